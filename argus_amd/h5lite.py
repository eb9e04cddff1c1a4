"""Minimal read-only HDF5 reader for the argus dataset files (no h5py in this environment).

Covers what h5py writes for argus (argus/data_generation.py:247,313-314; tests/conftest.py:43-57):
superblock v0/v1 (h5py's default "earliest" libver) and v2/v3; object headers v1 and v2 (with
continuation blocks); groups as old-style symbol tables (v1 B-tree + local heap) or link messages;
datasets with contiguous or compact layout (data layout message v1-v4); datatypes fixed-point,
IEEE float, fixed-length string and variable-length string (the form h5py>=3 gives a list of str,
as argus/data_generation.py:256,264 writes ``img_stems``; elements resolved through the global heap
collections, returned as bytes like h5py's ``[()]``); simple dataspaces; attributes (v1-v3).
Chunked/compressed datasets, dense (fractal-heap) link storage, variable-length sequences and
references are rejected with a clear error. Pure Python + numpy, read via mmap.
"""
from __future__ import annotations

import mmap
import struct
from typing import Any

import numpy as np

_SIG = b"\x89HDF\r\n\x1a\n"


class VlenStr:
    """Variable-length string datatype (HDF5 class 9, type 1): each stored element is a 4-byte byte
    count + a global heap ID (collection address, 4-byte object index)."""

    def __init__(self, so: int):
        self.itemsize = 4 + so + 4
        self.record = np.dtype([("len", "<u4"), ("addr", f"<u{so}"), ("idx", "<u4")])


class H5Error(ValueError):
    pass


class _Reader:
    def __init__(self, path: str):
        self._f = open(path, "rb")
        self.buf = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        for base in (0, 512, 1024, 2048, 4096, 8192):
            if self.buf[base:base + 8] == _SIG:
                break
        else:
            raise H5Error(f"{path}: not an HDF5 file")
        self.sb = base
        ver = self.buf[base + 8]
        if ver in (0, 1):
            self.so, self.sl = self.buf[base + 13], self.buf[base + 14]
            p = base + 24 + (4 if ver == 1 else 0)
            self.base_addr = self.off(p)
            p += 4 * self.so  # base, free-space, eof, driver addresses
            # root symbol table entry: link name offset, object header address, cache type, ...
            self.root = self.off(p + self.so)
        elif ver in (2, 3):
            self.so, self.sl = self.buf[base + 9], self.buf[base + 10]
            p = base + 12
            self.base_addr = self.off(p)
            self.root = self.off(p + 3 * self.so)
        else:
            raise H5Error(f"unsupported superblock version {ver}")

    def close(self):
        self.buf.close()
        self._f.close()

    def off(self, p: int) -> int:
        return int.from_bytes(self.buf[p:p + self.so], "little")

    def length(self, p: int) -> int:
        return int.from_bytes(self.buf[p:p + self.sl], "little")

    def u(self, p: int, n: int) -> int:
        return int.from_bytes(self.buf[p:p + n], "little")

    # ---------------------------------------------------------------- object headers
    def messages(self, addr: int):
        """Yield (type, data_offset, size) for every header message of the object at ``addr``."""
        b = self.buf
        if b[addr:addr + 4] == b"OHDR":
            yield from self._messages_v2(addr)
            return
        if b[addr] != 1:
            raise H5Error(f"unsupported object header version {b[addr]} at {addr}")
        nmsg = self.u(addr + 2, 2)
        size = self.u(addr + 8, 4)
        blocks = [(addr + 16, size)]
        seen = 0
        while blocks and seen < nmsg:
            p, n = blocks.pop(0)
            end = p + n
            while p + 8 <= end and seen < nmsg:
                mtype, msize = self.u(p, 2), self.u(p + 2, 2)
                data = p + 8
                seen += 1
                if mtype == 0x10:  # continuation
                    blocks.append((self.off(data), self.length(data + self.so)))
                else:
                    yield mtype, data, msize
                p = data + msize

    def _messages_v2(self, addr: int):
        b = self.buf
        flags = b[addr + 5]
        p = addr + 6
        if flags & 0x20:
            p += 16
        if flags & 0x10:
            p += 4
        csize_len = 1 << (flags & 3)
        csize = self.u(p, csize_len)
        p += csize_len
        blocks = [(p, csize)]
        track_order = bool(flags & 0x04)
        while blocks:
            p, n = blocks.pop(0)
            end = p + n
            while p + 4 <= end:
                mtype, msize, mflags = b[p], self.u(p + 1, 2), b[p + 3]
                p += 4 + (2 if track_order else 0)
                if mtype == 0x10:
                    caddr, clen = self.off(p), self.length(p + self.so)
                    blocks.append((caddr + 4, clen - 8))  # skip "OCHK" and trailing checksum
                elif mtype != 0:
                    yield mtype, p, msize
                p += msize
            del mflags

    # ---------------------------------------------------------------- messages
    def dataspace(self, p: int) -> tuple:
        ver, ndim, flags = self.buf[p], self.buf[p + 1], self.buf[p + 2]
        if ver == 1:
            q = p + 8
        elif ver == 2:
            if self.buf[p + 3] == 2:  # null dataspace
                return ()
            q = p + 4
        else:
            raise H5Error(f"dataspace version {ver}")
        return tuple(self.length(q + i * self.sl) for i in range(ndim))

    def datatype(self, p: int) -> np.dtype:
        cls_ver = self.buf[p]
        cls = cls_ver & 0x0F
        bits = self.u(p + 1, 3)
        size = self.u(p + 4, 4)
        be = ">" if bits & 1 else "<"
        if cls == 0:
            signed = bool(bits & 0x08)
            return np.dtype(f"{be}{'i' if signed else 'u'}{size}")
        if cls == 1:
            return np.dtype(f"{be}f{size}")
        if cls == 3:
            return np.dtype(f"S{size}")
        if cls == 9:
            if bits & 0x0F != 1:
                raise H5Error("variable-length sequences are not supported (only variable-length strings)")
            if size != 4 + self.so + 4:
                raise H5Error(f"unexpected variable-length string element size {size}")
            return VlenStr(self.so)
        raise H5Error(f"unsupported HDF5 datatype class {cls}")

    def global_heap_object(self, addr: int, idx: int) -> bytes:
        """Object ``idx`` of the global heap collection at ``addr`` (collections are cached)."""
        cache = self.__dict__.setdefault("_gcol", {})
        objs = cache.get(addr)
        if objs is None:
            b = self.buf
            if b[addr:addr + 4] != b"GCOL":
                raise H5Error(f"bad global heap collection at {addr}")
            end = addr + self.length(addr + 8)
            p = addr + 8 + self.sl
            objs = {}
            while p + 8 + self.sl <= end:
                oid = self.u(p, 2)
                n = self.length(p + 8)
                if oid == 0:  # free space: the rest of the collection
                    break
                objs[oid] = bytes(b[p + 8 + self.sl:p + 8 + self.sl + n])
                p += 8 + self.sl + ((n + 7) & ~7)
            cache[addr] = objs
        if idx not in objs:
            raise H5Error(f"global heap object {idx} missing in collection {addr}")
        return objs[idx]

    def layout(self, p: int, shape: tuple, dt: np.dtype):
        ver = self.buf[p]
        n = int(np.prod(shape)) if shape else 1
        nbytes = n * dt.itemsize
        if ver in (1, 2):
            ndim, cls = self.buf[p + 1], self.buf[p + 2]
            q = p + 8
            if cls == 0:  # compact: dims then size + data
                q += 4 * ndim
                size = self.u(q, 4)
                return ("raw", q + 4, size)
            addr = self.off(q)
            if cls == 1:
                return ("raw", addr, nbytes)
            raise H5Error("chunked HDF5 datasets are not supported")
        if ver in (3, 4):
            cls = self.buf[p + 1]
            if cls == 0:
                size = self.u(p + 2, 2)
                return ("raw", p + 4, size)
            if cls == 1:
                return ("raw", self.off(p + 2), nbytes)
            raise H5Error("chunked/virtual HDF5 datasets are not supported")
        raise H5Error(f"data layout version {ver}")

    def attribute(self, p: int) -> tuple[str, Any]:
        ver = self.buf[p]
        nlen, tlen, slen = self.u(p + 2, 2), self.u(p + 4, 2), self.u(p + 6, 2)
        pad = (lambda x: (x + 7) & ~7) if ver == 1 else (lambda x: x)
        q = p + 8 + (1 if ver == 3 else 0)
        name = bytes(self.buf[q:q + nlen]).split(b"\0", 1)[0].decode()
        q += pad(nlen)
        dt = self.datatype(q)
        q += pad(tlen)
        shape = self.dataspace(q)
        q += pad(slen)
        n = int(np.prod(shape)) if shape else 1
        arr = self.elements(dt, n, q)
        return name, (arr.reshape(shape) if shape else arr[0])

    def elements(self, dt, n: int, offset: int) -> np.ndarray:
        """``n`` stored elements of type ``dt`` at ``offset`` (variable-length strings resolved to
        bytes objects, as h5py returns them)."""
        if isinstance(dt, VlenStr):
            rec = np.frombuffer(self.buf, dtype=dt.record, count=n, offset=offset)
            out = np.empty(n, dtype=object)
            for i, (ln, addr, idx) in enumerate(rec):
                out[i] = self.global_heap_object(int(addr), int(idx))[:int(ln)] if addr else b""
            return out
        return np.frombuffer(self.buf, dtype=dt, count=n, offset=offset).copy()

    # ---------------------------------------------------------------- groups
    def children(self, addr: int) -> dict:
        out = {}
        for mtype, p, _ in self.messages(addr):
            if mtype == 0x11:  # symbol table
                self._btree_group(self.off(p), self.off(p + self.so), out)
            elif mtype == 0x06:  # link message
                name, target = self._link(p)
                if target is not None:
                    out[name] = target
            elif mtype == 0x02 and self.off(p + 2 + (8 if self.buf[p + 1] & 1 else 0)) != (1 << (8 * self.so)) - 1:
                raise H5Error("dense (fractal heap) HDF5 link storage is not supported")
        return out

    def _heap_data(self, heap_addr: int) -> int:
        if self.buf[heap_addr:heap_addr + 4] != b"HEAP":
            raise H5Error("bad local heap")
        return self.off(heap_addr + 8 + 2 * self.sl)

    def _btree_group(self, btree: int, heap: int, out: dict) -> None:
        data = self._heap_data(heap)
        b = self.buf
        if b[btree:btree + 4] != b"TREE":
            raise H5Error("bad group B-tree")
        level, used = b[btree + 5], self.u(btree + 6, 2)
        p = btree + 8 + 2 * self.so
        for i in range(used):
            child = self.off(p + self.sl + i * (self.sl + self.so))
            if level > 0:
                self._btree_group(child, heap, out)
                continue
            if b[child:child + 4] != b"SNOD":
                raise H5Error("bad symbol table node")
            nsym = self.u(child + 6, 2)
            e = child + 8
            esz = 2 * self.so + 24
            for j in range(nsym):
                name_off, obj = self.off(e + j * esz), self.off(e + j * esz + self.so)
                q = data + name_off
                name = bytes(b[q:b.find(b"\0", q)]).decode()
                out[name] = obj

    def _link(self, p: int):
        b = self.buf
        flags = b[p + 1]
        q = p + 2
        ltype = 0
        if flags & 0x08:
            ltype = b[q]
            q += 1
        if flags & 0x04:
            q += 8
        if flags & 0x10:
            q += 1
        nl = 1 << (flags & 3)
        nlen = self.u(q, nl)
        q += nl
        name = bytes(b[q:q + nlen]).decode()
        q += nlen
        return name, (self.off(q) if ltype == 0 else None)


class Dataset:
    def __init__(self, r: _Reader, addr: int):
        self._r, self._addr = r, addr
        shape, dt, lay = None, None, None
        for mtype, p, _ in r.messages(addr):
            if mtype == 0x01:
                shape = r.dataspace(p)
            elif mtype == 0x03:
                dt = r.datatype(p)
            elif mtype == 0x08:
                lay = p
        if shape is None or dt is None or lay is None:
            raise H5Error("not a dataset")
        self.shape, self.dtype = shape, dt
        self._layout = r.layout(lay, shape, dt)

    def __getitem__(self, key):
        kind, off, size = self._layout
        n = int(np.prod(self.shape)) if self.shape else 1
        if off == (1 << (8 * self._r.so)) - 1:  # never written -> fill value 0
            arr = np.full(n, b"", dtype=object) if isinstance(self.dtype, VlenStr) else np.zeros(n, dtype=self.dtype)
        else:
            arr = self._r.elements(self.dtype, n, off)
        arr = arr.reshape(self.shape) if self.shape else arr[0]
        return arr if key == () or key is Ellipsis else arr[key]


class Group:
    def __init__(self, r: _Reader, addr: int):
        self._r, self._addr = r, addr
        self._kids = r.children(addr)
        self.attrs = {}
        for mtype, p, _ in r.messages(addr):
            if mtype == 0x0C:
                k, v = r.attribute(p)
                self.attrs[k] = v

    def keys(self):
        return list(self._kids)

    def __contains__(self, k):
        return k in self._kids

    def __getitem__(self, path: str):
        node: Any = self
        for part in [x for x in path.split("/") if x]:
            addr = node._kids[part]
            kinds = {m for m, _, _ in self._r.messages(addr)}
            node = Dataset(self._r, addr) if 0x08 in kinds else Group(self._r, addr)
        return node


class File(Group):
    """``with File(path) as f: f["train"]["cube_poses"][()]; f.attrs["n_cams"]`` (h5py-like)."""

    def __init__(self, path: str, mode: str = "r"):
        if mode != "r":
            raise H5Error("h5lite is read-only")
        r = _Reader(path)
        super().__init__(r, r.root)

    def close(self):
        self._r.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
