"""Write small HDF5 dataset fixtures in the reference's on-disk format (tests/conftest.py:18-57,
argus/data.py:137-188) with REAL h5py — run with an interpreter that has h5py (build container:
/opt/conda/bin/python3.9). Two files: libver "earliest" (h5py default: superblock v0, symbol-table
groups) and libver "latest" (superblock v3, v2 object headers, link messages), both read back by
argus_amd.h5lite in tests/test_data.py. Values are seeded and also stored in fixtures.json so the
test compares element-for-element. Images are not stored: tests synthesise the PNGs with PIL.
"""
import json
import sys
from pathlib import Path

import h5py
import numpy as np

OUT = Path(__file__).resolve().parent / "h5"


def poses(rng, n):
    t = rng.normal(size=(n, 3))
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    return np.concatenate([t, q], 1)  # (x, y, z, qw, qx, qy, qz) as the datagen writes


def main():
    rng = np.random.default_rng(7)
    data = {"train": poses(rng, 10), "test": poses(rng, 5)}
    qleap = {"train": rng.normal(size=(10, 23)), "test": rng.normal(size=(5, 23))}
    stems = {"train": [f"img/img{i}" for i in range(10)], "test": [f"img/img{i}" for i in range(10, 15)]}
    # "vlen_*": img_stems written exactly as argus/data_generation.py:256,264 does (a plain list of
    # str, which h5py>=3 stores as variable-length UTF-8 strings in the global heap)
    for name, libver in (("earliest", "earliest"), ("latest", "latest"), ("vlen_earliest", "earliest"),
                         ("vlen_latest", "latest")):
        d = OUT / f"ds_{name}"
        d.mkdir(parents=True, exist_ok=True)
        with h5py.File(d / f"ds_{name}.hdf5", "w", libver=libver) as f:
            f.attrs["n_cams"] = 2
            f.attrs["W"] = 256
            f.attrs["H"] = 256
            for g in ("train", "test"):
                grp = f.create_group(g)
                grp.create_dataset("cube_poses", data=data[g])
                grp.create_dataset("q_leap", data=qleap[g])
                if name.startswith("vlen"):
                    grp.create_dataset("img_stems", data=list(stems[g]))
                    assert h5py.check_string_dtype(grp["img_stems"].dtype).length is None
                else:
                    grp.create_dataset("img_stems", data=np.array([s.encode("utf-8") for s in stems[g]]))
    with open(OUT / "fixtures.json", "w") as f:
        json.dump({"cube_poses": {k: v.tolist() for k, v in data.items()},
                   "q_leap": {k: v.tolist() for k, v in qleap.items()}, "img_stems": stems,
                   "attrs": {"n_cams": 2, "W": 256, "H": 256}, "h5py": h5py.__version__,
                   "python": sys.version.split()[0]}, f)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
