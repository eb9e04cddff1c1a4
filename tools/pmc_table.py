"""Per-kernel ratios from a tools/pmc_kernel.sh summary (dev tool): VALU / MFMA instruction ratio, MFMA-pipe and
VALU busy fractions, wave wait / issue-stall shares, LDS bank-conflict share.  python tools/pmc_table.py FILE"""
import re
import sys

cur, d = None, {}
for line in open(sys.argv[1]):
    if line.startswith("stats"):
        print(line.strip())
        continue
    if line.startswith("=="):
        cur = line[3:].strip()
        d[cur] = {}
        continue
    m = re.match(r"\s+(\S+)\s+(\S+)", line)
    if m and cur:
        d[cur][m.group(1)] = float(m.group(2))
for k, v in d.items():
    if "argus" not in k:
        continue
    simd_cycles = v.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024
    mf = max(1.0, v.get("SQ_INSTS_MFMA", 1))
    wc = v.get("SQ_WAVE_CYCLES", 1)
    print(f"{k[:64]:64s} valu/mfma {v.get('SQ_INSTS_VALU', 0) / mf:6.2f}  mfma_busy "
          f"{v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / simd_cycles:.3f}  valu_busy "
          f"{4 * v.get('SQ_ACTIVE_INST_VALU', 0) / simd_cycles:.3f}  wait {v.get('SQ_WAIT_ANY', 0) / wc:.2f}  "
          f"stall {v.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}  lds_conflict "
          f"{v.get('SQ_LDS_BANK_CONFLICT', 0) / max(1.0, v.get('SQ_LDS_IDX_ACTIVE', 1)):.2f}")
