"""Per-kernel VGPRs / spills / occupancy from a hipcc -Rpass-analysis=kernel-resource-usage
log (make -C gym-flock_amd/csrc asm 2> log). Usage: python scripts/resusage.py log [substring]"""
import re
import sys

want = sys.argv[2] if len(sys.argv) > 2 else "step"
cur, rows = None, {}
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s.*?(VGPRs Spill|VGPRs|AGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for name, r in rows.items():
    if want in name:
        short = re.sub(r"^_ZN2gf12_GLOBAL__N_1\d+", "", name)
        print("%-60s vgpr %3s spill %s occ %s" % (short[:60], r.get("VGPRs"), r.get("VGPRs Spill"),
                                                  r.get("Occupancy [waves/SIMD]")))
