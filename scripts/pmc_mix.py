"""Per-launch instruction counters of the step kernels from rocprofv3 --pmc csv dirs
(scripts/session_recipes.sh r03_s15): one line per configuration, per-wave VALU/SALU/LDS and the VALU
issue time they imply (wave64 VALU = 4 cycles of a 16-lane SIMD, 1024 SIMDs, 2.4 GHz).
  python scripts/pmc_mix.py gpurun_out/s15"""
import collections
import csv
import os
import sys

root = sys.argv[1]
for d in sorted(os.listdir(root)):
    f = os.path.join(root, d, "pmc_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(float)
    launches = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if "flock_step_kernel" not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        launches[r["Counter_Name"]].add(r["Dispatch_Id"])
    n = max(len(v) for v in launches.values())
    w = agg["SQ_WAVES"] / n
    v = agg["SQ_INSTS_VALU"] / n
    print("%-14s waves %6d  VALU/wave %6.0f  SALU/wave %6.0f  LDS/wave %5.0f  VMEM rd/wr per wave %5.1f/%5.1f  "
          "VALU issue %6.1f us  ACTIVE_VALU %6.1f us  WAVE_CYCLES/wave %8.0f" % (
              d, w, v / w, agg["SQ_INSTS_SALU"] / n / w, agg["SQ_INSTS_LDS"] / n / w,
              agg["SQ_INSTS_VMEM_RD"] / n / w, agg["SQ_INSTS_VMEM_WR"] / n / w,
              v * 4 / 1024 / 2.4e3, agg["SQ_ACTIVE_INST_VALU"] / n * 4 / 1024 / 2.4e3,
              agg["SQ_WAVE_CYCLES"] / n / w * 4))
