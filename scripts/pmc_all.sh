#!/bin/bash
# Summarise a profile session's PMC passes (scripts/session_recipes.sh r05_profile) into
# profiles/pmc_traffic.json: per-launch HBM bytes of each bench sub-line's kernel beside its
# algorithmic bytes per launch.   bash scripts/pmc_all.sh gpurun_out/r05_v2
D=$1
S() {  # S <name> <key> <kernel substring> <algorithmic bytes> [skip]
  python scripts/pmc_summary.py $D/pmc_$1_FETCH_SIZE/pmc_counter_collection.csv \
    $D/pmc_$1_WRITE_SIZE/pmc_counter_collection.csv "$2" "$3" "$4" ${5:-0}
}
S plain 1024x256 "flock_step_kernel<true, false, false, false, 0, 0, false, 0>" 1098909696 &&
S ctrl ctrl_1024x256 "flock_step_kernel<true, true, true, false, 0, 0, false, 0>" 1103104000 &&
S packed packed_1024x256 "flock_step_kernel<true, false, false, false, 0, 0, false, 0>" 59770880 &&
S knn knn7_1024x256 "flock_step_kernel<true, false, false, false, 0, 7, false, 0>" 1137707008 &&
S n8192 8192x32 "flock_step_kernel<true, false, false, false, 1, 0, false, 0>" 8615100672 &&
S cov coverage_r200x512 "cov_step_kernel<256, false>" 14344192 1
