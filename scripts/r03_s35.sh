#!/bin/bash
# Driver-window bench (20 steps after 5) with config 5 timed over the headline's K steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s35; mkdir -p $O
set -o pipefail
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
python -c "
import json;d=json.load(open('$O/bench20.json'))
print('plain', round(d['ms_per_step']*1e3,1), round(d['roofline']['frac'],3))
for k in ('step_with_controller','flocking_v0_knn7','coverage_config4','n8192_config5'):
  v=d[k]; print(k, v.get('steps'), round(v['ms_per_step']*1e3,2), round(v['roofline']['frac'],3))
"
