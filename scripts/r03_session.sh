#!/bin/bash
# Round-3 GPU session: GPU test suite, launcher refusal on a 1-GPU box, driver-window bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03s}
mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 5 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
python bench.py --gpus 2 --steps 5 > $O/launcher_2gpus.log 2>&1; echo "launcher --gpus 2 rc=$? (2 expected on a 1-GPU box)"; cat $O/launcher_2gpus.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 2 $O/smoke.log &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && tail -c 300 $O/bench20.json
echo "rc=$?"
