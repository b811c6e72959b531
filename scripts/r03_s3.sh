#!/bin/bash
# Round-3 session 3: Coverage kernel (first round trip before the dirty wait, tagged claim
# rounds) parity + A/B vs HEAD + phase timeline; N=8192 phase timeline; PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s3; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_cov.log 2>&1 || { tail -30 $O/pytest_cov.log; exit 1; }
tail -1 $O/pytest_cov.log
timeout -k 10 500 bash scripts/ab_cov.sh > $O/ab_cov.txt 2>&1 || { cat $O/ab_cov.txt; exit 1; }
grep -v "^$" $O/ab_cov.txt | tail -8
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > $O/cov_timeline.json 2>&1 || { cat $O/cov_timeline.json; exit 1; }
cat $O/cov_timeline.json
N=8192 B=16 GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/phase_timeline.py > $O/timeline_8192.txt 2>&1 || { cat $O/timeline_8192.txt; exit 1; }
head -30 $O/timeline_8192.txt
cd /tmp
R=$GRAFT_REPO_ROOT
N=8192 B=32 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc8192_f -o pmc -- python3 $R/scripts/pmc_step.py > $R/$O/pmc8192_f.log 2>&1 &&
N=8192 B=32 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc8192_w -o pmc -- python3 $R/scripts/pmc_step.py > $R/$O/pmc8192_w.log 2>&1 &&
KNN=1 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmcknn_f -o pmc -- python3 $R/scripts/pmc_step.py > $R/$O/pmcknn_f.log 2>&1 &&
KNN=1 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmcknn_w -o pmc -- python3 $R/scripts/pmc_step.py > $R/$O/pmcknn_w.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmccov_f -o pmc -- python3 $R/scripts/pmc_cov.py > $R/$O/pmccov_f.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmccov_w -o pmc -- python3 $R/scripts/pmc_cov.py > $R/$O/pmccov_w.log 2>&1
echo "pmc rc=$?"
ls -R $R/$O | grep -i csv | head
