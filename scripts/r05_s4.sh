# Round 5, session 4: Coverage greedy expert step in episodes vs steady state
# (scripts/cov_greedy_probe.py), with one and two launches per step, and a rocprofv3
# kernel trace of the probe.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r05_s4; mkdir -p $O
timeout -k 10 300 python scripts/cov_greedy_probe.py > $O/probe2.json 2> $O/probe2.err; rc=$?; echo "probe rc=$rc"; cat $O/probe2.json
[ $rc -ne 0 ] && { tail $O/probe2.err; exit $rc; }
STREAMS=1 timeout -k 10 300 python scripts/cov_greedy_probe.py > $O/probe1.json 2> $O/probe1.err; rc=$?; echo "probe1 rc=$rc"; cat $O/probe1.json
[ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/scripts/cov_greedy_probe.py > $O/trace.log 2>&1; rc=$?; echo "trace rc=$rc"
exit $rc
