# Round 5, session 15: the Coverage launch probe again (1 / 2 / 2-threaded launches per step),
# three rounds, for box-to-box spread.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s15; mkdir -p $O
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null
REPS=3 timeout -k 10 240 python scripts/cov_launch_probe.py > $O/cov_launch_probe.json 2>&1; r1=$?; cat $O/cov_launch_probe.json; cat $O/nproc.txt
exit $r1
