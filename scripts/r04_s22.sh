# Debug: RCCL teardown with torch's HIP runtime bound (scripts/dbg/comm_probe.py).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
for cfg in "1 init" "1 stats" "1 rewards"; do set -- $cfg
  GF_BT=1 TORCH=$1 MODE=$2 timeout -k 10 120 python -u scripts/dbg/comm_probe.py > $O/s22_$1_$2.log 2>&1; rc=$?
  echo "torch=$1 mode=$2 rc=$rc: $(grep -v '^Extension' $O/s22_$1_$2.log | grep -v '^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl' | tail -3 | tr '\n' ' ' | cut -c1-300)"
  [ $rc -ge 124 ] && [ $rc -ne 134 ] && exit $rc
done
exit 0
