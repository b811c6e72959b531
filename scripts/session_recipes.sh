#!/bin/bash
# Every per-session GPU driver of rounds 3-5, folded into one file: one shell function per
# session, named as the session (r05_s2 wrote gpurun_out/r05_s2/, r05_profile v7 wrote
# gpurun_out/r05_v7/, ...), each body the session's commands as run. profiles/r0N/SOURCES.md
# maps every committed profile file to the session (function) that produced it. Run one as
#   gpurun -- bash scripts/session_recipes.sh r05_s2
# (the tools they call, bench.py, scripts/*.py, profile_round.sh, pmc_all.sh, ab_*.sh,
# stay separate files).

r03_ab1() {
# Round-3 A/B: fused-kNN list insertion (med3) and rcp+Newton reciprocal; parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ab1; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
ROUNDS=3 timeout -k 10 900 bash scripts/ab_knn_libs.sh base med3 tree nr2 > $O/ab_knn.txt 2>&1 || { cat $O/ab_knn.txt; exit 1; }
cat $O/ab_knn.txt
ROUNDS=2 timeout -k 10 600 bash scripts/ab_plain_libs.sh base tree nr2 > $O/ab_plain.txt 2>&1 || { cat $O/ab_plain.txt; exit 1; }
cat $O/ab_plain.txt
for o in 0 1; do OTHER=$([ $o = 1 ] && echo 1) KSTEPS=200 WARM=5 timeout -k 10 120 python scripts/knn_line.py > $O/other$o.txt 2>&1; echo "other=$o $(tail -1 $O/other$o.txt)"; done
}

r03_ab2() {
# Round-3 A/B: N=8192 adjacency bits in a global scratch (L2) instead of LDS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ab2; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
for v in gb16 gb32; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "config5" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
ROUNDS=3 timeout -k 10 900 bash scripts/ab_n8192_libs.sh tree gb16 gb32 gb16w6 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
}

r03_profile() {
# A round-3 measurement set in one GPU session: the GPU suite, smoke, the default bench line
# (driver window and 200 steps), rocprofv3 kernel stats of the bench, and PMC HBM traffic
# (FETCH_SIZE and WRITE_SIZE passes) of every bench sub-line's kernel.
#   bash scripts/r03_profile.sh v1        -> gpurun_out/r03_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
R=$PWD
O=$R/gpurun_out/r03_$TAG
mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
timeout -k 10 500 python bench.py > $O/bench200.json 2> $O/bench200.err || { tail $O/bench200.err; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/rocprof_trace.log 2>&1 || { tail $O/rocprof_trace.log; exit 1; }
pmc() {  # pmc <name> <script> [env...]
  local name=$1 script=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${name}_$c -o pmc -- python3 $R/scripts/$script > $O/pmc_${name}_$c.log 2>&1 || return 1
  done
}
pmc plain pmc_step.py &&
pmc ctrl pmc_step.py MODE=ctrl &&
pmc packed pmc_step.py MODE=packed &&
pmc knn pmc_step.py KNN=1 &&
pmc n8192 pmc_step.py N=8192 B=32 &&
pmc cov pmc_cov.py
echo "pmc rc=$?"
}

r03_session() {
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
}

r03_s3() {
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
}

r03_s4() {
# Round-3 session 4: wide-env cell-list step: parity, then config 5 against the tiled build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s4; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -12 $O/pytest_grid.log
ROUNDS=3 timeout -k 10 600 bash scripts/ab_n8192_libs.sh old tree > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
}

r03_s5() {
# Round-3 session 5: cell-list step after the parallel prep scan: parity, config-5 A/B,
# rocprofv3 kernel stats of the config-5 line, and config 2 through the cell list (A/B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s5; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -1 $O/pytest_grid.log
ROUNDS=3 timeout -k 10 600 bash scripts/ab_n8192_libs.sh old tree > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8192 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n-agents 8192 --n-envs 32 --steps 20 --warmup 3 --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line > $GRAFT_REPO_ROOT/$O/prof8192.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof8192.log; exit 1; }
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03s5/prof8192/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print("%-70s %6s %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
ROUNDS=2 timeout -k 10 600 bash scripts/ab_plain_libs.sh tree grid1k > $O/ab_plain.txt 2>&1 || { cat $O/ab_plain.txt; exit 1; }
cat $O/ab_plain.txt
timeout -k 10 600 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_cov.log 2>&1 || { tail -30 $O/pytest_cov.log; exit 1; }
tail -1 $O/pytest_cov.log
timeout -k 10 500 bash scripts/ab_cov.sh > $O/ab_cov.txt 2>&1; rc=$?; grep -v "^$" $O/ab_cov.txt | tail -8; exit $rc
}

r03_s6() {
# Round-3 session 6: hashed cell-list step with the many-workgroup prep (bin, scan,
# scatter, order): parity at wide N and through the N=1024 variant; A/B and profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s6; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -1 $O/pytest_grid.log
GYMFLOCK_LIB=$PWD/build/lib_grid1k/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "not knn and not variant" > $O/pytest_grid1k.log 2>&1 || { tail -40 $O/pytest_grid1k.log; exit 1; }
tail -1 $O/pytest_grid1k.log
ROUNDS=3 timeout -k 10 600 bash scripts/ab_n8192_libs.sh old tree > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
ROUNDS=3 timeout -k 10 600 bash scripts/ab_plain_libs.sh tree grid1k > $O/ab_plain.txt 2>&1 || { cat $O/ab_plain.txt; exit 1; }
cat $O/ab_plain.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof8192 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --n-agents 8192 --n-envs 32 --steps 20 --warmup 3 --no-cpu-baseline --no-controller-line --no-packed-line --no-knn-line > $GRAFT_REPO_ROOT/$O/prof8192.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof8192.log; exit 1; }
GYMFLOCK_LIB=$GRAFT_REPO_ROOT/build/lib_grid1k/libgymflock.so KNN=0 KSTEPS=100 WARM=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof1k -o run -- python3 $GRAFT_REPO_ROOT/scripts/knn_line.py > $GRAFT_REPO_ROOT/$O/prof1k.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof1k.log; exit 1; }
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob
for tag in ("prof8192", "prof1k"):
    f = glob.glob("gpurun_out/r03s6/%s/**/*kernel_stats.csv" % tag, recursive=True)[0]
    print(tag)
    for r in list(csv.DictReader(open(f)))[:8]:
        print("  %-66s %6s %10.1f us" % (r["Name"][:66], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}

r03_s7() {
# Round-3 session 7: cell-list step, one vs two launches per step, vs the tiled kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s7; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_grid_step_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_grid.log 2>&1 || { tail -40 $O/pytest_grid.log; exit 1; }
tail -1 $O/pytest_grid.log
for r in 1 2; do
for lib in old tree; do for st in 1 2; do
  GYMFLOCK_LIB=$PWD/build/lib_$lib/libgymflock.so N=8192 B=32 STREAMS=$st timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1 | sed "s/^/$lib /"
done; done
for lib in old grid1k; do for st in 1 2; do
  GYMFLOCK_LIB=$PWD/build/lib_$lib/libgymflock.so N=1024 B=256 K=100 STREAMS=$st timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1 | sed "s/^/$lib /"
done; done
done
}

r03_s8() {
# Round-3 session 8: the store skeleton of the tiled step at N=8192 (diagnostic build):
# what the network stores alone cost, to bound what any compute restructuring can win.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  for d in 0 0x1A 0x41A 0x71A; do
    GYMFLOCK_LIB=$PWD/build/lib_diag/libgymflock.so DIAG=$d N=8192 B=32 K=20 timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1
  done
  for d in 0 0x1A 0x41A 0x71A; do
    GYMFLOCK_LIB=$PWD/build/lib_diag/libgymflock.so DIAG=$d N=1024 B=256 K=100 timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1
  done
  GYMFLOCK_LIB=$PWD/gym-flock_amd/lib/libgymflock.so N=8192 B=32 K=20 timeout -k 10 120 python scripts/time_grid.py 2>&1 | tail -1 | sed "s/^/grid /"
done
}

r03_s9() {
# Round-3 session 9: Coverage claim rounds tagged vs cleared (A/B, same box), the packed
# line's PMC, the Coverage timeline of the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r03s9; mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
GYMFLOCK_LIB=$R/build/lib_covtag/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_coverage_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_covtag.log 2>&1 || { tail -30 $O/pytest_covtag.log; exit 1; }
tail -1 $O/pytest_covtag.log
for i in 1 2 3 4; do
  timeout -k 10 200 python scripts/time_cov.py tree 2>&1 | tail -1
  GYMFLOCK_LIB=$R/build/lib_covtag/libgymflock.so timeout -k 10 200 python scripts/time_cov.py tagged 2>&1 | tail -1
done
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  MODE=packed timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_packed_$c -o pmc -- python3 $R/scripts/pmc_step.py > $O/pmc_packed_$c.log 2>&1 || exit 1
done
echo pmc ok
}

r03_s10() {
# Coverage node records: GPU Coverage tests, interleaved A/B against HEAD's library, timeline.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py > gpurun_out/s10_pytest.txt 2>&1
tail -2 gpurun_out/s10_pytest.txt
bash scripts/ab_cov_multi.sh lds0 nt128 > gpurun_out/s10_ab.txt 2>&1
cat gpurun_out/s10_ab.txt
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/s10_timeline.txt 2>&1
cat gpurun_out/s10_timeline.txt
}

r03_s11() {
# Coverage step: one launch per step vs the two-stream split, interleaved, same box.
set -e
mkdir -p gpurun_out
for i in 1 2 3; do
  STREAMS=1 timeout -k 10 200 python scripts/time_cov.py one
  STREAMS=2 timeout -k 10 200 python scripts/time_cov.py split
done
}

r03_s12() {
# Coverage step: one launch per step vs the two-stream split on the working tree, interleaved.
set -e
for i in 1 2 3; do
  STREAMS=1 timeout -k 10 200 python scripts/time_cov.py one
  STREAMS=2 timeout -k 10 200 python scripts/time_cov.py split
done
}

r03_s13() {
# Coverage: fewer dirty lines per step (constant tail stores skipped). GPU Coverage tests,
# A/B (split and one launch per step) against HEAD and the no-skip build, timeline.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py > gpurun_out/s13_pytest.txt 2>&1
tail -1 gpurun_out/s13_pytest.txt
bash scripts/ab_cov_multi.sh noskip > gpurun_out/s13_ab.txt 2>&1
for i in 1 2; do
  STREAMS=1 GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so timeout -k 10 200 python scripts/time_cov.py old-one
  STREAMS=1 timeout -k 10 200 python scripts/time_cov.py new-one
done >> gpurun_out/s13_ab.txt 2>&1
cat gpurun_out/s13_ab.txt
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/s13_timeline.txt 2>&1
}

r03_s14() {
# Instruction mix of the plain and Flocking-v0 step kernels (one launch per step, 5 steps):
# SQ instruction/cycle counters + GRBM_GUI_ACTIVE, one rocprofv3 --pmc pass each.
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/s14
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/plain -o pmc -- python3 scripts/pmc_step.py > $O/plain.log 2>&1
KNN=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/knn -o pmc -- python3 scripts/pmc_step.py > $O/knn.log 2>&1
C2="SQ_INSTS_VALU_FLOPS_FP64 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"
timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/plain2 -o pmc -- python3 scripts/pmc_step.py > $O/plain2.log 2>&1 || echo "pass2 plain rc=$?"
KNN=1 timeout -s KILL 120 rocprofv3 --pmc $C2 --output-format csv -d $O/knn2 -o pmc -- python3 scripts/pmc_step.py > $O/knn2.log 2>&1 || echo "pass2 knn rc=$?"
ls -R $O | head -30
}

r03_s15() {
# VALU/SALU/LDS instruction counts of the step kernels with parts switched off (diagnostic
# build, fe_diag switches), one rocprofv3 --pmc pass per configuration.
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/${S15_OUT:-s15}
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$n -o pmc -- python3 scripts/pmc_step.py > $O/$n.log 2>&1
}
run p_all DIAG=0 && run p_nofeat DIAG=2 && run p_nopass1 DIAG=8 && run p_nostage DIAG=16 && run p_conststore DIAG=1024 && run p_norowout DIAG=256 &&
run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && run k_noinsert KNN=1 DIAG=0x200000 && run k_nopred KNN=1 DIAG=0x20000 &&
run k_nogather KNN=1 DIAG=32 && run k_nofeat KNN=1 DIAG=2 && run k_norim KNN=1 DIAG=0x40000
echo "rc=$?"
}

r03_s16() {
# Pass 1 FMA + LDS-broadcast rows, network rows from an LDS nibble table: full GPU suite,
# then the bench A/B against HEAD's library.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s16_pytest.txt 2>&1 || { tail -30 gpurun_out/s16_pytest.txt; exit 1; }
tail -2 gpurun_out/s16_pytest.txt
ROUNDS=2 bash scripts/ab_bench.sh > gpurun_out/s16_ab.txt 2>&1
cat gpurun_out/s16_ab.txt
}

r03_s17() {
# Branch-free one-Newton reciprocal for the feature pair terms: GPU suite, bench A/B vs HEAD.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s17_pytest.txt 2>&1 || { tail -30 gpurun_out/s17_pytest.txt; exit 1; }
tail -2 gpurun_out/s17_pytest.txt
ROUNDS=2 bash scripts/ab_bench.sh > gpurun_out/s17_ab.txt 2>&1
cat gpurun_out/s17_ab.txt
}

r03_s18() {
# Instruction mix (SQ counters) of the current build's step kernels: plain, controller,
# Flocking-v0, N=8192 (one launch per step, 5 steps), one rocprofv3 --pmc pass each.
set -e
export TMPDIR=/tmp
O=$PWD/gpurun_out/s18
rm -rf $O; mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$n -o pmc -- python3 scripts/pmc_step.py > $O/$n.log 2>&1
}
run plain X=1 && run ctrl MODE=ctrl && run knn KNN=1 && run n8192 N=8192 B=32
python scripts/pmc_mix.py $O
}

r03_s19() {
# Coverage: hipLaunchKernel + bound Python call (host-bound split step): Coverage tests,
# time_cov A/B against HEAD's library (old Python path too: the tree's Python is used).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py > gpurun_out/s19_pytest.txt 2>&1
tail -1 gpurun_out/s19_pytest.txt
bash scripts/ab_cov_multi.sh > gpurun_out/s19_ab.txt 2>&1
cat gpurun_out/s19_ab.txt
}

r03_s20() {
# Coverage claim rounds tagged (no clears) with in-order LDS: A/B and both timelines.
set -e
mkdir -p gpurun_out
bash scripts/ab_cov_multi.sh covtag > gpurun_out/s20_ab.txt 2>&1
cat gpurun_out/s20_ab.txt
for v in stamps1 stamps_tag; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/s20_timeline_$v.json 2>&1
done
}

r03_s21() {
# Config 5 network store column-block-major: wide-env GPU tests, then N=8192 x 32 step
# time A/B (scripts/time_grid.py, two launches per step) against HEAD's library, plus the
# 8 GiB store probe of this box.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wide_step_gpu.py tests/test_flock_gpu.py > gpurun_out/s21_pytest.txt 2>&1 || { tail -30 gpurun_out/s21_pytest.txt; exit 1; }
tail -1 gpurun_out/s21_pytest.txt
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/old /'
  K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/new /'
done
hipcc -O3 --offload-arch=gfx950 scripts/storeprobe.hip -o /tmp/sp && timeout -k 10 200 /tmp/sp
}

r03_s22() {
# Plain step at 7 workgroups per CU (7-wave register budget, no LDS floor, rows read one
# at a time) against HEAD (6 per CU): headline-only bench A/B, 3 rounds, both 20 and 200 steps.
set -e
mkdir -p gpurun_out
X="--no-controller-line --no-packed-line --no-knn-line --no-other-configs"
ROUNDS=3 NEWLIB=$PWD/build/lib_w7/libgymflock.so bash scripts/ab_bench.sh $X > gpurun_out/s22_ab20.txt 2>&1
cat gpurun_out/s22_ab20.txt | grep -v "^setup\|^config\|^drop"
}

r03_s25() {
# Contiguous output buffers (>= 256 MiB): bench A/B (headline and config 5) against HEAD.
set -e
mkdir -p gpurun_out
X="--no-controller-line --no-packed-line --no-knn-line"
ROUNDS=3 bash scripts/ab_bench.sh $X > gpurun_out/s25_ab.txt 2>&1
grep -v "^setup\|^config\|^drop" gpurun_out/s25_ab.txt
}

r03_s26() {
# Contiguous buffers: config-5 store order A/B (row after row = HEAD vs column-block-major),
# wide-step tests on the block-major build, store probes in contiguous and default memory.
set -e
mkdir -p gpurun_out
GYMFLOCK_LIB=$PWD/build/lib_bm/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_wide_step_gpu.py > gpurun_out/s26_pytest.txt 2>&1 || { tail -30 gpurun_out/s26_pytest.txt; exit 1; }
tail -1 gpurun_out/s26_pytest.txt
for i in 1 2 3; do
  GYMFLOCK_LIB=$PWD/build/lib_old/libgymflock.so K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/row-major /'
  GYMFLOCK_LIB=$PWD/build/lib_bm/libgymflock.so K=40 timeout -k 10 200 python scripts/time_grid.py 2>&1 | sed 's/^/block-major /'
done
hipcc -O3 --offload-arch=gfx950 scripts/storeprobe.hip -o /tmp/sp
timeout -k 10 100 /tmp/sp c
timeout -k 10 100 /tmp/sp m
}

r03_s27() {
# Re-entry check after the container reset: GPU suite, smoke, driver-window bench at HEAD.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s27; mkdir -p $O
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
}

r03_s28() {
# Balanced feature pass (GF_FEAT_LIST: a row's pairs listed in LDS, dealt round robin over
# its slices) and lean pair terms (GF_PAIR_LEAN): flock/kNN GPU tests on the changed build,
# then Flocking-v0 and plain-step A/B, interleaved, against HEAD (lib_base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s28; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_listlean/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py > $O/pytest_listlean.txt 2>&1 || { tail -30 $O/pytest_listlean.txt; exit 1; }
tail -1 $O/pytest_listlean.txt
ROUNDS=2 bash scripts/ab_knn_libs.sh base list lean listlean 2>&1 | tee $O/ab_knn.txt
ROUNDS=2 bash scripts/ab_plain_libs.sh base lean 2>&1 | tee $O/ab_plain.txt
}

r03_s29() {
# Instruction counts (PMC) of the Flocking-v0 step on HEAD (lib_base), the balanced feature
# pass (lib_list) and lean pair terms (lib_lean): does the list cut VALU issue?
set -e
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/s29
mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
for n in base list lean; do
  GYMFLOCK_LIB=$PWD/build/lib_$n/libgymflock.so KNN=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/k_$n -o pmc -- python3 scripts/pmc_step.py > $O/k_$n.log 2>&1
done
python3 scripts/pmc_mix.py $O
}

r03_s30() {
# get_stats aggregates on the metrics path: the new GPU tests (summary vs oracle, RCCL
# all-gather at one rank), then the multi-rank bench path at one rank (--force-dist) with
# its gathered reward and stats checks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s30; mkdir -p $O
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_flock_gpu.py -k "stats" > $O/pytest_stats.txt 2>&1 || { tail -30 $O/pytest_stats.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/pytest_stats.txt | tail -5
timeout -k 10 300 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/bench_forcedist.json 2> $O/bench_forcedist.err || { tail -20 $O/bench_forcedist.err; exit 1; }
cat $O/bench_forcedist.json
}

r03_s31() {
# Fused kNN step with the plain step's paired row reads in pass 1 (GF_P1_PAIR_KNN):
# flock GPU tests on it, then Flocking-v0 A/B against HEAD (lib_base), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s31; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_pair/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py > $O/pytest_pair.txt 2>&1 || { tail -30 $O/pytest_pair.txt; exit 1; }
tail -1 $O/pytest_pair.txt
ROUNDS=3 bash scripts/ab_knn_libs.sh base pair 2>&1 | tee $O/ab_knn.txt
}

r03_s32() {
# Fused kNN step: paired row reads (lib_pair) and, on top, the predicted rows' candidate
# bounds and order from LDS tables with the mostly-predicted loop paired too (lib_ptab):
# flock GPU tests on lib_ptab, then Flocking-v0 A/B against HEAD (lib_base), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s32; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_ptab/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py > $O/pytest_ptab.txt 2>&1 || { tail -30 $O/pytest_ptab.txt; exit 1; }
tail -1 $O/pytest_ptab.txt
ROUNDS=3 bash scripts/ab_knn_libs.sh base pair ptab 2>&1 | tee $O/ab_knn.txt
}

r03_s33() {
# Instruction mix by part of the final round-3 build (diagnostic build, session r03_s15).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S15_OUT=s33 bash scripts/r03_s15.sh && python3 scripts/pmc_mix.py gpurun_out/s33
}

r03_s34() {
# Greedy expert: bounded block search over the cost row (in-tree lib) vs the whole-row scan
# (lib_gscan): Coverage GPU tests on the in-tree lib, then expert-step and time-matrix A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s34; mkdir -p $O
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py > $O/pytest_cov.txt 2>&1 || { tail -30 $O/pytest_cov.txt; exit 1; }
tail -1 $O/pytest_cov.txt
ROUNDS=3 bash scripts/ab_greedy_libs.sh tree gscan 2>&1 | tee $O/ab_greedy.txt
for n in tree gscan; do
  lib=$PWD/build/lib_$n/libgymflock.so; [ "$n" = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$lib timeout -k 10 200 python scripts/time_tm.py $n 2>&1 | tail -1 | tee -a $O/ab_tm.txt
done
}

r03_s35() {
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
}

r03_s36() {
# Greedy expert, uint8 rows: four targets per 32-bit operation (SWAR, in-tree lib) vs one
# (lib_gold = HEAD): Coverage GPU tests on the in-tree lib, then the expert-step A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s36; mkdir -p $O
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py > $O/pytest_cov.txt 2>&1 || { tail -30 $O/pytest_cov.txt; exit 1; }
tail -1 $O/pytest_cov.txt
ROUNDS=3 bash scripts/ab_greedy_libs.sh ${LIBS:-tree gold} 2>&1 | tee $O/ab_greedy.txt
}

r03_s37() {
# Greedy expert geometry after the SWAR search: lanes per robot and loads in flight.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s37; mkdir -p $O
set -o pipefail
GYMFLOCK_LIB=$PWD/build/lib_l4/libgymflock.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_coverage_greedy_gpu.py > $O/pytest_l4.txt 2>&1 || { tail -30 $O/pytest_l4.txt; exit 1; }
tail -1 $O/pytest_l4.txt
ROUNDS=2 bash scripts/ab_greedy_libs.sh tree l4 if2 l4if8 l16 2>&1 | tee $O/ab_greedy.txt
}

r03_s38() {
# Fused kNN merge with the exactness tests after the rounds (in-tree, GF_KNN_MERGE_LEAN=1)
# vs per round (lib_mold): flock GPU tests on the in-tree lib, then Flocking-v0 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s38; mkdir -p $O
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py > $O/pytest_flock.txt 2>&1 || { tail -30 $O/pytest_flock.txt; exit 1; }
tail -1 $O/pytest_flock.txt
ROUNDS=3 bash scripts/ab_knn_libs.sh tree mold 2>&1 | tee $O/ab_knn.txt
}

r03_s39() {
# Final check of the tree the round ends with: GPU suite and smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/s39; mkdir -p $O
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
}

r04_final() {
# Final check of the round-4 tree: GPU suite, smoke, a bench line (driver window) and the
# Flocking-v0 drop-in probe on the in-tree library.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04_final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -1 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.txt
[ $rc -ne 0 ] && exit $rc

timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err; rc=$?; echo "bench rc=$rc"
timeout -k 10 200 python scripts/dropin_knn_probe.py > $O/dropin_knn_probe.txt 2>&1; cat $O/dropin_knn_probe.txt

exit $rc
}

r04_profile() {
# A round-4 measurement set in one GPU session: the GPU suite, smoke, the default bench line
# (driver window and 200 steps), rocprofv3 kernel stats of the bench, and PMC HBM traffic
# (FETCH_SIZE and WRITE_SIZE passes) of every bench sub-line's kernel.
#   bash scripts/r04_profile.sh v1        -> gpurun_out/r04_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
R=$PWD
O=$R/gpurun_out/r04_$TAG
mkdir -p $O; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
timeout -k 10 500 python bench.py > $O/bench200.json 2> $O/bench200.err || { tail $O/bench200.err; exit 1; }
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
timeout -k 10 300 python scripts/dropin_probe.py > $O/dropin_probe.txt 2>&1 || { tail $O/dropin_probe.txt; exit 1; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/rocprof_trace.log 2>&1 || { tail $O/rocprof_trace.log; exit 1; }
pmc() {  # pmc <name> <script> [env...]
  local name=$1 script=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${name}_$c -o pmc -- python3 $R/scripts/$script > $O/pmc_${name}_$c.log 2>&1 || return 1
  done
}
pmc plain pmc_step.py &&
pmc ctrl pmc_step.py MODE=ctrl &&
pmc packed pmc_step.py MODE=packed &&
pmc knn pmc_step.py KNN=1 &&
pmc n8192 pmc_step.py N=8192 B=32 &&
pmc cov pmc_cov.py
echo "pmc rc=$?"
}

r04_session() {
# Round-4 GPU-box session. Modes (any combination, in order): test smoke bench bench200 prof
# Every GPU step has its own time limit; a crash/abort/timeout (exit >= 124, 134, 139)
# ends the session, an ordinary test failure (exit 1) does not.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${OUT:-gpurun_out/r04}; mkdir -p $O
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n ${TAILN:-15} "$O/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "ABORT after $name"; exit $rc; fi
  return 0
}
summ() {
python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", round(d["ms_per_step"] * 1e3, 1), "us frac", round(d["roofline"]["frac"], 3))
for k in ("step_with_controller", "packed_network", "flocking_v0_knn7", "coverage_config4", "n8192_config5"):
    v = d.get(k)
    if v:
        print(k, round(v["ms_per_step"] * 1e3, 2), "us frac", round(v["roofline"]["frac"], 3),
              "ratio", round(v.get("ratio_to_plain_step", 0), 3))
if d.get("dropin"):
    print("dropin", json.dumps(d["dropin"])[:900])
if d.get("coverage_config4", {}).get("greedy_expert"):
    print("greedy", json.dumps(d["coverage_config4"]["greedy_expert"])[:400])
PY
}
for MODE in "$@"; do
  case $MODE in
    test) step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider ;;
    testk) step pytest_gpu_k 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "$K" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench20 600 python bench.py --steps 20 --warmup 5 && (grep "^{" $O/bench20.log | tail -1 > $O/bench20.json; summ $O/bench20.json) ;;
    bench200) step bench200 600 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-other-configs && summ $O/bench200.log ;;
    prof) step rocprof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o trace -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    *) echo "unknown mode $MODE"; exit 2 ;;
  esac
done
echo "=== done"
}

r04_s3() {
bash scripts/r04_session.sh test smoke && ROUNDS=3 OUT=gpurun_out/r04/ab_ctrl timeout -k 10 900 python scripts/ab_multi.py old=build/lib_old/libgymflock.so rc0=build/lib_rc0/libgymflock.so rc1=build/lib_rc1/libgymflock.so rc2=build/lib_rc2/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s4() {
bash scripts/r04_session.sh test && ROUNDS=3 OUT=gpurun_out/r04/ab_plain timeout -k 10 900 python scripts/ab_multi.py old=build/lib_old/libgymflock.so new=gym-flock_amd/lib/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s5() {
bash scripts/r04_session.sh test && ROUNDS=3 OUT=gpurun_out/r04/ab_knn64 timeout -k 10 900 python scripts/ab_multi.py old=build/lib_old/libgymflock.so r32=build/lib_r32/libgymflock.so new=gym-flock_amd/lib/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s7() {
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/cov_tests.log 2>&1; echo "cov tests rc=$?"; tail -5 $O/cov_tests.log
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.log 2>&1 && grep "^{" $O/bench_cov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1e3, json.dumps(d.get('greedy_expert')))"
timeout -k 5 40 ./build/comm_probe 1 && timeout -k 5 40 ./build/comm_probe 0
echo "probe rc=$?"
}

r04_s8() {
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py tests/test_flock_gpu.py -k "coverage or greedy or wire or dropin or step_host" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/cov_tests.log 2>&1; echo "tests rc=$?"; tail -5 $O/cov_tests.log
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.log 2>&1 && grep "^{" $O/bench_cov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1e3, json.dumps(d.get('greedy_expert')))"
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench
class A: pass
print(json.dumps(bench.bench_dropin(A())))" > $O/dropin.log 2>&1; tail -3 $O/dropin.log
ROUNDS=2 OUT=gpurun_out/r04/ab_mode1 timeout -k 10 600 python scripts/ab_multi.py new=gym-flock_amd/lib/libgymflock.so mode1=build/lib_mode1/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
timeout -k 5 40 ./build/comm_probe 1 && timeout -k 5 40 ./build/comm_probe 0
echo "probe rc=$?"
}

r04_s9() {
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_metrics_gpu.py tests/test_flock_gpu.py -k "metrics or comm or gather or dropin or step_host or host_pool or stats" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s9_tests.log 2>&1; echo "tests rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed|lone-rank" $O/s9_tests.log | tail -30
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench
class A: pass
print(json.dumps(bench.bench_dropin(A())))" > $O/dropin2.log 2>&1; tail -1 $O/dropin2.log | cut -c1-900
}

r04_s10() {
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_metrics_gpu.py tests/test_flock_gpu.py -k "metrics or comm or gather or dropin or step_host or host_pool or stats" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s10_tests.log 2>&1; echo "tests rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/s10_tests.log | tail -40
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench.py']; sys.path.insert(0,'.')
import bench
class A: pass
print(json.dumps(bench.bench_dropin(A())))" > $O/dropin3.log 2>&1; tail -1 $O/dropin3.log | cut -c1-900
GYMFLOCK_LIB=$PWD/build/lib_v2/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py tests/test_flock_variants_gpu.py tests/test_stream_ordering_gpu.py -k "knn or v0 or variant or flocking" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s10_knn_v2.log 2>&1; echo "knn v2 tests rc=$?"; tail -5 $O/s10_knn_v2.log
ROUNDS=3 OUT=gpurun_out/r04/ab_v2 timeout -k 10 700 python scripts/ab_multi.py base=gym-flock_amd/lib/libgymflock.so v2=build/lib_v2/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
echo "== ctrl instruction mix by part"
export TMPDIR=/tmp
P=$PWD/gpurun_out/r04/pmc_ctrl; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run p_all DIAG=0 && run c_all MODE=ctrl DIAG=0 && run c_nofeat MODE=ctrl DIAG=2 && run c_nopass1 MODE=ctrl DIAG=8 &&
run c_recip MODE=ctrl DIAG=2048 && run c_nograd MODE=ctrl DIAG=4096 && run c_norowout MODE=ctrl DIAG=256 && run c_noreward MODE=ctrl DIAG=512 &&
python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt
echo "== coverage greedy timeline"
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so GREEDY=1 timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/r04/cov_timeline_greedy.json 2>&1; echo "tl rc=$?"; head -c 1500 gpurun_out/r04/cov_timeline_greedy.json
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so timeout -k 10 200 python scripts/cov_timeline.py > gpurun_out/r04/cov_timeline_random.json 2>&1; echo "tl rc=$?"
}

r04_s11() {
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r04/v2trace; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_v2/libgymflock.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O -o v2 -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-other-configs --no-packed-line --no-controller-line > $O/bench.log 2>&1; echo "rc=$?"
find $O -name "*kernel_stats.csv" | head -3
for f in $(find $O -name "*kernel_stats.csv"); do cut -d, -f1-8 $f | head -12; done
}

r04_s12() {
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_w6/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -k "knn or v0" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s12_knn_w6.log 2>&1; echo "knn w6 tests rc=$?"; tail -2 $O/s12_knn_w6.log
GYMFLOCK_LIB=$PWD/build/lib_c32/libgymflock.so timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -k "controller or ctrl or expert or closed" -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s12_ctrl_c32.log 2>&1; echo "ctrl c32 tests rc=$?"; tail -2 $O/s12_ctrl_c32.log
ROUNDS=3 OUT=gpurun_out/r04/ab_w6 timeout -k 10 900 python scripts/ab_multi.py base=gym-flock_amd/lib/libgymflock.so w6=build/lib_w6/libgymflock.so c32=build/lib_c32/libgymflock.so -- --no-other-configs --no-packed-line
echo "== knn instruction mix by part"
P=$PWD/gpurun_out/r04/pmc_knn; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run p_all DIAG=0 && run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && run k_noinsert KNN=1 DIAG=0x200000 && run k_nopred KNN=1 DIAG=0x20000 &&
run k_nogather KNN=1 DIAG=32 && run k_nofeat KNN=1 DIAG=2 && run k_nopass1 KNN=1 DIAG=8 && run k_norim KNN=1 DIAG=0x40000 &&
python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt
}

r04_s13() {
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_flock_gpu.py tests/test_stream_ordering_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s13_flock.log 2>&1; echo "flock tests rc=$?"; tail -2 $O/s13_flock.log
ROUNDS=3 OUT=gpurun_out/r04/ab_s13 timeout -k 10 900 python scripts/ab_multi.py c32=build/lib_c32/libgymflock.so new=gym-flock_amd/lib/libgymflock.so sf0=build/lib_sf0/libgymflock.so -- --no-other-configs --no-packed-line
P=$PWD/gpurun_out/r04/pmc_knn2; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt
}

r04_s14() {
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s14_cov.log 2>&1; echo "cov tests rc=$?"; tail -2 $O/s14_cov.log
for r in 0 1 2; do for L in old:build/lib_old new:gym-flock_amd/lib; do n=${L%%:*}; d=${L#*:}
GYMFLOCK_LIB=$PWD/$d/libgymflock.so timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/s14_${n}_$r.log 2>&1 || { echo "bench failed $n"; exit 1; }
grep "^{" $O/s14_${n}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('greedy_expert',{}); print('$r $n step %.2f us  expert %.2f  two_launch %.2f  episodes %.2f  tm %.1f ms' % (d['ms_per_step']*1e3, g['expert_step_ms']*1e3, g['expert_step_ms_two_launches']*1e3, g['expert_step_ms_in_episodes']*1e3, g['time_matrix_ms_all_envs']))"
done; done
GYMFLOCK_LIB=$PWD/build/lib_stamps1/libgymflock.so GREEDY=1 timeout -k 10 200 python scripts/cov_timeline.py > $O/cov_timeline_greedy2.json 2>&1; echo "tl rc=$?"; python -c "
import json; d=json.load(open('$O/cov_timeline_greedy2.json')); print(d['launch_span_us'], {k:(v['median'],v['p90'],v['max']) for k,v in d['phases_us'].items()})"
}

r04_s15() {
# Flocking-v0 A/B: superset pass 1 (sup), fast network store loop (sf), both (supsf) vs base.
# kNN-related GPU tests run on the sup+sf build first (parity), then the interleaved bench A/B.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_supsf/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s15_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/s15_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s15 timeout -k 10 900 python scripts/ab_multi.py base=build/lib_base/libgymflock.so sup=build/lib_sup/libgymflock.so sf=build/lib_sf/libgymflock.so supsf=build/lib_supsf/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s16() {
# Flocking-v0 A/B 2: kNN key by fma + saturating convert, exact words by LDS atomic clears
# (supsf2, sf2) vs supsf and base; sfp = supsf2 with the fast store loop for the plain step too.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_sfp/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py tests/test_stream_ordering_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s16_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/s16_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s16 timeout -k 10 900 python scripts/ab_multi.py base=build/lib_base/libgymflock.so supsf=build/lib_supsf/libgymflock.so supsf2=build/lib_supsf2/libgymflock.so sf2=build/lib_sf2/libgymflock.so sfp=build/lib_sfp/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s17() {
# PMC instruction mix of the Flocking-v0 step with the superset pass 1 + fast store loop
# (diagnostic build of supsf2): whole kernel and with parts switched off.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
P=$PWD/gpurun_out/r04/pmc_knn3; mkdir -p $P
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
L=$PWD/build/lib_diag2/libgymflock.so
run() {  # run <name> <env...>
  local n=$1; shift
  env GYMFLOCK_LIB=$L "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P/$n -o pmc -- python3 scripts/pmc_step.py > $P/$n.log 2>&1
}
run k_all KNN=1 DIAG=0 && run k_nomerge KNN=1 DIAG=1 && run k_nogather KNN=1 DIAG=32 && run k_noinsert KNN=1 DIAG=0x200000 && run k_nofeat KNN=1 DIAG=2 && run k_nopred KNN=1 DIAG=0x20000 && run p_all DIAG=0 && python scripts/pmc_mix.py $P > $P/mix.txt; cat $P/mix.txt
}

r04_s18() {
# Flocking-v0 A/B 3: the fused kNN step at 6 waves per SIMD (80 VGPRs; the superset pass 1
# leaves its spills outside the loops) vs 5 (supsf2); w6n = 6 waves without the superset.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_w6s/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s18_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/s18_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s18 timeout -k 10 900 python scripts/ab_multi.py supsf2=build/lib_supsf2/libgymflock.so w6s=build/lib_w6s/libgymflock.so w6n=build/lib_w6n/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s19() {
# Phase timelines (GF_STAMPS=1) of the plain and the Flocking-v0 step (supsf2 code).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
L=$PWD/build/lib_st1/libgymflock.so
GYMFLOCK_LIB=$L timeout -k 10 200 python scripts/phase_timeline.py > $O/s19_plain.txt 2>&1 && GYMFLOCK_LIB=$L KNN=1 timeout -k 10 200 python scripts/phase_timeline.py > $O/s19_knn.txt 2>&1; echo rc=$?
head -22 $O/s19_plain.txt; head -22 $O/s19_knn.txt
}

r04_s20() {
# Product build with the superset pass 1 + fast store loop for the fused kNN step:
# the GPU suite, smoke, a bench line, then phase timelines (GF_STAMPS build).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s20_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/s20_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/s20_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/s20_smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/s20_bench.json 2> $O/s20_bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
python - $O/s20_bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", round(d["ms_per_step"] * 1e3, 1), "us frac", round(d["roofline"]["frac"], 3))
for k in ("step_with_controller", "packed_network", "flocking_v0_knn7", "coverage_config4", "n8192_config5"):
    v = d.get(k)
    if v:
        print(k, round(v["ms_per_step"] * 1e3, 2), "us frac", round(v["roofline"]["frac"], 3), "ratio", round(v.get("ratio_to_plain_step", 0), 3))
PY
L=$PWD/build/lib_st1/libgymflock.so
GYMFLOCK_LIB=$L timeout -k 10 200 python scripts/phase_timeline.py > $O/s20_tl_plain.txt 2>&1 && GYMFLOCK_LIB=$L KNN=1 timeout -k 10 200 python scripts/phase_timeline.py > $O/s20_tl_knn.txt 2>&1; echo tl rc=$?
head -18 $O/s20_tl_plain.txt; head -18 $O/s20_tl_knn.txt
}

r04_s21() {
# Debug: does the HEAD library (build/lib_base) abort in the full GPU suite too?
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_base/libgymflock.so GF_ABORT_BT=1 timeout -k 10 600 python -u -m pytest -s -p no:faulthandler tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/s21_g.log 2>&1; echo "d rc=$?"; grep -v "^Extension" $O/s21_g.log | grep -v PASSED | tail -30
}

r04_s22() {
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
}

r04_s23() {
# Flocking-v0 A/B 4: inline-rim scan with 1 column in flight per lane (u1; its register
# peak set the kernel's) at 5 and 6 waves per SIMD, vs the current build.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_u1w6/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s23_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/s23_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s23 timeout -k 10 900 python scripts/ab_multi.py cur=build/lib_cur/libgymflock.so u1w5=build/lib_u1w5/libgymflock.so u1w6=build/lib_u1w6/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s24() {
# Phase timeline of the kNN step built for 6 waves per SIMD (inline rim U=1), to see where
# the 6-wave build loses (A/B: 225 vs 197 us) against the 5-wave timeline (s20_tl_knn.txt).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_st6/libgymflock.so KNN=1 timeout -k 10 200 python scripts/phase_timeline.py > $O/s24_tl_knn_w6.txt 2>&1; echo tl rc=$?
head -18 $O/s24_tl_knn_w6.txt
}

r04_s25() {
# Flocking-v0 A/B 5: hybrid pass 1 (superset on every tile but the last; the last tile's
# bits exact from the band sweep, its feature pass after the network stores) vs superset on
# every tile (cur).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_hyb/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s25_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/s25_tests.log
[ $rc -ge 124 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s25 timeout -k 10 900 python scripts/ab_multi.py cur=build/lib_cur/libgymflock.so hyb=build/lib_hyb/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s26() {
# One-tile envs take their rows from the tile staging; a single one-tile env's host actions travel
# in the kernel arguments (fe_step_host). GPU suite,
# the drop-in probe and a bench line (its dropin sub-object).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s26_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -2 $O/s26_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/dropin_probe.py > $O/s26_dropin_probe.txt 2>&1; echo "probe rc=$?"; tail -3 $O/s26_dropin_probe.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s26_bench.json 2> $O/s26_bench.err; echo "bench rc=$?"
python - $O/s26_bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", round(d["ms_per_step"] * 1e3, 1), "knn", round(d["flocking_v0_knn7"]["ms_per_step"] * 1e3, 1))
dd = d["dropin"]; print("dropin n100 direct", dd["n100"]["direct"], "pooled", dd["n100"]["pooled"])
PY
for r in 0 1; do for s in 1 2; do STREAMS=$s ROUNDS=3 timeout -k 10 120 python scripts/time_cov.py s$s > $O/s26_cov_s${s}_$r.txt 2>&1; echo "cov streams=$s round $r: $(tail -2 $O/s26_cov_s${s}_$r.txt | tr '\n' ' ')"; done; done
GYMFLOCK_LIB=$PWD/build/lib_cand/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s26_cand_tests.log 2>&1; echo "cand kNN tests rc=$?"; tail -1 $O/s26_cand_tests.log
ROUNDS=3 OUT=gpurun_out/r04/ab_s26 timeout -k 10 900 python scripts/ab_multi.py head=build/lib_head/libgymflock.so new=gym-flock_amd/lib/libgymflock.so cand=build/lib_cand/libgymflock.so -- --no-other-configs --no-packed-line
STEPS=200 WARMUP=20 ROUNDS=2 OUT=gpurun_out/r04/ab_s26_200 timeout -k 10 900 python scripts/ab_multi.py new=gym-flock_amd/lib/libgymflock.so cand=build/lib_cand/libgymflock.so -- --no-other-configs --no-packed-line
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline > $O/s26_forcedist.json 2> $O/s26_forcedist.err; echo "forcedist rc=$?"
python - $O/s26_forcedist.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print({k: d.get(k) for k in ("ms_per_step", "n_gpus", "gathered_rewards_ok", "gathered_stats_ok", "rccl")})
PY
}

r04_s27() {
# A/B of the round-4 latency changes' effect on the batched lines: head (before them),
# new (one-tile rows in the staging lambda + kernel-argument actions), new2 (one-tile rows
# copied from the staged tile after a barrier, outside the staging lambda), nouin (new2
# without the kernel-argument-action template parameter).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_new2/libgymflock.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s27_tests.log 2>&1; rc=$?; echo "new2 gpu suite rc=$rc"; tail -1 $O/s27_tests.log
[ $rc -ne 0 ] && exit $rc
ROUNDS=3 OUT=gpurun_out/r04/ab_s27 timeout -k 10 1000 python scripts/ab_multi.py head=build/lib_head/libgymflock.so new=gym-flock_amd/lib/libgymflock.so new2=build/lib_new2/libgymflock.so nouin=build/lib_nouin/libgymflock.so -- --no-other-configs --no-packed-line
}

r04_s28() {
# Flocking-v0 A/B 6: the predicted rows' candidate radius^2 factor (2.25 x the 7th-nearest
# r2 two states back, product) against 1.69 and 1.44, over 20 and 200 steps.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_cf144/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s28_tests.log 2>&1; rc=$?; echo "cf144 kNN tests rc=$rc"; tail -1 $O/s28_tests.log
[ $rc -ge 124 ] && exit $rc
STEPS=200 WARMUP=20 ROUNDS=2 OUT=gpurun_out/r04/ab_s28_200 timeout -k 10 900 python scripts/ab_multi.py cur=gym-flock_amd/lib/libgymflock.so cf169=build/lib_cf169/libgymflock.so cf144=build/lib_cf144/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
ROUNDS=3 OUT=gpurun_out/r04/ab_s28 timeout -k 10 900 python scripts/ab_multi.py cur=gym-flock_amd/lib/libgymflock.so cf169=build/lib_cf169/libgymflock.so cf144=build/lib_cf144/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
}

r04_s29() {
# The inline-action boundary tests, then the final round-4 profile set (v3).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flock_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "inline_actions or dropin" > $O/s29_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error|passed|failed" $O/s29_tests.log | tail -12
[ $rc -ne 0 ] && exit $rc
bash scripts/session_recipes.sh r04_profile v3
}

r04_s30() {
# Flocking-v0 drop-in step through fe_step_host_knn: GPU tests (flock file + the capi
# export check), then the latency probe (FlockingRelative direct, Flocking-v0 pooled/direct).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py tests/test_flock_variants_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/s30_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/s30_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/dropin_knn_probe.py
}

r04_s31() {
# Kernel trace of the drop-in Flocking-v0 step at N=100 (where its 68 us go).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r04/s31; mkdir -p $O
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o knn -- python3 $R/scripts/dbg/knn_dropin_loop.py > $O/log.txt 2>&1; echo rc=$?
cut -c1-200 $O/knn_kernel_stats.csv
python3 - $O/knn_kernel_trace.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-12:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    print("%-60s start %8.1f us  dur %6.1f us" % (r["Kernel_Name"][:60], (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
PY
}

r04_s32() {
# Small envs (N <= 128): every unranked row of the fused kNN step ranked by its wave's inline
# scan (no rim work). kNN tests on that build, then the drop-in probe: product vs ilim.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_ilim/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking or dropin" > $O/s32_tests.log 2>&1; rc=$?; echo "ilim tests rc=$rc"; tail -1 $O/s32_tests.log
[ $rc -ne 0 ] && exit $rc
for L in gym-flock_amd/lib build/lib_ilim; do echo $L; GYMFLOCK_LIB=$PWD/$L/libgymflock.so timeout -k 10 200 python scripts/dropin_knn_probe.py; done
}

r04_s33() {
# Fused kNN step: up to 4 unranked rows per wave ranked inline (ir4) vs 2 (ir2, product),
# 20 and 200 steps; kNN tests on ir4.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
GYMFLOCK_LIB=$PWD/build/lib_ir4/libgymflock.so timeout -k 10 600 python -u -m pytest tests/test_flock_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "knn or flocking_v0 or Flocking" > $O/s33_tests.log 2>&1; rc=$?; echo "ir4 tests rc=$rc"; tail -1 $O/s33_tests.log
ROUNDS=3 OUT=gpurun_out/r04/ab_s33 timeout -k 10 900 python scripts/ab_multi.py ir2=build/lib_ir2/libgymflock.so ir4=build/lib_ir4/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
STEPS=200 WARMUP=20 ROUNDS=2 OUT=gpurun_out/r04/ab_s33_200 timeout -k 10 900 python scripts/ab_multi.py ir2=build/lib_ir2/libgymflock.so ir4=build/lib_ir4/libgymflock.so -- --no-other-configs --no-packed-line --no-controller-line
}

r04_s34() {
# bench.py's dropin sub-object with the Flocking-v0 entries (driver window).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/s34_bench.json 2> $O/s34_bench.err; rc=$?; echo "bench rc=$rc"
python - $O/s34_bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 1) for kk, vv in v.items()} for k, v in d["dropin"][n].items()})
PY
exit $rc
}

r05_profile() {
# A round-5 measurement set in one GPU session: the GPU suite, smoke, the default bench line
# (driver window and 200 steps), the Coverage workload (with the greedy expert), the
# multi-rank path at one rank (--force-dist: the RCCL reward and stats gathers), a rocprofv3
# kernel trace + stats of a 100-step bench with its per-grid kernel stats and step periods
# (scripts/trace_by_grid.py), and PMC HBM traffic (FETCH_SIZE and WRITE_SIZE passes) of every
# bench sub-line's kernel (summarised here by scripts/pmc_all.sh).
#   bash scripts/r05_profile.sh v2        -> gpurun_out/r05_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
R=$PWD
O=$R/gpurun_out/r05_$TAG
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
echo "bench20 ok"
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench200.json 2> $O/bench200.err || { tail $O/bench200.err; exit 1; }
echo "bench200 ok"
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs > $O/bench_forcedist.json 2> $O/bench_forcedist.err || { tail $O/bench_forcedist.err; exit 1; }
echo "bench_forcedist ok"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/rocprof_trace.log 2>&1 || { tail $O/rocprof_trace.log; exit 1; }
cd $R
python scripts/trace_by_grid.py $O/trace/trace_kernel_trace.csv $O/trace_by_grid --steps 100 > $O/trace_by_grid.txt && cat $O/trace_by_grid.txt
cd /tmp
pmc() {  # pmc <name> <script> [env...]
  local name=$1 script=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${name}_$c -o pmc -- python3 $R/scripts/$script > $O/pmc_${name}_$c.log 2>&1 || return 1
  done
}
pmc plain pmc_step.py &&
pmc ctrl pmc_step.py MODE=ctrl &&
pmc packed pmc_step.py MODE=packed &&
pmc knn pmc_step.py KNN=1 &&
pmc n8192 pmc_step.py N=8192 B=32 &&
pmc cov pmc_cov.py
echo "pmc rc=$?"
# run-to-run spread of the headline on this box: three more driver-window lines
cd $R
for r in 1 2 3; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs > $O/bench20_rep$r.json 2>/dev/null; done
python - $O <<'PY'
import json, sys
for r in (1, 2, 3):
    d = json.loads(open("%s/bench20_rep%d.json" % (sys.argv[1], r)).read().strip().splitlines()[-1])
    print("rep", r, round(d["ms_per_step"] * 1e3, 2), "us", round(d["roofline"]["frac"], 3),
          "knn", round(d["flocking_v0_knn7"]["ms_per_step"] * 1e3, 2), round(d["flocking_v0_knn7"]["ratio_to_plain_step"], 3))
PY
# the GPU suite once more, after everything above (flakiness check)
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu_again.log 2>&1; echo "second suite rc=$?"; tail -1 $O/pytest_gpu_again.log
}

r05_s1() {
# Round 5, session 1: the GPU suite on the new tree (exact small-env kNN, fused
# Flocking-v0 expert action, staging stream of the metrics path, runtime binding tests),
# smoke, and one bench line in the driver's window with the drop-in probe.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -15 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench20.json 2> $O/bench20.err; rc=$?; echo "bench rc=$rc"
python - $O/bench20.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", d["ms_per_step"], d["roofline"]["frac"], "knn", d["flocking_v0_knn7"]["ms_per_step"], d["flocking_v0_knn7"]["ratio_to_plain_step"])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 1) for kk, vv in v.items()} for k, v in d["dropin"][n].items()})
print(d.get("runtime"))
for r in ("r6", "r200"):
    print(r, {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()} for k, v in d["dropin_coverage"][r].items()})
PY
exit $rc
}

r05_s2() {
# Round 5, session 2: the GPU suite on the tree, the kNN tests on the lean A/B library,
# the Flocking-v0 A/B (tree / lean / lean6 / w6u1), then one bench line with the drop-in
# probes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; rc=$?; echo "gpu suite rc=$rc"; tail -12 $O/pytest_gpu.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
GYMFLOCK_LIB=$PWD/build/lib_lean6/libgymflock.so timeout -k 10 300 python -u -m pytest tests/test_flock_gpu.py -m gpu -q -k "knn or flocking_v0 or golden" --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_lean6.log 2>&1; r2=$?; echo "lean6 knn tests rc=$r2"; tail -3 $O/pytest_lean6.log
[ $r2 -gt 1 ] && exit $r2
ROUNDS=2 timeout -k 10 400 bash scripts/ab_knn_libs.sh tree lean lean6 w6u1 > $O/ab_knn_lean.txt 2>&1; echo "ab rc=$?"; cat $O/ab_knn_lean.txt
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench20.json 2> $O/bench20.err; rc3=$?; echo "bench rc=$rc3"
python - $O/bench20.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", d["ms_per_step"], d["roofline"]["frac"], "knn", d["flocking_v0_knn7"]["ms_per_step"], d["flocking_v0_knn7"]["ratio_to_plain_step"])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 1) for kk, vv in v.items()} for k, v in d["dropin"][n].items()})
print(d.get("runtime"))
for r in ("r6", "r200"):
    print(r, {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()} for k, v in d["dropin_coverage"][r].items()})
PY
exit $rc
}

r05_s3() {
# Round 5, session 3: one bench line in the driver's window with every sub-object (drop-in
# probes for Flocking and Coverage included).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_cov.log 2>&1; r0=$?; echo "coverage tests rc=$r0"; tail -3 $O/pytest_cov.log
[ $r0 -gt 1 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --cpu-seconds 6 > $O/bench20.json 2> $O/bench20.err; rc=$?; echo "bench rc=$rc"; tail -3 $O/bench20.err
python - $O/bench20.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("plain", d["ms_per_step"], d["roofline"]["frac"], "knn", d["flocking_v0_knn7"]["ms_per_step"], d["flocking_v0_knn7"]["ratio_to_plain_step"])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 1) for kk, vv in v.items()} for k, v in d["dropin"][n].items()})
print(d.get("runtime"))
for r in ("r6", "r200"):
    print(r, {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()} for k, v in d["dropin_coverage"][r].items()})
PY
exit $rc
}

r05_s4() {
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
}

r05_s5() {
# Round 5, session 5: Coverage tests with the direct greedy path for short unvisited lists,
# then the greedy probe (steady state vs episodes).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_cov.log 2>&1; r0=$?; echo "coverage tests rc=$r0"; tail -15 $O/pytest_cov.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 300 python scripts/cov_greedy_probe.py > $O/probe2.json 2> $O/probe2.err; rc=$?; echo "probe rc=$rc"; cat $O/probe2.json
exit $rc
}

r05_s6() {
# Round 5, session 6: the greedy expert's fallback draws on the device (COV_GREEDY_RNG):
# Coverage tests, then the Coverage bench workload with the expert lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s6; mkdir -p $O
timeout -k 10 60 ./scripts/flagprobe.bin > $O/flagprobe.txt 2>&1; echo "flagprobe rc=$?"; cat $O/flagprobe.txt
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_cov.log 2>&1; r0=$?; echo "coverage tests rc=$r0"; tail -15 $O/pytest_cov.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s6/bench_cov.json").read().strip().splitlines()[-1])
def walk(o, p=""):
    for k, v in o.items():
        if isinstance(v, dict): walk(v, p + k + ".")
        elif "expert" in p + k or k in ("ms_per_step", "value"): print(p + k, "=", v)
walk(d)
PY
}

r05_s7() {
# Round 5, session 7: the drop-in steps wait for the kernel's completion flag; device
# fallback draws. Full GPU suite, the bench line (driver window) and the Coverage workload.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s7; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1; r0=$?; echo "gpu tests rc=$r0"; tail -5 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
echo "bench20 ok"
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
python - <<'PY'
import json
for f in ("bench20", "bench_cov"):
    d = json.loads(open("gpurun_out/r05_s7/%s.json" % f).read().strip().splitlines()[-1])
    def walk(o, p=""):
        for k, v in o.items():
            if isinstance(v, dict): walk(v, p + k + ".")
            elif "expert" in p + k or "dropin" in p or k in ("ms_per_step", "frac"): print(p + k, "=", v)
    walk(d)
PY
}

r05_s8() {
# Round 5, session 8: phase timelines of the plain and the Flocking-v0 step (config 2, one
# launch per step) from the stamps build (make -C gym-flock_amd/csrc stamps STAMPS=2).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s8; mkdir -p $O
export GYMFLOCK_LIB=$PWD/build/lib_stamps2/libgymflock.so
timeout -k 10 120 python scripts/phase_timeline.py > $O/tl_plain.txt 2>&1 || { tail $O/tl_plain.txt; exit 1; }
timeout -k 10 120 env KNN=1 python scripts/phase_timeline.py > $O/tl_knn.txt 2>&1 || { tail $O/tl_knn.txt; exit 1; }
head -22 $O/tl_plain.txt; echo ----; head -22 $O/tl_knn.txt
}

r05_s9() {
# Round 5, session 9: the drop-in Flocking-v0 step of a larger env waits for its rim kNN's
# completion flag. Flocking GPU tests, then the bench line (driver window).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s9; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_flock_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -5 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s9/bench20.json").read().strip().splitlines()[-1])
for n in ("n100", "n1024"):
    print(n, {k: {kk: round(vv * 1e3, 2) for kk, vv in v.items() if kk.endswith("_ms")} for k, v in d["dropin"][n].items() if isinstance(v, dict)})
print("plain", d["ms_per_step"], "knn", d["flocking_v0_knn7"]["ms_per_step"])
PY
}

r05_s10() {
# Round 5, session 10: the mid-run collective abort path (comm_event_wait timing out).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s10; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_metrics_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -30 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 timeout -k 10 300 ./build/asan/capi_asan > $O/asan.log 2>&1; ra=$?; echo "asan rc=$ra"; tail -5 $O/asan.log
[ $ra -ne 0 ] && exit $ra
timeout -k 10 120 python scripts/cov_launch_probe.py > $O/cov_launch_probe.json 2>&1; r1=$?; cat $O/cov_launch_probe.json
exit $r1
}

r05_s11() {
# Round 5, session 11: host launch cost of two streams from one thread vs two threads.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s11; mkdir -p $O
timeout -k 10 120 ./scripts/flagprobe.bin > $O/flagprobe.txt 2>&1; r=$?; cat $O/flagprobe.txt; exit $r
}

r05_s12() {
# Round 5, session 12: why the multi-rank path (--force-dist: one rank, reward all-gather
# every 8 steps) slows the plain step; kernel trace with queue ids.
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
O=$R/gpurun_out/r05_s12; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --force-dist --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
cd $R
timeout -k 10 300 python bench.py --force-dist --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/fd.json 2> $O/fd.err; echo "fd rc=$?"
timeout -k 10 300 python bench.py --force-dist --metrics-every 64 --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/fd64.json 2> $O/fd64.err; echo "fd64 rc=$?"
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line > $O/nofd.json 2> $O/nofd.err; echo "nofd rc=$?"
python - <<'PY'
import json
for f in ("fd", "fd64", "nofd"):
    d = json.loads(open("gpurun_out/r05_s12/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["config"]["parallelism"])
PY
ls $O/trace
}

r05_s13() {
# Round 5, session 13: the multi-rank path at one rank after re-warming the clocks that
# RCCL's initialisation let drop (bench.py REWARM_STEPS), against the plain line.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s13; mkdir -p $O
A="--steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --no-controller-line --no-packed-line --no-knn-line"
for r in 1 2; do
timeout -k 10 300 python bench.py --force-dist $A > $O/fd_$r.json 2> $O/fd_$r.err || { tail $O/fd_$r.err; exit 1; }
timeout -k 10 300 python bench.py $A > $O/nofd_$r.json 2> $O/nofd_$r.err || { tail $O/nofd_$r.err; exit 1; }
done
python - <<'PY'
import json
for f in ("fd_1", "nofd_1", "fd_2", "nofd_2"):
    d = json.loads(open("gpurun_out/r05_s13/%s.json" % f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"] * 1e3, 2), "us/step", d["config"]["parallelism"], d.get("clock_warmup"), d.get("gathered_rewards_ok"))
PY
}

r05_s14() {
# Round 5, session 14: Coverage split steps with the second half from a launcher thread
# (cov_set_streams 3) against one thread (2) and one launch (1); then the Coverage tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s14; mkdir -p $O
timeout -k 10 180 python scripts/cov_launch_probe.py > $O/cov_launch_probe.json 2>&1; r1=$?; cat $O/cov_launch_probe.json
[ $r1 -ne 0 ] && exit $r1
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -3 $O/pytest.log
exit $r0
}

r05_s15() {
# Round 5, session 15: the Coverage launch probe again (1 / 2 / 2-threaded launches per step),
# three rounds, for box-to-box spread.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s15; mkdir -p $O
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null
REPS=3 timeout -k 10 240 python scripts/cov_launch_probe.py > $O/cov_launch_probe.json 2>&1; r1=$?; cat $O/cov_launch_probe.json; cat $O/nproc.txt
exit $r1
}

r05_s16() {
# Round 5, session 16: Coverage steps with the automatic launch split (greedy steps in two
# halves, others one launch): tests, the Coverage workload, the greedy probe.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s16; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py tests/test_stream_ordering_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -3 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
for r in 1 2; do
timeout -k 10 300 python bench.py --workload coverage --steps 1000 --warmup 20 --no-cpu-baseline > $O/bench_cov_$r.json 2> $O/bench_cov_$r.err || { tail $O/bench_cov_$r.err; exit 1; }
done
timeout -k 10 300 python scripts/cov_greedy_probe.py > $O/probe.json 2> $O/probe.err; echo "probe rc=$?"
python - <<'PY'
import json
for r in (1, 2):
    d = json.loads(open("gpurun_out/r05_s16/bench_cov_%d.json" % r).read().strip().splitlines()[-1])
    print(r, round(d["ms_per_step"] * 1e3, 2), "us/step, frac", round(d["roofline"]["frac"], 3), "expert in episodes",
          round(d["greedy_expert"]["expert_step_ms_in_episodes"] * 1e3, 2), "us")
print(open("gpurun_out/r05_s16/probe.json").read())
PY
}

r05_s17() {
# Round 5, session 17: page-locked (completion flag) vs pageable (stream wait) drop-in outputs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s17; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_flock_gpu.py -m gpu -q -k "flag_and_stream or dropin" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -15 $O/pytest.log
exit $r0
}

r05_s18() {
# Round 5, session 18: the device fallback draws at the config-4 shape (64 envs, sampled).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s18; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py -m gpu -v -k "config4_batch" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -15 $O/pytest.log
exit $r0
}

r05_s19() {
# Round 5, session 19: reset()'s draws on the device (cov_reset_seeded): Coverage tests,
# the Coverage workload with the reset timings.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s19; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -15 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 300 python bench.py --workload coverage --steps 1000 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s19/bench_cov.json").read().strip().splitlines()[-1])
print(round(d["ms_per_step"] * 1e3, 2), {k: v for k, v in d["greedy_expert"].items() if "ms" in k})
PY
}

r05_s20() {
# Round 5, session 20: per-wave instruction mix (PMC) of the product build's step kernels:
# plain, step + controller, Flocking-v0 (scripts/pmc_mix.py summarises).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r05_s20; mkdir -p $O
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
cd /tmp
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$n -o pmc -- python3 $R/scripts/pmc_step.py > $O/$n.log 2>&1
}
run plain MODE=plain && run ctrl MODE=ctrl && run knn KNN=1
r=$?; echo "pmc rc=$r"
cd $R && python scripts/pmc_mix.py $O
exit $r
}

r05_s21() {
# Round 5, session 21: the Coverage expert / reset tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s21; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -8 $O/pytest.log
exit $r0
}

r05_s22() {
# Round 5, session 22: the Coverage workload with whole expert episodes.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s22; mkdir -p $O
timeout -k 10 300 python bench.py --workload coverage --steps 1000 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s22/bench_cov.json").read().strip().splitlines()[-1])
print(round(d["ms_per_step"] * 1e3, 2), {k: v for k, v in d["greedy_expert"].items() if "ms" in k or "per_s" in k})
PY
}

r05_s23() {
# Round 5, session 23: one-env Flocking-v0 handles ranked exactly in the step (tile = env,
# up to 1024 agents): Flocking GPU tests, then the drop-in probe lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s23; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_flock_gpu.py tests/test_wide_step_gpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; r0=$?; echo "tests rc=$r0"; tail -8 $O/pytest.log
[ $r0 -ne 0 ] && exit $r0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_s23/bench20.json").read().strip().splitlines()[-1])
for n in ("n100", "n1024"):
    print(n, {k: (round(v["step_ms"] * 1e3, 1), round(v["controller_plus_step_ms"] * 1e3, 1)) for k, v in d["dropin"][n].items() if isinstance(v, dict)})
print("plain", d["ms_per_step"], "knn", d["flocking_v0_knn7"]["ms_per_step"])
PY
}

r05_s24() {
# Round 5, session 24: A/B of the one-env exact in-step kNN threshold (1024: product build,
# 128: build/lib_exact128), drop-in Flocking-v0 per call over N, two rounds.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r05_s24; mkdir -p $O
for r in 1 2; do
timeout -k 10 200 python scripts/dropin_exact_probe.py >> $O/ab.txt 2>&1 || exit 1
timeout -k 10 200 env GYMFLOCK_LIB=$PWD/build/lib_exact128/libgymflock.so python scripts/dropin_exact_probe.py >> $O/ab.txt 2>&1 || exit 1
done
cat $O/ab.txt
}

r05_s25() {
# Deferred kNN ranking A/B (GF_KNN_DEFER): kNN GPU tests on the variants, then the
# Flocking-v0 line interleaved over base / noinl / d1 / d2 / d2i.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s25; mkdir -p $O
for v in d2 d2i; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_flock_gpu.py -m gpu -k "knn or flocking_v0 or Flocking" > $O/tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
ROUNDS=2 timeout -k 10 700 bash scripts/ab_knn_libs.sh base noinl d1 d2 d2i 2>&1 | tee $O/ab.txt
}

r05_s26() {
# Time-matrix schedule kernel (staged in LDS) and batch width A/B: Coverage GPU tests on
# the tree, then the drop-in first-step probe and the config-4 time matrix per library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s26; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
GYMFLOCK_LIB=$PWD/build/lib_tb16/libgymflock.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_coverage_greedy_gpu.py -m gpu > $O/tests_tb16.log 2>&1
rc=$?; echo "tests tb16 rc=$rc $(tail -1 $O/tests_tb16.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in tb8 tb16; do
    GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_${v}_$r.txt 2>&1 || exit 1
    echo "$v round $r first steps: $(grep 'step 0' $O/probe_${v}_$r.txt | awk '{print $5}' | tr '\n' ' ')"
    GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 300 python bench.py --workload coverage --steps 50 --warmup 10 --no-cpu-baseline > $O/cov_${v}_$r.json 2> $O/cov_${v}_$r.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$v round $r tm_all_envs_ms', round(d['greedy_expert']['time_matrix_ms_all_envs'],2))" $O/cov_${v}_$r.json
  done
done
}

r05_s27() {
# Multi-wave time-matrix passes for launches of few chunks: Coverage GPU tests on the tree
# (the drop-in and small-batch matrices now take it), then the drop-in first-step probe and
# the config-4 matrices, tree vs the one-wave form (GF_TM_FEW_CHUNKS=0), two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s27; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_coverage_greedy_gpu.py tests/test_coverage_gpu.py -m gpu > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in tree tm1w; do
    lib=$PWD/build/lib_$v/libgymflock.so; [ $v = tree ] && lib=$PWD/gym-flock_amd/lib/libgymflock.so
    GYMFLOCK_LIB=$lib timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_${v}_$r.txt 2>&1 || exit 1
    echo "$v round $r first steps: $(grep 'step 0' $O/probe_${v}_$r.txt | awk '{print $5}' | tr '\n' ' ')"
  done
done
GYMFLOCK_LIB=$PWD/gym-flock_amd/lib/libgymflock.so R=200 timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_r200.txt 2>&1 || exit 1
echo "tree R=200 first steps: $(grep 'step 0' $O/probe_r200.txt | awk '{print $5}' | tr '\n' ' ')"
}

r06_profile_a() {
# Round-6 measurement set, part A: the GPU suite, smoke, the default bench line (driver
# window, with the CPU baseline, the greedy expert and the new-map episode of config 4) and at
# 200 steps, the Coverage workload, the multi-rank path at one rank (--force-dist), and the
# time-matrix + greedy-list build of 512 distinct device maps (scripts/time_tm.py).
#   bash scripts/session_recipes.sh r06_profile_a v1   -> gpurun_out/r06_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
R=$PWD
O=$R/gpurun_out/r06_$TAG
mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
echo "bench20 ok"
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench200.json 2> $O/bench200.err || { tail $O/bench200.err; exit 1; }
echo "bench200 ok"
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
echo "bench_cov ok"
timeout -k 10 400 python bench.py --force-dist --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs > $O/bench_forcedist.json 2> $O/bench_forcedist.err || { tail $O/bench_forcedist.err; exit 1; }
echo "bench_forcedist ok"
ROUNDS=8 timeout -k 10 300 python scripts/time_tm.py r06 > $O/time_tm.json 2> $O/time_tm.err || { tail $O/time_tm.err; exit 1; }
cat $O/time_tm.json
}

r06_profile_b() {
# Round-6 measurement set, part B: a rocprofv3 kernel trace + stats of a 100-step bench with
# its per-grid kernel stats (scripts/trace_by_grid.py), PMC HBM traffic (FETCH_SIZE and
# WRITE_SIZE passes) of every bench sub-line's kernel (summarised by scripts/pmc_all.sh), and
# three more driver-window lines for the run-to-run spread.
#   bash scripts/session_recipes.sh r06_profile_b v1   -> gpurun_out/r06_<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-v1}
R=$PWD
O=$R/gpurun_out/r06_$TAG
mkdir -p $O; export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/rocprof_trace.log 2>&1 || { tail $O/rocprof_trace.log; exit 1; }
cd $R
python scripts/trace_by_grid.py $O/trace/trace_kernel_trace.csv $O/trace_by_grid --steps 100 > $O/trace_by_grid.txt && cat $O/trace_by_grid.txt
cd /tmp
pmc() {  # pmc <name> <script> [env...]
  local name=$1 script=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${name}_$c -o pmc -- python3 $R/scripts/$script > $O/pmc_${name}_$c.log 2>&1 || return 1
  done
}
pmc plain pmc_step.py &&
pmc ctrl pmc_step.py MODE=ctrl &&
pmc packed pmc_step.py MODE=packed &&
pmc knn pmc_step.py KNN=1 &&
pmc n8192 pmc_step.py N=8192 B=32 &&
pmc cov pmc_cov.py || { echo "pmc failed"; exit 1; }
cd $R
bash scripts/pmc_all.sh $O > $O/pmc_all.txt 2>&1; echo "pmc_all rc=$?"; cat $O/pmc_all.txt
for r in 1 2 3; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs > $O/bench20_rep$r.json 2>/dev/null || exit 1; done
python - $O <<'PY'
import json, sys
for r in (1, 2, 3):
    d = json.loads(open("%s/bench20_rep%d.json" % (sys.argv[1], r)).read().strip().splitlines()[-1])
    print("rep", r, round(d["ms_per_step"] * 1e3, 2), "us", round(d["roofline"]["frac"], 3),
          "knn", round(d["flocking_v0_knn7"]["ms_per_step"] * 1e3, 2), round(d["flocking_v0_knn7"]["ratio_to_plain_step"], 3))
PY
# the Coverage step's launch floor: wall, kernel and host enqueue time per step with one and
# two launches per step, with the runtime's kernel arguments in device memory (its default)
# and in host memory (HIP_FORCE_DEV_KERNARG=0)
for st in 2 1; do for ka in dflt 0; do
  if [ $ka = dflt ]; then e=""; else e="HIP_FORCE_DEV_KERNARG=0"; fi
  env $e STREAMS=$st ROUNDS=5 timeout -k 10 120 python scripts/time_cov.py s${st}_ka$ka >> $O/cov_launch_floor.txt 2>&1 || exit 1
done; done
cat $O/cov_launch_floor.txt
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_ka0.json 2> $O/bench20_ka0.err || { tail $O/bench20_ka0.err; exit 1; }
echo "bench20 (host kernargs) ok"
}

r06_s1() {
# Round 6, session 1 after the final set: host-action steps in 20- and 200-step windows
# (scripts/host_actions_probe.py); the time matrix with the XCD-grouped block mapping
# (product) against the grid-order build (build/lib_tm_noxcd, -DGF_TM_XCD=0) and the
# branch-free predecessor stores (build/lib_tm_buf, -DGF_TM_BUFSTORE=1; lib_tm_buf2 also
# -DGF_TM_BALLOT=1), interleaved;
# the Coverage expert/maps tests on the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s1; mkdir -p $O
timeout -k 10 200 python scripts/host_actions_probe.py > $O/host_actions_probe.txt 2>&1 || { cat $O/host_actions_probe.txt; exit 1; }
cat $O/host_actions_probe.txt
for r in 1 2; do for v in tm_noxcd prod tm_buf tm_buf2; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L timeout -k 10 120 python scripts/time_tm.py $v >> $O/ab_tm_xcd.txt 2>&1 || exit 1
done; done
cut -c1-110 $O/ab_tm_xcd.txt
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_maps_gpu.py tests/test_coverage_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for v in tm_buf tm_buf2; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 300 python -u -m pytest tests/test_coverage_greedy_gpu.py -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
}

r06_s2() {
# Round 6, session 2: the time matrix launched per occupancy class (product) against one
# launch sized to the largest env (build/lib_tm_buf, branch-free stores; build/lib_tm_noxcd,
# the build before both), interleaved; the Coverage tests and the Coverage bench on the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s2; mkdir -p $O
for r in 1 2; do for v in tm_noxcd tm_buf prod; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L timeout -k 10 120 python scripts/time_tm.py $v >> $O/ab_tm_classes.txt 2>&1 || exit 1
done; done
cut -c1-110 $O/ab_tm_classes.txt
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_maps_gpu.py tests/test_coverage_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
python - $O/bench_cov.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
g = d["greedy_expert"]
print("step", d["ms_per_step"], "tm", g["time_matrix_ms_all_envs"], "new-map episode", g["expert_episode_ms_all_envs_new_maps"],
      "maps+reset+tm", g["new_maps_reset_and_time_matrices_ms_all_envs"])
PY
}

r06_s3() {
# Round 6, session 3: the time matrix's edge schedule read in 64-slot windows by vector
# loads (build/lib_tm_vwin, -DGF_TM_VWIN=1) and, on top, batches software-pipelined within a
# conflict level (build/lib_tm_pipe, -DGF_TM_PIPE=1), against the product's per-batch scalar
# loads, three interleaved rounds; the Coverage greedy, maps and step tests on the variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s3; mkdir -p $O
for r in 1 2 3; do for v in prod tm_vwin tm_pipe; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L timeout -k 10 120 python scripts/time_tm.py $v >> $O/ab_tm_vwin.txt 2>&1 || exit 1
done; done
cut -c1-110 $O/ab_tm_vwin.txt
for v in tm_vwin tm_pipe prod; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_maps_gpu.py tests/test_coverage_gpu.py -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
}

r06_s6() {
# Round 6, session 6: the motion-graph kernel with its targets in LDS and the radius test
# decided from squared distances, and the map kernel's near-road test on a waypoint grid:
# the Coverage tests, the drop-in reset (scripts/cov_reset_probe.py, R=6 and 200) and the
# Coverage bench (map_ms_all_envs for 512 envs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_coverage_maps_gpu.py tests/test_coverage_gpu.py tests/test_coverage_greedy_gpu.py tests/test_coverage_wire_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/cov_reset_probe.py > $O/reset.txt 2>&1 && R=200 timeout -k 10 120 python scripts/cov_reset_probe.py >> $O/reset.txt 2>&1 || { cat $O/reset.txt; exit 1; }
cat $O/reset.txt
timeout -k 10 300 python bench.py --workload coverage --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_cov.json 2> $O/bench_cov.err || { tail $O/bench_cov.err; exit 1; }
python - $O/bench_cov.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
g, m = d["greedy_expert"], d["distinct_maps"]
print("maps 512:", m["map_ms_all_envs"], "ms; new-map episode", g["expert_episode_ms_all_envs_new_maps"], "ms; tm", g["time_matrix_ms_all_envs"])
PY
}

r06_s10() {
# Round 6, session 10: the drop-in greedy episode's first step (the new map's time matrix,
# cov_time_matrix_mw_kernel) with 2, 4 (product) and 8 waves per 64-source chunk
# (build/lib_tmw{2,8}, -DGF_TM_WAVES), interleaved, 8 episodes each; the Coverage greedy
# tests on the variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s10; mkdir -p $O
for r in 1 2; do for v in tmw2 prod tmw8; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L EPISODES=8 timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_${v}_$r.txt 2>&1 || exit 1
  echo "$v round $r first steps (us): $(grep 'step 0' $O/probe_${v}_$r.txt | awk '{print $5}' | tr '\n' ' ')"
done; done
for v in tmw2 tmw8; do
  GYMFLOCK_LIB=$PWD/build/lib_$v/libgymflock.so timeout -k 10 300 python -u -m pytest tests/test_coverage_greedy_gpu.py -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
}

r06_s11() {
# Round 6, session 11: the greedy lists' scan start kept per node across an episode
# (product) against the build before it (build/lib_gprev), interleaved
# (scripts/time_greedy_episodes.py), then the Coverage tests on the product; and the
# waves-per-chunk study of r06_s10 if its libraries are present.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s11; mkdir -p $O
for r in 1 2 3; do for v in gprev prod; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L timeout -k 10 120 python scripts/time_greedy_episodes.py $v >> $O/ab_gscan.txt 2>&1 || { tail -5 $O/ab_gscan.txt; exit 1; }
done; done
cut -c1-120 $O/ab_gscan.txt
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_maps_gpu.py tests/test_coverage_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/session_recipes.sh r06_s10
}

r06_s12() {
# Round 6, session 12: the drop-in first step with 8 waves per chunk (product) against 16
# (build/lib_tmw16), interleaved; the Coverage tests on the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s12; mkdir -p $O
for r in 1 2; do for v in prod tmw16; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L EPISODES=8 timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_${v}_$r.txt 2>&1 || exit 1
  echo "$v round $r first steps (us): $(grep 'step 0' $O/probe_${v}_$r.txt | awk '{print $5}' | tr '\n' ' ')"
done; done
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_maps_gpu.py tests/test_coverage_gpu.py tests/test_coverage_wire_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; exit $rc
}

r06_s19() {
# Round 6, session 19: the greedy-list block scan with its 32 masked flags loaded at once
# (product) against the build before it (build/lib_gprev), interleaved
# (scripts/time_greedy_episodes.py, then the drop-in expert loop's steps); the Coverage tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s19; mkdir -p $O
for r in 1 2 3; do for v in gprev prod; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L timeout -k 10 120 python scripts/time_greedy_episodes.py $v >> $O/ab_scan.txt 2>&1 || { tail -5 $O/ab_scan.txt; exit 1; }
done; done
cut -c1-120 $O/ab_scan.txt
timeout -k 10 400 python -u -m pytest tests/test_coverage_greedy_gpu.py tests/test_coverage_maps_gpu.py tests/test_coverage_gpu.py -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; exit $rc
}

r06_s20() {
# Round 6, session 20: the drop-in greedy episode's first step (cov_time_matrix_mw_kernel)
# with the predecessor LDS write under a per-edge branch (prod) against the branch-free
# write to the dummy column (build/lib_plsel, -DGF_TM_MW_PL_SELECT=1 on the tree before the
# branch-free write became the product and the switch was removed), interleaved, 8
# episodes each; the Coverage greedy tests on the variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06_s20; mkdir -p $O
for r in 1 2 3; do for v in prod plsel; do
  L=$PWD/build/lib_$v/libgymflock.so; [ $v = prod ] && L=$PWD/gym-flock_amd/lib/libgymflock.so
  GYMFLOCK_LIB=$L EPISODES=8 timeout -k 10 120 python scripts/cov_first_step_probe.py > $O/probe_${v}_$r.txt 2>&1 || exit 1
  echo "$v round $r first steps (us): $(grep 'step 0' $O/probe_${v}_$r.txt | awk '{print $5}' | tr '\n' ' ')"
done; done
GYMFLOCK_LIB=$PWD/build/lib_plsel/libgymflock.so timeout -k 10 300 python -u -m pytest tests/test_coverage_greedy_gpu.py -q --timeout 120 --timeout-method thread > $O/tests_plsel.log 2>&1; rc=$?; echo "plsel: $(tail -1 $O/tests_plsel.log)"; exit $rc
}

if [ $# -lt 1 ]; then
  echo "usage: $0 <session> [args]   sessions: r03_ab1 r03_ab2 r03_profile r03_session r03_s3 r03_s4 r03_s5 r03_s6 r03_s7 r03_s8 r03_s9 r03_s10 r03_s11 r03_s12 r03_s13 r03_s14 r03_s15 r03_s16 r03_s17 r03_s18 r03_s19 r03_s20 r03_s21 r03_s22 r03_s25 r03_s26 r03_s27 r03_s28 r03_s29 r03_s30 r03_s31 r03_s32 r03_s33 r03_s34 r03_s35 r03_s36 r03_s37 r03_s38 r03_s39 r04_final r04_profile r04_session r04_s3 r04_s4 r04_s5 r04_s7 r04_s8 r04_s9 r04_s10 r04_s11 r04_s12 r04_s13 r04_s14 r04_s15 r04_s16 r04_s17 r04_s18 r04_s19 r04_s20 r04_s21 r04_s22 r04_s23 r04_s24 r04_s25 r04_s26 r04_s27 r04_s28 r04_s29 r04_s30 r04_s31 r04_s32 r04_s33 r04_s34 r05_profile r05_s1 r05_s2 r05_s3 r05_s4 r05_s5 r05_s6 r05_s7 r05_s8 r05_s9 r05_s10 r05_s11 r05_s12 r05_s13 r05_s14 r05_s15 r05_s16 r05_s17 r05_s18 r05_s19 r05_s20 r05_s21 r05_s22 r05_s23 r05_s24 r05_s25 r05_s26 r05_s27 r06_profile_a r06_profile_b r06_s1 r06_s2 r06_s3 r06_s6 r06_s10 r06_s11 r06_s12 r06_s19 r06_s20"
  exit 2
fi
"$@"
