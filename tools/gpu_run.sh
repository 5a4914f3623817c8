#!/bin/bash
# gpu_run.sh TAG STEP... -- one parametrised GPU batch (run on the GPU box from the repo root; replaces
# round 4's one-off tools/gpu_*.sh).  Every step runs under its own time limit and the batch stops at
# the first failure.  Outputs: gpurun_out/TAG_*.  Steps:
#   tests[=PATHS]      pytest -m gpu (default: all of tests/), -x, 120 s per test
#   bench              bench.py (the driver's default line) -> TAG_bench.json
#   prof               tools/profile_pmc.sh TAG (kernel trace + PMC passes of the bench configuration)
#   pipes              tools/profile_pipes.sh TAG (LDS / TA / wait counters per kernel)
#   dpipes=BITS        the same over tools/recv_probe.py 28 BITS (distributed path, one key width)
#   probe              tools/dist_probe.py (2^28 keys, every distribution)
#   recv               tools/recv_probe.py 28 (receive-sort bucket sizes)
#   group=P[:LOG2[:LIB]]  tools/group_bench.py --ranks P (P in-process ranks on one GPU)
#   ab=LIB_A:LIB_B[:REPS]  tools/ab_lib.sh A B REPS (same-box A/B of two builds)
#   smoke              __graft_entry__.smoke()
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out
for step in "$@"; do
  name=${step%%=*}; arg=${step#*=}; [ "$arg" = "$step" ] && arg=""
  echo "== $TAG $step ($(date +%T))"
  case $name in
    tests) timeout -k 10 900 python -u -m pytest ${arg:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > $O/${TAG}_tests.txt 2>&1; rc=$?; tail -3 $O/${TAG}_tests.txt ;;
    bench) timeout -k 10 400 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err; rc=$? ;;
    prof) bash tools/profile_pmc.sh $TAG --steps 5 --warmup 2 > $O/${TAG}_prof.log 2>&1; rc=$? ;;
    pipes) bash tools/profile_pipes.sh $TAG --steps 5 --warmup 2 > $O/${TAG}_pipes.log 2>&1; rc=$? ;;
    dpipes) PIPES_CMD="python3 tools/recv_probe.py 28 $arg" bash tools/profile_pipes.sh ${TAG}_d$arg > $O/${TAG}_dpipes$arg.log 2>&1; rc=$? ;;
    probe) timeout -k 10 300 python3 tools/dist_probe.py > $O/${TAG}_dist_probe.txt 2>&1; rc=$? ;;
    recv) timeout -k 10 150 python3 tools/recv_probe.py 28 > $O/${TAG}_recv_probe.txt 2>&1; rc=$? ;;
    group) IFS=: read -r P LG LIB <<< "$arg"
           GSORT_LIB=${LIB:-} timeout -k 10 200 python3 tools/group_bench.py --ranks $P --keys-log2 ${LG:-28} --steps 5 > $O/${TAG}_group$P${LIB:+_$(basename $LIB .so)}.json 2> $O/${TAG}_group$P.err; rc=$?
           tail -1 $O/${TAG}_group$P${LIB:+_$(basename $LIB .so)}.json ;;
    ab) IFS=: read -r A B R <<< "$arg"
        bash tools/ab_lib.sh $A $B ${R:-2} partition_res local_sort_e gather_sort count_expand > $O/${TAG}_ab.txt 2>&1; rc=$? ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.txt 2>&1; rc=$? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  [ $rc -ne 0 ] && { echo "step $step failed rc=$rc"; exit $rc; }
done
echo "== $TAG done ($(date +%T))"
