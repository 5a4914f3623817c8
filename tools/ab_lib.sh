# Same-box A/B of two library builds (development): ab_lib.sh LIB_A LIB_B [reps] [pattern ...]
# Alternates bench.py runs under rocprofv3 --kernel-trace with GSORT_LIB=A / B (A B A B ...) and
# prints each run's GKeys/s and the median duration of every kernel matching the patterns.
# Build B = the working tree (make -C mpi-test_amd); A = e.g. a build of the previous commit:
#   git worktree add /tmp/wa HEAD~1 && make -C /tmp/wa/mpi-test_amd lib && cp /tmp/wa/mpi-test_amd/lib/libgsort.so mpi-test_amd/lib/libgsort_A.so  (A/B builds live beside the product in lib/ and are deleted after use: tools/ab/ is gpurun-ignored)
# AB_PLAIN=1: plain bench.py runs (no profiler; the step time as the driver sees it), 20 steps.
export TMPDIR=/tmp
A=$1; B=$2; R=${3:-2}; shift 3
EXTRA=${AB_BENCH_ARGS:-}
for i in $(seq 1 $R); do
  for L in A B; do
    lib=$A; [ $L = B ] && lib=$B
    d=gpurun_out/ablib_$L$i
    if [ -n "${AB_PLAIN:-}" ]; then
      GSORT_LIB=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 --warmup 3 $EXTRA > $d.json 2>$d.err || { echo "run $L$i failed"; grep -v "rocprofv3\]\|output_stream\|simple_timer" $d.err | tail -60; exit 1; }
    else
      GSORT_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $d -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 10 --warmup 2 $EXTRA > $d.json 2>$d.err || { echo "run $L$i failed"; grep -v "rocprofv3\]\|output_stream\|simple_timer" $d.err | tail -60; exit 1; }
    fi
    echo "== $L$i $(python3 -c "import json; d=json.load(open('$d.json')); print(d['value'], 'GKeys/s', d['ms_per_step'], 'ms', d['local_plan'])")"
    [ -n "${AB_PLAIN:-}" ] || python3 tools/kernel_grid.py $d/run_kernel_trace.csv "$@" | paste - - | sed "s/(unsigned.*median/ median/" | awk '{print "   ", $0}'
  done
done
