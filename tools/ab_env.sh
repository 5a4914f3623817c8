# Same-box A/B of library settings (development): ab_env.sh REPS "ENV_A" "ENV_B" ... -- [pattern ...]
# Alternates bench.py runs (A B .. A B ..) under rocprofv3 --kernel-trace, one per environment
# string per repetition, and prints each run's GKeys/s / ms per step plus the median duration
# of every kernel matching the patterns (tools/kernel_grid.py).  AB_BENCH_ARGS adds bench flags.
export TMPDIR=/tmp
R=$1; shift
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "$1" = "--" ] && shift
EXTRA=${AB_BENCH_ARGS:-}
for i in $(seq 1 $R); do
  j=0
  for E in "${ENVS[@]}"; do
    j=$((j+1))
    d=gpurun_out/abenv_${j}_$i
    env $E timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $d -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 10 --warmup 2 $EXTRA > $d.json 2>$d.err || { echo "run [$E] $i failed"; grep -v "rocprofv3\]\|output_stream\|simple_timer" $d.err | tail -60; exit 1; }
    echo "== [$E] rep $i: $(python3 -c "import json; d=json.load(open('$d.json')); print(d['value'], 'GKeys/s', d['ms_per_step'], 'ms', d['local_plan'], 'verified', d['verified'])")"
    python3 tools/kernel_grid.py $d/run_kernel_trace.csv "$@" | paste - - | sed "s/(unsigned.*median/ median/" | awk '{print "   ", $0}'
  done
done
