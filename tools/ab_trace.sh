# Same-box A/B of kernel times (development): ab_trace.sh "ENV_A" "ENV_B" [pattern ...]
# Runs bench.py under rocprofv3 --kernel-trace once per environment and prints the median
# duration of every kernel matching the patterns.
export TMPDIR=/tmp
A=$1; B=$2; shift 2
i=0
for E in "$A" "$B"; do
  i=$((i+1))
  env $E timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d gpurun_out/ab$i -o run -- python3 bench.py --no-cpu-baseline --steps 8 --warmup 2 > gpurun_out/ab$i.json 2>gpurun_out/ab$i.err || { echo "run $i failed"; tail -5 gpurun_out/ab$i.err; exit 1; }
  echo "== [$E] $(python3 -c "import json; d=json.load(open('gpurun_out/ab$i.json')); print(d['value'], 'GKeys/s', d['ms_per_step'], 'ms')")"
  python3 tools/kernel_grid.py gpurun_out/ab$i/run_kernel_trace.csv "$@" | paste - - | sed "s/(unsigned.*median/ median/"
done
