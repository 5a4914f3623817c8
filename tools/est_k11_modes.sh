# K11e experiment (development): kernel times per GSORT_EST_K11 mode (bit 0 store in place in
# y, bit 1 one workgroup per possible entry) and the exact plan (GSORT_EST=0) for reference
export TMPDIR=/tmp
for m in ${MODES:-0 1 2 3 x}; do
  if [ $m = x ]; then E="GSORT_EST=0"; else E="GSORT_EST_K11=$m"; fi
  env $E true
  if [ $m = x ]; then export GSORT_EST=0; else export GSORT_EST_K11=$m; unset GSORT_EST; fi
  timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d gpurun_out/k11m$m -o run -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/k11m$m.json 2>gpurun_out/k11m$m.err
  echo "== mode $m rc=$?"
  python3 tools/kernel_grid.py gpurun_out/k11m$m/run_kernel_trace.csv "local_sort"
done
