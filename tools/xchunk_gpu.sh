# chunked-exchange check (tools/, development): the GPU suite, the multi-rank tests at 1 and 8
# chunks with GSORT_CHECK, then the forced-distributed 1-rank bench per chunk count
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu ${ALL_K:+-k "$ALL_K"} > gpurun_out/xc_all.log 2>&1 || { tail -30 gpurun_out/xc_all.log; exit 1; }
tail -1 gpurun_out/xc_all.log
for x in 1 8; do
  GSORT_XCHUNKS=$x GSORT_CHECK=1 timeout -k 10 300 $T tests/test_gpu_sort.py -k "multirank" > gpurun_out/xc_$x.log 2>&1 || { tail -30 gpurun_out/xc_$x.log; exit 1; }
  tail -1 gpurun_out/xc_$x.log
done
for x in ${BENCH_X:-1 2 4 8}; do
  GSORT_XCHUNKS=$x GSORT_FORCE_DIST=1 timeout -k 10 120 python3 bench.py --no-cpu-baseline > gpurun_out/xc_b$x.json 2>gpurun_out/xc_b$x.err || { tail gpurun_out/xc_b$x.err; exit 1; }
done
