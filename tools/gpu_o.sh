# round-4 batch O: giant path with per-workgroup cold segments (no per-tile barriers) and the
# two-candidate skew aggregation -- tests + distribution probe
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_golden_large.py > gpurun_out/t_o.log 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpo.txt 2>&1
