# round-4 batch Z: K12s as two 64-block passes; K1e whole-wave aggregated sample adds -- tests,
# giant-path kernel trace, distribution probe
export TMPDIR=/tmp
O=gpurun_out/z_r04
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_golden_large.py > gpurun_out/t_z.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/t_bits16 -o run -- python3 tools/dist_probe.py 28 bits16 > $O/t_bits16.txt 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpz.txt 2>&1
