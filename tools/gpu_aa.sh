# round-4 batch AA: K1m as a majority vote -- tests, giant-path trace, distribution probe
export TMPDIR=/tmp
O=gpurun_out/aa_r04
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_golden_large.py tests/test_gpu_configs.py > gpurun_out/t_aa.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/t_bits16 -o run -- python3 tools/dist_probe.py 28 bits16 > $O/t_bits16.txt 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpaa.txt 2>&1
