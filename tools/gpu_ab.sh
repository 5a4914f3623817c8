# round-4 batch AB: K1g atomics without a per-item branch -- giant tests, 16-bit kernel trace, probe
export TMPDIR=/tmp
O=gpurun_out/ab_r04
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_golden_large.py > gpurun_out/t_ab.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/t_bits16 -o run -- python3 tools/dist_probe.py 28 bits16,zipf > $O/t_bits16.txt 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpab.txt 2>&1
