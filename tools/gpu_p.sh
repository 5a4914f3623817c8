# round-4 batch P: class 3 as 512 x 33 (16 896 keys) -- tests, receive probe, distribution probe,
# group emulation P = 2
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_est.py tests/test_gpu_recv.py tests/test_gpu_rccl.py > gpurun_out/t_p.log 2>&1 && \
timeout -k 10 150 python3 tools/recv_probe.py 28 > gpurun_out/rp_p.txt 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpp.txt 2>&1 && \
timeout -k 10 150 python3 tools/group_bench.py --ranks 2 --keys-log2 28 --steps 5 > gpurun_out/gp2.json 2> gpurun_out/gp2.err
