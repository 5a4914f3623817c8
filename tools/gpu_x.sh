# round-4 batch X: K12a with 32 partial loads in flight -- exact-plan / distributed tests, receive
# probe (sender hist phase), bench dist_p1
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_sort.py tests/test_gpu_rccl.py tests/test_gpu_recv.py tests/test_gpu_configs.py > gpurun_out/t_x.log 2>&1 && \
timeout -k 10 150 python3 tools/recv_probe.py 28 > gpurun_out/rp_x.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bx.json 2> gpurun_out/bx.err
