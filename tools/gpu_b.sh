# round-4 batch B: one-tile K3 A/B, K11g 10+6 on the receive shapes, IPC reopen probe
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_t1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_t1.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_t1.so 2 partition_res local_sort_e > gpurun_out/ab_t1.txt 2>&1 && \
timeout -k 10 200 python3 tools/recv_probe.py > gpurun_out/recv_base.txt 2>&1 && \
GSORT_LIB=$L/libgsort_a10.so timeout -k 10 200 python3 tools/recv_probe.py > gpurun_out/recv_a10.txt 2>&1 && \
timeout -k 10 120 tools/experiments/ipc_reopen.bin > gpurun_out/ipc_reopen.txt 2>&1
