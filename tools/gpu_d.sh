# round-4 batch D: K3p (pipelined persistent K3r / K3a) correctness + A/B; IPC free-vs-grow split
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_pipe.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_golden_large.py > gpurun_out/t_pipe.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_pipe.so 2 partition local_sort_e > gpurun_out/ab_pipe.txt 2>&1 ; \
for m in fresh keepgrow grow; do timeout -k 10 60 tools/experiments/ipc_group.bin 4 $m 64 >> gpurun_out/ipc_group2.txt 2>&1 || echo "P=4 $m rc=$?" >> gpurun_out/ipc_group2.txt; done
