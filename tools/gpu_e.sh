# round-4 batch E: K3p variants -- single-tile units at 2 WGs per CU (pipe1), late next-pair loads (pipe2)
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_pipe1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_pipe1.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_pipe1.so 2 partition > gpurun_out/ab_pipe1.txt 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_pipe2.so 1 partition > gpurun_out/ab_pipe2.txt 2>&1
