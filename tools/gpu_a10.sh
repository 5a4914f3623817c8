export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_a10.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_golden_large.py > gpurun_out/t_a10.log 2>&1 && \
GSORT_LIB=$L/libgsort_a11.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_a11.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_a10.so 2 local_sort_e > gpurun_out/ab_a10.txt 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_a11.so 1 local_sort_e > gpurun_out/ab_a11.txt 2>&1
