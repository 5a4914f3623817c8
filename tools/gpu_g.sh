# round-4 batch G: product with oversized children (K18c over Y), peaked-block retry, one-atomic
# K11 first pass -- tests, distribution probe and headline A/B against the round-3 library
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_recv.py tests/test_gpu_golden_large.py > gpurun_out/t_g2.log 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_new.txt 2>&1 && \
GSORT_LIB=$L/libgsort_r3.so timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_r3.txt 2>&1 && \
bash tools/ab_lib.sh $L/libgsort_r3.so $L/libgsort.so 2 local_sort_e partition_res count_expand > gpurun_out/ab_new.txt 2>&1
