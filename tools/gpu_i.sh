# round-4 batch I: product tests (K1e wrap-flag fix), padded-LDS K11 with hoisted read
# addresses (tests, distribution probe, headline A/B), one-tile K3a A/B
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_recv.py tests/test_gpu_golden_large.py > gpurun_out/t_i.log 2>&1; rc=$?; [ $rc -le 1 ] && \
GSORT_LIB=$L/libgsort_pad.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_recv.py > gpurun_out/t_ipad.log 2>&1; rc=$?; [ $rc -le 1 ] && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpi_new.txt 2>&1 && \
GSORT_LIB=$L/libgsort_pad.so timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpi_pad.txt 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_pad.so 3 local_sort_e count_expand > gpurun_out/abi_pad.txt 2>&1 && \
GSORT_LIB=$L/libgsort_a1.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_ia1.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_a1.so 2 partition_res > gpurun_out/abi_a1.txt 2>&1
