# round-4 batch G (combined): product tests (oversized children, peaked retry), padded-LDS K11
# variant (tests, distribution probe, headline A/B), reversed-input kernel trace, one-tile K3a A/B
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_PLAN_TRACE=1 timeout -k 10 200 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread "tests/test_gpu_est.py::test_giant_child_counted" > gpurun_out/t_trace.log 2>&1; rc=$?; [ $rc -le 1 ] && \
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_recv.py tests/test_gpu_golden_large.py > gpurun_out/t_g2.log 2>&1; rc=$?; [ $rc -le 1 ] && \
GSORT_LIB=$L/libgsort_pad.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_recv.py > gpurun_out/t_pad.log 2>&1; rc=$?; [ $rc -le 1 ] && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_new.txt 2>&1 && \
GSORT_LIB=$L/libgsort_pad.so timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_pad.txt 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_pad.so 2 local_sort_e count_expand > gpurun_out/ab_pad.txt 2>&1 && \
mkdir -p gpurun_out/prof_r04rev && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r04rev/t_reverse -o run -- python3 tools/dist_probe.py 28 reverse > gpurun_out/prof_r04rev/t_reverse.txt 2>&1 && \
GSORT_LIB=$L/libgsort_a1.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_a1.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_a1.so 1 partition_res > gpurun_out/ab_a1.txt 2>&1
