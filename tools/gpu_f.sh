# round-4 batch F: (c3) class 3 as 1024 x 16 instead of 512 x 32; (g) peaked blocks: eligibility at
# estimate + 4 sigma with clamped regions, offset retry when the first sample's counters wrapped;
# (one) g + one LDS atomic per thread in K11's first pass when every thread's keys share a digit
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_one.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py > gpurun_out/t_one.log 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_base.txt 2>&1 && \
GSORT_LIB=$L/libgsort_g.so timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_g.txt 2>&1 && \
GSORT_LIB=$L/libgsort_one.so timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_one.txt 2>&1 && \
GSORT_LIB=$L/libgsort_c3.so timeout -k 10 200 python3 tools/dist_probe.py 28 bits30,bits29,uniform31 > gpurun_out/dp_c3.txt 2>&1 && \
timeout -k 10 200 python3 tools/recv_probe.py > gpurun_out/rp_base.txt 2>&1 && \
GSORT_LIB=$L/libgsort_c3.so timeout -k 10 200 python3 tools/recv_probe.py > gpurun_out/rp_c3.txt 2>&1
