# round-4 batch F: class 3 (16 384-key buckets) as 1024 x 16 instead of 512 x 32 -- local (dist_probe
# bits30) and receive (recv_probe bits30) shapes, plus correctness of the variant
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_c3.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_recv.py > gpurun_out/t_c3.log 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 bits30,bits29,uniform31 > gpurun_out/dp_base.txt 2>&1 && \
GSORT_LIB=$L/libgsort_c3.so timeout -k 10 200 python3 tools/dist_probe.py 28 bits30,bits29,uniform31 > gpurun_out/dp_c3.txt 2>&1 && \
timeout -k 10 200 python3 tools/recv_probe.py > gpurun_out/rp_base.txt 2>&1 && \
GSORT_LIB=$L/libgsort_c3.so timeout -k 10 200 python3 tools/recv_probe.py > gpurun_out/rp_c3.txt 2>&1
