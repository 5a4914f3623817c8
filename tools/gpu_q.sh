# round-4 batch Q: sampled children of class 4 (16 897 .. 32 768 keys) to K18c (GSORT_EST_CX=4) vs K11e
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_ecx.so timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_qecx.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dq_A$i.txt 2>&1 || exit 1
  GSORT_LIB=$L/libgsort_ecx.so timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dq_B$i.txt 2>&1 || exit 1
done
