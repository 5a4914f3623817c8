# round-4 batch N: nontemporal K18c window stores (GSORT_NT_CX=1) -- receive probe A/B (alternating)
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_ntcx.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_recv.py tests/test_gpu_est.py > gpurun_out/t_nntcx.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 150 python3 tools/recv_probe.py 28 > gpurun_out/rp_A$i.txt 2>&1 || exit 1
  GSORT_LIB=$L/libgsort_ntcx.so timeout -k 10 150 python3 tools/recv_probe.py 28 > gpurun_out/rp_B$i.txt 2>&1 || exit 1
done
