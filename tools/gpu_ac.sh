# round-4 batch AC: K18g geometry (e1: 4096-key chunks x 512 threads; e2: + nontemporal stores)
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
for v in e1 e2; do
  GSORT_LIB=$L/libgsort_$v.so timeout -k 10 200 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_est.py -k giant > gpurun_out/t_ac_$v.log 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 120 python3 tools/dist_probe.py 28 bits16,bits8,zipf > gpurun_out/dac_A$i.txt 2>&1 || exit 1
  GSORT_LIB=$L/libgsort_e1.so timeout -k 10 120 python3 tools/dist_probe.py 28 bits16,bits8,zipf > gpurun_out/dac_B$i.txt 2>&1 || exit 1
  GSORT_LIB=$L/libgsort_e2.so timeout -k 10 120 python3 tools/dist_probe.py 28 bits16,bits8,zipf > gpurun_out/dac_C$i.txt 2>&1 || exit 1
done
