# round-4 batch V: end-of-call event sync (B) vs stream sync (A)
# -- bench alternating
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
O=gpurun_out/v_r04
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_recv.py > gpurun_out/t_v.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 30 --warmup 3 > $O/A$i.json 2> $O/A$i.err || exit 1
  GSORT_LIB=$L/libgsort_evd.so timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 30 --warmup 3 > $O/B$i.json 2> $O/B$i.err || exit 1
done
