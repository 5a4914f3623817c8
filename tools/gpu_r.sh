# round-4 batch R: end-of-call spin on a stream-written mailbox word (GSORT_SPIN_DONE=1) vs
# hipStreamSynchronize alone -- bench step time, alternating, no profiler
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
O=gpurun_out/r_r04
mkdir -p $O
GSORT_LIB=$L/libgsort_spin.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py > gpurun_out/t_rspin.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 30 --warmup 3 > $O/A$i.json 2> $O/A$i.err || exit 1
  GSORT_LIB=$L/libgsort_spin.so timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 30 --warmup 3 > $O/B$i.json 2> $O/B$i.err || exit 1
done
