# round-4 batch U: mailbox waits query the stream every 200 us (product) vs every 1024 spins
# (GSORT_QUERY_US=0) -- tests, bench alternating, no-stats kernel timeline
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
O=gpurun_out/u_r04
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_recv.py > gpurun_out/t_u.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 30 --warmup 3 > $O/A$i.json 2> $O/A$i.err || exit 1
  GSORT_LIB=$L/libgsort_q0.so timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 30 --warmup 3 > $O/B$i.json 2> $O/B$i.err || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 10 --warmup 2 --no-stats > $O/tr.json 2> $O/tr.err
