# round-4 batch J: est tests (dense / peaked 2^24), one-tile K3a at 80 VGPRs A/B, group emulation P = 2 / 4
# (wall time + kernel stats)
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
O=gpurun_out/grp_r04
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_j.log 2>&1 && \
GSORT_LIB=$L/libgsort_a1.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_ja1.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_a1.so 2 partition_res > gpurun_out/abj_a1.txt 2>&1 && \
for P in 2 4; do
  timeout -k 10 150 python3 tools/group_bench.py --ranks $P --keys-log2 28 --steps 5 > $O/g$P.json 2> $O/g$P.err || exit 1
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -f csv -d $O/k$P -o run -- python3 tools/group_bench.py --ranks $P --keys-log2 28 --steps 3 > $O/k$P.json 2> $O/k$P.err || exit 1
done
