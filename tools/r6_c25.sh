# kernel-level A/B of K11g class 3 (previous build A vs packed body B), P = 2 shape
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
A=mpi-test_amd/lib/libgsort_A.so; B=mpi-test_amd/lib/libgsort.so
for r in 1 2 3; do for L in A B; do
lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/r6c25_$L$r -o run -- python3 tools/recv_probe.py 28 30 > $O/r6c25_$L$r.log 2>&1 || { tail -5 $O/r6c25_$L$r.log; exit 1; }
f=$(find $O/r6c25_$L$r -name 'run_kernel_stats.csv' | head -1)
echo "== $L$r $(grep -E 'gather_sort' $f | awk -F, '{printf "%s calls %s avg %.1f us; ", substr($1,1,60), $3, $5/1000}')"
done; done
