set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
A=mpi-test_amd/lib/libgsort.so; B=mpi-test_amd/lib/libgsort_bperm.so
GSORT_LIB=$B timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_est.py tests/test_gpu_golden_large.py tests/test_gpu_recv.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r6c15_testsB.txt 2>&1; rc=$?; tail -2 $O/r6c15_testsB.txt; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib.sh $A $B 3 partition_res local_sort_e > $O/r6c15_ab.txt 2>&1 || { cat $O/r6c15_ab.txt; exit 1; }
cat $O/r6c15_ab.txt
for L in A B; do lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib timeout -k 10 200 python3 tools/recv_probe.py 28 31,30 > $O/r6c15_recv$L.txt 2>&1 || exit 1; echo "recv $L"; grep buckets $O/r6c15_recv$L.txt
done
for L in A B; do lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib bash tools/profile_pipes.sh r6c15_$L --steps 5 --warmup 2 > $O/r6c15_pipes$L.log 2>&1 || { tail -3 $O/r6c15_pipes$L.log; exit 1; }
done
echo done
