# packed class-3 bodies (K11e16 / K11g16): full GPU tests, then same-box A/B against the previous build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r6c24_tests.txt 2>&1; rc=$?; tail -3 $O/r6c24_tests.txt; [ $rc -ne 0 ] && exit $rc
A=mpi-test_amd/lib/libgsort_A.so; B=mpi-test_amd/lib/libgsort.so
for r in 1 2 3; do for L in A B; do
lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib timeout -k 10 120 python3 tools/dist_probe.py 28 bits30,bits29,uniform > $O/r6c24_d$L$r.txt 2>&1 || { tail -5 $O/r6c24_d$L$r.txt; exit 1; }
GSORT_LIB=$lib timeout -k 10 120 python3 tools/recv_probe.py 28 30 > $O/r6c24_p$L$r.txt 2>&1 || { tail -5 $O/r6c24_p$L$r.txt; exit 1; }
echo "== $L$r"; grep -E "bits30|bits29|uniform" $O/r6c24_d$L$r.txt; grep bits30 $O/r6c24_p$L$r.txt
done; done
