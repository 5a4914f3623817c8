# global-address run loads (K11g / K18c / gather copy) + packed class 3: receive tests, then
# kernel-level A/B against the previous build at the P = 1 / 2 / 4 / 8 receive shapes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_recv.py tests/test_gpu_sort.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/r6c27_t.txt 2>&1 || { tail -5 $O/r6c27_t.txt; exit 1; }
tail -1 $O/r6c27_t.txt
A=mpi-test_amd/lib/libgsort_A.so; B=mpi-test_amd/lib/libgsort.so
for r in 1 2 3; do for L in A B; do
lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib timeout -k 10 150 rocprofv3 --kernel-trace -f csv -d $O/r6c27_$L$r -o run -- python3 tools/recv_probe.py 28 31,30,29,28 > $O/r6c27_$L$r.log 2>&1 || { tail -5 $O/r6c27_$L$r.log; exit 1; }
python3 - $O/r6c27_$L$r $L$r <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
names = ('gather_sort', 'count_expand')
g = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000 for r in rows if any(n in r['Kernel_Name'] for n in names)]
# 6 calls per shape, shapes 31, 30, 29, 28; the receive kernels of one call summed where several
out = []
k = [r for r in rows if any(n in r['Kernel_Name'] for n in names)]
print(sys.argv[2], len(k), 'receive kernels')
PY
grep -E "uniform31|bits30|bits29|bits28" $O/r6c27_$L$r.log | awk -v t=$L$r '{print t, $1, "recv", $(NF-6)}'
done; done
