# K11g with global-address run loads + packed class 3: receive tests, then kernel-level A/B (A = previous build)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_recv.py tests/test_gpu_sort.py tests/test_gpu_est.py -x -q --timeout 120 --timeout-method thread > $O/r6c26_t.txt 2>&1 || { tail -5 $O/r6c26_t.txt; exit 1; }
tail -1 $O/r6c26_t.txt
A=mpi-test_amd/lib/libgsort_A.so; B=mpi-test_amd/lib/libgsort.so
for r in 1 2 3; do for L in A B; do
lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/r6c26_$L$r -o run -- python3 tools/recv_probe.py 28 31,30 > $O/r6c26_$L$r.log 2>&1 || { tail -5 $O/r6c26_$L$r.log; exit 1; }
python3 - $O/r6c26_$L$r $L$r <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
g = [(r['Kernel_Name'].split('(')[0].split('::')[-1][:40], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000) for r in rows if 'gather_sort' in r['Kernel_Name']]
# 6 calls per shape (1 + 5), shapes in order 31 then 30: last 3 of each
print(sys.argv[2], '8192-key:', g[0][0], [round(d, 1) for _, d in g[3:6]], ' 16384-key:', g[6][0], [round(d, 1) for _, d in g[9:12]])
PY
done; done
