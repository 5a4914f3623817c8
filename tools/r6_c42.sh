# A/B: K11g's direct loads with the piece deltas selected in registers (B) vs a per-key LDS read (A = HEAD);
# kernel-trace medians of the receive kernels in the P = 2 group emulation
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_recv.py tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread > $O/r6c42_t.txt 2>&1 || { tail -5 $O/r6c42_t.txt; exit 1; }
tail -1 $O/r6c42_t.txt
for r in 1 2 3; do for L in A B; do
GSORT_LIB=mpi-test_amd/lib/libgsort_$L.so timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/r6c42_$L$r -o run -- python3 tools/group_bench.py --ranks 2 --keys-log2 28 --algo radix --steps 5 > $O/r6c42_$L$r.json 2> $O/r6c42_$L$r.err || { tail -5 $O/r6c42_$L$r.err; exit 1; }
python3 - $O/r6c42_$L$r $L$r <<'PY'
import csv, sys, glob, statistics
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
def med(pat):
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000 for r in rows if pat in r['Kernel_Name']]
    return (round(statistics.median(d), 1), len(d)) if d else None
print(sys.argv[2], 'K11g16', med('k_gather_sort16'), 'K11g c2', med('k_gather_sortILi512ELi18'), 'K18c', med('k_count_expand'))
PY
done; done
