# A/B: K1e on u16 counters, adds without return (B) vs HEAD (A)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_est.py tests/test_gpu_golden_large.py -x -q --timeout 120 --timeout-method thread > $O/r6c41_t.txt 2>&1 || { tail -5 $O/r6c41_t.txt; exit 1; }
tail -1 $O/r6c41_t.txt
for r in 1 2 3; do for L in A B; do
GSORT_LIB=mpi-test_amd/lib/libgsort_$L.so timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/r6c41_$L$r -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c41_$L$r.json 2> $O/r6c41_$L$r.err || { tail -5 $O/r6c41_$L$r.err; exit 1; }
python3 - $O/r6c41_$L$r $L$r <<'PY'
import csv, sys, glob, statistics
f = glob.glob(sys.argv[1] + '/**/run_kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
def med(pat):
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000 for r in rows if pat in r['Kernel_Name']]
    return round(statistics.median(d), 2) if d else None
print(sys.argv[2], 'K1e', med('k_est_sample'), 'K12e', med('k_est_plan'), 'K12f', med('k_est_tiles'), 'K12g', med('k_est_classify'))
PY
done; done
for L in A B; do
GSORT_LIB=mpi-test_amd/lib/libgsort_$L.so timeout -k 10 300 python3 tools/dist_probe.py 28 > $O/r6c41_d$L.txt 2>&1 || { tail -5 $O/r6c41_d$L.txt; exit 1; }
done
paste <(awk '{print $1, $2, $NF}' $O/r6c41_dA.txt) <(awk '{print $2, $NF}' $O/r6c41_dB.txt)
