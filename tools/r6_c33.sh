# A/B: K3r / K3a ranks with the aggregated LDS atomics issued back to back (agg_rank_issue / _done, B)
# vs one wait per atomic (A = HEAD)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_est.py tests/test_gpu_golden_large.py tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread > $O/r6c33_t.txt 2>&1 || { tail -5 $O/r6c33_t.txt; exit 1; }
tail -1 $O/r6c33_t.txt
for r in 1 2 3 4; do for L in A B; do
lib=mpi-test_amd/lib/libgsort_$L.so
GSORT_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c33_$L$r.json 2> $O/r6c33_$L$r.err || { tail -5 $O/r6c33_$L$r.err; exit 1; }
python3 -c "import json;a=json.load(open('$O/r6c33_$L$r.json'));p=a['phases_ms_avg'];print('$L$r',a['value'],a['ms_per_step'],a['verified'],p['ms_level'][:2],'K11e',p['ms_bucket_sort'])"
done; done
for L in A B; do
GSORT_LIB=mpi-test_amd/lib/libgsort_$L.so timeout -k 10 200 python3 tools/dist_probe.py 28 sorted,zipf,bits16 > $O/r6c33_d$L.txt 2>&1 || { tail -5 $O/r6c33_d$L.txt; exit 1; }
echo "$L"; grep -E "^(sorted|zipf|bits16)" $O/r6c33_d$L.txt
done
