# A/B/C: A = HEAD; B = batched LDS reads in sort_bucket(16) + K3 scatter (packed ranks, pinned keys);
# C = B + K3 stores batched (keys, offsets, stores)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_est.py tests/test_gpu_golden_large.py tests/test_gpu_sort.py tests/test_gpu_recv.py -x -q --timeout 120 --timeout-method thread -k "not multirank_p8" > $O/r6c31_t.txt 2>&1 || { tail -5 $O/r6c31_t.txt; exit 1; }
tail -1 $O/r6c31_t.txt
for r in 1 2 3; do for L in A B C; do
lib=mpi-test_amd/lib/libgsort_$L.so
GSORT_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c31_$L$r.json 2> $O/r6c31_$L$r.err || { tail -5 $O/r6c31_$L$r.err; exit 1; }
python3 -c "import json;a=json.load(open('$O/r6c31_$L$r.json'));p=a['phases_ms_avg'];print('$L$r',a['value'],a['ms_per_step'],a['verified'],p['ms_level'][:2],'K11e',p['ms_bucket_sort'])"
done; done
