# A/B: K11e class 2 (the headline's dominant kernel) on the packed body (GSORT_EXP_C2U16) vs sort_bucket
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
GSORT_EXP_C2U16=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_est.py tests/test_gpu_golden_large.py -x -q --timeout 120 --timeout-method thread > $O/r6c28_t.txt 2>&1 || { tail -5 $O/r6c28_t.txt; exit 1; }
tail -1 $O/r6c28_t.txt
for r in 1 2 3; do for u in 0 1; do
if [ $u = 1 ]; then export GSORT_EXP_C2U16=1; else unset GSORT_EXP_C2U16; fi
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c28_b${u}_$r.json 2> $O/r6c28_b${u}_$r.err || { tail -5 $O/r6c28_b${u}_$r.err; exit 1; }
python3 -c "import json;a=json.load(open('$O/r6c28_b${u}_$r.json'));p=a['phases_ms_avg'];print('rep $r packed $u',a['value'],a['ms_per_step'],a['verified'],p['ms_level'][:2],'K11e',p['ms_bucket_sort'])"
done; done
