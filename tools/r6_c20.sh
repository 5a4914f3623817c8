# experiment: sampled plan shifted by 1 bit on 31-bit uniform keys (children 4096 keys, 15 bits)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do for sb in 0 1; do
GSORT_EXP_SB=$sb timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c20_s${sb}_$r.json 2> $O/r6c20_s${sb}_$r.err || { tail -5 $O/r6c20_s${sb}_$r.err; exit 1; }
python3 -c "import json;a=json.load(open('$O/r6c20_s${sb}_$r.json'));p=a['phases_ms_avg'];print('sb $sb',a['ms_per_step'],a['verified'],a['local_plan'],p['ms_hist'],p['ms_level'][:2],p['ms_bucket_sort'])"
done; done
