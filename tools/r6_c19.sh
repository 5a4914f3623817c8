# experiment: back-to-back untimed local sorts with and without the per-call stream sync
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2 3; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 40 --no-stats > $O/r6c19_u$r.json 2> $O/r6c19_u$r.err || exit 1
GSORT_ASYNC_EXP=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 40 --no-stats > $O/r6c19_a$r.json 2> $O/r6c19_a$r.err || { tail -5 $O/r6c19_a$r.err; exit 1; }
python3 -c "import json;a=json.load(open('$O/r6c19_u$r.json'));b=json.load(open('$O/r6c19_a$r.json'));print('sync',a['ms_per_step'],a['verified'],'async',b['ms_per_step'],b['verified'])"
done
