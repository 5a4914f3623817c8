# one round-closing GPU batch: tests, the driver's bench line, rocprofv3 kernel stats + PMC, smoke
set -o pipefail
export TMPDIR=/tmp
T=${1:-v37}
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_tests.txt 2>&1; rc=$?; tail -3 $O/${T}_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -5 $O/${T}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/${T}_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel'][:40],[(k,d[k]['ms_per_step']) for k in ('dist_p1','dist_p1_sample')])"
bash tools/profile_pmc.sh $T --steps 5 --warmup 2 > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.txt 2>&1 || { tail -5 $O/${T}_smoke.txt; exit 1; }
tail -2 $O/${T}_smoke.txt
