set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/r6c7_kb -o run -- ./tools/bin/kernel_boundary > $O/r6c7_kb.log 2>&1 || exit 1
python3 tools/boundary_gaps.py $O/r6c7_kb/run_kernel_trace.csv > $O/r6c7_kb_gaps.txt 2>&1; cat $O/r6c7_kb_gaps.txt
for i in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 > $O/r6c7_bs$i.json 2>/dev/null || exit 1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --no-stats > $O/r6c7_bn$i.json 2>/dev/null || exit 1
python3 -c "import json;a=json.load(open('$O/r6c7_bs$i.json'));b=json.load(open('$O/r6c7_bn$i.json'));print('stats',a['ms_per_step'],'no-stats',b['ms_per_step'])"
done
