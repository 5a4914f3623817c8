# untimed (no per-kernel events) local sort: step time and the call-boundary gap
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c18_t$r.json 2> $O/r6c18_t$r.err || exit 1
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 --no-stats > $O/r6c18_u$r.json 2> $O/r6c18_u$r.err || exit 1
python3 -c "import json;a=json.load(open('$O/r6c18_t$r.json'));b=json.load(open('$O/r6c18_u$r.json'));print('timed',a['ms_per_step'],'untimed',b['ms_per_step'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace -f csv -d $O/r6c18_tr -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 --no-stats > $O/r6c18_tr.log 2>&1 || exit 1
f=$(ls $O/r6c18_tr/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls $O/r6c18_tr/run_kernel_trace.csv)
python3 tools/step_timeline.py ${f%_kernel_trace.csv} k_est_sample > $O/r6c18_timeline.txt 2>&1 || exit 1
cat $O/r6c18_timeline.txt | head -40
