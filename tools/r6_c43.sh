# closing timeline of one 2^28-key sampled-plan sort (bench.py under rocprofv3 --kernel-trace)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $O/r6c43 -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 10 > $O/r6c43.json 2> $O/r6c43.err || { tail -5 $O/r6c43.err; exit 1; }
f=$(find $O/r6c43 -name run_kernel_trace.csv | head -1)
python3 tools/sort_timeline.py $f > $O/r6c43_timeline.txt || exit 1
cat $O/r6c43_timeline.txt
