set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/r6c11 -o run -- python3 tools/group_bench.py --ranks 8 --keys-log2 27 --algo sample --dist zipf --steps 2 --detail > $O/r6c11.json 2> $O/r6c11.err || { tail -5 $O/r6c11.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/r6c11.json'));print(d['median_ms_per_2p28_keys'], d['step_ms_in_order'])"
grep step $O/r6c11.err | head -16
head -15 $O/r6c11/run_kernel_stats.csv
