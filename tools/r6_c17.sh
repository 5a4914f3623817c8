set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r6c17_tests.txt 2>&1; rc=$?; tail -3 $O/r6c17_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -f csv -d $O/r6c17_dt -o run -- python3 tools/dist_p1_trace.py radix sample > $O/r6c17_dt.log 2>&1 || exit 1
grep -E "^(radix|sample) " $O/r6c17_dt.log
for P in 2 4; do for A in radix sample; do
timeout -k 10 200 python3 tools/group_bench.py --ranks $P --keys-log2 28 --algo $A --steps 7 > $O/r6c17_g$A$P.json 2> $O/r6c17_g$A$P.err || exit 1; python3 -c "import json;d=json.load(open('$O/r6c17_g$A$P.json'));print('$A',$P,d['median_ms_per_2p28_keys'],d['step_ms_in_order'])"
done; done
for A in sample radix; do
timeout -k 10 300 python3 tools/group_bench.py --ranks 8 --keys-log2 29 --algo $A --dist zipf --steps 3 > $O/r6c17_z$A.json 2> $O/r6c17_z$A.err || { tail -5 $O/r6c17_z$A.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/r6c17_z$A.json'));print('$A zipf P=8 2^29/rank', d['median_ms_per_2p28_keys'], d['step_ms_in_order'])"
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/r6c17_bench.json 2> $O/r6c17_bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/r6c17_bench.json'));print(d['value'],d['ms_per_step'],[(k,d[k]['ms_per_step'],d[k]['phases_ms_avg']['ms_total'],d[k]['receive_sort']['ms']) for k in ('dist_p1','dist_p1_sample')])"
