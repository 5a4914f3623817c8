set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for E in "GSORT_SAMPLE_INT32=0" "GSORT_SAMPLE_INT32=1"; do
for A in sample; do
env $E timeout -k 10 300 python3 tools/group_bench.py --ranks 8 --keys-log2 29 --algo $A --dist zipf --steps 3 > $O/r6c10_$A.json 2> $O/r6c10_$A.err || { tail -5 $O/r6c10_$A.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/r6c10_$A.json'));print('$E $A zipf P=8 2^29/rank', d['median_ms_per_2p28_keys'], d['step_ms_in_order'], d['sum_over_ranks_ms'])"
done; done
timeout -k 10 300 python3 tools/group_bench.py --ranks 8 --keys-log2 29 --algo radix --dist zipf --steps 3 > $O/r6c10_radix.json 2> $O/r6c10_radix.err || exit 1
python3 -c "import json;d=json.load(open('$O/r6c10_radix.json'));print('radix zipf P=8 2^29/rank', d['median_ms_per_2p28_keys'], d['step_ms_in_order'], d['sum_over_ranks_ms'])"
