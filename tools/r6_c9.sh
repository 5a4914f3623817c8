set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for q in 4 16; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 tools/group_bench.py --ranks 4 --keys-log2 28 --algo radix --steps 8 --detail > $O/r6c9_q$q.json 2> $O/r6c9_q$q.err || exit 1
python3 -c "import json;d=json.load(open('$O/r6c9_q$q.json'));print('hwq $q',d['median_ms_per_2p28_keys'],d['step_ms_in_order'])"
done
