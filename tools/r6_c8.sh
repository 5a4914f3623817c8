set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for i in 1 2; do
timeout -k 10 200 python3 tools/group_bench.py --ranks 4 --keys-log2 28 --algo radix --steps 8 --detail > $O/r6c8_g4r$i.json 2> $O/r6c8_g4r$i.err || exit 1
python3 -c "import json;d=json.load(open('$O/r6c8_g4r$i.json'));print(d['step_ms_in_order'])"
done
