# round-6 closing group emulation (P ranks sharing one GPU, in-process group): radix / sample at P = 2 / 4 / 8
# (2^28 keys per rank, uniform), and the configs[4] shape (8 x 2^29 Zipf keys); one JSON line each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
: > $O/r6c34_group_emulation.jsonl
for P in 2 4 8; do for A in radix sample; do
timeout -k 10 300 python3 tools/group_bench.py --ranks $P --keys-log2 28 --algo $A --steps 7 > $O/r6c34_g$A$P.json 2> $O/r6c34_g$A$P.err || { tail -5 $O/r6c34_g$A$P.err; exit 1; }
cat $O/r6c34_g$A$P.json >> $O/r6c34_group_emulation.jsonl
python3 -c "import json;d=json.load(open('$O/r6c34_g$A$P.json'));print('$A',$P,d['median_ms_per_2p28_keys'],d['step_ms_in_order'])"
done; done
for A in sample radix; do
timeout -k 10 300 python3 tools/group_bench.py --ranks 8 --keys-log2 29 --algo $A --dist zipf --steps 3 > $O/r6c34_z$A.json 2> $O/r6c34_z$A.err || { tail -5 $O/r6c34_z$A.err; exit 1; }
cat $O/r6c34_z$A.json >> $O/r6c34_group_emulation.jsonl
python3 -c "import json;d=json.load(open('$O/r6c34_z$A.json'));print('$A zipf P=8 2^29/rank', d['median_ms_per_2p28_keys'], d['step_ms_in_order'])"
done
