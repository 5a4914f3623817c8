# A/B: K11g class 3 on the packed u16 body (sort_bucket16) vs the u32 body, P = 2 shapes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2 3; do for u in 0 1; do
GSORT_K11G_U16=$u timeout -k 10 120 python3 tools/recv_probe.py 28 30 > $O/r6c22_p${u}_$r.txt 2>&1 || { tail -5 $O/r6c22_p${u}_$r.txt; exit 1; }
echo "rep $r u16 $u: $(grep bits30 $O/r6c22_p${u}_$r.txt)"
done; done
for r in 1 2; do for u in 0 1; do for A in radix sample; do
GSORT_K11G_U16=$u timeout -k 10 200 python3 tools/group_bench.py --ranks 2 --keys-log2 28 --algo $A --steps 7 > $O/r6c22_g${A}${u}_$r.json 2> $O/r6c22_g${A}${u}_$r.err || { tail -5 $O/r6c22_g${A}${u}_$r.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/r6c22_g${A}${u}_$r.json'));print('rep $r u16 $u $A P=2',d['median_ms_per_2p28_keys'],d['step_ms_in_order'])"
done; done; done
