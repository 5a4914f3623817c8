set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/r6c2_kb -o run -- ./tools/bin/kernel_boundary > $O/r6c2_kb.log 2>&1 || exit 1
python3 tools/boundary_gaps.py $O/r6c2_kb/run_kernel_trace.csv > $O/r6c2_kb_gaps.txt 2>&1; cat $O/r6c2_kb_gaps.txt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -f csv -d $O/r6c2_dt -o run -- python3 tools/dist_p1_trace.py radix sample > $O/r6c2_dt.log 2>&1 || exit 1
grep -E "^(radix|sample) " $O/r6c2_dt.log
for L in 28; do for P in 2 4; do
  timeout -k 10 200 python3 tools/group_bench.py --ranks $P --keys-log2 $L --algo sample --steps 5 > $O/r6c2_gs$P.json 2> $O/r6c2_gs$P.err || exit 1; tail -1 $O/r6c2_gs$P.json
  timeout -k 10 200 python3 tools/group_bench.py --ranks $P --keys-log2 $L --algo radix --steps 5 > $O/r6c2_gr$P.json 2> $O/r6c2_gr$P.err || exit 1; tail -1 $O/r6c2_gr$P.json
done; done
timeout -k 10 200 python3 tools/group_bench.py --ranks 8 --keys-log2 27 --algo sample --steps 5 > $O/r6c2_gs8.json 2> $O/r6c2_gs8.err || exit 1; tail -1 $O/r6c2_gs8.json
