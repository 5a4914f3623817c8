# round-4 batch H: reversed- and uniform-input kernel traces + LDS counters of the padded K11e
export TMPDIR=/tmp
O=gpurun_out/prof_r04rev
mkdir -p $O
for c in reverse uniform31; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/t_$c -o run -- python3 tools/dist_probe.py 28 $c > $O/t_$c.txt 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -f csv -d $O/p_$c -o run -- python3 tools/dist_probe.py 28 $c > $O/p_$c.txt 2>&1 || exit 1
done
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_final.txt 2>&1
