# round-4 batch H: why reversed input is slow in K11e -- kernel trace + LDS counters per case
export TMPDIR=/tmp
O=gpurun_out/prof_r04rev
mkdir -p $O
for c in reverse sorted uniform31; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/t_$c -o run -- python3 tools/dist_probe.py 28 $c > $O/t_$c.txt 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -f csv -d $O/p_$c -o run -- python3 tools/dist_probe.py 28 $c > $O/p_$c.txt 2>&1 || exit 1
done
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_a1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_a1.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_a1.so 2 partition_res > gpurun_out/ab_a1.txt 2>&1
