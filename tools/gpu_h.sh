# round-4 batch H: reversed-input K11e (kernel trace + LDS counters), padded K11 LDS key array
# (pad) and one-tile K3a (a1) against the product
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
O=gpurun_out/prof_r04rev
mkdir -p $O
for c in reverse uniform31; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/t_$c -o run -- python3 tools/dist_probe.py 28 $c > $O/t_$c.txt 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -f csv -d $O/p_$c -o run -- python3 tools/dist_probe.py 28 $c > $O/p_$c.txt 2>&1 || exit 1
done
GSORT_LIB=$L/libgsort_pad.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_recv.py > gpurun_out/t_pad.log 2>&1 && \
GSORT_LIB=$L/libgsort_pad.so timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dp_pad.txt 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_pad.so 2 local_sort_e > gpurun_out/ab_pad.txt 2>&1 && \
GSORT_LIB=$L/libgsort_a1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_a1.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_a1.so 2 partition_res > gpurun_out/ab_a1.txt 2>&1
