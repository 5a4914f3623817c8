set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_recv.py tests/test_gpu_configs.py tests/test_gpu_rccl.py tests/test_gpu_sort.py tests/test_gpu_golden_large.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r6c16_tests.txt 2>&1; rc=$?; tail -2 $O/r6c16_tests.txt; [ $rc -ne 0 ] && exit $rc
for A in sample radix; do
timeout -k 10 300 python3 tools/group_bench.py --ranks 8 --keys-log2 29 --algo $A --dist zipf --steps 3 > $O/r6c16_$A.json 2> $O/r6c16_$A.err || { tail -5 $O/r6c16_$A.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/r6c16_$A.json'));print('$A zipf P=8 2^29/rank', d['median_ms_per_2p28_keys'], d['step_ms_in_order'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/r6c16 -o run -- python3 tools/group_bench.py --ranks 8 --keys-log2 27 --algo sample --dist zipf --steps 2 > $O/r6c16.json 2> $O/r6c16.err || { tail -5 $O/r6c16.err; exit 1; }
