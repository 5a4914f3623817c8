set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r6c1_tests.txt 2>&1; rc=$?; tail -5 $O/r6c1_tests.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/r6c1_bench.json 2> $O/r6c1_bench.err; rc=$?; tail -3 $O/r6c1_bench.err; exit $rc
