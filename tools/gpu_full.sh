# full GPU check: every -m gpu test, then the driver's bench line (run from the repo root on the GPU box)
export TMPDIR=/tmp
TAG=${1:-r04}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
