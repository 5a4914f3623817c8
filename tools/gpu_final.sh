# round-4 closing batch: every -m gpu test, the driver's bench line, the PMC profile of the
# bench configuration (tools/profile_pmc.sh), reversed / uniform K11e counters, distribution probe
export TMPDIR=/tmp
TAG=${1:-r04_v27}
L=$PWD/mpi-test_amd/lib
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
bash tools/profile_pmc.sh $TAG --steps 5 --warmup 2 > gpurun_out/${TAG}_prof.log 2>&1 && \
bash tools/gpu_h.sh
