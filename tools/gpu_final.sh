# round-4 closing batch: every -m gpu test, the driver's bench line, the PMC profile of the
# bench configuration (tools/profile_pmc.sh), reversed / uniform K11e counters + distribution
# probe (tools/gpu_h.sh), receive probe and group emulation P = 2 / 4
export TMPDIR=/tmp
TAG=${1:-r04_v28}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
bash tools/profile_pmc.sh $TAG --steps 5 --warmup 2 > gpurun_out/${TAG}_prof.log 2>&1 && \
bash tools/gpu_h.sh && \
timeout -k 10 150 python3 tools/recv_probe.py 28 > gpurun_out/${TAG}_recv_probe.txt 2>&1 && \
for P in 2 4; do
  timeout -k 10 150 python3 tools/group_bench.py --ranks $P --keys-log2 28 --steps 5 > gpurun_out/${TAG}_group$P.json 2> gpurun_out/${TAG}_group$P.err || exit 1
done
