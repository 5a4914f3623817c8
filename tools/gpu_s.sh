# round-4 batch S: class-4 children of shifted plans back on K11e -- est tests + distribution probe
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_s.log 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dps.txt 2>&1
