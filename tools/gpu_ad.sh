# round-4 batch AD: K18g 4096 x 512 with NT stores on multi-bin chunks -- giant tests + probe
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_ad.log 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpad.txt 2>&1
