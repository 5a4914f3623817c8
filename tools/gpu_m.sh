# round-4 batch M: product with NT final stores (class >= 2) -- tests + A/B against the v27-era
# build (r3 lib is older; compare with ab of NT loads variant), and NT key loads variant
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_sort.py tests/test_gpu_recv.py tests/test_gpu_golden_large.py > gpurun_out/t_m.log 2>&1 && \
GSORT_LIB=$L/libgsort_ntl.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_mntl.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_ntl.so 3 partition_res local_sort_e est_sample > gpurun_out/abm_ntl.txt 2>&1 && \
timeout -k 10 200 python3 tools/dist_probe.py 28 > gpurun_out/dpm.txt 2>&1
