# round-4 batch L: nontemporal partition / sort stores (GSORT_NT_STORES=1 build) against the product
export TMPDIR=/tmp
L=$PWD/mpi-test_amd/lib
GSORT_LIB=$L/libgsort_nt.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_est.py > gpurun_out/t_lnt.log 2>&1 && \
bash tools/ab_lib.sh $L/libgsort.so $L/libgsort_nt.so 3 partition_res local_sort_e > gpurun_out/abl_nt.txt 2>&1
