# round-4 batch T: K1e / K12e level-3 sample partials bucket-major -- est tests + kernel times
export TMPDIR=/tmp
O=gpurun_out/t_r04
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_est.py tests/test_gpu_golden_large.py > gpurun_out/t_t.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/st -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 --warmup 3 > $O/st.json 2> $O/st.err
