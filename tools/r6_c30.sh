# A/B: sort_bucket scatters -- every digit start read (unpredicated) before any key is written -- and K3 stores: keys, offsets, then stores (B) vs interleaved (A = HEAD)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_est.py tests/test_gpu_golden_large.py -x -q --timeout 120 --timeout-method thread > $O/r6c30_t.txt 2>&1 || { tail -5 $O/r6c30_t.txt; exit 1; }
tail -1 $O/r6c30_t.txt
A=mpi-test_amd/lib/libgsort_A.so; B=mpi-test_amd/lib/libgsort.so
for r in 1 2 3 4; do for L in A B; do
lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c30_$L$r.json 2> $O/r6c30_$L$r.err || { tail -5 $O/r6c30_$L$r.err; exit 1; }
python3 -c "import json;a=json.load(open('$O/r6c30_$L$r.json'));p=a['phases_ms_avg'];print('$L$r',a['value'],a['ms_per_step'],a['verified'],p['ms_level'][:2],'K11e',p['ms_bucket_sort'])"
done; done
for r in 1 2; do for L in A B; do
lib=$A; [ $L = B ] && lib=$B
GSORT_LIB=$lib timeout -k 10 120 python3 tools/recv_probe.py 28 31,30 > $O/r6c30_p$L$r.txt 2>&1 || { tail -5 $O/r6c30_p$L$r.txt; exit 1; }
echo "$L$r $(grep -E 'uniform31|bits30' $O/r6c30_p$L$r.txt | awk '{print $1, $(NF-6)}' | tr '\n' ' ')"
done; done
