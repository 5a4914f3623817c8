# A/B: A = HEAD; B = batched digit-start reads in sort_bucket (classes 1-3) and sort_bucket16
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2 3; do for L in A B; do
lib=mpi-test_amd/lib/libgsort_$L.so
GSORT_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 > $O/r6c32_$L$r.json 2> $O/r6c32_$L$r.err || { tail -5 $O/r6c32_$L$r.err; exit 1; }
GSORT_LIB=$lib timeout -k 10 120 python3 tools/dist_probe.py 28 bits30 > $O/r6c32_d$L$r.txt 2>&1 || { tail -5 $O/r6c32_d$L$r.txt; exit 1; }
GSORT_LIB=$lib timeout -k 10 120 python3 tools/recv_probe.py 28 31,30 > $O/r6c32_p$L$r.txt 2>&1 || { tail -5 $O/r6c32_p$L$r.txt; exit 1; }
python3 -c "import json;a=json.load(open('$O/r6c32_$L$r.json'));p=a['phases_ms_avg'];print('$L$r',a['value'],a['ms_per_step'],a['verified'],p['ms_level'][:2],'K11e',p['ms_bucket_sort'])"
echo "   $(grep bits30 $O/r6c32_d$L$r.txt | awk '{print "bits30 local", $2, "K11", $(NF-4)}') | recv $(grep -E 'uniform31|bits30' $O/r6c32_p$L$r.txt | awk '{print $1, $(NF-6)}' | tr '\n' ' ')"
done; done
