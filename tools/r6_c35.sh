# same-box check of the P-rank group emulation: A = v38 code (f3b1992), B = this build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
for r in 1 2; do for L in A B; do for P in 2 4; do for A in radix sample; do
lib=mpi-test_amd/lib/libgsort.so; [ $L = A ] && lib=mpi-test_amd/lib/libgsort_A.so
GSORT_LIB=$lib timeout -k 10 300 python3 tools/group_bench.py --ranks $P --keys-log2 28 --algo $A --steps 7 > $O/r6c35_$L$r$A$P.json 2> $O/r6c35_$L$r$A$P.err || { tail -5 $O/r6c35_$L$r$A$P.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/r6c35_$L$r$A$P.json'));print('$L$r $A P=$P',d['median_ms_per_2p28_keys'],d['step_ms_in_order'])"
done; done; done; done
