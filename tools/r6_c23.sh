# A/B: K11g class 3 geometry -- u32 512x33 (0), u16 512x33 (1), u16 768x22 (2); P = 2 shape
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_recv.py -x -q --timeout 120 --timeout-method thread -k "class3 or classes" > $O/r6c23_t.txt 2>&1 || { tail -5 $O/r6c23_t.txt; exit 1; }
GSORT_K11G_U16=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_recv.py -x -q --timeout 120 --timeout-method thread -k "class3 or classes" > $O/r6c23_t2.txt 2>&1 || { tail -5 $O/r6c23_t2.txt; exit 1; }
tail -1 $O/r6c23_t.txt; tail -1 $O/r6c23_t2.txt
for r in 1 2 3; do for u in 0 1 2; do
GSORT_K11G_U16=$u timeout -k 10 120 python3 tools/recv_probe.py 28 30 > $O/r6c23_p${u}_$r.txt 2>&1 || { tail -5 $O/r6c23_p${u}_$r.txt; exit 1; }
echo "rep $r body $u: $(grep bits30 $O/r6c23_p${u}_$r.txt)"
done; done
