set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 python3 tools/recv_probe.py 28 > $O/r6c6_recv_probe.txt 2>&1 || exit 1
cat $O/r6c6_recv_probe.txt | grep buckets
for B in 30 29; do
PIPES_CMD="python3 tools/recv_probe.py 28 $B" bash tools/profile_pipes.sh r6c6_d$B > $O/r6c6_dpipes$B.log 2>&1 || { tail -5 $O/r6c6_dpipes$B.log; exit 1; }
done
echo done
