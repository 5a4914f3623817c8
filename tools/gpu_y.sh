# round-4 batch Y: kernel trace of the giant-child path (16-bit keys, Zipf) at 2^28
export TMPDIR=/tmp
O=gpurun_out/y_r04
mkdir -p $O
for c in bits16 zipf; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/t_$c -o run -- python3 tools/dist_probe.py 28 $c > $O/t_$c.txt 2>&1 || exit 1
done
