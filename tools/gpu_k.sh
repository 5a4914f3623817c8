# round-4 batch K: step time with and without the per-kernel stop events (gsort_stats timing),
# and the no-stats kernel timeline
export TMPDIR=/tmp
O=gpurun_out/k_r04
mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 --warmup 3 > $O/stats$i.json 2> $O/stats$i.err || exit 1
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 20 --warmup 3 --no-stats > $O/nostats$i.json 2> $O/nostats$i.err || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/tr_nostats -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 10 --warmup 2 --no-stats > $O/tr_nostats.json 2> $O/tr_nostats.err
