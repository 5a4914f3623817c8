# round-4 batch W: group emulation P = 4 repeated (noise check after the mailbox-poll change)
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 150 python3 tools/group_bench.py --ranks 4 --keys-log2 28 --steps 5 > gpurun_out/gw4_$i.json 2> gpurun_out/gw4_$i.err || exit 1
done
timeout -k 10 150 python3 tools/group_bench.py --ranks 2 --keys-log2 28 --steps 5 > gpurun_out/gw2.json 2> gpurun_out/gw2.err
