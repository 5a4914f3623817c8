# round-4 batch C: wave-time breakdown of the sort kernels (SQ wait / issue / active), P-process IPC probe
export TMPDIR=/tmp
O=gpurun_out/prof_r04wait
mkdir -p $O
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -f csv -d $O/w -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 4 --warmup 1 > $O/w.json 2> $O/w.err && \
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -f csv -d $O/i -o run -- python3 bench.py --no-cpu-baseline --no-dist-p1 --steps 4 --warmup 1 > $O/i.json 2> $O/i.err && \
python3 tools/pmc_summary.py $O > $O/summary.json; \
for P in 4 8; do for m in reexport grow once; do timeout -k 10 120 tools/experiments/ipc_group.bin $P $m 200 >> gpurun_out/ipc_group.txt 2>&1 || echo "P=$P $m rc=$?" >> gpurun_out/ipc_group.txt; done; done
