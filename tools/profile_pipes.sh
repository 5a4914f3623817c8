#!/bin/bash
# profile_pipes.sh TAG [bench args...] -- per-kernel pipe counters of one bench configuration
# (or of PIPES_CMD, e.g. PIPES_CMD="python3 tools/recv_probe.py 28 29" for the distributed path)
# (LDS array / bank conflicts / LDS instruction mix, vector-memory instruction cycles, TA busy),
# each group its own rocprofv3 --pmc pass (MI355X_MICROARCH.md: at most 8 SQ, 2 TA, 2 GRBM
# counters per pass).  Run on the GPU box from the repo root; summary in
# gpurun_out/pipes_TAG/summary.json (tools/pmc_summary.py).
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/pipes_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=("$@")
run() {  # name, rocprof options...
    local name=$1; shift
    timeout -k 10 120 rocprofv3 "$@" -f csv -d "$OUT/$name" -o run -- \
        ${PIPES_CMD:-python3 bench.py --no-cpu-baseline --no-dist-p1 "${ARGS[@]}"} > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run stats --kernel-trace --stats
run lds --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD SQ_LDS_ADDR_CONFLICT SQ_BUSY_CU_CYCLES
run vmem --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU
run wait --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU
run ta --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json"
echo "pipes $TAG done"
