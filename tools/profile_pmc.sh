#!/bin/bash
# profile_pmc.sh TAG [bench args...] -- rocprofv3 evidence for one bench configuration.
# Run on the GPU box from the repo root.  Writes gpurun_out/prof_TAG/{stats,fetch,write,sq,...}
# and summarises them into gpurun_out/prof_TAG/summary.json (tools/pmc_summary.py).
# Each counter group is its own run (MI355X_MICROARCH.md: rocprofv3 PMC slots; never --pmc
# together with a runtime/sys trace).
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=("$@")
run() {  # name, rocprof options...
    local name=$1; shift
    timeout -k 10 120 rocprofv3 "$@" -f csv -d "$OUT/$name" -o run -- \
        python3 bench.py --no-cpu-baseline --no-dist-p1 "${ARGS[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run stats --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS
run clk --pmc GRBM_GUI_ACTIVE GRBM_COUNT
# peer (xGMI) evidence for the exchange: EA requests that did not go to local DRAM
# (TCC_EA0_RDREQ - TCC_EA0_RDREQ_DRAM, TCC_EA0_WRREQ - TCC_EA0_WRREQ_DRAM)
run xgmi --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json"
echo "profile $TAG done"
