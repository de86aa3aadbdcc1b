#!/bin/bash
# PMC passes over the bench (run on the GPU box from the repo root).  Each pass is its own
# rocprofv3 invocation with --pmc only (no trace domains combined with counters).
# Usage: bash scripts/pmc.sh OUTDIR ["bench args"]; then scripts/pmc_summary.py OUTDIR --json ...
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
ARGS=${2:-"--steps 1 --warmup 0 --no-cpu-baseline --no-variant --no-pipeline"}
mkdir -p $OUT
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_THREAD_CYCLES_VALU" \
            "TCC_HIT TCC_MISS" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
            "GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS --no-clock > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
echo PMC_DONE
