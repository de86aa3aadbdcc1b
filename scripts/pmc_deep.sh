#!/bin/bash
# Where k_eval_nb's cycles go: texture-address / L1 / scalar-cache / LDS counters of the metric bench,
# one rocprofv3 --pmc pass per counter group (block limits: 8 SQ, 4 TCP, 2 TA, 2 GRBM per pass).
# Usage (GPU box, repo root): bash scripts/pmc_deep.sh OUTDIR ["bench args"]
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_deep}
ARGS=${2:-"--steps 1 --warmup 1 --timed-only"}
mkdir -p $OUT
i=10
for CTRS in "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum" \
            "TA_ADDR_STALLED_BY_TD_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
            "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_COALESCED_READ_CYCLES_sum" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
            "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_READ_sum" \
            "SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32" \
            "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_WAVES SQ_BUSY_CYCLES" \
            "GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python scripts/pmc_summary.py $OUT > $OUT/summary.txt
echo PMC_DEEP_DONE
