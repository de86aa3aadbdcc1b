#!/bin/bash
# Instruction-cache behaviour of the bench's kernels (one --pmc pass).  Usage: bash scripts/r03_icache_pmc.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-icache}
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/p -o run -- python3 bench.py --steps 1 --warmup 1 --timed-only --no-cpu-baseline --no-variant --no-pipeline --no-other-mode > $OUT/p.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/p.log; exit 1; }
python scripts/pmc_summary.py $OUT/p > $OUT/summary.txt 2>&1 || true
grep -A 8 "^k_eval_nb\|^k_eval_ref$" $OUT/summary.txt | head -30
echo ICACHE_DONE
