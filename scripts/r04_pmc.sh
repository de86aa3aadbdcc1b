#!/bin/bash
# Round-4 PMC passes (GPU box, repo root), each its own rocprofv3 --pmc run (no trace domains): the metric
# bench's five passes of scripts/pmc.sh (for profiles/pmc_propagate.json), then instruction and L2 passes
# at C3 (3200x1600 SPHERE V=15) and C2 (1600x1200 pinhole V=10).  Usage: bash scripts/r04_pmc.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_pmc}
mkdir -p $OUT
Q="--steps 1 --warmup 0 --no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
bash scripts/pmc.sh $OUT/metric "$Q" || exit 1
pass() {  # dir, bench args, counters...
  local d=$1 args=$2; shift 2
  mkdir -p $d
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $d -o run -- python3 bench.py $args > $d.log 2>&1 || { echo "pass $d failed"; tail -20 $d.log; exit 1; }
}
C3="--model sphere --width 3200 --height 1600 --n-src 15 $Q"
C2="--model pinhole --width 1600 --height 1200 --n-src 10 $Q"
pass $OUT/c3/p1 "$C3" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR
pass $OUT/c3/p2 "$C3" TCC_HIT TCC_MISS
pass $OUT/c3/p3 "$C3" FETCH_SIZE
pass $OUT/c3/p4 "$C3" WRITE_SIZE
pass $OUT/c2/p1 "$C2" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR
pass $OUT/c2/p2 "$C2" TCC_HIT TCC_MISS
pass $OUT/c2/p3 "$C2" FETCH_SIZE
pass $OUT/c2/p4 "$C2" WRITE_SIZE
echo PMC4_DONE
