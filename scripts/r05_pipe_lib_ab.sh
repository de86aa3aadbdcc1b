#!/bin/bash
# A/B of two library builds on the C2 49-view schedule (fast math), interleaved.  Usage:
#   bash scripts/r05_pipe_lib_ab.sh TAG "LIB1 LIB2" ROUNDS
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
for r in $(seq 1 ${3:-2}); do
  for lib in $2; do
    n=$(basename $lib .so)
    ACMMP_LIB=$lib timeout -k 10 300 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 \
      --n-src 10 --math fast > $OUT/c2_${n}_r$r.json 2> $OUT/c2_${n}_r$r.err || { echo "run failed"; tail -5 $OUT/c2_${n}_r$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/c2_${n}_r$r.json').read().strip().splitlines()[-1]); print('$n', d['total_s'], d['pass_compute_s'])" | tee -a $OUT/ab.txt
  done
done
echo PIPE_LIB_AB_DONE
