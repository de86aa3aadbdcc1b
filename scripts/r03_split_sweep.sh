#!/bin/bash
# Refinement split point (ACMMP_REF_SPLIT_AT) at C3 3200x1600 V=15 and C2 1600x1200 V=10, fast mode, plus a
# 2-rank rehearsal of bench.py --gpus 2 on one GPU.  Usage (GPU box, repo root): bash scripts/r03_split_sweep.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-split}
mkdir -p $OUT
ARGS="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
line() {  # label, env S, bench args
  ACMMP_REF_SPLIT_AT=$2 timeout -k 10 300 python bench.py $ARGS $3 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$1', 'S=$2', d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/split.txt
}
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
for rep in 1 2; do
  for S in 4 8 12; do line C3 $S "$C3" || exit 1; done
  for S in 2 4 6 8; do line C2 $S "$C2" || exit 1; done
done
timeout -k 10 300 python bench.py --gpus 2 --allow-shared-gpus --steps 3 --warmup 1 --no-cpu-baseline --no-variant > $OUT/gpus2.json 2> $OUT/gpus2.err || { echo "gpus 2 failed"; tail -30 $OUT/gpus2.err; exit 1; }
tail -1 $OUT/gpus2.json | cut -c1-600
echo SPLIT_DONE
