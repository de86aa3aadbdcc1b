#!/bin/bash
# Round-4 re-sweep of the refinement split point S (ACMMP_REF_SPLIT_AT) with 4-view tail chunks, at C3 and C2,
# both math modes at C3 (GPU box, repo root).  Usage: bash scripts/r04_split.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_split}
mkdir -p $OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for S in 8 10 12; do line c3_S$S ACMMP_REF_SPLIT_AT=$S timeout -k 10 400 python bench.py $C3 $Q; done
for S in 4 8; do line c3_exact_S$S ACMMP_REF_SPLIT_AT=$S timeout -k 10 400 python bench.py $C3 $Q --math exact; done
for S in 6 8; do line c2_S$S ACMMP_REF_SPLIT_AT=$S timeout -k 10 300 python bench.py $C2 $Q; done
line c3_S8 ACMMP_REF_SPLIT_AT=8 timeout -k 10 400 python bench.py $C3 $Q
echo SPLIT_DONE
