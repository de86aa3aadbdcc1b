#!/bin/bash
# Round-4 re-check of k_eval_nb's view chunking at C3 (ACMMP_NB_VIEW_CHUNK: 8 = default, 5, 15 = one launch)
# with the deferred fallbacks (GPU box, repo root).  Usage: bash scripts/r04_chunk.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_chunk}
mkdir -p $OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for c in 8 5 15 8; do line c3_chunk$c ACMMP_NB_VIEW_CHUNK=$c timeout -k 10 400 python bench.py $C3 $Q; done
echo CHUNK_DONE
