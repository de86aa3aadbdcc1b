#!/bin/bash
# Round-4 A/B (GPU box, repo root): C3 (3200x1600 SPHERE V=15) with the refinement tail in 4-view chunks
# (libacmmp_tailvb4) against the product's 2-view ones, and the metric line.  Usage: bash scripts/r04_ab6.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab6}
L=acmmp-spherical_amd/acmmp
mkdir -p $OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
line metric timeout -k 10 300 python bench.py $Q
for rep in 1 2; do
  line c3 timeout -k 10 400 python bench.py $C3 $Q
  line c3_tailvb4 ACMMP_LIB=$L/libacmmp_tailvb4.so timeout -k 10 400 python bench.py $C3 $Q
done
echo AB6_DONE
