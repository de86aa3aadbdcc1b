#!/bin/bash
# A/B of engine environment knobs on one bench config, interleaved.  Usage:
#   bash scripts/r05_env_ab.sh TAG REPS "CFG" "ENV1" "ENV2" ...   (ENVk: space-separated K=V, or "-" for none)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; REPS=$2; CFG=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq $REPS); do
  for ev in "$@"; do
    e=""; [ "$ev" != "-" ] && e="$ev"
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $CFG > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));r=d['roofline'];print('$ev', d['value'], d['ms_per_step'], r.get('half_sweep_kernels_ms'))" | tee -a $OUT/ab.txt
  done
done
echo ENV_AB_DONE
