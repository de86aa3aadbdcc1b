#!/bin/bash
# A/B of environment settings on one library (GPU box): alternated bench lines per setting and config.
# Usage: bash scripts/ab_env.sh TAG "ENV1 ENV2 ..." "CONFIG1" ...   (ENV "-" = none, else VAR=value; CONFIG "" = metric)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ENVS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for cfg in "$@"; do
  for rep in 1 2 3; do
    for e in $ENVS; do
      if [ "$e" = "-" ]; then E=""; else E="$e"; fi
      env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/b.json'));print('$e', '$cfg', d['value'], d['ms_per_step'], d['clock']['ghz'], d['stages_ms'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
echo AB_ENV_DONE
