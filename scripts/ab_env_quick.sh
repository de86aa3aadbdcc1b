#!/bin/bash
# A/B of run-time switches without the test pass: bench lines (both math modes) per environment setting.
# Usage: bash scripts/ab_env_quick.sh TAG "VAR=a VAR=b ..." ["bench args"]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ENVS=$2; ARGS=${3:-""}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for e in $ENVS; do
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline $ARGS > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$e', d['value'], d['other_math_mode']['value'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
  done
done
echo AB_DONE
