#!/bin/bash
# A/B of run-time switches (environment settings) on one library, after the GPU parity tests.
# Usage: bash scripts/ab_env.sh TAG "VAR=a VAR=b ..." "CONFIG1" "CONFIG2" ...   (CONFIG "" = the metric)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ENVS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in "$@"; do
  for rep in 1 2; do
    for e in $ENVS; do
      env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/b.json'));print('$e', '$cfg', d['value'], d['ms_per_depth_map'], d['stages_ms']['init'], d['roofline']['half_sweep_kernels_ms'])"
    done
  done
done
echo AB_DONE
