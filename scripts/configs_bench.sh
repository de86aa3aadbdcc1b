#!/bin/bash
# BASELINE.json's other configurations on one GPU: RunPatchMatch bench lines and the end-to-end
# ProcessProblem schedule.  Usage (GPU box, repo root): bash scripts/configs_bench.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 $t "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; exit 1; }
  tail -1 $OUT/$name.json | cut -c1-400
}
NOX="--no-cpu-baseline --no-variant --no-pipeline"
run c2_patchmatch 300 python bench.py --model pinhole --width 1600 --height 1200 --n-src 10 $NOX
run c3_patchmatch 400 python bench.py --model sphere --width 4096 --height 2048 --n-src 15 --steps 3 --warmup 1 $NOX
run c2_pipeline 400 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 --n-src 10
run c3_pipeline 500 python -u scripts/pipeline_bench.py --model sphere --width 4096 --height 2048 --views 16
echo CONFIGS_DONE
