#!/bin/bash
# BASELINE's multi-view schedules on one GPU (fast math): C2 (49 x 1600x1200 pinhole, 10 sources), the C4 shape
# (24 x 3200x2133 pinhole, 20 sources, three scales: bench.py --mode pipeline) and the C5 shape (300 x 1920x1080
# pinhole, 10 sources, two scales).  Usage: bash scripts/r05_pipelines.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pipelines}
mkdir -p $OUT
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 $t "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; exit 1; }
  tail -1 $OUT/$name.json | cut -c1-400
}
run c2_pipeline 500 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 --n-src 10 --math fast
run c4_pipeline 900 python -u bench.py --mode pipeline --math fast
run c5_pipeline 1200 python -u scripts/pipeline_bench.py --model pinhole --width 1920 --height 1080 --views 300 --n-src 10 --math fast --n-waves 12
echo PIPELINES_DONE
