#!/bin/bash
# GPU tests of the product build and the C2 49-view schedule's stages (device-resident geom-pass state).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_state}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 500 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 --n-src 10 > $OUT/c2_pipeline.json 2> $OUT/c2_pipeline.err || { echo "c2 pipeline failed"; tail -20 $OUT/c2_pipeline.err; exit 1; }
tail -c 600 $OUT/c2_pipeline.json
echo STATE_DONE
