#!/bin/bash
# GPU tests, the default bench line (end_to_end schedule) and the C2 49-view schedule.  Usage: bash scripts/r03_pipe_check.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pipe}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['end_to_end']['ms_per_view'], d['end_to_end']['stages_s'])"
timeout -k 10 500 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 --n-src 10 > $OUT/c2_pipeline.json 2> $OUT/c2_pipeline.err || { echo "c2 failed"; tail -20 $OUT/c2_pipeline.err; exit 1; }
tail -1 $OUT/c2_pipeline.json | cut -c1-600
echo PIPE_DONE
