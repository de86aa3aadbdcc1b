#!/bin/bash
# One GPU-box session: parity tests, the default bench line, and a kernel-trace profile of the bench.
# Usage (from the repo root, on the box): bash scripts/gpu_check.sh TAG [pytest-args]
set -o pipefail
TAG=${1:-dev}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-pipeline --no-variant > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
cat $OUT/prof_bench.json
echo GPU_CHECK_DONE
