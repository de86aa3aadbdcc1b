#!/bin/bash
# GPU box: parity tests, a quick bench line, then the fast-math floor measurement.  Usage: bash scripts/r03_check.sh TAG
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
if [ "${FLOOR:-1}" = "1" ]; then
  timeout -k 10 900 python -u scripts/fastmath_floor.py ${FLOOR_ARGS---quick} > $OUT/fastmath_floor.json 2> $OUT/fastmath_floor.err || { echo "floor failed"; tail -20 $OUT/fastmath_floor.err; exit 1; }
fi
echo CHECK_DONE
