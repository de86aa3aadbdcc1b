#!/bin/bash
# GPU parity tests only (no bench).  Usage (GPU box, repo root): bash scripts/gpu_tests.sh TAG [pytest-args]
set -o pipefail
TAG=${1:-dev}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -rA "$@" > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "PASSED|FAILED|ERROR" $OUT/pytest_gpu.log | tail -5; tail -40 $OUT/pytest_gpu.log; exit 1; }
grep -E "within 1%|passed|failed" $OUT/pytest_gpu.log | tail -8
echo GPU_TESTS_DONE
