#!/bin/bash
# Round-5 development check: the tests touched by a change first, then scripts/check.sh (GPU suite, smoke,
# bench line), then the T2 seed study.  Usage: bash scripts/r05_step.sh TAG "pytest node ids..."
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05}
mkdir -p $OUT
if [ -n "$2" ]; then
  ACMMP_TEST_REPORT_DIR=$OUT timeout -k 10 600 python -u -m pytest $2 -x -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_first.log 2>&1 || { echo "first tests failed"; grep -E "FAILED|ERROR|Error" $OUT/pytest_first.log | head -8; tail -40 $OUT/pytest_first.log; exit 1; }
  tail -1 $OUT/pytest_first.log
fi
bash scripts/check.sh ${1:-r05}/check || exit 1
if [ -n "$3" ]; then
  timeout -k 10 600 python -u scripts/t2_seeds.py $3 --out $OUT/t2_seeds.json > $OUT/t2_seeds.log 2>&1 || { echo "t2 failed"; tail -20 $OUT/t2_seeds.log; exit 1; }
  tail -2 $OUT/t2_seeds.log
fi
echo STEP_DONE
