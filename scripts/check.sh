#!/bin/bash
# Check of the in-tree build the round-end driver uses: GPU tests, smoke(), the default bench line.  Usage: bash scripts/check.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
ACMMP_TEST_REPORT_DIR=$OUT timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
echo LAST_DONE
