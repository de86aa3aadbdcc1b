#!/bin/bash
# Round-4 check of the working tree (GPU box, repo root): the per-query interpolation test first (with its
# report), the whole GPU suite, smoke(), the default bench line, then the C2 pinhole bench line and its PMC
# passes.  Usage: bash scripts/r04_check.sh TAG [quick]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_check}
mkdir -p $OUT
export ACMMP_TEST_REPORT_DIR=$OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_interp.py -x -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_interp.log 2>&1 || { echo "interp test failed"; grep -E "FAILED|ERROR|assert" $OUT/pytest_interp.log | head -20; tail -30 $OUT/pytest_interp.log; exit 1; }
tail -1 $OUT/pytest_interp.log
if [ "$2" != "quick" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread --deselect tests/test_gpu_interp.py > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
timeout -k 10 300 python bench.py $C2 --no-cpu-baseline --no-variant --no-pipeline > $OUT/c2.json 2> $OUT/c2.err || { echo "c2 failed"; tail -20 $OUT/c2.err; exit 1; }
cut -c1-300 $OUT/c2.json
bash scripts/pmc.sh $OUT/pmc_c2 "$C2 --steps 1 --warmup 1 --timed-only --no-cpu-baseline --no-variant --no-pipeline --no-other-mode" || exit 1
python scripts/pmc_summary.py $OUT/pmc_c2 --json $OUT/pmc_c2.json --width 1600 --height 1200 --n-src 10 --model pinhole > $OUT/pmc_c2_summary.txt || exit 1
echo CHECK_DONE
