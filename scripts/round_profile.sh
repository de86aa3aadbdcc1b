#!/bin/bash
# Full GPU-box record for one build: parity tests, the default bench line, a rocprofv3 kernel-trace of the
# same bench, and the PMC passes of the headline config.  Usage: bash scripts/round_profile.sh TAG
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-600 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-pipeline --no-variant --no-other-mode > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
bash scripts/pmc.sh $OUT/pmc "--steps 1 --warmup 0 --no-cpu-baseline --no-variant --no-pipeline --no-other-mode" || exit 1
python scripts/pmc_summary.py $OUT/pmc --json $OUT/pmc_propagate.json > $OUT/pmc_summary.txt || exit 1
echo ROUND_PROFILE_DONE
