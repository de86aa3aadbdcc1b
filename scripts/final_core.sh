#!/bin/bash
# Record of the committed tree (GPU box, repo root): parity tests, PMC passes of the headline
# config (their summary feeds the bench line's `traffic`), the default bench line, a rocprofv3 kernel trace
# of the same timed region (bench.py --timed-only, 20 steps so that the warmup's dispatches weigh little in
# rocprof's all-dispatch mean) with trace_window.py's recomputed frac, then scripts/configs.sh (C2 / C3
# PMC, bench lines and the C2 schedule).  Usage: bash scripts/final_core.sh TAG
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
bash scripts/pmc.sh $OUT/pmc "--steps 1 --warmup 1 --timed-only $Q" || exit 1
python scripts/pmc_summary.py $OUT/pmc --json $OUT/pmc_propagate.json > $OUT/pmc_summary.txt || exit 1
timeout -k 10 600 python bench.py --pmc $OUT/pmc_propagate.json > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --timed-only --steps 20 $Q --pmc $OUT/pmc_propagate.json > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python scripts/trace_window.py $OUT/prof/run_kernel_trace.csv $OUT/prof_bench.json --json $OUT/trace_window.json || exit 1
# (configs: scripts/configs.sh, a call of its own)
echo FINAL_DONE
