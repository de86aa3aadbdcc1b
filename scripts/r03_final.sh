#!/bin/bash
# Round-3 record of the committed tree (GPU box, repo root): parity tests, PMC passes of the headline
# config (their summary feeds the bench line's `traffic`), the default bench line, a rocprofv3 kernel trace
# of the same timed region (bench.py --timed-only) with trace_window.py's recomputed frac, and the
# refinement split sweep at V=20.  Usage: bash scripts/r03_final.sh TAG
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rA > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/pmc.sh $OUT/pmc "--steps 1 --warmup 1 --timed-only $Q" || exit 1
python scripts/pmc_summary.py $OUT/pmc --json $OUT/pmc_propagate.json > $OUT/pmc_summary.txt || exit 1
timeout -k 10 600 python bench.py --pmc $OUT/pmc_propagate.json > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --timed-only $Q --pmc $OUT/pmc_propagate.json > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python scripts/trace_window.py $OUT/prof/run_kernel_trace.csv $OUT/prof_bench.json --json $OUT/trace_window.json || exit 1
for S in 4 8 12; do
  ACMMP_REF_SPLIT_AT=$S timeout -k 10 300 python bench.py $Q --model pinhole --width 3200 --height 2133 --n-src 20 --steps 2 --warmup 1 > $OUT/v20.json 2> $OUT/v20.err || { tail $OUT/v20.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/v20.json'));print('V20 S=$S', d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/split_v20.txt
done
echo FINAL_DONE
