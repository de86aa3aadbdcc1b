#!/bin/bash
# Round 6: GPU tests of the in-tree build, the default bench line, and a rocprofv3 kernel-stats pass of the timed
# region.  Usage: bash scripts/r06_check.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 300 python bench.py $Q > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['clock']['ghz'], d['stages_ms'], d['roofline']['half_sweep_kernels_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --timed-only --steps 20 $Q > $OUT/prof_bench.json 2> $OUT/prof.err || { tail $OUT/prof.err; exit 1; }
python - <<PY
import csv
for r in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:14]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
echo CHECK_DONE
