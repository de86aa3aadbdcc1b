#!/bin/bash
# A/B of library variants in both math modes (GPU box, repo root), after the variants' GPU tests.
# Usage: bash scripts/ab_modes.sh TAG "LIB1 LIB2 ..." ["bench args"] ["pytest -k expr"]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; ARGS=${3:-"--no-cpu-baseline --no-variant --no-pipeline"}; K=${4:-""}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for lib in $LIBS; do
  ACMMP_LIB=$lib timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_$(basename $lib).log 2>&1 || { echo "pytest failed ($lib)"; tail -30 $OUT/pytest_$(basename $lib).log; exit 1; }
  echo "$(basename $lib): $(tail -1 $OUT/pytest_$(basename $lib).log)"
done
for rep in 1 2; do
  for lib in $LIBS; do
    for m in exact fast; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py $ARGS --math $m > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), '$m', d['value'], d['ms_per_step'], d['stages_ms']['init'], d['roofline']['half_sweep_kernels_ms'])"
    done
  done
done
echo AB_DONE
