#!/bin/bash
# A/B of library variants (GPU box, repo root): GPU tests on each TESTED lib, then alternating bench
# lines in both math modes.  Usage: bash scripts/ab_libs.sh TAG "TESTED_LIBS" "ALL_LIBS" ["bench args"]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; TESTED=$2; LIBS=$3; ARGS=${4:-"--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for lib in $TESTED; do
  ACMMP_LIB=$lib timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_$(basename $lib).log 2>&1 || { echo "pytest failed ($lib)"; tail -30 $OUT/pytest_$(basename $lib).log; exit 1; }
  echo "$(basename $lib): $(tail -1 $OUT/pytest_$(basename $lib).log)"
done
for rep in 1 2; do
  for lib in $LIBS; do
    for m in fast exact; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py $ARGS --math $m > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), '$m', d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'], d['stages_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
echo AB_DONE
