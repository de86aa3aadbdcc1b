#!/bin/bash
# Round-6 A/B: GPU tests on the candidate library, then bench lines of base vs candidate alternated.
# Usage: bash scripts/r06_ab.sh TAG CAND_LIB "CONFIG1" "CONFIG2" ...   (CONFIG "" = the metric)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; CAND=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
BASE=acmmp-spherical_amd/acmmp/libacmmp.so
ACMMP_LIB=$CAND ACMMP_TEST_REPORT_DIR=$OUT timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest $CAND"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -30 $OUT/pytest.log; exit 1; }
echo "$(basename $CAND): $(tail -1 $OUT/pytest.log)"
for cfg in "$@"; do
  for rep in 1 2; do
    for lib in $BASE $CAND; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), '$cfg', d['value'], d['ms_per_step'], d['clock']['ghz'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
echo AB_DONE
