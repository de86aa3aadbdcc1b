#!/bin/bash
# Round 6: GPU tests of the product build, the planar-prior stage timing, then an A/B of library variants
# (alternated bench lines).  Usage: bash scripts/r06_ab4.sh TAG "LIB1 LIB2 ..." "CONFIG1" ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
ACMMP_TEST_REPORT_DIR=$OUT timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $OUT/pytest.log | head; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python scripts/planar_timing.py 2000 1500 sphere > $OUT/planar_sphere.json || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --no-variant --no-other-mode > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], json.dumps(d['end_to_end']['stages_s']))"
for cfg in "$@"; do
  for rep in 1 2; do
    for lib in $LIBS; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), '$cfg', d['value'], d['ms_per_step'], d['clock']['ghz'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
echo AB_DONE
