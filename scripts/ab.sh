#!/bin/bash
# A/B timing of library variants on the GPU box (after the GPU tests pass on the product build).
# Usage: bash scripts/ab.sh TAG "LIB1 LIB2 ..." "CONFIG1" "CONFIG2" ...   (CONFIG "" = the metric)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for lib in $LIBS; do
  ACMMP_LIB=$lib timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest.log 2>&1 || { echo "$lib"; tail -30 $OUT/pytest.log; exit 1; }
  echo "$(basename $lib): $(tail -1 $OUT/pytest.log)"
done
for cfg in "$@"; do
  for lib in $LIBS; do
    ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), '$cfg', d['value'], d['ms_per_depth_map'], d['stages_ms']['init'], d['roofline']['half_sweep_kernels_ms'])"
  done
done
