#!/bin/bash
# GPU-box session: parity tests on the product build, then bench lines for each library variant.
# Usage: bash scripts/ab_bench.sh TAG "LIB1 LIB2 ..." ["bench args"]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; ARGS=${3:-"--no-cpu-baseline --no-variant --no-pipeline"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for rep in 1 2; do
  for lib in $LIBS; do
    ACMMP_LIB=$lib timeout -k 10 300 python bench.py $ARGS > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), d['value'], d['ms_per_depth_map'], d['stages_ms']['init'], d['roofline']['half_sweep_kernels_ms'])"
  done
done
echo AB_DONE
