#!/bin/bash
# Round-6 A/B of two library builds: the per-query interpolation tests (reports per build), then bench lines
# alternated.  Usage: bash scripts/r06_ab2.sh TAG BASE_LIB CAND_LIB "CONFIG1" ...   (CONFIG "" = the metric)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; BASE=$2; CAND=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT/base $OUT/cand
ACMMP_LIB=$BASE ACMMP_TEST_REPORT_DIR=$OUT/base timeout -k 10 600 python -u -m pytest tests/test_gpu_interp.py -q --timeout 300 --timeout-method thread -k "k_eval_nb_per_query" > $OUT/base.log 2>&1; echo base rc=$?
ACMMP_LIB=$CAND ACMMP_TEST_REPORT_DIR=$OUT/cand timeout -k 10 600 python -u -m pytest tests/test_gpu_interp.py -q --timeout 300 --timeout-method thread -k "k_eval_nb_per_query" > $OUT/cand.log 2>&1; echo cand rc=$?
for cfg in "$@"; do
  for rep in 1 2; do
    for lib in $BASE $CAND; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), '$cfg', d['value'], d['ms_per_step'], d['clock']['ghz'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
echo AB_DONE
