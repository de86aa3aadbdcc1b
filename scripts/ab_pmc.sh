#!/bin/bash
# PMC passes (scripts/pmc.sh counter sets) of the metric bench for each library variant, plus the
# counter list of the box.  Usage (GPU box, repo root): bash scripts/ab_pmc.sh TAG "LIBS"
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1 || echo "list-avail failed"
for lib in $LIBS; do
  n=$(basename $lib .so)
  ACMMP_LIB=$lib bash scripts/pmc.sh $OUT/$n "--steps 1 --warmup 1 --no-cpu-baseline --no-variant --no-pipeline --no-other-mode" || exit 1
  python scripts/pmc_summary.py $OUT/$n > $OUT/${n}_summary.txt || exit 1
done
echo AB_PMC_DONE
