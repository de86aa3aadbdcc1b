#!/bin/bash
# A/B of library variants at the metric, at C3's capped size (3200x1600 SPHERE, V = 15) and at C2
# (1600x1200 pinhole, V = 10), fast math, alternating, 2 reps.  Usage: bash scripts/ab_v15.sh TAG "LIBS"
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
NOX="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
for rep in 1 2; do
  for cfg in "metric|" "c3cap|--width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1" "c2|--model pinhole --width 1600 --height 1200 --n-src 10 --steps 3 --warmup 1"; do
    name=${cfg%%|*}; args=${cfg#*|}
    for lib in $LIBS; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py $NOX $args > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));print('$name', os.path.basename('$lib'), d['value'], d['ms_per_step'], d['stages_ms']['init'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
echo AB_DONE
