#!/bin/bash
# Alternating A/B of libraries on the end-to-end schedule (bench.py end_to_end) and the C2 49-view schedule.
# Usage: bash scripts/r03_pipe_ab.sh TAG "LIBS"
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
for rep in 1 2 3; do
  for lib in $2; do
    ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-other-mode > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json,os;d=json.load(open('$OUT/b.json'));e=d['end_to_end'];print(os.path.basename('$lib'), 'e2e', e['ms_per_view'], e['stages_s'])" | tee -a $OUT/ab.txt
  done
done
for lib in $2; do
  ACMMP_LIB=$lib timeout -k 10 500 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 --n-src 10 > $OUT/c2.json 2> $OUT/c2.err || { tail $OUT/c2.err; exit 1; }
  python -c "import json,os;d=json.loads(open('$OUT/c2.json').read().strip().splitlines()[-1]);print(os.path.basename('$lib'), 'c2', d['total_s'], d['stages_s'])" | tee -a $OUT/ab.txt
done
echo AB_DONE
