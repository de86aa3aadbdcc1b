#!/bin/bash
# A/B of the C2 49-view schedule (fast math) with the geom-pass overlap off / on, interleaved.
# Usage: bash scripts/r05_pipe_ab.sh TAG [rounds]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pipe_ab}
mkdir -p $OUT
for r in $(seq 1 ${2:-2}); do
  for g in 0 1; do
    ACMMP_PIPELINE_GEOM_OVERLAP=$g timeout -k 10 300 python -u scripts/pipeline_bench.py --model pinhole --width 1600 \
      --height 1200 --views 49 --n-src 10 --math fast > $OUT/c2_g${g}_r$r.json 2> $OUT/c2_g${g}_r$r.err || { echo "run failed"; tail -5 $OUT/c2_g${g}_r$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/c2_g${g}_r$r.json').read().strip().splitlines()[-1]); print('geom_overlap=$g', d['total_s'], d['pass_s'], d['pass_compute_s'])"
  done
done
echo PIPE_AB_DONE
