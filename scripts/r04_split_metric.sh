#!/bin/bash
# Round-4 re-sweep of the refinement split point at the metric (V = 4: S = 1, 2 = default, 3; and no split)
# with the compacted tail (GPU box, repo root).  Usage: bash scripts/r04_split_metric.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_split_metric}
mkdir -p $OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line metric_S2 ACMMP_REF_SPLIT_AT=2 timeout -k 10 300 python bench.py $Q
  line metric_S1 ACMMP_REF_SPLIT_AT=1 timeout -k 10 300 python bench.py $Q
  line metric_S3 ACMMP_REF_SPLIT_AT=3 timeout -k 10 300 python bench.py $Q
done
line metric_nosplit ACMMP_REF_SPLIT=0 timeout -k 10 300 python bench.py $Q
echo SPLITM_DONE
