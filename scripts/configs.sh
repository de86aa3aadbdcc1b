#!/bin/bash
# BASELINE.json's other single-GPU configurations: RunPatchMatch bench lines (C2 1600x1200 pinhole V=10,
# C3 at the 3200x1600 the reference scheduler runs 4096x2048 inputs at, V=15), their PMC passes, and the
# C2 / C3 ProcessProblem schedules.  Usage (GPU box, repo root): bash scripts/configs.sh TAG [no-pmc]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-configs}
mkdir -p $OUT
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 $t "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; exit 1; }
  tail -1 $OUT/$name.json | cut -c1-300
}
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
C3="--model sphere --width 3200 --height 1600 --n-src 15"
if [ "$2" != "no-pmc" ]; then
  bash scripts/pmc.sh $OUT/pmc_c2 "$C2 --steps 1 --warmup 1 --timed-only" || exit 1
  python scripts/pmc_summary.py $OUT/pmc_c2 --json $OUT/pmc_c2.json --width 1600 --height 1200 --n-src 10 --model pinhole > $OUT/pmc_c2_summary.txt || exit 1
  bash scripts/pmc.sh $OUT/pmc_c3 "$C3 --steps 1 --warmup 1 --timed-only" || exit 1
  python scripts/pmc_summary.py $OUT/pmc_c3 --json $OUT/pmc_c3.json --width 3200 --height 1600 --n-src 15 --model sphere > $OUT/pmc_c3_summary.txt || exit 1
fi
run c2_patchmatch 300 python bench.py $C2 --no-cpu-baseline --no-variant --no-pipeline --pmc $OUT/pmc_c2.json
run c3_patchmatch 400 python bench.py $C3 --steps 3 --warmup 1 --no-cpu-baseline --no-variant --no-pipeline --pmc $OUT/pmc_c3.json
run c2_pipeline 500 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 --n-src 10 --math fast
echo CONFIGS_DONE
