#!/bin/bash
# Round-2 record for one build (GPU box, repo root): round_profile (tests, bench, rocprof, PMC at the
# metric), the PMC passes at C3's V = 15 (3200x1600 SPHERE), and the configs bench.  Usage: TAG
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
bash scripts/round_profile.sh $TAG || exit 1
V15="--model sphere --width 3200 --height 1600 --n-src 15 --steps 1 --warmup 0 --no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
bash scripts/pmc.sh $OUT/pmc_v15 "$V15" || exit 1
python scripts/pmc_summary.py $OUT/pmc_v15 --json $OUT/pmc_v15.json --width 3200 --height 1600 --n-src 15 > $OUT/pmc_v15_summary.txt || exit 1
bash scripts/configs_bench.sh $TAG/configs || exit 1
echo ROUND2_FULL_DONE
