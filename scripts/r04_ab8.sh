#!/bin/bash
# Round-4 check + A/B (GPU box, repo root): the refinement-split parity tests (new k_tail_scan), then the
# SPHERE fast k_eval_nb at 6 waves without spills (libacmmp_sphw6) against the product's 7, at the metric
# and C3, with a kernel trace of the metric.  Usage: bash scripts/r04_ab8.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab8}
L=acmmp-spherical_amd/acmmp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or refinement" -x -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_split.log 2>&1 || { echo "split tests failed"; grep -E "^E  |FAILED" $OUT/pytest_split.log | cut -c1-300 | head; tail -3 $OUT/pytest_split.log; exit 1; }
tail -1 $OUT/pytest_split.log
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line metric timeout -k 10 300 python bench.py $Q
  line metric_sphw6 ACMMP_LIB=$L/libacmmp_sphw6.so timeout -k 10 300 python bench.py $Q
done
line c3 timeout -k 10 400 python bench.py $C3 $Q
line c3_sphw6 ACMMP_LIB=$L/libacmmp_sphw6.so timeout -k 10 400 python bench.py $C3 $Q
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --timed-only --steps 5 $Q > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 - $OUT <<'PY' || exit 1
import csv, sys, os
out = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(out, "prof", "run_kernel_stats.csv"))))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%-60s calls %6s avg_ms %.4f total_ms %.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
for lib in libacmmp libacmmp_sphw6; do
  timeout -k 10 300 env ACMMP_LIB=$L/$lib.so rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$lib -o run -- python3 bench.py --steps 1 --warmup 1 --timed-only $Q > $OUT/pmc_$lib.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc_$lib.log; exit 1; }
done
echo AB8_DONE
