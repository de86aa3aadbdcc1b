#!/bin/bash
# Round-4 kernel-level look at the SPHERE fast path (GPU box, repo root): a rocprofv3 kernel trace of the
# metric bench's timed region (product build), then bench lines of the spread-threshold variants
# (libacmmp_nofb: no interpolation fallback; libacmmp_thr256: 256-pixel threshold) with the fallbacks
# deferred and inline (ACMMP_NB_FIX=0), at the metric and C3.  Usage: bash scripts/r04_prof.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_prof}
mkdir -p $OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --timed-only --steps 5 $Q > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 - $OUT <<'PY' || exit 1
import csv, sys, collections, os
out = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(out, "prof", "run_kernel_stats.csv"))))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print("%-60s calls %6s avg_ms %.4f total_ms %.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
L=acmmp-spherical_amd/acmmp
for rep in 1 2; do
  line metric_queue64 timeout -k 10 300 python bench.py $Q
  line metric_nofb ACMMP_LIB=$L/libacmmp_nofb.so timeout -k 10 300 python bench.py $Q
  line metric_queue256 ACMMP_LIB=$L/libacmmp_thr256.so timeout -k 10 300 python bench.py $Q
  line metric_inline256 ACMMP_LIB=$L/libacmmp_thr256.so ACMMP_NB_FIX=0 timeout -k 10 300 python bench.py $Q
done
line c3_queue64 timeout -k 10 400 python bench.py $C3 $Q
line c3_nofb ACMMP_LIB=$L/libacmmp_nofb.so timeout -k 10 400 python bench.py $C3 $Q
line c3_queue256 ACMMP_LIB=$L/libacmmp_thr256.so timeout -k 10 400 python bench.py $C3 $Q
echo PROF_DONE
