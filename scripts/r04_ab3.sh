#!/bin/bash
# Round-4 A/B of the working tree (GPU box, repo root): a rocprofv3 kernel trace of the metric bench's timed
# region, bench lines -- metric with deferred fallbacks (product), inline (ACMMP_NB_FIX=0) and without
# fallbacks (libacmmp_nofb), metric exact, C3 fast / nofb / exact, C2 homogeneous 2-view and per-sample
# 4-view (libacmmp_pinvb4) -- then the fast-mode / per-query tests (reports).  Usage: bash scripts/r04_ab3.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab3}
L=acmmp-spherical_amd/acmmp
mkdir -p $OUT
export ACMMP_TEST_REPORT_DIR=$OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --timed-only --steps 5 $Q > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 - $OUT <<'PY' || exit 1
import csv, sys, os
out = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(out, "prof", "run_kernel_stats.csv"))))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print("%-60s calls %6s avg_ms %.4f total_ms %.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line metric timeout -k 10 300 python bench.py $Q
  line metric_inline ACMMP_NB_FIX=0 timeout -k 10 300 python bench.py $Q
  line metric_nofb ACMMP_LIB=$L/libacmmp_nofb.so timeout -k 10 300 python bench.py $Q
done
line metric_exact timeout -k 10 300 python bench.py $Q --math exact
line c3 timeout -k 10 400 python bench.py $C3 $Q
line c3_nofb ACMMP_LIB=$L/libacmmp_nofb.so timeout -k 10 400 python bench.py $C3 $Q
line c3_exact timeout -k 10 400 python bench.py $C3 $Q --math exact
line c2_homog2 timeout -k 10 300 python bench.py $C2 $Q
line c2_sample4 ACMMP_LIB=$L/libacmmp_pinvb4.so ACMMP_PIN_HOMOG=0 timeout -k 10 300 python bench.py $C2 $Q
timeout -k 10 600 python -u -m pytest tests/test_gpu_interp.py tests/test_gpu_fastmath.py tests/test_gpu_planar_state.py -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_fast.log 2>&1
rc=$?
tail -1 $OUT/pytest_fast.log
grep -E "^E  |FAILED" $OUT/pytest_fast.log | head -20
echo AB3_DONE rc=$rc
