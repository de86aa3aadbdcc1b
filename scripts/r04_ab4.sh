#!/bin/bash
# Round-4 A/B (GPU box, repo root): the deferred-fallback identity tests (row-parallel k_nb_fix, forced
# fallbacks), a rocprofv3 kernel trace of the metric bench, then bench lines of the refinement variants --
# libacmmp_refw5 (k_eval_ref at 5 waves per SIMD: the SPHERE V > 4 instance in 96 VGPRs) at C3 and
# libacmmp_refpin2 (fast pinhole k_eval_ref in 2-view chunks) at C2 -- against the product, and the
# fast-mode / planar-state tests.  Usage: bash scripts/r04_ab4.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab4}
L=acmmp-spherical_amd/acmmp
mkdir -p $OUT
export ACMMP_TEST_REPORT_DIR=$OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_interp.py tests/test_gpu_fastmath.py -k deferred -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_deferred.log 2>&1
rc=$?
tail -1 $OUT/pytest_deferred.log
grep -E "^E  |FAILED" $OUT/pytest_deferred.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "deferred tests aborted rc=$rc"; exit 1; fi
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --timed-only --steps 5 $Q > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
python3 - $OUT <<'PY' || exit 1
import csv, sys, os
out = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(out, "prof", "run_kernel_stats.csv"))))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
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
  line metric_nofb ACMMP_SPREAD_MAX=1e30 timeout -k 10 300 python bench.py $Q
  line c2 timeout -k 10 300 python bench.py $C2 $Q
  line c2_refpin2 ACMMP_LIB=$L/libacmmp_refpin2.so timeout -k 10 300 python bench.py $C2 $Q
done
line c3 timeout -k 10 400 python bench.py $C3 $Q
line c3_refw5 ACMMP_LIB=$L/libacmmp_refw5.so timeout -k 10 400 python bench.py $C3 $Q
line c3 timeout -k 10 400 python bench.py $C3 $Q
line c3_refw5 ACMMP_LIB=$L/libacmmp_refw5.so timeout -k 10 400 python bench.py $C3 $Q
timeout -k 10 600 python -u -m pytest tests/test_gpu_interp.py tests/test_gpu_fastmath.py tests/test_gpu_planar_state.py -v -rA --timeout 300 --timeout-method thread -k "not deferred" > $OUT/pytest_fast.log 2>&1
rc=$?
tail -1 $OUT/pytest_fast.log
grep -E "^E  |FAILED" $OUT/pytest_fast.log | head -20
echo AB4_DONE rc=$rc
