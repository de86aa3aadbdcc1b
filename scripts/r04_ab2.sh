#!/bin/bash
# Round-4 A/B of the working tree (GPU box, repo root): fast-mode / per-query tests (reports), the GPU suite,
# then bench lines -- metric with the deferred interpolation fallbacks (product) and inline (ACMMP_NB_FIX=0),
# metric exact, C3 fast / exact (dense XCD-segment refinement tail), C2 with the centre-relative homogeneous
# pinhole points on / off (2-view chunks) and round 3's per-sample 4-view chunks -- and the planar-prior timing.  Usage: bash scripts/r04_ab2.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab2}
V4=acmmp-spherical_amd/acmmp/libacmmp_pinvb4.so
mkdir -p $OUT
export ACMMP_TEST_REPORT_DIR=$OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_interp.py tests/test_gpu_fastmath.py -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_fast.log 2>&1
rc=$?
tail -1 $OUT/pytest_fast.log
if [ $rc -ne 0 ]; then
  grep -E "^E  |FAILED" $OUT/pytest_fast.log | head -20
  if [ $rc -ne 1 ]; then echo "fast-mode tests aborted rc=$rc"; exit 1; fi
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread --deselect tests/test_gpu_interp.py --deselect tests/test_gpu_fastmath.py > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^E  |FAILED" $OUT/pytest_gpu.log | head -20; tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line metric timeout -k 10 300 python bench.py $Q
  line metric_inline_fallback ACMMP_NB_FIX=0 timeout -k 10 300 python bench.py $Q
done
line metric_exact timeout -k 10 300 python bench.py $Q --math exact
line c3 timeout -k 10 400 python bench.py $C3 $Q
line c3_exact timeout -k 10 400 python bench.py $C3 $Q --math exact
for rep in 1 2; do
  line c2_homog2 timeout -k 10 300 python bench.py $C2 $Q
  line c2_sample2 ACMMP_PIN_HOMOG=0 timeout -k 10 300 python bench.py $C2 $Q
  line c2_sample4 ACMMP_LIB=$V4 ACMMP_PIN_HOMOG=0 timeout -k 10 300 python bench.py $C2 $Q
done
timeout -k 10 300 python scripts/planar_timing.py 2000 1500 sphere > $OUT/planar_2000x1500_sphere.json 2> $OUT/planar.err || { echo "planar timing failed"; tail -5 $OUT/planar.err; exit 1; }
timeout -k 10 300 python scripts/planar_timing.py 1600 1200 pinhole > $OUT/planar_1600x1200_pinhole.json 2>> $OUT/planar.err || { echo "planar timing failed"; tail -5 $OUT/planar.err; exit 1; }
cat $OUT/planar_*.json
echo AB2_DONE
