#!/bin/bash
# Round-4 check of the working tree (GPU box, repo root): the per-query and fast-mode tests first (with
# their reports), the whole GPU suite, then bench lines: C2 with the homogeneous pinhole points on / off
# (ACMMP_PIN_HOMOG) and with 2-view fast pinhole chunks (variant lib), C3 (the XCD-strip refinement tail),
# and the default line.  Usage: bash scripts/r04_pin.sh TAG [VARIANT_LIBS]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_pin}
VARS=${2:-acmmp-spherical_amd/acmmp/libacmmp_pinvb2.so}
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
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line c2_homog timeout -k 10 300 python bench.py $C2 $Q
  line c2_per_sample ACMMP_PIN_HOMOG=0 timeout -k 10 300 python bench.py $C2 $Q
  for lib in $VARS; do line c2_$(basename $lib .so) ACMMP_LIB=$lib timeout -k 10 300 python bench.py $C2 $Q; done
done
line c2_exact timeout -k 10 300 python bench.py $C2 $Q --math exact
line c3 timeout -k 10 400 python bench.py --model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1 $Q
line c3_exact timeout -k 10 400 python bench.py --model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1 $Q --math exact
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
echo PIN_DONE
