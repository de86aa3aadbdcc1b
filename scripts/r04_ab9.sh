#!/bin/bash
# Round-4 A/B (GPU box, repo root): homogeneous pinhole points in the unstaged fast chunks (k_init, the
# refinement tail, the per-sample hook) against libacmmp_hs0off (per-sample points there), at C2 and C5,
# then the pinhole fast-mode gates and per-query tests.  Usage: bash scripts/r04_ab9.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab9}
L=acmmp-spherical_amd/acmmp
mkdir -p $OUT
export ACMMP_TEST_REPORT_DIR=$OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
C5="--model pinhole --width 1920 --height 1080 --n-src 20"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['stages_ms'] if 'stages_ms' in d else '', d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line c2 timeout -k 10 300 python bench.py $C2 $Q
  line c2_hs0off ACMMP_LIB=$L/libacmmp_hs0off.so timeout -k 10 300 python bench.py $C2 $Q
done
line c5 timeout -k 10 300 python bench.py $C5 $Q
line c5_hs0off ACMMP_LIB=$L/libacmmp_hs0off.so timeout -k 10 300 python bench.py $C5 $Q
timeout -k 10 900 python -u -m pytest tests/test_gpu_fastmath.py tests/test_gpu_interp.py -k "pinhole or c2 or c5" -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_pin.log 2>&1
rc=$?
tail -1 $OUT/pytest_pin.log
grep -E "^E  |FAILED" $OUT/pytest_pin.log | cut -c1-300 | head -20
echo AB9_DONE rc=$rc
