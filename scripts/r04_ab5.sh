#!/bin/bash
# Round-4 check (GPU box, repo root): the deferred-fallback tests (queue only; forced fallbacks equal the
# per-sample fast arithmetic), bench lines -- metric, C2 against libacmmp_pinw6 (fast pinhole k_eval_nb at
# 6 waves per SIMD) -- then the whole GPU suite.  Usage: bash scripts/r04_ab5.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab5}
L=acmmp-spherical_amd/acmmp
mkdir -p $OUT
export ACMMP_TEST_REPORT_DIR=$OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_interp.py tests/test_gpu_fastmath.py -k deferred -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_deferred.log 2>&1
rc=$?
tail -1 $OUT/pytest_deferred.log
grep -E "^E  |FAILED" $OUT/pytest_deferred.log | cut -c1-300 | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "deferred tests aborted rc=$rc"; exit 1; fi
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line metric timeout -k 10 300 python bench.py $Q
  line c2 timeout -k 10 300 python bench.py $C2 $Q
  line c2_pinw6 ACMMP_LIB=$L/libacmmp_pinw6.so timeout -k 10 300 python bench.py $C2 $Q
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "^E  |FAILED" $OUT/pytest_gpu.log | cut -c1-300 | head -20; tail -3 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo AB5_DONE
