#!/bin/bash
# Re-entry check of the committed build (GPU tests + bench line) and the A/B of the interpolated k_eval_nb
# forms (bit identity against the committed build, then alternating fast-mode bench lines).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_ab_interp
mkdir -p $OUT
L=acmmp-spherical_amd/acmmp
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for lib in libacmmp.so libacmmp_f1.so libacmmp_f2.so; do
  ACMMP_LIB=$PWD/$L/$lib timeout -k 10 300 python scripts/ab_bitident.py run /tmp/$lib.npz || { echo "run failed $lib"; exit 1; }
done
python scripts/ab_bitident.py cmp /tmp/libacmmp.so.npz /tmp/libacmmp_f1.so.npz /tmp/libacmmp_f2.so.npz | tee $OUT/bitident.txt
for rep in 1 2; do
  for lib in libacmmp.so libacmmp_f1.so libacmmp_f2.so; do
    ACMMP_LIB=$PWD/$L/$lib timeout -k 10 300 python bench.py $Q --math fast > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$lib', 'fast', d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
  done
done
echo AB_DONE
