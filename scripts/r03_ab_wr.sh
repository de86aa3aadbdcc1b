#!/bin/bash
# A/B: product build vs libacmmp_wr.so (the interpolated k_eval_nb without the per-sample view guard): bit
# identity, GPU tests with the variant, alternating fast-mode bench lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_ab_wr
mkdir -p $OUT
L=$PWD/acmmp-spherical_amd/acmmp
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
for lib in libacmmp.so libacmmp_wr.so; do
  ACMMP_LIB=$L/$lib timeout -k 10 300 python scripts/ab_bitident.py run /tmp/$lib.npz || { echo "run failed $lib"; exit 1; }
done
python scripts/ab_bitident.py cmp /tmp/libacmmp.so.npz /tmp/libacmmp_wr.so.npz | tee $OUT/bitident.txt
ACMMP_LIB=$L/libacmmp_wr.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_g.log 2>&1 || { echo "pytest g failed"; grep -E "FAILED|ERROR" $OUT/pytest_g.log | head -5; tail -30 $OUT/pytest_g.log; exit 1; }
tail -1 $OUT/pytest_g.log
for rep in 1 2; do
  for lib in libacmmp.so libacmmp_wr.so; do
    ACMMP_LIB=$L/$lib timeout -k 10 300 python bench.py $Q --math fast > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$lib', 'fast', d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
  done
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" && echo SMOKE_OK
echo AB_DONE
