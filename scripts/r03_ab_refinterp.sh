#!/bin/bash
# GPU tests of the product build; the interpolated fast SPHERE refinement (libacmmp_ri.so) through the fast-mode
# tests, the fast-mode floor and alternating bench lines; the C2 49-view schedule's stages (device-resident
# geom-pass state).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_ab_refinterp
mkdir -p $OUT
L=$PWD/acmmp-spherical_amd/acmmp
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -5; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
ACMMP_LIB=$L/libacmmp_ri.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fastmath.py tests/test_gpu_band.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ri.log 2>&1 || { echo "pytest ri failed"; grep -E "FAILED|ERROR" $OUT/pytest_ri.log | head -5; tail -30 $OUT/pytest_ri.log; }
tail -1 $OUT/pytest_ri.log
for rep in 1 2; do
  for lib in libacmmp.so libacmmp_ri.so; do
    ACMMP_LIB=$L/$lib timeout -k 10 300 python bench.py $Q --math fast > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$lib', 'fast', d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
  done
done
ACMMP_LIB=$L/libacmmp_ri.so timeout -k 10 400 python -u scripts/fastmath_floor.py --quick > $OUT/floor_ri.json 2> $OUT/floor_ri.err || { echo "floor failed"; tail -5 $OUT/floor_ri.err; }
timeout -k 10 500 python -u scripts/pipeline_bench.py --model pinhole --width 1600 --height 1200 --views 49 --n-src 10 > $OUT/c2_pipeline.json 2> $OUT/c2_pipeline.err || { echo "c2 pipeline failed"; tail -20 $OUT/c2_pipeline.err; exit 1; }
tail -c 600 $OUT/c2_pipeline.json
echo AB_DONE
