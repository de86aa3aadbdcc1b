set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02_vchunk; mkdir -p $OUT
ACMMP_NB_VIEW_CHUNK=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_fastmath.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for cfg in "--width 3200 --height 1600 --n-src 15 --steps 2 --warmup 1" "--width 4096 --height 2048 --n-src 15 --steps 2 --warmup 1" "--model pinhole --width 1600 --height 1200 --n-src 10"; do
  for e in 0 4 8 5; do
    ACMMP_NB_VIEW_CHUNK=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));print('chunk=$e', '[$cfg]', d['value'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
  done
done
