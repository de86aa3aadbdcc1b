set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/xcd
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/xcd/pytest.log 2>&1 || { tail -30 gpurun_out/xcd/pytest.log; exit 1; }
tail -2 gpurun_out/xcd/pytest.log
for cfg in "" "--width 3200 --height 1600 --n-src 15" "--model pinhole --width 1600 --height 1200 --n-src 10"; do
  for lib in acmmp-spherical_amd/acmmp/libacmmp.so acmmp-spherical_amd/acmmp/libacmmp_exp.so; do
    ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant $cfg > gpurun_out/xcd/b.json 2>gpurun_out/xcd/b.err || { tail gpurun_out/xcd/b.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/xcd/b.json'));print('$lib'[-16:], '$cfg', d['value'], d['ms_per_depth_map'], d['stages_ms']['init'], d['roofline']['half_sweep_kernels_ms'])"
  done
done
