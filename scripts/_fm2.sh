set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02_fm2; mkdir -p $OUT
L=acmmp-spherical_amd/acmmp
for rep in 1 2; do
for cfg in "libacmmp.so exact" "libacmmp.so fast" "libacmmp_nbpipe.so fast" "libacmmp_nbw6.so fast" "libacmmp_nbpipe.so exact"; do
  set -- $cfg
  ACMMP_LIB=$L/$1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --math $2 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$1 $2', d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'], d['stages_ms']['init'])"
done
done
bash scripts/pmc.sh $OUT/pmc_fast "--steps 1 --warmup 0 --no-cpu-baseline --no-variant --no-pipeline --math fast" && python scripts/pmc_summary.py $OUT/pmc_fast > $OUT/pmc_fast_summary.txt && cat $OUT/pmc_fast_summary.txt | head -60
