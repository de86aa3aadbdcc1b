#!/bin/bash
# A/B of library builds on the GPU box: bit-identity of BASE and CAND (scripts/ab_bitident.py), alternated bench lines
# of every library in LIBS (ACMMP_LIB selects one; scripts/build_variants.py builds them), then the product's planar-prior
# timing and end-to-end line.  Usage: bash scripts/ab_libs.sh TAG BASE CAND "LIBS" "CONFIG1" ...   (CONFIG "" = metric)
set -o pipefail
export TMPDIR=/tmp
export ACMMP_KERNEL_TIMING=all   # every half-sweep bucket timed (the same event overhead in every library's line)
TAG=$1; BASE=$2; CAND=$3; LIBS=$4; shift 4
OUT=gpurun_out/$TAG; mkdir -p $OUT
ACMMP_LIB=$BASE timeout -k 10 300 python scripts/ab_bitident.py run $OUT/base.npz > $OUT/bit.log 2>&1 || { tail $OUT/bit.log; exit 1; }
ACMMP_LIB=$CAND timeout -k 10 300 python scripts/ab_bitident.py run $OUT/cand.npz >> $OUT/bit.log 2>&1 || { tail $OUT/bit.log; exit 1; }
python scripts/ab_bitident.py cmp $OUT/base.npz $OUT/cand.npz | tail -9
rm -f $OUT/base.npz $OUT/cand.npz
for cfg in "$@"; do
  for rep in 1 2; do
    for lib in $LIBS; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));print(os.path.basename('$lib'), '$cfg', d['value'], d['ms_per_step'], d['clock']['ghz'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
    done
  done
done
timeout -k 10 200 python scripts/planar_timing.py 2000 1500 sphere > $OUT/planar_sphere.json || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --no-variant --no-other-mode > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], json.dumps(d['end_to_end']['stages_s']))"
echo AB_DONE
