#!/bin/bash
# Round-5 A/B: bit identity of library variants (scripts/ab_bitident.py), then bench lines per variant and
# config, interleaved, REPS times.  Usage: bash scripts/r05_ab.sh TAG "LIB1 LIB2 ..." REPS "CFG1" "CFG2" ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; REPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -z "$NO_BITIDENT" ]; then
  NP=""
  for lib in $LIBS; do
    n=$(basename $lib .so)
    ACMMP_LIB=$lib timeout -k 10 400 python scripts/ab_bitident.py run $OUT/$n.npz --math fast > $OUT/bi_$n.log 2>&1 || { echo "bitident $n failed"; tail $OUT/bi_$n.log; exit 1; }
    NP="$NP $OUT/$n.npz"
  done
  python scripts/ab_bitident.py cmp $NP | tee $OUT/bitident.txt
  rm -f $NP                                            # (large: gpurun copies back at most 64 MiB)
fi
for cfg in "$@"; do
  for r in $(seq $REPS); do
    for lib in $LIBS; do
      ACMMP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-variant --no-pipeline --no-other-mode $cfg > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json,os;d=json.load(open('$OUT/b.json'));r=d['roofline'];print(os.path.basename('$lib'), '$cfg', d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], r.get('half_sweep_kernels_ms'))" | tee -a $OUT/ab.txt
    done
  done
done
echo AB_DONE
