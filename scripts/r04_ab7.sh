#!/bin/bash
# Round-4 A/B (GPU box, repo root): refinement-tail chunk width -- C3 with 8-view SPHERE tail chunks
# (libacmmp_tailvb8) and C2 with 8-view pinhole tail chunks (libacmmp_tailpin8) against the product's 4,
# then a rocprofv3 kernel trace of C3.  Usage: bash scripts/r04_ab7.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04_ab7}
L=acmmp-spherical_amd/acmmp
mkdir -p $OUT
Q="--no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
C2="--model pinhole --width 1600 --height 1200 --n-src 10"
C3="--model sphere --width 3200 --height 1600 --n-src 15 --steps 3 --warmup 1"
line() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" > $OUT/b.json 2> $OUT/b.err || { echo "bench failed ($tag)"; tail -20 $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));print('$tag', d['math'], d['value'], d['ms_per_step'], d['roofline']['half_sweep_kernels_ms'])" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  line c3 timeout -k 10 400 python bench.py $C3 $Q
  line c3_tailvb8 ACMMP_LIB=$L/libacmmp_tailvb8.so timeout -k 10 400 python bench.py $C3 $Q
  line c2 timeout -k 10 300 python bench.py $C2 $Q
  line c2_tailpin8 ACMMP_LIB=$L/libacmmp_tailpin8.so timeout -k 10 300 python bench.py $C2 $Q
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py $C3 --timed-only $Q > $OUT/prof_c3.json 2> $OUT/prof_c3.err || { echo "rocprof failed"; tail -20 $OUT/prof_c3.err; exit 1; }
python3 - $OUT <<'PY' || exit 1
import csv, sys, os
out = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(out, "prof_c3", "run_kernel_stats.csv"))))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-60s calls %6s avg_ms %.4f total_ms %.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
echo AB7_DONE
