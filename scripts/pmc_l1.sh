#!/bin/bash
# The L1 (TCP) pass alone for the metric, C2 and C3 bench configs: L1 hit rate and mean L2 read latency per kernel
# (scripts/pmc_summary.py derives them).  Usage (GPU box, repo root): bash scripts/pmc_l1.sh TAG
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_l1}
mkdir -p $OUT
Q="--steps 1 --warmup 1 --timed-only --no-cpu-baseline --no-variant --no-pipeline --no-other-mode"
for cfg in "metric|" "c2|--model pinhole --width 1600 --height 1200 --n-src 10" "c3|--model sphere --width 3200 --height 1600 --n-src 15"; do
  name=${cfg%%|*}; args=${cfg#*|}
  timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum \
    --output-format csv -d $OUT/$name/p1 -o run -- python3 bench.py $args $Q > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -20 $OUT/$name.log; exit 1; }
  python scripts/pmc_summary.py $OUT/$name > $OUT/${name}_summary.txt || exit 1
  python - "$OUT/${name}_summary.txt" "$name" <<'PY'
import sys, re
txt = open(sys.argv[1]).read()
for blk in re.split(r"\n(?=\S)", txt):
    lines = blk.strip().split("\n")
    if not lines or not any(k in lines[0] for k in ("k_eval_nb", "k_eval_ref", "k_select", "k_init", "k_nb_fix")):
        continue
    v = {l.split()[0]: float(l.split()[1].replace(",", "")) for l in lines[1:] if len(l.split()) == 2}
    acc, req = v.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0), v.get("TCP_TCC_READ_REQ_sum", 0)
    lat = v.get("TCP_TCC_READ_REQ_LATENCY_sum", 0)
    print(sys.argv[2], lines[0][:40], "L1 hit %.3f" % (1 - req / acc if acc else 0), "L2 read latency %.0f cyc" % (lat / req if req else 0))
PY
done
echo PMC_L1_DONE
