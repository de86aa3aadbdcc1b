#!/usr/bin/env python3
"""Recompute bench.py's roofline from a rocprofv3 kernel trace (reproducibility of the bench line).

The profiled command is `bench.py --timed-only ...`: after its W warmup and K timed RunPatchMatch calls
nothing else runs, so the last `launches` dispatches of the dominant kernel in the trace are exactly the
ones bench.py timed with HIP events (which also bracket k_nb_fix, reported beside it).  This prints (and with --json writes) their mean duration, the
all-dispatch mean rocprofv3's --stats reports, and roofline.frac recomputed from the bench line's
algorithmic FLOP per launch -- to compare with the line's own frac.

  python scripts/trace_window.py TRACE.csv BENCH.json [--kernel k_eval_nb] [--json OUT]
"""
import argparse
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--kernel", default="k_eval_nb")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    line = None
    for ln in open(a.bench):
        if ln.startswith("{"):
            line = json.loads(ln)
    rf = line["roofline"]
    rows = [r for r in csv.DictReader(open(a.trace)) if re.search(rf"\b{a.kernel}\b", r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]
    n = int(rf["launches"])
    win = dur[-n:]
    win_ms = sum(win) / len(win)
    all_ms = sum(dur) / len(dur)
    flop = float(rf["flop_per_launch"])
    peak = float(rf["peak"])
    # the bench's events bracket launch_eval_nb, which ends with k_nb_fix (the deferred interpolation
    # fallbacks, one dispatch per half-sweep when the fast SPHERE path interpolates): add its window
    fix = [r for r in csv.DictReader(open(a.trace)) if re.search(r"\bk_nb_fix\b", r["Kernel_Name"])]
    fix.sort(key=lambda r: int(r["Start_Timestamp"]))
    fix_dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in fix]
    fix_ms = sum(fix_dur[-n:]) / n if len(fix_dur) >= n else 0.0
    out = {"kernel": a.kernel, "dispatches_in_trace": len(dur), "timed_window": n,
           "k_nb_fix_window_mean_ms": round(fix_ms, 4),
           "window_with_fix_mean_ms": round(win_ms + fix_ms, 4),
           "window_with_fix_vs_events": round((win_ms + fix_ms) / rf["launch_ms"] - 1.0, 4),
           "frac_from_trace_window_with_fix": round(flop / ((win_ms + fix_ms) * 1e-3) / 1e12 / peak, 4),
           "window_mean_ms": round(win_ms, 4), "all_dispatch_mean_ms": round(all_ms, 4),
           "bench_event_mean_ms": rf["launch_ms"],
           "frac_from_trace_window": round(flop / (win_ms * 1e-3) / 1e12 / peak, 4),
           "frac_from_all_dispatches": round(flop / (all_ms * 1e-3) / 1e12 / peak, 4),
           "frac_bench_line": rf["frac"],
           "window_vs_events": round(win_ms / rf["launch_ms"] - 1.0, 4)}
    print(json.dumps(out, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
