#!/usr/bin/env python3
"""Measure the fast mode's T2 figures in geom / planar-prior / hierarchy passes:
after one half-sweep from the shared exact first-pass state, the share of pixels whose fast-mode plane equals
the exact mode's and the median |cost gap| of the flips, for seeds 72-75, on the pinhole, SPHERE and
interpolating SPHERE rigs of tests/test_gpu_fastmath.py.  Writes the JSON the test reads its floors from
(floor = four-seed mean - 0.5 pt; geom flip-gap bound = 2 x the largest measured median, at least 1e-4).

  python scripts/pass_gates.py [--out profiles/r06_pass_gates.json]   (GPU box, repo root)
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))

import numpy as np  # noqa: E402

import test_gpu_fastmath as T  # noqa: E402
from acmmp import capi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r06_pass_gates.json"))
    a = ap.parse_args()
    ctx = capi.Context(0)
    measured = {}
    for rig in T.PASS_RIGS:
        r = T.make_pass_rig(ctx, rig)
        measured[rig] = {}
        for kind in ("geom", "planar", "hierarchy"):
            setup = T.pass_setup(kind, *r[1:])
            got = [T.check_t2(ctx, setup, seed, rig.startswith("sphere"), init=False, hs_min=0.0, gap_max=None)
                   for seed in T.PASS_SEEDS]
            same = [g[0] for g in got]
            gaps = [g[1] for g in got]
            m = {"same_plane": same, "same_plane_mean": float(np.mean(same)), "same_plane_min": float(np.min(same)),
                 "flip_median_cost_gap": gaps}
            if kind == "geom":
                m["gap_bound"] = float(max(1e-4, 2.0 * max(gaps)))
            measured[rig][kind] = m
            print(rig, kind, json.dumps(m), flush=True)
    ctx.close()
    out = {"what": "fast vs exact after one half-sweep of a geom / planar / hierarchy pass from the exact first "
                   "pass's state (tests/test_gpu_fastmath.py PASS_RIGS, pass_setup); same_plane = share of pixels "
                   "with |fast - exact| <= 1e-4 max(1, |exact|) in every plane component",
           "seeds": list(T.PASS_SEEDS), "floor_rule": "same_plane_mean - 0.005 per (rig, kind), every seed",
           "geom_gap_rule": "max(1e-4, 2 x the largest seed's median flip gap)", "measured": measured}
    json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
