"""Summarise rocprofv3 --pmc CSVs (scripts/pmc.sh): mean counter value per dispatch for each kernel.

`--json OUT` also writes the traffic summary bench.py reads (profiles/pmc_propagate.json): HBM bytes
per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 -- rocprofv3 reports both in KiB, and on gfx950
FETCH_SIZE counts half the bytes of a wide read (MI355X_MICROARCH.md §HBM; cdna_hip_programming.md
§counter pitfalls).  Our reads are 8-byte-per-lane bilinear pairs and 16-byte state loads, so the x2
correction is the guide's prescription, not a calibration of this kernel.
"""
import argparse
import csv
import glob
import json
import re
from collections import defaultdict

SHORT = ("k_eval_nb", "k_select", "k_eval_ref", "k_eval_ref_tail", "k_pick", "k_finish", "k_init", "k_merge", "k_filter", "k_pad_image",
         "k_ray_tables", "k_spatial", "k_jbu")


def short_name(kernel_name: str) -> str:
    for k in SHORT:
        if re.search(rf"\b{k}\b", kernel_name):
            return k
    return kernel_name


def summarize(root):
    per = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
        rows = list(csv.DictReader(open(path)))
        acc = defaultdict(float)
        keyname, dur = {}, {}
        for r in rows:
            k = (r["Dispatch_Id"], r["Counter_Name"])
            acc[k] += float(r["Counter_Value"])
            keyname[r["Dispatch_Id"]] = r["Kernel_Name"]
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur[r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for (d, c), v in acc.items():
            per[short_name(keyname[d])][c].append(v)
            # the dispatch's effective shader clock: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / duration
            # (MI355X_MICROARCH.md "DVFS give-back"; reads high below ~0.3 ms dispatches)
            if c == "GRBM_GUI_ACTIVE" and dur.get(d, 0) > 0:
                per[short_name(keyname[d])]["effective_clock_ghz"].append(v / 8.0 / dur[d])
    out = {}
    for kern, cs in per.items():
        out[kern] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[kern]["_dispatches"] = max(len(v) for v in cs.values())
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    ap.add_argument("--width", type=int, default=2000)
    ap.add_argument("--height", type=int, default=1500)
    ap.add_argument("--n-src", type=int, default=4)
    ap.add_argument("--model", default="sphere")
    ap.add_argument("--math", default="fast")
    a = ap.parse_args()
    s = summarize(a.root)
    for k, v in sorted(s.items()):
        print(k)
        for c, val in sorted(v.items()):
            print(f"   {c:28s} {val:,.1f}")
    if a.json:
        kernels = {}
        for k, v in s.items():
            if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
                kernels[k] = {"FETCH_SIZE_KiB": v["FETCH_SIZE"], "WRITE_SIZE_KiB": v["WRITE_SIZE"],
                              "hbm_bytes_per_launch": (2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024.0,
                              "dispatches": v["_dispatches"]}
                for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                          "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "TCC_HIT", "TCC_MISS",
                          "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum", "TCP_TCC_READ_REQ_LATENCY_sum",
                          "TCP_PENDING_STALL_CYCLES_sum", "GRBM_GUI_ACTIVE", "effective_clock_ghz"):
                    if c in v:
                        kernels[k][c] = v[c]
                # SURVEY.md §8d's secondary gather roof: the L1 (TCP) hit rate -- the share of TCP accesses that
                # did not become an L2 read request -- and the mean L2 read latency the TCP saw
                if v.get("TCP_TOTAL_CACHE_ACCESSES_sum") and "TCP_TCC_READ_REQ_sum" in v:
                    kernels[k]["l1_hit_rate"] = 1.0 - v["TCP_TCC_READ_REQ_sum"] / v["TCP_TOTAL_CACHE_ACCESSES_sum"]
                if v.get("TCP_TCC_READ_REQ_sum") and "TCP_TCC_READ_REQ_LATENCY_sum" in v:
                    kernels[k]["l2_read_latency_cycles"] = v["TCP_TCC_READ_REQ_LATENCY_sum"] / v["TCP_TCC_READ_REQ_sum"]
                if "TCC_HIT" in v and "TCC_MISS" in v and v["TCC_HIT"] + v["TCC_MISS"] > 0:
                    kernels[k]["l2_hit_rate"] = v["TCC_HIT"] / (v["TCC_HIT"] + v["TCC_MISS"])
        json.dump({"config": {"width": a.width, "height": a.height, "n_src": a.n_src, "model": a.model, "math": a.math},
                   "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes per dispatch (gfx950 FETCH_SIZE counts 1/2)",
                   "kernels": kernels}, open(a.json, "w"), indent=1)
