"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch for each kernel."""
import csv
import glob
import json
import sys
from collections import defaultdict


def summarize(root):
    per = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(f"{root}/p*/run_counter_collection.csv"):
        rows = list(csv.DictReader(open(path)))
        acc = defaultdict(float)
        keyname = {}
        for r in rows:
            k = (r["Dispatch_Id"], r["Counter_Name"])
            acc[k] += float(r["Counter_Value"])
            keyname[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in acc.items():
            per[keyname[d]][c].append(v)
    out = {}
    for kern, cs in per.items():
        out[kern] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[kern]["_dispatches"] = max(len(v) for v in cs.values())
    return out


if __name__ == "__main__":
    s = summarize(sys.argv[1])
    for k, v in s.items():
        if "propagate" in k or len(sys.argv) > 2:
            print(k)
            for c, val in sorted(v.items()):
                print(f"   {c:28s} {val:,.0f}")
