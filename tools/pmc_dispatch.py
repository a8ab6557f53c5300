#!/usr/bin/env python3
"""Per-dispatch rocprofv3 counters of the checksum launches, first reads against later ones.

    python tools/pmc_dispatch.py DIR [DIR ...]

Each DIR is one `rocprofv3 --kernel-trace --pmc ... -- python3 bench.py --steps 20 --warmup 5`
output directory. For the kernel matching --kernel (default "chksum_batch"), prints per counter
the median over launches 1-3 (each rotation batch's first read after it was written) and over
launches 6-25 (the timed ones), with the dispatch duration. Not part of the product.
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def load(d, kernel):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None
    per = collections.OrderedDict()
    for r in csv.DictReader(open(f[0])):
        if kernel not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        e = per.setdefault(k, {})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        e["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    return list(per.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="chksum_batch")
    a = ap.parse_args()
    for d in a.dirs:
        rows = load(d, a.kernel)
        if not rows:
            print(json.dumps({"dir": d, "error": "no counters"}))
            continue
        first, timed = rows[:3], rows[5:25]
        out = {"dir": d, "launches": len(rows)}
        for c in rows[0]:
            out[c] = {"first3": round(statistics.median(r[c] for r in first), 3),
                      "timed": round(statistics.median(r[c] for r in timed), 3)}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
