#!/usr/bin/env python3
"""Summaries of a gpurun_out/<tag> directory: sweep medians, kernel-trace per-launch times,
PMC medians per kernel. Usage: python tools/summ.py gpurun_out/r02q"""
import collections, csv, glob, json, os, statistics, sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "sweep_*.jsonl"))):
    rows = [json.loads(l) for l in open(f)]
    print("%-28s" % os.path.basename(f),
          " ".join("%7.2f/%7.2f %s" % (r["median_us"], r["min_us"], "ok" if r["parity"] else "BAD")
                   for r in rows), " frac", " ".join("%.3f" % r["frac_8TBps"] for r in rows))
for f in sorted(glob.glob(os.path.join(d, "*", "run_kernel_trace.csv"))):
    if "pmc" in f or "sq" in os.path.basename(os.path.dirname(f)):
        continue
    ks = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        ks[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in ks.items():
        if len(v) > 3:
            name = k.split("::")[-1][:40]
            print(os.path.basename(os.path.dirname(f)), name, "n=%d avg=%.1f" % (len(v), sum(v) / len(v)),
                  " ".join("%.0f" % x for x in v))
for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    nm = {}
    for r in csv.DictReader(open(f)):
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        nm[r["Dispatch_Id"]] = r["Kernel_Name"]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for di, cc in agg.items():
        for k, v in cc.items():
            per[nm[di]][k].append(v)
    for k, cc in per.items():
        if "synth" in k:
            continue
        print(os.path.basename(os.path.dirname(f)), k.split("::")[-1][:40],
              {a: "%.4g" % statistics.median(b) for a, b in cc.items()})
