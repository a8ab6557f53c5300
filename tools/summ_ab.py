#!/usr/bin/env python3
"""A/B summary of the bench lines tools/r04.sh appends per variant (<name>.jsonl in one
directory): per variant, the per-launch kernel times of its processes and their parity.
Not part of the product.
    python tools/summ_ab.py gpurun_out/r04/gather2 A_stream A_gather ..."""
import json
import os
import sys

d = sys.argv[1]
names = sys.argv[2:] or sorted(f[:-6] for f in os.listdir(d) if f.endswith(".jsonl"))
for n in names:
    p = os.path.join(d, n + ".jsonl")
    if not os.path.exists(p):
        print(f"{n:24s} missing")
        continue
    rows = []
    for line in open(p):
        if not line.startswith("{"):
            continue
        x = json.loads(line)
        r = x.get("roofline") or {}
        rows.append((r.get("kernel_us"), (x.get("parity") or "")[:9], x.get("value"),
                     x.get("ms_per_step")))
    us = [r[0] for r in rows if r[0] is not None]
    print(f"{n:24s} us {us}  parity {sorted({r[1] for r in rows})}  "
          f"value {[r[2] for r in rows]}")
