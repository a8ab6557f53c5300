#!/usr/bin/env python3
"""One line per bench_<CFG>.json of a measurement directory: kernel us, frac, slot-ceiling
frac, traffic, parity, CPU baseline. Not part of the product.
    python tools/summ_bench.py gpurun_out/r03a"""
import glob
import json
import os
import sys

for p in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    try:
        d = json.loads(open(p).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        print(os.path.basename(p), "no line")
        continue
    r = d["roofline"]
    cpu = d.get("cpu_baseline") or {}
    print(f"{d['config']['config']:6s} {r['kernel_us']:8.2f} us  frac {r['frac']:.4f}  "
          f"slotfrac {r.get('frac_of_slot_read_ceiling')}  value {d['value']} GiB/s  "
          f"traffic {r.get('traffic')}  cpu1 {cpu.get('value')} all {cpu.get('all_cores', {}).get('value')}  "
          f"{(d.get('parity') or '')[:50]}")
