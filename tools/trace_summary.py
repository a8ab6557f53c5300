#!/usr/bin/env python3
"""Per-dispatch durations of the hot kernels in rocprofv3 kernel traces, as one JSON object
per trace directory: {"trace": dir, "kernel": name, "us": [...], "blocks_of_50": [...]}.
Not part of the product.

    python tools/trace_summary.py gpurun_out/r05/driver/tr_default [...] > per_launch.jsonl
"""
import csv
import json
import os
import statistics
import sys

HOT = ("chksum_batch_kernel", "chksum_chain_kernel", "frame_kernel")


def main():
    for d in sys.argv[1:]:
        path = os.path.join(d, "run_kernel_trace.csv")
        per = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                if any(h in k for h in HOT):
                    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
                    per.setdefault(k, []).append(round(us, 2))
        for k, us in per.items():
            blocks = [{"launches": f"{i}-{i + len(us[i:i + 50])}",
                       "mean": round(statistics.fmean(us[i:i + 50]), 2),
                       "min": min(us[i:i + 50])} for i in range(0, len(us), 50)]
            print(json.dumps({"trace": d, "kernel": k.split("(")[0], "n": len(us),
                              "mean": round(statistics.fmean(us), 2), "us": us,
                              "blocks_of_50": blocks}))


if __name__ == "__main__":
    main()
