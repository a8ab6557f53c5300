#!/usr/bin/env python3
"""Summarise tools/pmc_run.sh output into profiles/pmc_traffic.json (read by bench.py).

For each config directory <round>/pmc_<CFG>/{fetch,write,sq1,sq2}/run_counter_collection.csv
this takes, per counter, the median over the hot-path kernel's dispatches (excluding the
first, cold, dispatch), and applies the correction of MI355X_MICROARCH.md's HBM section:

    hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

(FETCH_SIZE is in KiB and counts wide streaming reads at half rate on gfx950.) The
algorithmic bytes per launch come from the same round's bench_<CFG>.json, so
`ratio` = measured / algorithmic HBM bytes (1.0 = no re-reads).

    python tools/pmc_summary.py gpurun_out/r01b profiles/pmc_traffic.json

Run it on the tree the counters were taken on: every entry records the digest of the kernel
sources (bench.kernel_source_digest) and of the library's device code (bench.device_code_digest:
the .hip_fatbin section of libaipstack_chksum.so), and bench.py reports an entry's traffic only
while the device code still matches; before that, while the
sources still match (else null, with the old value under roofline.traffic_stale). Existing
entries of other configs are kept.
"""
import csv
import glob
import json
import os
import statistics
import sys

HOT_KERNELS = ("chksum_batch_kernel", "chksum_chain_kernel", "frame_kernel",
               "tx_scatter_kernel")  # split Tx fill: read pass + scatter pass, summed
COUNTERS = ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_SALU", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES",
            "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")


def per_dispatch(csv_path):
    """{(hot kernel, counter): [value per dispatch of that kernel, in dispatch order]}"""
    acc = {}
    with open(csv_path) as f:
        for row in csv.DictReader(f):
            kern = next((k for k in HOT_KERNELS if k in row["Kernel_Name"]), None)
            if kern is None:
                continue
            key = (kern, int(row["Dispatch_Id"]), row["Counter_Name"])
            acc[key] = acc.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (kern, disp, name), v in sorted(acc.items()):
        out.setdefault((kern, name), []).append(v)
    return out


def summarise(round_dir, cfg):
    vals = {}
    for path in glob.glob(os.path.join(round_dir, f"pmc_{cfg}", "*", "run_counter_collection.csv")):
        for (kern, name), series in per_dispatch(path).items():  # a step's kernels summed
            warm = series[1:] if len(series) > 1 else series
            vals[name] = vals.get(name, 0.0) + statistics.median(warm)
    if "FETCH_SIZE" not in vals or "WRITE_SIZE" not in vals:
        return None
    hbm = int(round((2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024))
    rec = {"hbm_bytes_per_launch": hbm}
    bench = os.path.join(round_dir, f"bench_{cfg}.json")
    if os.path.exists(bench):
        with open(bench) as f:
            alg = json.load(f)["roofline"].get("algorithmic_bytes_per_launch")
        if alg:
            rec["algorithmic_bytes_per_launch"] = alg
            rec["ratio"] = round(hbm / alg, 4)
    rec["FETCH_SIZE_KiB"] = vals["FETCH_SIZE"]
    rec["WRITE_SIZE_KiB"] = vals["WRITE_SIZE"]
    for c in COUNTERS[2:]:
        if c in vals:
            rec[c] = vals[c]
    return rec


def main():
    round_dir, out_path = sys.argv[1], sys.argv[2]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import device_code_digest, kernel_source_digest  # the kernels measured
    digest = kernel_source_digest()
    code = device_code_digest()
    merge = os.path.exists(out_path)
    doc = {
        "source": f"tools/pmc_run.sh on MI355X ({round_dir}); median over dispatches "
                  "excluding the first",
        "formula": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024  (FETCH_SIZE x2: "
                   "gfx950 half-count for wide streaming reads, MI355X_MICROARCH.md HBM)",
    }
    if merge:  # keep the other configs' entries; replace the ones measured here
        with open(out_path) as f:
            old = json.load(f)
        doc = {**old, "source": doc["source"], "formula": doc["formula"]}
    for d in sorted(glob.glob(os.path.join(round_dir, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        cfg = os.path.basename(d)[len("pmc_"):]
        rec = summarise(round_dir, cfg)
        if rec:
            rec["kernel_sources"] = digest
            rec["device_code"] = code
            rec["measured_in"] = round_dir
            doc[cfg] = rec
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    for k, v in doc.items():
        if isinstance(v, dict):
            print(k, v["hbm_bytes_per_launch"], v.get("ratio"))


if __name__ == "__main__":
    main()
