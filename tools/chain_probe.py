"""Where CHAIN's extra traffic comes from (round 4): the chained batch over layouts that
differ in one thing each, five launches per layout, in a fixed order, so that a
`rocprofv3 --pmc FETCH_SIZE --kernel-trace` run of this script gives each layout's fetched
bytes per launch (tools/chain_probe.py --summarize <counter_collection.csv> pairs them up).

Layouts (n chains, 1460 payload bytes each, payloads back to back as in bench.py CHAIN):
  bench      20-B header node at a 32-B stride + the payload split in two (bench.py)
  hdr128     the same with one header per 128-B line
  hdr20      headers packed at a 20-B stride
  nohdr      the split payload alone (2 chunks per chain)
  whole      the payload as one chunk
  hdr_whole  32-B-stride header + the payload as one chunk
  nostate    bench without the pseudo-header states
  csr        the payloads as a CSR batch (chksum_batch_csr, stream mode): the same bytes
             without the gathered stream, for comparison
Launch variants (4 windows, nontemporal loads, short chunks first) come from the
environment (AIPSTACK_CHKSUM_*), as for bench.py.
Every launch is checked against the first launch of its layout (equal outputs); the
oracle check of the product is bench.py --config CHAIN.
"""
import argparse
import csv
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

LAYOUTS = ["bench", "hdr128", "hdr20", "nohdr", "whole", "hdr_whole", "nostate", "csr"]
PAYLOAD, HDR = 1460, 20


def tables(layout, n, base, rng):
    if layout == "csr":
        offsets = PAYLOAD * np.arange(n + 1, dtype=np.uint64)
        return offsets, None, None, None, PAYLOAD * n + 8 * (n + 1) + 2 * n, PAYLOAD * n
    stride = {"hdr128": 128, "hdr20": 20}.get(layout, 32)
    has_hdr = layout not in ("nohdr", "whole")
    split = layout not in ("whole", "hdr_whole")
    hdr_bytes = stride * n if has_hdr else 0
    pay = base + hdr_bytes + PAYLOAD * np.arange(n, dtype=np.uint64)
    per = (1 if has_hdr else 0) + (2 if split else 1)
    addr = np.empty(per * n, dtype=np.uint64)
    lens = np.empty(per * n, dtype=np.uint32)
    k = 0
    if has_hdr:
        addr[0::per] = base + stride * np.arange(n, dtype=np.uint64)
        lens[0::per] = HDR
        k = 1
    if split:
        cut = rng.integers(1, PAYLOAD, n).astype(np.uint64)
        addr[k::per], lens[k::per] = pay, cut
        addr[k + 1::per], lens[k + 1::per] = pay + cut, PAYLOAD - cut
    else:
        addr[k::per], lens[k::per] = pay, PAYLOAD
    index = np.arange(n + 1, dtype=np.uint64) * per
    alg = int(lens.sum(dtype=np.uint64)) + 12 * per * n + 8 * (n + 1) + 2 * n
    states = None if layout == "nostate" else rng.integers(0, 1 << 32, n, dtype=np.uint64)
    if states is not None:
        alg += 4 * n
    return addr, lens, index, states, alg, hdr_bytes + PAYLOAD * n


def run(n, reps, layouts):
    import torch
    from aipstack_amd import chksum, synth
    dev = torch.device("cuda:0")
    buf = torch.empty(128 * n + PAYLOAD * n, dtype=torch.uint8, device=dev)
    synth.fill_device(buf, 7)
    rng = np.random.default_rng(7)
    for layout in layouts:
        addr, lens, index, states, alg, span = tables(layout, n, buf.data_ptr(), rng)
        if layout == "csr":
            offs = torch.from_numpy(addr.view(np.int64)).to(dev)
            pay = buf[:PAYLOAD * n]
            launch = lambda: chksum.chksum_batch_csr(pay, offs, final=True)  # noqa: E731
        else:
            launch = None
        if launch is None:
            t_addr = torch.from_numpy(addr.view(np.int64)).to(dev)
            t_len = torch.from_numpy(lens.view(np.int32)).to(dev)
            t_idx = torch.from_numpy(index.view(np.int64)).to(dev)
            t_st = None if states is None else \
                torch.from_numpy(states.astype(np.uint32).view(np.int32)).to(dev)
            launch = lambda: chksum.chksum_batch_chain(  # noqa: E731
                t_addr, t_len, t_idx, t_st, final=True)
        torch.cuda.synchronize()
        first, ms = None, []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = launch()
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
            if first is None:
                first = out.clone()
            elif not torch.equal(out, first):
                raise SystemExit(f"{layout}: launches disagree")
        print(json.dumps({"layout": layout, "n": n, "alg_bytes": alg, "span_bytes": span,
                          "us_median": float(np.median(ms[1:])) * 1e3, "reps": reps}), flush=True)


def summarize(counter_csv, jsonl):
    lines = [json.loads(x) for x in open(jsonl) if x.startswith("{")]
    rows = [r for r in csv.DictReader(open(counter_csv))
            if ("chksum_chain_kernel" in r["Kernel_Name"] or "chksum_batch_kernel" in r["Kernel_Name"])
            and r["Counter_Name"] == "FETCH_SIZE"]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    fetch = [float(r["Counter_Value"]) * 2 * 1024 for r in rows]  # gfx950: x2, KiB
    if len(fetch) != sum(ln["reps"] for ln in lines):
        raise SystemExit(f"{len(fetch)} dispatches for {len(lines)} layouts")
    i0 = 0
    for ln in lines:
        mine = sorted(fetch[i0 + 1:i0 + ln["reps"]])  # the first (cold) launch excluded
        i0 += ln["reps"]
        f = mine[len(mine) // 2]
        ln["fetch_bytes"] = f
        ln["fetch_over_alg"] = f / ln["alg_bytes"]
        print(json.dumps(ln))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layouts", default=",".join(LAYOUTS))
    ap.add_argument("--summarize", nargs=2, metavar=("COUNTER_CSV", "PROBE_JSONL"))
    a = ap.parse_args()
    if a.summarize:
        summarize(*a.summarize)
    else:
        run(a.n, a.reps, a.layouts.split(","))
        sys.exit(0)
