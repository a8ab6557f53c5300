#!/usr/bin/env python3
"""In-place Tx fill forms, interleaved in ONE process (experiments; not part of the product).

    python tools/tx_sweep.py --config TX2K --variants "split=0,store=0;split=0,store=1;split=1"

TX   = 1 M frames (synth.frames_host, payload <= 1460) back to back at CSR offsets;
TX2K = the same frames in a ring of 2048-byte slots (the send ring).
A variant sets split (0 = one-pass fill, 1 = read pass + scatter pass) and any
aipstack_chksum_tune keys (store = "tx_store", gather = "tx_gather", frames, stream, ...).
Every variant's first launch is checked against the frame oracle (filled bytes and statuses);
then rounds of `--reps` launches per variant, each bracketed by HIP events on the launch
stream. Prints one JSON line per variant: median / min us per fill, fraction of 8 TB/s of
the algorithmic bytes (frame bytes + 8 B offset or 4 B length + 1 B status + 4 B fields).

Sweep-only tunables (unroll, packets, nontemporal, frames) need a library built with
-DAIPSTACK_ALL_VARIANTS (tools/build_variant.sh), passed with --lib (tools/sweep_common.py).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import sweep_common  # noqa: E402

ALIAS = {"store": "tx_store", "gather": "tx_gather"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="TX2K", choices=["TX", "TX2K"])
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    if args.lib:
        os.environ["AIPSTACK_AMD_LIB"] = os.path.abspath(args.lib)
    import torch
    import aipstack_amd as A
    from aipstack_amd import _lib, synth
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    n = 1 << 20
    fbuf, off = synth.frames_host(n, seed=synth.SEED_DATA, max_payload=1460)
    orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    vp, u64 = ctypes.c_void_p, ctypes.c_uint64
    orc.oracle_tx_fill_batch.argtypes = [vp, vp, u64, vp]
    orc.oracle_tx_fill_slotted.argtypes = [vp, u64, vp, u64, vp]
    want_st = np.empty(n, dtype=np.uint8)
    frame_bytes = int(off[-1])
    if args.config == "TX":
        want = fbuf.copy()
        o64 = off.astype(np.uint64)
        orc.oracle_tx_fill_batch(want.ctypes.data, o64.ctypes.data, n, want_st.ctypes.data)
        d = torch.from_numpy(fbuf).to(dev)
        d_off = torch.from_numpy(off).to(dev)
        alg = frame_bytes + 8 * (n + 1) + n + 4 * n
    else:
        ring, lens = synth.to_slots(fbuf, off, 2048)
        want = ring.copy()
        orc.oracle_tx_fill_slotted(want.ctypes.data, 2048, lens.ctypes.data, n,
                                   want_st.ctypes.data)
        d = torch.from_numpy(ring).to(dev)
        d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
        alg = frame_bytes + 4 * n + n + 4 * n
        del ring
    del fbuf
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    ws = torch.empty(8 * n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()

    variants = []
    for spec in args.variants.split(";"):
        kv = dict(x.split("=") for x in spec.split(",") if x)
        variants.append({ALIAS.get(k, k): int(v) for k, v in kv.items()})

    sweep_common.require_variants(lib, variants)  # sweep-only keys need an ALL_VARIANTS build

    def apply(v):
        for k in ("tx_store", "tx_gather"):
            assert lib.aipstack_chksum_tune(k.encode(), v.get(k, -1)) == 0
        for k in ("frames", "stream", "waves_per_cu", "chunk_packets"):
            assert lib.aipstack_chksum_tune(k.encode(), v.get(k, 0)) == 0

    def launch(v):
        split = bool(v.get("split", 0))
        if args.config == "TX":
            A.tx_fill(d, d_off, out=out, stream=stream, split=split, workspace=ws)
        else:
            A.tx_fill_slotted(d, 2048, d_len, out=out, stream=stream, split=split, workspace=ws)

    parity = []
    for v in variants:
        apply(v)
        launch(v)
        torch.cuda.synchronize()
        parity.append(bool(np.array_equal(out.cpu().numpy(), want_st) and
                           np.array_equal(d.cpu().numpy(), want)))
    times = [[] for _ in variants]
    for _ in range(args.rounds):
        for i, v in enumerate(variants):
            apply(v)
            for _ in range(3):
                launch(v)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for s, e in ev:
                s.record(stream)
                launch(v)
                e.record(stream)
            torch.cuda.synchronize()
            times[i].extend(s.elapsed_time(e) * 1e3 for s, e in ev)
    apply({})
    for v, t, ok in zip(variants, times, parity):
        med = float(np.median(t))
        print(json.dumps({"config": args.config, **v, "median_us": round(med, 2),
                          "min_us": round(float(np.min(t)), 2),
                          "frac_8TBps": round(alg / med / 1e3 / 8000.0, 4), "parity": ok}),
              flush=True)


if __name__ == "__main__":
    main()
