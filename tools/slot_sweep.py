#!/usr/bin/env python3
"""Launch-parameter sweep of the ring-slot kernels (C2K: aipstack_chksum_batch_slotted over
config C's packets in 2048-B slots; RX2K: aipstack_chksum_rx_verify_slotted over the RX
frames), variants interleaved round by round in ONE process, every variant's output checked
equal to the first's. Not part of the product.

    python tools/slot_sweep.py --config C2K --variants "stream=-1;stream=2,chunk_packets=16"

A variant is a list of aipstack_chksum_tune keys (0 / absent = automatic). Prints one JSON
line per variant: median / min kernel us and payload GB/s.

Sweep-only tunables (unroll, packets, nontemporal, frames) need a library built with
-DAIPSTACK_ALL_VARIANTS (tools/build_variant.sh), passed with --lib (tools/sweep_common.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import sweep_common  # noqa: E402

KEYS = ("waves_per_cu", "chunks_per_wave", "unroll", "packets", "frames", "stream",
        "chunk_packets", "tx_gather")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2K", choices=["C2K", "A2K", "RX2K"])
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--lib", default=None, help="another build of the library (experiments)")
    args = ap.parse_args()
    if args.lib:
        os.environ["AIPSTACK_AMD_LIB"] = os.path.abspath(args.lib)
    import torch
    import aipstack_amd as A
    from aipstack_amd import _lib, synth
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    if args.config == "C2K":
        buf, off = synth.mixed_batch(2 << 20)
    elif args.config == "A2K":  # 1 M x 1500 B in 2048-B slots (bench.py A2K's shape)
        n0 = 1 << 20
        buf = synth.random_bytes(42, n0 * 1500)
        off = np.arange(n0 + 1, dtype=np.int64) * 1500
    else:  # RX's frames, made valid by the frame oracle (as bench.py does; test infra)
        import ctypes
        buf, off = synth.frames_host(1 << 20, seed=synth.SEED_DATA, max_payload=1460)
        orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        orc.oracle_tx_fill_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]
        o64 = off.astype(np.uint64)
        st = np.empty(off.size - 1, dtype=np.uint8)
        orc.oracle_tx_fill_batch(buf.ctypes.data, o64.ctypes.data, off.size - 1, st.ctypes.data)
    ring, lens = synth.to_slots(buf, off, 2048)
    payload = int(lens.sum(dtype=np.uint64))
    d_ring = torch.from_numpy(ring).to(dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
    del buf, ring
    n = lens.size
    out = (torch.empty(n, dtype=torch.uint16, device=dev) if args.config != "RX2K"
           else torch.empty(n, dtype=torch.uint8, device=dev))
    stream = torch.cuda.current_stream()

    def launch():
        if args.config != "RX2K":
            A.chksum_batch_slotted(d_ring, 2048, d_lens, out=out, stream=stream)
        else:
            A.rx_verify_slotted(d_ring, 2048, d_lens, out=out, stream=stream)

    variants = []
    for spec in args.variants.split(";"):
        kv = dict(x.split("=") for x in spec.split(",") if x)
        variants.append({k: int(v) for k, v in kv.items()})

    sweep_common.require_variants(lib, variants)  # sweep-only keys need an ALL_VARIANTS build

    def apply(v):
        for k in KEYS:
            assert lib.aipstack_chksum_tune(k.encode(), v.get(k, -1 if k == "tx_gather" else 0)) == 0

    times = [[] for _ in variants]
    ref = None
    for r in range(args.rounds):
        for i, v in enumerate(variants):
            apply(v)
            launch()
            torch.cuda.synchronize()
            if r == 0:
                got = out.cpu().numpy().copy()
                if ref is None:
                    ref = got
                elif not np.array_equal(got, ref):
                    raise SystemExit(f"variant {v} differs from variant {variants[0]}")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                launch()
            e1.record(stream)
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) * 1e3 / args.reps)
    apply({})
    for v, t in zip(variants, times):
        t = sorted(t[1:])  # the first round warms up
        print(json.dumps({"config": args.config, "variant": v, "us_median": round(t[len(t) // 2], 2),
                          "us_min": round(t[0], 2),
                          "payload_GBps": round(payload / (t[len(t) // 2] * 1e-6) / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
