#!/usr/bin/env python3
"""Interleaved A/B timing of launch variants of the checksum batches, in ONE process.

Each variant is a set of library tunables (aipstack_chksum_tune); the variants take turns,
round by round (so clock and thermal drift hit them alike), each launch timed with its own
HIP event pair, over R rotated resident batches (bench.py's rotation: no launch finds its
bytes in the Infinity Cache). Every variant's output is checked equal to the oracle's on
every batch. One JSON object per variant on stdout. Not part of the product.

    python tools/ab.py --config A --variants "gather=0;gather=1;gather=1,lds_pad=33792"
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="A", choices=["A", "B", "C", "A2K", "C2K"])
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rotate", type=int, default=3)
    args = ap.parse_args()

    import torch
    import aipstack_amd as A
    from aipstack_amd import _lib, synth
    import bench

    lib = _lib.load()
    dev = torch.device("cuda", 0)
    layout, n, plen = bench.CONFIGS[args.config]
    spec = bench.shard_spec(args.config, 0, 1)
    stride = spec.get("stride", plen)
    total = spec["total"]
    bufs, wants = [], []
    d_off = torch.from_numpy(spec["offsets"]).to(dev) if layout == "csr" else None
    d_lens = None
    if layout == "csrslot":  # config C's packets in 2048-B ring slots, one ring per rotation
        orc = bench.ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        orc.oracle_batch_slotted.argtypes = [bench.ctypes.c_void_p, bench.ctypes.c_uint64,
                                             bench.ctypes.c_void_p, bench.ctypes.c_uint64,
                                             bench.ctypes.c_void_p, bench.ctypes.c_uint32]
        for r in range(args.rotate):
            sp = dict(spec, data_seed=synth.SEED_DATA + r)
            ring, lens = synth.to_slots(bench.host_shard(sp), spec["offsets"], 2048,
                                        slack_seed=99 + r)
            bufs.append(torch.from_numpy(ring).to(dev))
            w = np.empty(n, dtype=np.uint16)
            orc.oracle_batch_slotted(ring.ctypes.data, 2048, lens.ctypes.data, n, w.ctypes.data, 0)
            wants.append(w)
        d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
        total = int(lens.sum(dtype=np.uint64))
        spec["payload"] = total
    for r in range(args.rotate if layout != "csrslot" else 0):
        b = torch.empty(total, dtype=torch.uint8, device=dev)
        synth.fill_device(b, synth.SEED_DATA + r, spec["byte_offset"])
        if layout == "csr":
            synth.apply_classes_device(b, d_off, first_packet=spec["first_packet"])
        bufs.append(b)
        host = b.cpu().numpy()
        w = np.empty(n, dtype=np.uint16)
        orc = bench.ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        if layout == "csr":
            orc.oracle_batch_csr.argtypes = [bench.ctypes.c_void_p] * 2 + [
                bench.ctypes.c_uint64, bench.ctypes.c_void_p, bench.ctypes.c_uint32]
            o = spec["offsets"].astype(np.uint64)
            orc.oracle_batch_csr(host.ctypes.data, o.ctypes.data, n, w.ctypes.data, 0)
        else:
            orc.oracle_batch_strided.argtypes = [bench.ctypes.c_void_p, bench.ctypes.c_uint64,
                                                 bench.ctypes.c_uint32, bench.ctypes.c_uint64,
                                                 bench.ctypes.c_void_p, bench.ctypes.c_uint32]
            orc.oracle_batch_strided(host.ctypes.data, stride, plen, n, w.ctypes.data, 0)
        wants.append(w)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    stream = torch.cuda.current_stream()
    payload = spec.get("payload", total)
    alg = bench.algorithmic_bytes(layout, n, payload)

    variants = []
    for v in args.variants.split(";"):
        kv = {}
        for item in filter(None, v.split(",")):
            k, x = item.split("=")
            kv[k.strip()] = int(x)
        variants.append((v, kv))
    keys = sorted({k for _, kv in variants for k in kv})
    defaults = {"gather": 1, "lds_pad": 0, "stream": 0, "chunk_packets": 0, "tx_store": -1,
                "short_loads": -1, "slot_windows": 0}

    def apply(kv):
        for k in keys:
            val = kv.get(k, defaults.get(k, 0))
            if lib.aipstack_chksum_tune(k.encode(), val) != 0:
                raise SystemExit(f"tune {k}={val} rejected")

    def launch(r):
        if layout == "csrslot":
            A.chksum_batch_slotted(bufs[r], 2048, d_lens, out=out, stream=stream)
        elif layout == "csr":
            A.chksum_batch_csr(bufs[r], d_off, out=out, stream=stream)
        else:
            A.chksum_batch_strided(bufs[r], stride, plen, n, out=out, stream=stream)

    times = {name: [] for name, _ in variants}
    ok = {name: True for name, _ in variants}
    k = 0
    for rnd in range(args.rounds + 1):
        for name, kv in variants:
            apply(kv)
            evs = []
            for _ in range(args.reps):
                r = k % args.rotate
                k += 1
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                launch(r)
                b.record(stream)
                evs.append((a, b))
            torch.cuda.synchronize()
            if not np.array_equal(out.cpu().numpy(), wants[r]):
                ok[name] = False
            if rnd > 0:  # round 0: warm-up
                times[name] += [a.elapsed_time(b) * 1e3 for a, b in evs]
    apply({})
    for name, _ in variants:
        t = times[name]
        med = statistics.median(t)
        print(json.dumps({"config": args.config, "variant": name, "median_us": round(med, 2),
                          "mean_us": round(statistics.fmean(t), 2), "min_us": round(min(t), 2),
                          "frac_8TBps": round(alg / med / 1e-6 / 8e12, 4),
                          "launches": len(t), "rotate": args.rotate, "parity": ok[name]}),
              flush=True)


if __name__ == "__main__":
    main()
