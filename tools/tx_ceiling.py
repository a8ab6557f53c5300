#!/usr/bin/env python3
"""The in-place Tx fills' own ceiling: TX's (TX2K's) read pattern plus
the two 2-byte field stores per frame, without the checksum arithmetic (fp_fill in
tools/fresh_probe.hip), over R = 3 copies of the frame batch at distinct addresses (bench.py's
rotation). Sweeps the store density (a frame's fields written for every 1st, 2nd, 4th, 8th
frame) and the store policy (ordinary / nontemporal), and times the product's fill and Rx
verify on the same copies. One JSON line per measurement, median of 30 launches after 6.
Not part of the product.

    python tools/tx_ceiling.py [TX|TX2K ...]
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import aipstack_amd as A
    from aipstack_amd import synth
    import bench

    fp = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libfresh_probe.so"))
    fp.fp_fill_rec.restype = ctypes.c_int
    fp.fp_fill_rec.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p]
    fp.fp_fill.restype = ctypes.c_int
    fp.fp_fill.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                           ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    scratch = torch.zeros(1 << 16, dtype=torch.uint32, device=dev)
    R = 3
    for cfg in sys.argv[1:] or ["TX", "TX2K"]:
        spec = bench.shard_spec(cfg, 0, 1)
        n = spec["n"]
        compact = bench.host_shard(spec)
        if cfg == "TX":
            host, d_off, d_lens, stride = compact, torch.from_numpy(spec["offsets"]).to(dev), None, 0
            nbytes = int(spec["offsets"][-1])
        else:
            host, lens = synth.to_slots(compact, spec["offsets"], 2048)
            d_off, stride = None, 2048
            d_lens = torch.from_numpy(lens.view(np.int32)).to(dev)
            nbytes = int(lens.sum(dtype=np.uint64))
        copies = [torch.from_numpy(host).to(dev) for _ in range(R)]
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()

        def timed(launch, reps=30, warm=6):
            ts = []
            for k in range(warm + reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                launch(k % R)
                b.record(stream)
                b.synchronize()
                if k >= warm:
                    ts.append(a.elapsed_time(b) * 1e3)
            return statistics.median(ts)

        def probe(density, store):
            def run(r):
                st = fp.fp_fill(copies[r].data_ptr(), d_off.data_ptr() if d_off is not None else None,
                                stride, d_lens.data_ptr() if d_lens is not None else None, n,
                                density, store, scratch.data_ptr(), sh)
                if st != 0:
                    raise SystemExit(f"fp_fill {st}")
            return timed(run)

        def product(kind):
            def run(r):
                if cfg == "TX":
                    (A.tx_fill if kind == "fill" else A.rx_verify)(copies[r], d_off, out=status,
                                                                   stream=stream)
                else:
                    (A.tx_fill_slotted if kind == "fill" else A.rx_verify_slotted)(
                        copies[r], 2048, d_lens, out=status, stream=stream)
            return timed(run)

        t_read = probe(1, 0)
        print(json.dumps({"config": cfg, "what": "probe read only", "us": round(t_read, 2),
                          "payload_GBps": round(nbytes / t_read / 1e3, 1)}), flush=True)
        for store, name in ((1, "ordinary"), (2, "nontemporal")):
            for density in (1, 2, 4, 8):
                t = probe(density, store)
                stores = 2 * ((n + density - 1) // density)
                print(json.dumps({"config": cfg, "what": "probe read + field stores",
                                  "store": name, "density": density, "us": round(t, 2),
                                  "ns_per_store_over_read": round((t - t_read) * 1e3 / stores, 4)}),
                      flush=True)
        if cfg == "TX":  # the records pass's pattern: the read plus an 8-byte record per frame
            rec = torch.empty(n, dtype=torch.int64, device=dev)
            for store, name in ((3, "ordinary"), (4, "nontemporal")):
                def run(r, store=store):
                    if fp.fp_fill_rec(copies[r].data_ptr(), d_off.data_ptr(), 0, None, n, 1, store,
                                      scratch.data_ptr(), rec.data_ptr(), sh) != 0:
                        raise SystemExit("fp_fill_rec")
                t = timed(run)
                print(json.dumps({"config": cfg, "what": "probe read + 8-byte records",
                                  "store": name, "us": round(t, 2)}), flush=True)
            t = timed(lambda r: A.tx_fill_records(copies[r], d_off, out=rec, stream=stream))
            print(json.dumps({"config": cfg, "what": "product records pass", "us": round(t, 2)}),
                  flush=True)
        # the product on the same copies (the probe's junk fields are rewritten by the fill)
        for kind in ("fill", "verify"):
            t = product(kind)
            print(json.dumps({"config": cfg, "what": f"product {kind}", "us": round(t, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
