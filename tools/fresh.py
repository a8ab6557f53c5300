#!/usr/bin/env python3
"""Fresh-data experiments: the first read of a batch
that something has just written runs slower than later reads. Which writer, which reader,
what granularity, and does the effect age away?

Config A's batch (1 M x 1500 B, 1.57 GB), three working batches W0..W2 (bench.py's seeds
42..44). Every experiment prints one JSON line with the per-launch times (HIP events on the
launch stream, around the read only) of its read launches, in order, and every read's
output is checked against that batch's expected sums. Writers and the pure reader come from
tools/build/libfresh_probe.so (tools/fresh_probe.hip). Not part of the product.

    python tools/fresh.py [EXPERIMENT ...]      (default: all)
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import aipstack_amd as A
    from aipstack_amd import _lib, synth
    import bench

    lib = _lib.load()
    fp = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libfresh_probe.so"))
    for f in ("fp_read", "fp_touch", "fp_copy"):
        getattr(fp, f).restype = ctypes.c_int
    fp.fp_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int,
                           ctypes.c_void_p]
    fp.fp_touch.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    fp.fp_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                           ctypes.c_void_p]

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    layout, n, plen = bench.CONFIGS["A"]
    spec = bench.shard_spec("A", 0, 1)
    total, stride = spec["total"], spec.get("stride", plen)
    R = 3
    W = [torch.empty(total, dtype=torch.uint8, device=dev) for _ in range(R)]
    P = [torch.empty(total, dtype=torch.uint8, device=dev) for _ in range(R)]  # pristine
    spare = torch.empty(total, dtype=torch.uint8, device=dev)
    scratch = torch.zeros(1 << 16, dtype=torch.uint32, device=dev)
    out = torch.empty(n, dtype=torch.uint16, device=dev)
    for r in range(R):
        synth.fill_device(P[r], synth.SEED_DATA + r, spec["byte_offset"])
    synth.fill_device(spare, 7, 0)
    torch.cuda.synchronize()
    wants = []
    for r in range(R):
        A.chksum_batch_strided(P[r], stride, plen, n, out=out, stream=stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy().copy()
        check = bench.oracle_check(dict(spec, data_seed=synth.SEED_DATA + r), got, threads=16)
        if not check.startswith("bit-exact"):
            raise SystemExit(f"pristine batch {r}: {check}")
        wants.append(torch.from_numpy(got).to(dev))
    for r in range(R):
        W[r].copy_(P[r])
    pinned = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(P[0].cpu())
    torch.cuda.synchronize()

    def tune(**kv):
        for k, v in kv.items():
            if lib.aipstack_chksum_tune(k.encode(), int(v)) != 0:
                raise SystemExit(f"tune {k}={v} rejected")

    ok = [True]

    def read(r, reader="chksum"):
        """One timed read of W[r]; returns the event pair (checked later)."""
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        if reader.startswith("pure"):
            mode = int(reader[4:] or 0)
            if fp.fp_read(W[r].data_ptr(), total, scratch.data_ptr(), mode, sh) != 0:
                raise SystemExit("fp_read")
        else:
            A.chksum_batch_strided(W[r], stride, plen, n, out=out, stream=stream)
        b.record(stream)
        return a, b

    def check(r, want_r):
        torch.cuda.synchronize()
        if not torch.equal(out, wants[want_r]):
            ok[0] = False

    def restore(r, src=None):
        """W[r] = P[src if given else r] (D2D, hipMemcpyAsync), untimed."""
        W[r].copy_(P[r if src is None else src])

    def emit(name, times, **extra):
        print(json.dumps({"experiment": name, "us": [round(t, 2) for t in times],
                          "parity": ok[0], **extra}), flush=True)

    def timed_seq(seq, reader="chksum", want=None):
        times = []
        for r in seq:
            a, b = read(r, reader)
            if not reader.startswith("pure"):
                check(r, r if want is None else want)
            else:
                torch.cuda.synchronize()
            times.append(a.elapsed_time(b) * 1e3)
        return times

    def writer_events(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        fn()
        b.record(stream)
        return a, b

    exps = sys.argv[1:] or ["base", "base_stream", "base_gath", "base_pure", "idle", "evict",
                            "pure_first", "fresh_synth", "fresh_d2d", "fresh_kcopy",
                            "fresh_kcopy_nt", "fresh_h2d", "readers", "touch", "partial", "age"]
    seq9 = [0, 1, 2] * 3

    def setup_synth():
        for r in range(R):
            synth.fill_device(W[r], synth.SEED_DATA + r, spec["byte_offset"])
        torch.cuda.synchronize()

    def warm():  # every batch read twice: the steady state
        timed_seq([0, 1, 2, 0, 1, 2])

    for e in exps:
        ok[0] = True
        tune(gather=1)
        if e in ("base", "base_stream", "base_gath", "base_pure"):
            # bench.py's order: the three batches synthesised, then read in rotation
            if e == "base_stream":
                tune(gather=-1)
            if e == "base_gath":
                tune(gather=0)
            setup_synth()
            emit(e, timed_seq(seq9, "pure" if e == "base_pure" else "chksum"))
        elif e == "idle":
            # the same with 0.5 s of idle device between the writes and the reads
            setup_synth()
            time.sleep(0.5)
            emit(e, timed_seq(seq9))
        elif e == "evict":
            # written, then 3 x 1.57 GB of reads of another buffer (the caches hold none of
            # the written lines any more), then the rotation
            setup_synth()
            for _ in range(3):
                fp.fp_read(spare.data_ptr(), total, scratch.data_ptr(), 0, sh)
            torch.cuda.synchronize()
            emit(e, timed_seq(seq9))
        elif e == "pure_first":
            # written, then each batch once by the pure reader (timed), then the checksum
            setup_synth()
            t1 = timed_seq([0, 1, 2], "pure")
            t2 = timed_seq(seq9)
            emit(e, t1 + t2, note="first 3: pure reader; then the checksum")
        elif e.startswith("fresh_"):
            # every read right after its batch was rewritten (writer timed separately)
            warm()
            reads, writes = [], []
            for k in range(9):
                r = k % R
                if e == "fresh_synth":
                    wa, wb = writer_events(lambda: synth.fill_device(
                        W[r], synth.SEED_DATA + r, spec["byte_offset"]))
                    want = r
                elif e == "fresh_d2d":
                    wa, wb = writer_events(lambda: W[r].copy_(P[0]))
                    want = 0
                elif e in ("fresh_kcopy", "fresh_kcopy_nt"):
                    wa, wb = writer_events(lambda: fp.fp_copy(
                        W[r].data_ptr(), P[0].data_ptr(), total, int(e.endswith("_nt")), sh))
                    want = 0
                elif e == "fresh_h2d":
                    wa, wb = writer_events(lambda: W[r].copy_(pinned, non_blocking=True))
                    want = 0
                else:
                    raise SystemExit(f"unknown {e}")
                a, b = read(r)
                check(r, want)
                reads.append(a.elapsed_time(b) * 1e3)
                writes.append(wa.elapsed_time(wb) * 1e3)
            for r in range(R):
                restore(r)
            emit(e, reads, writer_us=[round(t, 2) for t in writes])
        elif e == "readers":
            # which reader pays: each fp_read mode (and the checksum) on batches just rewritten
            # by a plain-store copy, then the same on the steady state
            for reader in ("pure0", "pure1", "pure2", "pure3", "pure4", "chksum"):
                warm()
                fresh, steady = [], []
                for k in range(6):
                    r = k % R
                    fp.fp_copy(W[r].data_ptr(), P[r].data_ptr(), total, 0, sh)
                    fresh += timed_seq([r], reader)
                steady = timed_seq([0, 1, 2, 0, 1, 2], reader)
                emit(f"readers_{reader}", fresh, steady_us=[round(t, 2) for t in steady])
        elif e == "steady":
            # 30 launches over the rotation, after the warm-up
            warm()
            emit(e, timed_seq([0, 1, 2] * 10))
        elif e == "touch":
            # steady state, then one dword per STEP bytes rewritten in place before each read
            for step in (64, 128, 256, 4096, 65536, 2 << 20):
                warm()
                reads = []
                for k in range(6):
                    r = k % R
                    fp.fp_touch(W[r].data_ptr(), total, step, sh)
                    a, b = read(r)
                    check(r, r)
                    reads.append(a.elapsed_time(b) * 1e3)
                emit(f"touch_{step}", reads)
        elif e == "partial":
            # steady state, then the first FRAC of the batch rewritten (kernel copy) before
            # each read
            for frac in (0.125, 0.25, 0.5, 1.0):
                warm()
                reads = []
                nb = (int(total * frac) // 16) * 16
                for k in range(6):
                    r = k % R
                    fp.fp_copy(W[r].data_ptr(), P[r].data_ptr(), nb, 0, sh)
                    a, b = read(r)
                    check(r, r)
                    reads.append(a.elapsed_time(b) * 1e3)
                emit(f"partial_{frac}", reads)
        elif e == "age":
            # rewritten, then the device idle for T before the read
            for t_idle in (0.0, 0.001, 0.01, 0.1, 1.0):
                warm()
                reads = []
                for k in range(3):
                    r = k % R
                    fp.fp_copy(W[r].data_ptr(), P[r].data_ptr(), total, 0, sh)
                    torch.cuda.synchronize()
                    time.sleep(t_idle)
                    a, b = read(r)
                    check(r, r)
                    reads.append(a.elapsed_time(b) * 1e3)
                emit(f"age_{t_idle}", reads)
        else:
            raise SystemExit(f"unknown experiment {e}")
        # leave every working batch equal to its pristine copy
        for r in range(R):
            restore(r)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
