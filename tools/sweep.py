#!/usr/bin/env python3
"""Launch-parameter sweep of the batch checksum and frame kernels, interleaved in ONE process.

Each variant sets the library tunables (aipstack_chksum_tune), launches the batch, and is
timed with HIP events on the launch stream; variants are interleaved round by round (so
clock/thermal drift hits all of them alike) and every variant's output is checked equal
to the first one's and, for a prefix, to the oracle. Prints one JSON object per variant
(median/min kernel us, GB/s of algorithmic bytes, fraction of 8 TB/s) to stdout.

    python tools/sweep.py --config A --rounds 8 [--variants "U,P,NT,WPC;..."]
    python tools/sweep.py --config RX [--variants "F,WPC;..."]   (frames in flight, waves/CU)

U, P, NT and F (unroll, packets, nontemporal, frames) other than their defaults need a build
with every variant: tools/build_variant.sh NAME -DAIPSTACK_ALL_VARIANTS, then --lib
tools/build/lib_NAME.so (tools/sweep_common.py checks and says so).
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

DEFAULT_VARIANTS = {
    "A": "0,0,1,0;0,0,1,0,-1;0,0,1,0,2;0,0,1,0,8;0,0,1,32;0,0,1,128;0,0,1,256;0,0,1,32,8",
    "B": "0,0,1,0;0,0,1,0,-1;0,0,1,0,2;0,0,1,0,8;0,0,1,32;0,0,1,128;0,0,1,256;0,0,1,32,8",
    "A2K": "0,0,1,0;0,0,1,0,4;0,0,1,0,8;0,0,1,0,-1;0,4,1,0,-1;0,8,1,0,-1;0,0,1,32;0,0,1,128",
    "C": "0,0,1,0;0,0,1,0,-1;0,0,1,0,2;0,0,1,0,8;0,0,1,64;0,0,1,256;0,0,1,64,8;"
         "0,0,1,32;0,0,1,32,8;0,0,1,32,2",
    "RX": "0,0;0,0,-1;0,0,2;0,0,8;2,0;4,64;4,256;2,64,2;2,256,2",
    "TX": "0,0;0,0,-1;0,0,2;0,0,8;2,0;4,64;4,256;2,64,2;2,256,2",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="A", choices=["A", "B", "C", "A2K", "RX", "TX"])
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5, help="launches per variant per round")
    ap.add_argument("--variants", default=None,
                    help='"U,P,NT,WPC[,SU];..." or, for RX/TX, "F,WPC[,SU];..." (0 = automatic; '
                         'SU = stream-mode windows 2/4/8, -1 = stream mode off)')
    ap.add_argument("--tx-inplace", action="store_true",
                    help="TX: the one-pass in-place fill (default: split)")
    ap.add_argument("--lib", default=None,
                    help="load this build of libaipstack_chksum.so instead (experiments)")
    args = ap.parse_args()

    import torch

    if args.lib:  # before the package loads the library
        os.environ["AIPSTACK_AMD_LIB"] = os.path.abspath(args.lib)
    import aipstack_amd as A
    from aipstack_amd import _lib, synth
    print(f"library: {_lib.LIB_PATH}", file=sys.stderr)
    lib = _lib.load()

    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream()
    stride = None
    if args.config == "A":
        n, plen, layout = 1 << 20, 1500, "strided"
    elif args.config == "A2K":  # MTU packets in 2048-byte ring slots
        n, plen, layout, stride = 1 << 20, 1500, "strided", 2048
    elif args.config == "B":
        n, plen, layout = 256 << 10, 9000, "strided"
    elif args.config == "C":
        n, plen, layout = 2 << 20, None, "csr"
    else:
        n, plen, layout = 1 << 20, None, args.config.lower()
    if layout in ("rx", "tx"):
        fbuf, off = synth.frames_host(n, seed=synth.SEED_DATA, max_payload=1460)
        orc0 = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        orc0.oracle_tx_fill_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64,
                                                                      ctypes.c_void_p]
        orc0.oracle_rx_verify_batch.argtypes = orc0.oracle_tx_fill_batch.argtypes
        o64 = off.astype(np.uint64)
        st = np.empty(n, dtype=np.uint8)
        if layout == "rx":
            orc0.oracle_tx_fill_batch(fbuf.ctypes.data, o64.ctypes.data, n, st.ctypes.data)
            want_rx = np.empty(n, dtype=np.uint8)
            orc0.oracle_rx_verify_batch(fbuf.ctypes.data, o64.ctypes.data, n, want_rx.ctypes.data)
        else:
            want_tx = fbuf.copy()
            orc0.oracle_tx_fill_batch(want_tx.ctypes.data, o64.ctypes.data, n, st.ctypes.data)
        total = int(off[-1])
        buf = torch.from_numpy(fbuf).to(dev)
        d_off = torch.from_numpy(off).to(dev)
        alg = total + 8 * (n + 1) + n + (4 * n if layout == "tx" else 0)
    elif layout == "strided":
        stride = stride or plen
        total = n * plen
        buf = torch.empty(n * stride, dtype=torch.uint8, device=dev)
        synth.fill_device(buf, synth.SEED_DATA)
        alg = total + 2 * n
    else:
        off = synth.mixed_offsets(n)
        total = int(off[-1])
        buf = torch.empty(total, dtype=torch.uint8, device=dev)
        synth.fill_device(buf, synth.SEED_DATA)
        d_off = torch.from_numpy(off).to(dev)
        synth.apply_classes_device(buf, d_off)
        alg = total + 2 * n + 8 * (n + 1)
    out = torch.empty(n, dtype=torch.uint8 if layout in ("rx", "tx") else torch.uint16,
                      device=dev)

    tx_ws = torch.empty(8 * n, dtype=torch.uint8, device=dev) if layout == "tx" else None

    def run():
        if layout == "rx":
            A.rx_verify(buf, d_off, out=out, stream=stream)
        elif layout == "tx":
            A.tx_fill(buf, d_off, out=out, stream=stream, split=not args.tx_inplace,
                      workspace=tx_ws)
        elif layout == "strided":
            A.chksum_batch_strided(buf, stride, plen, n, out=out, stream=stream)
        else:
            A.chksum_batch_csr(buf, d_off, out=out, stream=stream)

    variants = []
    for v in (args.variants or DEFAULT_VARIANTS[args.config]).split(";"):
        if "=" in v:  # "key=value,...": any aipstack_chksum_tune keys (unset ones automatic)
            d = {"unroll": 0, "packets": 0, "waves_per_cu": 0, "stream": 0, "chunk_packets": 0}
            d.update({k: int(x) for k, x in (kv.split("=") for kv in v.split(","))})
            variants.append(d)
            continue
        if layout in ("rx", "tx"):
            f = [int(x) for x in v.split(",")]
            variants.append({"frames": f[0], "waves_per_cu": f[1],
                             "stream": f[2] if len(f) > 2 else 0})
            continue
        f = [int(x) for x in v.split(",")]
        u, p, nt, wpc = f[:4]
        su = f[4] if len(f) > 4 else 0
        variants.append({"unroll": u, "packets": p, "nontemporal": nt, "waves_per_cu": wpc,
                         "stream": su})

    sweep_common.require_variants(lib, variants)  # sweep-only keys need an ALL_VARIANTS build

    def apply(v):
        lib.aipstack_chksum_tune(b"chunks_per_wave", 0)
        for k, val in v.items():
            assert lib.aipstack_chksum_tune(k.encode(), val) == 0

    def check(got):
        if layout == "rx":
            return bool(np.array_equal(got, want_rx))
        if layout == "tx":
            return bool(np.array_equal(buf.cpu().numpy(), want_tx))
        return bool(np.array_equal(got[:m], want))

    # reference output: oracle on a prefix
    m = min(n, 65536)
    orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    host = buf.cpu().numpy()
    want = np.empty(m, dtype=np.uint16)
    if layout in ("rx", "tx"):
        pass
    elif layout == "strided":
        orc.oracle_batch_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
        orc.oracle_batch_strided(host.ctypes.data, stride, plen, m, want.ctypes.data, 0)
    else:
        orc.oracle_batch_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_uint32]
        o = off[:m + 1].astype(np.uint64)
        orc.oracle_batch_csr(host.ctypes.data, o.ctypes.data, m, want.ctypes.data, 0)

    first = None
    times = [[] for _ in variants]
    ok = [True] * len(variants)
    for vi, v in enumerate(variants):  # warm-up + correctness per variant
        apply(v)
        run()
        run()
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        if first is None:
            first = got.copy()
        ok[vi] = bool(np.array_equal(got, first) and check(got))
    for _ in range(args.rounds):
        for vi, v in enumerate(variants):
            apply(v)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.reps)]
            for s, e in ev:
                s.record(stream)
                run()
                e.record(stream)
            torch.cuda.synchronize()
            times[vi].extend(s.elapsed_time(e) * 1e3 for s, e in ev)
    for v, t, good in zip(variants, times, ok):
        med = float(np.median(t))
        print(json.dumps({"config": args.config, **v, "median_us": round(med, 2),
                          "min_us": round(float(np.min(t)), 2),
                          "GBps": round(alg / med / 1e3, 1),
                          "frac_8TBps": round(alg / med / 1e3 / 8000.0, 4), "parity": good}),
              flush=True)


if __name__ == "__main__":
    main()
