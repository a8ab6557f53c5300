#!/usr/bin/env python3
"""Benchmark: device-resident Internet checksum throughput on MI355X (GiB/s).

A "step" is one pass of the hot path -- one batched checksum launch
(aipstack_chksum_batch_strided / _csr of libaipstack_chksum.so) over one batch of
synthetic packets already resident in HBM. Default workload = BASELINE.json configs[1]
(config A): 1 M x 1500-byte packets per GPU. For A, B and C the timed loop rotates over
R = 3 distinct resident batches (--rotate; step k reads batch k mod R, every batch checked),
so that no launch finds its bytes in the 256 MiB Infinity Cache; the line also
carries the same box's pure-read probe rate (roofline.measured_peak: a reference, not a bound).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config A|B|C]
    torchrun --nproc-per-node N ... bench.py --gpus N     (one rank per GPU)

Multi-GPU: rank r owns a disjoint shard (packets [r*M, (r+1)*M) of one global batch,
generated in place on its own GPU); there is NO data-path collective. A gloo process
group is used only for the control plane (barriers around the timed region, max of the
per-rank times). value = bytes of all ranks x K / max-over-ranks time ("scaling": weak).

Prints ONE JSON line on stdout (everything else goes to stderr).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s checksummed (device-resident), 1M×1500B packets, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table), GB/s

CONFIGS = {
    # name: (layout, packets per GPU, packet bytes (strided) / None (mixed))
    "A": ("strided", 1 << 20, 1500),
    "B": ("strided", 256 << 10, 9000),
    # config A's packets in 2048-B ring slots (stride != len: the per-packet wave mode)
    "A2K": ("strided", 1 << 20, 1500),
    "C": ("csr", 2 << 20, None),
    # SURVEY 8(f) rows 2-3 (not BASELINE metric lines): raw Ethernet frames
    "RX": ("rx", 1 << 20, None),
    "TX": ("tx", 1 << 20, None),
    # the split fill's read pass alone (aipstack_chksum_tx_fill_records): the E2E Tx kernel
    "TXREC": ("txrec", 1 << 20, None),
    # ring slots (one frame / packet per 2048-B slot, a length per slot; TAP receive ring)
    "RX2K": ("rxslot", 1 << 20, None),
    "TX2K": ("txslot", 1 << 20, None),  # a send ring: Tx fill in place, one frame per slot
    "C2K": ("csrslot", 2 << 20, None),
    # chained + seeded (TCP Tx shape)
    "CHAIN": ("chain", 1 << 20, None),
}
SLOT_STRIDE = {"A2K": 2048, "RX2K": 2048, "TX2K": 2048, "C2K": 2048}  # layouts not back to back
WORKLOAD_NAMES = {
    "A": "1M x 1500B Ethernet-MTU packets per GPU, IP checksum (BASELINE configs[1]; x8 = configs[4])",
    "B": "256K x 9000B jumbo packets per GPU, IP checksum (BASELINE configs[2])",
    "A2K": "1M x 1500B packets per GPU in 2048B ring slots (stride != length: the packets' "
           "segments read as one gathered stream), IP checksum",
    "C": "2M mixed 64-1500B packets per GPU incl. odd lengths/starts, CSR (BASELINE configs[3])",
    "RX": "1M raw Ethernet frames per GPU (TCP/UDP/ICMP/other/ARP/fragments, 0-1460B payload), "
          "Rx verify: IPv4 header + L4 checksum verdicts",
    "TX": "1M raw Ethernet frames per GPU (same mix), Tx fill: IPv4 header + L4 checksums "
          "written in place",
    "TXREC": "1M raw Ethernet frames per GPU (same mix), Tx fill records: the split fill's read "
             "pass alone (8-B record per frame: both checksums, field offset, flags, status; "
             "nothing written into the frames)",
    "RX2K": "1M raw Ethernet frames per GPU (RX mix) in 2048B ring slots with a length per "
            "slot, Rx verify (aipstack_chksum_rx_verify_slotted)",
    "TX2K": "1M raw Ethernet frames per GPU (TX mix) in 2048B ring slots with a length per "
            "slot, Tx fill in place (aipstack_chksum_tx_fill_slotted)",
    "C2K": "2M mixed 64-1500B packets per GPU (config C's) in 2048B ring slots with a length "
           "per slot, IP checksum (aipstack_chksum_batch_slotted)",
    "CHAIN": "1M TCP-Tx-shaped chains per GPU: IpChksumAccumulator(pseudo-header State)"
             ".getChksum(20B header node + 1460B payload in 2 chunks split at a random point)",
}
CHAIN_HDR_STRIDE, CHAIN_HDR, CHAIN_PAYLOAD = 32, 20, 1460


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class stdout_to_stderr:
    """Point file descriptor 1 at stderr for the duration (C/C++ library chatter included;
    C stdio buffers are flushed before fd 1 is restored)."""

    def __enter__(self):
        sys.stdout.flush()
        self._saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        ctypes.CDLL(None).fflush(None)
        os.dup2(self._saved, 1)
        os.close(self._saved)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # Defaults sized for a fresh box: the first GPU-heavy second on a box runs ~3 % slow
    # (config A: 241 vs 233 us per launch, profiles/r02/warmup/), so ~0.5 s of untimed
    # launches come first, and 100 timed launches (~23 ms) average over transients.
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=2000)
    p.add_argument("--config", default="A", choices=sorted(CONFIGS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-reps", type=int, default=15,
                   help="timed single-thread passes of the CPU baseline sample")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--per-launch", action="store_true",
                   help="after the timed region, time each launch with its own event pair")
    p.add_argument("--e2e", action="store_true",
                   help="end-to-end mode: batch in HOST memory, results to HOST memory "
                        "(host-memory streaming engine; PCIe-inclusive). Prints its own line.")
    p.add_argument("--e2e-pageable", action="store_true",
                   help="with --e2e: do not page-lock the host batch (CPU copy to staging)")
    p.add_argument("--chain-fill", action="store_true",
                   help="CHAIN: the Tx form (aipstack_chksum_batch_chain_fill): each chain's "
                        "checksum is also stored big-endian into its 20-B header node")
    p.add_argument("--tx-split", action="store_true",
                   help="TX, TX2K: the two-pass split fill (read pass + scatter pass through a "
                        "workspace; default: the one-pass in-place fill, which measured faster "
                        "under the driver's protocol in round 5: TX 159.8 vs 161.6 us, TX2K "
                        "175.2 vs 178.9, profiles/r05/txsplit)")
    p.add_argument("--tx-inplace", action="store_true",
                   help="TX: the one-pass in-place fill (the default; kept for older scripts)")
    p.add_argument("--small", type=int, default=0, metavar="N",
                   help="small-batch mode (A or RX): batches of N packets/frames from a ring of "
                        "64 slots, eager launches vs the same launches replayed from a HIP "
                        "graph. Prints its own line.")
    p.add_argument("--e2e-streams", type=int, default=4)
    p.add_argument("--engines", type=int, default=0, metavar="N",
                   help="with --e2e: one process drives N devices through an engine group "
                        "(aipstack_chksum_engine_group_*; devices 0..N-1, or all "
                        "AIPSTACK_BENCH_FORCE_DEVICE), the batch split into N ranges")
    p.add_argument("--e2e-chunk-mib", type=int, default=64)
    p.add_argument("--no-ceiling", action="store_true",
                   help="skip the pure-read probe (roofline.measured_peak) and the Tx / records ceilings")
    p.add_argument("--rotate", type=int, default=3, metavar="R",
                   help="A, B, C, A2K: R distinct resident batches, step k reads batch k mod R "
                        "(3 x 1.5 GB for A: no launch can find its bytes in the 256 MiB "
                        "Infinity Cache); frames and ring slots (RX, TX, TXREC, RX2K, TX2K, "
                        "C2K): R copies of the batch at distinct addresses; 1 = one batch "
                        "read by every step")
    p.add_argument("--fresh", choices=FRESH_WRITERS, default=None,
                   help="fresh-data mode (DESIGN 6.1): before every launch (warm-ups included) "
                        "the batch it reads is rewritten from a pristine copy by WRITER -- dma "
                        "(pinned host -> device copy), nt (a device kernel with nontemporal "
                        "stores), plain (a device kernel with ordinary stores), d2d "
                        "(hipMemcpyAsync device -> device). Only the checksum launches are timed "
                        "(an event pair around each); the line carries 'fresh'")
    p.add_argument("--just-written", action="store_true",
                   help="pass the AIPSTACK_CHKSUM_JUST_WRITTEN hint (strided, ring-slot and "
                        "chain batches)")
    return p.parse_args()


FRESH_WRITERS = ("dma", "nt", "plain", "d2d")


def fresh_writer(kind, targets, stream):
    """writer(k): rewrite targets[k mod R] from a pristine copy taken now, on `stream` (the
    launch stream, so the checksum launch after it reads the new bytes). Bench plumbing."""
    import torch
    pristine = [t.clone() for t in targets]
    if kind == "dma":
        host = [torch.empty(t.numel(), dtype=torch.uint8, pin_memory=True) for t in targets]
        for h, t in zip(host, targets):
            h.copy_(t.cpu())
    lib = None
    if kind in ("nt", "plain"):
        lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libfresh_probe.so"))
        lib.fp_copy.restype = ctypes.c_int
        lib.fp_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                ctypes.c_void_p]
    torch.cuda.synchronize()

    def write(k):
        r = k % len(targets)
        t, p = targets[r], pristine[r]
        if kind == "dma":
            t.copy_(host[r], non_blocking=True)
        elif kind == "d2d":
            t.copy_(p)
        else:
            body = (t.numel() // 16) * 16
            if lib.fp_copy(t.data_ptr(), p.data_ptr(), body, int(kind == "nt"),
                           stream.cuda_stream) != 0:
                raise SystemExit("fresh writer: fp_copy failed")
            if body < t.numel():
                t[body:].copy_(p[body:])
    return write


# Layouts whose batch is synthesised on the host: rotated over copies at other addresses.
FRAME_LAYOUTS = ("rx", "tx", "txrec", "rxslot", "csrslot", "txslot")


def rotation_count(args, layout):
    """Batches the timed loop rotates over: the checksum batches (distinct data
    per batch), the frame and ring-slot batches and the chains (copies of the batch at other
    addresses, the chunk table rebased onto each; round 5)."""
    return max(1, args.rotate) if layout in ("strided", "csr", "chain") + FRAME_LAYOUTS else 1


def shard_spec(config, rank, world, n=None):
    """This rank's shard of the global batch: packets [rank*n, (rank+1)*n).

    Returns dict(layout, n, plen, byte_offset, offsets (local, CSR only), first_packet,
    total). The global batch is the same for every world size: strided shards are
    consecutive byte ranges of one splitmix64 stream; CSR shards are slices of one global
    offsets array, rebased to 0, whose bytes start at the global offset of their first
    packet (so classes and data come from global indices)."""
    from aipstack_amd import synth
    layout, n_default, plen = CONFIGS[config]
    n = n_default if n is None else n
    spec = {"layout": layout, "n": n, "plen": plen, "first_packet": rank * n}
    if layout == "strided":
        stride = SLOT_STRIDE.get(config, plen)
        spec["stride"] = stride
        spec["total"] = n * stride      # buffer bytes (slot gaps hold bytes no packet covers)
        spec["payload"] = n * plen
        spec["byte_offset"] = rank * n * stride
        spec["offsets"] = None
    elif layout in ("rx", "tx", "txrec", "rxslot", "txslot", "chain"):
        # each rank synthesises its own frames / chains (seed per rank): they are independent
        spec["seed"] = synth.SEED_DATA + 1000 * rank
        spec["byte_offset"] = 0
        spec["offsets"] = None  # known after synthesis
        spec["total"] = None
    else:  # csr, csrslot
        off_all = synth.mixed_offsets(n * world)
        spec["offsets"] = off_all[rank * n:(rank + 1) * n + 1] - off_all[rank * n]
        spec["byte_offset"] = int(off_all[rank * n])
        spec["total"] = int(spec["offsets"][-1])
    return spec


def host_shard(spec):
    """The shard's bytes in host memory (numpy), exactly as the device generators make them."""
    from aipstack_amd import synth
    if spec["layout"] in ("rx", "tx", "txrec", "rxslot", "txslot"):
        buf, off = synth.frames_host(spec["n"], seed=spec["seed"], max_payload=1460)
        spec["offsets"], spec["total"] = off, int(off[-1])
        if spec["layout"] in ("rx", "rxslot"):  # valid frames: filled by the oracle (test infra)
            lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
            lib.oracle_tx_fill_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64,
                                                                         ctypes.c_void_p]
            st = np.empty(spec["n"], dtype=np.uint8)
            o = off.astype(np.uint64)
            lib.oracle_tx_fill_batch(buf.ctypes.data, o.ctypes.data, spec["n"], st.ctypes.data)
        return buf
    host = np.empty(spec["total"], dtype=np.uint8)
    synth.fill_host(host, spec.get("data_seed", synth.SEED_DATA), spec["byte_offset"])
    if spec["layout"] in ("csr", "csrslot"):
        synth.apply_classes_host(host, spec["offsets"], first_packet=spec["first_packet"])
    return host


def algorithmic_bytes(layout, n, total_payload):
    """L bytes read + 2 bytes written per packet (+8 B offset for CSR).
    Frames: L read + 8 B offset + 1 B verdict/status (+ 4 B of checksums written, Tx);
    Tx records: L read + 8 B offset + 8 B record written.
    Chains: chunk bytes + 12 B (address, length) per chunk + 8 B index + 4 B state + 2 B
    result per chain (3 chunks per chain here)."""
    if layout == "chain":
        return total_payload + 3 * 12 * n + 8 * (n + 1) + 4 * n + 2 * n
    if layout == "txrec":
        return total_payload + 16 * n + 8
    if layout == "rxslot":  # frame bytes + 4 B length + 1 B verdict
        return total_payload + 5 * n
    if layout == "txslot":  # frame bytes + 4 B length + 1 B status + 4 B of checksums written
        return total_payload + 9 * n
    if layout == "csrslot":  # packet bytes + 4 B length + 2 B result
        return total_payload + 6 * n
    if layout in ("rx", "tx"):
        return total_payload + 9 * n + 8 + (4 * n if layout == "tx" else 0)
    b = total_payload + 2 * n
    if layout == "csr":
        b += 8 * (n + 1)
    return b


def dma_copy(t):
    """A copy of device tensor `t` at another address, written by DMA (pinned host -> device):
    the way the Rx path's bytes arrive. A device-side clone (ordinary stores) would leave its
    lines slow to read the first time."""
    import torch
    h = torch.empty(t.numel(), dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    out = torch.empty_like(t)
    out.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    return out


def dma_to(arr, dev):
    """numpy array -> device tensor through pinned host memory (DMA)."""
    import torch
    h = torch.from_numpy(arr).pin_memory()
    out = torch.empty(h.shape, dtype=h.dtype, device=dev)
    out.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    return out


def make_chains(spec, dev):
    """CHAIN workload: chain i = a 20-B header node (TCP header, 32-B stride header area)
    + 1460 payload bytes split into two chunks at a random point (a send ring wrapping,
    tcp/IpTcpProto_output.h:1251-1277), seeded with a random pseudo-header State. Device
    tensors plus the host copies parity needs."""
    import torch
    from aipstack_amd import synth
    n = spec["n"]
    hdr_bytes = CHAIN_HDR_STRIDE * n
    buf = torch.empty(hdr_bytes + CHAIN_PAYLOAD * n, dtype=torch.uint8, device=dev)
    synth.fill_device(buf, spec["seed"])
    rng = np.random.default_rng(spec["seed"])
    split = rng.integers(1, CHAIN_PAYLOAD, n).astype(np.uint64)
    base = buf.data_ptr()
    i = np.arange(n, dtype=np.uint64)
    addr = np.empty(3 * n, dtype=np.uint64)
    lens = np.empty(3 * n, dtype=np.uint32)
    addr[0::3] = base + CHAIN_HDR_STRIDE * i
    lens[0::3] = CHAIN_HDR
    addr[1::3] = base + hdr_bytes + CHAIN_PAYLOAD * i
    lens[1::3] = split
    addr[2::3] = addr[1::3] + split
    lens[2::3] = CHAIN_PAYLOAD - split
    index = np.arange(n + 1, dtype=np.uint64) * 3
    states = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    return {
        "buf": buf, "base": base, "n": n,
        "addr_host": addr, "len_host": lens, "index_host": index, "states_host": states,
        "addr": torch.from_numpy(addr.view(np.int64)).to(dev),
        "len": torch.from_numpy(lens.view(np.int32)).to(dev),
        "index": torch.from_numpy(index.view(np.int64)).to(dev),
        "states": torch.from_numpy(states.view(np.int32)).to(dev),
        # --chain-fill: each header's TCP checksum field (offset 16 of the 20-B node)
        "fields": torch.from_numpy((addr[0::3] + np.uint64(16)).view(np.int64)).to(dev),
        "payload": (CHAIN_HDR + CHAIN_PAYLOAD) * n,
    }


def chain_fill_check(chain):
    """--chain-fill: the timed launches kept refilling the fields, so zero them again, take
    the oracle's checksums over that state, fill once and compare both the returned values
    and every header's stored field (big-endian at header + 16)."""
    import aipstack_amd as A
    hdr = chain["buf"][:CHAIN_HDR_STRIDE * chain["n"]].view(-1, CHAIN_HDR_STRIDE)
    hdr[:, 16:18] = 0
    host = chain["buf"].cpu().numpy()
    want = chain_oracle(chain, host)
    got = A.chksum_chain_fill(chain["addr"], chain["len"], chain["index"], chain["states"],
                              chain["fields"]).cpu().numpy()
    fld = hdr[:, 16:18].cpu().numpy().astype(np.uint16)
    ok = np.array_equal(got, want) and np.array_equal((fld[:, 0] << 8) | fld[:, 1], want)
    return "bit-exact (every chain and stored field vs oracle)" if ok else "MISMATCH"


def chain_oracle(chain, host):
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    lib.oracle_batch_chain.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + \
        [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
    want = np.empty(chain["n"], dtype=np.uint16)
    lib.oracle_batch_chain(host.ctypes.data, chain["base"], chain["addr_host"].ctypes.data,
                           chain["len_host"].ctypes.data, chain["index_host"].ctypes.data,
                           chain["states_host"].ctypes.data, chain["n"], want.ctypes.data, 1)
    return want


def chain_check(chain, got):
    """Every chain against the C oracle (oracle_batch_chain) over a host copy."""
    host = chain["buf"].cpu().numpy()
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    lib.oracle_batch_chain.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + \
        [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
    want = np.empty(chain["n"], dtype=np.uint16)
    lib.oracle_batch_chain(host.ctypes.data, chain["base"], chain["addr_host"].ctypes.data,
                           chain["len_host"].ctypes.data, chain["index_host"].ctypes.data,
                           chain["states_host"].ctypes.data, chain["n"], want.ctypes.data, 1)
    return "bit-exact (every chain vs oracle)" if np.array_equal(got, want) else "MISMATCH"


def cpu_baseline(spec):
    """Reference scalar path on the host; bounded sample = this rank's whole batch."""
    layout, n, plen, off_host = spec["layout"], spec["n"], spec["plen"], spec["offsets"]
    total = spec.get("payload", spec["total"])
    stride = spec.get("stride", plen)
    host = host_shard(spec)
    out = np.empty(n, dtype=np.uint16)
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libref_chksum.so")
    cores_all = _affinity_cores()  # every core this process may run on
    if os.path.exists(ref_path):
        kind = "reference"
        lib = ctypes.CDLL(ref_path)
        lib.ref_time_batch_strided.restype = ctypes.c_double
        lib.ref_time_batch_strided.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                               ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                               ctypes.c_void_p]
        lib.ref_time_batch_csr.restype = ctypes.c_double
        lib.ref_time_batch_csr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]

        def timed(threads, reps):
            if layout == "csr":
                o = off_host.astype(np.uint64)
                return lib.ref_time_batch_csr(threads, reps, host.ctypes.data, o.ctypes.data, n,
                                              out.ctypes.data)
            return lib.ref_time_batch_strided(threads, reps, host.ctypes.data, stride, plen, n,
                                              out.ctypes.data)
    else:  # the C restatement (oracle/), single thread
        kind = "port"
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        lib.oracle_batch_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
        lib.oracle_batch_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_uint32]
        cores_all = 1

        def timed(threads, reps):
            ts = []
            o = off_host.astype(np.uint64) if layout == "csr" else None
            for _ in range(reps + 1):
                t0 = time.perf_counter()
                if layout == "csr":
                    lib.oracle_batch_csr(host.ctypes.data, o.ctypes.data, n, out.ctypes.data, 0)
                else:
                    lib.oracle_batch_strided(host.ctypes.data, stride, plen, n, out.ctypes.data, 0)
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts[1:]))
    t1 = timed(1, CPU_REPS)
    res = {
        "value": round(total / t1 / 2**30, 3),
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "sample": f"this rank's whole batch ({n} packets, {total} B of packets) in host memory, "
                  f"median of {CPU_REPS} passes after 1 warm-up, 1 thread"
                  + (" (reference Chksum.h:77-99 compiled -O2 from /root/reference)"
                     if kind == "reference" else " (oracle/chksum_oracle.c port)"),
    }
    if cores_all > 1:
        tn = timed(cores_all, 5)
        res["all_cores"] = {"value": round(total / tn / 2**30, 3), "cores": cores_all,
                            "threads": cores_all,
                            "sample": "same batch, disjoint packet ranges per std::thread, "
                                      "median of 5 passes"}
    res["cpu_model"] = _cpu_model()
    res["nproc"] = os.cpu_count()
    res["affinity_cores"] = _affinity_cores()
    hook = hook_baseline(spec, host, total, _affinity_cores(), out)
    if hook is not None:
        res["hook"] = hook
    return res, out


def hook_baseline(spec, host, total, cores_all, want):
    """The repo's own drop-in per-packet hook (libaipstack_chksum_hook: IpChksumInverted, the
    symbol the stack links under -DAIPSTACK_EXTERNAL_CHKSUM, reference Chksum.h:46-51) timed
    over the same host batch as the reference loop beside it, 1 thread and every affinity core
    (tools/hook_time.cpp, the reference leg's harness). Not the reference: labelled as the
    repo's drop-in. Its outputs are compared with the reference leg's (`want`). None when the
    harness is not built."""
    path = os.path.join(ROOT, "tools", "build", "libhook_time.so")
    if not os.path.exists(path):
        return None
    layout, n, plen, off_host = spec["layout"], spec["n"], spec["plen"], spec["offsets"]
    stride = spec.get("stride", plen)
    lib = ctypes.CDLL(path)
    lib.hook_time_batch_strided.restype = ctypes.c_double
    lib.hook_time_batch_strided.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                            ctypes.c_void_p]
    lib.hook_time_batch_csr.restype = ctypes.c_double
    lib.hook_time_batch_csr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    out = np.empty(n, dtype=np.uint16)
    o = off_host.astype(np.uint64) if layout == "csr" else None

    def timed(threads, reps):
        if layout == "csr":
            return lib.hook_time_batch_csr(threads, reps, host.ctypes.data, o.ctypes.data, n,
                                           out.ctypes.data)
        return lib.hook_time_batch_strided(threads, reps, host.ctypes.data, stride, plen, n,
                                           out.ctypes.data)

    t1 = timed(1, CPU_REPS)
    res = {"value": round(total / t1 / 2**30, 3), "unit": "GiB/s", "cores": 1,
           "kind": "repo drop-in hook (libaipstack_chksum_hook IpChksumInverted; AVX-512 / "
                   "AVX2 / SSE2 body picked at load), not the reference",
           "sample": f"the same batch as the reference leg, median of {CPU_REPS} passes, "
                     "1 thread",
           "matches_reference": bool(np.array_equal(out, want))}
    if cores_all > 1:
        tn = timed(cores_all, 5)
        res["all_cores"] = {"value": round(total / tn / 2**30, 3), "threads": cores_all,
                            "sample": "disjoint packet ranges per std::thread, median of 5"}
    return res


def cpu_baseline_chain(chain):
    """Reference IpChksumAccumulator(State).getChksum(IpBufRef chain) (Chksum.h:171-336)
    over every chain of this rank's CHAIN batch, on a host copy (nodes linked once, outside
    the timing); 1 thread and every affinity core. Kind "port" (the oracle's chain walk,
    oracle/chksum_oracle.c) where the reference build is absent."""
    host = chain["buf"].cpu().numpy()
    n = chain["n"]
    out = np.empty(n, dtype=np.uint16)
    bias = (chain["base"] - host.ctypes.data) % (1 << 64)
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libref_chksum.so")
    if os.path.exists(ref_path):
        kind = "reference"
        lib = ctypes.CDLL(ref_path)
        lib.ref_time_batch_chain.restype = ctypes.c_double
        lib.ref_time_batch_chain.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64] + \
            [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]

        def timed(threads, reps):
            return lib.ref_time_batch_chain(threads, reps, bias, chain["addr_host"].ctypes.data,
                                            chain["len_host"].ctypes.data,
                                            chain["index_host"].ctypes.data,
                                            chain["states_host"].ctypes.data, n,
                                            out.ctypes.data)
    else:
        kind = "port"
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        lib.oracle_batch_chain.argtypes = [ctypes.c_void_p, ctypes.c_uint64] + \
            [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]

        def timed(threads, reps):
            def one(lo, hi):
                k0 = int(chain["index_host"][lo])
                idx = chain["index_host"][lo:hi + 1] - np.uint64(k0)  # kept alive: a local
                lib.oracle_batch_chain(host.ctypes.data, chain["base"],
                                       chain["addr_host"][k0:].ctypes.data,
                                       chain["len_host"][k0:].ctypes.data, idx.ctypes.data,
                                       chain["states_host"][lo:hi].ctypes.data, hi - lo,
                                       out[lo:hi].ctypes.data, 1)
            return _timed_ranges(one, n, threads, reps)
    return _baseline_result(timed, chain["payload"], n, kind,
                            f"this rank's whole CHAIN batch ({n} chains of 3 chunks, "
                            f"{chain['payload']} B) in host memory",
                            "reference IpChksumAccumulator(State).getChksum(IpBufRef) from "
                            "Chksum.h compiled -O2 from /root/reference" if kind == "reference"
                            else "oracle/chksum_oracle.c chain walk")


def cpu_baseline_frames(spec, frames_host):
    """Rx verify / Tx fill on the host: the frame oracle (oracle/frame_oracle.c, a C
    restatement of the reference's receive checks and send-side fills whose arithmetic is
    the reference's IpChksum) over this rank's whole frame batch -- kind "port": the
    reference runs these checks inside its stack, one frame per call, with no entry point
    of its own to time. 1 thread and every affinity core (disjoint frame ranges; ctypes
    releases the GIL)."""
    n, off = spec["n"], spec["offsets"].astype(np.uint64)
    buf = frames_host.copy()
    status = np.empty(n, dtype=np.uint8)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    fn = lib.oracle_rx_verify_batch if spec["layout"] == "rx" else lib.oracle_tx_fill_batch
    fn.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]

    def timed(threads, reps):
        def one(lo, hi):  # offsets are absolute: pass the slice of n - lo + 1 entries
            fn(buf.ctypes.data, off[lo:].ctypes.data, hi - lo, status[lo:].ctypes.data)
        return _timed_ranges(one, n, threads, reps)
    what = "Rx verify" if spec["layout"] == "rx" else "Tx fill (in place, idempotent)"
    return _baseline_result(timed, spec["total"], n, "port",
                            f"{what} of this rank's whole frame batch ({n} frames, "
                            f"{spec['total']} B) in host memory",
                            "oracle/frame_oracle.c, compiled -O2")


def _timed_ranges(one, n, threads, reps):
    """Median of `reps` passes (after 1 warm-up) of one(lo, hi) over `threads` disjoint
    ranges run concurrently (Python threads; the ctypes calls run without the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    bounds = [(n * t // threads, n * (t + 1) // threads) for t in range(threads)]
    ts = []
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for _ in range(reps + 1):
            t0 = time.perf_counter()
            list(ex.map(lambda b: one(*b), bounds))
            ts.append(time.perf_counter() - t0)
    return float(np.median(ts[1:]))


def _baseline_result(timed, total, n, kind, sample, impl):
    reps = max(3, min(CPU_REPS, 5))
    t1 = timed(1, reps)
    cores_all = _affinity_cores()
    res = {"value": round(total / t1 / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": kind,
           "sample": f"{sample}, median of {reps} passes after 1 warm-up, 1 thread ({impl})"}
    if cores_all > 1:
        tn = timed(cores_all, 5)
        res["all_cores"] = {"value": round(total / tn / 2**30, 3), "cores": cores_all,
                            "threads": cores_all,
                            "sample": "same batch, disjoint ranges per thread, median of 5"}
    res["cpu_model"] = _cpu_model()
    res["nproc"] = os.cpu_count()
    res["affinity_cores"] = cores_all
    return res


def _affinity_cores():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


CPU_REPS = 15


def main():
    global CPU_REPS
    args = parse()
    CPU_REPS = max(1, args.cpu_reps)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    import aipstack_amd as A
    from aipstack_amd import synth

    if world > 1:
        # control plane only (barriers + max of times); no data-path collective. Gloo's C++
        # side prints "[Gloo] Rank r is connected to ..." on stdout: keep stdout for the one
        # JSON line.
        with stdout_to_stderr():
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
    # AIPSTACK_BENCH_FORCE_DEVICE: rehearsal of the multi-rank flow on a 1-GPU box (every
    # rank on that device). Never set by the driver; ranks then own their LOCAL_RANK GPU.
    device = int(os.environ.get("AIPSTACK_BENCH_FORCE_DEVICE", local_rank))
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)
    if A.device_check(device) != A.AIPSTACK_CHKSUM_OK:
        raise SystemExit(f"rank {rank}: device {device} is not a usable gfx950 device")

    layout, n, plen = CONFIGS[args.config]
    stream = torch.cuda.current_stream()
    if args.small:
        if args.config not in ("A", "RX", "TX") or world > 1:
            raise SystemExit("--small covers configs A, RX and TX on one GPU")
        return small_batches(args, layout, plen, dev)
    if args.e2e:
        if layout not in ("strided", "csr", "rx", "tx", "rxslot", "csrslot", "txslot"):
            raise SystemExit("--e2e covers the configs A, B, C, RX, TX, RX2K, TX2K and C2K")
        return e2e(args, rank, world, local_rank, layout, n, plen)

    # ---- this rank's shard, generated in place (global packets [rank*n, (rank+1)*n))
    spec = shard_spec(args.config, rank, world)
    if layout in ("rx", "tx", "txrec"):
        frames_host = host_shard(spec)          # frames are synthesised on the host
        buf = dma_to(frames_host, dev)
        d_off = torch.from_numpy(spec["offsets"]).to(dev)
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        tx_ws = torch.empty(8 * n, dtype=torch.uint8, device=dev)  # split fill's records
        records = torch.empty(n, dtype=torch.int64, device=dev)
    if layout in ("rxslot", "csrslot", "txslot"):
        # the shard's frames / packets laid into 2048-B ring slots (slack = random bytes)
        compact_host = host_shard(spec)
        ring_host, lens_host = synth.to_slots(compact_host, spec["offsets"], SLOT_STRIDE[args.config])
        buf = dma_to(ring_host, dev)
        d_lens = torch.from_numpy(lens_host.view(np.int32)).to(dev)
        status = torch.empty(n, dtype=torch.uint8, device=dev)
        tx_ws = torch.empty(8 * n, dtype=torch.uint8, device=dev)  # slotted split's records
        spec["total"] = int(lens_host.sum(dtype=np.uint64))
        spec["payload"] = spec["total"]
    if layout == "chain":
        chain = make_chains(spec, dev)
        spec["total"] = chain["payload"]
    off_host = spec["offsets"]
    byte_offset = spec["byte_offset"]
    total = spec["total"]
    stride = spec.get("stride", plen)
    # Rotation: R distinct resident batches, step k reads batch k mod R, so no
    # launch finds the previous launch's bytes in the 256 MiB Infinity Cache. Batch r is the
    # shard's packets over data seed SEED_DATA + r (same lengths / offsets); each is checked.
    rot = rotation_count(args, layout)
    bufs, outs = [], []
    if layout in ("strided", "csr"):
        if layout == "csr":
            d_off = torch.from_numpy(off_host).to(dev)
        for r in range(rot):
            b = torch.empty(total, dtype=torch.uint8, device=dev)
            synth.fill_device(b, synth.SEED_DATA + r, byte_offset)
            if layout == "csr":
                synth.apply_classes_device(b, d_off, first_packet=spec["first_packet"])
            bufs.append(b)
            outs.append(torch.empty(n, dtype=torch.uint16, device=dev))
        buf = bufs[0]
    chain_rot = []  # chains: copies of the buffer, each with its chunk table rebased onto it
    if layout == "chain" and rot > 1:
        for _ in range(rot - 1):
            bc = dma_copy(chain["buf"])
            delta = bc.data_ptr() - chain["base"]
            chain_rot.append({"buf": bc, "addr": chain["addr"] + delta,
                              "fields": chain["fields"] + delta})
    fbufs = [buf] if layout in FRAME_LAYOUTS else []  # frame / ring-slot batches: R copies
    if layout in FRAME_LAYOUTS and rot > 1:               # at distinct addresses
        fbufs += [dma_copy(buf) for _ in range(rot - 1)]
    out = outs[0] if outs else torch.empty(n, dtype=torch.uint16, device=dev)
    torch.cuda.synchronize()
    step_no = [0]

    def step():
        k = step_no[0]
        step_no[0] = k + 1
        if layout == "strided":
            A.chksum_batch_strided(bufs[k % rot], stride, plen, n, out=outs[k % rot],
                                   stream=stream, just_written=args.just_written)
        elif layout == "csr":
            A.chksum_batch_csr(bufs[k % rot], d_off, out=outs[k % rot], stream=stream)
        elif layout == "rx":
            A.rx_verify(fbufs[k % len(fbufs)], d_off, out=status, stream=stream)
        elif layout == "txrec":
            A.tx_fill_records(fbufs[k % len(fbufs)], d_off, out=records, stream=stream)
        elif layout == "rxslot":
            A.rx_verify_slotted(fbufs[k % len(fbufs)], 2048, d_lens, out=status, stream=stream)
        elif layout == "csrslot":
            A.chksum_batch_slotted(fbufs[k % len(fbufs)], 2048, d_lens, out=out, stream=stream,
                                   just_written=args.just_written)
        elif layout == "txslot":  # idempotent, as the CSR fill
            A.tx_fill_slotted(fbufs[k % len(fbufs)], 2048, d_lens, out=status, stream=stream,
                              split=args.tx_split, workspace=tx_ws if args.tx_split else None)
        elif layout == "chain":
            cc = chain if k % rot == 0 else chain_rot[k % rot - 1]
            if args.chain_fill:
                A.chksum_chain_fill(cc["addr"], chain["len"], chain["index"], chain["states"],
                                    cc["fields"], out=out, stream=stream,
                                    just_written=args.just_written)
            else:
                A.chksum_batch_chain(cc["addr"], chain["len"], chain["index"], chain["states"],
                                     out=out, final=True, stream=stream,
                                     just_written=args.just_written)
        else:  # tx: idempotent (the filled fields are excluded from their own sums)
            A.tx_fill(fbufs[k % len(fbufs)], d_off, out=status, stream=stream,
                      split=args.tx_split, workspace=tx_ws)

    # fresh-data mode: the buffers each step reads, rewritten before it
    writer = None
    if args.fresh:
        if layout in ("strided", "csr"):
            targets = bufs
        elif layout == "chain":
            targets = [chain["buf"]] + [cc["buf"] for cc in chain_rot]
        else:
            targets = fbufs
        writer = fresh_writer(args.fresh, targets, stream)

    def step_w():  # a step after the timing, on the timed steps' terms (fresh: rewrite first)
        if writer:
            writer(step_no[0])
        step()

    for _ in range(args.warmup):
        if writer:
            writer(step_no[0])
        step()
    torch.cuda.synchronize()

    # ---- solo phase (N > 1): each rank in turn runs the K steps alone while the others wait
    # at a barrier -- the per-GPU rate with no other GPU of the node busy, the denominator of
    # scaling_efficiency (SURVEY.md:445)
    solo_s = None
    if world > 1 and not writer:
        for r in range(world):
            dist.barrier()
            if r == rank:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    step()
                torch.cuda.synchronize()
                solo_s = time.perf_counter() - t0
        dist.barrier()

    # ---- timed region: barrier + synchronize on both sides; one HIP event pair on the
    # launch stream brackets the K launches, so the per-launch average includes the
    # kernel-to-kernel gaps (conservative for roofline.achieved)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    fresh_us = []
    if writer:
        # fresh data: an event pair around each checksum launch, the rewrite before it untimed;
        # elapsed = the sum of the launches' times
        pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                 for _ in range(args.steps)]
        for a, b in pairs:
            writer(step_no[0])
            a.record(stream)
            step()
            b.record(stream)
        torch.cuda.synchronize()
        fresh_us = [a.elapsed_time(b) * 1e3 for a, b in pairs]
        elapsed = sum(fresh_us) / 1e6
        avg_kernel_s = elapsed / args.steps
    else:
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(args.steps):
            step()
        ev1.record(stream)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        avg_kernel_s = ev0.elapsed_time(ev1) / 1e3 / args.steps
    if world > 1:
        dist.barrier()

    # Diagnostic, AFTER the timed region (not part of `value`): per-launch event pairs,
    # to expose outliers / clock ramps that the bracketed average smooths over.
    per_launch = []
    if args.per_launch and not writer:
        pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                 for _ in range(args.steps)]
        for a, b in pairs:
            a.record(stream)
            step()
            b.record(stream)
        torch.cuda.synchronize()
        per_launch = sorted(a.elapsed_time(b) * 1e3 for a, b in pairs)

    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    max_elapsed = float(t.item())
    # every rank's own wall time, kernel time and solo time (control plane only; after the
    # timed region)
    mine = torch.tensor([elapsed, avg_kernel_s, solo_s or 0.0], dtype=torch.float64)
    ranks = [torch.zeros(3, dtype=torch.float64) for _ in range(world)]
    if world > 1:
        dist.all_gather(ranks, mine)
    else:
        ranks = [mine]

    payload = spec.get("payload", total)
    alg = algorithmic_bytes(layout, n, payload)
    if layout == "chain" and args.chain_fill:
        alg += 10 * n  # + the field address read and the 2-byte field written per chain

    # ---- parity: EVERY rank checks its own shard (after the timed region) against the
    # oracle / the reference; then (after a barrier, so that no other rank's check competes
    # for the host cores) rank 0 times the CPU baseline on its shard
    parity = None
    rot_parity = None
    cpu = None
    baseline = None  # rank 0's CPU baseline, run after every rank's check
    if layout in FRAME_LAYOUTS and len(fbufs) > 1:
        # every copy processed at least once (the Tx fills write each in place); the last
        # step's outputs are checked below, and the copies must equal copy 0 afterwards
        while step_no[0] < len(fbufs) or (step_no[0] - 1) % len(fbufs) != 0:
            step_w()
        torch.cuda.synchronize()
        if not args.no_parity:
            same = all(torch.equal(fbufs[0], b) for b in fbufs[1:])
            rot_parity = (f"rotation copies 1..{len(fbufs) - 1} identical to copy 0 after the run"
                          if same else "MISMATCH")
    if layout in ("rx", "tx", "txrec"):
        if not args.no_parity and layout == "txrec":
            parity = records_check(spec, frames_host, buf.cpu().numpy(), records.cpu().numpy())
        elif not args.no_parity:
            parity = frames_check(spec, frames_host, buf.cpu().numpy(), status.cpu().numpy())
        baseline = lambda: cpu_baseline_frames(spec, frames_host)
    elif layout in ("rxslot", "csrslot", "txslot"):
        if not args.no_parity and layout == "txslot":
            parity = tx_slots_check(ring_host, lens_host, buf.cpu().numpy(),
                                    status.cpu().numpy())
        elif not args.no_parity:
            parity = slots_check(layout, ring_host, lens_host,
                                 (status if layout == "rxslot" else out).cpu().numpy())

        def baseline():
            # the same frames / packets in their compact (CSR) form: the same host work
            cspec = dict(spec, layout={"rxslot": "rx", "txslot": "tx"}.get(layout, "csr"),
                         total=int(spec["offsets"][-1]))
            cspec.pop("payload", None)
            c = cpu_baseline_frames(cspec, compact_host) if layout != "csrslot" \
                else cpu_baseline(cspec)[0]
            c["sample"] += " (the same packets in their compact CSR form)"
            return c
    elif layout == "chain":
        if chain_rot and not args.no_parity:
            # each copy once more into its own output: the same sums as copy 0 (and, for the
            # fill, the same headers afterwards). A fill sums its field, so two fills restore
            # it: every copy must have been filled equally often (step count a multiple of R)
            while step_no[0] < rot or step_no[0] % rot != 0:
                step_w()
            ref = A.chksum_batch_chain(chain["addr"], chain["len"], chain["index"],
                                       chain["states"], final=True, stream=stream)
            same = True
            for cc in chain_rot:
                o = A.chksum_batch_chain(cc["addr"], chain["len"], chain["index"],
                                         chain["states"], final=True, stream=stream)
                torch.cuda.synchronize()
                same = same and torch.equal(o, ref)
                if args.chain_fill:
                    same = same and torch.equal(cc["buf"], chain["buf"])
            rot_parity = (f"rotation copies 1..{rot - 1} give copy 0's sums" if same
                          else "MISMATCH")
        if not args.no_parity:
            parity = (chain_fill_check(chain) if args.chain_fill
                      else chain_check(chain, out.cpu().numpy()))
        baseline = lambda: cpu_baseline_chain(chain)
    else:
        # every rotation batch was read at least once (outside the timing if the run was
        # shorter than the rotation), and each is checked below
        while step_no[0] < rot:
            step_w()
        torch.cuda.synchronize()
        host_out = out.cpu().numpy()
        rot_parity = None
        if rot > 1 and not args.no_parity:
            thr = max(1, _affinity_cores() // world)
            checks = [oracle_check(dict(spec, data_seed=synth.SEED_DATA + r),
                                   outs[r].cpu().numpy(), threads=thr) for r in range(1, rot)]
            rot_parity = (f"rotation batches 1..{rot - 1} bit-exact" if
                          all(c.startswith("bit-exact") for c in checks) else "MISMATCH")
        if world == 1 and not args.no_cpu_baseline:
            # one rank: the baseline's own output (the reference over the whole shard) is
            # the check
            def baseline():
                nonlocal parity
                c, want = cpu_baseline(spec)
                if not args.no_parity:
                    parity = ("bit-exact (whole shard vs reference)"
                              if np.array_equal(host_out, want) else "MISMATCH")
                return c
        else:
            if not args.no_parity:
                parity = oracle_check(spec, host_out, threads=max(1, _affinity_cores() // world))
            baseline = lambda: cpu_baseline(spec)[0]
    if world > 1:
        dist.barrier()
    if rank == 0 and not args.no_cpu_baseline and baseline is not None:
        cpu = baseline()
    if rot_parity is not None and parity is not None:
        parity = "MISMATCH (a rotation batch)" if rot_parity == "MISMATCH" else \
            f"{parity}; {rot_parity}"
    # which device each rank ran on, gathered on the control plane with its parity
    props = torch.cuda.get_device_properties(device)
    mine_info = {"rank": rank, "device": device,
                 "pci": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
                 "uuid": str(getattr(props, "uuid", "")), "arch": props.gcnArchName,
                 "parity": parity}
    infos = [None] * world
    if world > 1:
        dist.all_gather_object(infos, mine_info)
    else:
        infos = [mine_info]
    if not args.no_parity:
        bad = [i["rank"] for i in infos if not str(i["parity"]).startswith("bit-exact")]
        parity = (f"bit-exact (each of {world} rank(s) checked its own shard: {parity})" if not bad
                  else f"MISMATCH on rank(s) {bad}")
    pcis = [i["pci"] for i in infos]

    traffic, traffic_stale = _pmc_traffic(args.config)
    slot_ceiling_fields = {}
    if layout in ("strided", "csr") and rank == 0 and not args.no_ceiling:
        ceil = hbm_read_ceiling()
        if ceil:
            slot_ceiling_fields["measured_peak"] = dict(
                ceil, frac=round(alg / avg_kernel_s / 1e9 / ceil["GBps"], 4),
                kind="pure-read probe in the kernels' load shapes on this box -- a reference "
                     "rate, not an upper bound: the checksum kernel can read faster (frac > 1)")
    if layout in ("tx", "txslot") and rank == 0 and not args.tx_split and not args.no_ceiling:
        fc = fill_ceiling(layout, fbufs, d_off if layout == "tx" else None,
                          d_lens if layout == "txslot" else None, n, stream)
        if fc:
            slot_ceiling_fields["fill_ceiling"] = fc
            slot_ceiling_fields["frac_of_fill_ceiling"] = round(fc["us"] / (avg_kernel_s * 1e6), 4)
    if layout == "txrec" and rank == 0 and not args.no_ceiling:
        rc = records_ceiling(fbufs, d_off, n, stream)
        if rc:
            slot_ceiling_fields["records_ceiling"] = rc
            slot_ceiling_fields["frac_of_records_ceiling"] = round(
                rc["us"] / (avg_kernel_s * 1e6), 4)
    if layout in ("rxslot", "csrslot", "txslot") and rank == 0:
        ceil = slot_read_ceiling(args.config, spec)
        if ceil:
            kernel_gbps = payload / avg_kernel_s / 1e9
            slot_ceiling_fields.update({"slot_read_ceiling": ceil,
                                        "payload_GBps": round(kernel_gbps, 1),
                                        "frac_of_slot_read_ceiling":
                                            round(kernel_gbps / ceil["payload_GBps"], 4)})
    bytes_all = payload * world  # weak scaling: every rank holds the same-size shard
    value = bytes_all * args.steps / max_elapsed / 2**30
    achieved = alg / avg_kernel_s / 1e9
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(max_elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (counter-based splitmix64 bytes, seed 42; generated on device)",
        "config": {
            "workload": WORKLOAD_NAMES[args.config],
            "config": args.config,
            "packets_per_gpu": n,
            **({"slot_stride": stride} if layout == "strided" and stride != plen else {}),
            **({"slot_stride": SLOT_STRIDE[args.config]}
               if layout in ("rxslot", "csrslot", "txslot") else {}),
            "packet_bytes": plen if plen else {"csr": "64-1500 (mixed)", "csrslot": "64-1500 (mixed)",
                                                "chain": "20 + 1460 in 3 chunks"}.get(
                                                    layout, "60-1514 (frames)"),
            "payload_bytes_per_gpu": payload,
            "layout": layout,
            "parallelism": f"disjoint packet shards x{world}, no collective",
            "rotation": {"batches": rot,
                         "resident_bytes_per_gpu": int(rot * (
                             buf.numel() if layout in FRAME_LAYOUTS else
                             chain["buf"].numel() if layout == "chain" else total)),
                         "note": ("one batch, read by every step" if rot == 1 else
                                  "step k reads copy k mod R of the batch (the same frames at "
                                  "R addresses), every copy checked" if layout in FRAME_LAYOUTS
                                  else "step k reads copy k mod R of the chains (the buffer "
                                  "cloned, the chunk table rebased), every copy checked"
                                  if layout == "chain"
                                  else "step k reads batch k mod R (data seeds 42..42+R-1), "
                                  "every batch checked")},
            **({"tx_fill": "split: read pass + scatter pass (both timed)" if args.tx_split else
                "in-place, one pass"} if layout in ("tx", "txslot") else {}),
            **({"chain_fill": "checksum also stored big-endian into each header node"}
               if layout == "chain" and args.chain_fill else {}),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            **({"traffic_stale": traffic_stale} if traffic_stale else {}),
            "device_code": device_code_digest(),
            "kernel_us": round(avg_kernel_s * 1e6, 2),
            **({"per_launch_us": {"min": round(per_launch[0], 2),
                                  "median": round(per_launch[len(per_launch) // 2], 2),
                                  "max": round(per_launch[-1], 2)}} if per_launch else {}),
            "algorithmic_bytes_per_launch": alg,
            **slot_ceiling_fields,
        },
        "per_gpu": {
            "GiB_s": [round(spec.get("payload", total) * args.steps / float(r[0]) / 2**30, 2)
                      for r in ranks],
            **({"solo_GiB_s": [round(payload * args.steps / float(r[2]) / 2**30, 2)
                               for r in ranks]} if world > 1 and not writer else {}),
            "kernel_us": [round(float(r[1]) * 1e6, 2) for r in ranks],
            "devices": pcis,
            "arch": [i["arch"] for i in infos],
            "distinct_devices": len(set(pcis)) == world,
            **({"note": "ranks share a device (AIPSTACK_BENCH_FORCE_DEVICE rehearsal): not a "
                        "multi-GPU measurement"} if len(set(pcis)) != world else {}),
            "parity": [i["parity"] for i in infos],
        },
        "cpu_baseline": cpu,
        "parity": parity,
    }
    if world > 1 and not writer:
        # value / (N x mean solo rate): 1.0 = every rank as fast with the node busy as alone
        solo_mean = sum(payload * args.steps / float(r[2]) / 2**30 for r in ranks) / world
        result["scaling_efficiency"] = round(value / (world * solo_mean), 4)
        result["scaling_efficiency_note"] = (
            "value / (N x mean of each rank's solo GiB/s: the same K steps on its own shard with "
            "the other ranks idle at a barrier)" + (
                "; ranks share a device (rehearsal): not a multi-GPU figure"
                if len(set(pcis)) != world else ""))
    if writer:
        srt = sorted(fresh_us)
        result["fresh"] = {
            "writer": args.fresh,
            "just_written_hint": bool(args.just_written),
            "timing": "checksum launches only: the batch each launch reads was rewritten from a "
                      "pristine copy right before it (untimed); value and kernel_us from the sum "
                      "of the launches' event pairs",
            "kernel_us": {"mean": round(sum(fresh_us) / len(fresh_us), 2),
                          "median": round(srt[len(srt) // 2], 2), "min": round(srt[0], 2),
                          "max": round(srt[-1], 2)}}
        result["metric"] = METRIC + " [fresh data: " + args.fresh + "-written]"
    elif args.just_written:
        result["just_written_hint"] = True
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity is not None and parity.startswith("MISMATCH"):
        sys.exit(1)


def small_batches(args, layout, plen, dev):
    """Launch-bound regime: a receive loop hands over small bursts (N packets or frames per
    batch), each its own launch on one stream. R = 64 ring slots, one batch per slot; K
    batches timed eagerly (one wrapper call and launch each) and then as replays of one HIP
    graph that holds the R launches (torch.cuda.CUDAGraph capture of the same calls). HIP
    events on the stream around K batches; the last batch of each form checked against the
    oracle."""
    import torch
    import aipstack_amd as A
    from aipstack_amd import synth
    N = args.small
    R = int(max(2, min(64, (4 << 30) // (N * (plen or 800)))))  # ring of at most ~4 GB
    K = max(R, (args.steps * 50) // R * R)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    if layout == "strided":
        buf = torch.empty(R * N * plen, dtype=torch.uint8, device=dev)
        synth.fill_device(buf, synth.SEED_DATA)
        outs = [torch.empty(N, dtype=torch.uint16, device=dev) for _ in range(R)]
        views = [buf[r * N * plen:(r + 1) * N * plen] for r in range(R)]

        def launch(r):
            A.chksum_batch_strided(views[r], plen, plen, N, out=outs[r])
        payload = N * plen

        def check(r):
            lib.oracle_batch_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
            host = views[r].cpu().numpy()
            want = np.empty(N, dtype=np.uint16)
            lib.oracle_batch_strided(host.ctypes.data, plen, plen, N, want.ctypes.data, 0)
            return np.array_equal(outs[r].cpu().numpy(), want)
    else:
        frames, off = synth.frames_host(R * N, seed=synth.SEED_DATA, max_payload=1460)
        lib.oracle_tx_fill_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]
        st = np.empty(R * N, dtype=np.uint8)
        off64 = off.astype(np.uint64)  # kept alive across the call
        lib.oracle_tx_fill_batch(frames.ctypes.data, off64.ctypes.data, R * N, st.ctypes.data)
        buf = torch.from_numpy(frames).to(dev)  # valid frames: Tx refills them unchanged
        offs = [torch.from_numpy((off[r * N:(r + 1) * N + 1]).copy()).to(dev) for r in range(R)]
        outs = [torch.empty(N, dtype=torch.uint8, device=dev) for _ in range(R)]
        ws = [torch.empty(8 * N, dtype=torch.uint8, device=dev) for _ in range(R)]

        def launch(r):
            if layout == "rx":
                A.rx_verify(buf, offs[r], out=outs[r])
            else:
                A.tx_fill(buf, offs[r], out=outs[r], workspace=ws[r], split=args.tx_split)
        payload = int(off[-1]) // R

        def check(r):
            fn = lib.oracle_rx_verify_batch if layout == "rx" else lib.oracle_tx_fill_batch
            fn.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]
            o = off[r * N:(r + 1) * N + 1].astype(np.uint64)
            want = np.empty(N, dtype=np.uint8)
            ref = frames.copy()
            fn(ref.ctypes.data, o.ctypes.data, N, want.ctypes.data)
            ok = np.array_equal(outs[r].cpu().numpy(), want)
            return ok and (layout == "rx" or np.array_equal(buf.cpu().numpy(), ref))
    stream = torch.cuda.current_stream()
    for r in range(R):
        launch(r)
    torch.cuda.synchronize()

    def timed(body):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        body()
        e1.record(stream)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K, e0.elapsed_time(e1) / 1e3 / K

    def eager():
        for k in range(K):
            launch(k % R)
    eager()  # warm-up
    wall_e, dev_e = timed(eager)
    ok_e = check((K - 1) % R)
    for o in outs:
        o.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for r in range(R):
            launch(r)
    stream = torch.cuda.current_stream()

    def replays():
        for _ in range(K // R):
            g.replay()
    replays()
    wall_g, dev_g = timed(replays)
    ok_g = check(R - 1)
    res = {
        "metric": f"small batches ({'packets' if layout == 'strided' else 'frames'} per batch = {N}): "
                  "us per batch, eager launches vs HIP graph replay",
        "value": round(wall_g * 1e6, 3), "unit": "us per batch (graph, wall)",
        "n_gpus": 1, "steps": K, "warmup": K, "higher_is_better": False,
        "config": {"workload": f"config {args.config} in batches of {N}"
                               + (" (split fill)" if layout == "tx" and args.tx_split
                                  else " (one-pass in-place fill)" if layout == "tx" else ""),
                   "ring_slots": R,
                   "tuning": {k: v for k, v in os.environ.items()
                              if k.startswith("AIPSTACK_CHKSUM_")},
                   "payload_bytes_per_batch": payload},
        "eager": {"wall_us": round(wall_e * 1e6, 3), "events_us": round(dev_e * 1e6, 3),
                  "GiB_s": round(payload / wall_e / 2**30, 2)},
        "graph": {"wall_us": round(wall_g * 1e6, 3), "events_us": round(dev_g * 1e6, 3),
                  "GiB_s": round(payload / wall_g / 2**30, 2)},
        "parity": "bit-exact" if ok_e and ok_g else "MISMATCH",
    }
    print(json.dumps(res), flush=True)
    if not (ok_e and ok_g):
        sys.exit(1)


def e2e(args, rank, world, local_rank, layout, n, plen):
    """Host memory in, host memory out, through aipstack_chksum_engine (PCIe-inclusive)."""
    import torch.distributed as dist
    import aipstack_amd as A
    from aipstack_amd import synth
    spec = shard_spec(args.config, rank, world)
    off, total = spec["offsets"], spec.get("payload", spec["total"])
    stride = spec.get("stride", plen)
    host = host_shard(spec)
    frames = layout in ("rx", "tx", "rxslot", "txslot")
    if frames:  # frames: synthesised (and, for RX, made valid) on the host by host_shard
        off, total = spec["offsets"], spec["total"]
    slot = SLOT_STRIDE.get(args.config)
    if layout in ("rxslot", "csrslot", "txslot"):  # a ring: one frame / packet per slot
        host, lens = synth.to_slots(host, off, slot)
        total = int(lens.sum(dtype=np.uint64))
    # Tx fill writes the frames in place: the fill ignores the fields' old contents, so
    # every step gives the same bytes; parity compares with the oracle's fill of a copy
    orig = host.copy() if layout in ("tx", "txslot") and not args.no_parity else None
    out = np.empty(n, dtype=np.uint8 if frames else np.uint16)
    if args.engines > 0:
        forced = os.environ.get("AIPSTACK_BENCH_FORCE_DEVICE")
        engine_devices = ([int(forced)] * args.engines if forced is not None
                          else list(range(args.engines)))
        eng = A.ChksumEngineGroup(engine_devices, chunk_bytes=args.e2e_chunk_mib << 20,
                                  nstreams=args.e2e_streams)
    else:
        engine_devices = [int(os.environ.get("AIPSTACK_BENCH_FORCE_DEVICE", local_rank))]
        eng = A.ChksumEngine(engine_devices[0], chunk_bytes=args.e2e_chunk_mib << 20,
                             nstreams=args.e2e_streams)
    if not args.e2e_pageable:
        eng.register(host)
    # where each engine's host threads run (its device's NUMA node, CPUs pinned)
    locality = eng.locality() if args.engines > 0 else [eng.locality()]

    def step():
        if layout == "strided":
            eng.strided(host, stride, plen, n, out=out)
        elif layout == "rx":
            eng.rx_verify(host, off, out=out)
        elif layout == "tx":
            eng.tx_fill(host, off, status=out)
        elif layout == "rxslot":
            eng.rx_verify_slotted(host, slot, lens, out=out)
        elif layout == "txslot":
            eng.tx_fill_slotted(host, slot, lens, status=out)
        elif layout == "csrslot":
            eng.slotted(host, slot, lens, out=out)
        else:
            eng.csr(host, off, out=out)

    for _ in range(max(1, args.warmup)):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    import torch
    # Diagnostic, AFTER the timed region (not part of `value`): wall time of each call
    # (every engine call is synchronous: H2D, kernels and D2H of the whole batch).
    per_launch = []
    if args.per_launch and not writer:
        for _ in range(args.steps):
            c0 = time.perf_counter()
            step()
            per_launch.append((time.perf_counter() - c0) * 1e6)
        per_launch.sort()

    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    max_elapsed = float(t.item())
    parity = None
    if not args.no_parity:  # every rank checks its own shard
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        want = np.empty(n, dtype=out.dtype)
        ok_bytes = True
        if layout == "tx":
            lib.oracle_tx_fill_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64,
                                                                         ctypes.c_void_p]
            o = off.astype(np.uint64)
            lib.oracle_tx_fill_batch(orig.ctypes.data, o.ctypes.data, n, want.ctypes.data)
            ok_bytes = np.array_equal(host, orig)
        elif layout == "rx":
            lib.oracle_rx_verify_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64,
                                                                           ctypes.c_void_p]
            o = off.astype(np.uint64)
            lib.oracle_rx_verify_batch(host.ctypes.data, o.ctypes.data, n, want.ctypes.data)
        elif layout == "txslot":
            lib.oracle_tx_fill_slotted.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                                   ctypes.c_void_p, ctypes.c_uint64,
                                                   ctypes.c_void_p]
            ln = np.ascontiguousarray(lens, dtype=np.uint32)
            lib.oracle_tx_fill_slotted(orig.ctypes.data, slot, ln.ctypes.data, n, want.ctypes.data)
            ok_bytes = np.array_equal(host, orig)
        elif layout in ("rxslot", "csrslot"):
            fn = lib.oracle_rx_verify_slotted if layout == "rxslot" else lib.oracle_batch_slotted
            fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                           ctypes.c_void_p] + ([] if layout == "rxslot" else [ctypes.c_uint32])
            ln = np.ascontiguousarray(lens, dtype=np.uint32)
            fn(host.ctypes.data, slot, ln.ctypes.data, n, want.ctypes.data,
               *([] if layout == "rxslot" else [0]))
        elif layout == "strided":
            lib.oracle_batch_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
            lib.oracle_batch_strided(host.ctypes.data, stride, plen, n, want.ctypes.data, 0)
        else:
            lib.oracle_batch_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_uint32]
            o = off.astype(np.uint64)
            lib.oracle_batch_csr(host.ctypes.data, o.ctypes.data, n, want.ctypes.data, 0)
        parity = "bit-exact" if ok_bytes and np.array_equal(out, want) else "MISMATCH"
    dev_index = int(os.environ.get("AIPSTACK_BENCH_FORCE_DEVICE", local_rank))
    props = torch.cuda.get_device_properties(dev_index)
    mine_info = {"rank": rank, "parity": parity, "arch": props.gcnArchName,
                 "pci": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"}
    infos = [mine_info]
    if world > 1:
        infos = [None] * world
        dist.all_gather_object(infos, mine_info)
    if not args.no_parity:
        bad = [i["rank"] for i in infos if i["parity"] != "bit-exact"]
        parity = (f"bit-exact (each of {world} rank(s) checked its own shard vs oracle)" if not bad
                  else f"MISMATCH on rank(s) {bad}")
    pcis = [i["pci"] for i in infos]
    value = total * world * args.steps / max_elapsed / 2**30
    if rank == 0:
        print(json.dumps({
            "metric": "GiB/s " + {"rx": "Rx-verified", "rxslot": "Rx-verified", "tx": "Tx-filled",
                                 "txslot": "Tx-filled"}.get(layout, "checksummed")
                      + " end-to-end (host memory in, host results out)",
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(max_elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u16",
            "data": "synthetic (splitmix64 bytes, seed 42; host memory)",
            "config": {"workload": WORKLOAD_NAMES[args.config], "config": args.config,
                       "host_memory": "pageable (CPU copy into pinned staging)"
                       if args.e2e_pageable else
                       ("registered (hipHostRegister; kernels read it in place, zero copy)"
                        if os.environ.get("AIPSTACK_ENGINE_ZERO_COPY", "1") != "0"
                        else "registered (hipHostRegister, DMA direct)"),
                       "streams": args.e2e_streams, "chunk_MiB": args.e2e_chunk_mib,
                       **({"slot_stride": slot, "ring_bytes": int(host.nbytes),
                           "value_counts": "frame/packet bytes (the lengths), not slot bytes"}
                          if layout in ("rxslot", "csrslot", "txslot") else {}),
                       **({"engines": args.engines, "engine_devices": engine_devices,
                           "engine_group": "one process, disjoint ranges of equal bytes per "
                                           "device; group tickets; pageable ranges staged by "
                                           "a worker thread per device"}
                          if args.engines > 0 else {}),
                       "engine_locality": [{"device": d, "numa_node": nn, "pinned_cpus": pc}
                                           for d, (nn, pc) in zip(engine_devices, locality)]},
            "per_gpu": {"devices": pcis, "arch": [i["arch"] for i in infos],
                        "distinct_devices": len(set(pcis)) == world,
                        "parity": [i["parity"] for i in infos]},
            **({"per_call_us": {"min": round(per_launch[0], 1),
                                "median": round(per_launch[len(per_launch) // 2], 1),
                                "max": round(per_launch[-1], 1)}} if per_launch else {}),
            "parity": parity}), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def frames_check(spec, frames_before, frames_after, status):
    """Frames: statuses (and, for Tx, the filled frames) vs the oracle on the host."""
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    o = spec["offsets"].astype(np.uint64)
    n = spec["n"]
    want = np.empty(n, dtype=np.uint8)
    fn = lib.oracle_rx_verify_batch if spec["layout"] == "rx" else lib.oracle_tx_fill_batch
    fn.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]
    ref = frames_before.copy()
    fn(ref.ctypes.data, o.ctypes.data, n, want.ctypes.data)
    ok = np.array_equal(status, want) and np.array_equal(frames_after, ref)
    return "bit-exact (verdicts/frames vs oracle)" if ok else "MISMATCH"


def slots_check(layout, ring, lens, got):
    """Ring slots: every verdict / checksum vs the C oracle over the same ring."""
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    n = lens.size
    if layout == "rxslot":
        want = np.empty(n, dtype=np.uint8)
        lib.oracle_rx_verify_slotted.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                 ctypes.c_uint64, ctypes.c_void_p]
        lib.oracle_rx_verify_slotted(ring.ctypes.data, 2048, lens.ctypes.data, n, want.ctypes.data)
    else:
        want = np.empty(n, dtype=np.uint16)
        lib.oracle_batch_slotted.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
        lib.oracle_batch_slotted(ring.ctypes.data, 2048, lens.ctypes.data, n, want.ctypes.data, 0)
    return "bit-exact (every slot vs oracle)" if np.array_equal(got, want) else "MISMATCH"


def slot_read_ceiling(config, spec):
    """tools/build/slot_peak on this shard's slot pattern (a child process, after the timed
    region): the payload GB/s a pure read of just the packets' bytes from their slots reaches
    on this GPU -- the ceiling the slotted kernels are compared with."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "build", "slot_peak")
    if not os.path.exists(exe):
        return None
    n = spec["n"]
    args = (["frames", str(n), str(spec["seed"]), "1460", "2048"] if config in ("RX2K", "TX2K")
            else ["mixed", str(n), "2048"])
    if config == "C2K" and spec["first_packet"] != 0:
        return None  # the probe regenerates shard 0's lengths only
    try:
        r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=120)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        d["source"] = "tools/build/slot_peak " + " ".join(args)
        return d
    except (OSError, ValueError, IndexError, subprocess.SubprocessError):
        return None


def fill_ceiling(layout, fbufs, d_off, d_lens, n, stream):
    """The in-place Tx fills' own ceiling (after the timed region): fp_fill of
    tools/fresh_probe.hip -- the fill's read pattern (TX: the chunk's frames streamed as one run;
    TX2K: each slot's frame bytes) plus the two 2-byte field stores per frame, ordinary stores
    as the fill's, no checksum arithmetic -- over copies of the rotation batches, median of 30
    launches after 6. None when the probe library is absent."""
    import statistics
    import torch
    path = os.path.join(ROOT, "tools", "build", "libfresh_probe.so")
    if not os.path.exists(path):
        return None
    fp = ctypes.CDLL(path)
    fp.fp_fill.restype = ctypes.c_int
    fp.fp_fill.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                           ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_void_p]
    copies = [b.clone() for b in fbufs]  # the probe's stores write junk into the fields
    scratch = torch.zeros(1 << 16, dtype=torch.uint32, device=copies[0].device)
    ts = []
    for k in range(36):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        st = fp.fp_fill(copies[k % len(copies)].data_ptr(),
                        d_off.data_ptr() if layout == "tx" else None,
                        0 if layout == "tx" else SLOT_STRIDE["TX2K"],
                        None if layout == "tx" else d_lens.data_ptr(), n, 1, 1,
                        scratch.data_ptr(), stream.cuda_stream)
        b.record(stream)
        b.synchronize()
        if st != 0:
            return None
        if k >= 6:
            ts.append(a.elapsed_time(b) * 1e3)
    del copies
    return {"us": round(statistics.median(ts), 2),
            "source": "tools/build/libfresh_probe.so fp_fill: the fill's read pattern plus its two "
                      "2-byte field stores per frame (ordinary stores), no checksum arithmetic, "
                      f"over {len(fbufs)} rotated copies, median of 30 launches after 6"}


def records_ceiling(fbufs, d_off, n, stream):
    """The records pass's own ceiling (after the timed region): fp_fill_rec of
    tools/fresh_probe.hip -- the frames' read pattern plus an 8-byte record per frame to a
    separate array (ordinary stores, coalesced), no checksum arithmetic -- over the rotation
    copies (read only), median of 30 launches after 6. None without the probe library."""
    import statistics
    import torch
    path = os.path.join(ROOT, "tools", "build", "libfresh_probe.so")
    if not os.path.exists(path):
        return None
    fp = ctypes.CDLL(path)
    fp.fp_fill_rec.restype = ctypes.c_int
    fp.fp_fill_rec.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    dev = fbufs[0].device
    scratch = torch.zeros(1 << 16, dtype=torch.uint32, device=dev)
    rec = torch.empty(n, dtype=torch.int64, device=dev)
    ts = []
    for k in range(36):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        st = fp.fp_fill_rec(fbufs[k % len(fbufs)].data_ptr(), d_off.data_ptr(), 0, None, n, 1, 3,
                            scratch.data_ptr(), rec.data_ptr(), stream.cuda_stream)
        b.record(stream)
        b.synchronize()
        if st != 0:
            return None
        if k >= 6:
            ts.append(a.elapsed_time(b) * 1e3)
    return {"us": round(statistics.median(ts), 2),
            "source": "tools/build/libfresh_probe.so fp_fill_rec: the frames' read pattern plus an "
                      "8-byte record per frame (ordinary stores, 256 B per wave), no checksum "
                      f"arithmetic, over {len(fbufs)} rotated copies, median of 30 launches after 6"}


def hbm_read_ceiling():
    """tools/build/hbm_peak ceiling (a child process, after the timed region): the best GB/s a
    pure 16-byte streaming read reaches on this GPU over 3 rotated 1.57 GB buffers, in the
    kernel's own load shapes -- the measured roofline beside the 8 TB/s spec peak."""
    import subprocess
    exe = os.path.join(ROOT, "tools", "build", "hbm_peak")
    if not os.path.exists(exe):
        return None
    try:
        r = subprocess.run([exe, "ceiling"], capture_output=True, text=True, timeout=120)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except (OSError, ValueError, IndexError, subprocess.SubprocessError):
        return None


def tx_slots_check(ring_before, lens, ring_after, status):
    """Send ring: the filled slots and the statuses vs the oracle's fill of a copy."""
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    n = lens.size
    want = np.empty(n, dtype=np.uint8)
    ref = ring_before.copy()
    lib.oracle_tx_fill_slotted.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p]
    lib.oracle_tx_fill_slotted(ref.ctypes.data, 2048, lens.ctypes.data, n, want.ctypes.data)
    ok = np.array_equal(status, want) and np.array_equal(ring_after, ref)
    return "bit-exact (every slot filled as the oracle fills it)" if ok else "MISMATCH"


def records_check(spec, frames_before, frames_after, records):
    """Tx records: the frames must be untouched; the records applied to a host copy (as the
    engine applies them) must give the oracle's Tx fill, statuses included."""
    import aipstack_amd as A
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    o = spec["offsets"].astype(np.uint64)
    n = spec["n"]
    want = np.empty(n, dtype=np.uint8)
    lib.oracle_tx_fill_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]
    ref = frames_before.copy()
    lib.oracle_tx_fill_batch(ref.ctypes.data, o.ctypes.data, n, want.ctypes.data)
    mine = frames_before.copy()
    got = A.apply_tx_records(mine, o, records)
    ok = (np.array_equal(frames_after, frames_before) and np.array_equal(got, want)
          and np.array_equal(mine, ref))
    return "bit-exact (records applied vs oracle Tx fill; frames untouched)" if ok else "MISMATCH"


def oracle_check(spec, got, threads=1):
    """Check this rank's whole output against the reference's own IpChksumInverted (oracle/_ref,
    `threads` std::threads; where it was built) or else the C oracle, on the same bytes."""
    host = host_shard(spec)
    n = spec["n"]
    want = np.empty(n, dtype=np.uint16)
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libref_chksum.so")
    if os.path.exists(ref_path):
        ref = ctypes.CDLL(ref_path)
        if spec["layout"] == "strided":
            ref.ref_time_batch_strided.restype = ctypes.c_double
            ref.ref_time_batch_strided.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                   ctypes.c_uint64, ctypes.c_uint32,
                                                   ctypes.c_uint64, ctypes.c_void_p]
            ref.ref_time_batch_strided(threads, 0, host.ctypes.data, spec["stride"], spec["plen"],
                                       n, want.ctypes.data)  # 0 timed passes: one pass
        else:
            ref.ref_time_batch_csr.restype = ctypes.c_double
            ref.ref_time_batch_csr.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
            o = spec["offsets"].astype(np.uint64)
            ref.ref_time_batch_csr(threads, 0, host.ctypes.data, o.ctypes.data, n,
                                   want.ctypes.data)
        return ("bit-exact (whole shard vs reference)" if np.array_equal(got, want)
                else "MISMATCH")
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    if spec["layout"] == "strided":
        lib.oracle_batch_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
        lib.oracle_batch_strided(host.ctypes.data, spec["stride"], spec["plen"], n,
                                 want.ctypes.data, 0)
    else:
        lib.oracle_batch_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_uint32]
        o = spec["offsets"].astype(np.uint64)
        lib.oracle_batch_csr(host.ctypes.data, o.ctypes.data, n, want.ctypes.data, 0)
    return "bit-exact (whole batch vs oracle)" if np.array_equal(got, want) else "MISMATCH"


KERNEL_SOURCES = ("aipstack_amd/csrc/chksum_device.h", "aipstack_amd/csrc/chksum_kernels.hip",
                  "aipstack_amd/csrc/frame_kernels.hip")


def device_code_digest(lib_path=None):
    """sha256 (16 hex digits) of the device code objects in libaipstack_chksum.so (its
    .hip_fatbin section, read with a minimal ELF64 section-table parser): identifies the
    kernels a PMC measurement was taken on, and changes only when device code does (host-side
    edits of the .hip files leave it alone). None if the section cannot be read."""
    import hashlib
    import struct
    path = lib_path or os.path.join(ROOT, "aipstack_amd", "lib", "libaipstack_chksum.so")
    try:
        with open(path, "rb") as f:
            data = f.read()
        if data[:4] != b"\x7fELF" or data[4] != 2:
            return None
        shoff, = struct.unpack_from("<Q", data, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
        def sec(i):
            name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize)
            return name, off, size
        _, stroff, _ = sec(shstrndx)
        for i in range(shnum):
            name, off, size = sec(i)
            end = data.index(b"\0", stroff + name)
            if data[stroff + name:end] == b".hip_fatbin":
                return hashlib.sha256(data[off:off + size]).hexdigest()[:16]
    except (OSError, ValueError, struct.error):
        return None
    return None


def kernel_source_digest():
    """sha256 (16 hex digits) of the device-code sources: identifies the kernels a PMC
    measurement was taken on (tools/pmc_summary.py records it with every entry)."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _pmc_traffic(config):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), measured
    by tools/pmc_run.sh on the same command: (2 x FETCH_SIZE + WRITE_SIZE) KiB, the x2
    being the gfx950 correction of MI355X_MICROARCH.md (HBM section). Reported only if the
    entry was measured on this library's device code (its device_code digest equals
    device_code_digest() of the loaded .so); a stale entry gives null here and its value
    under roofline.traffic_stale."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(config, {})
        v = e.get("hbm_bytes_per_launch")
        if v is None:
            return None, None
        if e.get("device_code") is None or e.get("device_code") != device_code_digest():
            return None, {"hbm_bytes_per_launch": int(v),
                          "measured_on_device_code": e.get("device_code"),
                          "note": "PMC entry predates the current device code"}
        return int(v), None
    except (OSError, ValueError):
        return None, None

if __name__ == "__main__":
    main()
