"""Golden cases for the reference stack's checksum call sequences (tests/cpp/call_sites.inc).

The same C++ text is compiled against the reference (oracle/_ref/libref_chksum.so, symbols
``ref_cs_*``) and against this repo's Chksum.hpp (tests/cpp/build/libhpp_shim.so,
``hpp_cs_*``). ``make_cases()`` builds deterministic inputs; ``evaluate(lib, prefix, case,
blob)`` runs one case through either library. make_golden.py records the reference's
answers into call_site_cases.json; tests/test_host_surface.py replays them on the repo's side.

A case's IpBufRef chain is an optional explicit first node (``hdr``, hex: a header built
here, e.g. an IPv4 header with a correct or corrupted checksum) followed by chunks of the
golden blob (``chunks``: [offset, length]); ``offset`` / ``tot_len`` as in IpBufRef.
"""
from __future__ import annotations

import ctypes

import numpy as np

SITES = ("tcp_rx", "udp_tx", "udp_rx", "tcp_tx", "ip4_tx", "ip4_rx", "icmp")


def _bind(lib, prefix):
    vp, sz, u16, u32, u8 = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint16, ctypes.c_uint32,
                            ctypes.c_uint8)
    chain = [vp, vp, sz, sz, sz]
    sig = {
        "tcp_rx": (u16, [u32, u32] + chain),
        "udp_tx": (u16, [u32, u32] + chain),
        "udp_rx": (ctypes.c_int, [u32, u32, u16] + chain),
        "tcp_tx": (u16, [u16, u16, u32, u16, u32, u32, u32, u16] + chain + [vp]),
        "ip4_tx": (u16, [u16, u8, u8, u32, u32, u16, u16, vp]),
        "ip4_rx": (ctypes.c_int, chain + [vp]),
        "icmp": (u16, chain),
    }
    fns = {}
    for name, (res, args) in sig.items():
        f = getattr(lib, f"{prefix}_cs_{name}")
        f.restype = res
        f.argtypes = args
        fns[name] = f
    return fns


def _chain_args(case, blob):
    """(keepalive, [ptrs, lens, nchunks, offset, tot_len]) for the case's chain."""
    ptrs, lens, keep = [], [], []
    if case.get("hdr"):
        h = np.frombuffer(bytes.fromhex(case["hdr"]), dtype=np.uint8).copy()
        keep.append(h)
        ptrs.append(h.ctypes.data)
        lens.append(h.size)
    for o, l in case["chunks"]:
        ptrs.append(blob.ctypes.data + o)
        lens.append(l)
    k = max(len(ptrs), 1)
    p = (ctypes.c_void_p * k)(*ptrs)
    ln = (ctypes.c_size_t * k)(*lens)
    keep += [p, ln]
    return keep, [p, ln, len(ptrs), case["offset"], case["tot_len"]]


def evaluate(lib, prefix, case, blob):
    """The library's answer for one case: an int, or [int, state] for the State sites."""
    fns = getattr(lib, "_cs_bound_" + prefix, None)
    if fns is None:
        fns = _bind(lib, prefix)
        setattr(lib, "_cs_bound_" + prefix, fns)
    site, a = case["site"], case["args"]
    if site == "ip4_tx":
        st = ctypes.c_uint32(0)
        r = fns[site](*a, ctypes.byref(st))
        return [int(r), int(st.value)]
    keep, ch = _chain_args(case, blob)
    if site == "tcp_tx":
        st = ctypes.c_uint32(0)
        r = fns[site](*a, *ch, ctypes.byref(st))
        return [int(r), int(st.value)]
    if site == "ip4_rx":
        dl = ctypes.c_size_t(0)
        r = fns[site](*ch, ctypes.byref(dl))
        return [int(r), int(dl.value)]
    r = fns[site](*a, *ch)
    del keep
    return int(r)


def _be16(x):
    return bytes([(x >> 8) & 0xFF, x & 0xFF])


def _ip4_header(rng, ihl, total_len, proto, good):
    """An IPv4 header of `ihl` words (version 4) with a correct (or corrupted) checksum."""
    h = bytearray(rng.integers(0, 256, size=4 * max(ihl, 5), dtype=np.uint8).tobytes())
    h[0] = 0x40 | (ihl & 0xF)
    h[2:4] = _be16(total_len)
    h[6:8] = _be16(int(rng.choice([0, 0x4000, 0x2000, 0x0123])))
    h[9] = proto
    h[10:12] = b"\x00\x00"
    s = 0
    for i in range(0, 4 * max(ihl, 5), 2):
        s += (h[i] << 8) | h[i + 1]
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    c = (~s) & 0xFFFF
    if not good:
        c ^= 1 << int(rng.integers(0, 16))
    h[10:12] = _be16(c)
    return bytes(h)


def make_cases(blob, seed=2024):
    rng = np.random.default_rng(seed)
    cases = []

    def u32():
        return int(rng.integers(0, 2**32))

    def u16():
        return int(rng.integers(0, 2**16))

    def chunks(max_n=4):
        n = int(rng.integers(1, max_n + 1))
        out = []
        for _ in range(n):
            ln = int(rng.choice([0, 1, 2, 3, int(rng.integers(0, 64)), int(rng.integers(0, 1500))]))
            out.append([int(rng.integers(0, 60000)), ln])
        return out

    def ref_span(ch, hdr_len=0, allow_short=True):
        lens = ([hdr_len] if hdr_len else []) + [l for _, l in ch]
        total = sum(lens)
        first = lens[0] if lens else 0
        offset = int(rng.integers(0, first + 1)) if rng.random() < 0.3 else 0
        tot_len = total - offset
        if allow_short and rng.random() < 0.25 and tot_len > 0:
            tot_len = int(rng.integers(0, tot_len + 1))
        return offset, tot_len

    for _ in range(150):
        ch = chunks()
        off, tl = ref_span(ch)
        cases.append({"site": "tcp_rx", "args": [u32(), u32()], "hdr": "", "chunks": ch,
                      "offset": off, "tot_len": tl})
        ch = chunks()
        off, tl = ref_span(ch)
        cases.append({"site": "udp_tx", "args": [u32(), u32()], "hdr": "", "chunks": ch,
                      "offset": off, "tot_len": tl})
        ch = chunks()
        off, tl = ref_span(ch)
        cases.append({"site": "udp_rx", "args": [u32(), u32(), int(rng.choice([0, u16()]))],
                      "hdr": "", "chunks": ch, "offset": off, "tot_len": tl})
        ch = chunks(3)
        off, tl = ref_span(ch)
        cases.append({"site": "tcp_tx",
                      "args": [u16(), u16(), u32(), u16(), u32(), u32(), u32(), u16()],
                      "hdr": "", "chunks": ch, "offset": off, "tot_len": tl})
        cases.append({"site": "ip4_tx",
                      "args": [int(rng.choice([0, 0x4000, u16()])), int(rng.integers(0, 256)),
                               int(rng.choice([1, 6, 17, int(rng.integers(0, 256))])), u32(),
                               u32(), u16(), u16()],
                      "hdr": "", "chunks": [], "offset": 0, "tot_len": 0})
        ch = chunks(3)
        off, tl = ref_span(ch)
        cases.append({"site": "icmp", "args": [], "hdr": "", "chunks": ch, "offset": off,
                      "tot_len": tl})
    # all-0xFF / all-zero data through the L4 sites (carry folding, 0 vs 0xFFFF)
    f0, z0 = 110000, 100000
    for o, ln in ((f0, 1023), (f0 + 1, 1460), (z0, 1460), (z0 + 3, 1)):
        for site in ("tcp_rx", "udp_tx", "icmp"):
            cases.append({"site": site, "args": [] if site == "icmp" else [0xFFFFFFFF, 0],
                          "hdr": "", "chunks": [[o, ln]], "offset": 0, "tot_len": ln})
    # Datagrams whose pseudo-header + data sum is 0xFFFF: a leading 2-byte node is set to
    # make it so. UDP Tx then computes 0 and sends 0xFFFF (udp/IpUdpProto.h:176-178); TCP
    # and UDP Rx verify them (getChksum == 0).
    for site, proto in (("udp_tx", 17), ("tcp_rx", 6), ("udp_rx", 17)):
        for _ in range(12):
            ch = chunks(3)
            a, b = u32(), u32()
            tot = 2 + sum(l for _, l in ch)
            s = (a >> 16) + (a & 0xFFFF) + (b >> 16) + (b & 0xFFFF) + proto + (tot & 0xFFFF)
            pos = 2
            for o, l in ch:
                d = blob[o:o + l]
                for i in range(l):
                    s += int(d[i]) << (8 if (pos + i) % 2 == 0 else 0)
                pos += l
            fix = (-s) % 0xFFFF
            args = [a, b] + ([u16() | 1] if site == "udp_rx" else [])
            cases.append({"site": site, "args": args, "hdr": _be16(fix).hex(), "chunks": ch,
                          "offset": 0, "tot_len": tot, "expect": {"udp_tx": 0xFFFF, "tcp_rx": 0,
                                                                  "udp_rx": 3}[site]})
    # IPv4 Rx header checks: fast path, options, bad version / IHL, header split over two
    # nodes (hasHeader fails), total length too small / too large, corrupted checksums
    for _ in range(250):
        ihl = int(rng.choice([5, 5, 5, 6, 8, 15, 4, 3]))
        hl = 4 * max(ihl, 5)
        payload = chunks(2)
        plen = sum(l for _, l in payload)
        kind = rng.random()
        total = hl + plen
        if kind < 0.1:
            total = hl - 2
        elif kind < 0.2:
            total = hl + plen + int(rng.integers(1, 40))
        elif kind < 0.4:
            total = hl + int(rng.integers(0, plen + 1))
        hdr = bytearray(_ip4_header(rng, ihl, total & 0xFFFF, int(rng.choice([1, 6, 17])),
                                    good=rng.random() < 0.8))
        if rng.random() < 0.08:
            hdr[0] = 0x55 if rng.random() < 0.5 else 0x65
        if rng.random() < 0.1:  # only part of the header in the first node: hasHeader fails
            cut = int(rng.integers(1, hl))
            cases.append({"site": "ip4_rx", "args": [], "hdr": bytes(hdr[:cut]).hex(),
                          "chunks": payload, "offset": 0, "tot_len": cut + plen})
            continue
        off = int(rng.integers(0, 3)) if rng.random() < 0.2 else 0
        pre = bytes(rng.integers(0, 256, size=off, dtype=np.uint8))
        cases.append({"site": "ip4_rx", "args": [], "hdr": (pre + bytes(hdr)).hex(),
                      "chunks": payload, "offset": off, "tot_len": hl + plen})
    return cases
