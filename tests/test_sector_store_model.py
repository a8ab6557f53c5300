"""CPU model of the in-place Tx fills' sector stores (frame_kernels.hip: FieldSectors,
pick_sectors, patch_be16, store_frame_sectors), step for step, checked before any GPU runs it.

A fill writes two big-endian 16-bit fields per frame (the IPv4 header checksum at frame byte
24, the L4 checksum at byte fld). The SECT form writes each field's whole 32-byte sector from
the header bytes the lane read, patched, instead of a 2-byte store. The model replays the
device's decisions (which sectors go out whole, which fields are patched into which sector,
which fields keep a 2-byte store) on a byte array for frames at every start alignment,
length and field offset, and checks the bytes against the plain 2-byte writes: only the
frame's own fields change, whatever the order of the stores, and no byte outside [S, E) is
written.
"""
import itertools

import numpy as np


def dword_keep(a, b):
    a, b = min(max(a, 0), 4), min(max(b, 0), 4)
    return ((0xFFFFFFFF >> (32 - 8 * (b - a))) << (8 * a)) & 0xFFFFFFFF if b > a else 0


def bswap16(x):
    return ((x & 0xFF) << 8) | ((x >> 8) & 0xFF)


def patch_be16(d, b, v):
    """patch_be16: d = 8 little-endian dwords of a sector; v big-endian at byte b (-1..31)."""
    w = bswap16(v)
    for k in range(8):
        p = b - 4 * k
        m = dword_keep(p, p + 2)
        val = ((w << ((8 * p) & 31)) & 0xFFFFFFFF) if p >= 0 else (w >> 8)
        d[k] = (d[k] & ~m & 0xFFFFFFFF) | (val & m)


def pick_sectors(mem, S, E, ip_ok, l4, fld):
    """pick_sectors: which sectors go out whole, and their bytes as read (from the lane's
    header blocks = memory before any store of this frame)."""
    xi, xl = S + 24, S + fld
    ai, al = xi & ~31, xl & ~31
    in_i = ip_ok and ai >= S and ai + 32 <= E
    in_l = l4 and al >= S and al + 32 <= E and not (in_i and al == ai)
    secs = [mem[a:a + 32].copy().view("<u4").astype(np.uint64).tolist() for a in (ai, al)]
    return (1 if in_i else 0) | (2 if in_l else 0), secs


def store_frame_sectors(mem, S, w0, wi, wl, fld, mode, secs, order):
    """store_frame_sectors; `order` permutes the stores: overlapping stores of one frame
    carry the same bytes, so the result must not depend on their order."""
    xi, xl = S + 24, S + fld
    sa, sb = xi & ~31, xl & ~31
    ia, la, ib, lb = xi - sa, xl - sa, xi - sb, xl - sb
    wa, wb = bool(mode & 1), bool(mode & 2)
    stores = []
    ci = cl = False
    if wa:
        d = secs[0]
        if wi:
            patch_be16(d, ia, w0 & 0xFFFF)
        if wl and -1 <= la <= 31:
            patch_be16(d, la, w0 >> 16)
        ci = ia <= 30
        cl = 0 <= la <= 30
        stores.append((sa, np.array(d, dtype=np.uint32).view(np.uint8)))
    if wb:
        d = secs[1]
        if wl:
            patch_be16(d, lb, w0 >> 16)
        if wi and -1 <= ib <= 31:
            patch_be16(d, ib, w0 & 0xFFFF)
        cl = cl or lb <= 30
        ci = ci or 0 <= ib <= 30
        stores.append((sb, np.array(d, dtype=np.uint32).view(np.uint8)))
    if wi and not ci:
        stores.append((xi, np.array([(w0 >> 8) & 0xFF, w0 & 0xFF], dtype=np.uint8)))
    if wl and not cl:
        stores.append((xl, np.array([(w0 >> 24) & 0xFF, (w0 >> 16) & 0xFF], dtype=np.uint8)))
    for k in order(len(stores)):
        a, data = stores[k]
        mem[a:a + data.size] = data
    return stores


def test_sector_stores_match_field_stores():
    rng = np.random.default_rng(5)
    fields = sorted({36, 40, 50} | set(range(36, 92, 2)))  # ICMP / UDP / TCP, IPv4 options
    lengths = [34, 42, 54, 59, 60, 61, 63, 64, 65, 70, 73, 90, 95, 96, 97, 100, 128, 200]
    cases = 0
    for s32, fld, ln in itertools.product(range(32), fields, lengths):
        if fld + 2 > ln:
            continue
        for ip_ok, l4 in ((True, True), (True, False)):
            S = 64 + s32
            E = S + ln
            mem = rng.integers(0, 256, S + ln + 96, dtype=np.uint8)
            w0 = int(rng.integers(0, 1 << 32))
            want = mem.copy()
            want[S + 24:S + 26] = [(w0 >> 8) & 0xFF, w0 & 0xFF]
            if l4:
                want[S + fld:S + fld + 2] = [(w0 >> 24) & 0xFF, (w0 >> 16) & 0xFF]
            mode, secs = pick_sectors(mem, S, E, ip_ok, l4, fld)
            for order in (lambda n: range(n), lambda n: reversed(range(n))):
                got = mem.copy()
                stores = store_frame_sectors(got, S, w0, ip_ok, l4, fld, mode,
                                             [list(x) for x in secs], order)
                assert np.array_equal(got, want), (s32, fld, ln, ip_ok, l4)
                for a, data in stores:  # nothing outside the frame is ever written
                    assert S <= a and a + data.size <= E
            cases += 1
    assert cases > 3000


def test_common_layouts_take_whole_sectors():
    """Slots (frames at 32-byte aligned starts) of 64+ bytes write both fields as whole sectors
    (TCP / UDP / ICMP); frames starting 1..7 bytes into a sector cannot (sector A starts
    before S) and keep the IPv4 field's 2-byte store."""
    mem = np.zeros(512, dtype=np.uint8)
    for fld in (36, 40, 50):
        mode, _ = pick_sectors(mem, 64, 64 + 1514, True, True, fld)
        assert mode == 3
        mode, _ = pick_sectors(mem, 64, 64 + 60, True, True, fld)
        assert mode == 1  # the L4 sector would pass a 60-byte frame's end
    for s32 in range(1, 8):
        mode, _ = pick_sectors(mem, 64 + s32, 64 + s32 + 1514, True, True, 50)
        assert not mode & 1
