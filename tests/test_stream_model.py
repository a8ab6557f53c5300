"""CPU model of the kernels' stream mode (chksum_device.h: stream_ok / sum_stream_chunk),
step for step, checked bit-exact against the oracle before any GPU runs it.

Stream mode reads a 64-packet chunk whose packets lie back to back as one contiguous run of
16-byte segments, 64 per window (one wave instruction), and gets each packet's exact sum of
little-endian 16-bit halves as a difference of prefixes H(S_{j+1}) - H(S_j) kept mod 2^32.
This model reproduces the windows, the lane scan, the per-boundary partial segment, the
bytes past the chunk end in its last segment, the mod-2^32 arithmetic and the finish
(fold, byte swap iff S even), so a wrong index or mask shows up here on the CPU.
"""
import zlib

import numpy as np
import pytest

M32 = 0xFFFFFFFF


def _halves_of_segments(buf, a, nseg, limit):
    """Per segment: sum of the 8 little-endian halves of buf[a + 16k : a + 16k + 16] (segments
    at or past `limit` bytes from a read as 0: the buffer descriptor's range check)."""
    raw = np.zeros(nseg * 16, dtype=np.uint8)
    take = min(nseg * 16, limit, buf.size - a)
    raw[:take] = buf[a:a + take]
    h = raw.view("<u2").astype(np.uint64).reshape(nseg, 8)
    return h.sum(axis=1), raw


def _below(raw_seg, t):
    """Halves-sum of the bytes [0, t) of one 16-byte segment (the rest as 0)."""
    s = raw_seg.copy()
    s[t:] = 0
    return int(s.view("<u2").astype(np.uint64).sum())


def stream_chunk_model(buf, S, E, cnt, U=4):
    """sum_stream_chunk for lanes 0..63 (S, E: per-lane packet bounds, lanes >= cnt ignored)."""
    X1 = int(E[cnt - 1])
    S = [int(S[j]) if j < cnt else X1 for j in range(64)]
    A = S[0] & ~15
    span = X1 - A
    nseg = (span + 15) >> 4
    nwin = (nseg + 63) >> 6
    padded = ((nwin + U - 1) // U) * U          # windows the loop touches (zeros past nseg)
    seg, raw = _halves_of_segments(buf, A, max(padded * 64, 1), nseg * 16)
    seg = seg[:padded * 64]
    hb = [0] * 64
    carry = 0
    x_hi = 0
    xt = span & 15
    for w in range(padded):
        s = seg[w * 64:(w + 1) * 64]
        incl = np.cumsum(s)
        excl = incl - s
        for j in range(64):
            boff = S[j] - A
            if boff >> 10 == w:
                o = (boff >> 4) & 63
                part = int(excl[o]) + _below(raw[(w * 64 + o) * 16:(w * 64 + o) * 16 + 16],
                                             boff & 15)
                hb[j] = (carry + part) & M32
        if nseg > 0 and w == (nseg - 1) >> 6 and xt != 0:
            k = nseg - 1
            full = int(seg[k])
            x_hi = full - _below(raw[k * 16:k * 16 + 16], xt)
        carry = (carry + int(incl[63])) & M32
    hx = (carry - x_hi) & M32
    for j in range(64):
        if S[j] == X1:
            hb[j] = hx
    sums = []
    for j in range(64):
        hn = hx if j == 63 else hb[j + 1]
        sums.append(((hn - hb[j]) & M32) if j < cnt else 0)
    return sums


def finish(sums, S, final=False):
    out = []
    for s, st in zip(sums, S):
        r = (s & 0xFFFF) + (s >> 16)
        r = (r & 0xFFFF) + (r >> 16)
        if (st & 1) == 0:
            r = ((r & 0xFF) << 8) | (r >> 8)
        out.append((~r & 0xFFFF) if final else r)
    return out


def stream_ok_model(S, E, cnt):
    for j in range(cnt):
        if E[j] - S[j] > (1 << 17) - 1 or E[j] < S[j]:
            return False
        if j + 1 < cnt and E[j] != S[j + 1]:
            return False
    return True


def model_batch_csr(buf, off, U=4):
    n = off.size - 1
    out = np.zeros(n, dtype=np.uint16)
    for p0 in range(0, n, 64):
        cnt = min(64, n - p0)
        S = [int(off[p0 + j]) for j in range(cnt)]
        E = [int(off[p0 + j + 1]) for j in range(cnt)]
        assert stream_ok_model(S, E, cnt)
        sums = stream_chunk_model(buf, S, E, cnt, U)
        out[p0:p0 + cnt] = finish(sums[:cnt], S)
    return out


def _layout(rng, n, lens_choice, base):
    lens = rng.choice(lens_choice, size=n)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return off + base


@pytest.mark.parametrize("U", [2, 4])
@pytest.mark.parametrize("case", ["tiny", "mixed", "mtu", "long", "empty_tail"])
def test_stream_model_matches_oracle(oracle, case, U):
    rng = np.random.default_rng(hash((case, U)) % 2**32)
    base = int(rng.integers(0, 16))
    if case == "tiny":          # many packets per 16-byte segment, empties, odd lengths
        off = _layout(rng, 300, [0, 0, 1, 2, 3, 5, 7, 16, 17, 31], base)
    elif case == "mixed":
        off = _layout(rng, 200, list(range(64, 1501, 97)) + [65, 1499], base)
    elif case == "mtu":
        off = _layout(rng, 130, [1500], base)
    elif case == "long":        # a chunk spanning many windows; 65535-byte packets
        off = _layout(rng, 70, [65535, 9000, 1, 0], base)
    else:                       # trailing empty packets at a 1 KiB-aligned chunk end
        lens = np.array([1024] * 10 + [0] * 54, dtype=np.int64)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    buf = rng.integers(0, 256, size=int(off[-1]) + 64, dtype=np.uint8)
    # some all-zero and all-0xFF packets
    for j in range(0, off.size - 1, 11):
        buf[off[j]:off[j + 1]] = 0 if j % 2 else 0xFF
    want = oracle.batch_csr(buf, off)
    got = model_batch_csr(buf, off, U)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def test_stream_model_halves_sum_is_exact_for_max_len():
    # 2^17 - 1 bytes of 0xFF: halves-sum = 65535 * 65535 + 0xFF < 2^32 (no wrap ambiguity)
    n = (1 << 17) - 1
    assert (n // 2) * 0xFFFF + 0xFF < 2 ** 32


# ---- gathered stream (chksum_device.h: sum_gathered_chunks, the chain kernel) ----------

def gathered_model(buf, a, l, U=4):
    """sum_gathered_chunks for one 64-chunk group: lane j = chunk [a[j], a[j] + l[j]) of buf
    (absolute offsets into buf). Cleaned segments (bytes outside the owner chunk masked by
    the loading lane), one boundary per lane at its chunk's first segment; returns each
    lane's halves-sum (mod 2^32)."""
    k = len(a)
    a = [int(x) for x in a] + [0] * (64 - k)
    l = [int(x) for x in l] + [0] * (64 - k)
    rs = [x & 15 for x in a]
    ns = [((rs[j] + l[j] + 15) >> 4) if l[j] else 0 for j in range(64)]
    incl = np.cumsum(ns)
    cs = [int(incl[j] - ns[j]) for j in range(64)]
    T = int(incl[63])
    if T == 0:
        return [0] * 64
    nwin = (T + 63) >> 6
    gbase = [(a[j] & ~15) - 16 * cs[j] for j in range(64)]
    first = [cs[j] for j in range(64)]
    last = [cs[j] + ns[j] - 1 for j in range(64)]
    tail_keep = [((rs[j] + l[j] - 1) & 15) + 1 for j in range(64)]
    g = [0] * 64
    cur, carry = 0, 0
    npairs = (nwin + 2 * U - 1) // (2 * U)
    for w in range(npairs * 2 * U):            # whole pairs of groups, as the kernel
        mark = [-1] * 64
        for j in range(64):
            if ns[j] and (cs[j] >> 6) == w:
                mark[cs[j] & 63] = j
        m = list(np.maximum.accumulate(mark))
        m = [cur if x < 0 else int(x) for x in m]
        cur = m[63]
        seg = np.zeros(64, dtype=np.uint64)
        for lane in range(64):
            c0 = w * 64 + lane
            c = min(c0, T - 1)
            o = m[lane]
            head = rs[o] if c == first[o] else 0
            tail = tail_keep[o] if c == last[o] else 16
            raw = np.zeros(16, dtype=np.uint8)
            addr = gbase[o] + 16 * c
            raw[:] = buf[addr:addr + 16]
            raw[:head] = 0
            raw[tail:] = 0
            if c0 < T:
                seg[lane] = int(raw.view("<u2").astype(np.uint64).sum())
        inc = np.cumsum(seg)
        exc = inc - seg
        for j in range(64):
            if cs[j] >> 6 == w:
                g[j] = (carry + int(exc[cs[j] & 63])) & M32
        carry = (carry + int(inc[63])) & M32
    for j in range(64):
        if cs[j] >> 6 >= nwin:
            g[j] = carry
    return [((g[j + 1] if j < 63 else carry) - g[j]) & M32 for j in range(64)]


def gathered_edge_model(buf, a, l, U=4):
    """sum_gathered_chunks in AIPSTACK_GATHER_MODE 2 (the default since round 4): the stream
    sums WHOLE segments; each window's chunk-start mask (one bit per non-empty chunk's first
    segment) and the end mask derived from it (the lane before a start, lane 63 when the next
    window starts with a chunk, and the stream's last segment) copy the loaded segment into
    the owner's LDS edge slots; each lane then subtracts the bytes of its first segment below
    its start and of its last segment from its end on. Returns each lane's halves-sum."""
    k = len(a)
    a = [int(x) for x in a] + [0] * (64 - k)
    l = [int(x) for x in l] + [0] * (64 - k)
    rs = [x & 15 for x in a]
    ns = [((rs[j] + l[j] + 15) >> 4) if l[j] else 0 for j in range(64)]
    incl = np.cumsum(ns)
    cs = [int(incl[j] - ns[j]) for j in range(64)]
    T = int(incl[63])
    if T == 0:
        return [0] * 64
    nwin = (T + 63) >> 6
    nonempty = [j for j in range(64) if ns[j]]
    rank = {j: r for r, j in enumerate(nonempty)}
    gbase = {rank[j]: (a[j] & ~15) - 16 * cs[j] for j in nonempty}
    starts = [0] * (nwin + 1)
    for j in nonempty:
        starts[cs[j] >> 6] |= 1 << (cs[j] & 63)
    edge = {}
    g = [0] * 64
    carry, base = 0, 0
    for w in range(nwin):
        ms = starts[w]
        me = (ms >> 1) | ((starts[w + 1] & 1) << 63)
        if (T - 1) >> 6 == w:
            me |= 1 << ((T - 1) & 63)
        seg = np.zeros(64, dtype=np.uint64)
        for lane in range(64):
            below = bin(ms & ((1 << (lane + 1)) - 1)).count("1")
            r = base + below - 1
            c0 = w * 64 + lane
            c = min(c0, T - 1)
            addr = gbase[r] + 16 * c
            raw = np.array(buf[addr:addr + 16], dtype=np.uint8)
            if (ms >> lane) & 1:
                edge[(r, 0)] = raw.copy()
            if (me >> lane) & 1:
                edge[(r, 1)] = raw.copy()
            if c0 < T:
                seg[lane] = int(raw.view("<u2").astype(np.uint64).sum())
        base += bin(ms).count("1")
        inc = np.cumsum(seg)
        exc = inc - seg
        for j in range(64):
            if cs[j] >> 6 == w:
                g[j] = (carry + int(exc[cs[j] & 63])) & M32
        carry = (carry + int(inc[63])) & M32
    for j in range(64):
        if cs[j] >> 6 >= nwin:
            g[j] = carry
    out = []
    for j in range(64):
        v = ((g[j + 1] if j < 63 else carry) - g[j]) & M32
        if ns[j]:
            first, last = edge[(rank[j], 0)].copy(), edge[(rank[j], 1)].copy()
            t = ((rs[j] + l[j] - 1) & 15) + 1
            first[rs[j]:] = 0          # the bytes below the start
            last[:t] = 0               # the bytes from the end on
            v = (v - int(first.view("<u2").astype(np.uint64).sum())
                 - int(last.view("<u2").astype(np.uint64).sum())) & M32
        out.append(v)
    return out


@pytest.mark.parametrize("model", ["masked", "edge"])
@pytest.mark.parametrize("U", [2, 4])
@pytest.mark.parametrize("case", ["headers_and_ring", "tiny", "sparse", "long", "shared_segments"])
def test_gathered_model_matches_oracle(oracle, case, U, model):
    rng = np.random.default_rng(hash(("g", case, U)) % 2**32)
    buf = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    buf[300000:310000] = 0xFF
    buf[310000:320000] = 0
    n = 64 if case != "tiny" else int(rng.integers(1, 65))
    if case == "headers_and_ring":   # 20-B headers at a 32-B stride, payload ring pieces
        a, l = [], []
        pay = 500000 + int(rng.integers(0, 16))
        for i in range(n):
            if i % 3 == 0:
                a.append(1000 + 32 * i)
                l.append(20)
            else:
                cut = int(rng.integers(1, 1460))
                a.append(pay)
                l.append(cut if i % 3 == 1 else 1460 - cut)
                pay += l[-1]
    elif case == "tiny":
        a = [int(x) for x in rng.integers(0, 200000, n)]
        l = [int(x) for x in rng.choice([0, 1, 2, 3, 15, 16, 17], n)]
    elif case == "sparse":           # far apart, odd addresses, some 0xFF / zero chunks
        a = [int(x) for x in rng.integers(0, 900000, n)]
        l = [int(x) for x in rng.integers(0, 1600, n)]
        a[5], l[5] = 300001, 999
        a[6], l[6] = 310003, 1001
    elif case == "long":             # chunks of up to 65535 bytes spanning many windows
        a = [int(x) for x in rng.integers(0, 900000, n)]
        l = [int(x) for x in rng.choice([0, 1, 65535, 9000, 17], n)]
    else:                            # back-to-back chunks sharing 16-B segments
        a, l = [], []
        p = 777
        for i in range(n):
            ln = int(rng.integers(0, 40))
            a.append(p)
            l.append(ln)
            p += ln
    sums = (gathered_model if model == "masked" else gathered_edge_model)(buf, a, l, U)
    for j in range(n):
        s = sums[j]
        r = (s & 0xFFFF) + (s >> 16)
        r = (r & 0xFFFF) + (r >> 16)
        if (a[j] & 1) == 0:
            r = ((r & 0xFF) << 8) | (r >> 8)
        assert r == oracle.inverted(buf, a[j], l[j]), (case, j, a[j], l[j])


# ---- frame stream with headers captured from the stream (frame_kernels.hip) -------------

def captured_frame_model(buf, S, E, l4s, l4e):
    """process_chunk's gathered stream for one back-to-back chunk: the union of the frames'
    header blocks [A0_j, (S_j + 128) & ~31) within the run goes to a compact array in
    window order (slot = union segments below), each lane reads its blocks back from its
    compact slot, and the L4 halves-sum is H(l4e) - H(l4s) from H at every A0_j. Returns
    (sums, blocks_ok); a frame whose L4 end lies past its blocks and before its end
    ('far') gets None."""
    cnt = len(S)
    A = S[0] & ~15
    X1 = E[-1]
    nseg = (X1 - A + 15) >> 4
    raw = np.zeros(nseg * 16, dtype=np.uint8)
    raw[:X1 - A] = buf[A:X1]
    full = raw.view("<u2").astype(np.uint64).reshape(nseg, 8).sum(axis=1)
    H = np.concatenate([[0], np.cumsum(full)])
    hx = int(H[nseg]) - (int(full[nseg - 1]) - _below(raw[(nseg - 1) * 16:nseg * 16],
                                                       (X1 - A) & 15 or 16))
    r0 = [((s & ~15) - A) >> 4 for s in S]
    r1 = [min(r0[j] + ((((s + 128) & ~31) - (s & ~15)) >> 4), nseg) for j, s in enumerate(S)]
    bit = np.zeros(nseg, dtype=bool)
    for j in range(cnt):
        bit[r0[j]:r1[j]] = True
    slots = [raw[g * 16:g * 16 + 16] for g in range(nseg) if bit[g]]   # window order
    cslot, prev = [], 0
    count = 0
    for j in range(cnt):
        u = max(r0[j], prev)
        nw = max(0, r1[j] - u)
        cslot.append(count - (u - r0[j]))
        count += nw
        prev = r1[j]
    assert count == len(slots)
    blocks_ok = True
    segs = []
    for j in range(cnt):
        mine = [slots[cslot[j] + i] if i < r1[j] - r0[j] else np.zeros(16, np.uint8)
                for i in range(8)]
        want = [raw[(r0[j] + i) * 16:(r0[j] + i + 1) * 16] if r0[j] + i < r1[j]
                else np.zeros(16, np.uint8) for i in range(8)]
        blocks_ok &= all(np.array_equal(a, b) for a, b in zip(mine, want))
        segs.append(np.concatenate(mine))
    hA = [int(H[r0[j]]) for j in range(cnt)]
    sums = []
    for j in range(cnt):
        A0 = S[j] & ~15
        blk = segs[j]
        below = lambda off: int(np.concatenate([blk[:off], np.zeros(off & 1, np.uint8)])
                                .view("<u2").astype(np.uint64).sum())
        h_s = hA[j] + below(l4s[j] - A0)
        if l4e[j] == X1:
            h_e = hx
        elif l4e[j] == E[j]:
            nb = segs[j + 1][:16]
            h_e = hA[j + 1] + _below(nb, E[j] & 15)
        elif l4e[j] - A0 < ((S[j] + 128) & ~31) - A0:     # e_off < hb_end
            h_e = hA[j] + below(l4e[j] - A0)
        else:
            sums.append(None)
            continue
        sums.append((h_e - h_s) & M32)
    return sums, blocks_ok


@pytest.mark.parametrize("case", ["mixed", "short", "padded", "mtu", "aligned_end", "tiny"])
def test_captured_frame_model_exact(case):
    rng = np.random.default_rng(hash(("capture", case)) % 2**32)
    for trial in range(40):
        cnt = int(rng.integers(1, 65))
        lo, hi = {"mixed": (34, 1515), "short": (34, 100), "padded": (60, 300),
                  "mtu": (1514, 1515), "aligned_end": (34, 200), "tiny": (0, 40)}[case]
        lens = rng.integers(lo, hi, cnt)
        base = 4096 + int(rng.integers(0, 64))
        S = [base + int(x) for x in np.concatenate([[0], np.cumsum(lens)[:-1]])]
        E = [s + int(n) for s, n in zip(S, lens)]
        if case == "aligned_end":
            shift = (16 - E[-1] % 16) % 16
            S = [s + shift for s in S]
            E = [e + shift for e in E]
        buf = rng.integers(0, 256, size=E[-1] + 4096, dtype=np.uint8)
        buf[S[0]:S[0] + 300] = 0xFF
        l4s, l4e = [], []
        for s, e in zip(S, E):
            hl = 4 * int(rng.integers(5, 16))
            start = min(s + 14 + hl, e)
            room = e - start
            ln = int(rng.integers(0, room + 1)) if case == "padded" and room else room
            l4s.append(start)
            l4e.append(start + ln)
        sums, ok = captured_frame_model(buf, S, E, l4s, l4e)
        assert ok, (case, trial)
        for j in range(cnt):
            if sums[j] is not None:
                assert sums[j] == _exact_halves(buf, l4s[j], l4e[j]) & M32, (case, trial, j)


def _exact_halves(buf, s, e):
    """Exact sum of little-endian 16-bit halves at even absolute addresses over [s, e)."""
    lo, hi = s & ~1, (e + 1) & ~1
    raw = np.zeros(hi - lo, dtype=np.uint8)
    raw[s - lo:e - lo] = buf[s:e]
    return int(raw.view("<u2").astype(np.uint64).sum())


# ---- column runs (round 5, sum_column_chunk) -------------------------------------------

def _below_uniform(raw_seg, o):
    """halves_below_uniform: the prefix of the dwords below o >> 2 (the window's own sum in
    dword order), plus dword o >> 2 masked to its o & 3 low bytes."""
    d = raw_seg.view("<u4").astype(np.uint64)
    q, m = o >> 2, (1 << (8 * (o & 3))) - 1
    acc = 0
    for k in range(q):
        acc += (int(d[k]) & 0xFFFF) + (int(d[k]) >> 16)
    x = int(d[q]) & m
    return acc + (x & 0xFFFF) + (x >> 16)


def column_chunk_model(buf, S, E, cnt, cpk, edge_loads=False):
    """sum_column_chunk, step for step: each lane's column sum C_L over the windows consumed,
    the boundary rows written when boundary j's window is consumed (the rest after the last
    window), then packet j = sum_L (X_{j+1,L} - X_{j,L}), all mod 2^32; the reduction as the
    kernel does it (64 / cpk lanes per packet, cpk columns each). edge_loads (the kernel's
    arithmetic in both its forms): X_{j,L} = C_L + (L < B_j ? s_L : 0), and P_j, the bytes of
    boundary j's segment below o_j, added as + P_{j+1} - P_j -- that segment from a separate
    default-policy load (the default) or captured from the stream into LDS (CAPTURE, the
    JUST_WRITTEN hint): the same bytes. Without edge_loads: the window-prefix variant measured
    in round 6 and not kept, X_{j,L} = C_L + (L < B_j ? s_L : L == B_j ? the bytes of the
    segment below o_j : 0) (halves_below_uniform)."""
    X1 = int(E[cnt - 1])
    b = [int(S[j]) if j < cnt else X1 for j in range(64)]
    A = b[0] & ~15
    nseg = (X1 - A + 15) >> 4
    nwin = (nseg + 63) >> 6
    seg, raw = _halves_of_segments(buf, A, max(nwin * 64, 1), nseg * 16)
    g = [(x - A) >> 4 for x in b]
    o = [(x - A) & 15 for x in b]
    rows = np.zeros((cnt + 1, 64), dtype=np.uint64)
    C = np.zeros(64, dtype=np.uint64)
    lanes = np.arange(64)
    jb = 0
    for w in range(nwin):
        s = seg[w * 64:(w + 1) * 64].astype(np.uint64)
        while jb <= cnt and (g[jb] >> 6) == w:
            B = g[jb] & 63
            x = np.where(lanes < B, s, 0)
            if not edge_loads:  # lane B: its own segment's bytes below o_j (0 past the run)
                x[B] = _below_uniform(raw[g[jb] * 16:g[jb] * 16 + 16], o[jb])
            rows[jb] = (C + x) & M32
            jb += 1
        C = (C + s) & M32
    while jb <= cnt:  # boundaries past the last window: X1 on a segment edge, o = 0
        assert o[jb] == 0
        rows[jb] = C
        jb += 1
    P = [(_below(raw[g[j] * 16:g[j] * 16 + 16], o[j]) if (edge_loads and j <= cnt and o[j])
          else 0) for j in range(64)]
    q = 64 // cpk
    sums = []
    for j in range(cnt):
        acc = 0
        for part in range(q):  # 64 / cpk lanes, cpk columns each, then the butterfly
            cols = range(part * cpk, (part + 1) * cpk)
            acc += sum(int(rows[j + 1][c]) - int(rows[j][c]) for c in cols)
        sums.append((acc + P[j + 1] - P[j]) & M32)
    return sums + [0] * (64 - cnt)


@pytest.mark.parametrize("edge_loads", [False, True])
@pytest.mark.parametrize("cpk", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("case", ["tiny", "mixed", "mtu", "jumbo", "aligned_end"])
def test_column_model_matches_oracle(oracle, case, cpk, edge_loads):
    rng = np.random.default_rng(hash((case, cpk, "col")) % 2**32)
    base = int(rng.integers(0, 16))
    if case == "tiny":
        off = _layout(rng, 100, [0, 0, 1, 2, 3, 5, 7, 16, 17, 31], base)
    elif case == "mixed":
        off = _layout(rng, 100, list(range(64, 1501, 97)) + [65, 1499], base)
    elif case == "mtu":
        off = _layout(rng, 64, [1500], base)
    elif case == "jumbo":
        off = _layout(rng, 20, [9000, 65535, 0, 1], base)
    else:                       # the run ending exactly on a window edge (X1 past the loop)
        lens = np.array([1024] * 16, dtype=np.int64)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    buf = rng.integers(0, 256, size=int(off[-1]) + 64, dtype=np.uint8)
    for j in range(0, off.size - 1, 7):
        buf[off[j]:off[j + 1]] = 0 if j % 2 else 0xFF
    n = off.size - 1
    got = np.zeros(n, dtype=np.uint16)
    for p0 in range(0, n, cpk):
        cnt = min(cpk, n - p0)
        S = [int(off[p0 + j]) for j in range(cnt)]
        E = [int(off[p0 + j + 1]) for j in range(cnt)]
        got[p0:p0 + cnt] = finish(column_chunk_model(buf, S, E, cnt, cpk, edge_loads)[:cnt], S)
    want = oracle.batch_csr(buf, off)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


# ---- chain column runs (round 6, chksum_chain_kernel COLS: the JUST_WRITTEN chains) -----

def chain_cols_model(buf, a, l, short_first=128, maxp=32):
    """One 64-chunk slice of the chain kernel's column-run form: the lone short chunks (at most
    short_first bytes, sharing no 128-byte line with their table neighbours -- lanes wrap as
    ds_bpermute does), the run chunks (every other non-empty one) in lanes 0.. in table order,
    the rest (empty) last; the run chunks must lie back to back (stream_ok), else None (the
    slice takes the gathered stream). Runs of at most maxp chunks by column_chunk_model (the
    kernel's edge-load arithmetic), the short chunks summed whole. Returns each chunk's
    halves-sum (mod 2^32) in table order."""
    k = len(a)
    a = [int(x) for x in a] + [0] * (64 - k)
    l = [int(x) for x in l] + [0] * (64 - k)
    M64 = (1 << 64) - 1
    line_s = [(x >> 7) & M32 for x in a]
    line_e = [(((a[j] + l[j] - 1) & M64) >> 7) & M32 for j in range(64)]
    sc = [l[j] != 0 and l[j] <= short_first and line_e[(j - 1) % 64] != line_s[j]
          and line_s[(j + 1) % 64] != line_e[j] for j in range(64)]
    run = [j for j in range(64) if l[j] and not sc[j]]
    for r in range(len(run)):
        j = run[r]
        if l[j] > (1 << 17) - 1:
            return None
        if r + 1 < len(run) and a[j] + l[j] != a[run[r + 1]]:
            return None
    out = [0] * 64
    for r0 in range(0, len(run), maxp):
        part = run[r0:r0 + maxp]
        S = [a[j] for j in part]
        E = [a[j] + l[j] for j in part]
        sums = column_chunk_model(buf, S, E, len(part), maxp, edge_loads=True)
        for i, j in enumerate(part):
            out[j] = sums[i]
    for j in range(64):
        if sc[j]:
            out[j] = _exact_halves(buf, a[j], a[j] + l[j]) & M32
    return out[:k]


def _tx_slice(rng, case):
    """One 64-chunk slice of a TCP-Tx chain table (header node, payload pieces back to back)."""
    a, l = [], []
    pay = 300000 + int(rng.integers(0, 16))
    i = 0
    while len(a) < 64:
        if case not in ("no_headers", "max_pieces"):
            a.append(100 + (20 if case == "adjacent_headers" else 32) * i)
            l.append(20)
        pieces = ([int(rng.integers(1, 3000))] if case == "no_headers" else
                  [int(rng.integers(1, 129)), int(rng.integers(1, 1460))] if case == "tx_short_pieces"
                  else [int(rng.integers(1, 1460)), int(rng.integers(1, 1460))])
        for ln in pieces:
            a.append(pay)
            l.append(ln)
            pay += ln
        i += 1
    a, l = a[:64], l[:64]
    if case == "max_pieces":  # 64 pieces of 30000 bytes: two runs of 32
        for j in range(64):
            a[j], l[j] = 10 + 30000 * j, 30000
    return a, l


@pytest.mark.parametrize("case", ["tx", "tx_short_pieces", "no_headers", "max_pieces",
                                  "adjacent_headers", "displaced"])
def test_chain_cols_model_matches_oracle(oracle, case):
    """The JUST_WRITTEN chain kernel's column-run form (chksum_kernels.hip, COLS) on TCP-Tx
    layouts, 12 seeded slices per case: each chunk's sum folded and oriented as the kernel
    does, against the oracle. A short first piece that ends on a 128-byte line edge shares no
    line with its table neighbours, so it counts as a lone short chunk and its slice takes the
    gathered stream (None) -- rare, and exact either way; most slices must take the runs."""
    column_path = 0
    for seed in range(12):
        rng = np.random.default_rng(zlib.crc32(f"cc-{case}-{seed}".encode()))
        buf = rng.integers(0, 256, size=(1 << 21) + 4096, dtype=np.uint8)
        buf[600000:620000] = 0xFF
        a, l = _tx_slice(rng, case)
        if case == "displaced":
            a[40] += 1  # a run chunk moved: not back to back any more
            assert chain_cols_model(buf, a, l) is None
            continue
        sums = chain_cols_model(buf, a, l)
        if sums is None:
            continue
        column_path += 1
        for j in range(64):
            r = finish([sums[j]], [a[j]])[0]
            assert r == oracle.inverted(buf, a[j], l[j]), (case, seed, j, a[j], l[j])
    assert case == "displaced" or column_path >= 9, (case, column_path)


# ---- slot windows (round 5, sum_slot_windows) ------------------------------------------

def slot_windows_model(buf, S, E, cnt):
    """sum_slot_windows: each packet's whole segments from A0 = S & ~15 (a descriptor of
    exactly nseg segments: lanes past it read 0), lane partials per slot added in groups of 8
    slots, minus the foreign bytes of the packet's first and last segment."""
    out = []
    for j in range(cnt):
        s, e = int(S[j]), int(E[j])
        ln = e - s
        if ln == 0:
            out.append(0)
            continue
        a0 = s & ~15
        rs = s & 15
        nseg = (rs + ln + 15) >> 4
        te = ((rs + ln - 1) & 15) + 1
        seg, raw = _halves_of_segments(buf, a0, max(((nseg + 63) >> 6) * 64, 1), nseg * 16)
        lanes = [int(seg[L::64].sum()) for L in range(64)]  # each lane's windows
        whole = sum(lanes) & M32
        first = raw[:16]
        last = raw[(nseg - 1) * 16:nseg * 16]
        foreign = _below(first, rs) + (int(last.view("<u2").astype(np.uint64).sum())
                                       - _below(last, te))
        out.append((whole - foreign) & M32)
    return out


@pytest.mark.parametrize("stride", [64, 1517, 2048, 9216])
def test_slot_windows_model_matches_oracle(oracle, stride):
    rng = np.random.default_rng(stride)
    n = 300
    cap = min(stride, 65535)
    lens = rng.integers(0, cap + 1, n).astype(np.uint32)
    lens[:6] = [0, 1, 15, 16, 17, cap]
    base = 5
    ring = rng.integers(0, 256, size=n * stride + base + 32, dtype=np.uint8)
    ring[base:base + stride] = 0xFF
    S = [base + i * stride for i in range(n)]
    E = [S[i] + int(lens[i]) for i in range(n)]
    got = finish(slot_windows_model(ring, S, E, n), S)
    want = oracle.batch_slotted(np.ascontiguousarray(ring[base:base + n * stride]), stride, lens)
    assert np.array_equal(np.array(got, dtype=np.uint16), want)


# ---- gapped column runs (round 5, sum_gapped_column_chunk) ------------------------------

def gapped_column_chunk_model(buf, s0, stride, ln, cnt, cpk):
    """sum_gapped_column_chunk, step for step: compact segment c of the chunk is loaded from
    B0 + k * gap + 16 c with k = mulhi(c, ceil(2^32 / ns)) (checked against c // ns), the
    columns and boundary rows as in column runs with boundaries at j * ns (no partial
    segment), then each packet's foreign edge bytes subtracted."""
    rs = s0 & 15
    B0 = s0 & ~15
    ns = (rs + ln + 15) >> 4
    magic = ((1 << 32) + ns - 1) // ns
    gap = stride - 16 * ns
    T = cnt * ns
    nwin = (T + 63) >> 6
    span = (cnt - 1) * stride + 16 * ns
    C = np.zeros(64, dtype=np.uint64)
    rows = np.zeros((cnt + 1, 64), dtype=np.uint64)
    jb = 0
    for w in range(nwin):
        s = np.zeros(64, dtype=np.uint64)
        for lane in range(64):
            c = min(w * 64 + lane, T - 1)
            k = (c * magic) >> 32
            assert k == c // ns
            off = k * gap + 16 * c
            assert 0 <= off and off + 16 <= span
            if w * 64 + lane < T:
                raw = np.array(buf[B0 + off:B0 + off + 16], dtype=np.uint8)
                s[lane] = int(raw.view("<u2").astype(np.uint64).sum())
        while jb <= cnt and ((jb * ns) >> 6) == w:
            B = (jb * ns) & 63
            rows[jb] = (C + np.where(np.arange(64) < B, s, 0)) & M32
            jb += 1
        C = (C + s) & M32
    while jb <= cnt:
        rows[jb] = C
        jb += 1
    te = ((rs + ln - 1) & 15) + 1
    out = []
    q = 64 // cpk
    for j in range(cnt):
        acc = 0
        for part in range(q):
            cols = range(part * cpk, (part + 1) * cpk)
            acc += sum(int(rows[j + 1][c]) - int(rows[j][c]) for c in cols)
        a0 = B0 + j * stride
        first = np.array(buf[a0:a0 + 16], dtype=np.uint8)
        last = np.array(buf[a0 + 16 * (ns - 1):a0 + 16 * ns], dtype=np.uint8)
        foreign = _below(first, rs) + (int(last.view("<u2").astype(np.uint64).sum())
                                       - _below(last, te))
        out.append((acc - foreign) & M32)
    return out


@pytest.mark.parametrize("stride,ln", [(2048, 1500), (1504, 1500), (16, 40), (0, 100),
                                       (48, 1), (2048, 2048 - 16), (9216, 9000), (64, 16)])
def test_gapped_column_model_matches_oracle(oracle, stride, ln):
    """Strides a multiple of 16, packets at any start offset within a segment: gaps, packets
    sharing their edge segments (1504 / 1500 at an odd offset), overlapping and zero strides."""
    rng = np.random.default_rng(stride * 7 + ln)
    n = 40
    for base in (0, 3, 12, 15):
        cp = 1
        while cp < 16 and 2 * cp * ln <= 12288:
            cp *= 2
        ring = rng.integers(0, 256, size=n * max(stride, 16) + ln + base + 64, dtype=np.uint8)
        ring[base:base + ln] = 0xFF
        got = np.zeros(n, dtype=np.uint16)
        for p0 in range(0, n, cp):
            cnt = min(cp, n - p0)
            s0 = base + p0 * stride
            S = [s0 + j * stride for j in range(cnt)]
            got[p0:p0 + cnt] = finish(gapped_column_chunk_model(ring, s0, stride, ln, cnt, cp), S)
        want = oracle.batch_strided(ring, stride, ln, n, base_off=base)
        assert np.array_equal(got, want), (base, np.nonzero(got != want)[0][:8])


# ---- segment-table runs (round 5, sum_segtab_chunk) ------------------------------------

def segtab_chunk_model(buf, S, E, cnt, cpk):
    """sum_segtab_chunk: the run's per-segment halves-sums in a table, packet j = its whole
    segments [g_j, g_{j+1}) added in 64 / cpk contiguous shares, + P_{j+1} - P_j, mod 2^32."""
    X1 = int(E[cnt - 1])
    b = [int(S[j]) if j < cnt else X1 for j in range(64)]
    A = b[0] & ~15
    nseg = (X1 - A + 15) >> 4
    nwin = (nseg + 63) >> 6
    seg, raw = _halves_of_segments(buf, A, max(nwin * 64, 1), nseg * 16)
    g = [(x - A) >> 4 for x in b]
    o = [(x - A) & 15 for x in b]
    P = [(_below(raw[g[j] * 16:g[j] * 16 + 16], o[j]) if (j <= cnt and o[j]) else 0)
         for j in range(64)]
    q = 64 // cpk
    sums = []
    for j in range(cnt):
        lo, hi = g[j], g[j + 1]
        per = (hi - lo + q - 1) // q
        acc = 0
        for part in range(q):
            a = lo + part * per
            acc += int(seg[a:min(a + per, hi)].sum()) if a < hi else 0
        sums.append((acc + P[j + 1] - P[j]) & M32)
    return sums + [0] * (64 - cnt)


@pytest.mark.parametrize("cpk", [1, 4, 16, 32])
@pytest.mark.parametrize("case", ["tiny", "mixed", "mtu", "aligned_end"])
def test_segtab_model_matches_oracle(oracle, case, cpk):
    rng = np.random.default_rng(hash((case, cpk, "segtab")) % 2**32)
    base = int(rng.integers(0, 16))
    if case == "tiny":
        off = _layout(rng, 200, [0, 0, 1, 2, 3, 5, 7, 16, 17, 31], base)
    elif case == "mixed":
        off = _layout(rng, 100, list(range(64, 1501, 97)) + [65, 1499], base)
    elif case == "mtu":
        off = _layout(rng, 64, [1500], base)
    else:
        lens = np.array([1024] * 16, dtype=np.int64)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    buf = rng.integers(0, 256, size=int(off[-1]) + 64, dtype=np.uint8)
    for j in range(0, off.size - 1, 7):
        buf[off[j]:off[j + 1]] = 0 if j % 2 else 0xFF
    n = off.size - 1
    got = np.zeros(n, dtype=np.uint16)
    for p0 in range(0, n, cpk):
        cnt = min(cpk, n - p0)
        S = [int(off[p0 + j]) for j in range(cnt)]
        E = [int(off[p0 + j + 1]) for j in range(cnt)]
        got[p0:p0 + cnt] = finish(segtab_chunk_model(buf, S, E, cnt, cpk)[:cnt], S)
    want = oracle.batch_csr(buf, off)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
