"""CPU model of the kernels' stream mode (chksum_device.h: stream_ok / sum_stream_chunk),
step for step, checked bit-exact against the oracle before any GPU runs it.

Stream mode reads a 64-packet chunk whose packets lie back to back as one contiguous run of
16-byte segments, 64 per window (one wave instruction), and gets each packet's exact sum of
little-endian 16-bit halves as a difference of prefixes H(S_{j+1}) - H(S_j) kept mod 2^32.
This model reproduces the windows, the lane scan, the per-boundary partial segment, the
bytes past the chunk end in its last segment, the mod-2^32 arithmetic and the finish
(fold, byte swap iff S even), so a wrong index or mask shows up here on the CPU.
"""
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
