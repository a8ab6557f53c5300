"""Host-side surface: the IpChksumInverted hook of libaipstack_chksum.so, the Python
mirror (aipstack_amd.chksum) and the C++ header mirror (include/aipstack_amd/Chksum.hpp),
each against the reference's golden vectors. Structured like the reference's own
tests/ip_chksum_test.cpp (known answer + chain-equals-flat property)."""
import ctypes
import itertools
import os
import subprocess

import numpy as np
import pytest

import aipstack_amd as A
from conftest import ROOT, chain_to_chunks


def test_hook_flat_cases(golden):
    b = golden["blob"]
    bad = [(o, l) for o, l, inv, fin in golden["flat"]["flat"]
           if A.IpChksumInverted(b[o:o + l]) != inv or A.IpChksum(b[o:o + l]) != fin]
    assert not bad, bad[:10]


def test_hook_edge_cases():
    assert A.IpChksumInverted(b"") == 0
    assert A.IpChksum(b"") == 0xFFFF
    assert A.IpChksumInverted(b"\xff\xff") == 0xFFFF
    assert A.IpChksumInverted(b"\x00" * 64) == 0
    assert A.IpChksumInverted(b"\x12") == 0x1200     # odd tail = high byte
    assert A.IpChksumInverted(b"\x12\x34") == 0x1234  # big-endian words
    with pytest.raises(ValueError):
        A.IpChksumInverted(bytes(65536))


def test_hook_unaligned_and_random(oracle):
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, size=80000, dtype=np.uint8)
    for _ in range(3000):
        o = int(rng.integers(0, 64))
        ln = int(rng.integers(0, 9001))
        assert A.IpChksumInverted(buf[o:o + ln]) == oracle.inverted(buf, o, ln)


def _python_chain(case, blob):
    nodes = None
    for o, l in reversed(case["chunks"]):
        nodes = A.IpBufNode(blob[o:o + l], l, nodes)
    acc = A.IpChksumAccumulator(case["state"])
    return acc.getChksum(A.IpBufRef(nodes, case["offset"], case["tot_len"]))


def test_reference_kat_python_mirror(golden):
    # tests/ip_chksum_test.cpp:45-62, on the Python mirror of IpBufNode/IpBufRef
    data = np.full(1023, 0xFF, dtype=np.uint8)
    nodes = None
    for i in reversed(range(512)):
        nodes = A.IpBufNode(data, 1 if i == 255 else 2, nodes)
    chain = A.IpChksum(A.IpBufRef(nodes, 0, 1023))
    assert chain == A.IpChksum(data) == 0x00FF


def test_chain_property_python_mirror():
    # tests/ip_chksum_test.cpp:64-106 (deterministic seed, fewer iterations)
    rng = np.random.default_rng(1)
    brk = [33, 34, 50, 51]
    for _ in range(200):
        buf = rng.integers(0, 256, size=101, dtype=np.uint8)
        good = A.IpChksum(buf)
        for k in (1, 2, 3):
            for cuts in itertools.combinations(brk, k):
                bounds = [0, *cuts, 101]
                nodes = None
                for i in reversed(range(len(bounds) - 1)):
                    s, e = bounds[i], bounds[i + 1]
                    nodes = A.IpBufNode(buf[s:e], e - s, nodes)
                assert A.IpChksum(A.IpBufRef(nodes, 0, 101)) == good


def test_chain_golden_python_mirror(golden):
    b = golden["blob"]
    cases = golden["chain"]["chains"]
    bad = [c for c in cases[::3] if _python_chain(c, b) != c["chksum"]]
    assert not bad, bad[:2]


def test_accumulate_golden_python_mirror(golden):
    b = golden["blob"]
    for c in golden["chain"]["accumulate"]:
        acc = A.IpChksumAccumulator()
        for w in c["w16"]:
            acc.addWord16(w)
        for w in c["w32"]:
            acc.addWord32(w)
        ho, hl = c["hdr"]
        acc.addEvenBytes(b[ho:ho + hl])
        assert acc.getState() == c["state"]
        resumed = A.IpChksumAccumulator(acc.getState())  # export / resume (Chksum.h:171-184)
        po, pl = c["payload"]
        node = A.IpBufNode(b[po:po + pl], pl)
        assert resumed.getChksum(A.IpBufRef(node, 0, pl)) == c["chksum"]


def test_add_even_bytes_rejects_odd():
    with pytest.raises(AssertionError):
        A.IpChksumAccumulator().addEvenBytes(b"abc")


def test_ipbuf_process_bytes_eager_walk():
    n3 = A.IpBufNode(b"", 0)
    n2 = A.IpBufNode(b"cd", 2, n3)
    n1 = A.IpBufNode(b"ab", 2, n2)
    seen = []
    rest = A.ipBufProcessBytes(A.IpBufRef(n1, 1, 3), 3,
                               lambda mv, n: seen.append(bytes(mv[:n])) or n)
    assert seen == [b"b", b"cd"]
    assert rest.tot_len == 0 and rest.node is n3   # moved on eagerly (BufUtils.h:165-170)


def _hpp():
    so = os.path.join(ROOT, "tests", "cpp", "build", "libhpp_shim.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp"), "all"], check=True)
    lib = ctypes.CDLL(so)
    lib.hpp_chksum_chain.restype = ctypes.c_uint16
    lib.hpp_chksum_chain.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
    lib.hpp_accumulate.restype = ctypes.c_uint16
    lib.hpp_accumulate.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    return lib


def test_cpp_header_chain_golden(golden):
    lib = _hpp()
    b = golden["blob"]
    for c in golden["chain"]["chains"]:
        k = max(len(c["chunks"]), 1)
        ptrs = (ctypes.c_void_p * k)(*[b.ctypes.data + o for o, _ in c["chunks"]])
        lens = (ctypes.c_size_t * k)(*[l for _, l in c["chunks"]])
        got = lib.hpp_chksum_chain(c["state"], ptrs, lens, len(c["chunks"]), c["offset"],
                                   c["tot_len"])
        assert got == c["chksum"], c


def test_cpp_header_accumulate_golden(golden):
    lib = _hpp()
    b = golden["blob"]
    for c in golden["chain"]["accumulate"]:
        w16 = np.array(c["w16"], dtype=np.uint16)
        w32 = np.array(c["w32"], dtype=np.uint32)
        st = ctypes.c_uint32(0)
        ho, hl = c["hdr"]
        po, pl = c["payload"]
        got = lib.hpp_accumulate(w16.ctypes.data, w16.size, w32.ctypes.data, w32.size,
                                 b.ctypes.data + ho, hl, b.ctypes.data + po, pl, ctypes.byref(st))
        assert st.value == c["state"] and got == c["chksum"], c


def test_chain_to_chunks_covers_tot_len(golden):
    for c in golden["chain"]["chains"]:
        assert sum(l for _, l in chain_to_chunks(c)) == c["tot_len"]


def test_host_hook_variants_match_oracle(oracle):
    """Portable / SSE2 / AVX2 / AVX-512 bodies of the hook (host_hook.cc) against the oracle
    (a body the CPU lacks falls back to the next one down)."""
    lib = A._lib.load()
    f = lib.aipstack_chksum_host_variant
    f.restype = ctypes.c_uint16
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    rng = np.random.default_rng(17)
    buf = rng.integers(0, 256, size=140000, dtype=np.uint8)
    buf[70000:] = 0xFF
    for t in range(4000):
        o = int(rng.integers(0, 70000 if t % 2 else 64))
        ln = min(int(rng.integers(0, 65536 if t % 50 == 0 else 3000)), 65535, buf.size - o)
        want = oracle.inverted(buf, o, ln)
        for v in (0, 1, 2, 3):
            assert f(v, buf.ctypes.data + o, ln) == want, (v, o, ln)


def test_engine_host_arrays_view_or_convert():
    """The engine wrappers hand offsets / lengths to the C-ABI as uint64 / uint32: contiguous
    int64 / int32 arrays as views (no per-call copy of a 1 M-entry array), the rest converted;
    the bit patterns are those of the conversion either way."""
    from aipstack_amd.chksum import _host_u32, _host_u64
    o = np.arange(0, 10 * 1500, 1500, dtype=np.int64)
    v = _host_u64(o)
    assert v.dtype == np.uint64 and np.shares_memory(v, o)
    assert np.array_equal(v, o.astype(np.uint64))
    neg = np.array([0, -1], dtype=np.int64)
    assert int(_host_u64(neg)[1]) == 2**64 - 1  # rejected by the engine's offset check
    for src in (o.astype(np.int32), o.astype(np.uint64), o[::2], list(o)):
        c = _host_u64(src)
        assert c.dtype == np.uint64 and c.flags.c_contiguous
        assert np.array_equal(c, np.asarray(src, dtype=np.int64).astype(np.uint64))
    ln = np.array([60, 1514, 0], dtype=np.int32)
    assert _host_u32(ln).dtype == np.uint32 and np.shares_memory(_host_u32(ln), ln)
    assert int(_host_u32(np.array([-1], dtype=np.int32))[0]) == 2**32 - 1
    assert np.array_equal(_host_u32([60, 1514]), np.array([60, 1514], dtype=np.uint32))
