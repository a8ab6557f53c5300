"""The C++ side of the boundary, on the CPU:

* the reference's OWN tests/ip_chksum_test.cpp, compiled in place with
  -DAIPSTACK_EXTERNAL_CHKSUM and linked to libaipstack_chksum.so (oracle/_ref/
  ip_chksum_test_external; only where the reference was present at build time);
* the repo's counterpart tests/cpp/ip_chksum_test.cpp on Chksum.hpp;
* the reference stack's checksum call sequences (tests/cpp/call_sites.inc: TCP/UDP Rx and
  Tx, IPv4 header Tx/Rx, ICMP) compiled against Chksum.hpp, checked against the answers
  the same text gives when compiled against the reference (tests/golden/
  call_site_cases.json), through ctypes and as a standalone program;
* the C-ABI's argument validation (tests/cpp/capi_validation_test.cpp);
* all of the above again under AddressSanitizer + UBSan (make -C tests/cpp asan; the
  reference's nix build uses both, default.nix:5-6).
"""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

import call_sites

CPP = os.path.join(ROOT, "tests", "cpp")
BUILD = os.path.join(CPP, "build")
REF_EXT = os.path.join(ROOT, "oracle", "_ref", "ip_chksum_test_external")
REF_HOOK_ONLY = os.path.join(ROOT, "oracle", "_ref", "ip_chksum_test_hook_only")
HOOK_SO = os.path.join(ROOT, "aipstack_amd", "lib", "libaipstack_chksum_hook.so")
HOOK_A = os.path.join(ROOT, "aipstack_amd", "lib", "libaipstack_chksum_hook.a")
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libref_chksum.so")
ASAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _built(*targets):
    """Bring the programs up to date (make is incremental) and return their paths."""
    subprocess.run(["make", "-j8", "-C", CPP, *[os.path.join("build", t) for t in targets]],
                   check=True, stdout=subprocess.DEVNULL)
    return [os.path.join(BUILD, t) for t in targets]


def _run(cmd, env=None, timeout=300):
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (cmd, r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


@pytest.fixture(scope="module")
def cases():
    with open(os.path.join(GOLDEN, "call_site_cases.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.skipif(not os.path.exists(REF_EXT),
                    reason="reference test not built here (no /root/reference at build time)")
def test_reference_ip_chksum_test_on_our_hook():
    """/root/reference/tests/ip_chksum_test.cpp, unmodified, linked to our IpChksumInverted
    (Chksum.h:50-51): the 0x00FF chain known answer + 10 M random chain-vs-flat splits."""
    _run([REF_EXT], timeout=600)


def test_hook_library_needs_no_rocm():
    """libaipstack_chksum_hook.{so,a}: IpChksumInverted alone (host_hook.cc), for a stack
    built with -DAIPSTACK_EXTERNAL_CHKSUM (Chksum.h:46-51) on a host without ROCm."""
    subprocess.run(["make", "-C", os.path.join(ROOT, "aipstack_amd", "csrc")], check=True,
                   stdout=subprocess.DEVNULL)
    deps = _run(["ldd", HOOK_SO])
    libs = [ln.split()[0] for ln in deps.splitlines() if ln.strip()]
    assert not [l for l in libs if "hip" in l or "hsa" in l or "amd" in l or "rocm" in l], deps
    assert all(l.startswith(("linux-vdso", "libc.so", "/lib64/ld-linux", "libstdc++", "libm.so",
                             "libgcc_s")) for l in libs), deps
    for lib in (HOOK_SO, HOOK_A):
        syms = _run(["nm", "-D" if lib.endswith(".so") else "-g", "--defined-only", lib])
        assert any(ln.split()[-1] == "IpChksumInverted" and " T " in ln
                   for ln in syms.splitlines() if ln.strip()), lib
    ctl = ctypes.CDLL(HOOK_SO)
    ctl.IpChksumInverted.restype = ctypes.c_uint16
    ctl.IpChksumInverted.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    assert ctl.IpChksumInverted(b"\xff\xff", 2) == 0xFFFF  # SURVEY 8(c) edge case


@pytest.mark.skipif(not os.path.exists(REF_HOOK_ONLY),
                    reason="reference test not built here (no /root/reference at build time)")
def test_reference_ip_chksum_test_on_rocm_free_hook():
    """The reference's own tests/ip_chksum_test.cpp linked to libaipstack_chksum_hook.so only
    (no HIP runtime in the process)."""
    deps = _run(["ldd", REF_HOOK_ONLY])
    assert "amdhip" not in deps and "hsa-runtime" not in deps, deps
    _run([REF_HOOK_ONLY], timeout=600)


def test_repo_ip_chksum_test():
    (exe,) = _built("ip_chksum_test")
    assert "OK" in _run([exe])


def test_call_sites_golden_ctypes(cases, golden):
    lib = ctypes.CDLL(_built("libhpp_shim.so")[0])
    blob = golden["blob"]
    bad = [c for c in cases if call_sites.evaluate(lib, "hpp", c, blob) != c["want"]]
    assert not bad, bad[:3]
    sites = {c["site"] for c in cases}
    assert sites == set(call_sites.SITES)


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="reference library not built here")
def test_call_sites_live_vs_reference(golden):
    """Fresh inputs (another seed) through both compilations of call_sites.inc."""
    ref = ctypes.CDLL(REF_LIB)
    hpp = ctypes.CDLL(_built("libhpp_shim.so")[0])
    blob = golden["blob"]
    for c in call_sites.make_cases(blob, seed=777):
        c.pop("expect", None)
        assert call_sites.evaluate(hpp, "hpp", c, blob) == call_sites.evaluate(ref, "ref", c, blob), c


def _walk(lib, prefix, blob, lens, offset, tot_len, process_len, budget):
    fn = getattr(lib, f"{prefix}_cs_walk")
    fn.restype = ctypes.c_size_t
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                   ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                   ctypes.c_size_t, ctypes.c_void_p]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]) if len(lens) else np.zeros(0, np.int64)
    k = max(len(lens), 1)
    ptrs = (ctypes.c_void_p * k)(*[blob.ctypes.data + int(o) for o in starts])
    ln = (ctypes.c_size_t * k)(*[int(l) for l in lens])
    pieces = np.zeros(2 * 64, dtype=np.uint64)
    out = np.zeros(3, dtype=np.uint64)
    cnt = fn(ptrs, ln, len(lens), offset, tot_len, process_len, budget, pieces.ctypes.data, 64,
             out.ctypes.data)
    rel = [(int(pieces[2 * i]) - blob.ctypes.data, int(pieces[2 * i + 1]))
           for i in range(min(cnt, 64))]
    return cnt, rel, [int(x) for x in out]


def _walk_py(blob, lens, offset, tot_len, process_len, budget):
    """The same walk through the Python mirror (aipstack_amd.ipBufProcessBytes)."""
    import aipstack_amd as A
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    nodes = [A.IpBufNode(blob[int(o):int(o) + int(l)], int(l)) for o, l in zip(starts, lens)]
    for a, b in zip(nodes, nodes[1:]):
        a.next = b
    offered, left = [], [budget]

    def visit(mv, n):
        addr = np.frombuffer(mv, dtype=np.uint8).ctypes.data
        offered.append((addr - blob.ctypes.data, n))
        took = min(n, left[0])
        left[0] -= took
        return took
    r = A.ipBufProcessBytes(A.IpBufRef(nodes[0], offset, tot_len), process_len, visit)
    return len(offered), offered[:64], [nodes.index(r.node), r.offset, r.tot_len]


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="reference library not built here")
def test_ip_buf_process_bytes_vs_reference(golden):
    """ipBufProcessBytes (BufUtils.h:129-178) itself, compiled from call_sites.inc against the
    reference and against Chksum.hpp: the pieces offered, the returned node / offset /
    tot_len, with visitors that stop early (budget), empty nodes (the eager advance steps
    over them), process_len below tot_len and offsets inside the first node."""
    ref = ctypes.CDLL(REF_LIB)
    hpp = ctypes.CDLL(_built("libhpp_shim.so")[0])
    blob = golden["blob"]
    rng = np.random.default_rng(2024)
    n_cases = 0
    for _ in range(3000):
        nn = int(rng.integers(1, 7))
        lens = [int(x) for x in rng.integers(0, 9, size=nn)]
        if rng.random() < 0.5:
            lens = [l * int(rng.integers(1, 40)) for l in lens]
        total = sum(lens)
        offset = int(rng.integers(0, lens[0] + 1))
        tot_len = int(rng.integers(0, total - offset + 1))
        process_len = int(rng.integers(0, tot_len + 1))
        budget = int(rng.integers(0, process_len + 2)) if rng.random() < 0.5 else 1 << 40
        args = (blob, lens, offset, tot_len, process_len, budget)
        want = _walk(ref, "ref", *args)
        assert _walk(hpp, "hpp", *args) == want, (lens, offset, tot_len, process_len, budget)
        assert _walk_py(*args) == want, ("python", lens, offset, tot_len, process_len, budget)
        n_cases += 1
    assert n_cases == 3000


def _write_case_files(tmp_path, cases, blob):
    blob_path = tmp_path / "blob.bin"
    blob.tofile(blob_path)
    lines = []
    for c in cases:
        want = c["want"] if isinstance(c["want"], list) else [c["want"]]
        ch = " ".join(f"{o} {l}" for o, l in c["chunks"])
        lines.append(" ".join(map(str, [c["site"], len(c["args"]), *c["args"],
                                        c["hdr"] or "-", len(c["chunks"])]))
                     + (" " + ch if ch else "")
                     + " " + " ".join(map(str, [c["offset"], c["tot_len"], len(want), *want])))
    case_path = tmp_path / "cases.txt"
    case_path.write_text("\n".join(lines) + "\n")
    return str(blob_path), str(case_path)


def test_call_sites_program(tmp_path, cases, golden):
    (exe,) = _built("call_sites_test")
    b, c = _write_case_files(tmp_path, cases, golden["blob"])
    assert f"{len(cases)} cases, 0 mismatches" in _run([exe, b, c])


def test_capi_validation():
    (exe,) = _built("capi_validation_test")
    assert "OK" in _run([exe])


def test_host_threads():
    """The engines' host-thread layer: sysfs CPU-list parsing and the persistent HostPool
    (every part once, concurrent callers, pools with 0-7 workers)."""
    (exe,) = _built("host_threads_test")
    assert "OK" in _run([exe])


@pytest.mark.parametrize("prog", ["ip_chksum_test", "call_sites_test", "capi_validation_test",
                                  "host_threads_test"])
def test_asan_ubsan(prog, tmp_path, cases, golden):
    (exe,) = _built(f"asan/{prog}")
    args = [exe]
    if prog == "call_sites_test":
        args += list(_write_case_files(tmp_path, cases, golden["blob"]))
    elif prog == "ip_chksum_test":
        args.append("300000")
    out = _run(args, env=ASAN_ENV, timeout=600)
    assert "OK" in out or "0 mismatches" in out


def test_add_even_bytes_asserts_an_even_count():
    """Chksum.hpp's addEvenBytes asserts an even count as the reference does (Chksum.h:227),
    under the reference's assertion configuration (AIPSTACK_CONFIG_ENABLE_ASSERTIONS)."""
    (exe,) = _built("assert_test")
    assert "sum" in _run([exe, "even"])
    r = subprocess.run([exe, "odd"], capture_output=True, text=True, timeout=60)
    assert r.returncode < 0 and "num_bytes % 2 == 0" in r.stderr, (r.returncode, r.stderr)
