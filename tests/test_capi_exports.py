"""The C-ABI library loads and exports every symbol include/*.h declares; argument
validation and diagnostics work without a GPU (no compute calls here)."""
import ctypes
import os
import re
import subprocess

import aipstack_amd as A
from aipstack_amd import _lib
from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", "aipstack_amd", h) for h in ("chksum.h", "synth.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name not in ("if", "defined"):
                names.add(name)
    return names


def test_header_declarations_found():
    names = declared_functions()
    assert "IpChksumInverted" in names
    assert "aipstack_chksum_batch_strided" in names
    assert len(names) >= 12


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], check=True,
                         capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared_functions() - exported
    assert not missing, missing


def test_ctypes_signatures_cover_headers():
    assert declared_functions() == set(_lib.SIGNATURES)


def test_library_is_in_tree_and_gfx950():
    assert A.LIB_PATH.startswith(os.path.join(ROOT, "aipstack_amd", "lib"))
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list",
                          "--type=o", f"--input={A.LIB_PATH}"], capture_output=True, text=True)
    if out.returncode == 0 and out.stdout.strip():
        assert "gfx950" in out.stdout
    else:  # fall back to scanning the embedded code-object target string
        assert b"gfx950" in open(A.LIB_PATH, "rb").read()


def test_status_strings_and_abi():
    lib = _lib.load()
    assert lib.aipstack_chksum_abi_version() == 1
    for st, word in ((0, b"ok"), (-1, b"invalid"), (-2, b"HIP"), (-3, b"gfx950")):
        assert word in lib.aipstack_chksum_strerror(st)
    assert lib.aipstack_chksum_strerror(-99) == b"unknown status"


def test_argument_validation_without_gpu():
    lib = _lib.load()
    buf = ctypes.create_string_buffer(16)
    out = ctypes.create_string_buffer(16)
    p, o = ctypes.addressof(buf), ctypes.addressof(out)
    # n == 0 is a no-op and never touches the device
    assert lib.aipstack_chksum_batch_strided(p, 1, 1, 0, o, 0, None) == 0
    assert lib.aipstack_chksum_batch_csr(p, p, 0, o, 0, None) == 0
    assert lib.aipstack_chksum_batch_seeded_csr(p, p, p, 0, o, None) == 0
    # bad arguments are rejected before any HIP call
    assert lib.aipstack_chksum_batch_strided(None, 1, 1, 1, o, 0, None) == A.AIPSTACK_CHKSUM_EINVAL
    assert lib.aipstack_chksum_batch_strided(p, 1, 1, 1, None, 0, None) == A.AIPSTACK_CHKSUM_EINVAL
    assert lib.aipstack_chksum_batch_strided(p, 1, 65536, 1, o, 0, None) == A.AIPSTACK_CHKSUM_EINVAL
    assert lib.aipstack_chksum_batch_csr(p, None, 1, o, 0, None) == A.AIPSTACK_CHKSUM_EINVAL
    assert lib.aipstack_chksum_batch_seeded_csr(p, p, None, 1, o, None) == A.AIPSTACK_CHKSUM_EINVAL
    # split Tx fill: 8 workspace bytes per frame, 8-byte aligned, checked before any launch
    assert lib.aipstack_chksum_tx_fill_workspace_bytes(1000) == 8000
    assert lib.aipstack_chksum_tx_fill_split(p, p, 0, o, None, 0, None) == 0
    assert lib.aipstack_chksum_tx_fill_split(p, p, 2, o, o, 15, None) == A.AIPSTACK_CHKSUM_EINVAL
    assert lib.aipstack_chksum_tx_fill_split(p, p, 2, o, None, 16, None) == A.AIPSTACK_CHKSUM_EINVAL
    assert lib.aipstack_chksum_tx_fill_split(p, p, 1, o, o + 1, 15, None) == A.AIPSTACK_CHKSUM_EINVAL


def test_python_batch_api_requires_device_tensors():
    import pytest
    import torch
    with pytest.raises(ValueError):
        A.chksum_batch_strided(torch.zeros(16, dtype=torch.uint8), 16, 16, 1)


def test_launch_shape_small_and_large_batches():
    """aipstack_chksum_launch_shape (host-side, no GPU): a batch that fills at least 16 waves
    per CU at 64 packets per chunk keeps 64-packet chunks and the family's windows (2
    strided, 8 CSR); smaller batches shrink the chunk to ~8 waves per CU and stream 8
    windows."""
    lib = _lib.load()
    cp, w = ctypes.c_uint32(0), ctypes.c_int(0)

    def shape(n, csr=0, cus=256):
        assert lib.aipstack_chksum_launch_shape(n, cus, csr, ctypes.byref(cp), ctypes.byref(w)) == 0
        return cp.value, w.value

    assert shape(1 << 20) == (64, 2) and shape(1 << 20, csr=1) == (64, 8)
    assert shape(262144) == (64, 2)          # 4096 chunks of 64 = 16 waves per CU
    assert shape(4095 * 64) == (64, 8)       # one chunk fewer: small regime, 64-packet chunks
    assert shape(65536) == (32, 8)           # ~8 waves per CU
    assert shape(32768) == (16, 8)
    assert shape(4096) == (2, 8)
    assert shape(1) == (1, 8) and shape(0) == (1, 8)
    assert shape(65536, cus=32) == (64, 2)   # a smaller device fills sooner
    for n in (1, 100, 5000, 70000, 200000, 1 << 22):
        c, _ = shape(n)
        assert c in (1, 2, 4, 8, 16, 32, 64)
    assert lib.aipstack_chksum_launch_shape(1, 0, 0, ctypes.byref(cp), ctypes.byref(w)) == \
        A.AIPSTACK_CHKSUM_EINVAL
    assert lib.aipstack_chksum_launch_shape(1, 256, 0, None, ctypes.byref(w)) == \
        A.AIPSTACK_CHKSUM_EINVAL
    # the tunable overrides the chunk size (and is restored)
    assert lib.aipstack_chksum_tune(b"chunk_packets", 16) == 0
    try:
        assert shape(1 << 20)[0] == 16
    finally:
        assert lib.aipstack_chksum_tune(b"chunk_packets", 0) == 0


def test_library_matches_its_sources():
    """The library carries the digest of the sources it was built from
    (aipstack_chksum_source_digest); it must equal the digest of the sources in the tree, so
    a stale prebuilt .so fails here (and in the GPU suite's loaded-library test)."""
    lib = _lib.load()
    built = lib.aipstack_chksum_source_digest().decode()
    assert len(built) == 64
    assert built == _lib.tree_source_digest(), (
        "libaipstack_chksum.so was not built from the sources in the tree: "
        "make -C aipstack_amd/csrc")


def test_source_digest_detects_a_changed_source(tmp_path):
    """A one-byte change in any digested source changes the tree digest (what a stale
    library is caught by): a copy of the sources with one byte flipped."""
    import shutil
    pkg = tmp_path / "aipstack_amd"
    shutil.copytree(os.path.join(ROOT, "aipstack_amd", "csrc"), pkg / "csrc",
                    ignore=shutil.ignore_patterns("build"))
    shutil.copytree(os.path.join(ROOT, "include"), tmp_path / "include")
    assert _lib.tree_source_digest(str(pkg)) == _lib.tree_source_digest()
    f = pkg / "csrc" / "frame_kernels.hip"
    data = bytearray(f.read_bytes())
    data[100] ^= 1
    f.write_bytes(bytes(data))
    assert _lib.tree_source_digest(str(pkg)) != _lib.load().aipstack_chksum_source_digest().decode()
