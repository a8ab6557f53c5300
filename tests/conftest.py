import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _ensure_built():
    lib = os.path.join(ROOT, "aipstack_amd", "lib", "libaipstack_chksum.so")
    orc = os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "aipstack_amd", "csrc")], check=True)
    if not os.path.exists(orc):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)


_ensure_built()


class Oracle:
    """ctypes view of oracle/build/libchksum_oracle.so (the CPU checker)."""

    def __init__(self):
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        vp, u64, u32, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_size_t
        lib.oracle_chksum_inverted.restype = ctypes.c_uint16
        lib.oracle_chksum_inverted.argtypes = [vp, sz]
        lib.oracle_chksum.restype = ctypes.c_uint16
        lib.oracle_chksum.argtypes = [vp, sz]
        lib.oracle_chksum_chain.restype = ctypes.c_uint16
        lib.oracle_chksum_chain.argtypes = [u32, vp, vp, sz]
        lib.oracle_batch_strided.argtypes = [vp, u64, u32, u64, vp, u32]
        lib.oracle_batch_csr.argtypes = [vp, vp, u64, vp, u32]
        lib.oracle_batch_seeded_csr.argtypes = [vp, vp, vp, u64, vp]
        lib.oracle_rx_verify.restype = ctypes.c_int
        lib.oracle_rx_verify.argtypes = [vp, sz]
        lib.oracle_tx_fill.restype = ctypes.c_int
        lib.oracle_tx_fill.argtypes = [vp, sz]
        lib.oracle_rx_verify_batch.argtypes = [vp, vp, u64, vp]
        lib.oracle_tx_fill_batch.argtypes = [vp, vp, u64, vp]
        lib.oracle_batch_slotted.argtypes = [vp, u64, vp, u64, vp, u32]
        lib.oracle_rx_verify_slotted.argtypes = [vp, u64, vp, u64, vp]
        lib.oracle_tx_fill_slotted.argtypes = [vp, u64, vp, u64, vp]
        self.lib = lib

    def batch_slotted(self, buf, stride, lens, final=False):
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.empty(ln.size, dtype=np.uint16)
        self.lib.oracle_batch_slotted(buf.ctypes.data, stride, ln.ctypes.data, ln.size,
                                      out.ctypes.data, 1 if final else 0)
        return out

    def rx_verify_slotted(self, buf, stride, lens):
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.empty(ln.size, dtype=np.uint8)
        self.lib.oracle_rx_verify_slotted(buf.ctypes.data, stride, ln.ctypes.data, ln.size,
                                          out.ctypes.data)
        return out

    def tx_fill_slotted(self, buf, stride, lens):
        """In place on the numpy buffer; returns statuses."""
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.empty(ln.size, dtype=np.uint8)
        self.lib.oracle_tx_fill_slotted(buf.ctypes.data, stride, ln.ctypes.data, ln.size,
                                        out.ctypes.data)
        return out

    def rx_verify_batch(self, buf, offsets):
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        out = np.empty(o.size - 1, dtype=np.uint8)
        self.lib.oracle_rx_verify_batch(buf.ctypes.data, o.ctypes.data, o.size - 1, out.ctypes.data)
        return out

    def tx_fill_batch(self, buf, offsets):
        """In place on the numpy buffer; returns statuses."""
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        out = np.empty(o.size - 1, dtype=np.uint8)
        self.lib.oracle_tx_fill_batch(buf.ctypes.data, o.ctypes.data, o.size - 1, out.ctypes.data)
        return out

    def inverted(self, arr: np.ndarray, off: int, length: int) -> int:
        return int(self.lib.oracle_chksum_inverted(arr.ctypes.data + off, length))

    def final(self, arr: np.ndarray, off: int, length: int) -> int:
        return int(self.lib.oracle_chksum(arr.ctypes.data + off, length))

    def chain(self, state: int, arr: np.ndarray, chunks) -> int:
        """chunks: list of (offset into arr, length) taken as a chain from its start."""
        k = max(len(chunks), 1)
        ptrs = (ctypes.c_void_p * k)(*[arr.ctypes.data + o for o, _ in chunks])
        lens = (ctypes.c_size_t * k)(*[l for _, l in chunks])
        return int(self.lib.oracle_chksum_chain(state, ptrs, lens, len(chunks)))

    def batch_strided(self, arr, stride, length, n, final=False, base_off=0):
        out = np.empty(n, dtype=np.uint16)
        self.lib.oracle_batch_strided(arr.ctypes.data + base_off, stride, length, n,
                                      out.ctypes.data, 1 if final else 0)
        return out

    def batch_csr(self, arr, offsets, final=False):
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = o.size - 1
        out = np.empty(n, dtype=np.uint16)
        self.lib.oracle_batch_csr(arr.ctypes.data, o.ctypes.data, n, out.ctypes.data,
                                  1 if final else 0)
        return out

    def batch_seeded_csr(self, arr, offsets, states):
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        s = np.ascontiguousarray(states, dtype=np.uint32)
        n = o.size - 1
        out = np.empty(n, dtype=np.uint16)
        self.lib.oracle_batch_seeded_csr(arr.ctypes.data, o.ctypes.data, s.ctypes.data, n,
                                         out.ctypes.data)
        return out


def load_frame_ref_sets():
    """(frame_ref_cases.json, {set name: (buf, offsets)}, the frame_ref module): the frame
    batches the reference-composed fixtures cover, regenerated from their specs."""
    import frame_ref
    import make_golden
    with open(os.path.join(GOLDEN, "frame_ref_cases.json")) as f:
        doc = json.load(f)
    sets, _ = make_golden.frame_sets()
    mb, mo = sets["mix"]
    sets["mix_filled"] = (make_golden.fill_and_corrupt(mb, mo, doc["mix"], frame_ref), mo)
    return doc, sets, frame_ref


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


def chain_to_chunks(case):
    """Resolve a golden chain case (node list + IpBufRef offset/tot_len) into the list of
    (blob offset, length) chunks ipBufProcessBytes would visit (BufUtils.h:129-178)."""
    chunks = []
    remaining = case["tot_len"]
    offset = case["offset"]
    for i, (o, l) in enumerate(case["chunks"]):
        start = offset if i == 0 else 0
        take = min(l - start, remaining)
        if take > 0:
            chunks.append((o + start, take))
        remaining -= max(take, 0)
        if remaining <= 0:
            break
    return chunks


@pytest.fixture(scope="session")
def golden():
    from golden_data import blob
    with open(os.path.join(GOLDEN, "flat_cases.json")) as f:
        flat = json.load(f)
    with open(os.path.join(GOLDEN, "chain_cases.json")) as f:
        chain = json.load(f)
    with open(os.path.join(GOLDEN, "batch_cases.json")) as f:
        batch = json.load(f)
    return {"blob": blob(), "flat": flat, "chain": chain, "batch": batch}
