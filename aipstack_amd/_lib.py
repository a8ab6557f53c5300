"""Loader for the in-tree product library ``aipstack_amd/lib/libaipstack_chksum.so``.

The library is the C-ABI of ``include/aipstack_amd/chksum.h`` (+ ``synth.h``). There is
no pure-Python or CPU fallback for the batch entry points: if the library is missing
this module raises ``ImportError`` loudly (build it with ``make -C aipstack_amd/csrc`` or
``python -c "import __graft_entry__ as g; g.build()"``).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# AIPSTACK_AMD_LIB: load another build instead (A/B experiments, tools/sweep.py --lib).
LIB_PATH = os.environ.get("AIPSTACK_AMD_LIB") or os.path.join(_HERE, "lib", "libaipstack_chksum.so")

# Every symbol include/aipstack_amd/*.h declares, with its ctypes signature.
_c_u16 = ctypes.c_uint16
_c_u32 = ctypes.c_uint32
_c_u64 = ctypes.c_uint64
_c_int = ctypes.c_int
_c_vp = ctypes.c_void_p
_c_size = ctypes.c_size_t

SIGNATURES = {
    # chksum.h
    "IpChksumInverted": (_c_u16, [_c_vp, _c_size]),
    "aipstack_chksum_batch_strided": (_c_int, [_c_vp, _c_u64, _c_u32, _c_u64, _c_vp, _c_u32, _c_vp]),
    "aipstack_chksum_batch_csr": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u32, _c_vp]),
    "aipstack_chksum_batch_seeded_csr": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_batch_chain": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_u32, _c_vp]),
    "aipstack_chksum_batch_chain_fill": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_u64, _c_vp,
                                                  _c_u32, _c_vp]),
    "aipstack_chksum_rx_verify": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_tx_fill": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_tx_fill_workspace_bytes": (_c_u64, [_c_u64]),
    "aipstack_chksum_tx_fill_split": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_vp, _c_u64, _c_vp]),
    "aipstack_chksum_strerror": (ctypes.c_char_p, [_c_int]),
    "aipstack_chksum_last_hip_error": (_c_int, []),
    "aipstack_chksum_device_check": (_c_int, [_c_int]),
    "aipstack_chksum_abi_version": (_c_int, []),
    "aipstack_chksum_tune": (_c_int, [ctypes.c_char_p, _c_int]),
    "aipstack_chksum_launch_shape": (_c_int, [_c_u64, _c_int, _c_int, _c_vp, _c_vp]),
    "aipstack_chksum_contract_violations": (_c_int, [_c_int, ctypes.POINTER(_c_u32), _c_int]),
    "aipstack_chksum_engine_create": (_c_int, [_c_int, _c_u64, _c_int, ctypes.POINTER(_c_vp)]),
    "aipstack_chksum_engine_destroy": (None, [_c_vp]),
    "aipstack_chksum_engine_register": (_c_int, [_c_vp, _c_vp, _c_u64]),
    "aipstack_chksum_engine_unregister": (_c_int, [_c_vp, _c_vp]),
    "aipstack_chksum_engine_host_strided": (_c_int, [_c_vp, _c_vp, _c_u64, _c_u32, _c_u64, _c_vp, _c_u32]),
    "aipstack_chksum_engine_host_csr": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_u32]),
    "aipstack_chksum_engine_host_rx_verify": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp]),
    "aipstack_chksum_engine_host_tx_fill": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp]),
    "aipstack_chksum_engine_submit_tx_fill": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_tx_fill_records": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_batch_slotted": (_c_int, [_c_vp, _c_u64, _c_vp, _c_u64, _c_vp, _c_u32, _c_vp]),
    "aipstack_chksum_rx_verify_slotted": (_c_int, [_c_vp, _c_u64, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_tx_fill_slotted": (_c_int, [_c_vp, _c_u64, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_tx_fill_slotted_split": (_c_int, [_c_vp, _c_u64, _c_vp, _c_u64, _c_vp, _c_vp,
                                                       _c_u64, _c_vp]),
    "aipstack_chksum_tx_fill_records_slotted": (_c_int, [_c_vp, _c_u64, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_submit_rx_verify": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_submit_strided": (_c_int, [_c_vp, _c_vp, _c_u64, _c_u32, _c_u64, _c_vp,
                                                       _c_u32, ctypes.POINTER(_c_u64)]),
    "aipstack_chksum_engine_submit_csr": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_u32,
                                                   ctypes.POINTER(_c_u64)]),
    "aipstack_chksum_engine_host_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64, _c_vp, _c_u32]),
    "aipstack_chksum_engine_submit_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64, _c_vp, _c_u32,
                                                       ctypes.POINTER(_c_u64)]),
    "aipstack_chksum_engine_host_rx_verify_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64, _c_vp]),
    "aipstack_chksum_engine_submit_rx_verify_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64,
                                                                 _c_vp, ctypes.POINTER(_c_u64)]),
    "aipstack_chksum_engine_host_tx_fill_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64, _c_vp]),
    "aipstack_chksum_engine_submit_tx_fill_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64,
                                                               _c_vp, ctypes.POINTER(_c_u64)]),
    "aipstack_chksum_engine_poll": (_c_int, [_c_vp, _c_u64]),
    "aipstack_chksum_engine_wait": (_c_int, [_c_vp, _c_u64]),
    "aipstack_chksum_engine_group_create": (_c_int, [_c_vp, _c_int, _c_u64, _c_int, ctypes.POINTER(_c_vp)]),
    "aipstack_chksum_engine_group_destroy": (None, [_c_vp]),
    "aipstack_chksum_engine_group_size": (_c_int, [_c_vp]),
    "aipstack_chksum_engine_group_register": (_c_int, [_c_vp, _c_vp, _c_u64]),
    "aipstack_chksum_engine_group_unregister": (_c_int, [_c_vp, _c_vp]),
    "aipstack_chksum_engine_group_engine": (_c_vp, [_c_vp, _c_int]),
    "aipstack_chksum_engine_group_region_mapped": (_c_int, [_c_vp, _c_vp]),
    "aipstack_chksum_engine_group_submit_strided": (_c_int, [_c_vp, _c_vp, _c_u64, _c_u32, _c_u64, _c_vp,
                                                             _c_u32, _c_vp]),
    "aipstack_chksum_engine_group_submit_csr": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_u32, _c_vp]),
    "aipstack_chksum_engine_group_submit_rx_verify": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_group_submit_tx_fill": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_group_submit_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64, _c_vp,
                                                             _c_u32, _c_vp]),
    "aipstack_chksum_engine_group_submit_rx_verify_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp,
                                                                       _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_group_submit_tx_fill_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp,
                                                                     _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_group_poll": (_c_int, [_c_vp, _c_u64, _c_vp]),
    "aipstack_chksum_engine_group_wait": (_c_int, [_c_vp, _c_u64, _c_vp]),
    "aipstack_chksum_source_digest": (ctypes.c_char_p, []),
    "aipstack_chksum_engine_locality": (_c_int, [_c_vp, _c_vp, _c_vp]),
    "aipstack_chksum_engine_region_mapped": (_c_int, [_c_vp, _c_vp]),
    "aipstack_chksum_engine_group_host_strided": (_c_int, [_c_vp, _c_vp, _c_u64, _c_u32, _c_u64, _c_vp,
                                                           _c_u32, _c_vp]),
    "aipstack_chksum_engine_group_host_csr": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_u32, _c_vp]),
    "aipstack_chksum_engine_group_host_rx_verify": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_group_host_tx_fill": (_c_int, [_c_vp, _c_vp, _c_vp, _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_group_host_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp, _c_u64, _c_vp,
                                                           _c_u32, _c_vp]),
    "aipstack_chksum_engine_group_host_rx_verify_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp,
                                                                     _c_u64, _c_vp, _c_vp]),
    "aipstack_chksum_engine_group_host_tx_fill_slotted": (_c_int, [_c_vp, _c_vp, _c_u64, _c_vp,
                                                                   _c_u64, _c_vp, _c_vp]),
    # synth.h
    "aipstack_synth_fill_host": (None, [_c_vp, _c_u64, _c_u64, _c_u64]),
    "aipstack_synth_mixed_offsets_host": (_c_u64, [_c_vp, _c_u64, _c_u64]),
    "aipstack_synth_apply_classes_host": (None, [_c_vp, _c_vp, _c_u64, _c_u64, _c_u64]),
    "aipstack_synth_fill_device": (_c_int, [_c_vp, _c_u64, _c_u64, _c_u64, _c_vp]),
    "aipstack_synth_apply_classes_device": (_c_int, [_c_vp, _c_vp, _c_u64, _c_u64, _c_u64, _c_vp]),
    "aipstack_synth_frames_host": (_c_u64, [_c_vp, _c_vp, _c_u64, _c_u64, _c_u32]),
}

ABI_VERSION = 1

_lib = None


def load() -> ctypes.CDLL:
    """Load (once) and return the product library; raise ImportError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"aipstack_amd: native library not built: {LIB_PATH} is missing "
            "(run `make -C aipstack_amd/csrc`). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError = library/header mismatch: loud
        fn.restype = res
        fn.argtypes = args
    if lib.aipstack_chksum_abi_version() != ABI_VERSION:
        raise ImportError("aipstack_amd: library ABI version mismatch")
    _lib = lib
    return lib


def tree_source_digest(package_dir: str = _HERE) -> str:
    """The digest aipstack_chksum_source_digest() reports, recomputed from the source tree
    (the files and order of the Makefile's DIGEST_SRCS; `package_dir` = the aipstack_amd
    directory whose csrc/ and ../include/ are read): equal iff the loaded library was built
    from the sources beside it."""
    import glob
    import hashlib
    csrc = os.path.join(package_dir, "csrc")
    names = []
    for pat in ("*.hip", "*.cpp", "*.cc", "*.h"):
        names += [os.path.basename(p) for p in glob.glob(os.path.join(csrc, pat))]
    names += [os.path.relpath(p, csrc) for p in
              glob.glob(os.path.join(package_dir, "..", "include", "aipstack_amd", "*.h"))]
    names.append("Makefile")
    h = hashlib.sha256()
    for n in sorted(set(names)):
        with open(os.path.join(csrc, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()
