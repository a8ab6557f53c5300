"""aipstack_amd -- MI355X-native Internet-checksum engine for aipstack's packet path.

The product is ``aipstack_amd/lib/libaipstack_chksum.so`` (host C++ + CDNA4 HIP
kernels) behind the C-ABI in ``include/aipstack_amd/chksum.h``; this package is its
Python host-side mirror (``chksum``) plus synthetic-batch plumbing (``synth``).
Importing it loads the native library and fails loudly if it was not built.
"""
from . import _lib

_lib.load()

from .chksum import (  # noqa: E402
    AIPSTACK_CHKSUM_EHIP,
    AIPSTACK_CHKSUM_EINVAL,
    AIPSTACK_CHKSUM_ENODEV,
    AIPSTACK_CHKSUM_FINAL,
    AIPSTACK_CHKSUM_JUST_WRITTEN,
    AIPSTACK_CHKSUM_MAX_LEN,
    AIPSTACK_CHKSUM_OK,
    ChksumEngine,
    ChksumEngineGroup,
    ChksumError,
    IpBufNode,
    IpBufRef,
    IpChksum,
    IpChksumAccumulator,
    IpChksumInverted,
    chksum_batch_chain,
    chksum_chain_fill,
    chksum_batch_csr,
    chksum_batch_seeded_csr,
    chksum_batch_slotted,
    chksum_batch_strided,
    contract_violations,
    device_check,
    VIOLATION_CHUNK_LEN,
    VIOLATION_PACKET_LEN,
    VIOLATION_SPAN,
    flatten_chains,
    ipBufProcessBytes,
    RX_VERDICTS,
    rx_verify,
    rx_verify_slotted,
    slots_to_offsets,
    tx_fill,
    tx_fill_records,
    tx_fill_records_slotted,
    tx_fill_slotted,
    apply_tx_records,
)

LIB_PATH = _lib.LIB_PATH

__all__ = [
    "AIPSTACK_CHKSUM_EHIP", "AIPSTACK_CHKSUM_EINVAL", "AIPSTACK_CHKSUM_ENODEV",
    "AIPSTACK_CHKSUM_FINAL", "AIPSTACK_CHKSUM_JUST_WRITTEN", "AIPSTACK_CHKSUM_MAX_LEN", "AIPSTACK_CHKSUM_OK", "ChksumEngine",
    "ChksumError",
    "IpBufNode", "IpBufRef", "IpChksum", "IpChksumAccumulator", "IpChksumInverted",
    "chksum_batch_chain", "chksum_chain_fill", "chksum_batch_csr", "chksum_batch_seeded_csr", "flatten_chains", "chksum_batch_strided", "device_check",
    "ipBufProcessBytes", "LIB_PATH", "RX_VERDICTS", "rx_verify", "tx_fill", "tx_fill_records",
    "apply_tx_records", "contract_violations", "VIOLATION_CHUNK_LEN", "VIOLATION_PACKET_LEN",
    "VIOLATION_SPAN", "chksum_batch_slotted", "rx_verify_slotted", "slots_to_offsets",
    "tx_fill_records_slotted", "tx_fill_slotted", "ChksumEngineGroup",
]
