"""Deterministic synthetic packet batches (include/aipstack_amd/synth.h).

The same counter-based byte stream is produced three ways, which tests check agree:
numpy (here), the host C functions and the device kernels of libaipstack_chksum.so.
Bench / test plumbing only.
"""
from __future__ import annotations

import numpy as np

from . import _lib

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
CLASS_SALT = 0xC1A55EED
MIN_LEN, MAX_LEN = 64, 1500

# BASELINE.json configs (binary K/M)
SEED_DATA = 42
SEED_LENGTHS = 43


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def words(seed: int, k0: int, count: int) -> np.ndarray:
    """word(seed, k) for k in [k0, k0 + count) as uint64."""
    with np.errstate(over="ignore"):
        k = np.arange(k0, k0 + count, dtype=np.uint64)
        return _mix(np.uint64(seed) + (k + np.uint64(1)) * GOLDEN)


def random_bytes(seed: int, nbytes: int, byte_offset: int = 0) -> np.ndarray:
    """byte(seed, byte_offset + i) for i < nbytes (uint8)."""
    k0 = byte_offset >> 3
    k1 = (byte_offset + nbytes + 7) >> 3
    w = words(seed, k0, k1 - k0).view(np.uint8)  # little-endian host
    s = byte_offset - 8 * k0
    return w[s:s + nbytes].copy()


def mixed_lengths(n: int, len_seed: int = SEED_LENGTHS) -> np.ndarray:
    return (MIN_LEN + (words(len_seed, 0, n) % np.uint64(MAX_LEN - MIN_LEN + 1))).astype(np.int64)


def mixed_classes(n: int, len_seed: int = SEED_LENGTHS) -> np.ndarray:
    return (words(len_seed ^ CLASS_SALT, 0, n) % np.uint64(100)).astype(np.int64)


def mixed_offsets(n: int, len_seed: int = SEED_LENGTHS) -> np.ndarray:
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(mixed_lengths(n, len_seed), out=off[1:])
    return off


def apply_classes(buf: np.ndarray, offsets: np.ndarray, len_seed: int = SEED_LENGTHS,
                  first_packet: int = 0) -> None:
    """In place: class 0 -> 0xFF, 1 -> 0x00, 2 -> nonzero with word sum = 0 mod 0xFFFF.
    Local packet p (offsets are local) is global packet first_packet + p."""
    n = offsets.size - 1
    cls = mixed_classes(first_packet + n, len_seed)[first_packet:]
    for p in np.nonzero(cls <= 2)[0]:
        s, e = int(offsets[p]), int(offsets[p + 1])
        c = int(cls[p])
        if c == 1:
            buf[s:e] = 0x00
        else:
            buf[s:e] = 0xFF
            if c == 2 and (e - s) & 1:
                buf[s] = 0x00


def mixed_batch(n: int, data_seed: int = SEED_DATA, len_seed: int = SEED_LENGTHS):
    """(buf uint8, offsets int64) of BASELINE config C's construction, on the host."""
    off = mixed_offsets(n, len_seed)
    buf = random_bytes(data_seed, int(off[-1]))
    apply_classes(buf, off, len_seed)
    return buf, off


# ---- native (C / HIP) generators --------------------------------------------------------

def fill_host(buf: np.ndarray, seed: int, byte_offset: int = 0) -> None:
    _lib.load().aipstack_synth_fill_host(buf.ctypes.data, buf.nbytes, seed, byte_offset)


def fill_device(tensor, seed: int, byte_offset: int = 0, stream=None) -> None:
    import torch
    s = torch.cuda.current_stream() if stream is None else stream
    st = _lib.load().aipstack_synth_fill_device(tensor.data_ptr(), tensor.numel() * tensor.element_size(),
                                                seed, byte_offset, int(s.cuda_stream))
    if st != 0:
        raise RuntimeError(f"aipstack_synth_fill_device failed ({st})")


def apply_classes_host(buf: np.ndarray, offsets: np.ndarray, len_seed: int = SEED_LENGTHS,
                       first_packet: int = 0) -> None:
    o = np.ascontiguousarray(offsets, dtype=np.uint64)
    _lib.load().aipstack_synth_apply_classes_host(buf.ctypes.data, o.ctypes.data, o.size - 1,
                                                  len_seed, first_packet)


def apply_classes_device(tensor, d_offsets, len_seed: int = SEED_LENGTHS, first_packet: int = 0,
                         stream=None) -> None:
    import torch
    s = torch.cuda.current_stream() if stream is None else stream
    st = _lib.load().aipstack_synth_apply_classes_device(
        tensor.data_ptr(), d_offsets.data_ptr(), d_offsets.numel() - 1, len_seed, first_packet,
        int(s.cuda_stream))
    if st != 0:
        raise RuntimeError(f"aipstack_synth_apply_classes_device failed ({st})")


def frames_host(n: int, seed: int = SEED_DATA, max_payload: int = 1400):
    """(buf uint8, offsets int64) of n raw Ethernet frames with zero checksum fields
    (aipstack_synth_frames_host; see include/aipstack_amd/synth.h for the mix)."""
    lib = _lib.load()
    off = np.zeros(n + 1, dtype=np.uint64)
    total = lib.aipstack_synth_frames_host(None, off.ctypes.data, n, seed, max_payload)
    buf = np.empty(max(total, 1), dtype=np.uint8)
    lib.aipstack_synth_frames_host(buf.ctypes.data, off.ctypes.data, n, seed, max_payload)
    return buf[:total], off.astype(np.int64)


def to_slots(buf: np.ndarray, offsets: np.ndarray, slot_stride: int, slack_seed: int = 99):
    """Packets / frames buf[offsets[i]:offsets[i+1]] laid into a ring of fixed slots (one per
    slot at i * slot_stride, the rest of each slot filled with splitmix64 bytes of
    `slack_seed`, so that a kernel reading past a length would see garbage). Returns
    (ring uint8 of n * slot_stride bytes, lens uint32)."""
    o = np.asarray(offsets, dtype=np.int64)
    n = o.size - 1
    lens = np.diff(o).astype(np.int64)
    if n and int(lens.max()) > slot_stride:
        raise ValueError("a packet is longer than the slot")
    ring = np.empty(n * slot_stride, dtype=np.uint8)
    fill_host(ring, slack_seed)  # the same splitmix64 bytes as random_bytes, in C
    if n == 0:
        return ring, lens.astype(np.uint32)
    so = np.arange(n, dtype=np.int64) * slot_stride
    for d0, s0, s1 in zip(so.tolist(), o[:-1].tolist(), o[1:].tolist()):
        ring[d0:d0 + s1 - s0] = buf[s0:s1]
    return ring, lens.astype(np.uint32)
