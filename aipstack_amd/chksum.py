"""Host-side mirror of aipstack's checksum interface + the batched GPU entry points.

Reference interface mirrored (ambrop72/aipstack, ``src/aipstack/infra``):

=========================================  ================================================
reference (file:line)                      here
=========================================  ================================================
``IpChksumInverted`` Chksum.h:77-99        :func:`IpChksumInverted` (host C hook in the .so)
``IpChksum(ptr,len)`` Chksum.h:122-125     :func:`IpChksum` (bytes-like argument)
``IpChksum(IpBufRef)`` Chksum.h:332-336    :func:`IpChksum` (``IpBufRef`` argument)
``IpChksumAccumulator`` Chksum.h:148-316   :class:`IpChksumAccumulator`
``IpBufNode`` Buf.h:68-83                  :class:`IpBufNode`
``IpBufRef`` Buf.h:118-251                 :class:`IpBufRef`
``ipBufProcessBytes`` BufUtils.h:129-178   :func:`ipBufProcessBytes`
=========================================  ================================================

The per-packet functions run on the host (one packet is ~0.35 us of scalar work; a GPU
launch costs more). Batches go to the GPU through :func:`chksum_batch_strided`,
:func:`chksum_batch_csr` and :func:`chksum_batch_seeded_csr`, which call the C-ABI
(``include/aipstack_amd/chksum.h``) on device-resident torch tensors. torch is only the
device-memory / stream plumbing here; there is no CPU fallback for the batch calls.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional

import numpy as np

from . import _lib

AIPSTACK_CHKSUM_OK = 0
AIPSTACK_CHKSUM_EINVAL = -1
AIPSTACK_CHKSUM_EHIP = -2
AIPSTACK_CHKSUM_ENODEV = -3
AIPSTACK_CHKSUM_FINAL = 1
AIPSTACK_CHKSUM_ZERO_AS_FFFF = 2
AIPSTACK_CHKSUM_JUST_WRITTEN = 4  # hint: written by device stores since last read (chksum.h)
AIPSTACK_CHKSUM_MAX_LEN = 65535


class ChksumError(RuntimeError):
    """A batch entry point returned a negative status."""

    def __init__(self, status: int, where: str):
        lib = _lib.load()
        msg = lib.aipstack_chksum_strerror(status).decode()
        hip = lib.aipstack_chksum_last_hip_error()
        super().__init__(f"{where}: {msg} (status {status}, hip error {hip})")
        self.status = status
        self.hip_error = hip


def _check(status: int, where: str) -> None:
    if status != AIPSTACK_CHKSUM_OK:
        raise ChksumError(status, where)


# --------------------------------------------------------------------------------------
# Per-packet host functions
# --------------------------------------------------------------------------------------

def _as_pointer(data, length: Optional[int]):
    """(keepalive, address, length) of a bytes-like object's first `length` bytes."""
    arr = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) \
        else data.reshape(-1).view(np.uint8)
    n = arr.nbytes if length is None else int(length)
    if n < 0 or n > arr.nbytes:
        raise ValueError("length exceeds the buffer")
    if n == 0:  # the hook requires a non-null pointer even for len 0
        arr = np.zeros(1, dtype=np.uint8)
    return arr, arr.ctypes.data, n


def IpChksumInverted(data, length: Optional[int] = None) -> int:
    """Inverted IP checksum (ones'-complement sum of big-endian 16-bit words) of the first
    `length` bytes of `data` (default: all). Reference Chksum.h:77-99; len <= 65535."""
    keep, addr, n = _as_pointer(data, length)
    if n > AIPSTACK_CHKSUM_MAX_LEN:
        raise ValueError("IpChksumInverted: len must not exceed 65535 (Chksum.h:73-74)")
    r = _lib.load().IpChksumInverted(addr, n)
    del keep
    return int(r)


def IpChksum(data, length: Optional[int] = None) -> int:
    """IP checksum. With a bytes-like `data`: ``~IpChksumInverted`` (Chksum.h:122-125).
    With an :class:`IpBufRef`: the checksum of the referenced chain (Chksum.h:332-336)."""
    if isinstance(data, IpBufRef):
        return IpChksumAccumulator().getChksum(data)
    return (~IpChksumInverted(data, length)) & 0xFFFF


# --------------------------------------------------------------------------------------
# Buffer chains (Buf.h / BufUtils.h)
# --------------------------------------------------------------------------------------

class IpBufNode:
    """Node of a buffer chain: ``ptr`` (a bytes-like object; its first ``len`` bytes are
    the node's data), ``len`` and ``next`` (reference Buf.h:68-83)."""

    __slots__ = ("ptr", "len", "next")

    def __init__(self, ptr=b"", len: int = 0, next: "Optional[IpBufNode]" = None):
        self.ptr = memoryview(ptr).cast("B") if ptr is not None else memoryview(b"")
        self.len = int(len)
        self.next = next
        if self.len > self.ptr.nbytes:
            raise ValueError("IpBufNode: len exceeds the buffer")


class IpBufRef:
    """Reference to ``tot_len`` bytes of a chain starting at ``offset`` in ``node``
    (reference Buf.h:118-251)."""

    __slots__ = ("node", "offset", "tot_len")

    def __init__(self, node: Optional[IpBufNode] = None, offset: int = 0, tot_len: int = 0):
        self.node = node
        self.offset = int(offset)
        self.tot_len = int(tot_len)

    def _assert_sanity(self) -> None:  # Buf.h:242-246
        assert self.node is not None and self.offset <= self.node.len

    def getChunkPtr(self) -> memoryview:  # Buf.h:137-142
        self._assert_sanity()
        return self.node.ptr[self.offset:]

    def getChunkLength(self) -> int:  # Buf.h:149-154
        self._assert_sanity()
        return min(self.tot_len, self.node.len - self.offset)

    def revealHeader(self, amount: int) -> "IpBufRef":  # Buf.h:166-175
        assert amount <= self.offset
        return IpBufRef(self.node, self.offset - amount, self.tot_len + amount)

    def hasHeader(self, amount: int) -> bool:  # Buf.h:184-189
        self._assert_sanity()
        return amount <= self.tot_len and amount <= self.node.len - self.offset

    def hideHeader(self, amount: int) -> "IpBufRef":  # Buf.h:201-212
        self._assert_sanity()
        assert amount <= self.tot_len and amount <= self.node.len - self.offset
        return IpBufRef(self.node, self.offset + amount, self.tot_len - amount)

    def subTo(self, new_tot_len: int) -> "IpBufRef":  # Buf.h:226-235
        assert new_tot_len <= self.tot_len
        return IpBufRef(self.node, self.offset, new_tot_len)


def ipBufProcessBytes(buf: IpBufRef, processLen: int,
                      processChunk: Callable[[memoryview, int], int]) -> IpBufRef:
    """BufUtils.h:129-178 (same contract): hands ``processChunk(piece, piece_len)`` the
    non-empty pieces of the first `processLen` bytes of `buf`, node by node; it returns how
    many bytes of its piece it took, and taking fewer ends the walk inside that node. The
    returned reference starts after the bytes taken and keeps everything not taken. A used-up
    node is left behind whenever it has a successor, even when nothing more is wanted (the
    reference's eager advance, which also steps over empty nodes)."""
    assert buf.node is not None and processLen <= buf.tot_len
    untouched = buf.tot_len - processLen
    at, pos, want = buf.node, buf.offset, processLen
    while True:
        assert pos <= at.len
        avail = at.len - pos
        uses_up_node = want >= avail
        piece = avail if uses_up_node else want
        if piece:
            took = processChunk(at.ptr[pos:pos + piece], piece)
            assert 0 <= took <= piece
            pos += took
            want -= took
            if took != piece:  # the visitor stopped early
                break
        if not uses_up_node or at.next is None:
            break
        at, pos = at.next, 0
    return IpBufRef(at, pos, want + untouched)


# --------------------------------------------------------------------------------------
# Incremental accumulator (Chksum.h:148-316)
# --------------------------------------------------------------------------------------

class IpChksumAccumulator:
    """Incremental IP checksum of header words followed by data.

    ``State`` is the exported 32-bit running sum (Chksum.h:156, getState :181,
    resume :171). Header words are added without carry handling, as the reference does
    (addWord :191-217); chunk sums are added with end-around carry and the odd-chunk
    byte-swap rule (addIpBuf :283-315); getChksum folds twice and inverts (:245-250)."""

    __slots__ = ("_sum",)

    def __init__(self, state: Optional[int] = None):
        self._sum = 0 if state is None else int(state) & 0xFFFFFFFF

    def getState(self) -> int:
        return self._sum

    def addWord16(self, word: int) -> None:  # addWord(WrapType<uint16_t>) :191-194
        self._sum = (self._sum + (int(word) & 0xFFFF)) & 0xFFFFFFFF

    def addWordOctets(self, high_octet: int, low_octet: int) -> None:  # :202-206
        self.addWord16(((int(high_octet) & 0xFF) << 8) | (int(low_octet) & 0xFF))

    def addWord32(self, word: int) -> None:  # addWord(WrapType<uint32_t>) :213-217
        self.addWord16((int(word) >> 16) & 0xFFFF)
        self.addWord16(int(word) & 0xFFFF)

    def addEvenBytes(self, data, num_bytes: Optional[int] = None) -> None:  # :225-235
        mv = memoryview(data).cast("B")
        n = mv.nbytes if num_bytes is None else int(num_bytes)
        assert n % 2 == 0, "addEvenBytes: odd byte count"
        for i in range(0, n, 2):
            self.addWord16((mv[i] << 8) | mv[i + 1])

    @staticmethod
    def _swap(x: int) -> int:  # swapBytes :277-281
        return ((x >> 8) & 0x00FF00FF) | ((x << 8) & 0xFF00FF00)

    def _addIpBuf(self, buf: IpBufRef) -> None:  # :283-315
        swapped = [False]

        def chunk(mv: memoryview, n: int) -> int:
            b = IpChksumInverted(mv, n)
            s = self._sum + b
            if s > 0xFFFFFFFF:  # end-around carry
                s = (s & 0xFFFFFFFF) + 1
            if n % 2:
                s = self._swap(s)
                swapped[0] = not swapped[0]
            self._sum = s
            return n

        ipBufProcessBytes(buf, buf.tot_len, chunk)
        if swapped[0]:
            self._sum = self._swap(self._sum)

    def getChksum(self, buf: Optional[IpBufRef] = None) -> int:  # :245-250, :263-269
        if buf is not None and buf.tot_len > 0:
            self._addIpBuf(buf)
        s = self._sum
        s = (s & 0xFFFF) + (s >> 16)
        s = (s & 0xFFFF) + (s >> 16)
        return (~s) & 0xFFFF


# --------------------------------------------------------------------------------------
# Batched GPU entry points (device-resident torch tensors)
# --------------------------------------------------------------------------------------

def _torch():
    import torch  # plumbing only: device memory and streams
    return torch


def _stream_handle(stream, like=None) -> int:
    """The raw hipStream_t of `stream`; for None, torch's current stream of `like`'s device
    (a tensor), so every wrapper launches on the stream of the device its data lives on."""
    torch = _torch()
    if stream is None:  # torch's current stream, as a raw handle
        dev = like.device.index if like is not None and like.device.index is not None \
            else torch.cuda.current_device()
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:  # skips building a Stream object per call (small batches)
            return int(raw(dev))
        stream = torch.cuda.current_stream(dev)
    return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)


def _require_device(t, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _require_offsets(offsets, name: str = "offsets") -> None:
    """CSR offsets: a contiguous device tensor of 64-bit integers (the C-ABI reads uint64)."""
    torch = _torch()
    _require_device(offsets, name)
    if offsets.dtype not in (torch.int64, torch.uint64):
        raise ValueError(f"{name} must be an int64/uint64 device tensor")


def _same_device(a, b, names: str) -> None:
    if a.device != b.device:
        raise ValueError(f"{names} must be on the same device")


def _out_tensor(out, n: int, like):
    torch = _torch()
    if out is None:
        return torch.empty(n, dtype=torch.uint16, device=like.device)
    _require_device(out, "out")
    if out.dtype not in (torch.uint16, torch.int16) or out.numel() < n:
        raise ValueError("out must be a uint16/int16 device tensor with >= n elements")
    _same_device(out, like, "out and the input")
    return out


def chksum_batch_strided(buf, stride: int, length: int, n: int, *, out=None,
                         final: bool = False, byte_offset: int = 0, stream=None,
                         just_written: bool = False):
    """``out[i] = IpChksumInverted(buf[byte_offset + i*stride :][:length])`` for i < n
    (``IpChksum`` with ``final=True``), on the GPU. ``buf`` is a device uint8 tensor.
    ``just_written``: the AIPSTACK_CHKSUM_JUST_WRITTEN hint (the bytes were written by device
    kernels with ordinary stores since they were last read); the results do not change."""
    _require_device(buf, "buf")
    if n and byte_offset + (n - 1) * stride + length > buf.numel() * buf.element_size():
        raise ValueError("batch exceeds buf")
    out = _out_tensor(out, n, buf)
    flags = (AIPSTACK_CHKSUM_FINAL if final else 0) | (
        AIPSTACK_CHKSUM_JUST_WRITTEN if just_written else 0)
    st = _lib.load().aipstack_chksum_batch_strided(
        buf.data_ptr() + byte_offset, stride, length, n, out.data_ptr(), flags,
        _stream_handle(stream, buf))
    _check(st, "aipstack_chksum_batch_strided")
    return out


def chksum_batch_csr(buf, offsets, *, out=None, final: bool = False, stream=None):
    """``out[i] = IpChksumInverted(buf[offsets[i]:offsets[i+1]])`` on the GPU. ``offsets``
    is a device int64/uint64 tensor of n+1 non-decreasing byte offsets."""
    _require_device(buf, "buf")
    _require_offsets(offsets)
    _same_device(buf, offsets, "buf and offsets")
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets must hold n+1 entries")
    out = _out_tensor(out, n, buf)
    st = _lib.load().aipstack_chksum_batch_csr(
        buf.data_ptr(), offsets.data_ptr(), n, out.data_ptr(),
        AIPSTACK_CHKSUM_FINAL if final else 0, _stream_handle(stream, buf))
    _check(st, "aipstack_chksum_batch_csr")
    return out


def _require_lens(lens, n_slots_bytes, slot_stride, buf):
    torch = _torch()
    _require_device(lens, "lens")
    if lens.dtype not in (torch.int32, torch.uint32):
        raise ValueError("lens must be an int32/uint32 device tensor")
    _same_device(buf, lens, "buf and lens")
    if slot_stride <= 0 or lens.numel() * slot_stride > n_slots_bytes:
        raise ValueError("buf must hold n whole slots of slot_stride bytes")
    return lens.numel()


def chksum_batch_slotted(buf, slot_stride: int, lens, *, out=None, final: bool = False,
                         stream=None, just_written: bool = False):
    """Ring slots on the GPU: ``out[i] = IpChksumInverted(buf[i*slot_stride:][:lens[i]])``
    (``IpChksum`` with ``final=True``). ``lens``: int32/uint32 device tensor of n lengths,
    each <= min(slot_stride, 65535); ``buf`` holds n whole slots."""
    _require_device(buf, "buf")
    n = _require_lens(lens, buf.numel() * buf.element_size(), slot_stride, buf)
    out = _out_tensor(out, n, buf)
    _check(_lib.load().aipstack_chksum_batch_slotted(
        buf.data_ptr(), slot_stride, lens.data_ptr(), n, out.data_ptr(),
        (AIPSTACK_CHKSUM_FINAL if final else 0) | (AIPSTACK_CHKSUM_JUST_WRITTEN if just_written else 0),
        _stream_handle(stream, buf)),
        "aipstack_chksum_batch_slotted")
    return out


def rx_verify_slotted(frames, slot_stride: int, lens, *, out=None, stream=None):
    """Rx verify of a ring of frame slots on the GPU (frame i = the lens[i] bytes at
    frames[i*slot_stride:]); one AIPSTACK_RX_* verdict per frame."""
    _require_device(frames, "frames")
    n = _require_lens(lens, frames.numel() * frames.element_size(), slot_stride, frames)
    out = _u8_out(out, n, frames)
    _check(_lib.load().aipstack_chksum_rx_verify_slotted(
        frames.data_ptr(), slot_stride, lens.data_ptr(), n, out.data_ptr(),
        _stream_handle(stream, frames)), "aipstack_chksum_rx_verify_slotted")
    return out


def tx_fill_slotted(frames, slot_stride: int, lens, *, out=None, stream=None, split=False,
                    workspace=None):
    """Tx fill, in place, of a ring of frame slots on the GPU; one status per frame.
    ``split=True`` runs ``aipstack_chksum_tx_fill_slotted_split`` (records pass + scatter pass
    through a workspace of 8 bytes per frame, as :func:`tx_fill`); both write the same bytes."""
    _require_device(frames, "frames")
    n = _require_lens(lens, frames.numel() * frames.element_size(), slot_stride, frames)
    out = _u8_out(out, n, frames)
    lib = _lib.load()
    if not split:
        _check(lib.aipstack_chksum_tx_fill_slotted(
            frames.data_ptr(), slot_stride, lens.data_ptr(), n, out.data_ptr(),
            _stream_handle(stream, frames)), "aipstack_chksum_tx_fill_slotted")
        return out
    _split_call(lib, "aipstack_chksum_tx_fill_slotted_split", frames, n, stream, workspace,
                lambda ws, ws_bytes, h: (frames.data_ptr(), slot_stride, lens.data_ptr(), n,
                                         out.data_ptr(), ws, ws_bytes, h))
    return out


def tx_fill_records_slotted(frames, slot_stride: int, lens, *, out=None, stream=None):
    """The Tx records (see :func:`tx_fill_records`) of a ring of frame slots."""
    torch = _torch()
    _require_device(frames, "frames")
    n = _require_lens(lens, frames.numel() * frames.element_size(), slot_stride, frames)
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=frames.device)
    _check(_lib.load().aipstack_chksum_tx_fill_records_slotted(
        frames.data_ptr(), slot_stride, lens.data_ptr(), n, out.data_ptr(),
        _stream_handle(stream, frames)), "aipstack_chksum_tx_fill_records_slotted")
    return out


def chksum_batch_seeded_csr(buf, offsets, states, *, out=None, stream=None):
    """``out[i] = IpChksumAccumulator(State(states[i])).getChksum(IpBufRef(packet i))`` on
    the GPU (final checksum). ``states`` is a device int32/uint32 tensor of n states."""
    _require_device(buf, "buf")
    _require_offsets(offsets)
    _require_device(states, "states")
    _same_device(buf, offsets, "buf and offsets")
    _same_device(buf, states, "buf and states")
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets must hold n+1 entries")
    if states.numel() < n or states.element_size() != 4:
        raise ValueError("states must hold n 32-bit entries")
    out = _out_tensor(out, n, buf)
    st = _lib.load().aipstack_chksum_batch_seeded_csr(
        buf.data_ptr(), offsets.data_ptr(), states.data_ptr(), n, out.data_ptr(),
        _stream_handle(stream, buf))
    _check(st, "aipstack_chksum_batch_seeded_csr")
    return out


def _host_u64(a):
    """Host offsets as the C-ABI's uint64: a contiguous int64 array is passed as it is (a
    view; the engine rejects the huge values a negative entry becomes, as non-decreasing
    offsets within the frames), anything else is converted (a copy)."""
    if isinstance(a, np.ndarray) and a.dtype == np.int64 and a.flags.c_contiguous:
        return a.view(np.uint64)
    return np.ascontiguousarray(a, dtype=np.uint64)


def _host_u32(a):
    """Host lengths as the C-ABI's uint32 (int32 viewed, as _host_u64; the engine rejects
    lengths above the slot stride)."""
    if isinstance(a, np.ndarray) and a.dtype == np.int32 and a.flags.c_contiguous:
        return a.view(np.uint32)
    return np.ascontiguousarray(a, dtype=np.uint32)


class ChksumEngine:
    """Host-memory streaming engine (C-ABI ``aipstack_chksum_engine_*``): checksums
    batches held in HOST memory (numpy arrays) and returns results in host memory,
    pipelining H2D / kernel / D2H over ``nstreams`` HIP streams. ``strided`` / ``csr`` are
    synchronous; ``submit_strided`` / ``submit_csr`` return a ticket at once and
    ``poll`` / ``wait`` complete it, so the caller can prepare its next batch meanwhile."""

    def __init__(self, device: int = 0, chunk_bytes: int = 0, nstreams: int = 2):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _check(self._lib.aipstack_chksum_engine_create(device, chunk_bytes, nstreams,
                                                       ctypes.byref(h)),
               "aipstack_chksum_engine_create")
        self._h = h
        self._registered = []
        self._inflight = {}

    def close(self) -> None:
        if self._h:
            self._lib.aipstack_chksum_engine_destroy(self._h)  # waits for every stream
            self._h = None
            self._registered = []
            self._inflight = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def register(self, arr: np.ndarray) -> None:
        """Page-lock `arr` (kept alive by the engine) so that the kernels read batches in it
        where they lie (zero copy; or DMA'd directly with tune("engine_zero_copy", 0))."""
        _check(self._lib.aipstack_chksum_engine_register(self._h, arr.ctypes.data, arr.nbytes),
               "aipstack_chksum_engine_register")
        self._registered.append(arr)

    def unregister(self, arr: np.ndarray) -> None:
        """Unpin `arr`; batches still in flight are completed first (C engine)."""
        _check(self._lib.aipstack_chksum_engine_unregister(self._h, arr.ctypes.data),
               "aipstack_chksum_engine_unregister")
        self._registered = [a for a in self._registered if a is not arr]

    @staticmethod
    def _host_args(buf: np.ndarray, out, n: int, dtype=np.uint16) -> np.ndarray:
        if not isinstance(buf, np.ndarray) or not buf.flags.c_contiguous:
            raise ValueError("buf must be a C-contiguous numpy array")
        if out is None:
            return np.empty(max(n, 0), dtype=dtype)
        if (not isinstance(out, np.ndarray) or out.dtype != dtype
                or not out.flags.c_contiguous or not out.flags.writeable or out.size < n):
            raise ValueError(f"out must be a writable C-contiguous {np.dtype(dtype).name} array "
                             "of >= n elements")
        return out

    def strided(self, buf: np.ndarray, stride: int, length: int, n: int, *, out=None,
                final: bool = False) -> np.ndarray:
        if n and (n - 1) * stride + length > buf.nbytes:
            raise ValueError("batch exceeds buf")
        out = self._host_args(buf, out, n)
        _check(self._lib.aipstack_chksum_engine_host_strided(
            self._h, buf.ctypes.data, stride, length, n, out.ctypes.data,
            AIPSTACK_CHKSUM_FINAL if final else 0), "aipstack_chksum_engine_host_strided")
        return out

    # ---- asynchronous batches: submit returns a ticket, poll / wait complete it --------

    def submit_strided(self, buf: np.ndarray, stride: int, length: int, n: int, *, out=None,
                       final: bool = False):
        """Enqueue a strided batch; returns (ticket, out). `out` is filled when the batch
        completes (wait / poll); a registered `buf` must not change until then."""
        if n and (n - 1) * stride + length > buf.nbytes:
            raise ValueError("batch exceeds buf")
        out = self._host_args(buf, out, n)
        t = ctypes.c_uint64(0)
        st = self._lib.aipstack_chksum_engine_submit_strided(
            self._h, buf.ctypes.data, stride, length, n, out.ctypes.data,
            AIPSTACK_CHKSUM_FINAL if final else 0, ctypes.byref(t))
        self._submitted(st, t.value, "aipstack_chksum_engine_submit_strided", buf, out)
        return t.value, out

    def submit_csr(self, buf: np.ndarray, offsets: np.ndarray, *, out=None,
                   final: bool = False):
        """Enqueue a CSR batch; returns (ticket, out) (see submit_strided)."""
        o = _host_u64(offsets)
        n = o.size - 1
        if n > 0 and int(o[-1]) > buf.nbytes:
            raise ValueError("offsets exceed buf")
        out = self._host_args(buf, out, n)
        t = ctypes.c_uint64(0)
        st = self._lib.aipstack_chksum_engine_submit_csr(
            self._h, buf.ctypes.data, o.ctypes.data, max(n, 0), out.ctypes.data,
            AIPSTACK_CHKSUM_FINAL if final else 0, ctypes.byref(t))
        self._submitted(st, t.value, "aipstack_chksum_engine_submit_csr", buf, o, out)
        return t.value, out

    def _keep(self, ticket, *arrays):
        # the buffers the GPU and the completion still use stay alive until completion
        if ticket:
            self._inflight[ticket] = arrays

    def _submitted(self, st, ticket, where, *arrays):
        """After a submit_* C call: keep the arrays of a batch in flight, or, if the submit
        failed part-way, complete the pieces it did enqueue (they still read `arrays` and,
        for Tx, write into the frames) before raising."""
        if st != AIPSTACK_CHKSUM_OK:
            if ticket:
                self._lib.aipstack_chksum_engine_wait(self._h, ticket)
            raise ChksumError(st, where)
        self._keep(ticket, *arrays)

    def locality(self):
        """(NUMA node of the device or -1, CPUs the engine's host threads are pinned to)."""
        node, cpus = ctypes.c_int(-1), ctypes.c_int(0)
        _check(self._lib.aipstack_chksum_engine_locality(self._h, ctypes.byref(node),
                                                         ctypes.byref(cpus)),
               "aipstack_chksum_engine_locality")
        return node.value, cpus.value

    def poll(self, ticket: int) -> bool:
        """True once batch `ticket` is complete (its `out` filled); False while running."""
        st = self._lib.aipstack_chksum_engine_poll(self._h, ticket)
        if st == 1:
            return False
        self._inflight.pop(ticket, None)
        _check(st, "aipstack_chksum_engine_poll")
        return True

    def wait(self, ticket: int) -> None:
        """Block until batch `ticket` is complete."""
        st = self._lib.aipstack_chksum_engine_wait(self._h, ticket)
        self._inflight.pop(ticket, None)
        _check(st, "aipstack_chksum_engine_wait")

    def rx_verify(self, frames: np.ndarray, offsets: np.ndarray, *, out=None) -> np.ndarray:
        """Rx verify of raw Ethernet frames in HOST memory (frame i =
        ``frames[offsets[i]:offsets[i+1]]``): one AIPSTACK_RX_* verdict per frame (uint8),
        as :func:`rx_verify` on the device."""
        o = _host_u64(offsets)
        n = o.size - 1
        if n > 0 and int(o[-1]) > frames.nbytes:
            raise ValueError("offsets exceed frames")
        out = self._host_args(frames, out, n, np.uint8)
        _check(self._lib.aipstack_chksum_engine_host_rx_verify(
            self._h, frames.ctypes.data, o.ctypes.data, max(n, 0), out.ctypes.data),
            "aipstack_chksum_engine_host_rx_verify")
        return out

    def submit_rx_verify(self, frames: np.ndarray, offsets: np.ndarray, *, out=None):
        """Enqueue an Rx verify batch; returns (ticket, out) (see submit_strided)."""
        o = _host_u64(offsets)
        n = o.size - 1
        if n > 0 and int(o[-1]) > frames.nbytes:
            raise ValueError("offsets exceed frames")
        out = self._host_args(frames, out, n, np.uint8)
        t = ctypes.c_uint64(0)
        st = self._lib.aipstack_chksum_engine_submit_rx_verify(
            self._h, frames.ctypes.data, o.ctypes.data, max(n, 0), out.ctypes.data,
            ctypes.byref(t))
        self._submitted(st, t.value, "aipstack_chksum_engine_submit_rx_verify", frames, o, out)
        return t.value, out

    @staticmethod
    def _tx_args(frames, offsets, status):
        if not isinstance(frames, np.ndarray) or not frames.flags.writeable:
            raise ValueError("frames must be a writable numpy array (filled in place)")
        o = _host_u64(offsets)
        n = o.size - 1
        if n > 0 and int(o[-1]) > frames.nbytes:
            raise ValueError("offsets exceed frames")
        return o, n, ChksumEngine._host_args(frames, status, n, np.uint8)

    def tx_fill(self, frames: np.ndarray, offsets: np.ndarray, *, status=None) -> np.ndarray:
        """Tx fill of raw Ethernet frames in HOST memory, IN PLACE (frame i =
        ``frames[offsets[i]:offsets[i+1]]``): the IPv4 header and L4 checksum fields are
        written as :func:`tx_fill` does on the device; returns the per-frame AIPSTACK_TX_*
        statuses (uint8)."""
        o, n, status = self._tx_args(frames, offsets, status)
        _check(self._lib.aipstack_chksum_engine_host_tx_fill(
            self._h, frames.ctypes.data, o.ctypes.data, max(n, 0), status.ctypes.data),
            "aipstack_chksum_engine_host_tx_fill")
        return status

    def submit_tx_fill(self, frames: np.ndarray, offsets: np.ndarray, *, status=None):
        """Enqueue a Tx fill batch; returns (ticket, status). The frames are filled and
        `status` written when the batch completes (wait / poll); `frames` must not be
        touched until then."""
        o, n, status = self._tx_args(frames, offsets, status)
        # the completion reads the offsets again (it writes the fields into the frames, on
        # the engine's applier thread): a private copy, so the caller may reuse its array
        o = o.copy()
        t = ctypes.c_uint64(0)
        st = self._lib.aipstack_chksum_engine_submit_tx_fill(
            self._h, frames.ctypes.data, o.ctypes.data, max(n, 0), status.ctypes.data,
            ctypes.byref(t))
        # the completion reads the offsets again (it writes the fields into the frames)
        self._submitted(st, t.value, "aipstack_chksum_engine_submit_tx_fill", frames, o, status)
        return t.value, status

    # ---- ring slots: frame i = the lens[i] bytes at buf[i * slot_stride:] ----------------

    @staticmethod
    def _slot_args(buf, slot_stride: int, lens):
        ln = _host_u32(lens)
        n = ln.size
        if slot_stride <= 0 or n * slot_stride > buf.nbytes:
            raise ValueError("the buffer must hold n whole slots of slot_stride bytes")
        return ln, n

    def slotted(self, buf: np.ndarray, slot_stride: int, lens, *, out=None,
                final: bool = False) -> np.ndarray:
        """Checksums of the packets of a ring of slots in HOST memory
        (``aipstack_chksum_engine_host_slotted``)."""
        ln, n = self._slot_args(buf, slot_stride, lens)
        out = self._host_args(buf, out, n)
        _check(self._lib.aipstack_chksum_engine_host_slotted(
            self._h, buf.ctypes.data, slot_stride, ln.ctypes.data, n, out.ctypes.data,
            AIPSTACK_CHKSUM_FINAL if final else 0), "aipstack_chksum_engine_host_slotted")
        return out

    def submit_slotted(self, buf: np.ndarray, slot_stride: int, lens, *, out=None,
                       final: bool = False):
        ln, n = self._slot_args(buf, slot_stride, lens)
        out = self._host_args(buf, out, n)
        t = ctypes.c_uint64(0)
        st = self._lib.aipstack_chksum_engine_submit_slotted(
            self._h, buf.ctypes.data, slot_stride, ln.ctypes.data, n, out.ctypes.data,
            AIPSTACK_CHKSUM_FINAL if final else 0, ctypes.byref(t))
        self._submitted(st, t.value, "aipstack_chksum_engine_submit_slotted", buf, ln, out)
        return t.value, out

    def rx_verify_slotted(self, frames: np.ndarray, slot_stride: int, lens, *,
                          out=None) -> np.ndarray:
        """Rx verify of a ring of frame slots in HOST memory."""
        ln, n = self._slot_args(frames, slot_stride, lens)
        out = self._host_args(frames, out, n, np.uint8)
        _check(self._lib.aipstack_chksum_engine_host_rx_verify_slotted(
            self._h, frames.ctypes.data, slot_stride, ln.ctypes.data, n, out.ctypes.data),
            "aipstack_chksum_engine_host_rx_verify_slotted")
        return out

    def submit_rx_verify_slotted(self, frames: np.ndarray, slot_stride: int, lens, *,
                                 out=None):
        """Enqueue an Rx verify batch of frame slots; returns (ticket, out). The slots must
        not be refilled until the ticket completes (the receive loop of a TAP ring:
        tap/linux/TapDeviceLinux.cpp:156-178)."""
        ln, n = self._slot_args(frames, slot_stride, lens)
        out = self._host_args(frames, out, n, np.uint8)
        t = ctypes.c_uint64(0)
        st = self._lib.aipstack_chksum_engine_submit_rx_verify_slotted(
            self._h, frames.ctypes.data, slot_stride, ln.ctypes.data, n, out.ctypes.data,
            ctypes.byref(t))
        self._submitted(st, t.value, "aipstack_chksum_engine_submit_rx_verify_slotted", frames,
                        ln, out)
        return t.value, out

    def submit_tx_fill_slotted(self, frames: np.ndarray, slot_stride: int, lens, *,
                               status=None):
        """Enqueue a Tx fill of frame slots, in place; returns (ticket, status). The frames
        are filled when the ticket completes and must not be touched until then."""
        if not frames.flags.writeable:
            raise ValueError("frames must be writable (filled in place)")
        ln, n = self._slot_args(frames, slot_stride, lens)
        status = self._host_args(frames, status, n, np.uint8)
        t = ctypes.c_uint64(0)
        st = self._lib.aipstack_chksum_engine_submit_tx_fill_slotted(
            self._h, frames.ctypes.data, slot_stride, ln.ctypes.data, n, status.ctypes.data,
            ctypes.byref(t))
        self._submitted(st, t.value, "aipstack_chksum_engine_submit_tx_fill_slotted", frames,
                        ln, status)
        return t.value, status

    def tx_fill_slotted(self, frames: np.ndarray, slot_stride: int, lens, *,
                        status=None) -> np.ndarray:
        """Tx fill, in place, of a ring of frame slots in HOST memory."""
        if not frames.flags.writeable:
            raise ValueError("frames must be writable (filled in place)")
        ln, n = self._slot_args(frames, slot_stride, lens)
        status = self._host_args(frames, status, n, np.uint8)
        _check(self._lib.aipstack_chksum_engine_host_tx_fill_slotted(
            self._h, frames.ctypes.data, slot_stride, ln.ctypes.data, n, status.ctypes.data),
            "aipstack_chksum_engine_host_tx_fill_slotted")
        return status

    def csr(self, buf: np.ndarray, offsets: np.ndarray, *, out=None,
            final: bool = False) -> np.ndarray:
        o = _host_u64(offsets)
        n = o.size - 1
        if n > 0 and int(o[-1]) > buf.nbytes:
            raise ValueError("offsets exceed buf")
        out = self._host_args(buf, out, n)
        _check(self._lib.aipstack_chksum_engine_host_csr(
            self._h, buf.ctypes.data, o.ctypes.data, n, out.ctypes.data,
            AIPSTACK_CHKSUM_FINAL if final else 0), "aipstack_chksum_engine_host_csr")
        return out


class ChksumEngineGroup:
    """Several devices behind one host-memory batch in ONE process (C-ABI
    ``aipstack_chksum_engine_group_*``): one engine per entry of ``devices`` (repeats
    allowed), each batch split into contiguous ranges of about equal bytes run concurrently
    (small batches go whole to one device, round robin). The synchronous calls return the
    results; ``submit_*`` return ``(ticket, out)`` at once, ``poll`` / ``wait`` complete a
    ticket. ``last_status`` holds each engine's status of the last completed call."""

    def __init__(self, devices, chunk_bytes: int = 0, nstreams: int = 4):
        self._lib = _lib.load()
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        h = ctypes.c_void_p()
        _check(self._lib.aipstack_chksum_engine_group_create(devs, len(devices), chunk_bytes,
                                                             nstreams, ctypes.byref(h)),
               "aipstack_chksum_engine_group_create")
        self._h = h
        self.size = len(devices)
        self._registered = []
        self._inflight = {}
        self.last_status = [0] * self.size

    def close(self) -> None:
        if self._h:
            self._lib.aipstack_chksum_engine_group_destroy(self._h)  # completes every batch
            self._h = None
            self._registered = []
            self._inflight = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def register(self, arr: np.ndarray) -> None:
        _check(self._lib.aipstack_chksum_engine_group_register(self._h, arr.ctypes.data,
                                                               arr.nbytes),
               "aipstack_chksum_engine_group_register")
        self._registered.append(arr)

    def unregister(self, arr: np.ndarray) -> None:
        _check(self._lib.aipstack_chksum_engine_group_unregister(self._h, arr.ctypes.data),
               "aipstack_chksum_engine_group_unregister")
        self._registered = [a for a in self._registered if a is not arr]

    def _call(self, fn, where, *args):
        ds = (ctypes.c_int * self.size)()
        st = getattr(self._lib, fn)(self._h, *args, ds)
        self.last_status = list(ds)
        _check(st, where)

    def _submit(self, fn, arrays, *args):
        """A submit_* C call; the arrays of the batch stay referenced until it completes."""
        t = ctypes.c_uint64(0)
        st = getattr(self._lib, fn)(self._h, *args, ctypes.byref(t))
        if st != AIPSTACK_CHKSUM_OK:
            if t.value:  # ranges already enqueued still read (and, Tx, write) the arrays
                self._lib.aipstack_chksum_engine_group_wait(self._h, t.value, None)
            raise ChksumError(st, fn)
        self._inflight[t.value] = arrays
        return t.value

    def poll(self, ticket: int) -> bool:
        """True once group batch `ticket` is complete; False while a device still works."""
        ds = (ctypes.c_int * self.size)()
        st = self._lib.aipstack_chksum_engine_group_poll(self._h, ticket, ds)
        if st == 1:
            return False
        self._inflight.pop(ticket, None)
        self.last_status = list(ds)
        _check(st, "aipstack_chksum_engine_group_poll")
        return True

    def wait(self, ticket: int) -> None:
        """Block until group batch `ticket` is complete."""
        ds = (ctypes.c_int * self.size)()
        st = self._lib.aipstack_chksum_engine_group_wait(self._h, ticket, ds)
        self._inflight.pop(ticket, None)
        self.last_status = list(ds)
        _check(st, "aipstack_chksum_engine_group_wait")

    def locality(self):
        """Per engine: (NUMA node of its device or -1, CPUs its host threads are pinned to)."""
        out = []
        for k in range(self.size):
            e = self._lib.aipstack_chksum_engine_group_engine(self._h, k)
            node, cpus = ctypes.c_int(-1), ctypes.c_int(0)
            _check(self._lib.aipstack_chksum_engine_locality(e, ctypes.byref(node),
                                                             ctypes.byref(cpus)),
                   "aipstack_chksum_engine_locality")
            out.append((node.value, cpus.value))
        return out

    def region_mapped(self, arr: np.ndarray) -> bool:
        """Whether every device's kernels read the registered `arr` in place (zero copy)."""
        st = self._lib.aipstack_chksum_engine_group_region_mapped(self._h, arr.ctypes.data)
        _check(min(st, 0), "aipstack_chksum_engine_group_region_mapped")
        return st == 1

    def submit_strided(self, buf, stride: int, length: int, n: int, *, out=None, final=False):
        if n and (n - 1) * stride + length > buf.nbytes:
            raise ValueError("batch exceeds buf")
        out = ChksumEngine._host_args(buf, out, n)
        t = self._submit("aipstack_chksum_engine_group_submit_strided", (buf, out),
                         buf.ctypes.data, stride, length, n, out.ctypes.data,
                         AIPSTACK_CHKSUM_FINAL if final else 0)
        return t, out

    def submit_csr(self, buf, offsets, *, out=None, final=False):
        # a copy: a range may be submitted later on its device's worker thread, after this
        # returns, and must not see the caller refill its offsets (the bounds checked here)
        o = _host_u64(offsets).copy()
        n = o.size - 1
        if n > 0 and int(o[-1]) > buf.nbytes:
            raise ValueError("offsets exceed buf")
        out = ChksumEngine._host_args(buf, out, n)
        t = self._submit("aipstack_chksum_engine_group_submit_csr", (buf, o, out),
                         buf.ctypes.data, o.ctypes.data, max(n, 0), out.ctypes.data,
                         AIPSTACK_CHKSUM_FINAL if final else 0)
        return t, out

    def submit_rx_verify(self, frames, offsets, *, out=None):
        o = _host_u64(offsets).copy()  # (as submit_csr)
        n = o.size - 1
        if n > 0 and int(o[-1]) > frames.nbytes:
            raise ValueError("offsets exceed frames")
        out = ChksumEngine._host_args(frames, out, n, np.uint8)
        t = self._submit("aipstack_chksum_engine_group_submit_rx_verify", (frames, o, out),
                         frames.ctypes.data, o.ctypes.data, max(n, 0), out.ctypes.data)
        return t, out

    def submit_tx_fill(self, frames, offsets, *, status=None):
        o, n, status = ChksumEngine._tx_args(frames, offsets, status)
        o = o.copy()  # read again when the fields are applied (see ChksumEngine.submit_tx_fill)
        t = self._submit("aipstack_chksum_engine_group_submit_tx_fill", (frames, o, status),
                         frames.ctypes.data, o.ctypes.data, max(n, 0), status.ctypes.data)
        return t, status

    def submit_slotted(self, buf, slot_stride: int, lens, *, out=None, final=False):
        ln, n = ChksumEngine._slot_args(buf, slot_stride, lens)
        ln = ln.copy()  # (as submit_csr: the lengths are read again on a worker thread)
        out = ChksumEngine._host_args(buf, out, n)
        t = self._submit("aipstack_chksum_engine_group_submit_slotted", (buf, ln, out),
                         buf.ctypes.data, slot_stride, ln.ctypes.data, n, out.ctypes.data,
                         AIPSTACK_CHKSUM_FINAL if final else 0)
        return t, out

    def submit_rx_verify_slotted(self, frames, slot_stride: int, lens, *, out=None):
        ln, n = ChksumEngine._slot_args(frames, slot_stride, lens)
        ln = ln.copy()  # (as submit_slotted)
        out = ChksumEngine._host_args(frames, out, n, np.uint8)
        t = self._submit("aipstack_chksum_engine_group_submit_rx_verify_slotted",
                         (frames, ln, out), frames.ctypes.data, slot_stride, ln.ctypes.data, n,
                         out.ctypes.data)
        return t, out

    def submit_tx_fill_slotted(self, frames, slot_stride: int, lens, *, status=None):
        if not frames.flags.writeable:
            raise ValueError("frames must be writable (filled in place)")
        ln, n = ChksumEngine._slot_args(frames, slot_stride, lens)
        ln = ln.copy()  # (as submit_slotted)
        status = ChksumEngine._host_args(frames, status, n, np.uint8)
        t = self._submit("aipstack_chksum_engine_group_submit_tx_fill_slotted",
                         (frames, ln, status), frames.ctypes.data, slot_stride, ln.ctypes.data,
                         n, status.ctypes.data)
        return t, status

    def strided(self, buf, stride: int, length: int, n: int, *, out=None, final=False):
        if n and (n - 1) * stride + length > buf.nbytes:
            raise ValueError("batch exceeds buf")
        out = ChksumEngine._host_args(buf, out, n)
        self._call("aipstack_chksum_engine_group_host_strided", "engine group strided",
                   buf.ctypes.data, stride, length, n, out.ctypes.data,
                   AIPSTACK_CHKSUM_FINAL if final else 0)
        return out

    def csr(self, buf, offsets, *, out=None, final=False):
        o = _host_u64(offsets)
        n = o.size - 1
        if n > 0 and int(o[-1]) > buf.nbytes:
            raise ValueError("offsets exceed buf")
        out = ChksumEngine._host_args(buf, out, n)
        self._call("aipstack_chksum_engine_group_host_csr", "engine group csr", buf.ctypes.data,
                   o.ctypes.data, max(n, 0), out.ctypes.data, AIPSTACK_CHKSUM_FINAL if final else 0)
        return out

    def rx_verify(self, frames, offsets, *, out=None):
        o = _host_u64(offsets)
        n = o.size - 1
        if n > 0 and int(o[-1]) > frames.nbytes:
            raise ValueError("offsets exceed frames")
        out = ChksumEngine._host_args(frames, out, n, np.uint8)
        self._call("aipstack_chksum_engine_group_host_rx_verify", "engine group rx_verify",
                   frames.ctypes.data, o.ctypes.data, max(n, 0), out.ctypes.data)
        return out

    def tx_fill(self, frames, offsets, *, status=None):
        o, n, status = ChksumEngine._tx_args(frames, offsets, status)
        self._call("aipstack_chksum_engine_group_host_tx_fill", "engine group tx_fill",
                   frames.ctypes.data, o.ctypes.data, max(n, 0), status.ctypes.data)
        return status

    # ring slots: frame i = the lens[i] bytes at buf[i * slot_stride:]
    def slotted(self, buf, slot_stride: int, lens, *, out=None, final=False):
        ln, n = ChksumEngine._slot_args(buf, slot_stride, lens)
        out = ChksumEngine._host_args(buf, out, n)
        self._call("aipstack_chksum_engine_group_host_slotted", "engine group slotted",
                   buf.ctypes.data, slot_stride, ln.ctypes.data, n, out.ctypes.data,
                   AIPSTACK_CHKSUM_FINAL if final else 0)
        return out

    def rx_verify_slotted(self, frames, slot_stride: int, lens, *, out=None):
        ln, n = ChksumEngine._slot_args(frames, slot_stride, lens)
        out = ChksumEngine._host_args(frames, out, n, np.uint8)
        self._call("aipstack_chksum_engine_group_host_rx_verify_slotted",
                   "engine group rx_verify_slotted", frames.ctypes.data, slot_stride,
                   ln.ctypes.data, n, out.ctypes.data)
        return out

    def tx_fill_slotted(self, frames, slot_stride: int, lens, *, status=None):
        if not frames.flags.writeable:
            raise ValueError("frames must be writable (filled in place)")
        ln, n = ChksumEngine._slot_args(frames, slot_stride, lens)
        status = ChksumEngine._host_args(frames, status, n, np.uint8)
        self._call("aipstack_chksum_engine_group_host_tx_fill_slotted",
                   "engine group tx_fill_slotted", frames.ctypes.data, slot_stride,
                   ln.ctypes.data, n, status.ctypes.data)
        return status


def chksum_batch_chain(chunk_addr, chunk_len, chunk_index, states=None, *, out=None,
                       final: bool = False, stream=None, just_written: bool = False):
    """Chained (scatter-gather) batch on the GPU: chain i = chunks
    ``[chunk_index[i], chunk_index[i+1])``, chunk k = ``chunk_len[k]`` bytes at DEVICE
    address ``chunk_addr[k]``. ``final=True`` gives
    ``IpChksumAccumulator(State(states[i])).getChksum(chain i)``; ``final=False`` its NOT.
    Tensors: int64 addresses, int32 lengths, int64 index (n+1), int32 states (or None)."""
    for t, name in ((chunk_addr, "chunk_addr"), (chunk_len, "chunk_len"),
                    (chunk_index, "chunk_index")):
        _require_device(t, name)
    if chunk_addr.element_size() != 8 or chunk_len.element_size() != 4 \
            or chunk_index.element_size() != 8:
        raise ValueError("chunk_addr/chunk_index must be 64-bit, chunk_len 32-bit")
    n = chunk_index.numel() - 1
    if n < 0:
        raise ValueError("chunk_index must hold n+1 entries")
    sp = 0
    if states is not None:
        _require_device(states, "states")
        if states.numel() < n or states.element_size() != 4:
            raise ValueError("states must hold n 32-bit entries")
        sp = states.data_ptr()
    out = _out_tensor(out, n, chunk_index)
    st = _lib.load().aipstack_chksum_batch_chain(
        chunk_addr.data_ptr(), chunk_len.data_ptr(), chunk_index.data_ptr(), sp or None, n,
        out.data_ptr(),
        (AIPSTACK_CHKSUM_FINAL if final else 0) | (AIPSTACK_CHKSUM_JUST_WRITTEN if just_written else 0),
        _stream_handle(stream, chunk_index))
    _check(st, "aipstack_chksum_batch_chain")
    return out


def chksum_chain_fill(chunk_addr, chunk_len, chunk_index, states, fields, *, out=None,
                      zero_as_ffff: bool = False, stream=None, just_written: bool = False):
    """The Tx form of :func:`chksum_batch_chain`: chain i's final checksum
    (``IpChksumAccumulator(State(states[i])).getChksum(chain i)``) is stored big-endian at
    DEVICE address ``fields[i]`` (int64 tensor; 0 = no store) -- the checksum field of the
    header the chain starts with, which must read 0 when the batch runs, as the reference
    sets it before summing (tcp/IpTcpProto_output.h:1251-1277, udp/IpUdpProto.h:164-179).
    ``zero_as_ffff`` sends a computed 0 as 0xFFFF (UDP). ``just_written``: the
    AIPSTACK_CHKSUM_JUST_WRITTEN hint (results unchanged). Returns the checksums (``out``)."""
    for t, name in ((chunk_addr, "chunk_addr"), (chunk_len, "chunk_len"),
                    (chunk_index, "chunk_index"), (fields, "fields")):
        _require_device(t, name)
    if chunk_addr.element_size() != 8 or chunk_len.element_size() != 4 \
            or chunk_index.element_size() != 8 or fields.element_size() != 8:
        raise ValueError("chunk_addr/chunk_index/fields must be 64-bit, chunk_len 32-bit")
    n = chunk_index.numel() - 1
    if n < 0:
        raise ValueError("chunk_index must hold n+1 entries")
    if fields.numel() < n:
        raise ValueError("fields must hold n entries")
    sp = 0
    if states is not None:
        _require_device(states, "states")
        if states.numel() < n or states.element_size() != 4:
            raise ValueError("states must hold n 32-bit entries")
        sp = states.data_ptr()
    out = _out_tensor(out, n, chunk_index)
    st = _lib.load().aipstack_chksum_batch_chain_fill(
        chunk_addr.data_ptr(), chunk_len.data_ptr(), chunk_index.data_ptr(), sp or None,
        fields.data_ptr(), n, out.data_ptr(),
        (AIPSTACK_CHKSUM_ZERO_AS_FFFF if zero_as_ffff else 0) |
        (AIPSTACK_CHKSUM_JUST_WRITTEN if just_written else 0),
        _stream_handle(stream, chunk_index))
    _check(st, "aipstack_chksum_batch_chain_fill")
    return out


def _u8_out(out, n, like):
    torch = _torch()
    if out is None:
        return torch.empty(n, dtype=torch.uint8, device=like.device)
    _require_device(out, "out")
    if out.element_size() != 1 or out.numel() < n:
        raise ValueError("out must be a uint8 device tensor with >= n elements")
    _same_device(out, like, "out and frames")
    return out


def rx_verify(frames, offsets, *, out=None, stream=None):
    """Rx verify on the GPU: frame i = ``frames[offsets[i]:offsets[i+1]]`` (raw Ethernet);
    returns one AIPSTACK_RX_* verdict per frame (uint8 device tensor). Read-only."""
    _require_device(frames, "frames")
    _require_offsets(offsets)
    _same_device(frames, offsets, "frames and offsets")
    n = offsets.numel() - 1
    out = _u8_out(out, max(n, 0), frames)
    _check(_lib.load().aipstack_chksum_rx_verify(frames.data_ptr(), offsets.data_ptr(), n,
                                                 out.data_ptr(), _stream_handle(stream, frames)),
           "aipstack_chksum_rx_verify")
    return out


def tx_fill(frames, offsets, *, out=None, stream=None, split=None, workspace=None):
    """Tx fill on the GPU, IN PLACE: writes the IPv4 header checksum and the TCP / UDP /
    ICMP checksum of every frame; returns one status per frame (AIPSTACK_RX_* codes).

    ``split=True`` runs the two-pass ``aipstack_chksum_tx_fill_split`` with a workspace of
    8 bytes per frame (``workspace``: a device tensor of at least that many bytes, else one
    is taken from torch's allocator); ``split=False`` the one-pass
    ``aipstack_chksum_tx_fill``; ``None`` (default) the one pass, the faster at every batch
    size measured (round 5, driver protocol, 1 M frames: 193.4 against 194.5 us on rotated
    batches, 159.8 against 161.6 on one buffer, profiles/r05/txrot, txsplit; round 2: 57
    against 61 us at 256 K). Both write the same bytes."""
    _require_device(frames, "frames")
    _require_offsets(offsets)
    _same_device(frames, offsets, "frames and offsets")
    n = offsets.numel() - 1
    out = _u8_out(out, max(n, 0), frames)
    lib = _lib.load()
    if split is None:
        split = False
    if not split:
        _check(lib.aipstack_chksum_tx_fill(frames.data_ptr(), offsets.data_ptr(), n,
                                           out.data_ptr(), _stream_handle(stream, frames)),
               "aipstack_chksum_tx_fill")
        return out
    _split_call(lib, "aipstack_chksum_tx_fill_split", frames, n, stream, workspace,
                lambda ws, ws_bytes, h: (frames.data_ptr(), offsets.data_ptr(), n,
                                         out.data_ptr(), ws, ws_bytes, h))
    return out


def _split_call(lib, name, frames, n, stream, workspace, args):
    """A split Tx fill (read pass + scatter pass through a workspace of 8 bytes per frame):
    ``args(workspace_ptr, workspace_bytes, stream_handle)`` gives the entry point's arguments."""
    torch = _torch()
    need = int(lib.aipstack_chksum_tx_fill_workspace_bytes(max(n, 0)))
    if workspace is None:
        workspace = torch.empty(max(need, 8), dtype=torch.uint8, device=frames.device)
    else:
        _require_device(workspace, "workspace")
        _same_device(frames, workspace, "frames and workspace")
    ws_bytes = workspace.numel() * workspace.element_size()
    launch_stream = torch.cuda.current_stream(frames.device) if stream is None else stream
    if not hasattr(launch_stream, "cuda_stream"):  # a raw hipStream_t handle
        launch_stream = torch.cuda.ExternalStream(int(launch_stream), device=frames.device)
    _check(getattr(lib, name)(*args(workspace.data_ptr(), ws_bytes,
                                    _stream_handle(launch_stream))), name)
    # The caching allocator must not hand the workspace out again before both passes on
    # the launch stream are done with it (it may not be torch's current stream).
    workspace.record_stream(launch_stream)


def tx_fill_records(frames, offsets, *, out=None, stream=None):
    """The split Tx fill's read pass alone (``aipstack_chksum_tx_fill_records``): one 8-byte
    record per frame, nothing written into the frames. Record i = ``w0 | w1 << 32`` with
    ``w0`` = IPv4 header checksum | L4 checksum << 16 and ``w1`` = L4 field offset (bits
    0-7) | write the IPv4 field (8) | write the L4 field (9) | status (16-23); the host
    applies them (:func:`apply_tx_records`). Returns the records (int64 device tensor)."""
    torch = _torch()
    _require_device(frames, "frames")
    _require_offsets(offsets)
    _same_device(frames, offsets, "frames and offsets")
    n = max(offsets.numel() - 1, 0)
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=frames.device)
    else:
        _require_device(out, "out")
        if out.element_size() != 8 or out.numel() < n:
            raise ValueError("out must be a 64-bit device tensor with >= n elements")
        _same_device(out, frames, "out and frames")
    _check(_lib.load().aipstack_chksum_tx_fill_records(frames.data_ptr(), offsets.data_ptr(), n,
                                                       out.data_ptr(), _stream_handle(stream, frames)),
           "aipstack_chksum_tx_fill_records")
    return out


def slots_to_offsets(n: int, slot_stride: int) -> np.ndarray:
    """Frame start offsets of n ring slots (for :func:`apply_tx_records`): i * slot_stride."""
    return np.arange(n + 1, dtype=np.uint64) * np.uint64(slot_stride)


def apply_tx_records(frames: np.ndarray, offsets: np.ndarray, records: np.ndarray,
                     status: Optional[np.ndarray] = None) -> np.ndarray:
    """Apply Tx fill records (:func:`tx_fill_records`) to frames in HOST memory (numpy, in
    place), as the engine's completion does: the IPv4 header checksum big-endian at frame
    byte 24, the L4 checksum at the record's field offset, each when its flag is set.
    Returns the per-frame statuses (uint8)."""
    rec = np.ascontiguousarray(records).view(np.uint64)
    o = np.ascontiguousarray(offsets, dtype=np.uint64)[:rec.size]
    w0 = (rec & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    w1 = (rec >> np.uint64(32)).astype(np.uint32)
    if status is None:
        status = np.empty(rec.size, dtype=np.uint8)
    status[:rec.size] = (w1 >> 16) & 0xFF
    flat = frames.reshape(-1).view(np.uint8)
    for flag, at, val in ((0x100, o + np.uint64(24), w0 & 0xFFFF),
                          (0x200, o + (w1 & 0xFF).astype(np.uint64), w0 >> 16)):
        sel = (w1 & flag) != 0
        a = at[sel].astype(np.int64)
        v = val[sel]
        flat[a] = (v >> 8).astype(np.uint8)
        flat[a + 1] = (v & 0xFF).astype(np.uint8)
    return status


RX_VERDICTS = {0: "NOT_IP4", 1: "DROP_IP_MALFORMED", 2: "DROP_IP_CHKSUM", 3: "FRAGMENT",
               4: "DROP_L4_MALFORMED", 5: "DROP_L4_CHKSUM", 6: "ACCEPT",
               7: "ACCEPT_NO_CHKSUM", 8: "ACCEPT_OTHER"}


def flatten_chains(refs, host_base: np.ndarray, device_base: int):
    """Flatten IpBufRef chains whose nodes point into `host_base` (a numpy byte array
    mirrored on the device at `device_base`) into the chunk table of
    :func:`chksum_batch_chain`: the non-empty chunks ipBufProcessBytes visits
    (BufUtils.h:129-178), translated to device addresses. Returns numpy
    (addr uint64, len uint32, index uint64)."""
    base_ptr = host_base.ctypes.data
    addrs, lens, index = [], [], [0]
    for ref in refs:
        if ref.tot_len > 0:
            def visit(mv, n):
                ptr = np.frombuffer(mv, dtype=np.uint8).ctypes.data
                if not base_ptr <= ptr < base_ptr + host_base.nbytes:
                    raise ValueError("chain node outside host_base")
                addrs.append(device_base + (ptr - base_ptr))
                lens.append(n)
                return n
            ipBufProcessBytes(ref, ref.tot_len, visit)
        index.append(len(addrs))
    return (np.array(addrs, dtype=np.uint64), np.array(lens, dtype=np.uint32),
            np.array(index, dtype=np.uint64))


VIOLATION_PACKET_LEN = 1
VIOLATION_CHUNK_LEN = 2
VIOLATION_SPAN = 4


def contract_violations(device: int = 0, clear: bool = True) -> int:
    """Sticky contract-violation bits (VIOLATION_*) the kernels met on `device` since the
    last clear (``aipstack_chksum_contract_violations``; waits for the device to go idle)."""
    m = ctypes.c_uint32(0)
    _check(_lib.load().aipstack_chksum_contract_violations(device, ctypes.byref(m), int(clear)),
           "aipstack_chksum_contract_violations")
    return int(m.value)


def device_check(device: int = 0) -> int:
    """AIPSTACK_CHKSUM_OK if `device` is a gfx950 device the library can launch on."""
    return int(_lib.load().aipstack_chksum_device_check(device))
