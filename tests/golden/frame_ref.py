"""TEST INFRASTRUCTURE -- reference-produced answers for the frame-level rows (SURVEY.md 8(f)
rows 2-3), composed from the reference's OWN checksum call sites.

`oracle/_ref/libref_chksum.so` exports the stack's checksum call sequences compiled against
the reference's Chksum.h/Buf.h (tests/cpp/call_sites.inc, `ref_cs_*`):
  ref_cs_ip4_rx  ip/IpStack.h:936-1018  IPv4 header checks + header checksum (getChksum())
  ref_cs_tcp_rx  tcp/IpTcpProto_input.h:92-100  pseudo-header + segment
  ref_cs_udp_rx  udp/IpUdpProto.h:631-652  verifyChecksum (bit 0 verified, bit 1 has_checksum)
  ref_cs_udp_tx  udp/IpUdpProto.h:169-179  pseudo-header + datagram, 0 -> 0xFFFF
  ref_cs_icmp    ip/IpStack.h:1127  IpChksum(dgram)
`reference_values` runs them per frame (the send side on a copy with the field set to 0, as
the reference sums before it writes) and records every value; the stack itself is not run
(its harness was denied in round 1). What stays restated is only the
glue between the calls: the Ethernet type test (eth/EthIpIface.h:367-390), the fragment test
(ip/IpStack.h:1020) and the TCP/UDP/ICMP length tests (tcp/IpTcpProto_input.h:77,
udp/IpUdpProto.h:473-489, ip/IpStack.h:1113) -- `verdict` and `fill_fields` below.

Record per frame (ints, -1 = not reached):
  [ip4_rx, ip4_fill, l4_rx, l4_fill]
  ip4_rx    ref_cs_ip4_rx on the frame: -1 = header dropped before its checksum test, else
            getChksum() (0 = header checksum good)
  ip4_fill  ref_cs_ip4_rx with the header checksum field 0: the value the send side writes
  l4_rx     TCP/ICMP: the getChksum value (0 = good); UDP: verifyChecksum's bits
  l4_fill   the L4 checksum the send side writes (UDP: 0 sent as 0xFFFF)
"""
import ctypes

import numpy as np

VP, SZ = ctypes.c_void_p, ctypes.c_size_t


def load(path):
    lib = ctypes.CDLL(path)
    chain = [ctypes.POINTER(VP), ctypes.POINTER(SZ), SZ, SZ, SZ]
    lib.ref_cs_ip4_rx.restype = ctypes.c_int
    lib.ref_cs_ip4_rx.argtypes = chain + [ctypes.POINTER(SZ)]
    lib.ref_cs_tcp_rx.restype = ctypes.c_uint16
    lib.ref_cs_tcp_rx.argtypes = [ctypes.c_uint32, ctypes.c_uint32] + chain
    lib.ref_cs_udp_rx.restype = ctypes.c_int
    lib.ref_cs_udp_rx.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16] + chain
    lib.ref_cs_udp_tx.restype = ctypes.c_uint16
    lib.ref_cs_udp_tx.argtypes = [ctypes.c_uint32, ctypes.c_uint32] + chain
    lib.ref_cs_icmp.restype = ctypes.c_uint16
    lib.ref_cs_icmp.argtypes = chain
    return lib


def _be16(b, o):
    return (int(b[o]) << 8) | int(b[o + 1])


def _be32(b, o):
    return (_be16(b, o) << 16) | _be16(b, o + 2)


def _one(arr, off, length):
    """(ptrs, lens, nchunks, offset, tot_len) of one IpBufNode over arr[off:off+length]"""
    ptrs = (VP * 1)(arr.ctypes.data + off)
    lens = (SZ * 1)(length)
    return ptrs, lens, 1, 0, length


def _l4_shape(f):
    """(proto, hl, dlen, l4 length the checksum covers, field offset in the dgram) after the
    IPv4 header passed; None where a restated length test drops the datagram."""
    hl = (int(f[14]) & 15) * 4
    total = _be16(f, 16)
    proto = int(f[23])
    dlen = total - hl
    dg = 14 + hl
    if proto == 6:
        return (6, hl, dlen, dlen, 16) if dlen >= 20 else None
    if proto == 17:
        if dlen < 8:
            return None
        ulen = _be16(f, dg + 4)
        return (17, hl, dlen, ulen, 6) if 8 <= ulen <= dlen else None
    if proto == 1:
        return (1, hl, dlen, dlen, 2) if dlen >= 8 else None
    return (proto, hl, dlen, 0, -1)


def reference_values(lib, buf, offsets):
    """The record above for every frame buf[offsets[i]:offsets[i+1]]."""
    out = []
    for i in range(offsets.size - 1):
        s, e = int(offsets[i]), int(offsets[i + 1])
        f = np.ascontiguousarray(buf[s:e])
        rec = [-1, -1, -1, -1]
        if f.size < 14 or _be16(f, 12) != 0x0800:
            out.append(rec)
            continue
        dl = SZ(0)
        rec[0] = lib.ref_cs_ip4_rx(*_one(f, 14, f.size - 14), ctypes.byref(dl))
        if rec[0] < 0:
            out.append(rec)
            continue
        z = f.copy()
        z[24:26] = 0
        rec[1] = lib.ref_cs_ip4_rx(*_one(z, 14, z.size - 14), ctypes.byref(SZ(0)))
        shape = _l4_shape(f)
        frag = (_be16(f, 20) & 0x3FFF) != 0
        if frag or shape is None or shape[4] < 0:
            out.append(rec)
            continue
        proto, hl, dlen, cover, fo = shape
        dg = 14 + hl
        src, dst = _be32(f, 26), _be32(f, 30)
        zl = f.copy()
        zl[dg + fo:dg + fo + 2] = 0
        if proto == 6:
            rec[2] = lib.ref_cs_tcp_rx(src, dst, *_one(f, dg, cover))
            rec[3] = lib.ref_cs_tcp_rx(src, dst, *_one(zl, dg, cover))
        elif proto == 17:
            rec[2] = lib.ref_cs_udp_rx(src, dst, _be16(f, dg + 6), *_one(f, dg, cover))
            rec[3] = lib.ref_cs_udp_tx(src, dst, *_one(zl, dg, cover))
        else:
            rec[2] = lib.ref_cs_icmp(*_one(f, dg, cover))
            rec[3] = lib.ref_cs_icmp(*_one(zl, dg, cover))
        out.append([int(x) for x in rec])
    return out


# AIPSTACK_RX_* (include/aipstack_amd/chksum.h)
NOT_IP4, DROP_IP_MALFORMED, DROP_IP_CHKSUM, FRAGMENT, DROP_L4_MALFORMED, DROP_L4_CHKSUM, \
    ACCEPT, ACCEPT_NO_CHKSUM, ACCEPT_OTHER = range(9)


def verdict(frame, rec):
    """The Rx verdict from the reference's recorded answers plus the restated glue."""
    f = frame
    if f.size < 14 or _be16(f, 12) != 0x0800:
        return NOT_IP4
    ip4_rx, _, l4_rx, _ = rec
    if ip4_rx < 0:
        return DROP_IP_MALFORMED
    if ip4_rx != 0:
        return DROP_IP_CHKSUM
    if (_be16(f, 20) & 0x3FFF) != 0:
        return FRAGMENT
    shape = _l4_shape(f)
    if shape is None:
        return DROP_L4_MALFORMED
    if shape[4] < 0:
        return ACCEPT_OTHER
    if shape[0] == 17:
        if l4_rx & 1 == 0:
            return DROP_L4_CHKSUM
        return ACCEPT if l4_rx & 2 else ACCEPT_NO_CHKSUM
    return ACCEPT if l4_rx == 0 else DROP_L4_CHKSUM


def fill_fields(frame, rec):
    """[(frame offset, value)] the send side writes, from the recorded answers: the IPv4
    header checksum at 24 and the L4 checksum at its field."""
    _, ip4_fill, _, l4_fill = rec
    out = []
    if ip4_fill >= 0:
        out.append((24, ip4_fill))
        shape = _l4_shape(frame)
        if l4_fill >= 0 and shape is not None and shape[4] >= 0:
            out.append((14 + shape[1] + shape[4], l4_fill))
    return out
