"""TEST INFRASTRUCTURE -- deterministic edge-case frames for the Rx-verify / Tx-fill parity
tests: the GPU kernels against oracle/frame_oracle.c.

`frames(seed, n)` builds n Ethernet frames: TCP (with and without options, SYN/ACK/FIN
mixes), UDP, ICMP echo and other ICMP types, and protocols without a checksum here; IPv4
headers with and without options; Ethernet padding and trailing bytes beyond total_len;
L4 payloads crafted so the checksum sum is 0 mod 0xFFFF (both zero representations in
the field). A fraction then gets one mutation (header fields, lengths, checksums,
fragments, ethertype, truncation), so every Rx verdict code occurs.

Only `random.Random(seed).getrandbits` is used (a stable Mersenne Twister stream).
"""
import random
import struct

LOCAL_IP = bytes([10, 20, 30, 40])     # destination of every frame
LOCAL_MAC = bytes([0x02, 0x00, 0x5E, 0x10, 0x20, 0x30])
NUM_PEERS = 4
SYN_PORT = 80


def peer_ip(i):
    return bytes([10, 20, 30, 100 + i])


def peer_mac(i):
    return bytes([0x02, 0x11, 0x22, 0x33, 0x44, 0x50 + i])


class _Rng:
    def __init__(self, seed):
        self._r = random.Random(seed)

    def below(self, n):
        """uniform in [0, n) from getrandbits only (rejection sampling)"""
        if n <= 1:
            return 0
        b = (n - 1).bit_length()
        while True:
            v = self._r.getrandbits(b)
            if v < n:
                return v

    def span(self, lo, hi):
        return lo + self.below(hi - lo + 1)

    def chance(self, num, den):
        return self.below(den) < num

    def bytes(self, n):
        return bytes(self._r.getrandbits(8) for _ in range(n))

    def pick(self, seq):
        return seq[self.below(len(seq))]


def be_sum(data):
    """sum of big-endian 16-bit words (odd tail byte as a high byte); plain integer"""
    if len(data) & 1:
        data = data + b"\0"
    return sum(struct.unpack(">%dH" % (len(data) // 2), data))


def chksum(data, extra=0):
    s = be_sum(data) + extra
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def _pseudo(src, dst, proto, length):
    return be_sum(src) + be_sum(dst) + proto + length


def _ip_header(rng, src, proto, payload_len, ihl=5, flags_off=0x4000):
    opts = b""
    if ihl > 5:
        # option bytes: NOP/EOL and random filler (the receive path only sums them)
        opts = bytes(rng.pick([0x01, 0x00, rng.below(256)]) for _ in range(4 * (ihl - 5)))
    h = bytearray(struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, rng.below(256),
                              4 * ihl + payload_len, rng.below(65536), flags_off,
                              rng.span(1, 255), proto, 0, src, LOCAL_IP)) + opts
    struct.pack_into(">H", h, 10, chksum(bytes(h)))
    return h


def _fix_ip_chksum(frame):
    ihl = (frame[14] & 0xF) * 4
    struct.pack_into(">H", frame, 24, 0)
    struct.pack_into(">H", frame, 24, chksum(bytes(frame[14:14 + ihl])))


def _craft_zero_sum(l4, csum_off, extra):
    """Adjust one even-aligned payload word so the L4 sum (with the checksum field 0) is
    == 0 mod 0xFFFF: the computed checksum is then 0x0000, and 0xFFFF verifies as well."""
    for w in range((len(l4) - 2) & ~1, csum_off + 1, -2):
        t = bytearray(l4)
        struct.pack_into(">H", t, csum_off, 0)
        s = (be_sum(bytes(t)) + extra) % 0xFFFF
        old = struct.unpack_from(">H", t, w)[0]
        struct.pack_into(">H", t, w, (old - s) % 0xFFFF)
        return t
    return bytearray(l4)


def _tcp(rng, dst_port, flags, payload, opts=b""):
    doff = 5 + len(opts) // 4
    h = bytearray(struct.pack(">HHIIHHHH", rng.span(1024, 65535), dst_port, rng.below(1 << 32),
                              rng.below(1 << 32), (doff << 12) | flags, rng.span(0, 65535), 0,
                              0)) + opts + payload
    return h, 16, 6


def _build(rng, peer):
    """one valid frame: (frame, kind, L4 checksum offset in the frame or -1, L4 offset,
    protocol)"""
    src = peer_ip(peer)
    kind = rng.below(100)
    craft = rng.chance(1, 12)
    if kind < 40:                                       # TCP
        if rng.chance(1, 4):
            flags = rng.pick([0x02, 0x02, 0x10, 0x18])   # SYN or ACK to a service port
            dport = SYN_PORT
        else:
            flags = rng.pick([0x10, 0x18, 0x11, 0x02, 0x00, 0x12, 0x29, 0x04])
            dport = rng.span(1, 65535)
            if dport == SYN_PORT:
                dport += 1
        opts = b""
        r = rng.below(4)
        if r == 1:
            opts = struct.pack(">BBH", 2, 4, rng.span(200, 1460))            # MSS
        elif r == 2:
            opts = struct.pack(">BBHBBBB", 2, 4, 1460, 1, 3, 3, rng.below(15))  # MSS, NOP, WS
        elif r == 3:
            opts = bytes([1]) * 4 * rng.span(1, 10)
        payload = rng.bytes(rng.pick([0, 0, rng.span(1, 64), rng.span(1, 1400)]))
        if len(opts) + 20 + len(payload) > 1480:
            payload = payload[:1480 - 20 - len(opts)]
        l4, coff, proto = _tcp(rng, dport, flags, payload, opts)
        cat = "tcp"
    elif kind < 70:                                     # UDP
        payload = rng.bytes(rng.pick([0, rng.span(1, 32), rng.span(1, 1472)]))
        l4 = bytearray(struct.pack(">HHHH", rng.span(1, 65535), rng.span(1, 65535),
                                   8 + len(payload), 0)) + payload
        coff, proto, cat = 6, 17, "udp"
    elif kind < 90:                                     # ICMP echo request
        payload = rng.bytes(rng.pick([0, rng.span(1, 56), rng.span(1, 1472)]))
        l4 = bytearray(struct.pack(">BBHHH", 8, 0, 0, rng.below(65536), rng.below(65536))) + payload
        coff, proto, cat = 2, 1, "icmp_echo"
    elif kind < 95:                                     # other ICMP types
        payload = rng.bytes(rng.span(0, 200))
        l4 = bytearray(struct.pack(">BBHI", rng.pick([0, 13, 14, 17, 30]), 0, 0,
                                   rng.below(1 << 32))) + payload
        coff, proto, cat = 2, 1, "icmp_other"
    else:                                               # a protocol without a checksum here
        l4 = bytearray(rng.bytes(rng.span(0, 600)))
        coff, proto, cat = -1, rng.pick([47, 50, 132, 255, 2]), "other"
    if coff >= 0:
        extra = _pseudo(src, LOCAL_IP, proto, len(l4)) if proto in (6, 17) else 0
        if craft and len(l4) >= coff + 6:
            l4 = _craft_zero_sum(l4, coff, extra)
        struct.pack_into(">H", l4, coff, 0)
        c = chksum(bytes(l4), extra)
        if proto == 17 and rng.chance(1, 10):
            c = 0                                       # UDP without a checksum
        elif proto == 17 and c == 0:
            c = 0xFFFF                                  # udp/IpUdpProto.h:176-178
        elif craft and c == 0 and rng.chance(1, 2):
            c = 0xFFFF                                  # the other zero, must verify too
        struct.pack_into(">H", l4, coff, c)
    ihl = 5 if rng.chance(4, 5) else rng.span(6, 15)
    ip = _ip_header(rng, src, proto, len(l4), ihl=ihl,
                    flags_off=rng.pick([0x4000, 0x0000, 0x4000]))
    frame = bytearray(LOCAL_MAC + peer_mac(peer) + b"\x08\x00") + ip + l4
    if len(frame) < 60:
        frame += rng.bytes(60 - len(frame)) if rng.chance(1, 2) else bytes(60 - len(frame))
    elif rng.chance(1, 10):
        frame += rng.bytes(rng.span(1, 20))             # trailing bytes beyond total_len
    l4_off = 14 + 4 * ihl
    return frame, cat, (l4_off + coff) if coff >= 0 else -1, l4_off, proto


MUTATIONS = ["l4_byte", "l4_chk", "ip_chk", "ip_ver", "ihl_small", "ihl_big", "tot_big",
             "tot_small", "tot_trunc", "udp_len", "frag", "ethertype", "short", "alt_zero"]


def _mutate(rng, frame, m, l4_chk_off, l4_off, proto):
    hl = (frame[14] & 0xF) * 4
    if m == "l4_byte" and len(frame) > l4_off:
        end = 14 + struct.unpack_from(">H", frame, 16)[0]
        if end > l4_off:
            frame[rng.span(l4_off, end - 1)] ^= 1 << rng.below(8)
    elif m == "l4_chk" and l4_chk_off >= 0:
        frame[l4_chk_off + rng.below(2)] ^= 1 << rng.below(8)
    elif m == "ip_chk":
        frame[24 + rng.below(2)] ^= 1 << rng.below(8)
        return
    elif m == "ip_ver":
        frame[14] = (rng.pick([0, 6, 5, 15]) << 4) | (frame[14] & 0xF)
    elif m == "ihl_small":
        frame[14] = 0x40 | rng.below(5)
    elif m == "ihl_big":
        # IHL past the frame (truncate the frame to just after the base header)
        frame[14] = 0x4F
        del frame[14 + 20 + rng.below(40):]
    elif m == "tot_big":
        struct.pack_into(">H", frame, 16, len(frame) - 14 + rng.span(1, 100))
    elif m == "tot_small":
        struct.pack_into(">H", frame, 16, rng.below(hl))
    elif m == "tot_trunc":
        tot = struct.unpack_from(">H", frame, 16)[0]
        struct.pack_into(">H", frame, 16, rng.span(hl, max(hl, tot - 1)))
    elif m == "udp_len" and proto == 17 and len(frame) >= l4_off + 8:
        dlen = struct.unpack_from(">H", frame, 16)[0] - hl
        struct.pack_into(">H", frame, l4_off + 4,
                         rng.pick([rng.below(8), dlen + rng.span(1, 50), max(8, dlen - rng.span(1, 8))]))
    elif m == "frag":
        struct.pack_into(">H", frame, 20, rng.pick([0x2000, 0x2000 | rng.span(1, 100),
                                                    rng.span(1, 0x1FFF)]))
    elif m == "ethertype":
        struct.pack_into(">H", frame, 12, rng.pick([0x86DD, 0x8100, 0x88CC, 0x0801]))
        return
    elif m == "short":
        del frame[rng.below(34):]
        return
    elif m == "alt_zero" and l4_chk_off >= 0:
        c = struct.unpack_from(">H", frame, l4_chk_off)[0]
        if c in (0, 0xFFFF):
            struct.pack_into(">H", frame, l4_chk_off, c ^ 0xFFFF)
        return
    _fix_ip_chksum(frame)


def frames(seed=20251015, n=3000):
    rng = _Rng(seed)
    out = []
    for _ in range(n):
        peer = rng.below(NUM_PEERS)
        frame, _, l4_chk_off, l4_off, proto = _build(rng, peer)
        if rng.chance(2, 5) and len(frame) >= 34:
            _mutate(rng, frame, MUTATIONS[rng.below(len(MUTATIONS))], l4_chk_off, l4_off, proto)
        out.append(bytes(frame))
    return out


def pack(frs):
    """frames -> (uint8 numpy buffer, uint64 CSR offsets of n+1 entries), back to back"""
    import numpy as np
    offs = np.zeros(len(frs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(fr) for fr in frs])
    buf = np.frombuffer(b"".join(frs) or b"\0", dtype=np.uint8).copy()
    return buf, offs
