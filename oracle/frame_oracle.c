/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle for the frame-level rows of SURVEY.md 8(f):
 *   row 2  batched Rx verify of raw Ethernet frames (the checksum decisions the
 *          reference's receive path makes), and
 *   row 3  batched Tx fill (the checksums the reference's send paths write).
 * Restated from the reference source (cited per check); the checksum arithmetic itself is
 * chksum_oracle.c (pinned against the reference's own Chksum.h by tests/golden/).
 *
 * A frame is one contiguous buffer as the TAP driver delivers it (one IpBufNode,
 * tap/linux/TapDeviceLinux.cpp:172-178), so every hasHeader() check of the reference is
 * a length check on that buffer.
 */
#include <stddef.h>
#include <stdint.h>

#include "chksum_oracle.h"
#include "frame_oracle.h"

static inline uint32_t rd8(const uint8_t *p) { return p[0]; }
static inline uint32_t rd16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static inline uint32_t rd32(const uint8_t *p) { return (rd16(p) << 16) | rd16(p + 2); }
static inline void wr16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* IpChksumAccumulator with header words then getChksum(IpBufRef{one buffer})
 * (Chksum.h:191-217 addWord without carry, :263-315 one chunk, :245-250 fold + invert). */
static uint16_t accum_chksum(uint32_t words_sum, const uint8_t *data, size_t len)
{
    const void *p = data;
    return oracle_chksum_chain(words_sum, &p, &len, len ? 1 : 0);
}

/* TCP/UDP pseudo-header words: addWord32(src), addWord32(dst), addWord16(proto),
 * addWord16(len) (tcp/IpTcpProto_input.h:93-97, udp/IpUdpProto.h:640-643). */
static uint32_t pseudo(uint32_t src, uint32_t dst, uint32_t proto, uint32_t len)
{
    return (src >> 16) + (src & 0xFFFF) + (dst >> 16) + (dst & 0xFFFF) + proto + (len & 0xFFFF);
}

struct parsed {
    uint32_t hl, total_len, flags_off, proto, src, dst;
};

/* Ethernet + IPv4 header checks of EthIpIface::recvFrame (eth/EthIpIface.h:367-390) and
 * IpStack::processRecvedIp4Packet (ip/IpStack.h:936-990). Returns -1 when the frame is an
 * IPv4 packet with a sane header, else the verdict (>= 0). */
static int parse_ip4(const uint8_t *f, size_t len, struct parsed *ps)
{
    if (len < 14)                                   /* hasHeader(EthHeader::Size) :370 */
        return AIPSTACK_RX_NOT_IP4;
    if (rd16(f + 12) != 0x0800)                     /* EthType::Ipv4 :383 */
        return AIPSTACK_RX_NOT_IP4;
    const uint8_t *ip = f + 14;
    const size_t plen = len - 14;
    if (plen < 20)                                  /* IpStack.h:939 */
        return AIPSTACK_RX_DROP_IP_MALFORMED;
    const uint32_t vihl = rd8(ip);
    uint32_t hl;
    if (vihl == 0x45) {                             /* :959 fast path */
        hl = 20;
    } else {
        if ((vihl >> 4) != 4)                       /* :965 */
            return AIPSTACK_RX_DROP_IP_MALFORMED;
        hl = (vihl & 0xF) * 4;                      /* :971 */
        if (hl < 20 || hl > plen)                   /* :972-976 */
            return AIPSTACK_RX_DROP_IP_MALFORMED;
    }
    const uint32_t total_len = rd16(ip + 2);
    if (total_len < hl || total_len > plen)         /* :988 */
        return AIPSTACK_RX_DROP_IP_MALFORMED;
    ps->hl = hl;
    ps->total_len = total_len;
    ps->flags_off = rd16(ip + 6);
    ps->proto = rd8(ip + 9);
    ps->src = rd32(ip + 12);
    ps->dst = rd32(ip + 16);
    return -1;
}

/* Sum of the header's 16-bit words, skipping the word at `skip_off` (or none if >= hl):
 * the addWord/addEvenBytes sequence of IpStack.h:950-1013 (receive) / :425-453 (send). */
static uint32_t header_words(const uint8_t *ip, uint32_t hl, uint32_t skip_off)
{
    uint32_t s = 0;
    for (uint32_t o = 0; o < hl; o += 2)
        if (o != skip_off)
            s += rd16(ip + o);
    return s;
}

static uint16_t fold_not(uint32_t s)
{
    s = (s & 0xFFFF) + (s >> 16);
    s = (s & 0xFFFF) + (s >> 16);
    return (uint16_t)~s;
}

int oracle_rx_verify(const void *frame, size_t len)
{
    const uint8_t *f = (const uint8_t *)frame;
    struct parsed ps;
    int v = parse_ip4(f, len, &ps);
    if (v >= 0)
        return v;
    const uint8_t *ip = f + 14;
    if (fold_not(header_words(ip, ps.hl, 0xFFFFFFFFu)) != 0)   /* :1016 */
        return AIPSTACK_RX_DROP_IP_CHKSUM;
    if ((ps.flags_off & 0x3FFF) != 0)               /* MF | OffsetMask :1020 */
        return AIPSTACK_RX_FRAGMENT;                /* -> host reassembly :1022-1043 */
    const uint8_t *dg = ip + ps.hl;
    const uint32_t dlen = ps.total_len - ps.hl;     /* pkt.hideHeader().subTo() :993 */
    switch (ps.proto) {
    case 6:                                         /* TCP, tcp/IpTcpProto_input.h:68-100 */
        if (dlen < 20)                              /* :77 hasHeader(Tcp4Header::Size) */
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        if (accum_chksum(pseudo(ps.src, ps.dst, 6, dlen), dg, dlen) != 0)   /* :93-100 */
            return AIPSTACK_RX_DROP_L4_CHKSUM;
        return AIPSTACK_RX_ACCEPT;
    case 17: {                                      /* UDP, udp/IpUdpProto.h:470-490 */
        if (dlen < 8)                               /* :473 */
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        const uint32_t ulen = rd16(dg + 4);
        if (ulen < 8 || ulen > dlen)                /* :484-489 */
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        if (rd16(dg + 6) == 0)                      /* has_checksum = false :637-639 */
            return AIPSTACK_RX_ACCEPT_NO_CHKSUM;
        if (accum_chksum(pseudo(ps.src, ps.dst, 17, ulen), dg, ulen) != 0)  /* :640-648 */
            return AIPSTACK_RX_DROP_L4_CHKSUM;
        return AIPSTACK_RX_ACCEPT;
    }
    case 1:                                         /* ICMP, ip/IpStack.h:1093-1130 */
        if (dlen < 8)                               /* :1113 hasHeader(Icmp4Header::Size) */
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        if (accum_chksum(0, dg, dlen) != 0)         /* IpChksum(dgram) :1126-1129 */
            return AIPSTACK_RX_DROP_L4_CHKSUM;
        return AIPSTACK_RX_ACCEPT;
    default:
        return AIPSTACK_RX_ACCEPT_OTHER;
    }
}

int oracle_tx_fill(void *frame, size_t len)
{
    uint8_t *f = (uint8_t *)frame;
    struct parsed ps;
    int v = parse_ip4(f, len, &ps);
    if (v >= 0)
        return v;
    uint8_t *ip = f + 14;
    /* IPv4 header checksum over the header words with the checksum field as 0
     * (ip/IpStack.h:425-453 computes it over the fields it writes; options included). */
    wr16(ip + 10, fold_not(header_words(ip, ps.hl, 10)));
    if ((ps.flags_off & 0x3FFF) != 0)               /* a fragment: the L4 checksum covers */
        return AIPSTACK_RX_FRAGMENT;                /* the whole datagram, not this piece */
    uint8_t *dg = ip + ps.hl;
    const uint32_t dlen = ps.total_len - ps.hl;
    switch (ps.proto) {
    case 6: {                                       /* tcp/IpTcpProto_output.h:1251-1277 */
        if (dlen < 20)
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        wr16(dg + 16, 0);
        wr16(dg + 16, accum_chksum(pseudo(ps.src, ps.dst, 6, dlen), dg, dlen));
        return AIPSTACK_RX_ACCEPT;
    }
    case 17: {                                      /* udp/IpUdpProto.h:152-184 */
        if (dlen < 8)
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        const uint32_t ulen = rd16(dg + 4);
        if (ulen < 8 || ulen > dlen)
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        wr16(dg + 6, 0);
        uint16_t c = accum_chksum(pseudo(ps.src, ps.dst, 17, ulen), dg, ulen);
        wr16(dg + 6, c == 0 ? 0xFFFF : c);          /* :176-178 */
        return AIPSTACK_RX_ACCEPT;
    }
    case 1: {                                       /* ip/IpStack.h:1164-1190 */
        if (dlen < 8)
            return AIPSTACK_RX_DROP_L4_MALFORMED;
        wr16(dg + 2, 0);
        wr16(dg + 2, accum_chksum(0, dg, dlen));
        return AIPSTACK_RX_ACCEPT;
    }
    default:
        return AIPSTACK_RX_ACCEPT_OTHER;
    }
}

void oracle_rx_verify_batch(const void *base, const uint64_t *offsets, uint64_t n,
                            uint8_t *verdict)
{
    const uint8_t *b = (const uint8_t *)base;
    for (uint64_t i = 0; i < n; i++)
        verdict[i] = (uint8_t)oracle_rx_verify(b + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
}

void oracle_tx_fill_batch(void *base, const uint64_t *offsets, uint64_t n, uint8_t *status)
{
    uint8_t *b = (uint8_t *)base;
    for (uint64_t i = 0; i < n; i++)
        status[i] = (uint8_t)oracle_tx_fill(b + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
}

/* Ring slots: frame i = the lens[i] bytes at base + i * stride. */
void oracle_rx_verify_slotted(const void *base, uint64_t stride, const uint32_t *lens,
                              uint64_t n, uint8_t *verdict)
{
    const uint8_t *b = (const uint8_t *)base;
    for (uint64_t i = 0; i < n; i++)
        verdict[i] = (uint8_t)oracle_rx_verify(b + i * stride, lens[i]);
}

void oracle_tx_fill_slotted(void *base, uint64_t stride, const uint32_t *lens, uint64_t n,
                            uint8_t *status)
{
    uint8_t *b = (uint8_t *)base;
    for (uint64_t i = 0; i < n; i++)
        status[i] = (uint8_t)oracle_tx_fill(b + i * stride, lens[i]);
}
