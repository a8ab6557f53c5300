// aipstack_amd -- frame-level batch kernels on raw Ethernet frames:
//   Rx verify: the reference's receive-path checksum decisions for n frames at once
//              (eth/EthIpIface.h:367-390, ip/IpStack.h:936-1018 and :1093-1130,
//              tcp/IpTcpProto_input.h:68-100, udp/IpUdpProto.h:470-490, :631-652);
//   Tx fill:   the checksums the reference's send paths write, filled in place
//              (ip/IpStack.h:425-453, tcp/IpTcpProto_output.h:1251-1277,
//              udp/IpUdpProto.h:164-179, ip/IpStack.h:1164-1190).
//
// 64-frame chunks per wave (CSR frame offsets, as the checksum CSR batch). The header
// decisions run one frame per LANE (VALU), from the frame's first 112 aligned bytes; the
// L4 checksums run one frame per WAVE over just the bytes they cover, with the CSR
// batch's loads, masks and DPP reduction. Each frame's bytes come from HBM once (the
// header bytes are re-read from L2 by the L4 pass).

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "aipstack_amd/chksum.h"
#include "chksum_device.h"
#include "chksum_internal.h"

namespace aipstack_amd {
namespace {

// Frame bytes [0, 82) hold every header field the kernels read: 14 (Ethernet) + 60 (IPv4
// with options) + 8 (UDP header); from A0 = S & ~15 that is at most 97 bytes. The header
// pass loads from A0 up to the next 32-byte boundary past them (7 or 8 segments), so the
// L4 pass starts on a fresh 32-byte sector and no sector is fetched twice.
constexpr int kHdrSegs = 8;
constexpr int kHdrDwords = 23;  // frame bytes [0, 92) realigned to the frame start
constexpr uint32_t kHdrNeed = 97;
constexpr uint64_t kMaxSlotStride = AIPSTACK_CHKSUM_MAX_SLOT_STRIDE;
// Records (the split fill's read pass, the records-only pass): nontemporal stores (1) or
// ordinary ones (0), an A/B build switch.
#ifndef AIPSTACK_FRAME_REC_NT
#define AIPSTACK_FRAME_REC_NT 1
#endif
// The in-place Tx fills' field stores by default (tunable "tx_store", FieldSectors below).
#ifndef AIPSTACK_TX_STORE_DEFAULT
#define AIPSTACK_TX_STORE_DEFAULT 0
#endif
constexpr int kTxStoreDefault = AIPSTACK_TX_STORE_DEFAULT;


__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
    return __builtin_bswap32(x);
}

// (a & ~m) | (b & m): one v_bfi_b32. Used instead of `c ? x[i + k] : x[i]`, which LLVM
// canonicalises into a dynamically indexed load (a private array in scratch).
__device__ __forceinline__ uint32_t blend(uint32_t m, uint32_t a, uint32_t b) {
    return (a & ~m) | (b & m);
}

__device__ __forceinline__ uint32_t be16_at(uint32_t le_dword, int byte) {  // byte 0 or 2
    return ((le_dword >> (8 * byte)) & 0xFFu) << 8 | ((le_dword >> (8 * byte + 8)) & 0xFFu);
}

// One global_store_short at any byte address: ROCm runs gfx9 in unaligned-access mode, so
// an odd address is one store instruction, not two byte stores (the frame fields sit at
// S + 24 and S + fld, odd whenever the frame starts at an odd address).
typedef uint16_t u16_any_align __attribute__((aligned(1)));
#ifndef AIPSTACK_TX_STORE_MODE  // experiments only (tools/sweep.py --lib): 1 = nontemporal,
#define AIPSTACK_TX_STORE_MODE 0   // 2 = no field stores (measures their cost; wrong output)
#endif
__device__ __forceinline__ void store_be16(uint64_t addr, uint32_t v) {
#if AIPSTACK_TX_STORE_MODE == 0
    *reinterpret_cast<u16_any_align *>(addr) = (uint16_t)bswap16(v);
#elif AIPSTACK_TX_STORE_MODE == 1
    __builtin_nontemporal_store((uint16_t)bswap16(v), reinterpret_cast<u16_any_align *>(addr));
#else
    asm volatile("" ::"v"(v), "v"(addr));  // keep the value live, store nothing
#endif
}

// Sector stores (round 4, the in-place Tx fills' `SECT` form). A 2-byte field store makes a
// partial 32-byte sector that the memory side has to merge with the bytes around it; the
// lane holds those bytes already (its header blocks), so it writes each field's whole
// sector instead -- the sector's bytes as read, the field patched in -- as two 16-byte
// stores. Only sectors inside the frame's own bytes [S, E) are written whole (no byte of
// another frame or of a slot's slack is ever rewritten). Every written field that overlaps a
// whole-written sector, even by one byte, is patched into it; a field that no written sector
// holds whole keeps its 2-byte store as well (the same value, so their order is free).
// sec[0..1] = sector A (holding frame byte 24, the IPv4 checksum field's first), sec[2..3] =
// sector B (holding the L4 field's first byte; not written when it is A).
struct FieldSectors {
    u32x4 sec[4];
    uint32_t mode;  // bit 0: write A whole; bit 1: write B whole
};

// One frame's result, as the finish step produces it (lane j <-> frame j of the chunk):
//   w0 = IPv4 header checksum (bits 0-15) | L4 checksum (16-31)
//   w1 = L4 field offset from the frame start (0-7) | write the IPv4 field (8) | write the
//        L4 field (9) | status / verdict (16-23)
// Also the split Tx fill's workspace record (w0 | w1 << 32), scattered by tx_scatter_kernel.
struct FrameOut {
    uint64_t S;  // frame start (absolute address)
    uint32_t w0, w1;
    FieldSectors fs;  // SECT launches only
};

__device__ __forceinline__ uint32_t frame_w1(int fld, bool ip, bool l4, int status) {
    return (uint32_t)(fld & 0xFF) | (uint32_t)ip << 8 | (uint32_t)l4 << 9 |
           (uint32_t)(uint8_t)status << 16;
}

// The stores of one frame: its status byte, and for Tx the two checksum fields in place.
#ifndef AIPSTACK_TX_RETOUCH  // experiment: load the field dwords again right before the stores
#define AIPSTACK_TX_RETOUCH 0
#endif
template <bool TX>
__device__ __forceinline__ void store_frame(uint64_t S, uint32_t w0, uint32_t w1,
                                            uint8_t *__restrict__ status, uint64_t i) {
    status[i] = (uint8_t)(w1 >> 16);
    if constexpr (TX && AIPSTACK_TX_RETOUCH) {
        typedef __attribute__((address_space(1))) const uint32_t gdw;
        uint32_t t0 = 0, t1 = 0;
        if (w1 & 0x100u) t0 = *(const gdw *)((S + 24) & ~(uint64_t)3);
        if (w1 & 0x200u) t1 = *(const gdw *)((S + (w1 & 0xFFu)) & ~(uint64_t)3);
        asm volatile("" ::"v"(t0), "v"(t1));
    }
    if constexpr (TX) {
        if (w1 & 0x100u) store_be16(S + 24, w0);
        if (w1 & 0x200u) store_be16(S + (w1 & 0xFFu), w0 >> 16);
    }
}

// The 16-bit value v written big-endian at byte b of a sector held as 8 little-endian
// dwords (d[k] = sector bytes [4k, 4k + 4)); b = -1 or 31: only the byte inside the sector.
// Branch-free over the 8 dwords.
__device__ __forceinline__ void patch_be16(u32x4 &lo, u32x4 &hi, int b, uint32_t v) {
    const uint32_t w = bswap16(v);  // low byte = the byte at b
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int p = b - 4 * k;  // the field's first byte within dword k (-1: its 2nd)
        const uint32_t m = dword_keep(p, p + 2);
        const uint32_t val = p >= 0 ? w << ((8 * p) & 31) : w >> 8;
        if (k < 4)
            lo[k] = (lo[k] & ~m) | (val & m);
        else
            hi[k - 4] = (hi[k - 4] & ~m) | (val & m);
    }
}

// Sector stores of one frame (FieldSectors above): the written sectors whole, each with
// every written field overlapping it patched in, and 2-byte stores of the fields no written
// sector holds whole. The sector addresses are recomputed from S and fld.
__device__ __forceinline__ void store_frame_sectors(uint64_t S, uint32_t w0, uint32_t w1,
                                                    FieldSectors fs, uint8_t *__restrict__ status,
                                                    uint64_t i) {
    status[i] = (uint8_t)(w1 >> 16);
    const bool wi = (w1 & 0x100u) != 0, wl = (w1 & 0x200u) != 0;
    const uint64_t xi = S + 24, xl = S + (w1 & 0xFFu);
    const uint64_t sa = xi & ~(uint64_t)31, sb = xl & ~(uint64_t)31;
    // field positions relative to each sector (the first byte; -1 .. 31 = overlaps it)
    const int ia = (int)(xi - sa), la = (int)(int64_t)(xl - sa);
    const int ib = (int)(int64_t)(xi - sb), lb = (int)(xl - sb);
    const bool wa = (fs.mode & 1u) != 0, wb = (fs.mode & 2u) != 0;
    bool ci = false, cl = false;  // held whole by a written sector
    if (wa) {
        if (wi) patch_be16(fs.sec[0], fs.sec[1], ia, w0);
        if (wl && la >= -1 && la <= 31) patch_be16(fs.sec[0], fs.sec[1], la, w0 >> 16);
        ci = ia <= 30;
        cl = la >= 0 && la <= 30;
        u32x4 *p = reinterpret_cast<u32x4 *>(sa);
        p[0] = fs.sec[0];
        p[1] = fs.sec[1];
    }
    if (wb) {
        if (wl) patch_be16(fs.sec[2], fs.sec[3], lb, w0 >> 16);
        if (wi && ib >= -1 && ib <= 31) patch_be16(fs.sec[2], fs.sec[3], ib, w0);
        cl = cl || lb <= 30;
        ci = ci || (ib >= 0 && ib <= 30);
        u32x4 *p = reinterpret_cast<u32x4 *>(sb);
        p[0] = fs.sec[2];
        p[1] = fs.sec[3];
    }
    if (wi && !ci) store_be16(xi, w0);
    if (wl && !cl) store_be16(xl, w0 >> 16);
}

// Second pass of the split Tx fill: one frame per thread, the stores of every frame after
// the whole read pass (stream-ordered behind frame_kernel<TX, ..., SPLIT>).
__global__ __launch_bounds__(kBlock) void tx_scatter_kernel(uint64_t base,
                                                            const uint64_t *__restrict__ offsets,
                                                            const uint64_t *__restrict__ records,
                                                            uint8_t *__restrict__ status,
                                                            uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const uint64_t rec = records[i];
        store_frame<true>(base + offsets[i], (uint32_t)rec, (uint32_t)(rec >> 32), status, i);
    }
}

// The same for ring slots: frame i starts at base + i * stride.
__global__ __launch_bounds__(kBlock) void tx_scatter_slotted_kernel(uint64_t base, uint64_t stride,
                                                                    const uint64_t *__restrict__ records,
                                                                    uint8_t *__restrict__ status,
                                                                    uint64_t n) {
    const uint64_t step = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += step) {
        const uint64_t rec = records[i];
        store_frame<true>(base + i * stride, (uint32_t)rec, (uint32_t)(rec >> 32), status, i);
    }
}

// Halves-sum (the stream's H metric: little-endian 16-bit halves at even absolute
// addresses) of the bytes [0, o) of one aligned 16-byte segment.
__device__ __forceinline__ uint32_t halves_below(const u32x4 &x, uint32_t o) {
    uint32_t acc = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) acc = halves(x[d] & dword_keep(0, (int)o - 4 * d), acc);
    return acc;
}

// The same for the segment at byte `off` (< 128) of a lane's header blocks (aligned
// segments from A0): the bytes of that segment below `off`. Branch-free 8-way select.
__device__ __forceinline__ uint32_t seg_below(const u32x4 (&seg)[kHdrSegs], uint32_t off) {
    const uint32_t si = off >> 4;
    u32x4 x = seg[0];
#pragma unroll
    for (int i = 1; i < kHdrSegs; ++i) {
        const uint32_t m = si == (uint32_t)i ? ~0u : 0u;
#pragma unroll
        for (int d = 0; d < 4; ++d) x[d] = (x[d] & ~m) | (seg[i][d] & m);
    }
    return halves_below(x, off & 15u);
}

// What the header pass decides for one frame (lane j <-> frame j of the chunk).
struct FrameLane {
    uint64_t l4s;       // first byte the L4 checksum covers (its parity orients the sum)
    uint64_t l4e;       // one past the last (stream mode)
    uint32_t fhalf;     // Tx, stream mode: the checksum field's bytes as they enter H
    uint64_t cs, ce;    // the L4 bytes past the header pass's blocks: [cs, ce), maybe empty
    uint32_t part;      // ones'-complement sum of the L4 bytes inside the header blocks
    bool l4;            // an L4 checksum is computed
    uint32_t words;     // IpChksumAccumulator words added before them (pseudo-header)
    uint32_t hchk;      // IPv4 header checksum over the header (Tx: with the field as 0)
    int fld;            // Tx: L4 checksum field, bytes from the frame start
    int pre;            // the verdict / status when no L4 sum decides it
    bool ip_ok;         // the IPv4 header parsed (Tx writes its checksum)
    bool udp;           // Tx: a computed 0 is sent as 0xFFFF
};

// Header pass, one frame per lane, all in VALU: realign the frame's first bytes from the
// aligned segments, then the checks of EthIpIface::recvFrame (eth/EthIpIface.h:367-390),
// IpStack::processRecvedIp4Packet (ip/IpStack.h:936-1044) and the L4 entry checks
// (tcp/IpTcpProto_input.h:68-100, udp/IpUdpProto.h:470-490, 631-652, ip/IpStack.h:1093-1130);
// the send side fills the same fields (ip/IpStack.h:425-453, tcp/IpTcpProto_output.h:1251-1277,
// udp/IpUdpProto.h:164-179, ip/IpStack.h:1164-1190).
// STREAM: the L4 sum comes from stream prefixes over [l4s, l4e) (minus the Tx field's
// bytes, fhalf), so the partial sum over the header blocks and [cs, ce) are not needed.
template <bool TX, bool STREAM>
__device__ __forceinline__ FrameLane parse_lane(const u32x4 (&seg)[kHdrSegs], uint64_t S,
                                                int len, uint32_t hb_end) {
    uint32_t raw[4 * kHdrSegs];
#pragma unroll
    for (int i = 0; i < kHdrSegs; ++i)
#pragma unroll
        for (int d = 0; d < 4; ++d) raw[4 * i + d] = seg[i][d];
    // f[i] = frame bytes [4i, 4i + 4) as a little-endian dword: shift by S & 15 bytes
    const uint32_t rs = (uint32_t)S & 15u;
    const uint32_t q2 = (rs & 8u) ? ~0u : 0u, q1 = (rs & 4u) ? ~0u : 0u;
    uint32_t t1[kHdrDwords + 2], t2[kHdrDwords + 1], f[kHdrDwords];
#pragma unroll
    for (int i = 0; i < kHdrDwords + 2; ++i) t1[i] = blend(q2, raw[i], raw[i + 2]);
#pragma unroll
    for (int i = 0; i < kHdrDwords + 1; ++i) t2[i] = blend(q1, t1[i], t1[i + 1]);
#pragma unroll
    for (int i = 0; i < kHdrDwords; ++i) f[i] = __builtin_amdgcn_alignbyte(t2[i + 1], t2[i], rs & 3u);

    FrameLane r;
    r.l4s = r.l4e = r.cs = r.ce = S;
    r.fhalf = 0;
    r.part = 0;
    r.l4 = false;
    r.words = 0;
    r.fld = 0;
    r.udp = false;
    r.ip_ok = false;
    // ---- Ethernet + IPv4 header checks (eth/EthIpIface.h:370-384, ip/IpStack.h:938-990)
    const uint32_t ethertype = be16_at(f[3], 0);
    const uint32_t vihl = (f[3] >> 16) & 0xFFu;
    const int hl = vihl == 0x45u ? 20 : (int)(vihl & 0xFu) * 4;
    const int total_len = (int)be16_at(f[4], 0);
    const int plen = len - 14;
    if (len < 14 || ethertype != 0x0800u) {
        r.pre = AIPSTACK_RX_NOT_IP4;
    } else if (plen < 20 || (vihl >> 4) != 4u || hl < 20 || hl > plen || total_len < hl ||
               total_len > plen) {
        r.pre = AIPSTACK_RX_DROP_IP_MALFORMED;
    } else {
        r.ip_ok = true;
        r.pre = -1;
    }
    // ---- IPv4 header sum: dwords of frame bytes [14 + 4m, 18 + 4m), m < hl / 4. Their
    // little-endian halves pair (14 + 2i, 15 + 2i) with the even byte low: byte-swapped
    // big-endian words, so the folded sum is swapped back once (x * 256 * 256 = x).
    Eac hs;
#pragma unroll
    for (int m = 0; m < 15; ++m) {
        uint32_t w = __builtin_amdgcn_alignbyte(f[4 + m], f[3 + m], 2);
        if (TX && m == 2) w &= 0xFFFFu;  // header checksum field as 0 (bytes 24-25)
        hs.add(w & (4 * m < hl ? ~0u : 0u));
    }
    r.hchk = (~bswap16(fold16(hs.finish()))) & 0xFFFFu;
    if (!r.ip_ok)
        return r;
    if (!TX && r.hchk != 0) {                                       // ip/IpStack.h:1016
        r.pre = AIPSTACK_RX_DROP_IP_CHKSUM;
        return r;
    }
    const uint32_t flags_off = be16_at(f[5], 0);
    const uint32_t proto = f[5] >> 24;
    if ((flags_off & 0x3FFFu) != 0) {                               // ip/IpStack.h:1020
        r.pre = AIPSTACK_RX_FRAGMENT;
        return r;
    }
    const uint32_t src = bswap32(__builtin_amdgcn_alignbyte(f[7], f[6], 2));
    const uint32_t dst = bswap32(__builtin_amdgcn_alignbyte(f[8], f[7], 2));
    const uint32_t pseudo = (src >> 16) + (src & 0xFFFFu) + (dst >> 16) + (dst & 0xFFFFu);
    const int dg = 14 + hl;
    const int dlen = total_len - hl;
    // UDP length + checksum: frame bytes [dg + 4, dg + 8), i.e. dwords 4 + hl/4 and 5 + hl/4
    const int h = hl >> 2;
    uint32_t ulo = f[9], uhi = f[10];
#pragma unroll
    for (int hh = 6; hh <= 15; ++hh) {
        const uint32_t sel = h == hh ? ~0u : 0u;
        ulo = blend(sel, ulo, f[4 + hh]);
        uhi = blend(sel, uhi, f[5 + hh]);
    }
    const uint32_t uw = __builtin_amdgcn_alignbyte(uhi, ulo, 2);
    int l4len = -1, fo = 0;
    r.pre = AIPSTACK_RX_ACCEPT_OTHER;
    if (proto == 6) {                                               // TCP
        if (dlen < 20) r.pre = AIPSTACK_RX_DROP_L4_MALFORMED;
        else { l4len = dlen; fo = 16; r.words = pseudo + 6u + (uint32_t)dlen; }
    } else if (proto == 17) {                                       // UDP
        const int ulen = (int)be16_at(uw, 0);
        if (dlen < 8 || ulen < 8 || ulen > dlen) {
            r.pre = AIPSTACK_RX_DROP_L4_MALFORMED;
        } else if (!TX && be16_at(uw, 2) == 0) {
            r.pre = AIPSTACK_RX_ACCEPT_NO_CHKSUM;                   // udp/IpUdpProto.h:637
        } else {
            l4len = ulen; fo = 6; r.words = pseudo + 17u + (uint32_t)ulen; r.udp = true;
        }
    } else if (proto == 1) {                                        // ICMP
        if (dlen < 8) r.pre = AIPSTACK_RX_DROP_L4_MALFORMED;
        else { l4len = dlen; fo = 2; }
    }
    if (l4len >= 0) {
        r.pre = AIPSTACK_RX_ACCEPT;
        r.l4 = true;
        r.l4s = S + (uint64_t)dg;
        r.fld = dg + fo;
        if constexpr (STREAM) {
            r.l4e = r.l4s + (uint64_t)l4len;
            if constexpr (TX) {
                // the field (frame bytes fld, fld + 1; fld = 0 or 2 mod 4, fld <= 90) is
                // half fld & 2 of f[fld / 4]; in H its two bytes pair with their absolute
                // neighbours: as stored if S + fld is even, byte-swapped if odd
                const int k = r.fld >> 2;
                uint32_t fw = f[9];
#pragma unroll
                for (int i = 10; i < kHdrDwords; ++i) fw = blend(k == i ? ~0u : 0u, fw, f[i]);
                const uint32_t fv = (fw >> (8 * (r.fld & 2))) & 0xFFFFu;
                r.fhalf = ((S + (uint64_t)r.fld) & 1u) ? bswap16(fv) : fv;
            }
            return r;
        }
        // L4 bytes inside the loaded blocks [A0, A0 + hb_end): summed here, from the aligned
        // dwords (little-endian halves at even absolute addresses, as the L4 pass sums); the
        // rest, [A0 + hb_end, end), by the L4 pass. For Tx the checksum field (always in
        // the header blocks: fld + 2 <= 92) is summed as 0.
        const int lo = (int)rs + dg, hi = (int)rs + dg + l4len;
        const int fx = TX ? (int)rs + r.fld : -64;
        Eac ps;
#pragma unroll
        for (int i = 0; i < 4 * kHdrSegs; ++i) {
            uint32_t m = dword_keep(lo - 4 * i, min(hi, (int)hb_end) - 4 * i);
            if (TX) m &= ~dword_keep(fx - 4 * i, fx + 2 - 4 * i);
            ps.add(raw[i] & m);
        }
        r.part = ps.finish();
        const uint64_t a0 = S & ~(uint64_t)15;
        r.cs = a0 + hb_end;
        r.ce = hi > (int)hb_end ? a0 + (uint64_t)hi : r.cs;
    }
    return r;
}

// Halves-sum of a whole 16-byte segment.
__device__ __forceinline__ uint32_t seg_halves(const u32x4 &x) {
    return halves(x[0], halves(x[1], halves(x[2], halves(x[3], 0u))));
}

// Halves-sum of the bytes [A0, A0 + off) of a lane's header blocks (off < 16 * kHdrSegs):
// the whole segments below off's segment (per-segment sums hs) plus that segment's bytes.
__device__ __forceinline__ uint32_t hdr_below(const u32x4 (&seg)[kHdrSegs],
                                              const uint32_t (&hs)[kHdrSegs], uint32_t off) {
    const uint32_t si = off >> 4;
    uint32_t acc = seg_below(seg, off);
#pragma unroll
    for (int i = 0; i < kHdrSegs - 1; ++i) acc += (uint32_t)i < si ? hs[i] : 0u;
    return acc;
}

// Gathered frame stream (stream mode, round 2): the chunk's header segments -- the union
// over its frames of [A0_j, A0_j + hb_end_j), within the run -- are copied out of the stream
// windows into a compact LDS array as they pass (a segment's slot = the union segments
// before it), instead of being loaded per lane before the stream: a header line loaded up
// front has left L2 by the time the stream reaches it, so it was fetched twice (RX 1.11x).
// Which lanes of window w hold header segments is word w of an LDS mask table, so runs of at
// most kGatherWindows windows take this path; chunks of at most kCaptureFrames frames (the
// launch's 32, round 4), so that the compact slots take 4 KiB per wave (round 5: 64 frames'
// 8 KiB held the kernel at 4 waves per SIMD by LDS alone).
constexpr uint32_t kGatherWindows = 64;
constexpr uint32_t kCaptureFrames = 32;
#ifndef AIPSTACK_FRAME_NT  // experiments: 0 = the frame stream loads with the default policy
#define AIPSTACK_FRAME_NT 1
#endif
constexpr uint32_t kHdrSlots = kCaptureFrames * kHdrSegs;  // at most 8 segments per frame

// Round 5 (AIPSTACK_FRAME_HCAP): the capture also stores H at each captured segment's start,
// so a frame's H(A0) is read from LDS after the stream instead of fetched per window with a
// ds_bpermute (and its wait) as a stream boundary.
#ifndef AIPSTACK_FRAME_HCAP
#define AIPSTACK_FRAME_HCAP 1
#endif
struct FrameLds {
    uint64_t wmask[kGatherWindows + 8];  // per window: the lanes holding header segments
                                         // (+8: whole groups past the last window read 0)
    u32x4 slots[kHdrSlots];          // the compact header segments
    uint32_t hslot[AIPSTACK_FRAME_HCAP ? kHdrSlots : 1];  // H at each slot's segment start
};

// Capture hook: group(w) fetches the group's U window masks into SGPRs (broadcast LDS
// reads); window(v, w) writes the lanes of the mask to consecutive compact slots.
template <int U>
struct HeaderCapture {
    static constexpr bool kWantH = AIPSTACK_FRAME_HCAP != 0;
    const uint64_t *wmask;
    u32x4 *slots;
    uint32_t *hslot;
    uint32_t count;  // header segments before the current window (wave-uniform)
    uint64_t mk[U];
    __device__ __forceinline__ void group(uint32_t w) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t wu = w + (uint32_t)u;
            const uint64_t x = wmask[wu];  // wu < kGatherWindows + U: zeroed
            mk[u] = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
        }
    }
    // The store runs under exec = the window's mask, set and restored inside one asm
    // statement (the compiler would test each lane's bit with VALU instead). The statement
    // declares SCC clobbered (s_and_saveexec_b64 writes it): without that, LLVM may keep a
    // scalar compare's SCC live across it -- an s_cmp before, an s_cselect after, selecting
    // between the masks of two windows in flight. Round 5's copy of this store in the gathered
    // stream lacked the clobber and did swap two windows' start masks; EXEC is
    // restored inside the statement, and LDS stores complete in order, so the compiler's own
    // lgkmcnt waits stay conservative. tools/asm_scc_scan.py checks a build for SCC read after
    // any such statement before it is written again.
    __device__ __forceinline__ void window(const u32x4 &v, uint32_t w, uint32_t hv) {
        static_assert(U <= 8, "wmask holds 8 zero words past the last window");
        const uint64_t m = mk[w & (uint32_t)(U - 1)];
        const uint32_t below =
            __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        typedef __attribute__((address_space(3))) u32x4 lds_seg;
        const uint32_t addr = (uint32_t)(uintptr_t)(lds_seg *)(slots + count) + 16u * below;
        uint64_t save;
        if constexpr (kWantH) {
            typedef __attribute__((address_space(3))) uint32_t lds_h;
            const uint32_t haddr = (uint32_t)(uintptr_t)(lds_h *)(hslot + count) + 4u * below;
            asm volatile(
                "s_and_saveexec_b64 %0, %2\n\t"
                "ds_write_b128 %1, %3\n\t"
                "ds_write_b32 %4, %5\n\t"
                "s_mov_b64 exec, %0"
                : "=&s"(save)
                : "v"(addr), "s"(m), "v"(v), "v"(haddr), "v"(hv)
                : "memory", "scc");
        } else {
            asm volatile(
                "s_and_saveexec_b64 %0, %2\n\t"
                "ds_write_b128 %1, %3\n\t"
                "s_mov_b64 exec, %0"
                : "=&s"(save)
                : "v"(addr), "s"(m), "v"(v)
                : "memory", "scc");
        }
        count += (uint32_t)__builtin_popcountll(m);
    }
};

// Bits [lo, hi) of a 64-bit word (lo < 64, lo <= hi).
__device__ __forceinline__ uint64_t bit_range(uint32_t lo, uint32_t hi) {
    const uint64_t top = hi >= 64u ? ~0ull : ((1ull << hi) - 1ull);
    return top & ~((1ull << lo) - 1ull);
}

// H(l4s) - H(A0) from the header blocks: l4s - A0 = (S & 15) + 14 + IHL * 4 lies in
// [34, 89], i.e. in segment 2..5 (any other offset only feeds lanes whose sum is unused).
__device__ __forceinline__ uint32_t l4s_below(const u32x4 (&seg)[kHdrSegs], uint32_t off) {
    const uint32_t si = off >> 4;
    u32x4 x = seg[2];
#pragma unroll
    for (int i = 3; i <= 5; ++i) {
        const uint32_t m = si == (uint32_t)i ? ~0u : 0u;
#pragma unroll
        for (int d = 0; d < 4; ++d) x[d] = (x[d] & ~m) | (seg[i][d] & m);
    }
    uint32_t acc = halves_below(x, off & 15u) + seg_halves(seg[0]) + seg_halves(seg[1]);
#pragma unroll
    for (int i = 2; i <= 4; ++i) acc += (uint32_t)i < si ? seg_halves(seg[i]) : 0u;
    return acc;
}

// The sectors of a frame's two checksum fields, taken from its header blocks right after
// the parse (FieldSectors): sector A holds frame byte 24, B frame byte fld; A0 = S & ~15, so
// A lies at segment 0..2 and B at segment 1..6 of the blocks, and both end inside them (the
// blocks end on the first 32-byte boundary at or past frame byte 97).
__device__ __forceinline__ FieldSectors pick_sectors(const u32x4 (&seg)[kHdrSegs], uint64_t S,
                                                     uint64_t E, const FrameLane &fl) {
    const uint64_t A0 = S & ~(uint64_t)15;
    const uint64_t xi = S + 24, xl = S + (uint64_t)fl.fld;
    const uint64_t ai = xi & ~(uint64_t)31, al = xl & ~(uint64_t)31;
    const bool in_i = fl.ip_ok && ai >= S && ai + 32 <= E;
    const bool in_l = fl.l4 && al >= S && al + 32 <= E && !(in_i && al == ai);
    FieldSectors fs;
    fs.mode = (in_i ? 1u : 0u) | (in_l ? 2u : 0u);
    const uint32_t ia = (uint32_t)(ai - A0) >> 4, il = (uint32_t)(al - A0) >> 4;
    fs.sec[0] = seg[0];
    fs.sec[1] = seg[1];
    fs.sec[2] = seg[1];
    fs.sec[3] = seg[2];
#pragma unroll
    for (int i = 1; i <= 6; ++i) {
        const uint32_t ma = i <= 2 && ia == (uint32_t)i ? ~0u : 0u;
        const uint32_t mb = i >= 2 && il == (uint32_t)i ? ~0u : 0u;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            if (i <= 2) {
                fs.sec[0][d] = blend(ma, fs.sec[0][d], seg[i][d]);
                fs.sec[1][d] = blend(ma, fs.sec[1][d], seg[i + 1][d]);
            }
            if (i >= 2) {
                fs.sec[2][d] = blend(mb, fs.sec[2][d], seg[i][d]);
                fs.sec[3][d] = blend(mb, fs.sec[3][d], seg[i + 1][d]);
            }
        }
    }
    return fs;
}

// Rx verify / Tx fill of one 64-frame chunk (CSR offsets), lane j <-> frame j:
//   (B) lane j loads frame j's first 112 aligned bytes (one buffer descriptor per chunk)
//       and parses its headers (parse_lane): the L4 byte range, pseudo-header words and
//       the verdict when no L4 sum is needed;
//   (C) the frames that need an L4 sum are summed one per wave, P in flight, exactly as
//       the CSR checksum batch sums packets (PacketLoad over the L4 range); for Tx the
//       checksum field is masked out of the sum;
//   (D) lane j finishes frame j: the verdict, and for Tx the IPv4 header and L4 checksums.
// Returns lane j's FrameOut; the caller stores it (store_frame) now or later.
//
// Stream mode (SU > 0, chunks whose frames lie back to back): (C) is replaced by stream
// prefixes over the chunk's frames (chksum_device.h): each frame's L4 sum is
// H(l4e) - H(l4s), minus the Tx checksum field's bytes; no per-frame loads or reductions.
// Stream windows issued before the header parse (the rest after it): all of them hold
// ~4 * SU more VGPRs through the parse.
#ifndef AIPSTACK_FRAME_PREFETCH
#define AIPSTACK_FRAME_PREFETCH(SU) ((SU) / 2)
#endif
// Frames whose headers are captured from the stream: the next group of windows issued before
// the current one is summed (StreamRun's DB; round 4, profiles/r04/fdb: RX 120.1 -> 117.6 us,
// split Tx fill 161.2 -> 155.8, records pass 129.2 -> 127.6; 128 VGPRs at 8 windows, no
// spill, the same 4 waves per SIMD). A/B build switch: -DAIPSTACK_FRAME_DB=0.
#ifndef AIPSTACK_FRAME_DB
#define AIPSTACK_FRAME_DB 1
#endif
// Ring slots: the L4 bytes past the header blocks read as one gathered stream of the chunk's
// frames (1) or one frame per wave instruction pair (0, rounds 3-4), an A/B build switch.
#ifndef AIPSTACK_FRAME_SLOT_GATHER
#define AIPSTACK_FRAME_SLOT_GATHER 1
#endif
// GATHER: where the parse's header segments come from (launch_frames picks it):
//   kHdrLoads    per-lane loads before the stream (default policy);
//   kHdrCapture  copied out of the stream windows as they pass (Rx, the records-only pass);
//   kHdrCaptureTouch  the same, plus two dword loads per frame at the default policy before
//                the stream, on the lines holding the IPv4 and (usually) the L4 checksum
//                field, so that the in-place field stores find those lines in the caches
//                (split fill 168 vs 178 us, one pass 174 vs 186).
constexpr int kHdrLoads = 0, kHdrCapture = 1, kHdrCaptureTouch = 2;
template <class Desc, bool TX, int U, int P, bool NT, int SU, int GATHER, int STORE>
__device__ __forceinline__ FrameOut process_chunk(const Desc &desc, uint64_t p0, uint64_t n,
                                                  uint32_t cpk, int lane, uint32_t voff,
                                                  uint32_t not_lane0, FrameLds *lds,
                                                  GatherLds *glds, u32x4 *lines, int &cnt_out) {
    constexpr bool SECT = STORE == kTxStoreSectors;
    const int cnt = (int)min((uint64_t)cpk, n - p0);
    // the chunk's own table entries only (lanes past it re-read entry p0 + cnt)
    const auto chunk = desc.begin_chunk(p0, p0 + (uint64_t)cnt, lane);
    cnt_out = cnt;
    uint64_t S, E;
    desc.lane_bounds(chunk, lane, S, E);
    const uint64_t l64 = E - S;
    // a frame over 65535 bytes (or E < S) is outside the contract: NOT_IP4, reported
    const bool too_long = l64 > (uint64_t)AIPSTACK_CHKSUM_MAX_LEN;
    note_violation(lane < cnt && too_long, AIPSTACK_CHKSUM_VIOLATION_PACKET_LEN);
    const int len = (lane >= cnt || too_long) ? 0 : (int)l64;  // 0: NOT_IP4
    // (B) headers: aligned segments [A0_j, A0_j + 112) through one range-checked
    // descriptor over the chunk's aligned span (never past the 16-byte blocks holding
    // the chunk's bytes; slots past it read 0). A span beyond what 64 frames of at most
    // 65535 bytes can cover (offsets outside the contract, chksum.h) reads nothing.
    const uint64_t base = (__builtin_amdgcn_readfirstlane((uint32_t)S) & ~15u) |
                          ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(S >> 32)) << 32);
    const uint64_t span = ((desc.chunk_end(chunk, cnt) + 15u) & ~(uint64_t)15) - base;
    const bool span_bad = span > (uint64_t)kWave * 65536u + 16u;
    note_violation(span_bad && lane == 0, AIPSTACK_CHKSUM_VIOLATION_SPAN);
    const uint32_t hrec = __builtin_amdgcn_readfirstlane(
        span_bad ? 0u : (uint32_t)span);  // uniform: SGPR descriptor
    const __amdgpu_buffer_rsrc_t hrsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(base), (short)0, hrec, 0x00020000);
    const uint32_t hoff = (uint32_t)((S & ~(uint64_t)15) - base);
    // this lane's blocks: A0 up to the first 32-byte boundary past the header bytes
    // (A0 % 32 + 15 + 97 + 31 < 160, so at most 128 bytes = kHdrSegs segments)
    const uint32_t a0_32 = (uint32_t)S & 16u;
    const uint32_t hb_end = ((a0_32 + ((uint32_t)S & 15u) + kHdrNeed + 31u) & ~31u) - a0_32;
    u32x4 seg[kHdrSegs];
    auto load_headers = [&]() {
#pragma unroll
        for (int i = 0; i < kHdrSegs; ++i)  // past hb_end or the chunk: out of range, reads 0
            seg[i] = load_segment<false>(
                hrsrc, 16u * i < hb_end && lane < cnt ? hoff + 16u * i : 0xFFFFFFF0u, 0u);
    };
    FrameLane fl;
    FieldSectors fsec;
    fsec.mode = 0;
    uint32_t r;
    bool streamed = false, have_headers = false;
    if constexpr (SU > 0) {
      if (stream_ok(S, E, lane, cnt)) {
        const int lastl = cnt - 1;
        const uint64_t X1 =
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(E >> 32), lastl)
             << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)E, lastl);
        const uint32_t nseg = ((uint32_t)(X1 - base) + 15u) >> 4;
        if (GATHER != kHdrLoads && cnt <= (int)kCaptureFrames &&
            ((nseg + 63u) >> 6) <= kGatherWindows) {
            // (B'+C') one pass: the stream gives H at every frame's aligned start A0_j and
            // hands the header segments to LDS; the parse runs on them after the stream.
            const uint64_t A0 = S & ~(uint64_t)15;
            const bool act = lane < cnt;
            const uint32_t r0 = act ? (uint32_t)((A0 - base) >> 4) : nseg;
            const uint32_t r1 = min(r0 + (hb_end >> 4), nseg);
            // the window masks: each lane ORs its header segments in (at most two windows)
            {
                uint32_t z;  // made here (a zero quad kept live across the loop was spilled)
                asm volatile("v_mov_b32 %0, 0" : "=v"(z));
                static_assert((kGatherWindows + 8) % 2 == 0 && (kGatherWindows + 8) / 2 <= kWave,
                              "one 16-byte store per lane clears the masks");
                if (lane < (int)(kGatherWindows + 8) / 2)
                    reinterpret_cast<u32x4 *>(lds->wmask)[lane] = u32x4{z, z, z, z};
            }
            __builtin_amdgcn_wave_barrier();
            if (r1 > r0) {
                const uint32_t w0 = r0 >> 6, e0 = r1 - (w0 << 6);
                __hip_atomic_fetch_or(&lds->wmask[w0], bit_range(r0 & 63u, min(e0, 64u)),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                if (e0 > 64u)
                    __hip_atomic_fetch_or(&lds->wmask[w0 + 1u], bit_range(0u, e0 - 64u),
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // the field lines (frame bytes 24 and 50: IPv4, and TCP / UDP / ICMP behind a
            // 20-byte IPv4 header) into the caches before the nontemporal stream passes them
            uint32_t touch0 = 0, touch1 = 0;
            if constexpr (TX && GATHER == kHdrCaptureTouch) {
                const uint32_t fo = (uint32_t)(S - base);
                touch0 = __builtin_amdgcn_raw_buffer_load_b32(
                    hrsrc, act ? (fo + 24u) & ~3u : 0xFFFFFFF0u, 0u, 0);
                touch1 = __builtin_amdgcn_raw_buffer_load_b32(
                    hrsrc, act ? (fo + 50u) & ~3u : 0xFFFFFFF0u, 0u, 0);
            }
            StreamRun<SU, NT, SU, AIPSTACK_FRAME_DB != 0> run;
            run.begin(base, X1, voff);
            // compact slot of r0: the union segments below it. Regions start and end in
            // lane order, so region j adds [max(r0_j, r1_{j-1}), r1_j) to the union.
            const uint32_t r1p = (uint32_t)__builtin_amdgcn_ds_bpermute(
                ((lane + 63) & 63) << 2, (int)(lane == 63 ? 0u : r1));
            const uint32_t uj = max(r0, r1p);
            const uint32_t nw = r1 > uj ? r1 - uj : 0u;
            const uint32_t cslot = (wave_incl_scan(nw) - nw) - (uj - r0);
            const uint32_t nmine = r1 - r0;
            HeaderCapture<SU> cap;
            cap.wmask = lds->wmask;
            cap.slots = lds->slots;
            cap.hslot = lds->hslot;
            cap.count = 0;
            // (HCAP: no stream boundary but X1; H(A0) comes from the capture after the stream)
            const uint64_t bs[1] = {act && !AIPSTACK_FRAME_HCAP ? A0 : X1};
            uint32_t hA[1], hx;
            run.template prefixes<1, true>(bs, hA, hx, voff, cap);
            __builtin_amdgcn_wave_barrier();
            if constexpr (AIPSTACK_FRAME_HCAP)  // r0 < nseg: its segment was captured at cslot
                hA[0] = act && nmine ? lds->hslot[min(cslot, kHdrSlots - 1u)] : hx;
            // this lane's header blocks, and the next frame's first block (its start)
#pragma unroll
            for (int i = 0; i < kHdrSegs; ++i) {
                const u32x4 x = lds->slots[min(cslot + (uint32_t)i, kHdrSlots - 1u)];
                seg[i] = (uint32_t)i < nmine ? x : u32x4{0u, 0u, 0u, 0u};
            }
            const uint32_t cs_n = from_next_lane(cslot, 0u, lane);
            const uint32_t nm_n = from_next_lane(nmine, 0u, lane);
            const uint32_t hA_n = from_next_lane(hA[0], 0u, lane);
            // H(E) - H(A0 of the next frame): its first block's bytes below E
            const uint32_t pn =
                nm_n ? halves_below(lds->slots[min(cs_n, kHdrSlots - 1u)], (uint32_t)E & 15u) : 0u;
            fl = parse_lane<TX, true>(seg, S, len, hb_end);
            if constexpr (SECT) fsec = pick_sectors(seg, S, E, fl);
            const bool use = act && fl.l4;
            // H(l4s): l4s lies in the own header blocks (l4s - A0 <= 89 < hb_end)
            const uint32_t h_s = hA[0] + l4s_below(seg, (uint32_t)(fl.l4s - A0));
            // H(l4e): X1 (exact), or the next frame's start (its A0 plus the bytes below it
            // in its first block), or inside the own header blocks (a short frame with
            // padding); else (bytes after the IPv4 total length in a long frame) the chunk
            // takes the per-frame path below.
            const uint32_t e_off = (uint32_t)(fl.l4e - A0);
            uint32_t h_e = hx;
            bool far = false;
            const bool pad = use && fl.l4e != X1 && fl.l4e != E;
            if (use && fl.l4e != X1 && fl.l4e == E) h_e = hA_n + pn;
            if (__builtin_amdgcn_ballot_w64(pad)) {  // short frames with padding
                uint32_t hs[kHdrSegs];
#pragma unroll
                for (int i = 0; i < kHdrSegs; ++i) hs[i] = seg_halves(seg[i]);
                if (pad) {
                    if (e_off < hb_end)
                        h_e = hA[0] + hdr_below(seg, hs, e_off);
                    else
                        far = true;
                }
            }
            if (!__builtin_amdgcn_ballot_w64(far)) {
                r = fold16(h_e - h_s - fl.fhalf);  // exact halves-sum, < 2^32
                streamed = true;
            }
            if constexpr (TX && GATHER == kHdrCaptureTouch)
                asm volatile("" ::"v"(touch0), "v"(touch1));  // loaded, never used
            have_headers = true;  // the parse's inputs are the loaded header blocks
        } else {
            // (C') long runs: header blocks loaded per lane, stream prefixes at each frame's
            // L4 start and end. The first windows' loads go out behind the header loads
            // and arrive during the parse.
            load_headers();
            have_headers = true;
            StreamRun<SU, NT, AIPSTACK_FRAME_PREFETCH(SU)> run;
            run.begin(base, X1, voff);
            fl = parse_lane<TX, true>(seg, S, len, hb_end);
            // (no sector stores here: their 16 VGPRs would live through the stream)
            // frames without an L4 sum (and lanes past the batch) put both at X1
            const bool use = lane < cnt && fl.l4;
            const uint64_t bs[2] = {use ? fl.l4s : X1, use ? fl.l4e : X1};
            // The stream gives H at the start of each boundary's segment; the bytes of that
            // segment below the boundary come from header registers, once per chunk:
            //  - l4s lies in the frame's own header blocks (l4s - A0 <= 89 < hb_end);
            //  - l4e is usually the frame's end = the next frame's start, whose segment is
            //    the next lane's header block 0; or it lies in the own header blocks (a short
            //    frame with padding); or it is X1 (H(X1) is exact); else (bytes after the IPv4
            //    total length in a long frame) that one segment is loaded here.
            const uint64_t A0 = S & ~(uint64_t)15;
            u32x4 nb;
#pragma unroll
            for (int d = 0; d < 4; ++d) nb[d] = from_next_lane(seg[0][d], 0u, lane);
            const uint32_t p0 = use ? seg_below(seg, (uint32_t)(fl.l4s - A0)) : 0u;
            uint32_t p1 = 0;
            const bool e_mid = use && fl.l4e != X1;
            const uint32_t e_off = (uint32_t)(fl.l4e - A0);
            if (e_mid) {
                if (fl.l4e == E)
                    p1 = halves_below(nb, (uint32_t)E & 15u);
                else if (e_off < hb_end)
                    p1 = seg_below(seg, e_off);
            }
            const bool far = e_mid && fl.l4e != E && e_off >= hb_end;
            if (__builtin_amdgcn_ballot_w64(far)) {
                const u32x4 fs = load_segment<false>(
                    hrsrc, far ? (uint32_t)((fl.l4e & ~(uint64_t)15) - base) : 0xFFFFFFF0u, 0u);
                if (far) p1 = halves_below(fs, (uint32_t)fl.l4e & 15u);
            }
            uint32_t h[2], hx;
            run.template prefixes<2, true>(bs, h, hx, voff);
            r = fold16((h[1] + p1) - (h[0] + p0) - fl.fhalf);  // exact halves-sum, < 2^32
            streamed = true;
        }
      }
    }
    if (!streamed) {
        if (!have_headers) load_headers();
        if constexpr (STORE == kTxStoreLines) {
            // line stores: this lane's first 128 bytes (its header blocks: A0 = S on a
            // 128-byte-aligned slot) kept in LDS until the checksums are known
#pragma unroll
            for (int i = 0; i < kHdrSegs; ++i) lines[lane * kHdrSegs + i] = seg[i];
        }
        fl = parse_lane<TX, false>(seg, S, len, hb_end);
        // sector stores: ring slots (this is their only path), not the rare CSR chunks that
        // are not back to back (16 more VGPRs through the per-frame loop)
        if constexpr (SECT && !Desc::kStream) fsec = pick_sectors(seg, S, E, fl);
        uint32_t sums;
        if constexpr (!Desc::kStream && AIPSTACK_FRAME_SLOT_GATHER && Desc::kEdge) {
            // (C) ring slots: the remaining L4 bytes of the chunk's frames as one gathered
            // stream of just their segments (chksum_device.h; round 4)
            const uint32_t l4rest = lane < cnt ? (uint32_t)(fl.ce - fl.cs) : 0u;
            sums = sum_gathered_chunks<4, NT>(fl.cs, l4rest, lane, glds, nullptr);
        } else {
            const bool need = fl.ce != fl.cs;
            const LaneMeta meta = lane_meta(fl.cs, fl.ce);
            // (C) the remaining L4 bytes, one frame per wave, P frames' loads in flight
            NoMaskHook hook;
            sums = sum_lane_packets<U, P, AIPSTACK_ROWS_FRAMES, NT>(
                meta, __builtin_amdgcn_ballot_w64(need), lane, voff, not_lane0, hook);
        }
        // both parts (< 2^24 + 2^17), folded
        r = fold16(sums + fold16(fl.part));
    }
    // (D) per-lane finish: oriented by the L4 start
    if ((fl.l4s & 1u) == 0)  // L4 start even: little-endian pairing -> big-endian
        r = bswap16(r);
    const uint64_t m = (uint64_t)fl.words + r;
    uint32_t chk = (~fold16((uint32_t)m + (uint32_t)(m >> 32))) & 0xFFFFu;
    int v = fl.pre;
    if (TX) {
        if (fl.udp && chk == 0) chk = 0xFFFFu;                      // udp/IpUdpProto.h:176-178
    } else if (fl.l4) {
        v = chk == 0 ? AIPSTACK_RX_ACCEPT : AIPSTACK_RX_DROP_L4_CHKSUM;
    }
    FrameOut o;
    o.S = S;
    o.w0 = (fl.hchk & 0xFFFFu) | chk << 16;
    o.w1 = frame_w1(fl.fld, TX && fl.ip_ok, TX && fl.l4, v);
    o.fs = fsec;
    return o;
}

// Line stores (round 5, the send ring's in-place fill, tx_store = 2): a 2-byte field store
// leaves a partly written line that the memory side merges with the bytes around it (TX2K:
// ~49 us of its 170 for 2 M field stores, WRITE_SIZE ~52 B per frame). On a ring of slots
// that start on 128-byte boundaries, a frame's first line [S, S + 128) is its own and holds
// both fields of a 20-byte IPv4 header (bytes 24 and 36 / 40 / 50); the kernel loaded it
// whole for the parse. It is kept in LDS, the fields are patched in there, and the line is
// written back whole: eight lanes store one frame's line as 8 x 16 contiguous bytes in one
// wave instruction. Bytes of the line past a short frame are the slot's own slack, rewritten
// with the values just read. A field past byte 127 (IPv4 options) keeps its 2-byte store.
__device__ __forceinline__ void store_frame_lines(const FrameOut &o, uint32_t fld_line_ok,
                                                 uint64_t slot0, uint64_t stride, int cnt,
                                                 int lane, u32x4 *lines,
                                                 uint8_t *__restrict__ status, uint64_t i) {
    const bool act = lane < cnt;
    const bool wi = act && (o.w1 & 0x100u) != 0, wl = act && (o.w1 & 0x200u) != 0;
    const uint32_t fld = o.w1 & 0xFFu;
    typedef __attribute__((address_space(3))) uint16_t lds16;
    lds16 *lb = reinterpret_cast<lds16 *>(reinterpret_cast<uintptr_t>(lines)) +
                (uint32_t)lane * (kHdrSegs * 8u);
    const bool l_in = wl && fld + 2u <= 16u * kHdrSegs && fld_line_ok;
    if (wi && fld_line_ok) lb[12] = (uint16_t)bswap16(o.w0);  // byte 24
    if (l_in) lb[fld >> 1] = (uint16_t)bswap16(o.w0 >> 16);    // (fld is even)
    if (act) status[i] = (uint8_t)(o.w1 >> 16);
    if (!fld_line_ok) {  // slots off the 128-byte grid: the 2-byte stores
        if (wi) store_be16(o.S + 24, o.w0);
        if (wl) store_be16(o.S + fld, o.w0 >> 16);
        return;
    }
    if (wl && !l_in) store_be16(o.S + fld, o.w0 >> 16);
    const bool mine = wi || wl;  // this frame's line is written
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t sub = (uint32_t)lane & 7u;
    for (int f0 = 0; f0 < cnt; f0 += 8) {
        const int f = f0 + (lane >> 3);
        const int src = f < kWave ? f : 0;
        const bool w = __builtin_amdgcn_ds_bpermute(src << 2, mine ? 1 : 0) != 0;
        if (f < cnt && w) {
            const u32x4 x = lines[f * kHdrSegs + sub];
            *reinterpret_cast<u32x4 *>(slot0 + (uint64_t)f * stride + 16u * sub) = x;
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// The classic kernel: a wave walks its chunks and stores each chunk's results right after
// it. SPLIT (Tx only): lane j writes frame j's record (w0 | w1 << 32) to a workspace
// instead, and tx_scatter_kernel stores the fields after the whole read pass.
#ifndef AIPSTACK_FRAME_WAVES_PER_SIMD  // occupancy the register budget is fitted to
#define AIPSTACK_FRAME_WAVES_PER_SIMD 4
#endif
#ifndef AIPSTACK_FRAME_RX_WAVES_PER_SIMD  // the same for Rx verify (no field stores)
#define AIPSTACK_FRAME_RX_WAVES_PER_SIMD AIPSTACK_FRAME_WAVES_PER_SIMD
#endif
template <class Desc, bool TX, int U, int P, bool NT, int SU, bool SPLIT, int GATHER, int STORE>
__global__ __launch_bounds__(kBlock, TX ? AIPSTACK_FRAME_WAVES_PER_SIMD
                                        : AIPSTACK_FRAME_RX_WAVES_PER_SIMD) void frame_kernel(Desc desc, uint64_t n,
                                                       uint32_t chunks_per_wave,
                                                       uint32_t chunk_packets,
                                                       uint8_t *__restrict__ status,
                                                       uint64_t *__restrict__ records) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wave_in_block;
    const uint64_t cpk = chunk_packets;  // frames per chunk, 1..64 (launch_frames)
    const uint64_t nchunks = (n + cpk - 1) / cpk;
    uint64_t c = wave * chunks_per_wave;
    const uint64_t c_end = min(c + chunks_per_wave, nchunks);
    const uint32_t voff = (uint32_t)lane * 16u;
    const uint32_t not_lane0 = lane == 0 ? 0u : ~0u;
    constexpr bool kGather = SU > 0 && GATHER != kHdrLoads;
    __shared__ FrameLds lds[kGather ? kWavesPerBlock : 1];  // 9 KiB per wave (gathered stream)
    FrameLds *my = &lds[kGather ? wave_in_block : 0];
    constexpr bool kSlotGather = !Desc::kStream && AIPSTACK_FRAME_SLOT_GATHER && Desc::kEdge;
    __shared__ GatherLds glds[kSlotGather ? kWavesPerBlock : 1];  // ring slots' L4 stream
    GatherLds *mg = &glds[kSlotGather ? wave_in_block : 0];
    constexpr bool kLines = STORE == kTxStoreLines;  // ring slots only (launch_frames_slotted_d)
    __shared__ u32x4 line_lds[kLines ? kWavesPerBlock * kWave * kHdrSegs : 1];  // 8 KiB per wave
    u32x4 *ml = &line_lds[kLines ? wave_in_block * kWave * kHdrSegs : 0];
    for (; c < c_end; ++c) {
        const uint64_t p0 = c * cpk;
        int cnt;
        const FrameOut o = process_chunk<Desc, TX, U, P, NT, SU, GATHER, STORE>(
            desc, p0, n, (uint32_t)cpk, lane, voff, not_lane0, my, mg, ml, cnt);
        if constexpr (kLines && !Desc::kStream) {
            const uint64_t slot0 = desc.begin_chunk(p0, p0, lane).s0;
            const bool grid = ((slot0 | desc.stride) & 127u) == 0;  // wave-uniform
            store_frame_lines(o, grid ? 1u : 0u, slot0, desc.stride, cnt, lane, ml, status,
                              p0 + lane);
        } else if (lane < cnt) {
            if constexpr (SPLIT)
#if AIPSTACK_EXP_NO_RECORDS  // experiment: price of the record stores (wrong output)
                asm volatile("" ::"v"(o.w0), "v"(o.w1));
#elif AIPSTACK_FRAME_REC_NT
                // nontemporal (round 6): the records pass 126.5-130.9 us against 128.3-130.3
                // (profiles/r06/recnt), its probe 127.7 against 130.1; and a reader of the
                // records (the scatter pass, a D2H copy) then finds no freshly written lines
                // 
                __builtin_nontemporal_store((uint64_t)o.w0 | (uint64_t)o.w1 << 32,
                                            records + p0 + lane);
#else
                records[p0 + lane] = (uint64_t)o.w0 | (uint64_t)o.w1 << 32;
#endif
            else if constexpr (STORE == kTxStoreSectors)
                store_frame_sectors(o.S, o.w0, o.w1, o.fs, status, p0 + lane);
            else
                store_frame<TX>(o.S, o.w0, o.w1, status, p0 + lane);
        }
    }
}

template <class Desc, bool TX, bool SPLIT, int GATHER, int STORE = kTxStoreFields>
int launch_frames_g(const Desc &desc, uint64_t n, uint8_t *d_status, uint64_t *d_records,
                    hipStream_t stream, int cus) {
    // small batches: fewer frames per chunk, so that they spread over many waves (as the
    // checksum batches, chksum_kernels.hip pick_shape)
    uint32_t cpk = frames_per_chunk(n, cus);
    const int wpc = tuning_waves_per_cu();
    // Ring slots: 32-frame chunks, one per wave (RX2K, profiles/r03/ssweep: 130 us against
    // 136 with 64-frame chunks in runs per wave; 16-frame chunks 160; 1 segment per lane up
    // front instead of 2: 144, profiles/r03/fsweep)
    // Back-to-back frames too, since round 4: RX 120.6 us against 123.0 with 64-frame chunks,
    // the split Tx fill 161.4 against 168.9 (16-frame chunks 141.6 / 179.3;
    // profiles/r04/chunks).
    const bool big = cpk == (uint32_t)kWave && tuning_chunk_packets() == 0;
    const bool slots = !Desc::kStream && big;
    if (big) cpk = 32;
    const uint64_t nchunks = (n + cpk - 1) / cpk;
    // stream windows per group: round 4 measured 8 > 4 > off > 2 for RX and TX at steady
    // state; under the driver's protocol 4 runs RX 122.9-124.7 us against 124.5-127.3, the
    // records pass 130.5-132.3 against 132.3-132.9 and the split fill 161.1 against
    // 163.3-165.0 (profiles/r05/shape6)
    const int su = tuning_stream_windows(4);
    const uint64_t target_waves =
        (slots && wpc <= 0) ? nchunks : (uint64_t)cus * (wpc > 0 ? wpc : 128);
    uint64_t cpw = (nchunks + target_waves - 1) / target_waves;
    if (cpw == 0) cpw = 1;
    const uint64_t waves = (nchunks + cpw - 1) / cpw;
    const uint64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7FFFFFFFull || cpw > 0xFFFFFFFFull) return AIPSTACK_CHKSUM_EINVAL;
#define AIPSTACK_LAUNCH_FRAMES(P, SU)                                                          \
    hipLaunchKernelGGL((frame_kernel<Desc, TX, 2, P, AIPSTACK_FRAME_NT != 0, SU, SPLIT, GATHER,  \
                                     STORE>),                                                    \
                       dim3((unsigned)blocks), dim3(kBlock), tuning_lds_pad(0), stream, desc, n, \
                       (uint32_t)cpw,                                                           \
                       cpk, d_status, d_records)
#define AIPSTACK_LAUNCH_FRAMES_SU(P)                  \
    if constexpr (!Desc::kStream) {                   \
        AIPSTACK_LAUNCH_FRAMES(P, 0);                 \
    } else {                                          \
        switch (su) {                                 \
            case 0: AIPSTACK_LAUNCH_FRAMES(P, 0); break; \
            case 2: AIPSTACK_LAUNCH_FRAMES(P, 2); break; \
            case 8: AIPSTACK_LAUNCH_FRAMES(P, 8); break; \
            default: AIPSTACK_LAUNCH_FRAMES(P, 4);     \
        }                                             \
    }
#ifdef AIPSTACK_ALL_VARIANTS  // frames in flight 2 / 8: sweep builds only (tools/build_variant.sh)
    switch (tuning_frames_in_flight()) {
        case 2: AIPSTACK_LAUNCH_FRAMES_SU(2); break;
        case 8: AIPSTACK_LAUNCH_FRAMES_SU(8); break;
        default: AIPSTACK_LAUNCH_FRAMES_SU(4);
    }
#else
    AIPSTACK_LAUNCH_FRAMES_SU(4);
#endif
#undef AIPSTACK_LAUNCH_FRAMES_SU
#undef AIPSTACK_LAUNCH_FRAMES
    return check_hip(hipGetLastError());
}

// Rx verify; Tx fill in one pass; the split fill's read pass (SPLIT), followed by the
// scatter pass unless `scatter` is false (the records-only call). Where the header segments
// come from (GATHER): Rx and the records-only pass capture them from the stream; both fills
// that store fields in place capture them too and touch the two field lines up front at the
// default cache policy, so that the stores find those lines cached: split fill 168 vs 178 us,
// one pass 174 vs 186, against per-lane header loads.
template <bool TX, bool SPLIT = false>
int launch_frames(const void *d_base, const uint64_t *d_offsets, uint64_t n, uint8_t *d_status,
                  uint64_t *d_records, hipStream_t stream, bool scatter = true) {
    const int cus = device_cu_count(stream);
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    CsrDesc desc{(uint64_t)(uintptr_t)d_base, d_offsets};
    int st;
    if constexpr (TX && !SPLIT) {
      if (tuning_tx_store(kTxStoreDefault) == kTxStoreSectors) {
        // whole sectors need no line in the caches: captured headers, no touches by default
        if (tuning_tx_header_mode(kHdrCapture) == kHdrCaptureTouch)
            st = launch_frames_g<CsrDesc, true, false, kHdrCaptureTouch, kTxStoreSectors>(
                desc, n, d_status, d_records, stream, cus);
        else
            st = launch_frames_g<CsrDesc, true, false, kHdrCapture, kTxStoreSectors>(
                desc, n, d_status, d_records, stream, cus);
        return st;
      }
    }
    if constexpr (TX) {
        const int mode = tuning_tx_header_mode(SPLIT && !scatter ? kHdrCapture : kHdrCaptureTouch);
        if (mode == kHdrCaptureTouch)
            st = launch_frames_g<CsrDesc, true, SPLIT, kHdrCaptureTouch>(desc, n, d_status, d_records,
                                                                        stream, cus);
        else if (mode == kHdrCapture)
            st = launch_frames_g<CsrDesc, true, SPLIT, kHdrCapture>(desc, n, d_status, d_records,
                                                                   stream, cus);
        else
            st = launch_frames_g<CsrDesc, true, SPLIT, kHdrLoads>(desc, n, d_status, d_records,
                                                                 stream, cus);
    } else {
        st = launch_frames_g<CsrDesc, false, SPLIT, kHdrCapture>(desc, n, d_status, d_records,
                                                                stream, cus);
    }
    if (st != AIPSTACK_CHKSUM_OK) return st;
    if (SPLIT && scatter) {
        const uint64_t sblocks = min((n + kBlock - 1) / kBlock, (uint64_t)cus * 64);
        hipLaunchKernelGGL(tx_scatter_kernel, dim3((unsigned)sblocks), dim3(kBlock), 0, stream,
                           desc.base, d_offsets, d_records, d_status, n);
        return check_hip(hipGetLastError());
    }
    return AIPSTACK_CHKSUM_OK;
}

}  // namespace

// Ring slots (SlottedDesc): per-lane header loads, then the L4 bytes past the header blocks as
// one gathered stream of the chunk's frames -- or, for slots read over the link from host
// memory (the engine's zero-copy pieces, host_bytes), one frame per wave instruction pair
// (SlottedHostDesc), where the gathered stream's second read of an edge segment would cross
// the link again. No stream mode, so the header capture does not apply either.
template <bool TX, bool SPLIT, class D>
int launch_frames_slotted_d(const D &desc, uint64_t n, uint8_t *d_status, uint64_t *d_records,
                            hipStream_t stream, int cus) {
    if constexpr (TX && !SPLIT) {
        const int ts = tuning_tx_store(kTxStoreDefault);
        if (ts == kTxStoreSectors)
            return launch_frames_g<D, true, false, kHdrLoads, kTxStoreSectors>(
                desc, n, d_status, d_records, stream, cus);
        // line stores: device-memory rings (over the link a line store is no cheaper)
        if constexpr (!std::is_same<D, SlottedHostDesc>::value)
            if (ts == kTxStoreLines)
                return launch_frames_g<D, true, false, kHdrLoads, kTxStoreLines>(
                    desc, n, d_status, d_records, stream, cus);
    }
    return launch_frames_g<D, TX, SPLIT, kHdrLoads>(desc, n, d_status, d_records, stream, cus);
}

template <bool TX, bool SPLIT>
int launch_frames_slotted(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                          uint64_t n, uint8_t *d_status, uint64_t *d_records, hipStream_t stream,
                          bool host_bytes = false) {
    const int cus = device_cu_count(stream);
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    SlottedDesc desc;
    desc.base = (uint64_t)(uintptr_t)d_base;
    desc.stride = slot_stride;
    desc.lens = d_len;
    desc.cap = (uint32_t)(slot_stride < AIPSTACK_CHKSUM_MAX_LEN ? slot_stride : AIPSTACK_CHKSUM_MAX_LEN);
    int st;
    if (host_bytes) {
        SlottedHostDesc h;
        static_cast<SlottedDesc &>(h) = desc;
        st = launch_frames_slotted_d<TX, SPLIT>(h, n, d_status, d_records, stream, cus);
    } else {
        st = launch_frames_slotted_d<TX, SPLIT>(desc, n, d_status, d_records, stream, cus);
    }
    if (st != AIPSTACK_CHKSUM_OK || !SPLIT || !d_status) return st;
    // the split slotted fill's scatter pass (records pass above: d_status is null for the
    // records-only call)
    const uint64_t sblocks = min((n + kBlock - 1) / kBlock, (uint64_t)cus * 64);
    hipLaunchKernelGGL(tx_scatter_slotted_kernel, dim3((unsigned)sblocks), dim3(kBlock), 0, stream,
                       desc.base, slot_stride, d_records, d_status, n);
    return check_hip(hipGetLastError());
}

int take_violations_frames(uint32_t *mask, bool clear) {
    return take_violations_here(mask, clear);
}

int rx_verify_slotted_from(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                           uint64_t n, uint8_t *d_verdict, void *stream, bool host_bytes) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_len || !d_verdict || slot_stride == 0 ||
        slot_stride > kMaxSlotStride || n > (1ull << 40))
        return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames_slotted<false, false>(d_base, slot_stride, d_len, n, d_verdict, nullptr,
                                               (hipStream_t)stream, host_bytes);
}

int tx_fill_records_slotted_from(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                                 uint64_t n, uint64_t *d_records, void *stream, bool host_bytes) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_len || !d_records || slot_stride == 0 ||
        slot_stride > kMaxSlotStride || n > (1ull << 40) ||
        ((uintptr_t)d_records & 7u) != 0)
        return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames_slotted<true, true>(d_base, slot_stride, d_len, n, nullptr, d_records,
                                             (hipStream_t)stream, host_bytes);
}

}  // namespace aipstack_amd

using namespace aipstack_amd;

extern "C" int aipstack_chksum_rx_verify(const void *d_base, const uint64_t *d_offsets, uint64_t n,
                                         uint8_t *d_verdict, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_verdict || n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames<false>(d_base, d_offsets, n, d_verdict, nullptr, (hipStream_t)stream);
}

extern "C" int aipstack_chksum_tx_fill(void *d_base, const uint64_t *d_offsets, uint64_t n,
                                       uint8_t *d_status, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_status || n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames<true>(d_base, d_offsets, n, d_status, nullptr, (hipStream_t)stream);
}

extern "C" uint64_t aipstack_chksum_tx_fill_workspace_bytes(uint64_t n) {
    return n * sizeof(uint64_t);
}

extern "C" int aipstack_chksum_tx_fill_records(const void *d_base, const uint64_t *d_offsets,
                                               uint64_t n, uint64_t *d_records, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_records || n > (1ull << 40) ||
        ((uintptr_t)d_records & 7u) != 0)
        return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames<true, true>(const_cast<void *>(d_base), d_offsets, n, nullptr, d_records,
                                     (hipStream_t)stream, false);
}

extern "C" int aipstack_chksum_tx_fill_split(void *d_base, const uint64_t *d_offsets, uint64_t n,
                                             uint8_t *d_status, void *d_workspace,
                                             uint64_t workspace_bytes, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_status || !d_workspace || n > (1ull << 40) ||
        workspace_bytes < aipstack_chksum_tx_fill_workspace_bytes(n) ||
        ((uintptr_t)d_workspace & 7u) != 0)
        return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames<true, true>(d_base, d_offsets, n, d_status,
                                     static_cast<uint64_t *>(d_workspace), (hipStream_t)stream);
}

extern "C" int aipstack_chksum_rx_verify_slotted(const void *d_base, uint64_t slot_stride,
                                                 const uint32_t *d_len, uint64_t n,
                                                 uint8_t *d_verdict, void *stream) {
    return rx_verify_slotted_from(d_base, slot_stride, d_len, n, d_verdict, stream, false);
}

extern "C" int aipstack_chksum_tx_fill_slotted(void *d_base, uint64_t slot_stride,
                                               const uint32_t *d_len, uint64_t n,
                                               uint8_t *d_status, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_len || !d_status || slot_stride == 0 ||
        slot_stride > kMaxSlotStride || n > (1ull << 40))
        return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames_slotted<true, false>(d_base, slot_stride, d_len, n, d_status, nullptr,
                                              (hipStream_t)stream);
}

extern "C" int aipstack_chksum_tx_fill_slotted_split(void *d_base, uint64_t slot_stride,
                                                     const uint32_t *d_len, uint64_t n,
                                                     uint8_t *d_status, void *d_workspace,
                                                     uint64_t workspace_bytes, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_len || !d_status || !d_workspace || slot_stride == 0 ||
        slot_stride > kMaxSlotStride || n > (1ull << 40) ||
        workspace_bytes < aipstack_chksum_tx_fill_workspace_bytes(n) ||
        ((uintptr_t)d_workspace & 7u) != 0)
        return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames_slotted<true, true>(d_base, slot_stride, d_len, n, d_status,
                                             static_cast<uint64_t *>(d_workspace),
                                             (hipStream_t)stream);
}

extern "C" int aipstack_chksum_tx_fill_records_slotted(const void *d_base, uint64_t slot_stride,
                                                       const uint32_t *d_len, uint64_t n,
                                                       uint64_t *d_records, void *stream) {
    return tx_fill_records_slotted_from(d_base, slot_stride, d_len, n, d_records, stream, false);
}
