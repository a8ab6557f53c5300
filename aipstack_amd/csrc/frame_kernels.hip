// aipstack_amd -- frame-level batch kernels on raw Ethernet frames:
//   Rx verify: the reference's receive-path checksum decisions for n frames at once
//              (eth/EthIpIface.h:367-390, ip/IpStack.h:936-1018 and :1093-1130,
//              tcp/IpTcpProto_input.h:68-100, udp/IpUdpProto.h:470-490, :631-652);
//   Tx fill:   the checksums the reference's send paths write, filled in place
//              (ip/IpStack.h:425-453, tcp/IpTcpProto_output.h:1251-1277,
//              udp/IpUdpProto.h:164-179, ip/IpStack.h:1164-1190).
//
// One wave per frame, 64-frame chunks per wave (CSR frame offsets, as the checksum CSR
// batch). A frame is read ONCE from HBM: the aligned segments covering it are loaded
// through a range-checked buffer descriptor (as PacketLoad does); lanes 0-7 copy the first
// 128 bytes into the wave's LDS slot, where the Ethernet / IPv4 / L4 header fields are
// parsed and the IPv4 header words are summed (one lane per word); the L4 checksum is a
// masked sum over the same loaded segments (segment range, head/tail byte masks and, for
// Tx, the checksum field itself masked out), reduced across the wave with DPP.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "aipstack_amd/chksum.h"
#include "chksum_device.h"
#include "chksum_internal.h"

namespace aipstack_amd {
namespace {

constexpr int kStageBytes = 128;  // bytes [A0, A0 + 128) cover frame bytes [0, 112)

// Zero bytes b and b+1 (b+1 < 16) of a 16-byte segment, as four dwords.
constexpr uint32_t not_pair_dword(int b, int d) {
    uint32_t m = 0xFFFFFFFFu;
    for (int i = 0; i < 4; ++i)
        if (4 * d + i == b || 4 * d + i == b + 1) m &= ~(0xFFu << (8 * i));
    return m;
}
#define AIPSTACK_NOT_PAIR(b) \
    {not_pair_dword(b, 0), not_pair_dword(b, 1), not_pair_dword(b, 2), not_pair_dword(b, 3)}
__constant__ uint32_t kMaskNotPair[16][4] = {
    AIPSTACK_NOT_PAIR(0),  AIPSTACK_NOT_PAIR(1),  AIPSTACK_NOT_PAIR(2),  AIPSTACK_NOT_PAIR(3),
    AIPSTACK_NOT_PAIR(4),  AIPSTACK_NOT_PAIR(5),  AIPSTACK_NOT_PAIR(6),  AIPSTACK_NOT_PAIR(7),
    AIPSTACK_NOT_PAIR(8),  AIPSTACK_NOT_PAIR(9),  AIPSTACK_NOT_PAIR(10), AIPSTACK_NOT_PAIR(11),
    AIPSTACK_NOT_PAIR(12), AIPSTACK_NOT_PAIR(13), AIPSTACK_NOT_PAIR(14), AIPSTACK_NOT_PAIR(15)};
#undef AIPSTACK_NOT_PAIR

__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
    return __builtin_bswap32(x);
}

// Wave-uniform read of 4 frame bytes [x, x+4) (x relative to A0) from the LDS stage, as a
// little-endian dword.
__device__ __forceinline__ uint32_t stage4(const uint32_t *st, int x) {
    const uint32_t lo = st[x >> 2], hi = st[(x >> 2) + 1];
    const uint32_t r = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(x & 3));
    return __builtin_amdgcn_readfirstlane(r);
}
// This lane's share of the masked sum of the frame bytes [r0, r1) relative to A0, except
// the two bytes at fx (fx < 0: none), over the segments the wave has loaded (group 0 in
// fl.v, further groups loaded here): the lane's 18-bit folded ones'-complement sum. Summed
// over the wave (< 2^24) it is congruent mod 0xFFFF to the little-endian 16-bit halves of
// those bytes and 0 iff they are all 0.
template <int U, bool NT>
__device__ __forceinline__ uint32_t range_lane(PacketLoad<U, NT> &fl, int r0, int r1, int fx,
                                               int lane, uint32_t voff) {
    if (r1 <= r0)
        return 0;
    const int k0 = r0 >> 4, k1 = (r1 - 1) >> 4;
    const u32x4 hm = load_mask(kMaskFrom[r0 & 15]);
    const u32x4 tm = load_mask(kMaskTo[r1 - 16 * k1]);
    const int kx = fx >= 0 ? fx >> 4 : -2;
    const int bx = fx >= 0 ? fx & 15 : 0;
    const u32x4 xm = load_mask(kMaskNotPair[bx]);   // bytes bx, bx+1 of segment kx
    const u32x4 xm2 = load_mask(kMaskFrom[1]);      // byte 0 of segment kx+1 (bx == 15)
    const int kx2 = (fx >= 0 && bx == 15) ? kx + 1 : -2;
    Eac a0, a1;
    for (int g = 0; g <= k1; g += kWave * U) {
        if (g > 0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                fl.v[u] = load_segment<NT>(fl.rsrc, voff, (uint32_t)((g + u * kWave) * 16));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = g + u * kWave + lane;
            const uint32_t in = (k >= k0 && k <= k1) ? ~0u : 0u;
            u32x4 x = fl.v[u];
            apply_mask(x, hm, k == k0 ? 0u : ~0u);
            apply_mask(x, tm, k == k1 ? 0u : ~0u);
            if (fx >= 0) {  // wave-uniform: Tx only
                apply_mask(x, xm, k == kx ? 0u : ~0u);
                apply_mask(x, xm2, k == kx2 ? 0u : ~0u);
            }
            a0.add(x[0] & in);
            a1.add(x[1] & in);
            a0.add(x[2] & in);
            a1.add(x[3] & in);
        }
    }
    const uint32_t s0 = a0.finish(), s1 = a1.finish();
    return (s0 & 0xFFFFu) + (s0 >> 16) + (s1 & 0xFFFFu) + (s1 >> 16);
}

// Two wave sums at once: the two DPP chains interleave, so neither waits on its own
// data-hazard slots. Results wave-uniform.
__device__ __forceinline__ void wave_sum2(uint32_t &a, uint32_t &b) {
#define AIPSTACK_DPP2(ctrl, rowmask)                                                     \
    a += __builtin_amdgcn_update_dpp(0u, a, ctrl, rowmask, 0xF, false);                  \
    b += __builtin_amdgcn_update_dpp(0u, b, ctrl, rowmask, 0xF, false);
    AIPSTACK_DPP2(0x111, 0xF)
    AIPSTACK_DPP2(0x112, 0xF)
    AIPSTACK_DPP2(0x114, 0xF)
    AIPSTACK_DPP2(0x118, 0xF)
    AIPSTACK_DPP2(0x142, 0xA)
    AIPSTACK_DPP2(0x143, 0xC)
#undef AIPSTACK_DPP2
    a = __builtin_amdgcn_readlane(a, 63);
    b = __builtin_amdgcn_readlane(b, 63);
}

// IpChksumAccumulator(words).getChksum() over a little-endian range sum `t` of bytes that
// start at absolute address `start`: orient (big-endian pairing from `start`), add the
// header/pseudo-header words with end-around carry, fold, invert (Chksum.h:245-300).
__device__ __forceinline__ uint32_t finish_chksum(uint32_t words, uint32_t t, uint64_t start) {
    uint32_t r = fold16(t);
    if ((start & 1) == 0)
        r = bswap16(r);
    const uint64_t m = (uint64_t)words + r;
    return (~fold16((uint32_t)m + (uint32_t)(m >> 32))) & 0xFFFFu;
}

__device__ __forceinline__ void store_be16(uint64_t addr, uint32_t v) {
    uint8_t *p = reinterpret_cast<uint8_t *>(addr);
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

// One frame, its segment loads already issued into fl: stage the header, parse, sum,
// decide (and for Tx, write the checksums). Returns the AIPSTACK_RX_* verdict / status.
template <bool TX, int U, bool NT>
__device__ __forceinline__ int process_frame(PacketLoad<U, NT> &fl, uint64_t S, int len,
                                             uint32_t *st, int lane, uint32_t voff) {
    const int rs = fl.rel_s;
    // stage frame bytes [0, 112) (segments 0..7) in this wave's LDS slot
    if (lane < kStageBytes / 16) {
        st[4 * lane + 0] = fl.v[0][0];
        st[4 * lane + 1] = fl.v[0][1];
        st[4 * lane + 2] = fl.v[0][2];
        st[4 * lane + 3] = fl.v[0][3];
    }
    __builtin_amdgcn_wave_barrier();
    // all fixed-offset header dwords in one batch of LDS reads
    const uint32_t w12 = stage4(st, rs + 12);  // EtherType | version/IHL | TOS
    const uint32_t w16 = stage4(st, rs + 16);  // total length | ident
    const uint32_t w20 = stage4(st, rs + 20);  // flags/offset | TTL | protocol
    const uint32_t w28 = stage4(st, rs + 28);
    const uint32_t w24 = stage4(st, rs + 24);
    const uint32_t w32 = stage4(st, rs + 32);
    const uint32_t ethertype = ((w12 & 0xFFu) << 8) | ((w12 >> 8) & 0xFFu);
    // ---- Ethernet (EthIpIface.h:370-384)
    if (len < 14 || ethertype != 0x0800)
        return AIPSTACK_RX_NOT_IP4;
    // ---- IPv4 header checks (IpStack.h:938-990)
    const int plen = len - 14;
    if (plen < 20)
        return AIPSTACK_RX_DROP_IP_MALFORMED;
    const uint32_t vihl = (w12 >> 16) & 0xFFu;
    int hl = 20;
    if (vihl != 0x45) {
        hl = (int)(vihl & 0xFu) * 4;
        if ((vihl >> 4) != 4 || hl < 20 || hl > plen)
            return AIPSTACK_RX_DROP_IP_MALFORMED;
    }
    const int total_len = (int)(((w16 & 0xFFu) << 8) | ((w16 >> 8) & 0xFFu));
    if (total_len < hl || total_len > plen)
        return AIPSTACK_RX_DROP_IP_MALFORMED;
    const uint32_t flags_off = ((w20 & 0xFFu) << 8) | ((w20 >> 8) & 0xFFu);
    const bool fragment = (flags_off & 0x3FFFu) != 0;                  // IpStack.h:1020
    const uint32_t proto = w20 >> 24;
    const uint32_t src = bswap32((w24 >> 16) | (w28 << 16));
    const uint32_t dst = bswap32((w28 >> 16) | (w32 << 16));
    // ---- L4: which bytes the checksum covers, or a verdict without one
    const int dg = 14 + hl;
    const int dlen = total_len - hl;
    const uint32_t pseudo_sa = (src >> 16) + (src & 0xFFFFu) + (dst >> 16) + (dst & 0xFFFFu);
    int l4len = -1, fld = 0, l4verdict = AIPSTACK_RX_ACCEPT_OTHER;
    uint32_t words = 0;
    bool udp = false;
    if (!fragment) {
        if (proto == 6) {                                              // TCP
            if (dlen < 20) l4verdict = AIPSTACK_RX_DROP_L4_MALFORMED;
            else { l4len = dlen; fld = dg + 16; words = pseudo_sa + 6 + (uint32_t)dlen; }
        } else if (proto == 17) {                                      // UDP
            if (dlen < 8) {
                l4verdict = AIPSTACK_RX_DROP_L4_MALFORMED;
            } else {
                const uint32_t w = stage4(st, rs + dg + 4);
                const int ulen = (int)(((w & 0xFFu) << 8) | ((w >> 8) & 0xFFu));
                const uint32_t ucs = ((w >> 8) & 0xFF00u) | (w >> 24);
                if (ulen < 8 || ulen > dlen) {
                    l4verdict = AIPSTACK_RX_DROP_L4_MALFORMED;
                } else if (!TX && ucs == 0) {
                    l4verdict = AIPSTACK_RX_ACCEPT_NO_CHKSUM;          // IpUdpProto.h:637
                } else {
                    l4len = ulen; fld = dg + 6; words = pseudo_sa + 17 + (uint32_t)ulen;
                    udp = true;
                }
            }
        } else if (proto == 1) {                                       // ICMP
            if (dlen < 8) l4verdict = AIPSTACK_RX_DROP_L4_MALFORMED;
            else { l4len = dlen; fld = dg + 2; }
        }
    }
    // ---- both sums, one interleaved reduction: header word `lane` (LDS), L4 bytes (regs)
    uint32_t hw = 0;
    if (2 * lane < hl && !(TX && lane == 5)) {
        const uint8_t *sb = reinterpret_cast<const uint8_t *>(st);
        const int o = rs + 14 + 2 * lane;
        hw = ((uint32_t)sb[o] << 8) | sb[o + 1];
    }
    const int r0 = rs + dg;
    uint32_t lw = l4len >= 0 ? range_lane<U, NT>(fl, r0, r0 + l4len, TX ? rs + fld : -1, lane, voff)
                             : 0u;
    wave_sum2(hw, lw);
    const uint32_t hchk = (~fold16(hw)) & 0xFFFFu;                     // IpStack.h:1016
    if (TX) {
        if (lane == 0) store_be16(S + 24, hchk);
    } else if (hchk != 0) {
        return AIPSTACK_RX_DROP_IP_CHKSUM;
    }
    if (fragment)
        return AIPSTACK_RX_FRAGMENT;
    if (l4len < 0)
        return l4verdict;
    uint32_t chk = finish_chksum(words, lw, S + (uint64_t)dg);
    if (TX) {
        if (udp && chk == 0) chk = 0xFFFFu;                            // IpUdpProto.h:176-178
        if (lane == 0) store_be16(S + (uint64_t)fld, chk);
        return AIPSTACK_RX_ACCEPT;
    }
    return chk == 0 ? AIPSTACK_RX_ACCEPT : AIPSTACK_RX_DROP_L4_CHKSUM;
}

template <bool TX, int U, int P, bool NT>
__global__ __launch_bounds__(kBlock) void frame_kernel(CsrDesc desc, uint64_t n,
                                                       uint32_t chunks_per_wave,
                                                       uint8_t *__restrict__ status) {
    __shared__ uint32_t stage_all[kWavesPerBlock][P][kStageBytes / 4 + 1];
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wave_in_block;
    const uint64_t nchunks = (n + kWave - 1) / kWave;
    uint64_t c = wave * chunks_per_wave;
    const uint64_t c_end = min(c + chunks_per_wave, nchunks);
    const uint32_t voff = (uint32_t)lane * 16u;

    for (; c < c_end; ++c) {
        const uint64_t p0 = c * kWave;
        const auto chunk = desc.begin_chunk(p0, n, lane);
        const int cnt = (int)min((uint64_t)kWave, n - p0);
        uint32_t verdicts = 0;
        for (int j0 = 0; j0 < cnt; j0 += P) {
            PacketLoad<U, NT> fl[P];
            uint64_t S[P];
            int len[P];
#pragma unroll
            for (int q = 0; q < P; ++q) {  // P frames' loads in flight
                uint64_t s = 0, e = 0;
                if (j0 + q < cnt)
                    desc.bounds(chunk, j0 + q, s, e);
                const uint64_t l64 = e - s;
                len[q] = l64 >= (1ull << 31) ? 0 : (int)l64;  // out of contract: empty
                S[q] = s;
                fl[q].issue(s, s + (uint64_t)len[q], voff);
            }
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const int v = process_frame<TX, U, NT>(fl[q], S[q], len[q],
                                                       stage_all[wave_in_block][q], lane, voff);
                verdicts = (lane == j0 + q) ? (uint32_t)v : verdicts;
            }
            // the stage slots are rewritten by the next frames: reads before writes
            __builtin_amdgcn_wave_barrier();
        }
        if (lane < cnt)
            status[p0 + lane] = (uint8_t)verdicts;
    }
}

template <bool TX>
int launch_frames(const void *d_base, const uint64_t *d_offsets, uint64_t n, uint8_t *d_status,
                  hipStream_t stream) {
    const uint64_t nchunks = (n + kWave - 1) / kWave;
    const int cus = device_cu_count();
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    const uint64_t target_waves = (uint64_t)cus * 128;
    uint64_t cpw = (nchunks + target_waves - 1) / target_waves;
    if (cpw == 0) cpw = 1;
    const uint64_t waves = (nchunks + cpw - 1) / cpw;
    const uint64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7FFFFFFFull || cpw > 0xFFFFFFFFull) return AIPSTACK_CHKSUM_EINVAL;
    CsrDesc desc{(uint64_t)(uintptr_t)d_base, d_offsets};
    switch (tuning_frames_in_flight()) {
        case 1:
            hipLaunchKernelGGL((frame_kernel<TX, 2, 1, true>), dim3((unsigned)blocks), dim3(kBlock),
                               0, stream, desc, n, (uint32_t)cpw, d_status);
            break;
        case 4:
            hipLaunchKernelGGL((frame_kernel<TX, 2, 4, true>), dim3((unsigned)blocks), dim3(kBlock),
                               0, stream, desc, n, (uint32_t)cpw, d_status);
            break;
        default:
            hipLaunchKernelGGL((frame_kernel<TX, 2, 2, true>), dim3((unsigned)blocks), dim3(kBlock),
                               0, stream, desc, n, (uint32_t)cpw, d_status);
    }
    return check_hip(hipGetLastError());
}

}  // namespace
}  // namespace aipstack_amd

using namespace aipstack_amd;

extern "C" int aipstack_chksum_rx_verify(const void *d_base, const uint64_t *d_offsets, uint64_t n,
                                         uint8_t *d_verdict, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_verdict || n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames<false>(d_base, d_offsets, n, d_verdict, (hipStream_t)stream);
}

extern "C" int aipstack_chksum_tx_fill(void *d_base, const uint64_t *d_offsets, uint64_t n,
                                       uint8_t *d_status, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_status || n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    return launch_frames<true>(d_base, d_offsets, n, d_status, (hipStream_t)stream);
}
