// aipstack_amd -- CDNA4 (gfx950) batch Internet-checksum kernels + their C-ABI launchers.
//
// What is computed (reference semantics, src/aipstack/infra/Chksum.h):
//   IpChksumInverted(p, L)  (Chksum.h:77-99): ones'-complement sum of the big-endian
//   16-bit words of p[0..L), odd tail byte as a high byte, folded twice to 16 bits.
//   IpChksum = ~that (Chksum.h:122-125). IpChksumAccumulator(State s).getChksum(buf)
//   (Chksum.h:171-174, 263-315) = the same sum seeded with the 32-bit state s.
//
// How (MI355X-first; see DESIGN.md "Kernel arithmetic"):
//   * One packet per 64-lane wavefront at a time. A wave owns a contiguous run of
//     64-packet chunks; lane j of the wave keeps packet j's result and the chunk ends
//     in ONE coalesced 128-byte store of 64 uint16 results.
//   * A packet [S, E) (absolute byte addresses) is read as the 16-byte-aligned
//     segments A0 = S & ~15, A0+16, ... covering it: lane k loads segment k with a
//     global_load_dwordx4 (a wave instruction reads 1 KiB contiguous). Every segment
//     loaded contains at least one byte of the packet, so no load leaves the pages
//     of the caller's buffer (a 16-byte block never straddles a page).
//   * Segments are summed unmasked: each dword as its two little-endian 16-bit halves
//     into a per-lane uint32 (exact up to 4 MiB packets); the 64 lane sums are added by
//     a DPP reduction. The bytes of the head and tail segments that lie outside
//     [S, E) are read back with v_readlane and subtracted on the scalar unit, so the
//     sum is exact (not just congruent) and can be folded like the reference's.
//   * Little-endian halves at even absolute addresses pair byte (2i, 2i+1) with 2i as
//     the LOW byte; the reference pairs relative to the packet start with p[0] as the
//     HIGH byte. So the folded sum is byte-swapped iff S is even (for odd S the two
//     pairings coincide with the roles already swapped). Byte-swap is x*256 mod 0xFFFF,
//     and folding never turns a nonzero sum into 0, so the 0x0000-vs-0xFFFF
//     representation matches the reference exactly (0 iff every byte is 0).
//   * HBM-bound integer reduction: no MFMA, no LDS needed (the cross-lane sum is DPP).

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "aipstack_amd/chksum.h"
#include "chksum_internal.h"

namespace aipstack_amd {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

// ---------------------------------------------------------------------------------
// Packet descriptors. A wave walks 64-packet chunks; per chunk the descriptor may fetch
// per-lane data (lane j <-> packet j of the chunk), then gives
//   bounds(j)      the wave-uniform absolute byte range [S, E) of packet j (SGPRs), and
//   lane_start()   the start address of this lane's packet (VGPR, for the finalisation).
// ---------------------------------------------------------------------------------

// A copy of x in a fresh VGPR. The compiler waits for the load that produced x here,
// once per chunk, instead of before every later v_readlane of it (where, inside the
// packet loop, the wait would also drain the packet loads already in flight).
__device__ __forceinline__ uint32_t settle(uint32_t x) {
    uint32_t y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
    return y;
}

struct StridedDesc {
    static constexpr bool kCsr = false;
    uint64_t base;    // absolute address of packet 0
    uint64_t stride;  // bytes between packet starts
    uint32_t len;     // bytes per packet

    struct Chunk {
        uint64_t s0;  // start of the chunk's first packet
    };
    __device__ __forceinline__ Chunk begin_chunk(uint64_t p0, uint64_t, int) const {
        return Chunk{base + p0 * stride};
    }
    __device__ __forceinline__ void bounds(const Chunk &c, int j, uint64_t &S,
                                           uint64_t &E) const {
        S = c.s0 + (uint64_t)j * stride;
        E = S + len;
    }
    __device__ __forceinline__ uint64_t lane_start(const Chunk &c, int lane) const {
        return c.s0 + (uint64_t)lane * stride;
    }
    __device__ __forceinline__ uint32_t lane_seed(const Chunk &) const { return 0; }
};

struct CsrDesc {
    static constexpr bool kCsr = true;
    uint64_t base;            // absolute address offsets are relative to
    const uint64_t *offsets;  // n+1 byte offsets

    struct Chunk {
        uint32_t off_lo, off_hi;  // lane j: offsets[c0 + j] (settled)
        uint64_t end_off;         // offsets[min(c0 + 64, n)] (scalar load)
    };
    // Lane j fetches offsets[c0 + j]: one coalesced 512-B load per chunk.
    __device__ __forceinline__ Chunk begin_chunk(uint64_t c0, uint64_t n, int lane) const {
        Chunk c;
        const uint64_t i = c0 + (uint64_t)lane;
        const uint64_t o = offsets[i <= n ? i : n];
        c.off_lo = settle((uint32_t)o);
        c.off_hi = settle((uint32_t)(o >> 32));
        const uint64_t last = c0 + kWave < n ? c0 + kWave : n;
        c.end_off = offsets[last];
        return c;
    }
    __device__ __forceinline__ uint64_t offset_of(const Chunk &c, int j) const {
        const uint32_t lo = __builtin_amdgcn_readlane(c.off_lo, j);
        const uint32_t hi = __builtin_amdgcn_readlane(c.off_hi, j);
        return ((uint64_t)hi << 32) | lo;
    }
    __device__ __forceinline__ void bounds(const Chunk &c, int j, uint64_t &S,
                                           uint64_t &E) const {
        S = base + offset_of(c, j);
        E = base + ((j + 1 < kWave) ? offset_of(c, j + 1) : c.end_off);
    }
    __device__ __forceinline__ uint64_t lane_start(const Chunk &c, int) const {
        return base + (((uint64_t)c.off_hi << 32) | c.off_lo);
    }
    __device__ __forceinline__ uint32_t lane_seed(const Chunk &) const { return 0; }
};

struct SeededCsrDesc : CsrDesc {
    const uint32_t *states;  // n accumulator states (IpChksumAccumulator::State)

    struct Chunk : CsrDesc::Chunk {
        uint32_t state;  // lane j: states[c0 + j]
    };
    __device__ __forceinline__ Chunk begin_chunk(uint64_t c0, uint64_t n, int lane) const {
        Chunk c;
        static_cast<CsrDesc::Chunk &>(c) = CsrDesc::begin_chunk(c0, n, lane);
        const uint64_t i = c0 + (uint64_t)lane;
        c.state = i < n ? states[i] : 0u;
        return c;
    }
    __device__ __forceinline__ uint32_t lane_seed(const Chunk &c) const { return c.state; }
};

// ---------------------------------------------------------------------------------
// Per-lane pieces
// ---------------------------------------------------------------------------------

// Ones'-complement (end-around-carry) accumulator over 32-bit words: the add-with-carry
// chain compiles to one v_addc_co_u32 per word; the carry out of each add is folded into
// the next one, and finish() adds the last carry (twice at most). 2^32 = 1 (mod 0xFFFF),
// so the 32-bit ones'-complement sum is congruent to the sum of the 16-bit halves, and it
// is 0 only if every word was 0.
struct Eac {
    uint32_t s = 0, c = 0;
    __device__ __forceinline__ void add(uint32_t x) { s = __builtin_addc(s, x, c, &c); }
    __device__ __forceinline__ uint32_t finish() {
        uint32_t c2;
        uint32_t r = __builtin_addc(s, c, 0u, &c2);
        return r + c2;
    }
};

// Byte masks of a 16-byte segment as four dwords, in constant memory so that a wave
// fetches them with one s_load_dwordx4 each (scalar cache) instead of computing them:
//   kMaskFrom[f] keeps bytes [f, 16)  (head segment, f = S & 15)
//   kMaskTo[t]   keeps bytes [0, t)   (tail segment, t in 1..16)
constexpr uint32_t byte_range_dword(int lo, int hi, int d) {
    uint32_t m = 0;
    for (int b = 0; b < 4; ++b)
        if (4 * d + b >= lo && 4 * d + b < hi) m |= 0xFFu << (8 * b);
    return m;
}
#define AIPSTACK_MASK_FROM(f) \
    {byte_range_dword(f, 16, 0), byte_range_dword(f, 16, 1), byte_range_dword(f, 16, 2), \
     byte_range_dword(f, 16, 3)}
#define AIPSTACK_MASK_TO(t) \
    {byte_range_dword(0, t, 0), byte_range_dword(0, t, 1), byte_range_dword(0, t, 2), \
     byte_range_dword(0, t, 3)}
__constant__ uint32_t kMaskFrom[16][4] = {
    AIPSTACK_MASK_FROM(0),  AIPSTACK_MASK_FROM(1),  AIPSTACK_MASK_FROM(2),  AIPSTACK_MASK_FROM(3),
    AIPSTACK_MASK_FROM(4),  AIPSTACK_MASK_FROM(5),  AIPSTACK_MASK_FROM(6),  AIPSTACK_MASK_FROM(7),
    AIPSTACK_MASK_FROM(8),  AIPSTACK_MASK_FROM(9),  AIPSTACK_MASK_FROM(10), AIPSTACK_MASK_FROM(11),
    AIPSTACK_MASK_FROM(12), AIPSTACK_MASK_FROM(13), AIPSTACK_MASK_FROM(14), AIPSTACK_MASK_FROM(15)};
__constant__ uint32_t kMaskTo[17][4] = {
    AIPSTACK_MASK_TO(0),  AIPSTACK_MASK_TO(1),  AIPSTACK_MASK_TO(2),  AIPSTACK_MASK_TO(3),
    AIPSTACK_MASK_TO(4),  AIPSTACK_MASK_TO(5),  AIPSTACK_MASK_TO(6),  AIPSTACK_MASK_TO(7),
    AIPSTACK_MASK_TO(8),  AIPSTACK_MASK_TO(9),  AIPSTACK_MASK_TO(10), AIPSTACK_MASK_TO(11),
    AIPSTACK_MASK_TO(12), AIPSTACK_MASK_TO(13), AIPSTACK_MASK_TO(14), AIPSTACK_MASK_TO(15),
    AIPSTACK_MASK_TO(16)};
#undef AIPSTACK_MASK_FROM
#undef AIPSTACK_MASK_TO

__device__ __forceinline__ u32x4 load_mask(const uint32_t (&m)[4]) {
    return u32x4{m[0], m[1], m[2], m[3]};
}

// v & (m | sel): sel = ~0 keeps v (lanes the mask does not apply to), sel = 0 masks it.
// One v_bitop3_b32 per dword.
__device__ __forceinline__ void apply_mask(u32x4 &v, const u32x4 &m, uint32_t sel) {
#pragma unroll
    for (int d = 0; d < 4; ++d) v[d] &= (m[d] | sel);
}

// Buffer-load cache policy (aux): 2 = nt (streaming), 0 = default.
template <bool NT>
__device__ __forceinline__ u32x4 load_segment(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                              uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, soff, NT ? 2 : 0);
}

// Sum over the 64 lanes (defined below).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v);

// One packet's aligned-segment loads, split into issue() and finish() so that a wave
// can keep several packets' loads in flight before it reduces the first of them.
//
// The packet [S, E) is read as the 16-byte-aligned segments A0 = S & ~15, A0 + 16, ...
// through a buffer descriptor whose base is A0 and whose size is 16 * nseg: lane k reads
// segment k (voffset = 16 * lane, soffset = 1 KiB per slot), and the hardware range check
// returns zeros for segments past the end, with no exec masking. Bytes of the head
// segment before S and of the tail segment from E on are masked off. Each lane keeps a
// ones'-complement sum of its dwords; finish() folds it to 18 bits and adds the 64 lanes
// exactly (< 2^24), returning a wave-uniform value that is 0 iff every byte is 0 and is
// congruent (mod 0xFFFF) to the sum of the little-endian 16-bit halves.
// U = segments per lane issued up front (group 0 = the first 64*U segments); longer
// packets loop over further groups inside finish().
template <int U, bool NT>
struct PacketLoad {
    uint64_t A0;
    int rel_s;  // S - A0 (0..15)
    int rel_e;  // E - A0
    int nseg;   // aligned segments covering [S, E); 0 for an empty packet
    __amdgpu_buffer_rsrc_t rsrc;
    u32x4 v[U];

    u32x4 hm, tm;  // head / tail byte masks

    __device__ __forceinline__ void issue(uint64_t S, uint64_t E, uint32_t voff) {
        A0 = S & ~(uint64_t)15;
        rel_s = (int)(S - A0);
        // Lengths of 2 GiB or more, and E < S, are outside every contract: empty packet.
        const uint64_t len = E - S;
        const bool empty = len == 0 || len >= (1ull << 31);
        rel_e = empty ? rel_s : rel_s + (int)len;
        nseg = empty ? 0 : (rel_e + 15) >> 4;
        hm = load_mask(kMaskFrom[rel_s]);
        tm = load_mask(kMaskTo[empty ? 16 : rel_e - 16 * (nseg - 1)]);
        rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(A0), (short)0,
                                                 nseg * 16, 0x00020000);
        // Unconditional: slots past the packet fail the descriptor's range check and
        // return zeros without touching memory. Keeping the loads straight-line lets the
        // compiler count them, so finishing packet q waits only for q's loads
        // (s_waitcnt vmcnt(N)), not for every packet in flight (a branch -> vmcnt(0)).
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = load_segment<NT>(rsrc, voff, (uint32_t)(u * kWave * 16));
    }

    // Mask the tail segment `last` (lane lt of slot (last - g) >> 6) if it is in group g.
    __device__ __forceinline__ void mask_tail(int g, int last, const u32x4 &tm,
                                              uint32_t not_lt) {
        if (last >= g && last < g + kWave * U) {
            const int ut = (last - g) >> 6;
            // Branch-free slot choice: an `if (u == ut)` chain gets merged by LLVM into one
            // dynamically indexed v[ut], which lives in scratch.
#pragma unroll
            for (int u = 0; u < U; ++u)
                apply_mask(v[u], tm, u == ut ? not_lt : ~0u);
        }
    }

    // Two interleaved carry chains (even / odd dwords): independent v_addc_co_u32 fill
    // each other's carry-hazard wait states.
    __device__ __forceinline__ void accumulate(Eac &a0, Eac &a1) const {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a0.add(v[u][0]);
            a1.add(v[u][1]);
            a0.add(v[u][2]);
            a1.add(v[u][3]);
        }
    }

    // not_lane0 = ~0 on every lane but lane 0 (where it is 0).
    __device__ __forceinline__ uint32_t finish(int lane, uint32_t voff, uint32_t not_lane0) {
        if (nseg == 0)
            return 0;
        const int last = nseg - 1;
        const uint32_t not_lt = (lane == (last & (kWave - 1))) ? 0u : ~0u;
        apply_mask(v[0], hm, not_lane0);  // head: segment 0 = slot 0, lane 0
        mask_tail(0, last, tm, not_lt);
        Eac acc0, acc1;
        accumulate(acc0, acc1);
        for (int g = kWave * U; g < nseg; g += kWave * U) {  // packets > 64*U segments
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[u] = load_segment<NT>(rsrc, voff, (uint32_t)((g + u * kWave) * 16));
            mask_tail(g, last, tm, not_lt);
            accumulate(acc0, acc1);
        }
        // fold each chain to 17 bits (nonzero stays nonzero): 2 x 64 lanes x 0x1FFFE < 2^24
        const uint32_t s0 = acc0.finish(), s1 = acc1.finish();
        return wave_sum((s0 & 0xFFFFu) + (s0 >> 16) + (s1 & 0xFFFFu) + (s1 >> 16));
    }
};

// Sum over the 64 lanes (DPP row scan + row broadcasts); result valid in lane 63,
// returned wave-uniform via readlane.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    // dpp_ctrl: row_shr:n = 0x110 + n; row_bcast:15 = 0x142; row_bcast:31 = 0x143.
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ uint32_t fold16(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) {
    return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
}

// ---------------------------------------------------------------------------------
// The kernel: wave w handles 64-packet chunks [w*cpw, (w+1)*cpw).
// ---------------------------------------------------------------------------------
template <class Desc, int U, int P, bool NT, bool SEEDED>
__global__ __launch_bounds__(kBlock) void chksum_batch_kernel(Desc desc, uint64_t n,
                                                              uint32_t chunks_per_wave,
                                                              uint16_t *__restrict__ out,
                                                              uint32_t flags) {
    const int lane = threadIdx.x & (kWave - 1);
    // threadIdx.x >> 6 is wave-uniform but the compiler cannot prove it: readfirstlane
    // keeps the whole packet walk (bounds, loop counters) in SGPRs.
    const uint32_t wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wave_in_block;
    const uint64_t nchunks = (n + kWave - 1) / kWave;
    uint64_t c = wave * chunks_per_wave;
    const uint64_t c_end = min(c + chunks_per_wave, nchunks);
    const bool final_flag = (flags & AIPSTACK_CHKSUM_FINAL) != 0;
    const uint32_t voff = (uint32_t)lane * 16u;          // this lane's segment in a slot
    const uint32_t not_lane0 = lane == 0 ? 0u : ~0u;     // head-mask lane select

    for (; c < c_end; ++c) {
        const uint64_t p0 = c * kWave;
        const auto chunk = desc.begin_chunk(p0, n, lane);
        const int cnt = (int)min((uint64_t)kWave, n - p0);
        uint32_t sums = 0;  // lane j: exact halves-sum of packet j (< 2^24)
        // P packets at a time: all their first-group loads in flight, then reduce each.
        for (int j0 = 0; j0 < cnt; j0 += P) {
            PacketLoad<U, NT> pk[P];
#pragma unroll
            for (int q = 0; q < P; ++q) {
                uint64_t s = 0, e = 0;
                if (j0 + q < cnt)
                    desc.bounds(chunk, j0 + q, s, e);
                pk[q].issue(s, e, voff);
            }
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const uint32_t t = pk[q].finish(lane, voff, not_lane0);  // wave-uniform
                sums = (lane == j0 + q) ? t : sums;
            }
        }
        // Finalise the chunk's 64 results together (VALU, one packet per lane).
        uint32_t r = fold16(sums);
        if ((desc.lane_start(chunk, lane) & 1) == 0)
            r = bswap16(r);  // little-endian pairing -> the reference's big-endian words
        if constexpr (SEEDED) {
            // IpChksumAccumulator(State): m_sum = state; m_sum += r with end-around
            // carry (Chksum.h:294-300); getChksum: fold twice, invert (:245-250).
            const uint64_t t = (uint64_t)desc.lane_seed(chunk) + r;
            const uint32_t m = (uint32_t)t + (uint32_t)(t >> 32);
            r = (~fold16(m)) & 0xFFFFu;
        } else if (final_flag) {
            r = (~r) & 0xFFFFu;
        }
        if (lane < cnt)
            out[p0 + lane] = (uint16_t)r;
    }
}

// ---------------------------------------------------------------------------------
// Chained batch: IpChksumAccumulator(State{states[i]})
// .getChksum(IpBufRef{chain i}) (Chksum.h:171-174, 263-315) for n chains. Chain i is the
// chunks [index[i], index[i+1]) of a chunk table (absolute address, length), in order:
// the IpBufRef's nodes as ipBufProcessBytes visits them (BufUtils.h:129-178).
//
// The reference adds each chunk's IpChksumInverted with end-around carry and byte-swaps
// the running sum after every odd-length chunk, once more at the end if the count of
// swaps is odd (Chksum.h:294-314). A swap is x*256 mod 0xFFFF, so chunk k contributes
// its big-endian sum times 256^(parity of its logical position q_k), and the state is
// swapped an even number of times. With the kernel's little-endian sum of the chunk at
// address a_k, that is: byte-swap the folded chunk sum iff parity(a_k) == parity(q_k).
// ---------------------------------------------------------------------------------
template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void chksum_chain_kernel(
    const uint64_t *__restrict__ chunk_addr, const uint32_t *__restrict__ chunk_len,
    const uint64_t *__restrict__ index, const uint32_t *__restrict__ states, uint64_t n,
    uint32_t chunks_per_wave, uint16_t *__restrict__ out, uint32_t flags) {
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wave_in_block;
    const uint64_t nchunks = (n + kWave - 1) / kWave;
    uint64_t c = wave * chunks_per_wave;
    const uint64_t c_end = min(c + chunks_per_wave, nchunks);
    const bool final_flag = (flags & AIPSTACK_CHKSUM_FINAL) != 0;
    const uint32_t voff = (uint32_t)lane * 16u;
    const uint32_t not_lane0 = lane == 0 ? 0u : ~0u;
    CsrDesc idx_desc{0, index};  // reuse the CSR offset walk for the chunk index

    for (; c < c_end; ++c) {
        const uint64_t p0 = c * kWave;
        const auto chunk = idx_desc.begin_chunk(p0, n, lane);
        const int cnt = (int)min((uint64_t)kWave, n - p0);
        uint32_t state = 0;
        if (states != nullptr && p0 + lane < n)
            state = states[p0 + lane];
        uint32_t sums = 0;  // lane j: sum of chain j's orientation-corrected chunk sums
        for (int j = 0; j < cnt; ++j) {
            uint64_t k0, k1;
            idx_desc.bounds(chunk, j, k0, k1);
            uint32_t acc = 0;   // <= nchunks * 0xFFFF
            uint32_t pos = 0;   // parity of the logical position
            for (uint64_t k = k0; k < k1; ++k) {
                const uint64_t a = chunk_addr[k];
                const uint32_t l = chunk_len[k];
                PacketLoad<U, NT> pk;
                pk.issue(a, a + l, voff);
                uint32_t r = fold16(pk.finish(lane, voff, not_lane0));
                if ((uint32_t)(a & 1) == pos)
                    r = bswap16(r);
                acc += r;
                pos ^= l & 1;
            }
            sums = (lane == j) ? acc : sums;
        }
        // m_sum = state (+) chain sum with end-around carry; getChksum folds and inverts.
        const uint64_t t = (uint64_t)state + fold16(sums);
        uint32_t r = fold16((uint32_t)t + (uint32_t)(t >> 32));
        r = final_flag ? (~r & 0xFFFFu) : r;
        if (lane < cnt)
            out[p0 + lane] = (uint16_t)r;
    }
}

// ---------------------------------------------------------------------------------
// Launch configuration
// ---------------------------------------------------------------------------------

// Tunables (0 = automatic). Set from the environment once, or at run time through
// aipstack_chksum_tune() (benchmark sweeps); read at every launch.
struct Tuning {
    std::atomic<int> waves_per_cu{0};     // resident-wave budget per CU the grid is sized to
    std::atomic<int> chunks_per_wave{0};  // 64-packet chunks per wave (overrides the above)
    std::atomic<int> unroll{0};           // U: segments per lane issued up front (1..4)
    std::atomic<int> packets{0};          // P: packets whose loads a wave keeps in flight
    std::atomic<int> nontemporal{1};      // 1 = nontemporal (streaming) loads: every byte is
                                          // read once; measured faster on configs A and B

    Tuning() {
        auto env = [](const char *k, std::atomic<int> &v) {
            if (const char *s = std::getenv(k)) v = std::atoi(s);
        };
        env("AIPSTACK_CHKSUM_WAVES_PER_CU", waves_per_cu);
        env("AIPSTACK_CHKSUM_CHUNKS_PER_WAVE", chunks_per_wave);
        env("AIPSTACK_CHKSUM_UNROLL", unroll);
        env("AIPSTACK_CHKSUM_PACKETS", packets);
        env("AIPSTACK_CHKSUM_NT", nontemporal);
    }
};

Tuning &tuning() {
    static Tuning t;
    return t;
}

constexpr int kDefaultWavesPerCu = 64;

// U: enough segments per lane to cover a typical packet in one group.
int pick_unroll(uint32_t max_len) {
    const int t = tuning().unroll.load(std::memory_order_relaxed);
    if (t >= 1 && t <= 4) return t;
    const uint32_t max_seg = (max_len + 30u) / 16u;           // worst-case alignment
    const uint32_t q = (max_seg + kWave - 1) / kWave;         // groups of 64 segments
    if (q <= 1) return 1;
    if (q == 2) return 2;
    if (q % 3 == 0 || q == 3) return 3;
    return 4;
}

// P: packets whose loads a wave keeps in flight. Measured (tools/sweep.py, MI355X):
// 1500 B strided best at P = 4..8, 9000 B at P = 1 (U = 3 already has 3 KiB in flight
// per wave), mixed CSR at P = 2.
int pick_packets(int u, bool csr) {
    const int t = tuning().packets.load(std::memory_order_relaxed);
    if (t == 1 || t == 2 || t == 4 || t == 8) return t;
    if (csr) return 2;
    return u <= 2 ? 4 : 1;
}

template <class Desc, int U, int P, bool NT, bool SEEDED>
int launch_k(const Desc &desc, uint64_t n, uint16_t *d_out, uint32_t flags,
             hipStream_t stream) {
    const uint64_t nchunks = (n + kWave - 1) / kWave;
    const int cus = device_cu_count();
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    uint64_t cpw = (uint64_t)tuning().chunks_per_wave.load(std::memory_order_relaxed);
    if (cpw == 0) {
        int wpc = tuning().waves_per_cu.load(std::memory_order_relaxed);
        if (wpc <= 0) wpc = Desc::kCsr ? 2 * kDefaultWavesPerCu : kDefaultWavesPerCu;
        const uint64_t target_waves = (uint64_t)cus * (uint64_t)wpc;
        cpw = (nchunks + target_waves - 1) / target_waves;
        if (cpw == 0) cpw = 1;
    }
    const uint64_t waves = (nchunks + cpw - 1) / cpw;
    const uint64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7FFFFFFFull || cpw > 0xFFFFFFFFull) return AIPSTACK_CHKSUM_EINVAL;
    hipLaunchKernelGGL((chksum_batch_kernel<Desc, U, P, NT, SEEDED>), dim3((unsigned)blocks),
                       dim3(kBlock), 0, stream, desc, n, (uint32_t)cpw, d_out, flags);
    return check_hip(hipGetLastError());
}

template <class Desc, int U, bool SEEDED>
int launch_u(const Desc &desc, uint64_t n, uint16_t *d_out, uint32_t flags,
             hipStream_t stream) {
    const bool nt = tuning().nontemporal.load(std::memory_order_relaxed) != 0;
    const int p = pick_packets(U, Desc::kCsr);
#define AIPSTACK_LAUNCH_P(PP)                                                               \
    case PP:                                                                                \
        return nt ? launch_k<Desc, U, PP, true, SEEDED>(desc, n, d_out, flags, stream)      \
                  : launch_k<Desc, U, PP, false, SEEDED>(desc, n, d_out, flags, stream);
    switch (p) {
        AIPSTACK_LAUNCH_P(1)
        AIPSTACK_LAUNCH_P(2)
        AIPSTACK_LAUNCH_P(4)
        AIPSTACK_LAUNCH_P(8)
    }
#undef AIPSTACK_LAUNCH_P
    return AIPSTACK_CHKSUM_EINVAL;
}

template <class Desc, bool SEEDED>
int launch(const Desc &desc, uint64_t n, uint32_t max_len, uint16_t *d_out, uint32_t flags,
           hipStream_t stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    switch (pick_unroll(max_len)) {
        case 1: return launch_u<Desc, 1, SEEDED>(desc, n, d_out, flags, stream);
        case 2: return launch_u<Desc, 2, SEEDED>(desc, n, d_out, flags, stream);
        case 3: return launch_u<Desc, 3, SEEDED>(desc, n, d_out, flags, stream);
        case 4: return launch_u<Desc, 4, SEEDED>(desc, n, d_out, flags, stream);
    }
    return AIPSTACK_CHKSUM_EINVAL;
}

template <int U, bool NT>
int launch_chain(const uint64_t *d_addr, const uint32_t *d_len, const uint64_t *d_index,
                 const uint32_t *d_states, uint64_t n, uint16_t *d_out, uint32_t flags,
                 hipStream_t stream) {
    const uint64_t nchunks = (n + kWave - 1) / kWave;
    const int cus = device_cu_count();
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    const uint64_t target_waves = (uint64_t)cus * 2 * kDefaultWavesPerCu;
    uint64_t cpw = (nchunks + target_waves - 1) / target_waves;
    if (cpw == 0) cpw = 1;
    const uint64_t waves = (nchunks + cpw - 1) / cpw;
    const uint64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7FFFFFFFull || cpw > 0xFFFFFFFFull) return AIPSTACK_CHKSUM_EINVAL;
    hipLaunchKernelGGL((chksum_chain_kernel<U, NT>), dim3((unsigned)blocks), dim3(kBlock), 0,
                       stream, d_addr, d_len, d_index, d_states, n, (uint32_t)cpw, d_out, flags);
    return check_hip(hipGetLastError());
}

}  // namespace
}  // namespace aipstack_amd

using namespace aipstack_amd;

extern "C" int aipstack_chksum_batch_strided(const void *d_base, uint64_t stride, uint32_t len,
                                             uint64_t n, uint16_t *d_out, uint32_t flags,
                                             void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_out || len > AIPSTACK_CHKSUM_MAX_LEN) return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    StridedDesc d{(uint64_t)(uintptr_t)d_base, stride, len};
    return launch<StridedDesc, false>(d, n, len, d_out, flags, (hipStream_t)stream);
}

extern "C" int aipstack_chksum_batch_csr(const void *d_base, const uint64_t *d_offsets,
                                         uint64_t n, uint16_t *d_out, uint32_t flags,
                                         void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    CsrDesc d{(uint64_t)(uintptr_t)d_base, d_offsets};
    // Typical network packets (<= ~2 KiB) fit one group at U = 2; longer ones loop.
    return launch<CsrDesc, false>(d, n, 1500u, d_out, flags, (hipStream_t)stream);
}

extern "C" int aipstack_chksum_batch_seeded_csr(const void *d_base, const uint64_t *d_offsets,
                                                const uint32_t *d_states, uint64_t n,
                                                uint16_t *d_out, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_states || !d_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    SeededCsrDesc d;
    d.base = (uint64_t)(uintptr_t)d_base;
    d.offsets = d_offsets;
    d.states = d_states;
    return launch<SeededCsrDesc, true>(d, n, 1500u, d_out, AIPSTACK_CHKSUM_FINAL,
                                       (hipStream_t)stream);
}

extern "C" int aipstack_chksum_tune(const char *key, int value) {
    if (!key) return AIPSTACK_CHKSUM_EINVAL;
    Tuning &t = tuning();
    if (!std::strcmp(key, "waves_per_cu")) t.waves_per_cu = value;
    else if (!std::strcmp(key, "chunks_per_wave")) t.chunks_per_wave = value;
    else if (!std::strcmp(key, "unroll")) t.unroll = value;
    else if (!std::strcmp(key, "packets")) t.packets = value;
    else if (!std::strcmp(key, "nontemporal")) t.nontemporal = value;
    else return AIPSTACK_CHKSUM_EINVAL;
    return AIPSTACK_CHKSUM_OK;
}

extern "C" int aipstack_chksum_batch_chain(const uint64_t *d_chunk_addr,
                                           const uint32_t *d_chunk_len,
                                           const uint64_t *d_chunk_index,
                                           const uint32_t *d_states, uint64_t n,
                                           uint16_t *d_out, uint32_t flags, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_chunk_addr || !d_chunk_len || !d_chunk_index || !d_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    // Chains are mostly short pieces (headers, ring-buffer halves): U = 2 covers 2 KiB.
    return tuning().nontemporal.load(std::memory_order_relaxed)
               ? launch_chain<2, true>(d_chunk_addr, d_chunk_len, d_chunk_index, d_states, n,
                                       d_out, flags, (hipStream_t)stream)
               : launch_chain<2, false>(d_chunk_addr, d_chunk_len, d_chunk_index, d_states, n,
                                        d_out, flags, (hipStream_t)stream);
}
