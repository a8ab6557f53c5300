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
// Packet descriptors: give the absolute byte range [S, E) of packet p.
// Wave-uniform in, wave-uniform out (the compiler keeps S/E in SGPRs).
// ---------------------------------------------------------------------------------

struct StridedDesc {
    uint64_t base;    // absolute address of packet 0
    uint64_t stride;  // bytes between packet starts
    uint32_t len;     // bytes per packet

    // Per-chunk prologue (nothing to fetch for a fixed stride).
    struct Chunk {};
    __device__ __forceinline__ Chunk begin_chunk(uint64_t, uint64_t, int) const { return {}; }
    __device__ __forceinline__ void bounds(const Chunk &, uint64_t p, int, uint64_t &S,
                                           uint64_t &E) const {
        S = base + p * stride;
        E = S + len;
    }
    __device__ __forceinline__ uint32_t seed(const Chunk &, int) const { return 0; }
};

struct CsrDesc {
    uint64_t base;            // absolute address offsets are relative to
    const uint64_t *offsets;  // n+1 byte offsets

    struct Chunk {
        uint64_t lane_off;  // lane j: offsets[c0 + j]
        uint64_t end_off;   // offsets[min(c0 + 64, n)]
    };
    // Lane j fetches offsets[c0 + j] (one coalesced 512-B load per chunk).
    __device__ __forceinline__ Chunk begin_chunk(uint64_t c0, uint64_t n, int lane) const {
        Chunk c;
        const uint64_t i = c0 + (uint64_t)lane;
        c.lane_off = offsets[i <= n ? i : n];
        const uint64_t last = c0 + kWave < n ? c0 + kWave : n;
        c.end_off = offsets[last];
        return c;
    }
    __device__ __forceinline__ void bounds(const Chunk &c, uint64_t, int j, uint64_t &S,
                                           uint64_t &E) const {
        const uint64_t s = readlane64(c.lane_off, j);
        const uint64_t e = (j + 1 < kWave) ? readlane64(c.lane_off, j + 1) : c.end_off;
        S = base + s;
        E = base + e;
    }
    __device__ __forceinline__ uint32_t seed(const Chunk &, int) const { return 0; }

    __device__ __forceinline__ static uint64_t readlane64(uint64_t v, int j) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, j);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), j);
        return ((uint64_t)hi << 32) | lo;
    }
};

struct SeededCsrDesc : CsrDesc {
    const uint32_t *states;  // n accumulator states (IpChksumAccumulator::State)

    struct Chunk : CsrDesc::Chunk {
        uint32_t lane_state;
    };
    __device__ __forceinline__ Chunk begin_chunk(uint64_t c0, uint64_t n, int lane) const {
        Chunk c;
        static_cast<CsrDesc::Chunk &>(c) = CsrDesc::begin_chunk(c0, n, lane);
        const uint64_t i = c0 + (uint64_t)lane;
        c.lane_state = i < n ? states[i] : 0u;
        return c;
    }
    __device__ __forceinline__ uint32_t seed(const Chunk &c, int j) const {
        return __builtin_amdgcn_readlane(c.lane_state, j);
    }
};

// ---------------------------------------------------------------------------------
// Per-lane pieces
// ---------------------------------------------------------------------------------

// Keep the bytes [lo, hi) of a 16-byte segment that fall in dword d (bytes 4d..4d+3).
__device__ __forceinline__ uint32_t dword_mask(int lo, int hi, int d) {
    const int l = min(max(lo - 4 * d, 0), 4);
    const int h = min(max(hi - 4 * d, 0), 4);
    // low 32 bits of 64-bit shifts: shift by 32 gives 0, as wanted.
    const uint32_t keep_from = (uint32_t)(0xFFFFFFFFull << (8 * l));
    const uint32_t drop_from = (uint32_t)(0xFFFFFFFFull << (8 * h));
    return keep_from & ~drop_from;
}

// Sum of the two little-endian 16-bit halves of x.
__device__ __forceinline__ uint32_t halves(uint32_t x) { return (x & 0xFFFFu) + (x >> 16); }

// Halves-sum of the bytes of a (wave-uniform) 16-byte segment OUTSIDE the window
// [lo, hi): what the unmasked per-lane sum over-counted. Runs on the scalar unit.
__device__ __forceinline__ uint32_t outside_sum(u32x4 w, int lo, int hi) {
    uint32_t s = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) s += halves(w[d] & ~dword_mask(lo, hi, d));
    return s;
}

__device__ __forceinline__ u32x4 readlane4(const u32x4 &v, int lane) {
    return u32x4{(uint32_t)__builtin_amdgcn_readlane(v[0], lane),
                 (uint32_t)__builtin_amdgcn_readlane(v[1], lane),
                 (uint32_t)__builtin_amdgcn_readlane(v[2], lane),
                 (uint32_t)__builtin_amdgcn_readlane(v[3], lane)};
}

template <bool NT>
__device__ __forceinline__ u32x4 load_segment(uint64_t addr) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(addr);
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// Sum over the 64 lanes (defined below).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v);

// Exact little-endian 16-bit-halves sum (64-bit, wave-uniform) of the bytes [S, E).
// S, E wave-uniform. Lane k loads the aligned segment k unmasked; the bytes of the
// first and last segment that lie outside [S, E) are subtracted afterwards on the
// scalar unit. U = segments each lane has in flight per group (1 KiB per wave each).
template <int U, bool NT>
__device__ __forceinline__ uint64_t packet_sum(uint64_t S, uint64_t E, int lane) {
    if (E <= S)
        return 0;
    const uint64_t A0 = S & ~(uint64_t)15;
    const int rel_s = (int)(S - A0);                  // 0..15
    const int rel_e = (int)(E - A0);                  // len + rel_s
    const int nseg = (rel_e + 15) >> 4;
    const int last = nseg - 1;
    uint32_t acc = 0;   // per lane: <= 2^19 per segment, exact up to 4 MiB packets
    uint32_t corr = 0;  // wave-uniform over-count of the head/tail segments
    for (int g = 0; g < nseg; g += kWave * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = g + u * kWave + lane;
            v[u] = u32x4{0u, 0u, 0u, 0u};
            if (k < nseg)
                v[u] = load_segment<NT>(A0 + 16ull * (uint64_t)k);
        }
        if (g == 0)  // head segment (also the tail when nseg == 1)
            corr += outside_sum(readlane4(v[0], 0), rel_s, rel_e);
        if (last > 0 && last < g + kWave * U) {  // tail segment is in this group
            const int ut = (last - g) >> 6;
            const int lt = last & (kWave - 1);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (u == ut)
                    corr += outside_sum(readlane4(v[u], lt), 0, rel_e - 16 * last);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int d = 0; d < 4; ++d)
                acc += halves(v[u][d]);
    }
    uint64_t total;
    if (nseg <= 8192) {  // 64 lanes * 2^19 * ceil(nseg/64) < 2^32
        total = wave_sum(acc);
    } else {             // longer than any reference packet: split to stay exact
        total = (uint64_t)wave_sum(acc & 0xFFFFu) + ((uint64_t)wave_sum(acc >> 16) << 16);
    }
    return total - corr;
}

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

// Fold a 64-bit sum to 16 bits; 2^32 = 2^16 = 1 (mod 0xFFFF), nonzero stays nonzero.
__device__ __forceinline__ uint32_t fold64(uint64_t t) {
    t = (t & 0xFFFFFFFFull) + (t >> 32);
    t = (t & 0xFFFFFFFFull) + (t >> 32);
    uint32_t s = (uint32_t)t;
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;
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
template <class Desc, int U, bool NT, bool SEEDED>
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

    for (; c < c_end; ++c) {
        const uint64_t p0 = c * kWave;
        const auto chunk = desc.begin_chunk(p0, n, lane);
        const int cnt = (int)min((uint64_t)kWave, n - p0);
        uint32_t mine = 0;
        for (int j = 0; j < cnt; ++j) {
            uint64_t S, E;
            desc.bounds(chunk, p0 + j, j, S, E);
            uint32_t r = fold64(packet_sum<U, NT>(S, E, lane));
            if ((S & 1) == 0)
                r = bswap16(r);
            if constexpr (SEEDED) {
                // IpChksumAccumulator(State): m_sum = state; m_sum += r with end-around
                // carry (Chksum.h:294-300); getChksum: fold twice, invert (:245-250).
                uint64_t t = (uint64_t)desc.seed(chunk, j) + r;
                uint32_t m = (uint32_t)t + (uint32_t)(t >> 32);
                r = (~fold16(m)) & 0xFFFFu;
            } else if (final_flag) {
                r = (~r) & 0xFFFFu;
            }
            mine = (lane == j) ? r : mine;
        }
        if (lane < cnt)
            out[p0 + lane] = (uint16_t)mine;
    }
}

// ---------------------------------------------------------------------------------
// Launch configuration
// ---------------------------------------------------------------------------------

struct Tuning {
    int waves_per_cu = 64;      // target resident-wave budget per CU the grid is sized to
    int chunks_per_wave = 0;    // 0 = derived from waves_per_cu
    int unroll = 0;             // 0 = derived from packet length (segments in flight/lane)
    int nontemporal = 0;        // 1 = nontemporal (streaming) loads
};

Tuning read_tuning() {
    Tuning t;
    if (const char *s = std::getenv("AIPSTACK_CHKSUM_WAVES_PER_CU")) t.waves_per_cu = std::atoi(s);
    if (const char *s = std::getenv("AIPSTACK_CHKSUM_CHUNKS_PER_WAVE")) t.chunks_per_wave = std::atoi(s);
    if (const char *s = std::getenv("AIPSTACK_CHKSUM_UNROLL")) t.unroll = std::atoi(s);
    if (const char *s = std::getenv("AIPSTACK_CHKSUM_NT")) t.nontemporal = std::atoi(s);
    if (t.waves_per_cu < 1) t.waves_per_cu = 1;
    return t;
}

const Tuning &tuning() {
    static const Tuning t = read_tuning();
    return t;
}

// Segments per lane in flight per group: enough to cover a typical packet in one group.
int pick_unroll(uint32_t max_len) {
    if (tuning().unroll >= 1 && tuning().unroll <= 4) return tuning().unroll;
    const uint32_t max_seg = (max_len + 30u) / 16u;           // worst-case alignment
    const uint32_t q = (max_seg + kWave - 1) / kWave;         // groups of 64 segments
    if (q <= 1) return 1;
    if (q == 2) return 2;
    if (q % 3 == 0) return 3;
    if (q == 3) return 3;
    return 4;
}

template <class Desc, int U, bool NT, bool SEEDED>
int launch_u(const Desc &desc, uint64_t n, uint16_t *d_out, uint32_t flags,
             hipStream_t stream) {
    const uint64_t nchunks = (n + kWave - 1) / kWave;
    int cus = device_cu_count();
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    uint64_t cpw = (uint64_t)tuning().chunks_per_wave;
    if (cpw == 0) {
        const uint64_t target_waves = (uint64_t)cus * (uint64_t)tuning().waves_per_cu;
        cpw = (nchunks + target_waves - 1) / target_waves;
        if (cpw == 0) cpw = 1;
    }
    const uint64_t waves = (nchunks + cpw - 1) / cpw;
    const uint64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7FFFFFFFull || cpw > 0xFFFFFFFFull) return AIPSTACK_CHKSUM_EINVAL;
    hipLaunchKernelGGL((chksum_batch_kernel<Desc, U, NT, SEEDED>), dim3((unsigned)blocks),
                       dim3(kBlock), 0, stream, desc, n, (uint32_t)cpw, d_out, flags);
    return check_hip(hipGetLastError());
}

template <class Desc, bool SEEDED>
int launch(const Desc &desc, uint64_t n, uint32_t max_len, uint16_t *d_out, uint32_t flags,
           hipStream_t stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    const int u = pick_unroll(max_len);
    const bool nt = tuning().nontemporal != 0;
#define AIPSTACK_LAUNCH_U(UU)                                                             \
    case UU:                                                                              \
        return nt ? launch_u<Desc, UU, true, SEEDED>(desc, n, d_out, flags, stream)       \
                  : launch_u<Desc, UU, false, SEEDED>(desc, n, d_out, flags, stream);
    switch (u) {
        AIPSTACK_LAUNCH_U(1)
        AIPSTACK_LAUNCH_U(2)
        AIPSTACK_LAUNCH_U(3)
        AIPSTACK_LAUNCH_U(4)
    }
#undef AIPSTACK_LAUNCH_U
    return AIPSTACK_CHKSUM_EINVAL;
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
