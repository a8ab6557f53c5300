// aipstack_amd -- device-side building blocks shared by the batch kernels
// (chksum_kernels.hip: flat / CSR / seeded / chained batches; frame_kernels.hip: Rx verify
// and Tx fill on raw frames). Included by .hip translation units only; everything lives
// in an anonymous namespace, so each TU has its own copy.
#ifndef AIPSTACK_AMD_CHKSUM_DEVICE_H
#define AIPSTACK_AMD_CHKSUM_DEVICE_H

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "aipstack_amd/chksum.h"
#include "chksum_internal.h"

namespace aipstack_amd {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

// Contract violations seen by this translation unit's kernels on this device: sticky bits
// (AIPSTACK_CHKSUM_VIOLATION_*, chksum.h), read and cleared from the host through
// aipstack_chksum_contract_violations(). Each .hip file has its own copy (anonymous
// namespace); the host side reads them all. Set only on the rare path, with a vector atomic.
__device__ uint32_t g_violations;

__device__ __forceinline__ void note_violation(bool bad, uint32_t bit) {
    if (__builtin_amdgcn_ballot_w64(bad) != 0 && bad)
        __hip_atomic_fetch_or(&g_violations, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Reads this translation unit's violation word into *out -- and clears it in the same atomic
// exchange when `clear`, so a bit a kernel sets meanwhile is either returned or kept, never
// lost (a read and a separate clear could drop it). One thread, on its own stream.
__global__ void take_violations_kernel(uint32_t *out, uint32_t clear) {
    out[0] = clear ? __hip_atomic_exchange(&g_violations, 0u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT)
                   : __hip_atomic_load(&g_violations, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Host side of the above for the current device: ORs the word into *mask.
inline int take_violations_here(uint32_t *mask, bool clear) {
    uint32_t *h = nullptr;
    int st = check_hip(hipHostMalloc(reinterpret_cast<void **>(&h), sizeof(uint32_t),
                                     hipHostMallocMapped));
    if (st != AIPSTACK_CHKSUM_OK) return st;
    *h = 0;
    hipStream_t s = nullptr;
    st = check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (st == AIPSTACK_CHKSUM_OK) {
        hipLaunchKernelGGL(take_violations_kernel, dim3(1), dim3(1), 0, s, h, clear ? 1u : 0u);
        st = check_hip(hipGetLastError());
    }
    if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipStreamSynchronize(s));
    if (st == AIPSTACK_CHKSUM_OK) *mask |= *h;
    if (s) (void)hipStreamDestroy(s);
    (void)hipHostFree(h);
    return st;
}

// ---------------------------------------------------------------------------------
// Packet descriptors. A wave walks 64-packet chunks; per chunk the descriptor may fetch
// per-lane data (lane j <-> packet j of the chunk), then gives
//   bounds(j)      the wave-uniform absolute byte range [S, E) of packet j (SGPRs), and
//   lane_bounds()  [S, E) of this lane's packet (VGPRs; vectorised per-chunk metadata).
// ---------------------------------------------------------------------------------

// A copy of x in a fresh VGPR. The compiler waits for the load that produced x here,
// once per chunk, instead of before every later v_readlane of it (where, inside the
// packet loop, the wait would also drain the packet loads already in flight).
__device__ __forceinline__ uint32_t settle(uint32_t x) {
    uint32_t y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
    return y;
}

// Lane i gets lane i+1's v; lane 63 gets `last`. The choice is made on the source side
// (lane 0 supplies `last`) and the ds_bpermute always runs on the full wave. Written as
// `lane == 63 ? last : __shfl_down(v, 1)`, LLVM may run the permute under an exec mask
// without lane 63 -- and a permute that reads an inactive lane gets garbage.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v, uint32_t last, int lane) {
    const uint32_t src = lane == 0 ? last : v;
    return (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + 1) & 63) << 2, (int)src);
}

// Lane l's 64-bit v, wave-uniform.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

struct StridedDesc {
    static constexpr bool kCsr = false;
    static constexpr bool kStream = true;  // SU > 0: stream mode for back-to-back chunks
    static constexpr bool kEdge = true;    // (gathered descriptors only)
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
    // This lane's packet (chunk packet `lane`) as [S, E) in VGPRs.
    __device__ __forceinline__ void lane_bounds(const Chunk &c, int lane, uint64_t &S,
                                                uint64_t &E) const {
        S = c.s0 + (uint64_t)lane * stride;
        E = S + len;
    }
    __device__ __forceinline__ uint32_t lane_seed(const Chunk &) const { return 0; }
    // Host: every chunk's packets lie back to back (stream mode always applies).
    bool back_to_back() const { return stride == len && len < (1u << 17); }
};

// Fixed-length packets at a stride other than their length (gaps between them, as
// `aipstack_chksum_batch_strided` with stride != len: 1500-B packets in 2048-B slots): not one
// contiguous run, so they take the gathered stream of just their segments (round 4: config
// A2K 241.6 us in the per-packet wave mode, ~224 us gathered) -- a ring of slots with one
// length for all.
struct GappedDesc {
    static constexpr bool kCsr = false;
    static constexpr bool kStream = false;
    static constexpr bool kEdge = true;  // gathered stream: edge segments read up front
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
    __device__ __forceinline__ void lane_bounds(const Chunk &c, int lane, uint64_t &S,
                                                uint64_t &E) const {
        S = c.s0 + (uint64_t)lane * stride;
        E = S + len;
    }
    __device__ __forceinline__ uint32_t lane_seed(const Chunk &) const { return 0; }
    bool back_to_back() const { return false; }
    __device__ __forceinline__ uint64_t chunk_end(const Chunk &c, int cnt) const {
        return c.s0 + (uint64_t)cnt * stride;
    }
};

// Gapped packets whose segments can be counted without a table (round 5): the stride a
// multiple of 16, so every packet starts at the same offset rs within its segment and spans
// the same ns segments. Compact segment c of a chunk (its packets' segments in order) is
// segment c - k ns of packet k = c / ns (magic = ceil(2^32 / ns), exact for c < 2^16 and
// ns <= 2048), at byte k (stride - 16 ns) + 16 c from the chunk's first aligned start: the
// column runs' loop over a gathered stream whose owners are arithmetic (no LDS lookups).
struct GappedColDesc : GappedDesc {
    uint32_t ns;     // segments per packet
    uint32_t magic;  // ceil(2^32 / ns)
    int32_t gap;     // stride - 16 * ns (negative when packets share their edge segments)
};

struct CsrDesc {
    static constexpr bool kCsr = true;
    static constexpr bool kStream = true;
    static constexpr bool kEdge = true;  // (gathered descriptors only)
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
    // This lane's packet as [S, E): its offset and the next lane's (lane 63: end_off).
    __device__ __forceinline__ void lane_bounds(const Chunk &c, int lane, uint64_t &S,
                                                uint64_t &E) const {
        const uint32_t nlo = from_next_lane(c.off_lo, (uint32_t)c.end_off, lane);
        const uint32_t nhi = from_next_lane(c.off_hi, (uint32_t)(c.end_off >> 32), lane);
        const uint64_t next = ((uint64_t)nhi << 32) | nlo;
        S = base + (((uint64_t)c.off_hi << 32) | c.off_lo);
        E = base + next;
    }
    __device__ __forceinline__ uint32_t lane_seed(const Chunk &) const { return 0; }
    bool back_to_back() const { return false; }  // known per chunk only
    // End of the chunk's bytes (absolute): one past its last packet.
    __device__ __forceinline__ uint64_t chunk_end(const Chunk &c, int) const {
        return base + c.end_off;
    }
};

// Ring slots: packet i is the lens[i] bytes at base + i * stride -- a receive ring that
// holds one frame per fixed-size slot with its length beside it (the TAP driver reads one
// frame per buffer, reference tap/linux/TapDeviceLinux.cpp:156-178). The buffer holds n
// whole slots. A length above cap = min(stride, 65535) is outside the contract: it is
// clamped to cap (nothing outside the slot is read) and reported (note_violation).
struct SlottedDesc {
    static constexpr bool kCsr = false;
    static constexpr bool kStream = false;  // slots are not back to back: no contiguous run,
                                            // but the gathered stream (SU > 0) reads just the
                                            // packets' segments as one stream
    static constexpr bool kEdge = true;     // edge segments read up front (sum_gathered_chunks)
    uint64_t base;          // absolute address of slot 0
    uint64_t stride;        // slot size in bytes
    const uint32_t *lens;   // n packet lengths
    uint32_t cap;           // min(stride, 65535)

    struct Chunk {
        uint64_t s0;   // start of the chunk's first slot
        uint32_t len;  // lane j: packet j's length (settled)
    };
    __device__ __forceinline__ Chunk begin_chunk(uint64_t c0, uint64_t n, int lane) const {
        const uint64_t i = c0 + (uint64_t)lane;
        const uint32_t l = i < n ? lens[i] : 0u;
        note_violation(l > cap, AIPSTACK_CHKSUM_VIOLATION_PACKET_LEN);
        return Chunk{base + c0 * stride, settle(l < cap ? l : cap)};
    }
    __device__ __forceinline__ void bounds(const Chunk &c, int j, uint64_t &S,
                                           uint64_t &E) const {
        S = c.s0 + (uint64_t)j * stride;
        E = S + (uint32_t)__builtin_amdgcn_readlane(c.len, j);
    }
    __device__ __forceinline__ void lane_bounds(const Chunk &c, int lane, uint64_t &S,
                                                uint64_t &E) const {
        S = c.s0 + (uint64_t)lane * stride;
        E = S + c.len;
    }
    __device__ __forceinline__ uint32_t lane_seed(const Chunk &) const { return 0; }
    bool back_to_back() const { return false; }
    __device__ __forceinline__ uint64_t chunk_end(const Chunk &c, int cnt) const {
        return c.s0 + (uint64_t)cnt * stride;
    }
};

// CSR packets read by the gathered stream (round 4, the default for the CSR checksum batch):
// the same descriptor without stream mode. A chunk holding a packet over 65535 bytes (outside
// the contract; its halves-sum could pass 2^32) takes the per-packet wave mode instead.
struct GatheredCsrDesc : CsrDesc {
    static constexpr bool kStream = false;
    static constexpr bool kEdge = true;
    bool back_to_back() const { return false; }
};

// Ring slots the kernel reads over the link from page-locked host memory (the engine's
// zero-copy pieces): edges masked in the stream, so no segment crosses the link twice.
struct SlottedHostDesc : SlottedDesc {
    static constexpr bool kEdge = false;
};

// The same for fixed-length packets at a gap read over the link.
struct GappedHostDesc : GappedDesc {
    static constexpr bool kEdge = false;
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

// Per-packet load parameters, computed for 64 packets at once (lane j <-> packet j, VALU)
// and fetched per packet with three v_readlane: the aligned base A0 = S & ~15 and a
// packed word {rel_s = S & 15 : 4 | tail bytes t (1..16) : 5 | nseg : 23}. Lengths of
// 2^26 bytes or more, and E < S, are outside every contract and packed as empty.
struct LaneMeta {
    uint32_t a0_lo, a0_hi, packed;
};

__device__ __forceinline__ LaneMeta lane_meta(uint64_t S, uint64_t E) {
    const uint64_t len = E - S;
    const bool empty = ((len - 1) >> 26) != 0;
    const uint32_t rs = (uint32_t)S & 15u;
    const uint32_t re = rs + (empty ? 0u : (uint32_t)len);
    const uint32_t nseg = empty ? 0u : (re + 15u) >> 4;
    const uint32_t t = empty ? 16u : ((re - 1u) & 15u) + 1u;
    const uint64_t a0 = S & ~(uint64_t)15;
    return LaneMeta{(uint32_t)a0, (uint32_t)(a0 >> 32), rs | (t << 4) | (nseg << 9)};
}

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
        rel_s = (int)(S & 15);
        // Lengths of 2 GiB or more, and E < S, are outside every contract: empty packet.
        // ((len - 1) >> 31) != 0  <=>  len == 0 || len >= 2^31, in SALU-only 64-bit ops
        // (gfx950 SALU has no unsigned 64-bit ordered compare).
        const uint64_t len = E - S;
        const bool empty = ((len - 1) >> 31) != 0;
        rel_e = rel_s + (empty ? 0 : (int)(uint32_t)len);
        nseg = empty ? 0 : (rel_e + 15) >> 4;
        hm = load_mask(kMaskFrom[rel_s]);
        tm = load_mask(kMaskTo[empty ? 16 : ((rel_e - 1) & 15) + 1]);  // tail bytes, 1..16
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

    // issue() from a packed LaneMeta (wave-uniform values read back with v_readlane).
    __device__ __forceinline__ void issue_meta(uint64_t a0, uint32_t packed, uint32_t voff) {
        A0 = a0;
        rel_s = (int)(packed & 15u);
        const int t = (int)((packed >> 4) & 31u);
        nseg = (int)(packed >> 9);
        rel_e = nseg > 0 ? 16 * (nseg - 1) + t : rel_s;
        hm = load_mask(kMaskFrom[rel_s]);
        tm = load_mask(kMaskTo[t]);
        rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(A0), (short)0,
                                                 nseg * 16, 0x00020000);
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
        return wave_sum(lane_partial(lane, voff, not_lane0));
    }

    // This lane's share of finish() before the cross-lane sum (< 2^18 per lane), so that a
    // wave can reduce several packets' partials together (wave_sum_n).
    __device__ __forceinline__ uint32_t lane_partial(int lane, uint32_t voff, uint32_t not_lane0) {
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
        return (s0 & 0xFFFFu) + (s0 >> 16) + (s1 & 0xFFFFu) + (s1 >> 16);
    }
};

// wave_sum of N values at once: the N DPP chains interleave, so each chain's data-hazard
// wait states are filled by the others' instructions instead of s_nop. Results
// wave-uniform.
template <int N>
__device__ __forceinline__ void wave_sum_n(uint32_t (&v)[N]) {
#define AIPSTACK_DPP_N(ctrl, rowmask)                                                     \
    _Pragma("unroll") for (int i = 0; i < N; ++i)                                         \
        v[i] += __builtin_amdgcn_update_dpp(0u, v[i], ctrl, rowmask, 0xF, false);
    AIPSTACK_DPP_N(0x111, 0xF)
    AIPSTACK_DPP_N(0x112, 0xF)
    AIPSTACK_DPP_N(0x114, 0xF)
    AIPSTACK_DPP_N(0x118, 0xF)
    AIPSTACK_DPP_N(0x142, 0xA)
    AIPSTACK_DPP_N(0x143, 0xC)
#undef AIPSTACK_DPP_N
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = __builtin_amdgcn_readlane(v[i], 63);
}

// No per-packet adjustment (see sum_lane_packets).
struct NoMaskHook {
    static constexpr bool kField = false;
    template <class PK>
    __device__ __forceinline__ void issue(int, int) {}
    template <class PK>
    __device__ __forceinline__ void apply(int, PK &, int) {}
    __device__ __forceinline__ int row_field(int) { return -64; }
};

// ---------------------------------------------------------------------------------
// Row mode: packets of at most 16 aligned segments (<= 241 bytes at worst alignment),
// four per wave instruction. Row r (lanes 16r..16r+15) holds one packet; lane k of the
// row loads the packet's segment k with a per-lane address (its row's LaneMeta fetched
// with ds_bpermute), masks its own head/tail bytes in VALU, and the 16 lanes of a row are
// added by a 4-step row DPP scan. Same sum as the wave mode (an end-around-carry sum of
// the masked little-endian dwords), at a quarter of the per-packet instructions.
// ---------------------------------------------------------------------------------
constexpr uint32_t kRowSegs = 16;

// Row groups (of four packets) a kernel keeps in flight; 0 = no row mode. Per kernel
// family, measured; overridable at build time for experiments.
#ifndef AIPSTACK_ROWS_STRIDED
#define AIPSTACK_ROWS_STRIDED 0
#endif
#ifndef AIPSTACK_ROWS_CSR
#define AIPSTACK_ROWS_CSR 0
#endif
#ifndef AIPSTACK_ROWS_FRAMES
#define AIPSTACK_ROWS_FRAMES 0
#endif

__device__ u32x4 g_zero_segment;  // a valid address for rows without a packet

// Keep bytes [a, b) of a little-endian dword (a, b clamped to 0..4).
__device__ __forceinline__ uint32_t dword_keep(int a, int b) {
    a = min(max(a, 0), 4);
    b = min(max(b, 0), 4);
    return b > a ? ((0xFFFFFFFFu >> (32 - 8 * (b - a))) << (8 * a)) : 0u;
}

// Edge / boundary segments (the few per chunk read outside the stream): their cache policy.
// 0 = default (the stream reads the same line again and finds it in L2), 1 = nontemporal.
#ifndef AIPSTACK_EDGE_NT
#define AIPSTACK_EDGE_NT 0
#endif
constexpr bool kEdgeNT = AIPSTACK_EDGE_NT != 0;

// `nt` (wave-uniform, run time): the AIPSTACK_CHKSUM_JUST_WRITTEN hint -- on lines ordinary
// stores wrote since they were last read, a cached read is the expensive one.
__device__ __forceinline__ u32x4 load_edge_segment(uint64_t addr, bool nt = false) {
    typedef __attribute__((address_space(1))) const u32x4 gseg;
    const gseg *p = (const gseg *)addr;
    if (kEdgeNT || nt)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
__device__ __forceinline__ u32x4 load_edge_segment(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                                   bool nt = false) {
    return (kEdgeNT || nt) ? load_segment<true>(rsrc, voff, 0u) : load_segment<false>(rsrc, voff, 0u);
}

template <bool NT>
__device__ __forceinline__ u32x4 load_lane_segment(uint64_t addr) {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(addr);
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

template <int kRowGroups, bool NT, class Hook>
__device__ __forceinline__ uint32_t sum_row_packets(const LaneMeta &meta, uint64_t todo,
                                                    int lane, uint32_t sums, Hook &hook) {
    const int row = lane >> 4, k = lane & 15;
    while (todo) {
        u32x4 v[kRowGroups];
        int jr[kRowGroups][4];
        uint32_t packed_l[kRowGroups];
        int src_l[kRowGroups];
#pragma unroll
        for (int g = 0; g < kRowGroups; ++g) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const bool valid = todo != 0;
                jr[g][r] = valid ? (int)__builtin_ctzll(todo) : -1;
                todo &= todo - 1;
            }
            int src = jr[g][0];
            src = row == 1 ? jr[g][1] : src;
            src = row == 2 ? jr[g][2] : src;
            src = row == 3 ? jr[g][3] : src;
            const int from = max(src, 0) << 2;
            const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)meta.a0_lo);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)meta.a0_hi);
            const uint32_t packed = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)meta.packed);
            const uint32_t nseg = packed >> 9;  // 1..16 for a row packet
            const uint32_t kk = min((uint32_t)k, nseg - 1u);
            const uint64_t addr = src >= 0
                                      ? ((((uint64_t)hi << 32) | lo) + 16u * (uint64_t)kk)
                                      : (uint64_t)(uintptr_t)&g_zero_segment;
            v[g] = load_lane_segment<NT>(addr);
            packed_l[g] = packed;
            src_l[g] = src;
        }
        uint32_t part[kRowGroups];
#pragma unroll
        for (int g = 0; g < kRowGroups; ++g) {
            const uint32_t packed = packed_l[g];
            const int nseg = (int)(packed >> 9);
            const bool in = src_l[g] >= 0 && k < nseg;
            const int lo = k == 0 ? (int)(packed & 15u) : 0;
            const int hi = k == nseg - 1 ? (int)((packed >> 4) & 31u) : 16;
            int fx = -64;  // a 2-byte field summed as 0, bytes from the packet's A0
            if constexpr (Hook::kField)
                fx = hook.row_field(max(src_l[g], 0)) - 16 * k;
            Eac a;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                uint32_t m = dword_keep(lo - 4 * d, hi - 4 * d);
                if constexpr (Hook::kField)
                    m &= ~dword_keep(fx - 4 * d, fx + 2 - 4 * d);
                a.add(v[g][d] & (in ? m : 0u));
            }
            const uint32_t s0 = a.finish();
            part[g] = (s0 & 0xFFFFu) + (s0 >> 16);  // < 2^17; 16 lanes < 2^21
        }
        // row sums: 4-step row scan, interleaved across the groups; lane 16r+15 = row r
#define AIPSTACK_ROW_STEP(ctrl)                                                             \
    _Pragma("unroll") for (int g = 0; g < kRowGroups; ++g)                                   \
        part[g] += __builtin_amdgcn_update_dpp(0u, part[g], ctrl, 0xF, 0xF, false);
        AIPSTACK_ROW_STEP(0x111)
        AIPSTACK_ROW_STEP(0x112)
        AIPSTACK_ROW_STEP(0x114)
        AIPSTACK_ROW_STEP(0x118)
#undef AIPSTACK_ROW_STEP
#pragma unroll
        for (int g = 0; g < kRowGroups; ++g)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t t = (uint32_t)__builtin_amdgcn_readlane(part[g], 16 * r + 15);
                sums = (lane == jr[g][r]) ? t : sums;
            }
    }
    return sums;
}

// The packets of a 64-packet chunk whose lanes are set in `todo` (wave-uniform): with
// RG > 0, those of at most 16 segments four per wave instruction (sum_row_packets, RG
// groups in flight); the others each
// summed by the whole wave with P packets' loads in flight; lane j receives packet j's
// exact halves-sum (< 2^24; 0 iff all its bytes are 0), other lanes 0. `meta` is the
// per-lane LaneMeta. hook.issue(q, j) runs when packet j's loads are issued into slot q,
// hook.apply(q, pk, lane) just before slot q is reduced (e.g. to mask a field).
template <int U, int P, int RG, bool NT, class Hook>
__device__ __forceinline__ uint32_t sum_lane_packets(const LaneMeta &meta, uint64_t todo,
                                                     int lane, uint32_t voff,
                                                     uint32_t not_lane0, Hook &hook) {
    uint32_t sums = 0;
    if constexpr (RG > 0) {
        const uint64_t small =
            todo & __builtin_amdgcn_ballot_w64((meta.packed >> 9) <= kRowSegs);
        if (small) {
            sums = sum_row_packets<RG, NT>(meta, small, lane, sums, hook);
            todo &= ~small;
        }
    }
    while (todo) {
        PacketLoad<U, NT> pk[P];
        int jq[P];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const bool valid = todo != 0;
            const int j = valid ? (int)__builtin_ctzll(todo) : 0;
            todo &= todo - 1;
            jq[q] = valid ? j : -1;
            const uint64_t a0 = ((uint64_t)__builtin_amdgcn_readlane(meta.a0_hi, j) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane(meta.a0_lo, j);
            const uint32_t packed =
                valid ? (uint32_t)__builtin_amdgcn_readlane(meta.packed, j) : 16u << 4;
            hook.template issue<PacketLoad<U, NT>>(q, j);
            pk[q].issue_meta(a0, packed, voff);
        }
        uint32_t part[P];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            hook.apply(q, pk[q], lane);
            part[q] = pk[q].lane_partial(lane, voff, not_lane0);
        }
        wave_sum_n<P>(part);  // wave-uniform
#pragma unroll
        for (int q = 0; q < P; ++q) sums = (lane == jq[q]) ? part[q] : sums;
    }
    return sums;
}

// ---------------------------------------------------------------------------------
// Stream mode: a chunk whose 64 packets lie back to back in memory (packet j ends where
// packet j+1 starts: every CSR batch with non-decreasing offsets, strided batches with
// stride == len) is read as ONE contiguous byte run, 1 KiB per wave instruction, with no
// per-packet loads, masks or reductions. Packet sums come from prefix differences:
//
//   H(x)  = exact sum of the little-endian 16-bit halves of the bytes [A, x), A = S_0 & ~15
//           (bytes read through their aligned dwords, the bytes at or above x as 0);
//   sum_j = H(S_{j+1}) - H(S_j) = the exact halves-sum of packet j's masked dwords.
//
// The halves-sum (v_sad_u16 against 0 adds a dword's two halves, one VALU op) is exact,
// so sum_j is 0 iff every byte of packet j is 0 and is congruent mod 0xFFFF to the
// little-endian ones'-complement sum: the same value the wave mode produces, folded and
// oriented identically. A packet of at most 2^17 - 1 bytes has sum_j < 2^32, so H is
// kept modulo 2^32 (wrap-around subtraction stays exact).
//
// Per 1 KiB window: lane k loads segment k (buffer_load_dwordx4, range-checked to the
// chunk), adds its halves (4 v_sad_u16), and an inclusive DPP scan gives each segment's
// prefix. Lane j evaluates H(S_j) in the window holding S_j: the prefix before S_j's
// segment and that segment's dwords (ds_bpermute from the lane that loaded it), masked
// below S_j. All 64 boundaries are evaluated in parallel, so the cost per window does
// not depend on how many packets it holds.
// ---------------------------------------------------------------------------------
constexpr uint32_t kStreamMaxLen = (1u << 17) - 1u;

__device__ __forceinline__ uint32_t halves(uint32_t x, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(x, 0u, acc);  // (x & 0xFFFF) + (x >> 16) + acc
}

// Halves-sum of bytes [0, o) of one aligned 16-byte segment (o < 16).
__device__ __forceinline__ uint32_t halves_below_seg(const u32x4 &x, uint32_t o) {
    uint32_t acc = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) acc = halves(x[d] & dword_keep(0, (int)o - 4 * d), acc);
    return acc;
}

// Inclusive prefix sum over the 64 lanes (row scan + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);
    return v;
}

// Whether the chunk can take stream mode (wave-uniform): lanes < cnt hold packets
// [S, E) with E - S <= kStreamMaxLen, and each packet ends where the next one starts.
__device__ __forceinline__ bool stream_ok(uint64_t S, uint64_t E, int lane, int cnt) {
    const uint32_t s_lo = (uint32_t)S, s_hi = (uint32_t)(S >> 32);
    const uint64_t next = ((uint64_t)from_next_lane(s_hi, 0u, lane) << 32) |
                          from_next_lane(s_lo, 0u, lane);
    const bool bad = lane < cnt && ((E - S) > kStreamMaxLen || (lane + 1 < cnt && E != next));
    return __builtin_amdgcn_ballot_w64(bad) == 0;
}

// H at NB boundaries per lane over the wave-uniform byte run [A, X1) (A 16-aligned, the run
// < 2^32 bytes). begin() issues the first U windows' loads, so that a kernel can overlap
// them with other work (the frame kernels' header parse); prefixes() then gives
// h[k] = H(b[k]) for every b[k] in [A, X1], and hx = H(X1). Windows past the run read
// zeros (range check) and change nothing.
struct NoStreamHook {
    static constexpr bool kWantH = false;  // window() gets H at each segment start (else 0)
    __device__ __forceinline__ void group(uint32_t) {}
    __device__ __forceinline__ void window(const u32x4 &, uint32_t, uint32_t) {}
};

// DB (round 4): the next group of U windows is issued before the current one is summed (two
// register sets, as the gathered stream does, §5.2 of DESIGN.md), so a wave always has
// U..2U windows in flight; without it the next group goes out only after the current one is
// summed.
#ifndef AIPSTACK_STREAM_DB  // the checksum batches' stream mode with DB (A/B build switch;
#define AIPSTACK_STREAM_DB 0  // round 4: A 233.2 vs 233.6 us, so off)
#endif
// GL (round 5, the short runs' experiment switch): global_load_dwordx4 from the wave-uniform
// run start plus a 32-bit lane offset (the gathered stream's load form) instead of a buffer
// descriptor; segments past the run re-read its last segment and are summed as 0.
template <int U, bool NT, int PRE = U, bool DB = false, bool GL = false>
struct StreamRun {
    uint64_t A, X1;
    uint32_t nseg, nwin;
    __amdgpu_buffer_rsrc_t rsrc;
    u32x4 v[U];
    u32x4 v2[DB ? U : 1];

    __device__ __forceinline__ u32x4 load_win(uint32_t voff, uint32_t w) const {
        if constexpr (GL) {
            // an empty run (a chunk of empty packets on a segment boundary, possibly at the
            // very end of an allocation) has no segment to clamp to: no load at all
            if (nseg == 0u) return u32x4{0u, 0u, 0u, 0u};
            const uint32_t k = min(w * 64u + (voff >> 4), nseg - 1u);
            typedef __attribute__((address_space(1))) const u32x4 gseg;
            const gseg *p = (const gseg *)(A + 16ull * k);
            return NT ? __builtin_nontemporal_load(p) : *p;
        } else {
            return load_segment<NT>(rsrc, voff, w * 1024u);
        }
    }

    // Issues windows [0, PRE) now (the rest of the first U when prefixes() starts): a
    // kernel that overlaps begin() with register-hungry work keeps only PRE in flight.
    __device__ __forceinline__ void begin(uint64_t a, uint64_t x1, uint32_t voff) {
        A = a;
        X1 = x1;
        nseg = ((uint32_t)(X1 - A) + 15u) >> 4;
        nwin = (nseg + (uint32_t)kWave - 1u) >> 6;
        rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(A), (short)0,
                                                 (int)(nseg * 16u), 0x00020000);
        issue<0, PRE>(0, voff);
    }

    // Slots [U0, U1) <- windows w + U0 .. w + U1 - 1, in window order: the loop consumes
    // them in that order with counted waits (s_waitcnt vmcnt(U - 1 - u)); the scheduler
    // barriers stop LLVM from reordering them.
    template <int U0, int U1>
    __device__ __forceinline__ void issue(uint32_t w, uint32_t voff) {
#pragma unroll
        for (int u = U0; u < U1; ++u) {
            v[u] = load_win(voff, w + (uint32_t)u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    template <int N>
    __device__ __forceinline__ void issue_into(u32x4 (&dst)[N], uint32_t w, uint32_t voff) {
#pragma unroll
        for (int u = 0; u < N; ++u) {
            dst[u] = load_win(voff, w + (uint32_t)u);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // h[k] = H(b[k]) for every b[k] in [A, X1], and hx = H(X1). ALIGNED: h[k] = H at the
    // start of b[k]'s 16-byte segment instead (one ds_bpermute per boundary and window, no
    // partial segment; the caller adds the bytes of that segment below b[k] from data it
    // holds itself), except h[k] = hx for b[k] == X1.
    // hook.group(w) runs before the windows [w, w + U) are consumed, hook.window(v, w) once
    // per window with its data (the frame kernels copy header segments out of the stream).
    template <int NB, bool ALIGNED = false, class Hook = NoStreamHook>
    __device__ __forceinline__ void prefixes(const uint64_t (&b)[NB], uint32_t (&h)[NB],
                                             uint32_t &hx, uint32_t voff, Hook &&hook = Hook()) {
        // each boundary: its window, owner lane (x4 for ds_bpermute), dword masks below it
        uint32_t bwin[NB];
        int bsrc[NB];
        uint32_t below[NB][4];
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const uint32_t boff = (uint32_t)(b[k] - A);
            bwin[k] = boff >> 10;
            bsrc[k] = (int)(((boff >> 4) & 63u) << 2);
#pragma unroll
            for (int d = 0; d < 4; ++d)
                below[k][d] = ALIGNED ? 0u : dword_keep(0, (int)(boff & 15u) - 4 * d);
            h[k] = 0;
        }
        // X1's segment (the last one; past X1 it holds bytes outside the run): window, lane
        const uint32_t xt = (uint32_t)(X1 - A) & 15u;
        const uint32_t xwin = (nseg - 1u) >> 6;
        const int xlane = (int)((nseg - 1u) & 63u);
        uint32_t xabove[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) xabove[d] = ~dword_keep(0, (int)xt - 4 * d);

        if constexpr (PRE < U) issue<PRE, U>(0, voff);
        uint32_t carry = 0;  // H(start of the current window), mod 2^32
        uint32_t x_hi = 0;   // halves of the last segment's bytes at or above X1
        // one group of U windows [w, w + U) held in vv
        auto consume = [&](const u32x4 (&vv)[U], uint32_t w) {
            hook.group(w);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t wu = w + (uint32_t)u;
                uint32_t s =
                    halves(vv[u][0], halves(vv[u][1], halves(vv[u][2], halves(vv[u][3], 0u))));
                if constexpr (GL)  // past the run: a re-read of its last segment, counted 0
                    s = wu * 64u + (voff >> 4) < nseg ? s : 0u;
                const uint32_t incl = wave_incl_scan(s);
                const uint32_t excl = incl - s;
#pragma unroll
                for (int k = 0; k < NB; ++k) {
                    if (__builtin_amdgcn_ballot_w64(bwin[k] == wu)) {  // boundaries in window
                        uint32_t part = (uint32_t)__builtin_amdgcn_ds_bpermute(bsrc[k], (int)excl);
                        if constexpr (!ALIGNED) {
#pragma unroll
                            for (int d = 0; d < 4; ++d)
                                part = halves((uint32_t)__builtin_amdgcn_ds_bpermute(
                                                  bsrc[k], (int)vv[u][d]) &
                                                  below[k][d],
                                              part);
                        }
                        if (bwin[k] == wu) h[k] = carry + part;
                    }
                }
                if (wu == xwin && xt != 0) {  // wave-uniform: X1 falls inside this segment
                    uint32_t hh = 0;
#pragma unroll
                    for (int d = 0; d < 4; ++d) hh = halves(vv[u][d] & xabove[d], hh);
                    x_hi = (uint32_t)__builtin_amdgcn_readlane((int)hh, xlane);
                }
                // H at this lane's segment start, for hooks that keep it (frames' capture)
                const uint32_t hseg = std::remove_reference_t<Hook>::kWantH ? carry + excl : 0u;
                carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                hook.window(vv[u], wu, hseg);
            }
        };
        if constexpr (DB) {
            // as the gathered stream: group g + 1 is issued before group g is summed; the loop
            // runs while at least three groups remain (both issues needed and unconditional,
            // so every wait is counted), the last one or two groups straight-line
            const uint32_t groups = (nwin + U - 1u) / U;
            uint32_t g = 0;
            for (; g + 2u < groups; g += 2u) {
                issue_into(v2, (g + 1u) * U, voff);
                consume(v, g * U);
                issue<0, U>((g + 2u) * U, voff);
                consume(v2, (g + 1u) * U);
            }
            if (g + 2u == groups) {
                issue_into(v2, (g + 1u) * U, voff);
                consume(v, g * U);
                consume(v2, (g + 1u) * U);
            } else {
                consume(v, g * U);
            }
        } else {
            for (uint32_t w = 0; w < nwin; w += U) {
                consume(v, w);
                if (w + U < nwin) issue<0, U>(w + U, voff);
            }
        }
        hx = carry - x_hi;  // H(X1)
#pragma unroll
        for (int k = 0; k < NB; ++k)
            if (b[k] == X1) h[k] = hx;  // a boundary at X1 may lie past the last window
    }
};

// Inclusive max-scan over the 64 lanes (-1 = unset).
__device__ __forceinline__ int wave_max_scan(int v) {
#define AIPSTACK_MAXSCAN(ctrl, rowmask) \
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, ctrl, rowmask, 0xF, false));
    AIPSTACK_MAXSCAN(0x111, 0xF)
    AIPSTACK_MAXSCAN(0x112, 0xF)
    AIPSTACK_MAXSCAN(0x114, 0xF)
    AIPSTACK_MAXSCAN(0x118, 0xF)
    AIPSTACK_MAXSCAN(0x142, 0xA)
    AIPSTACK_MAXSCAN(0x143, 0xC)
#undef AIPSTACK_MAXSCAN
    return v;
}

// Exact halves-sum of lane j's own short chunk [a, a + l) (l <= 128 B here: at most 9
// segments), read by the lane itself: its aligned 16-byte segments, nontemporal, the bytes
// outside the chunk masked off; kmax = the wave's largest segment count (uniform). The chain
// kernel's header nodes (round 6, chain runs): side by side in memory, adjacent lanes read
// adjacent segments, so one wave instruction fetches whole lines.
__device__ __forceinline__ uint32_t sum_own_short_chunk(uint64_t a, uint32_t l, uint32_t kmax) {
    typedef __attribute__((address_space(1))) const u32x4 gseg;
    const uint32_t rs = (uint32_t)a & 15u;
    const uint32_t nsg = l ? (rs + l + 15u) >> 4 : 0u;
    const uint32_t te = ((rs + l - 1u) & 15u) + 1u;  // the chunk's end in its last segment
    const gseg *p = (const gseg *)(a & ~(uint64_t)15);
    uint32_t acc = 0;
    for (uint32_t k = 0; k < kmax; ++k) {
        if (k < nsg) {
            const u32x4 x = __builtin_nontemporal_load(p + k);
            const int lo = k == 0 ? (int)rs : 0, hi = k + 1 == nsg ? (int)te : 16;
#pragma unroll
            for (int d = 0; d < 4; ++d) acc = halves(x[d] & dword_keep(lo - 4 * d, hi - 4 * d), acc);
        }
    }
    return acc;
}

// The same with the chunk's first two segments already loaded (x0, x1: issued early, so that
// their latency hides behind other loads); segments 2.. are loaded here.
__device__ __forceinline__ uint32_t sum_short_chunk_from(const u32x4 &x0, const u32x4 &x1,
                                                         uint64_t a, uint32_t l, uint32_t kmax) {
    typedef __attribute__((address_space(1))) const u32x4 gseg;
    const uint32_t rs = (uint32_t)a & 15u;
    const uint32_t nsg = l ? (rs + l + 15u) >> 4 : 0u;
    const uint32_t te = ((rs + l - 1u) & 15u) + 1u;
    const gseg *p = (const gseg *)(a & ~(uint64_t)15);
    uint32_t acc = 0;
    for (uint32_t k = 0; k < kmax; ++k) {
        if (k < nsg) {
            const u32x4 x = k == 0 ? x0 : k == 1 ? x1 : __builtin_nontemporal_load(p + k);
            const int lo = k == 0 ? (int)rs : 0, hi = k + 1 == nsg ? (int)te : 16;
#pragma unroll
            for (int d = 0; d < 4; ++d) acc = halves(x[d] & dword_keep(lo - 4 * d, hi - 4 * d), acc);
        }
    }
    return acc;
}

// ---------------------------------------------------------------------------------
// Gathered stream (the chain kernel): up to 64 chunks anywhere in memory (lane j: chunk
// [a_j, a_j + l_j), l_j <= 65535, empty chunks allowed) read as ONE stream of just their
// 16-byte segments. The segments of chunk j, in order, get the compact indices
// [cs_j, cs_j + ns_j) (cs = exclusive scan of the counts); window w is compact indices
// [64w, 64w + 64), and lane k loads index c = 64w + k from the chunk that owns it, at
// gbase_owner + 16 c (gbase_j = (a_j & ~15) - 16 cs_j).
//
// Owners: the non-empty chunks' load parameters sit in LDS by rank; per group of U windows
// each chunk starting there ORs its start lane into its window's 64-bit mask, and lane k of
// window w takes rank base_w - 1 + popcount(mask bits <= k) (two mbcnt; round 2 -- a mark
// table and a DPP max-scan per window before). With G_j = the prefix of whole-segment
// halves-sums up to segment cs_j (a segment-aligned position: no partial segment to fetch),
// G_{j+1} - G_j is the sum of chunk j's segments: one boundary per lane, evaluated with one
// ds_bpermute of the window's exclusive scan. Those segments also hold bytes that are not the
// chunk's -- below a_j & 15 in its first segment, from its end on in its last -- and lane j
// subtracts them: it reads its chunk's two edge segments itself before the stream starts
// (round 4, EDGE; rounds 2-3 masked them off in the stream, every lane of every window
// looking up a keep mask -- kept for bytes read over the link, !EDGE). A segment shared by two chunks is loaded once
// for each (the second time from L2); bytes outside every chunk's segments are never read,
// so chunks may sit in separate allocations (a 16-byte segment around a mapped byte is
// mapped). Lanes past the stream re-read its last segment and count 0, so every address
// stays inside a chunk.
//
// Software-pipelined: group g + 1's owners and loads are issued before group g is
// consumed; the next group is issued unconditionally while at least three groups remain
// (the last one or two are finished straight-line), so the loads stay straight-line and
// every wait is counted (vmcnt(N)), also across the back edge. Windows of the last group
// past the stream are loaded with it but not summed.
// ---------------------------------------------------------------------------------
// How a chunk's first and last segments lose the bytes that are not the chunk's (template
// flag EDGE): true (round 4, the default) = the stream sums whole segments, and each lane
// reads its chunk's two edge segments itself up front and subtracts their foreign bytes;
// false = every loaded segment masked in the stream (a keep-table index per lane and window,
// rounds 2-3), kept for bytes read over the link from host memory, where an edge segment
// read twice crosses the link twice (the engine's zero-copy ring slots). Round 4
// (profiles/r04/edge): masked C2K 262.4 / CHAIN 241.2 us, edge loads 256.1 / 236.0 us
// (VALU -21 / -26 %; CHAIN's FETCH_SIZE +2 %: an edge line read up front is sometimes gone
// when the stream gets to it). Copying the edge segments out of the stream windows into LDS
// instead (exec-masked ds_write per window) cut VALU as far but cost SALU and ran
// 264.6 / 241.8 us.

// Per-wave LDS scratch of the gathered stream: the owners' load parameters by rank (rank =
// non-empty chunks before it), and the chunk-start masks of the current group's windows.
struct GatherLds {
    u32x4 owner[kWave];   // {gbase lo, gbase hi, first_info, last_info}
    uint64_t starts[8];   // per window of the group: bit k = a chunk starts at lane k
};

// LDS table of byte masks: entry head * 16 + (tail - 1) keeps bytes [head, tail) of a
// 16-byte segment (head 0..15, tail 1..16). Filled once per block by fill_keep_table().
typedef u32x4 KeepTable[256];

__device__ __forceinline__ void fill_keep_table(KeepTable &t) {
    for (int i = (int)threadIdx.x; i < 256; i += (int)blockDim.x) {
        const int head = i >> 4, tail = (i & 15) + 1;
        t[i] = u32x4{dword_keep(head, tail), dword_keep(head - 4, tail - 4),
                     dword_keep(head - 8, tail - 8), dword_keep(head - 12, tail - 12)};
    }
}

// The bytes of a chunk's first segment below its start (h = start & 15) and of its last
// segment from its end on (t = ((end - 1) & 15) + 1), as a halves-sum.
__device__ __forceinline__ uint32_t foreign_halves(const u32x4 &first, const u32x4 &last, int h,
                                                   int t) {
    uint32_t f = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        f = halves(first[d] & dword_keep(-4 * d, h - 4 * d), f);
        f = halves(last[d] & dword_keep(t - 4 * d, 16 - 4 * d), f);
    }
    return f;
}

template <int U, bool NT, bool EDGE>
struct ChunkLoader {
    static_assert(U <= 8, "GatherLds holds 8 window masks");
    uint32_t T;
    uint32_t start_win;     // the window its chunk starts in (~0: empty chunk)
    uint32_t start_bit;     // the lane its chunk starts at, within that window
    uint32_t base;          // non-empty chunks starting before the next group (uniform)
    int lane;
    GatherLds *g;

    // Windows [w, w + U): loads into v, and (!EDGE) each lane's keep-table index into
    // keep. The owner of compact index 64w + k is the last chunk starting at or before it:
    // its rank is base_w - 1 + (starts at lanes <= k of window w)
    // = base_w + bit0 - 1 + mbcnt(m >> 1).
    __device__ __forceinline__ void issue(uint32_t w, u32x4 (&v)[U], uint32_t (&keep)[U]) {
        uint64_t mk[U];
        if (lane < U) g->starts[lane] = 0ull;
        __builtin_amdgcn_wave_barrier();
        const uint32_t du = start_win - w;  // < U: starts in this group
        if (du < (uint32_t)U)
            __hip_atomic_fetch_or(&g->starts[du], 1ull << start_bit, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WAVEFRONT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t x = g->starts[u];
            mk[u] = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
                    (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t m1 = mk[u] >> 1;
            const uint32_t rank = base + ((uint32_t)mk[u] & 1u) - 1u +
                                  __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
            base += (uint32_t)__builtin_popcountll(mk[u]);
            const u32x4 od = g->owner[rank & (uint32_t)(kWave - 1)];
            const uint32_t c0 = (w + (uint32_t)u) * (uint32_t)kWave + (uint32_t)lane;
            const uint32_t c = min(c0, T - 1u);
            if constexpr (!EDGE) {
                const uint32_t fi = od[2], li = od[3];
                const uint32_t head = c == (fi & 0xFFFFFFu) ? fi >> 24 : 0u;
                const uint32_t tail = c == (li & 0xFFFFFFu) ? li >> 24 : 16u;
                keep[u] = head * 16u + tail - 1u;
            }
            const uint64_t addr = (((uint64_t)od[1] << 32) | od[0]) + 16ull * c;
            typedef __attribute__((address_space(1))) const u32x4 gseg;
            const gseg *p = (const gseg *)(addr);
            if constexpr (NT)
                v[u] = __builtin_nontemporal_load(p);
            else
                v[u] = *p;
        }
    }
};

// The chain kernel's 64 chunk sums (also the ring slots' chunks). `g`: this wave's LDS
// scratch; `keep_table`: the block's mask table (fill_keep_table; !EDGE only, else unused and
// may be null). Returns lane j's
// exact halves-sum of its chunk.
template <int U, bool NT, bool EDGE = true>
__device__ __forceinline__ uint32_t sum_gathered_chunks(uint64_t a, uint32_t l, int lane,
                                                        GatherLds *glds,
                                                        const KeepTable *keep_table,
                                                        bool edge_nt = false) {
    const uint32_t rs = (uint32_t)a & 15u;
    const uint32_t ns = l ? (rs + l + 15u) >> 4 : 0u;
    const uint32_t ns_incl = wave_incl_scan(ns);
    const uint32_t cs = ns_incl - ns;
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)ns_incl, 63);
    if (T == 0) return 0;
    const uint32_t nwin = (T + (uint32_t)kWave - 1u) >> 6;
    ChunkLoader<U, NT, EDGE> ld;
    ld.T = T;
    const uint64_t gbase = (a & ~(uint64_t)15) - 16ull * cs;
    // the owners' load parameters, by rank among the non-empty chunks
    const uint64_t ne = __builtin_amdgcn_ballot_w64(ns != 0u);
    const uint32_t rank =
        __builtin_amdgcn_mbcnt_hi((uint32_t)(ne >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ne, 0u));
    if (ns)
        glds->owner[rank] = u32x4{(uint32_t)gbase, (uint32_t)(gbase >> 32), cs | rs << 24,
                               (cs + ns - 1u) | ((((rs + l - 1u) & 15u) + 1u) << 24)};
    __builtin_amdgcn_wave_barrier();
    ld.start_win = ns ? (cs >> 6) : ~0u;
    ld.start_bit = cs & 63u;
    ld.base = 0;
    ld.lane = lane;
    ld.g = glds;
    // this lane's boundary: G at segment cs (an empty chunk's cs is the next one's)
    const uint32_t bwin = cs >> 6;
    const int bsrc = (int)((cs & 63u) << 2);
    uint32_t gsum = 0, carry = 0;  // carry: prefix at the current window's start, mod 2^32
    auto consume = [&](uint32_t w, const u32x4 (&v)[U], const uint32_t (&keep)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t wu = w + (uint32_t)u;
            // windows past the stream (the last group's tail) sum zeros and hold no boundary:
            // their loads went out with the group, their scans are skipped (wave-uniform)
            if (wu >= nwin) break;
            const uint32_t c0 = wu * (uint32_t)kWave + (uint32_t)lane;
            uint32_t s;
            if constexpr (!EDGE) {
                const u32x4 km = (*keep_table)[keep[u]];
                s = halves(v[u][0] & km[0],
                           halves(v[u][1] & km[1],
                                  halves(v[u][2] & km[2], halves(v[u][3] & km[3], 0u))));
            } else {
                s = halves(v[u][0], halves(v[u][1], halves(v[u][2], halves(v[u][3], 0u))));
            }
            s = c0 < T ? s : 0u;  // lanes past the stream re-read its last segment
            const uint32_t incl = wave_incl_scan(s);
            if (__builtin_amdgcn_ballot_w64(bwin == wu)) {
                const uint32_t part = (uint32_t)__builtin_amdgcn_ds_bpermute(bsrc, (int)(incl - s));
                if (bwin == wu) gsum = carry + part;
            }
            carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
    };
    u32x4 va[U], vb[U];
    uint32_t ka[U], kb[U];
    // Groups of U windows, double-buffered: group g+1's loads go out before group g is
    // consumed. The loop runs while at least three groups remain, so both of its issues are
    // needed and unconditional (counted waits across the back edge); the last one or two
    // groups are finished straight-line, issuing nothing past the stream.
    const uint32_t groups = (nwin + U - 1u) / U;
    // EDGE: the lane reads its chunk's two edge segments itself (they lie inside the chunk's
    // segments, so they are mapped) before the stream's first group, at the default cache
    // policy (the stream reads the same lines later). Read after the stream's last group was
    // issued instead, they miss L2 more often (the stream's nontemporal lines do not stay):
    // C2K 282 against 268 us, FETCH_SIZE +12 %, CHAIN 271 against 261 (profiles/r05/edgeafter).
    // (none where the chunk starts or ends on a segment boundary: nothing foreign there)
    u32x4 fseg = {0u, 0u, 0u, 0u}, lseg = {0u, 0u, 0u, 0u};
    const uint32_t te = ((rs + l - 1u) & 15u) + 1u;  // the chunk's end in its last segment
    if constexpr (EDGE) {
        if (ns && rs != 0u) fseg = load_edge_segment(a & ~(uint64_t)15, edge_nt);
        if (ns && te != 16u) lseg = load_edge_segment((a + l - 1u) & ~(uint64_t)15, edge_nt);
    }
    ld.issue(0, va, ka);
    const uint32_t foreign = EDGE && ns ? foreign_halves(fseg, lseg, (int)rs, (int)te) : 0u;
    uint32_t g = 0;
    for (; g + 2u < groups; g += 2u) {
        ld.issue((g + 1u) * U, vb, kb);
        consume(g * U, va, ka);
        ld.issue((g + 2u) * U, va, ka);
        consume((g + 1u) * U, vb, kb);
    }
    if (g + 2u == groups) {
        ld.issue((g + 1u) * U, vb, kb);
        consume(g * U, va, ka);
        consume((g + 1u) * U, vb, kb);
    } else {
        consume(g * U, va, ka);
    }
    if (bwin >= nwin) gsum = carry;  // cs == T on a multiple of 64: past the last window
    // chunk j ends where chunk j + 1 starts (lane 63: at T, prefix = the final carry)
    return from_next_lane(gsum, carry, lane) - gsum - foreign;
}

// Segment-table runs (round 5, SU = 96): the run read as in column runs, and each window's 64
// segment sums written to a per-wave LDS table (one ds_write_b32 per window); no per-boundary
// work in the stream at all. After it, packet j's whole segments [g_j, g_{j+1}) are added from
// the table by its 64 / cp lanes (a contiguous share each), then a butterfly, and the partial
// segments at both ends as in column runs: + P_{j+1} - P_j. Runs longer than kSegTabMax
// segments (chunks of very long packets) take the per-packet wave mode.
constexpr uint32_t kSegTabMax = 1536;  // 24 windows: 16 packets of up to ~1.5 KiB
typedef uint32_t SegTab[kSegTabMax];

template <bool NT>
__device__ __forceinline__ uint32_t sum_segtab_chunk(uint64_t S, uint64_t E, int lane, int cnt,
                                                     uint32_t voff, uint32_t cpk, uint32_t *tab) {
    const uint64_t X1 = readlane64(E, cnt - 1);
    if (lane >= cnt) S = X1;
    const uint64_t A =
        (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(S >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)S)) & ~(uint64_t)15;
    const uint32_t nseg = ((uint32_t)(X1 - A) + 15u) >> 4;  // <= kSegTabMax (caller)
    const uint32_t nwin = (nseg + (uint32_t)kWave - 1u) >> 6;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(A), (short)0, (int)(nseg * 16u), 0x00020000);
    const uint32_t rel = (uint32_t)(S - A);
    const uint32_t g = rel >> 4, o = rel & 15u;
    u32x4 bseg = {0u, 0u, 0u, 0u};
    if (lane <= cnt && o != 0u) bseg = load_segment<kEdgeNT>(rsrc, g * 16u, 0u);
    constexpr int U = 8;
    u32x4 va[U], vb[U];
    auto issue = [&](u32x4 (&v)[U], uint32_t w) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = load_segment<NT>(rsrc, voff, (w + (uint32_t)u) * 1024u);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto consume = [&](const u32x4 (&v)[U], uint32_t w) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t wu = w + (uint32_t)u;
            if (wu >= nwin) break;
            tab[wu * kWave + (uint32_t)lane] =
                halves(v[u][0], halves(v[u][1], halves(v[u][2], halves(v[u][3], 0u))));
        }
    };
    const uint32_t groups = (nwin + U - 1u) / U;
    issue(va, 0);
    uint32_t gi = 0;
    for (; gi + 2u < groups; gi += 2u) {
        issue(vb, (gi + 1u) * U);
        consume(va, gi * U);
        issue(va, (gi + 2u) * U);
        consume(vb, (gi + 1u) * U);
    }
    if (gi + 2u == groups) {
        issue(vb, (gi + 1u) * U);
        consume(va, gi * U);
        consume(vb, (gi + 1u) * U);
    } else {
        consume(va, gi * U);
    }
    const uint32_t P = halves_below_seg(bseg, o);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // packet j = lane >> ql: segments [g_j, g_{j+1}) in 2^ql contiguous shares
    const uint32_t ql = 6u - (uint32_t)__builtin_ctz(cpk);  // cpk: a power of two <= 32
    const uint32_t j = (uint32_t)lane >> ql, part = (uint32_t)lane & ((1u << ql) - 1u);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(j, 63u) << 2), (int)g);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(min(j + 1u, 63u) << 2), (int)g);
    uint32_t acc = 0;
    if (j < (uint32_t)cnt) {
        const uint32_t per = ((hi - lo) + (1u << ql) - 1u) >> ql;
        const uint32_t a = lo + part * per;
        const uint32_t b = min(a + per, hi);
        for (uint32_t k = a; k < b; ++k) acc += tab[k];
    }
    for (uint32_t m = 1; m < (1u << ql); m <<= 1)
        acc += (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((uint32_t)lane ^ m) << 2), (int)acc);
    __builtin_amdgcn_wave_barrier();
    const uint32_t col = (uint32_t)__builtin_amdgcn_ds_bpermute(
        (int)((((uint32_t)lane << ql) & 63u) << 2), (int)acc);
    const uint32_t pn = from_next_lane(P, 0u, lane);  // P_{j+1} (lane cnt: X1's)
    __builtin_amdgcn_wave_barrier();  // (the table is rewritten by the next chunk)
    return lane < cnt ? col + pn - P : 0u;
}

// Slot windows (round 5, SU = 128): packets that each lie on their own (ring slots, a fixed
// length at another stride) summed without compacting their segments. Slot k's packet [S, E)
// is read from A0 = S & ~15 as whole 1 KiB windows, lane L taking segment L of each window,
// through a buffer descriptor of exactly its 16 * nseg bytes: lanes past the packet read 0 and
// fetch nothing, so only the packet's own lines cross from HBM. Eight slots' first two windows
// (packets of up to ~2 KiB) are issued together, 16 loads per wave up front; longer packets add
// their further windows after. A lane adds its segments per slot with v_sad_u16 -- no mask and no
// cross-lane work per window -- and the 8 x 64 partial sums are added through a transpose in LDS
// (8 lanes per slot) and a 3-step butterfly. Each packet's first and last segment also hold
// bytes that are not its own; lane k reads them itself before the windows (as the gathered
// stream's edges, foreign_halves) and subtracts them. Per wave of 8 slots: 64 v_sad_u16 for the
// windows, against a DPP scan, an owner lookup and a 64-bit address per window in the gathered
// stream.
constexpr int kSlotGroup = 8;            // slots whose first two windows go out together
typedef uint32_t SlotRows[kSlotGroup * kWave];

template <bool NT>
__device__ __forceinline__ uint32_t sum_slot_windows(uint64_t S, uint64_t E, int lane, int cnt,
                                                     uint32_t voff, uint32_t *rows) {
    const uint64_t A0 = S & ~(uint64_t)15;
    const uint32_t rs = (uint32_t)S & 15u;
    const uint32_t len = lane < cnt ? (uint32_t)(E - S) : 0u;
    const uint32_t nseg = len ? (rs + len + 15u) >> 4 : 0u;
    const uint32_t te = ((rs + len - 1u) & 15u) + 1u;  // the packet's end in its last segment
    // the edge segments' foreign bytes (none on a segment edge), read before the windows
    u32x4 fseg = {0u, 0u, 0u, 0u}, lseg = {0u, 0u, 0u, 0u};
    if (nseg && rs != 0u) fseg = load_edge_segment(A0);
    if (nseg && te != 16u) lseg = load_edge_segment(A0 + 16ull * (nseg - 1u));
    uint32_t mine = 0;  // lane j < cnt: packet j's exact halves-sum (whole segments)
    for (int k0 = 0; k0 < cnt; k0 += kSlotGroup) {
        u32x4 v[kSlotGroup][2];
        __amdgpu_buffer_rsrc_t rs_k[kSlotGroup];
        uint32_t n_k[kSlotGroup];
#pragma unroll
        for (int k = 0; k < kSlotGroup; ++k) {
            const int src = min(k0 + k, kWave - 1);
            const uint64_t a = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(A0 >> 32), src) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)A0, src);
            n_k[k] = k0 + k < cnt ? (uint32_t)__builtin_amdgcn_readlane((int)nseg, src) : 0u;
            rs_k[k] = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(a), (short)0,
                                                        (int)(n_k[k] * 16u), 0x00020000);
        }
#pragma unroll
        for (int k = 0; k < kSlotGroup; ++k) {
            v[k][0] = load_segment<NT>(rs_k[k], voff, 0u);
            __builtin_amdgcn_sched_barrier(0);
            v[k][1] = load_segment<NT>(rs_k[k], voff, 1024u);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int k = 0; k < kSlotGroup; ++k) {
            uint32_t p = halves(v[k][0][0], halves(v[k][0][1], halves(v[k][0][2], halves(v[k][0][3], 0u))));
            p = halves(v[k][1][0], halves(v[k][1][1], halves(v[k][1][2], halves(v[k][1][3], p))));
            for (uint32_t w = 2; w * 64u < n_k[k]; ++w) {  // packets over ~2 KiB (uniform)
                const u32x4 x = load_segment<NT>(rs_k[k], voff, w * 1024u);
                p = halves(x[0], halves(x[1], halves(x[2], halves(x[3], p))));
            }
            rows[k * kWave + lane] = p;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // lane t: slot t >> 3, the partials of lanes 8 (t & 7) .. 8 (t & 7) + 7
        const u32x4 *r = reinterpret_cast<const u32x4 *>(rows + (lane >> 3) * kWave + (lane & 7) * 8);
        const u32x4 a = r[0], b = r[1];
        uint32_t acc = a[0] + a[1] + a[2] + a[3] + b[0] + b[1] + b[2] + b[3];
        acc += (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ 1) << 2, (int)acc);
        acc += (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ 2) << 2, (int)acc);
        acc += (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ 4) << 2, (int)acc);
        // slot k's total is on lanes 8k..8k+7: lane k0 + k takes it from lane 8k
        const int j = lane - k0;
        const uint32_t tot = (uint32_t)__builtin_amdgcn_ds_bpermute(((j & 7) * 8) << 2, (int)acc);
        if (j >= 0 && j < kSlotGroup) mine = tot;
        __builtin_amdgcn_wave_barrier();  // (the rows are rewritten by the next group)
    }
    const uint32_t foreign = nseg ? foreign_halves(fseg, lseg, (int)rs, (int)te) : 0u;
    return lane < cnt ? mine - foreign : 0u;
}

// Stream mode for one chunk (stream_ok). Lane j < cnt holds packet j = [S, E); returns
// lane j's exact halves-sum (0 on lanes >= cnt).
// SU <= 8: SU windows issued together, the next group after the current one is summed (rounds
// 1-4). SU > 8 (round 5, short runs): groups of AIPSTACK_SHORT_RUN_WINDOWS windows,
// double-buffered -- the next group goes out before the current one is summed, so a wave of
// one short chunk issues all of its ~12 KiB before it sums the first window (the gathered
// stream's issue pattern, without its per-window owner lookup and address arithmetic).
// Short runs' stream prefixes: packet starts' partial segments loaded per lane up front (1) or
// taken from the stream (0). Driver protocol (profiles/r05/edge): config C 247.9-250.1 us with
// the loads against 240.5-243.5 without (2 M extra loads); A in stream prefixes 223.4-224.2
// against 230.3-230.5 (A's default, column runs, does this already). A/B build switch.
#ifndef AIPSTACK_STREAM_EDGE_LOADS
#define AIPSTACK_STREAM_EDGE_LOADS 0
#endif
template <int SU, bool NT>
__device__ __forceinline__ uint32_t sum_stream_chunk(uint64_t S, uint64_t E, int lane, int cnt,
                                                     uint32_t voff) {
    constexpr bool kDb = SU > 8 || AIPSTACK_STREAM_DB != 0;
// Short runs' windows per group, double-buffered (A/B build switch): config C under the
// driver's protocol 241.7-242.5 us at 6 against 242.1-249.3 at 8 and 247.3-248.4 at 4
// (profiles/r05/sru): ~12 KiB chunks load 12 windows instead of 16.
#ifndef AIPSTACK_SHORT_RUN_WINDOWS
#define AIPSTACK_SHORT_RUN_WINDOWS 6
#endif
    constexpr int U = SU > 8 ? AIPSTACK_SHORT_RUN_WINDOWS : SU;
    constexpr bool kGl = SU == 32;  // (SU 32: SU 16 through global loads, StreamRun GL)
    // X1 = end of the chunk's last packet; lanes past the batch sit at X1 (empty)
    const int lastl = cnt - 1;
    const uint64_t X1 =
        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(E >> 32), lastl) << 32) |
        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)E, lastl);
    if (lane >= cnt) S = X1;
    const uint64_t S0 =
        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(S >> 32)) << 32) |
        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)S);
    // the run spans <= 64 * 2^17 + 15 bytes (stream_ok)
    StreamRun<U, NT, U, kDb, kGl> run;
    const uint64_t bs[1] = {S};
    uint32_t hb[1], hx;
    if constexpr (AIPSTACK_STREAM_EDGE_LOADS && SU > 8) {
        // Short runs (device memory only): H at each packet start's segment (one ds_bpermute
        // per window with starts, no partial segment from the stream) plus the bytes of that
        // segment below the start, from one segment load per lane before the stream (as column
        // runs; the stream reads that line again later). A start at X1 (lanes past the batch,
        // empty tail packets) is exact. Stream mode (SU <= 8) also reads host memory over the
        // link, where the edge segment would cross it twice.
        const uint64_t A = S0 & ~(uint64_t)15;
        const uint32_t o = (uint32_t)S & 15u;
        u32x4 bseg = {0u, 0u, 0u, 0u};
        if (S != X1 && o != 0u) bseg = load_edge_segment(S & ~(uint64_t)15);
        run.begin(A, X1, voff);
        run.template prefixes<1, true>(bs, hb, hx, voff);
        hb[0] += S != X1 ? halves_below_seg(bseg, o) : 0u;
    } else {
        run.begin(S0 & ~(uint64_t)15, X1, voff);
        run.prefixes(bs, hb, hx, voff);
    }
    const uint32_t hn = from_next_lane(hb[0], hx, lane);  // H(S_{j+1}); lane 63: H(X1)
    return lane < cnt ? hn - hb[0] : 0u;
}

// Column runs (round 5, SU = 64): a short chunk of back-to-back packets (at most
// kColMaxPackets) read as one run of 16-byte segments, 64 per wave instruction (lane L of
// window w loads segment 64w + L), groups of 8 windows double-buffered -- and no cross-lane
// work per window. Each lane keeps the sum of its own column (its segments of the windows
// consumed so far, C). Boundary j of the chunk (packet starts S_0..S_{cnt-1} and the run's end
// X1, lane j holding b_j) lies at byte o_j of segment g_j = 64 W + B; when window W is
// consumed, every lane writes X_{j,L} = C_L + (L < B ? s_L : 0) to row j of an LDS table, so
// that the sum over L of X_{j,L} is the halves-sum of the whole segments before b_j. P_j, the
// halves of segment g_j's bytes below o_j, is added per packet at the end:
//     packet j = sum over L of (X_{j+1,L} - X_{j,L}) + P_{j+1} - P_j   (mod 2^32, exact),
// the column differences added by 64 / cp lanes per packet from the table, then a butterfly.
// Per window: 4 v_sad_u16 and one add per lane; per boundary a select, an add and an LDS write
// (stream mode: a 6-step DPP scan per window and 5 ds_bpermute per boundary).
//
// Where P_j's bytes come from:
//   CAPTURE = false (the default): one default-policy segment load per lane ahead of the
//     stream (the stream finds those lines in L2 later). Steady state 219-223 us on A.
//   CAPTURE = true (AIPSTACK_CHKSUM_JUST_WRITTEN, round 6): captured from the stream -- lane B
//     writes the boundary's segment to a 17-entry LDS table as window W passes (one
//     ds_write_b128 under a one-lane exec mask), lane j reads entry j after the stream; no
//     line of the batch is read through the L2-allocating path. Steady state 228-235 us.
// A default-policy read of a line that plain (write-back) stores wrote since it was last read
// costs the memory side far more than a nontemporal one, and slows the whole stream, not just
// that load: A's first read after a plain-store writer 285-312 us with the loads against
// 242-258 captured; after DMA or nontemporal stores 221-231 against 231-240 (DESIGN 6.1,
// tools/fresh.py, profiles/r06/).
constexpr int kColMaxPackets = 16;
constexpr uint32_t kColSegTab = (kColMaxPackets + 1) * kWave;  // dword offset of the segments
typedef uint32_t ColRows[(kColMaxPackets + 1) * kWave + (kColMaxPackets + 1) * 4];
// MAXP: boundaries per run at most MAXP + 1 (rows of MAXP + 1 columns, then MAXP + 1 segments)
template <int MAXP>
using ColRowsN = uint32_t[(MAXP + 1) * kWave + (MAXP + 1) * 4];

// U: windows per group (8; 6 for chunks of one long packet, launch_short_runs). MAXP: the
// most packets a run holds (rows: a ColRowsN<MAXP>); cpk = 64 / (64 lanes / MAXP per packet).
template <bool NT, int U = 8, bool CAPTURE = false, int MAXP = kColMaxPackets>
__device__ __forceinline__ uint32_t sum_column_chunk(uint64_t S, uint64_t E, int lane, int cnt,
                                                     uint32_t voff, uint32_t cpk, uint32_t *rows) {
    const uint64_t X1 = readlane64(E, cnt - 1);  // end of the chunk's last packet
    if (lane >= cnt) S = X1;                      // lane cnt: boundary X1; past it: unused
    const uint64_t A =
        (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(S >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)S)) & ~(uint64_t)15;
    const uint32_t nseg = ((uint32_t)(X1 - A) + 15u) >> 4;  // the run < 17 * 2^17 bytes
    const uint32_t nwin = (nseg + (uint32_t)kWave - 1u) >> 6;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(A), (short)0, (int)(nseg * 16u), 0x00020000);
    const uint32_t rel = (uint32_t)(S - A);  // lane j: boundary j's byte in the run
    const uint32_t o = rel & 15u;
    uint32_t *const segs = rows + (MAXP + 1) * kWave;  // (CAPTURE) boundary j's segment: entry j
    u32x4 bseg = {0u, 0u, 0u, 0u};            // boundary j's segment (lanes 0..cnt, o != 0)
    if (!CAPTURE && lane <= cnt && o != 0u)
        bseg = load_segment<kEdgeNT>(rsrc, (rel >> 4) * 16u, 0u);
    u32x4 va[U], vb[U];
    auto issue = [&](u32x4 (&v)[U], uint32_t w) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = load_segment<NT>(rsrc, voff, (w + (uint32_t)u) * 1024u);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    uint32_t C = 0;                                                   // this lane's column sum
    uint32_t jb = 0;                                                  // next boundary (uniform)
    uint32_t rj = (uint32_t)__builtin_amdgcn_readlane((int)rel, 0);  // its byte in the run
    auto consume = [&](const u32x4 (&v)[U], uint32_t w) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t wu = w + (uint32_t)u;
            if (wu >= nwin) break;
            const uint32_t s =
                halves(v[u][0], halves(v[u][1], halves(v[u][2], halves(v[u][3], 0u))));
            while (jb <= (uint32_t)cnt && (rj >> 10) == wu) {
                const uint32_t B = (rj >> 4) & 63u;  // the lane holding the boundary's segment
                rows[jb * kWave + (uint32_t)lane] = C + ((uint32_t)lane < B ? s : 0u);
                if constexpr (CAPTURE) {
                    if ((rj & 15u) != 0u && (uint32_t)lane == B)
                        *reinterpret_cast<u32x4 *>(segs + jb * 4u) = v[u];
                }
                ++jb;
                rj = jb <= (uint32_t)cnt ? (uint32_t)__builtin_amdgcn_readlane((int)rel, (int)jb)
                                         : ~0u;
            }
            C += s;
        }
    };
    const uint32_t groups = (nwin + U - 1u) / U;
    issue(va, 0);
    uint32_t gi = 0;
    for (; gi + 2u < groups; gi += 2u) {
        issue(vb, (gi + 1u) * U);
        consume(va, gi * U);
        issue(va, (gi + 2u) * U);
        consume(vb, (gi + 1u) * U);
    }
    if (gi + 2u == groups) {
        issue(vb, (gi + 1u) * U);
        consume(va, gi * U);
        consume(vb, (gi + 1u) * U);
    } else {
        consume(va, gi * U);
    }
    // boundaries at the run's end (X1 on a segment edge: nothing of its segment below it)
    for (; jb <= (uint32_t)cnt; ++jb) rows[jb * kWave + (uint32_t)lane] = C;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (CAPTURE && lane <= cnt && o != 0u)  // every such boundary's window was consumed
        bseg = *reinterpret_cast<const u32x4 *>(segs + (uint32_t)lane * 4u);
    const uint32_t P = halves_below_seg(bseg, o);
    // packet j = lane >> ql: its 2^ql lanes add cpk column differences each
    const uint32_t ql = 6u - (uint32_t)__builtin_ctz(cpk);  // cpk: a power of two <= MAXP
    const uint32_t j = (uint32_t)lane >> ql, part = (uint32_t)lane & ((1u << ql) - 1u);
    uint32_t acc = 0;
    if (j < (uint32_t)cnt) {
        const uint32_t *r0 = rows + j * kWave + part * cpk;
        const uint32_t *r1 = r0 + kWave;
        if (cpk >= 4u) {
            for (uint32_t i = 0; i < cpk; i += 4u) {
                const u32x4 a = *reinterpret_cast<const u32x4 *>(r0 + i);
                const u32x4 b = *reinterpret_cast<const u32x4 *>(r1 + i);
                acc += (b[0] - a[0]) + (b[1] - a[1]) + (b[2] - a[2]) + (b[3] - a[3]);
            }
        } else {
            for (uint32_t i = 0; i < cpk; ++i) acc += r1[i] - r0[i];
        }
    }
    for (uint32_t m = 1; m < (1u << ql); m <<= 1)
        acc += (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((uint32_t)lane ^ m) << 2), (int)acc);
    __builtin_amdgcn_wave_barrier();
    const uint32_t col = (uint32_t)__builtin_amdgcn_ds_bpermute(
        (int)((((uint32_t)lane << ql) & 63u) << 2), (int)acc);
    const uint32_t pn = from_next_lane(P, 0u, lane);  // P_{j+1} (lane cnt: X1's)
    __builtin_amdgcn_wave_barrier();  // (the table is rewritten by the next chunk)
    return lane < cnt ? col + pn - P : 0u;
}

// Gapped column runs (round 5, GappedColDesc, SU = 64): the column runs' loop (each lane adds
// its own column of segments; per-boundary snapshots in LDS) over a chunk's packets read as one
// compact stream of just their segments, lane L of window w loading compact segment 64w + L
// through one buffer descriptor over the chunk's span at k gap + 16 c (five VALU per window,
// against the gathered stream's owner lookup, 64-bit address and DPP scan). Packet j's whole
// segments are [j ns, (j + 1) ns): no boundary falls inside a segment; the bytes of its first
// and last segments that are not its own (below rs, from its end on) come from the two edge
// segments lane j reads up front and are subtracted (foreign_halves).
template <bool NT>
__device__ __forceinline__ uint32_t sum_gapped_column_chunk(uint64_t s0, int lane, int cnt,
                                                            uint32_t cpk, uint32_t *rows,
                                                            const GappedColDesc &d,
                                                            bool edge_nt = false) {
    const uint32_t ns = d.ns;
    const uint32_t rs = (uint32_t)s0 & 15u;
    const uint64_t B0 = s0 & ~(uint64_t)15;
    const uint32_t T = (uint32_t)cnt * ns;  // < 2^16 (launch)
    const uint32_t nwin = (T + (uint32_t)kWave - 1u) >> 6;
    const uint32_t span = (uint32_t)((uint64_t)(cnt - 1) * d.stride) + 16u * ns;  // < 2^31
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void *>(B0), (short)0, (int)span, 0x00020000);
    // edge segments (default cache policy; the stream reads them again later)
    const uint32_t te = ((rs + d.len - 1u) & 15u) + 1u;
    const uint32_t pkoff = (uint32_t)lane * (uint32_t)d.stride;  // lanes < cnt: < span
    u32x4 fseg = {0u, 0u, 0u, 0u}, lseg = {0u, 0u, 0u, 0u};
    if (lane < cnt && rs != 0u) fseg = load_edge_segment(rsrc, pkoff, edge_nt);
    if (lane < cnt && te != 16u) lseg = load_edge_segment(rsrc, pkoff + 16u * (ns - 1u), edge_nt);
// windows per group (A/B build switch; A2K 228.9-229.7 us at 6 and 228.9-229.6 at 8,
// profiles/r05/gcu)
#ifndef AIPSTACK_GAPCOL_WINDOWS
#define AIPSTACK_GAPCOL_WINDOWS 8
#endif
    constexpr int U = AIPSTACK_GAPCOL_WINDOWS;
    u32x4 va[U], vb[U];
    auto issue = [&](u32x4 (&v)[U], uint32_t w) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = min((w + (uint32_t)u) * (uint32_t)kWave + (uint32_t)lane, T - 1u);
            const uint32_t k = __umulhi(c, d.magic);
            const uint32_t off = (uint32_t)(__mul24((int)k, d.gap) + (int)(c << 4));
            v[u] = load_segment<NT>(rsrc, off, 0u);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    uint32_t C = 0;   // this lane's column sum
    uint32_t jb = 0;  // next boundary (uniform): compact segment jb * ns
    auto consume = [&](const u32x4 (&v)[U], uint32_t w) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t wu = w + (uint32_t)u;
            if (wu >= nwin) break;
            uint32_t s = halves(v[u][0], halves(v[u][1], halves(v[u][2], halves(v[u][3], 0u))));
            if (wu + 1u == nwin)  // lanes past the stream re-read its last segment
                s = wu * (uint32_t)kWave + (uint32_t)lane < T ? s : 0u;
            while (jb <= (uint32_t)cnt && ((jb * ns) >> 6) == wu) {
                rows[jb * kWave + (uint32_t)lane] =
                    C + ((uint32_t)lane < ((jb * ns) & 63u) ? s : 0u);
                ++jb;
            }
            C += s;
        }
    };
    const uint32_t groups = (nwin + U - 1u) / U;
    issue(va, 0);
    uint32_t gi = 0;
    for (; gi + 2u < groups; gi += 2u) {
        issue(vb, (gi + 1u) * U);
        consume(va, gi * U);
        issue(va, (gi + 2u) * U);
        consume(vb, (gi + 1u) * U);
    }
    if (gi + 2u == groups) {
        issue(vb, (gi + 1u) * U);
        consume(va, gi * U);
        consume(vb, (gi + 1u) * U);
    } else {
        consume(va, gi * U);
    }
    for (; jb <= (uint32_t)cnt; ++jb) rows[jb * kWave + (uint32_t)lane] = C;  // at T
    const uint32_t foreign = lane < cnt ? foreign_halves(fseg, lseg, (int)rs, (int)te) : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // packet j = lane >> ql: its 2^ql lanes add cpk column differences each
    const uint32_t ql = 6u - (uint32_t)__builtin_ctz(cpk);  // cpk: a power of two <= 16
    const uint32_t j = (uint32_t)lane >> ql, part = (uint32_t)lane & ((1u << ql) - 1u);
    uint32_t acc = 0;
    if (j < (uint32_t)cnt) {
        const uint32_t *r0 = rows + j * kWave + part * cpk;
        const uint32_t *r1 = r0 + kWave;
        if (cpk >= 4u) {
            for (uint32_t i = 0; i < cpk; i += 4u) {
                const u32x4 a = *reinterpret_cast<const u32x4 *>(r0 + i);
                const u32x4 b = *reinterpret_cast<const u32x4 *>(r1 + i);
                acc += (b[0] - a[0]) + (b[1] - a[1]) + (b[2] - a[2]) + (b[3] - a[3]);
            }
        } else {
            for (uint32_t i = 0; i < cpk; ++i) acc += r1[i] - r0[i];
        }
    }
    for (uint32_t m = 1; m < (1u << ql); m <<= 1)
        acc += (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((uint32_t)lane ^ m) << 2), (int)acc);
    __builtin_amdgcn_wave_barrier();
    const uint32_t col = (uint32_t)__builtin_amdgcn_ds_bpermute(
        (int)((((uint32_t)lane << ql) & 63u) << 2), (int)acc);
    __builtin_amdgcn_wave_barrier();  // (the table is rewritten by the next chunk)
    return lane < cnt ? col - foreign : 0u;
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

__device__ __forceinline__ uint32_t fold16(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return s;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x) {
    return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
}

}  // namespace
}  // namespace aipstack_amd

#endif
