// aipstack_amd -- CDNA4 (gfx950) batch Internet-checksum kernels + their C-ABI launchers.
//
// What is computed (reference semantics, src/aipstack/infra/Chksum.h):
//   IpChksumInverted(p, L)  (Chksum.h:77-99): ones'-complement sum of the big-endian
//   16-bit words of p[0..L), odd tail byte as a high byte, folded twice to 16 bits.
//   IpChksum = ~that (Chksum.h:122-125). IpChksumAccumulator(State s).getChksum(buf)
//   (Chksum.h:171-174, 263-315) = the same sum seeded with the 32-bit state s.
//
// How (MI355X-first; DESIGN.md sections 4-5):
//   * A wave owns a contiguous run of 64-packet chunks. Per chunk, lane j computes packet
//     j's load parameters (aligned base, segment count, head/tail mask indices) in VALU,
//     and lane j ends up holding packet j's result: ONE coalesced 128-byte store.
//   * Packets are processed one per wave, P at a time: packet [S, E) is read as the
//     16-byte-aligned segments A0 = S & ~15, A0+16, ... through a buffer descriptor of
//     16 * nseg bytes (lane k loads segment k; buffer_load_dwordx4 ... nt, 1 KiB per wave
//     instruction; the range check zeroes slots past the packet). The head segment's bytes
//     before S and the tail segment's bytes from E on are masked (constant tables, one
//     v_bitop3 per dword on the lane that holds them).
//   * Each lane accumulates its dwords in two add-with-carry chains (v_addc_co_u32, one op
//     per dword): a ones'-complement sum, congruent mod 0xFFFF to the sum of the 16-bit
//     halves and 0 only for all-zero input. Folded to 17 bits per chain, the 64 lanes are
//     added exactly (< 2^24) by a DPP row scan.
//   * Little-endian halves at even absolute addresses pair byte (2i, 2i+1) with 2i as the
//     LOW byte; the reference pairs relative to the packet start with p[0] as the HIGH
//     byte. So the folded sum is byte-swapped iff S is even. A byte swap is x*256 mod
//     0xFFFF and folding never turns a nonzero sum into 0, so the 0x0000-vs-0xFFFF
//     representation matches the reference exactly (0 iff every byte is 0).
//   * Stream mode (chksum_device.h): a chunk whose packets lie back to back (CSR with
//     non-decreasing offsets, stride == len) skips the per-packet work entirely. The wave
//     reads the chunk as one contiguous run, 1 KiB per instruction, keeps an exact prefix
//     of 16-bit-half sums (v_sad_u16 + DPP scan), and each packet's sum is the difference
//     of the prefixes at its two ends -- the same exact halves-sum as above.
//   * HBM-bound integer reduction: no MFMA, no LDS (the cross-lane sum is DPP).

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "aipstack_amd/chksum.h"
#include "chksum_internal.h"

#include "chksum_device.h"

namespace aipstack_amd {
namespace {

// ---------------------------------------------------------------------------------
// The kernel: wave w handles chunks [w*cpw, (w+1)*cpw) of `chunk_packets` (<= 64) packets
// each: 64 for large batches, fewer for small ones, so that a small batch still spreads
// over many waves (launch(): the small-batch regime).
// ---------------------------------------------------------------------------------
template <class Desc, int U, int P, bool NT, bool SEEDED, int SU>
__global__ __launch_bounds__(kBlock) void chksum_batch_kernel(Desc desc, uint64_t n,
                                                              uint32_t chunks_per_wave,
                                                              uint32_t chunk_packets,
                                                              uint16_t *__restrict__ out,
                                                              uint32_t flags) {
    const int lane = threadIdx.x & (kWave - 1);
    // threadIdx.x >> 6 is wave-uniform but the compiler cannot prove it: readfirstlane
    // keeps the whole packet walk (bounds, loop counters) in SGPRs.
    const uint32_t wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wave_in_block;
    const uint64_t cpk = chunk_packets;  // 1..64 (launch_k)
    const uint64_t nchunks = (n + cpk - 1) / cpk;
    uint64_t c = wave * chunks_per_wave;
    const uint64_t c_end = min(c + chunks_per_wave, nchunks);
    const bool final_flag = (flags & AIPSTACK_CHKSUM_FINAL) != 0;
    // the JUST_WRITTEN hint: the read forms' few loads outside their streams nontemporal too
    const bool edge_nt = (flags & AIPSTACK_CHKSUM_JUST_WRITTEN) != 0;
    const uint32_t voff = (uint32_t)lane * 16u;          // this lane's segment in a slot
    const uint32_t not_lane0 = lane == 0 ? 0u : ~0u;     // head-mask lane select
    // Ring slots with SU > 0: the chunk's 64 packets read as ONE gathered stream of just
    // their 16-byte segments (the chain kernel's loader, chksum_device.h), 1 KiB per wave
    // instruction however short the packets are, instead of one packet per wave instruction.
    // SU = 128 (slot windows, sum_slot_windows): each packet read on its own, no compaction
    constexpr bool kSlotWin = !Desc::kStream && SU == 128;
    // gapped column runs (sum_gapped_column_chunk): owners by arithmetic, no gathered stream
    constexpr bool kGapCols = std::is_same<Desc, GappedColDesc>::value;
    constexpr bool kGathered = !Desc::kStream && SU > 0 && !kSlotWin && !kGapCols;
    // 16-byte aligned by construction: the tables are read with ds_read_b128 (u32x4)
    alignas(16) __shared__ typename std::conditional<kSlotWin, SlotRows[kWavesPerBlock], char>::type slot_rows;
    struct GatheredShared {
        GatherLds g[kWavesPerBlock];
        // the byte-mask table, for edges masked in the stream only
        typename std::conditional<Desc::kEdge, char, KeepTable>::type keep;
    };
    __shared__ typename std::conditional<kGathered, GatheredShared, char>::type gsh;
    // column runs (sum_column_chunk): SU 64 = groups of 8 windows, 48 = groups of 6; 66 / 50
    // the same with the boundary segments captured from the stream (AIPSTACK_CHKSUM_JUST_WRITTEN)
    constexpr bool kColumns = Desc::kStream && (SU == 64 || SU == 48 || SU == 66 || SU == 50);
    constexpr bool kColCapture = SU == 66 || SU == 50;
    alignas(16) __shared__ typename std::conditional<kColumns || kGapCols, ColRows[kWavesPerBlock], char>::type
        col_rows;
    constexpr bool kSegTab = Desc::kStream && SU == 96;   // segment tables (sum_segtab_chunk)
    alignas(16) __shared__ typename std::conditional<kSegTab, SegTab[kWavesPerBlock], char>::type seg_tab;
    if constexpr (kGathered) {
        if constexpr (!Desc::kEdge) {  // edges masked in the stream: the mask table
            fill_keep_table(gsh.keep);
            __syncthreads();
        }
    }

    for (; c < c_end; ++c) {
        const uint64_t p0 = c * cpk;
        const int cnt = (int)min(cpk, n - p0);
        // the chunk's own table entries only (offsets, lengths, states): lanes past it re-read
        // entry p0 + cnt, so a wave of a short chunk fetches no other chunk's table lines
        const auto chunk = desc.begin_chunk(p0, p0 + (uint64_t)cnt, lane);
        // every packet's load parameters at once: lane j <-> packet j (VALU, vectorised)
        uint64_t lS, lE;
        desc.lane_bounds(chunk, lane, lS, lE);
        if (lane >= cnt) lE = lS;  // past the batch: empty
        if constexpr (Desc::kCsr)  // len > 65535 or E < S: outside the contract (chksum.h)
            note_violation(lE - lS > (uint64_t)AIPSTACK_CHKSUM_MAX_LEN,
                           AIPSTACK_CHKSUM_VIOLATION_PACKET_LEN);
        // lane j: exact halves-sum of packet j (0 iff all its bytes are 0)
        uint32_t sums = 0;
        bool streamed = false;
        if constexpr (kSlotWin) {
            sums = sum_slot_windows<NT>(lS, lE, lane, cnt, voff, slot_rows[wave_in_block]);
            streamed = true;
        } else if constexpr (kGapCols) {
            sums = sum_gapped_column_chunk<NT>(chunk.s0, lane, cnt, chunk_packets,
                                               col_rows[wave_in_block], desc, edge_nt);
            streamed = true;
        } else if constexpr (kGathered) {
            // (CSR: every packet within the contract, else the wave mode below)
            if (!Desc::kCsr || __builtin_amdgcn_ballot_w64(lE - lS > (uint64_t)AIPSTACK_CHKSUM_MAX_LEN) == 0) {
                if constexpr (Desc::kEdge)
                    sums = sum_gathered_chunks<SU, NT, true>(lS, (uint32_t)(lE - lS), lane,
                                                             &gsh.g[wave_in_block], nullptr,
                                                             edge_nt);
                else
                    sums = sum_gathered_chunks<SU, NT, false>(lS, (uint32_t)(lE - lS), lane,
                                                              &gsh.g[wave_in_block], &gsh.keep);
                streamed = true;
            }
        } else if constexpr (SU > 0) {
            if (stream_ok(lS, lE, lane, cnt) &&
                (!kSegTab ||
                 ((uint32_t)(readlane64(lE, cnt - 1) -
                             (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(lS >> 32)) << 32) |
                              ((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lS) & ~15u))) +
                  15u) >> 4 <= kSegTabMax)) {
                // back-to-back packets: the chunk read as one contiguous run
                if constexpr (kSegTab)
                    sums = sum_segtab_chunk<NT>(lS, lE, lane, cnt, voff, chunk_packets,
                                                seg_tab[wave_in_block]);
                else if constexpr (kColumns)
                    sums = sum_column_chunk<NT, (SU == 48 || SU == 50) ? 6 : 8, kColCapture>(
                        lS, lE, lane, cnt, voff,
                                                                   chunk_packets,
                                                                   col_rows[wave_in_block]);
                else
                    sums = sum_stream_chunk<SU, NT>(lS, lE, lane, cnt, voff);
                streamed = true;
            }
        }
        if (!streamed) {
            // one packet per wave, P in flight; empty packets are skipped
            const LaneMeta meta = lane_meta(lS, lE);
            NoMaskHook hook;
            sums = sum_lane_packets<U, P, Desc::kCsr ? AIPSTACK_ROWS_CSR : AIPSTACK_ROWS_STRIDED,
                                    NT>(meta, __builtin_amdgcn_ballot_w64((meta.packed >> 9) != 0),
                                        lane, voff, not_lane0, hook);
        }
        // Finalise the chunk's 64 results together (VALU, one packet per lane).
        uint32_t r = fold16(sums);
        if ((lS & 1u) == 0)  // S even
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
//
// A wave owns 64 chains and walks their chunks (contiguous in the table) 64 at a time,
// chunk <-> lane: coalesced loads of the chunk table; the chunk's chain from the chain
// starts marked in LDS and a max-scan; its logical-position parity from a ballot of odd
// lengths (prefix popcounts) plus the parity carried in from the previous 64 chunks; the
// 64 chunk sums from one gathered stream over just their bytes (sum_gathered_chunks,
// chksum_device.h); then each oriented chunk sum is added into its chain's 64-bit LDS
// accumulator, exact for any number of chunks per chain.
// ---------------------------------------------------------------------------------

// A 16-bit store at any byte address (one global_store_short: gfx9 runs in unaligned mode).
#ifndef AIPSTACK_CHAIN_FIELD_NT
#define AIPSTACK_CHAIN_FIELD_NT 1
#endif
typedef uint16_t u16_any_align __attribute__((aligned(1)));

// Second pass of the chain fill: chain i's checksum (from the chained batch's output) stored
// big-endian into its header field, one chain per thread, after every chain has been read
// (no field store can race a read of the same chain). CHAIN bench shape, 1 M chains: 13.5 us
// here, but the chain kernel of the next launch then runs ~37 us longer (the partially
// written lines go back to HBM under its stream): 299 us per fill against 298 with the
// stores inside the chain kernel and 248 for the chained batch alone.
__global__ __launch_bounds__(kBlock) void chain_field_scatter_kernel(
    const uint64_t *__restrict__ fields, const uint16_t *__restrict__ sums, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const uint64_t fa = fields[i];
#if AIPSTACK_CHAIN_FIELD_NT  // nontemporal field stores (round 6): the header lines they write
                             // carry no first-read cost into the next batch: chain
                             // fill 265.6-265.8 us against 307.1-308.3 (profiles/r06/hint6)
        if (fa) __builtin_nontemporal_store((uint16_t)bswap16(sums[i]), reinterpret_cast<u16_any_align *>(fa));
#else
        if (fa) *reinterpret_cast<u16_any_align *>(fa) = (uint16_t)bswap16(sums[i]);
#endif
    }
}

__device__ __forceinline__ uint32_t parity_below(uint64_t mask, uint32_t s) {  // s in 0..64
    const uint64_t below = s == 0 ? 0ull : (~0ull >> (64u - s));
    return (uint32_t)__builtin_popcountll(mask & below) & 1u;
}

// SU = 4 (the default since round 4) holds four more segment quads per lane than SU = 2 and
// gets 4 waves per SIMD (at 5 it spilled 68 bytes per lane at 96 VGPRs); SU = 2 keeps 5.
// Chain runs (round 6; A/B build switch AIPSTACK_CHAIN_RUNS): long chunks that lie back to
// back read as one stream-prefix run, short ones by their own lanes. Bit-exact (the chain
// tests), but slower on CHAIN: 261.0-261.5 us against 251.8-254.5 for the gathered stream
// (profiles/r06/chain6): a 31 KiB run with 43 boundaries per group costs the stream prefixes'
// per-window scan and boundary evaluation more than the gathered stream's owner lookup. Off.
#ifndef AIPSTACK_CHAIN_RUNS
#define AIPSTACK_CHAIN_RUNS 0
#endif
constexpr bool kChainRuns = AIPSTACK_CHAIN_RUNS != 0;
// Chain column runs (round 6; COLS): as chain runs, but the run chunks -- every non-empty
// chunk that is not a lone short one (the short_first rule: header nodes apart from the
// payload), in table order -- are read as column runs of at most kChainColMax chunks each
// (sum_column_chunk, capture form: no per-window scan, no owner lookup, no line read through
// the L2-allocating path), and the lone short ones each by its own lane (their first two
// segments loaded before the runs). Any other layout: the gathered stream below. The kernel
// for AIPSTACK_CHKSUM_JUST_WRITTEN (launch_chain): on plain-written CHAIN 323.5 against the
// gathered stream's 367.3 us; on bytes read before, 279-283 against 253-255 (more per-boundary
// work at 45 segments per boundary, 4 waves per SIMD against 5), so not the default
// (profiles/r06/ccols/). AIPSTACK_CHAIN_COLS=1: every launch (A/B build switch).
#ifndef AIPSTACK_CHAIN_COLS
#define AIPSTACK_CHAIN_COLS 0
#endif
constexpr bool kChainCols = AIPSTACK_CHAIN_COLS != 0;
#ifndef AIPSTACK_CHAIN_COLS_MAXP
#define AIPSTACK_CHAIN_COLS_MAXP 32
#endif
constexpr int kChainColMax = AIPSTACK_CHAIN_COLS_MAXP;  // run chunks per column run (16 or 32)
#ifndef AIPSTACK_CHAIN_COLS_U
#define AIPSTACK_CHAIN_COLS_U 6
#endif
constexpr int kChainColU = AIPSTACK_CHAIN_COLS_U;  // windows per group in those runs
template <bool NT, int SU, bool COLS = false>
__global__ __launch_bounds__(kBlock, SU > 2 ? 4 : 5) void chksum_chain_kernel(
    const uint64_t *__restrict__ chunk_addr, const uint32_t *__restrict__ chunk_len,
    const uint64_t *__restrict__ index, const uint32_t *__restrict__ states, uint64_t n,
    uint32_t chunks_per_wave, uint32_t chains_per_group, uint16_t *__restrict__ out,
    uint32_t flags, uint32_t short_first) {
    __shared__ uint64_t lds_acc[kWavesPerBlock][kWave];  // per-chain sum of chunk sums
    __shared__ int lds_mark[kWavesPerBlock][kWave];      // chain starting at chunk lane
    constexpr bool kCols = (COLS || kChainCols) && SU > 2;
    // gathered stream owners (chain column runs: in the wave's column rows, which a slice that
    // takes the gathered stream does not use)
    __shared__ typename std::conditional<kCols, char, GatherLds[kWavesPerBlock]>::type lds_gather;
    alignas(16) __shared__
        typename std::conditional<kCols, ColRowsN<kChainColMax>[kWavesPerBlock], char>::type col_rows;
    const int lane = threadIdx.x & (kWave - 1);
    const uint32_t wave_in_block = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t wave = (uint64_t)blockIdx.x * kWavesPerBlock + wave_in_block;
    const uint64_t cpg = chains_per_group;  // 1..64: fewer for small batches (pick_shape)
    const uint64_t ngroups = (n + cpg - 1) / cpg;
    uint64_t c = wave * chunks_per_wave;
    const uint64_t c_end = min(c + chunks_per_wave, ngroups);
    const bool final_flag = (flags & AIPSTACK_CHKSUM_FINAL) != 0;
    const bool edge_nt = (flags & AIPSTACK_CHKSUM_JUST_WRITTEN) != 0;  // 
    uint64_t *acc = lds_acc[wave_in_block];
    int *mark = lds_mark[wave_in_block];
    const uint32_t voff = (uint32_t)lane * 16u;  // (chain runs: this lane's segment in a window)
    auto gather_lds = [&]() -> GatherLds * {
        if constexpr (kCols)
            return reinterpret_cast<GatherLds *>(col_rows[wave_in_block]);
        else
            return &lds_gather[wave_in_block];
    };
    CsrDesc idx_desc{0, index};  // the chain index walks like CSR offsets

    for (; c < c_end; ++c) {
        const uint64_t p0 = c * cpg;
        const int cnt = (int)min(cpg, n - p0);
        // only the group's cnt + 1 index entries and cnt states: lanes past them re-read
        // entry p0 + cnt (one line), so no wave fetches the next groups' table lines
        const auto grp = idx_desc.begin_chunk(p0, p0 + (uint64_t)cnt, lane);
        const uint32_t state = (states != nullptr && lane < cnt) ? states[p0 + lane] : 0u;
        // chain `lane` = chunks [cs, ce) (relative to the group's first chunk K0)
        uint64_t cs64, ce64;
        idx_desc.lane_bounds(grp, lane, cs64, ce64);
        const uint64_t K0 = idx_desc.offset_of(grp, 0);
        // the group's chunks end where chain p0 + cnt starts (lane cnt's index entry)
        const uint64_t K1 =
            cnt < kWave ? idx_desc.offset_of(grp, cnt)
                        : ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(grp.end_off >> 32))
                           << 32) | __builtin_amdgcn_readfirstlane((uint32_t)grp.end_off);
        const bool chain_nonempty = lane < cnt && ce64 > cs64;
        const uint32_t cs = (uint32_t)(cs64 - K0);  // < 2^32 chunks per group (contract)
        acc[lane] = 0;
        int carry_cid = -1;      // chain of the last chunk of the previous 64
        uint32_t carry_par = 0;  // its logical position parity after that chunk
        for (uint64_t kb = K0; kb < K1; kb += kWave) {
            const uint32_t kr = (uint32_t)(kb - K0);
            const uint64_t k = kb + (uint64_t)lane;
            const bool valid = k < K1;
            uint64_t a = 0;
            uint32_t l = 0;
            if (valid) {
                a = chunk_addr[k];
                l = chunk_len[k];
            }
            // a chunk over 65535 bytes (outside the contract) is summed as empty: the
            // gathered stream's compact indices (24 bits) then cannot overflow, so no load
            // leaves the chunks
            note_violation(l > AIPSTACK_CHKSUM_MAX_LEN, AIPSTACK_CHKSUM_VIOLATION_CHUNK_LEN);
            if (l > AIPSTACK_CHKSUM_MAX_LEN) l = 0;
            // which chain: the last chain starting at or before this chunk
            mark[lane] = -1;
            __builtin_amdgcn_wave_barrier();
            if (chain_nonempty && cs >= kr && cs - kr < (uint32_t)kWave)
                mark[cs - kr] = lane;
            __builtin_amdgcn_wave_barrier();
            int cid = wave_max_scan(mark[lane]);
            if (cid < 0) cid = carry_cid;  // continues a chain from the previous 64
            __builtin_amdgcn_wave_barrier();
            // logical position parity: odd lengths before this chunk within its chain
            const uint64_t odd = __builtin_amdgcn_ballot_w64(valid && (l & 1u));
            const uint32_t scs = (uint32_t)__builtin_amdgcn_ds_bpermute(max(cid, 0) << 2, (int)cs);
            const bool before = scs < kr;  // the chain began in an earlier 64
            const uint32_t s = before ? 0u : scs - kr;
            uint32_t q = parity_below(odd, (uint32_t)lane) ^ parity_below(odd, s);
            if (before) q ^= carry_par;
            // the 64 chunk sums: one gathered stream over just the chunks' bytes. With
            // short_first (tunable "chain_short", default 128 since round 4; 0 = the table's
            // order), chunks of at most that many bytes that share no line with their
            // neighbours in the table go first in the stream, so that header nodes lying side
            // by side are read together as whole lines rather than one 32-byte piece between
            // two payloads' windows each (the nontemporal stream keeps no line cached until
            // the next header's turn). Any order gives the same sums: each chunk's sum
            // returns to its lane through the inverse permutation. CHAIN: FETCH_SIZE -1.3 %,
            // 241.0-241.7 vs 241.9-242.9 us (profiles/r04/short, probe).
            uint32_t sums = 0;
            const uint32_t lv = valid ? l : 0u;
            bool done = false;
            if constexpr (kChainRuns && SU > 2) {  // (SU 2, 5 waves per SIMD: would spill)
                // Chain runs (round 6): when the group's long chunks, in table order, lie back
                // to back -- the payload pieces of consecutive segments cut from one send
                // buffer, tcp/IpTcpProto_output.h:1251-1277 -- they are read as ONE run with
                // stream prefixes (sum_stream_chunk, C's loader: no owner lookup, no 64-bit
                // address per window) in lanes 0..nl-1, and the short ones (header nodes, at
                // most short_first bytes) each by its own lane. Any other layout: the gathered
                // stream below. Each chunk's sum returns to its lane through the inverse
                // permutation, as there.
                const bool shortc = short_first != 0u && lv != 0u && lv <= short_first;
                const uint64_t lm = __builtin_amdgcn_ballot_w64(lv != 0u && !shortc);
                const uint32_t nl = (uint32_t)__builtin_popcountll(lm);
                const uint32_t below_l = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
                const bool longc = ((lm >> lane) & 1ull) != 0;
                const uint32_t rank = longc ? below_l : nl + (uint32_t)lane - below_l;
                const int to = (int)(rank << 2);
                const uint32_t a_lo = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)a);
                const uint32_t a_hi = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)(a >> 32));
                const uint32_t l_p = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)lv);
                const uint64_t a_p = ((uint64_t)a_hi << 32) | a_lo;
                if (nl != 0u && stream_ok(a_p, a_p + l_p, lane, (int)nl)) {
                    const uint32_t s_long = sum_stream_chunk<16, NT>(a_p, a_p + l_p, lane,
                                                                     (int)nl, voff);
                    // the short ones: lanes nl.. hold them (and the empty chunks, l_p = 0)
                    const uint32_t nsg = ((uint32_t)lane >= nl && l_p)
                                             ? (((uint32_t)a_p & 15u) + l_p + 15u) >> 4 : 0u;
                    const uint32_t kmax = (uint32_t)__builtin_amdgcn_readlane(
                        wave_max_scan((int)nsg), kWave - 1);
                    const uint32_t s_short = sum_own_short_chunk(a_p, (uint32_t)lane >= nl ? l_p : 0u,
                                                                 kmax);
                    const uint32_t s_p = (uint32_t)lane < nl ? s_long : s_short;
                    sums = (uint32_t)__builtin_amdgcn_ds_bpermute(to, (int)s_p);
                    done = true;
                }
            }
            if constexpr (kCols) {
                if (short_first != 0u) {
                    // lone short chunks (the short_first rule below), run chunks, empty ones
                    const uint32_t line_s = (uint32_t)(a >> 7);
                    const uint32_t line_e = (uint32_t)((a + lv - 1u) >> 7);
                    const uint32_t prev_e =
                        (uint32_t)__builtin_amdgcn_ds_bpermute((lane - 1) << 2, (int)line_e);
                    const uint32_t next_s =
                        (uint32_t)__builtin_amdgcn_ds_bpermute((lane + 1) << 2, (int)line_s);
                    const bool sc = lv != 0 && lv <= short_first && prev_e != line_s &&
                                    next_s != line_e;
                    const bool rc = lv != 0 && !sc;
                    const uint64_t rm = __builtin_amdgcn_ballot_w64(rc);
                    const uint64_t sm = __builtin_amdgcn_ballot_w64(sc);
                    const uint32_t nr = (uint32_t)__builtin_popcountll(rm);
                    const uint32_t ns_ = (uint32_t)__builtin_popcountll(sm);
                    const uint32_t below_r = __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u));
                    const uint32_t below_s = __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                    // run chunks in lanes 0..nr-1 (table order), then the short ones, then
                    // the empty ones
                    const uint32_t rank = rc ? below_r
                                          : sc ? nr + below_s
                                               : nr + ns_ + (uint32_t)lane - below_r - below_s;
                    const int to = (int)(rank << 2);
                    const uint32_t a_lo = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)a);
                    const uint32_t a_hi = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)(a >> 32));
                    const uint32_t l_p = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)lv);
                    const uint64_t a_p = ((uint64_t)a_hi << 32) | a_lo;
                    if (stream_ok(a_p, a_p + l_p, lane, (int)nr)) {  // back to back
                        // the short ones' first two segments go out ahead of the runs
                        typedef __attribute__((address_space(1))) const u32x4 gseg;
                        const bool mine = (uint32_t)lane >= nr && (uint32_t)lane < nr + ns_;
                        const uint32_t nsg = mine ? (((uint32_t)a_p & 15u) + l_p + 15u) >> 4 : 0u;
                        const gseg *hp = (const gseg *)(a_p & ~(uint64_t)15);
                        u32x4 h0 = {0u, 0u, 0u, 0u}, h1 = {0u, 0u, 0u, 0u};
                        if (nsg > 0u) h0 = __builtin_nontemporal_load(hp);
                        if (nsg > 1u) h1 = __builtin_nontemporal_load(hp + 1);
                        uint32_t s_p = 0;
                        // (cpk as a run-time value: the column differences' loop stays rolled)
                        const uint32_t cpk = (uint32_t)kChainColMax | (flags & 0x80000000u);
                        for (uint32_t r0 = 0; r0 < nr; r0 += (uint32_t)kChainColMax) {
                            const int cnt_r = (int)min(nr - r0, (uint32_t)kChainColMax);
                            const int src = (int)((((uint32_t)lane + r0) & 63u) << 2);
                            const uint64_t S = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)a_hi) << 32) |
                                               (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)a_lo);
                            const uint64_t E = S + (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)l_p);
                            uint32_t sr;
                            if (COLS || edge_nt)  // (the COLS kernel runs for the hint alone)
                                sr = sum_column_chunk<NT, kChainColU, true, kChainColMax>(
                                    S, E, lane, cnt_r, voff, cpk, col_rows[wave_in_block]);
                            else
                                sr = sum_column_chunk<NT, kChainColU, false, kChainColMax>(
                                    S, E, lane, cnt_r, voff, cpk, col_rows[wave_in_block]);
                            const uint32_t back = (uint32_t)__builtin_amdgcn_ds_bpermute(
                                (int)((((uint32_t)lane - r0) & 63u) << 2), (int)sr);
                            if ((uint32_t)lane >= r0 && (uint32_t)lane < r0 + (uint32_t)cnt_r)
                                s_p = back;
                        }
                        const uint32_t kmax = (uint32_t)__builtin_amdgcn_readlane(
                            wave_max_scan((int)nsg), kWave - 1);
                        if (mine) s_p = sum_short_chunk_from(h0, h1, a_p, l_p, kmax);
                        sums = (uint32_t)__builtin_amdgcn_ds_bpermute(to, (int)s_p);
                        done = true;
                    }
                }
            }
            if (done) {
            } else if (short_first) {
                // a short chunk goes first only if it shares no line with its neighbours in
                // the table (a header node apart from the payload; a short payload piece
                // stays beside the pieces it shares lines with)
                const uint32_t line_s = (uint32_t)(a >> 7);
                const uint32_t line_e = (uint32_t)((a + lv - 1u) >> 7);
                const uint32_t prev_e =
                    (uint32_t)__builtin_amdgcn_ds_bpermute((lane - 1) << 2, (int)line_e);
                const uint32_t next_s =
                    (uint32_t)__builtin_amdgcn_ds_bpermute((lane + 1) << 2, (int)line_s);
                const bool sc = lv != 0 && lv <= short_first && prev_e != line_s &&
                                next_s != line_e;
                const uint64_t sm = __builtin_amdgcn_ballot_w64(sc);
                const uint32_t below_s = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                const uint32_t rank = sc ? below_s
                                         : (uint32_t)__builtin_popcountll(sm) + (uint32_t)lane - below_s;
                const int to = (int)(rank << 2);
                const uint32_t a_lo = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)a);
                const uint32_t a_hi = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)(a >> 32));
                const uint32_t l_p = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)lv);
                const uint32_t s_p = sum_gathered_chunks<SU, NT>(
                    ((uint64_t)a_hi << 32) | a_lo, l_p, lane, gather_lds(), nullptr,
                    edge_nt);
                sums = (uint32_t)__builtin_amdgcn_ds_bpermute(to, (int)s_p);
            } else {
                sums = sum_gathered_chunks<SU, NT>(a, lv, lane, gather_lds(),
                                                   nullptr, edge_nt);
            }
            uint32_t r = fold16(sums);
            if ((uint32_t)(a & 1) == q)
                r = bswap16(r);
            if (valid && r != 0)
                __hip_atomic_fetch_add(&acc[cid], (uint64_t)r, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            // carry to the next 64 chunks
            const int last = (int)min((uint64_t)(kWave - 1), K1 - kb - 1);
            carry_cid = __builtin_amdgcn_readlane(cid, last);
            carry_par = __builtin_amdgcn_readlane(q ^ (l & 1u), last);
        }
        __builtin_amdgcn_wave_barrier();
        const uint64_t sum = acc[lane];  // <= chunks * 0xFFFF: exact for any chunk count
        __builtin_amdgcn_wave_barrier();
        // fold to 16 bits keeping the residue mod 0xFFFF and zero-ness (2^32 = 1)
        uint64_t s33 = (sum & 0xFFFFFFFFull) + (sum >> 32);
        const uint32_t s32 = (uint32_t)s33 + (uint32_t)(s33 >> 32);
        // m_sum = state (+) chain sum with end-around carry; getChksum folds and inverts.
        const uint64_t t = (uint64_t)state + fold16(s32);
        uint32_t r = fold16((uint32_t)t + (uint32_t)(t >> 32));
        r = final_flag ? (~r & 0xFFFFu) : r;
        if ((flags & AIPSTACK_CHKSUM_ZERO_AS_FFFF) && r == 0)  // udp/IpUdpProto.h:176-178
            r = 0xFFFFu;
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
    std::atomic<int> frames{0};           // frames in flight per wave (frame kernels)
    std::atomic<int> nontemporal{1};      // 1 = nontemporal (streaming) loads: every byte is
                                          // read once; measured faster on configs A and B
    std::atomic<int> stream{0};           // stream mode for back-to-back chunks: windows
                                          // issued together (2, 4, 8); -1 = off
    std::atomic<int> chunk_packets{0};    // packets per chunk (1, 2, 4, ..., 64); 0 = by
                                          // batch size (pick_shape)
    std::atomic<int> tx_gather{-1};       // Tx header segments: 0 per-lane loads, 1 captured
                                          // from the stream, 2 captured + field lines
                                          // touched up front; else by kind of Tx launch
    std::atomic<int> tx_store{-1};        // in-place Tx fills: 0 = 2-byte field stores, 1 =
                                          // whole sectors; else the default
    std::atomic<int> gather{1};           // back-to-back batches: -1 stream mode with 64-packet
                                          // chunks (rounds 1-3), 0 the gathered stream (round
                                          // 4), 1 (or 2) short runs (round 5, launch_short_runs)
    std::atomic<int> short_loads{-1};     // short runs: 0 stream prefixes (buffer loads), 1 the
                                          // same through global loads, 2 column runs; -1 by
                                          // packet length (launch_short_runs)
    std::atomic<int> slot_windows{0};     // ring slots / gaps: 1 = slot windows (SU 128)
    std::atomic<int> lds_pad{0};          // bytes of dynamic LDS per batch block (occupancy;
                                          // 0 = the launch's own, -1 = none)
    std::atomic<int> chain_short{-1};      // chains: chunks of at most this many bytes first in
                                          // the gathered stream (0 = table order; measured:
                                          // CHAIN 250.0-250.6 us at 128 against 248.0-248.9,
                                          // FETCH_SIZE -0.5 %, profiles/r04/kern)
    // host engine (read when an engine is created, chksum_engine.cpp):
    std::atomic<int> engine_zero_copy{1};         // kernels read registered input in place
    std::atomic<int> engine_zero_copy_small{65536};  // pieces of at most this many packets
                                                     // keep offsets / results in pinned staging
    std::atomic<int> engine_pageable_rows{1};  // pageable ring slots: frame bytes staged
                                               // and read in place (0: whole slots DMA'd)

    Tuning() {
        auto env = [](const char *k, std::atomic<int> &v) {
            if (const char *s = std::getenv(k)) v = std::atoi(s);
        };
        env("AIPSTACK_CHKSUM_WAVES_PER_CU", waves_per_cu);
        env("AIPSTACK_CHKSUM_CHUNKS_PER_WAVE", chunks_per_wave);
        env("AIPSTACK_CHKSUM_UNROLL", unroll);
        env("AIPSTACK_CHKSUM_PACKETS", packets);
        env("AIPSTACK_CHKSUM_NT", nontemporal);
        env("AIPSTACK_CHKSUM_FRAMES", frames);
        env("AIPSTACK_CHKSUM_STREAM", stream);
        env("AIPSTACK_CHKSUM_CHUNK_PACKETS", chunk_packets);
        env("AIPSTACK_CHKSUM_TX_GATHER", tx_gather);
        env("AIPSTACK_CHKSUM_TX_STORE", tx_store);
        env("AIPSTACK_CHKSUM_CHAIN_SHORT", chain_short);
        env("AIPSTACK_CHKSUM_GATHER", gather);
        env("AIPSTACK_CHKSUM_SHORT_LOADS", short_loads);
        env("AIPSTACK_CHKSUM_LDS_PAD", lds_pad);
        env("AIPSTACK_CHKSUM_SLOT_WINDOWS", slot_windows);
        env("AIPSTACK_ENGINE_ZERO_COPY", engine_zero_copy);
        env("AIPSTACK_ENGINE_ZERO_COPY_SMALL", engine_zero_copy_small);
        env("AIPSTACK_ENGINE_PAGEABLE_ROWS", engine_pageable_rows);

    }
};

Tuning &tuning() {
    static Tuning t;
    return t;
}

constexpr int kDefaultWavesPerCu = 64;
constexpr int kShortRunLds = 0;  // dynamic LDS per short-run block (none: 5 waves per SIMD)

// The product build compiles the launch shapes the pick_* functions choose, plus the runtime
// forms the tests exercise (stream windows 2 / 4 / 8 / off, the gathered stream's window
// counts, chunk sizes): about 60 batch kernels. tools/build_variant.sh NAME -DAIPSTACK_ALL_VARIANTS
// builds every U x P x NT combination as well (the "unroll", "packets" and "nontemporal"
// tunables of tools/sweep.py; round 4's product build held all of them, 565 kernels).
#ifdef AIPSTACK_ALL_VARIANTS
constexpr bool kAllVariants = true;
#else
constexpr bool kAllVariants = false;
#endif

// U: enough segments per lane to cover a typical packet in one group.
int pick_unroll(uint32_t max_len) {
    const int t = tuning().unroll.load(std::memory_order_relaxed);
    if (kAllVariants && t >= 1 && t <= 4) return t;
    const uint32_t max_seg = (max_len + 30u) / 16u;           // worst-case alignment
    const uint32_t q = (max_seg + kWave - 1) / kWave;         // groups of 64 segments
    if (q <= 1) return 1;
    if (q == 2) return 2;
    if (q % 3 == 0 || q == 3) return 3;
    return 4;
}

// P: packets whose loads a wave keeps in flight. Measured (tools/sweep.py, MI355X,
// profiles/r01/sweep_*.jsonl): 1500 B strided best at P = 8, 9000 B at P = 1 (U = 3
// already has 3 KiB in flight per wave), mixed 64-1500 B CSR at P = 4.
[[maybe_unused]] int pick_packets(int u, bool csr) {
    const int t = tuning().packets.load(std::memory_order_relaxed);
    if (t == 1 || t == 2 || t == 4 || t == 8) return t;
    if (csr) return 4;
    return u <= 2 ? 8 : 1;
}

// SU: stream-mode windows issued together (0 = stream mode off). Measured (tools/sweep.py,
// profiles/r01e): 1500/9000 B strided best at 2 (a wave streams 94-141 KiB per chunk, and
// occupancy covers the latency), mixed CSR at 8 (stream 2 / 4 / 8 / off: 262 / 258 / 255 /
// 266 us on config C).
int pick_stream(bool csr) { return tuning_stream_windows(csr ? 8 : 2); }

// Small batches. A 64-packet chunk per wave leaves a small batch on a few waves, each
// streaming ~100 KB with 2 windows (2 KiB) in flight: latency-bound (a 64-packet batch
// took 23 us, a 4096-packet one 33 us). Below kSmallWavesPerCu waves per CU at 64 packets
// per chunk, chunks shrink (packets per chunk = the power of two that gives about
// kSmallTargetPerCu waves per CU, at least 1) and every wave keeps 8 windows in flight.
// Chosen from a sweep of 8 K..512 K packets / frames per batch (profiles/r02/small_batches/
// shape_sweep.jsonl): config A in batches of 32 K 9.9 us at 16 packets per chunk (11.7 at
// 32, 34.5 at 64 with 2 windows), 128 K 32.0 us at 64 packets with 8 windows (41.5 with 2);
// from 256 K on the large-batch shape is as fast.
constexpr uint64_t kSmallWavesPerCu = 16;
constexpr uint64_t kSmallTargetPerCu = 8;

struct Shape {
    uint32_t chunk_packets;  // packets per chunk (64: the large-batch shape)
    bool small;
};

Shape pick_shape(uint64_t n, int cus) {
    const int t = tuning().chunk_packets.load(std::memory_order_relaxed);
    if (t >= 1 && t <= kWave && (t & (t - 1)) == 0) return Shape{(uint32_t)t, t < kWave};
    const uint64_t chunks64 = (n + kWave - 1) / kWave;
    if (chunks64 >= (uint64_t)cus * kSmallWavesPerCu) return Shape{(uint32_t)kWave, false};
    const uint64_t per = (n + (uint64_t)cus * kSmallTargetPerCu - 1) / ((uint64_t)cus * kSmallTargetPerCu);
    uint32_t cpk = 1;
    while (cpk < per && cpk < (uint32_t)kWave) cpk <<= 1;
    return Shape{cpk, true};
}

// SU for a launch: the tuned value, else 8 windows in the small-batch regime, else the
// family default.
int pick_stream_for(bool csr, const Shape &sh) {
    const int t = tuning().stream.load(std::memory_order_relaxed);
    if (t < 0 || t == 2 || t == 4 || t == 8) return tuning_stream_windows(0);
    return sh.small ? 8 : pick_stream(csr);
}

template <class Desc, int U, int P, bool NT, bool SEEDED, int SU>
int launch_k(const Desc &desc, uint64_t n, const Shape &sh, uint16_t *d_out, uint32_t flags,
             hipStream_t stream, bool one_per_wave = false, int dyn_lds = 0) {
    const uint64_t nchunks = (n + sh.chunk_packets - 1) / sh.chunk_packets;
    const int cus = device_cu_count(stream);
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    uint64_t cpw = (uint64_t)tuning().chunks_per_wave.load(std::memory_order_relaxed);
    if (cpw == 0 && (one_per_wave || !Desc::kStream) &&
        tuning().waves_per_cu.load(std::memory_order_relaxed) == 0)
        cpw = 1;  // short chunks: one per wave, the waves scheduled as CUs free up
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
    // (tunable lds_pad: dynamic LDS per block, so that fewer blocks fit a CU -- occupancy
    // experiments only; 0 by default)
    hipLaunchKernelGGL((chksum_batch_kernel<Desc, U, P, NT, SEEDED, SU>), dim3((unsigned)blocks),
                       dim3(kBlock), tuning_lds_pad(dyn_lds), stream, desc, n, (uint32_t)cpw,
                       sh.chunk_packets, d_out, flags);
    return check_hip(hipGetLastError());
}

template <class Desc, int U, int P, bool SEEDED>
int launch_s(const Desc &desc, uint64_t n, const Shape &sh, uint16_t *d_out, uint32_t flags,
             hipStream_t stream) {
    if constexpr (!Desc::kStream) {  // ring slots, per-packet wave mode (launch: gathered)
        return launch_k<Desc, U, P, true, SEEDED, 0>(desc, n, sh, d_out, flags, stream);
    } else if constexpr (!kAllVariants && std::is_same<Desc, StridedDesc>::value &&
                         (U != 1 || P != 1)) {
        // fixed-length packets back to back: stream mode runs at U = P = 1 (launch), so the
        // U / P forms are the per-packet wave mode only (tunable stream = -1)
        return launch_k<Desc, U, P, true, SEEDED, 0>(desc, n, sh, d_out, flags, stream);
    } else {
        if constexpr (kAllVariants) {
            if (tuning().nontemporal.load(std::memory_order_relaxed) == 0)  // sweeps only
                return launch_k<Desc, U, P, false, SEEDED, 0>(desc, n, sh, d_out, flags, stream);
        }
        switch (pick_stream_for(Desc::kCsr, sh)) {
            case 0: return launch_k<Desc, U, P, true, SEEDED, 0>(desc, n, sh, d_out, flags, stream);
            case 2: return launch_k<Desc, U, P, true, SEEDED, 2>(desc, n, sh, d_out, flags, stream);
            case 8: return launch_k<Desc, U, P, true, SEEDED, 8>(desc, n, sh, d_out, flags, stream);
            default: return launch_k<Desc, U, P, true, SEEDED, 4>(desc, n, sh, d_out, flags, stream);
        }
    }
}

template <class Desc, int U, bool SEEDED>
int launch_u(const Desc &desc, uint64_t n, const Shape &sh, uint16_t *d_out, uint32_t flags,
             hipStream_t stream) {
    if constexpr (!kAllVariants) {
        // P for this U: pick_packets' measured choice, except P = 4 for U <= 2 where it took 8
        // (the per-packet wave mode is a fallback since round 4 -- tunable stream = -1 -- and
        // at P = 8 it spilled 62-65 SGPRs)
        return launch_s<Desc, U, (Desc::kCsr || U <= 2) ? 4 : 1, SEEDED>(desc, n, sh, d_out,
                                                                        flags, stream);
    } else {
        int p = pick_packets(U, Desc::kCsr);
        if (Desc::kStream && desc.back_to_back() && pick_stream_for(Desc::kCsr, sh) > 0 &&
            tuning().nontemporal.load(std::memory_order_relaxed) != 0 &&
            tuning().packets.load(std::memory_order_relaxed) == 0)
            p = 1;
        switch (p) {
            case 1: return launch_s<Desc, U, 1, SEEDED>(desc, n, sh, d_out, flags, stream);
            case 2: return launch_s<Desc, U, 2, SEEDED>(desc, n, sh, d_out, flags, stream);
            case 4: return launch_s<Desc, U, 4, SEEDED>(desc, n, sh, d_out, flags, stream);
            case 8: return launch_s<Desc, U, 8, SEEDED>(desc, n, sh, d_out, flags, stream);
        }
        return AIPSTACK_CHKSUM_EINVAL;
    }
}

template <class Desc, bool SEEDED>
int launch(const Desc &desc, uint64_t n, uint32_t max_len, uint16_t *d_out, uint32_t flags,
           hipStream_t stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    const int cus = device_cu_count(stream);
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    Shape sh = pick_shape(n, cus);
    if constexpr (!Desc::kStream) {
        // Ring slots: the gathered stream, 4 windows per group, 8-packet chunks, one chunk
        // per wave ("stream" tunable: 2 = 2 windows, -1 = the per-packet wave mode). C2K
        // (profiles/r03/ssweep): 263 us against 278 with 64-packet chunks and runs of chunks
        // per wave, and 265 for the wave mode in the same shape; round 4, once the stream
        // summed whole segments (fewer VGPRs): 8-packet chunks 244.2 us, 16 248.8, 4 291.9
        // (A2K 224.2 / 225.8 / 221.9; profiles/r04/shape2).
        // CSR packets in the gathered stream (config C, 64-1500 B): 16-packet chunks 231.0 us,
        // 8 242.3, 32 233.6 (profiles/r04/chunks) -- about 12 KiB per chunk, as A's 8 x 1500 B.
        // Round 5, the driver's protocol (--steps 20 --warmup 5, profiles/r05/shape5): ring
        // slots of mixed lengths (C2K) run 254.8-256.6 us in 16-packet chunks against
        // 281.9-284.2 in 8 (32: 262), the per-chunk setup spread over twice the bytes; fixed
        // 1500-B packets at a stride (A2K) 231.6-233.1 against 231.5-232.1, so they keep 8.
        if (!sh.small && tuning().chunk_packets.load(std::memory_order_relaxed) == 0)
            sh.chunk_packets =
                (Desc::kCsr || std::is_base_of<SlottedDesc, Desc>::value) ? 16 : 8;
        // 4 windows per group. Round 4 took 8 for fixed-length packets of 1 KiB or more (A
        // 213.4 against 217.1 us at 4, steady state; C and C2K lost at 8: 233.3 / 267.1 against
        // 229.9 / 243.4; profiles/r04/su8); under the driver's protocol A2K runs 230.4-230.8
        // at 4 against 232.1-232.9 at 8 (profiles/r05/shape6), so 4 everywhere.
        const int su = tuning_stream_windows(4);
        // slot windows (SU 128, sum_slot_windows): tunable slot_windows = 1 (device-memory
        // slots and gaps; the host-memory form keeps the masked gathered stream)
        if constexpr (Desc::kEdge) {
            if (su != 0 && tuning().slot_windows.load(std::memory_order_relaxed) == 1)
                return launch_k<Desc, 1, 1, true, SEEDED, 128>(desc, n, sh, d_out, flags, stream);
        }
        if (su == 4) return launch_k<Desc, 1, 1, true, SEEDED, 4>(desc, n, sh, d_out, flags, stream);
        if (su == 8) return launch_k<Desc, 1, 1, true, SEEDED, 8>(desc, n, sh, d_out, flags, stream);
        if (su != 0) return launch_k<Desc, 1, 1, true, SEEDED, 2>(desc, n, sh, d_out, flags, stream);
    }
    if constexpr (!kAllVariants && std::is_same<Desc, StridedDesc>::value) {
        // Every chunk takes stream mode: the per-packet path never runs, so it is built with the
        // fewest registers (U = P = 1; the kernel's occupancy is set by the larger path).
        if (desc.back_to_back() && pick_stream_for(false, sh) > 0)
            return launch_s<Desc, 1, 1, SEEDED>(desc, n, sh, d_out, flags, stream);
    }
    if constexpr (!kAllVariants && Desc::kCsr) {
        // CSR entry points pass max_len 1500: U = 2 (pick_unroll)
        return launch_u<Desc, 2, SEEDED>(desc, n, sh, d_out, flags, stream);
    } else if constexpr (!kAllVariants && std::is_base_of<SlottedDesc, Desc>::value) {
        // ring slots pass max_len <= 2000: U <= 2 (batch_slotted_from)
        if (pick_unroll(max_len) <= 1) return launch_u<Desc, 1, SEEDED>(desc, n, sh, d_out, flags, stream);
        return launch_u<Desc, 2, SEEDED>(desc, n, sh, d_out, flags, stream);
    } else {
        switch (pick_unroll(max_len)) {
            case 1: return launch_u<Desc, 1, SEEDED>(desc, n, sh, d_out, flags, stream);
            case 2: return launch_u<Desc, 2, SEEDED>(desc, n, sh, d_out, flags, stream);
            case 3: return launch_u<Desc, 3, SEEDED>(desc, n, sh, d_out, flags, stream);
            case 4: return launch_u<Desc, 4, SEEDED>(desc, n, sh, d_out, flags, stream);
        }
        return AIPSTACK_CHKSUM_EINVAL;
    }
}

// Short runs (round 5, the default for back-to-back strided packets): stream mode on chunks of
// about 12 KiB (8 x 1500 B; one 9000-B packet), one chunk per wave, groups of 8 windows
// double-buffered (SU = 16), so a wave has all of its chunk's loads out before it sums the first
// window -- the round-4 gathered stream's issue pattern at stream mode's instruction count.
// Config A, driver protocol (--steps 20 --warmup 5): the gathered stream's higher VALU rate
// brings a clock dip ~3 ms into a run (launches 14-45 at 250-273 us against 220 after it,
// profiles/r05/driver); stream mode with 64-packet chunks has none but runs 233 us.
template <class Desc, bool SEEDED>
int launch_short_runs(const Desc &desc, uint64_t n, uint32_t len, uint16_t *d_out, uint32_t flags,
                      hipStream_t stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    const int cus = device_cu_count(stream);
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    if (tuning_stream_windows(2) == 0)  // tunable stream = -1: the per-packet wave mode
        return launch<Desc, SEEDED>(desc, n, len, d_out, flags, stream);
    Shape sh = pick_shape(n, cus);  // (tunable chunk_packets: short runs of that many)
    if (tuning().chunk_packets.load(std::memory_order_relaxed) == 0) {
        if (sh.small) return launch<Desc, SEEDED>(desc, n, len, d_out, flags, stream);
        uint32_t cp = 1;  // the largest power of two with cp * len <= 12 KiB (at least 1)
        while (cp < (uint32_t)kWave && (uint64_t)(2 * cp) * len <= 12288u) cp <<= 1;
        sh.chunk_packets = cp;
    }
    // Occupancy: the 5 waves per SIMD its 96 VGPRs allow. At 3 (tunable lds_pad = 41984: 3
    // blocks of 4 waves per CU's 160 KiB) config A's steady state is 222.5 us against 230.1
    // (tools/ab.py, one process, rotated batches, profiles/r05/occ), but the faster kernel
    // draws the clock dip described above into the driver's 25-launch protocol: 243-247 us
    // there against 228-229 (profiles/r05/driver2). B loses at 3 (366.9 vs 331.8 us).
    // Column runs (SU 64, sum_column_chunk) for fixed-length packets of 1 KiB or more; stream
    // prefixes for shorter and mixed lengths (several packet starts per window: config C
    // 235.9 us with stream prefixes against 242.7 in columns). Config A: 223.2 us against 229.6
    // at steady state (tools/ab.py), and 218.6 under the driver's protocol (--steps 20
    // --warmup 5; the gathered stream 230-237, stream prefixes 228-231), 35.0 M VALU per
    // launch against 50.9 M and 74.5 M (profiles/r05/col, shape). Tunable short_loads: 0
    // stream prefixes, 1 the same through global loads, 2 columns (-1: automatic).
    int mode = tuning().short_loads.load(std::memory_order_relaxed);
    if (mode < 0) mode = (!Desc::kCsr && len >= 1024u) ? 2 : 0;
    if (mode == 3) {  // segment tables (SU 96): lane cnt holds the run's end, so cnt < 64
        if (sh.chunk_packets > 32u) sh.chunk_packets = 32u;
        return launch_k<Desc, 1, 1, true, SEEDED, 96>(desc, n, sh, d_out, flags, stream, true,
                                                      kShortRunLds);
    }
    if (mode == 2) {  // column runs (SU 64)
        if (sh.chunk_packets > (uint32_t)kColMaxPackets) sh.chunk_packets = kColMaxPackets;
        // chunks of one packet over 8 KiB (B: 9000 B, 8.8 windows) in groups of 6 windows: 12
        // loaded against 16 in groups of 8; under the driver's protocol B 336.8-337.7 us
        // against 338.3-344.0 (A, 12 KiB chunks, keeps 8: 220.9-221.9 against 222.7-223.1;
        // profiles/r05/colu)
        // AIPSTACK_CHKSUM_JUST_WRITTEN: the form that reads no line of the batch through the
        // L2-allocating path (sum_column_chunk CAPTURE)
        const bool fresh = (flags & AIPSTACK_CHKSUM_JUST_WRITTEN) != 0;
        if constexpr (!Desc::kCsr) {
            if (sh.chunk_packets == 1u && len > 8192u)
                return fresh ? launch_k<Desc, 1, 1, true, SEEDED, 50>(desc, n, sh, d_out, flags,
                                                                      stream, true, kShortRunLds)
                             : launch_k<Desc, 1, 1, true, SEEDED, 48>(desc, n, sh, d_out, flags,
                                                                      stream, true, kShortRunLds);
        }
        return fresh ? launch_k<Desc, 1, 1, true, SEEDED, 66>(desc, n, sh, d_out, flags, stream,
                                                              true, kShortRunLds)
                     : launch_k<Desc, 1, 1, true, SEEDED, 64>(desc, n, sh, d_out, flags, stream,
                                                              true, kShortRunLds);
    }
    if (mode == 1)  // global loads (SU 32)
        return launch_k<Desc, 1, 1, true, SEEDED, 32>(desc, n, sh, d_out, flags, stream, true,
                                                      kShortRunLds);
    return launch_k<Desc, 1, 1, true, SEEDED, 16>(desc, n, sh, d_out, flags, stream, true,
                                                  kShortRunLds);
}

// Gapped column runs (round 5, the default for fixed-length packets at a stride that is a
// multiple of 16, in device memory): chunks of the largest power of two of packets with
// <= 12 KiB (at most 16), one per wave, through sum_gapped_column_chunk. Strides from 8 MiB,
// packets over 32 KiB, small batches and tunable gather = 0 keep the gathered stream.
int launch_gapped(const GappedDesc &g, uint64_t n, uint16_t *d_out, uint32_t flags,
                  hipStream_t stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    const int cus = device_cu_count(stream);
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    const uint32_t rs = (uint32_t)g.base & 15u;
    const uint32_t ns = (rs + g.len + 15u) >> 4;
    Shape sh = pick_shape(n, cus);
    const int gm = tuning().gather.load(std::memory_order_relaxed);
    const bool cols = gm != 0 && g.len > 0 && (g.stride & 15u) == 0 && g.stride < (1u << 23) &&
                      ns <= 2048u && tuning_stream_windows(4) != 0 &&
                      (!sh.small || tuning().chunk_packets.load(std::memory_order_relaxed) != 0);
    if (!cols) return launch<GappedDesc, false>(g, n, g.len, d_out, flags, stream);
    if (tuning().chunk_packets.load(std::memory_order_relaxed) == 0) {
        uint32_t cp = 1;
        while (cp < (uint32_t)kColMaxPackets && (uint64_t)(2 * cp) * g.len <= 12288u) cp <<= 1;
        sh.chunk_packets = cp;
    }
    if (sh.chunk_packets > (uint32_t)kColMaxPackets) sh.chunk_packets = kColMaxPackets;
    uint32_t cp2 = 1;  // a power of two (the column sums' lane split)
    while (cp2 * 2u <= sh.chunk_packets) cp2 <<= 1;
    sh.chunk_packets = cp2;
    GappedColDesc d;
    static_cast<GappedDesc &>(d) = g;
    d.ns = ns;
    d.magic = (uint32_t)(((1ull << 32) + ns - 1u) / ns);
    d.gap = (int32_t)((int64_t)g.stride - 16 * (int64_t)ns);
    return launch_k<GappedColDesc, 1, 1, true, false, 64>(d, n, sh, d_out, flags, stream, true,
                                                          kShortRunLds);
}

template <bool NT, int SU>
int launch_chain(const uint64_t *d_addr, const uint32_t *d_len, const uint64_t *d_index,
                 const uint32_t *d_states, const uint64_t *d_fields, uint64_t n,
                 uint16_t *d_out, uint32_t flags, hipStream_t stream) {
    const int cus = device_cu_count(stream);
    if (cus <= 0) return AIPSTACK_CHKSUM_EHIP;
    // chains per group: 32 for large batches (CHAIN 230.8 us against 233.2 at 64 and 231.9 at
    // 16, profiles/r04/shape2), fewer for small ones, or the chunk_packets tunable
    uint32_t cpg = pick_shape(n, cus).chunk_packets;
    if (cpg > 32u && tuning().chunk_packets.load(std::memory_order_relaxed) == 0) cpg = 32u;
    const uint64_t nchunks = (n + cpg - 1) / cpg;
    const uint64_t target_waves = (uint64_t)cus * 2 * kDefaultWavesPerCu;
    uint64_t cpw = (nchunks + target_waves - 1) / target_waves;
    const int cpw_t = tuning().chunks_per_wave.load(std::memory_order_relaxed);
    // groups per wave (tunable; default one for large batches: CHAIN 249.9-254.9 us against
    // 262.6-266.2 at 2, 267.1-267.3 at 4, 273.9-277.9 at 8, profiles/r06/chshape/)
    if (cpw_t > 0) cpw = (uint64_t)cpw_t;
    if (cpw == 0) cpw = 1;
    const uint64_t waves = (nchunks + cpw - 1) / cpw;
    const uint64_t blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > 0x7FFFFFFFull || cpw > 0xFFFFFFFFull) return AIPSTACK_CHKSUM_EINVAL;
    // just-written bytes: the column-run kernel (SU 4 only; see chksum_chain_kernel)
    bool cols = false;
    if constexpr (SU > 2) {
        cols = (flags & AIPSTACK_CHKSUM_JUST_WRITTEN) && tuning_chain_short() != 0;
        if (cols)
            hipLaunchKernelGGL((chksum_chain_kernel<NT, SU, true>), dim3((unsigned)blocks),
                               dim3(kBlock), tuning_lds_pad(0), stream, d_addr, d_len, d_index,
                               d_states, n, (uint32_t)cpw, cpg, d_out, flags,
                               (uint32_t)tuning_chain_short());
    }
    if (!cols)
        hipLaunchKernelGGL((chksum_chain_kernel<NT, SU>), dim3((unsigned)blocks), dim3(kBlock),
                           tuning_lds_pad(0), stream, d_addr, d_len, d_index, d_states, n,
                           (uint32_t)cpw, cpg, d_out, flags, (uint32_t)tuning_chain_short());
    if (d_fields) {  // chain fill: the field stores as a pass of their own
        const int st = check_hip(hipGetLastError());
        if (st != AIPSTACK_CHKSUM_OK) return st;
        const uint64_t sblocks = min((n + kBlock - 1) / kBlock, (uint64_t)cus * 64);
        hipLaunchKernelGGL(chain_field_scatter_kernel, dim3((unsigned)sblocks), dim3(kBlock), 0,
                           stream, d_fields, d_out, n);
    }
    return check_hip(hipGetLastError());
}

}  // namespace

int take_violations_batch(uint32_t *mask, bool clear) {
    return take_violations_here(mask, clear);
}

int tuning_waves_per_cu() {
    return tuning().waves_per_cu.load(std::memory_order_relaxed);
}

int tuning_engine_zero_copy() { return tuning().engine_zero_copy.load(std::memory_order_relaxed); }
int tuning_engine_zero_copy_small() {
    return tuning().engine_zero_copy_small.load(std::memory_order_relaxed);
}
int tuning_engine_pageable_rows() {
    return tuning().engine_pageable_rows.load(std::memory_order_relaxed);
}

int tuning_stream_windows(int family_default) {
    const int t = tuning().stream.load(std::memory_order_relaxed);
    if (t < 0) return 0;
    if (t == 2 || t == 4 || t == 8) return t;
    return family_default;
}

uint32_t frames_per_chunk(uint64_t n, int cus) { return pick_shape(n, cus).chunk_packets; }

int tuning_chunk_packets() { return tuning().chunk_packets.load(std::memory_order_relaxed); }

unsigned tuning_lds_pad(int family_default) {
    int pad = tuning().lds_pad.load(std::memory_order_relaxed);
    if (pad == 0) pad = family_default;
    return (unsigned)(pad > 0 && pad <= 65536 ? pad : 0);
}

int tuning_tx_header_mode(int family_default) {
    const int t = tuning().tx_gather.load(std::memory_order_relaxed);
    return (t >= 0 && t <= 2) ? t : family_default;
}

int tuning_chain_short() {
    const int t = tuning().chain_short.load(std::memory_order_relaxed);
    return t < 0 ? 128 : (t > 65535 ? 65535 : t);
}

int tuning_tx_store(int family_default) {
    const int t = tuning().tx_store.load(std::memory_order_relaxed);
    return (t == kTxStoreFields || t == kTxStoreSectors || t == kTxStoreLines) ? t
                                                                                : family_default;
}

int tuning_frames_in_flight() {
    const int f = tuning().frames.load(std::memory_order_relaxed);
    return (f == 2 || f == 4 || f == 8) ? f : 4;
}

}  // namespace aipstack_amd

using namespace aipstack_amd;

namespace aipstack_amd {

int batch_strided_from(const void *d_base, uint64_t stride, uint32_t len, uint64_t n,
                       uint16_t *d_out, uint32_t flags, void *stream, bool host_bytes) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_out || len > AIPSTACK_CHKSUM_MAX_LEN) return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    // The gathered stream (round 4), also for packets back to back: config A 217.2 us against
    // 232.5 in stream mode, B 336.2 / 337.7 (profiles/r04/gatherA). Stream mode stays for
    // stride == len where the bytes are read over the link from host memory (the engine's
    // zero-copy pieces: A end to end 49.7 vs 48.7 GiB/s, profiles/r04/final/e2e.jsonl) or
    // when tunable "gather" = -1.
    // Round 5: back-to-back packets in device memory take short runs (launch_short_runs);
    // tunable "gather" 0 = the round-4 gathered stream, -1 = rounds 1-3 stream mode.
    const int gm = tuning().gather.load(std::memory_order_relaxed);
    if (stride != len && host_bytes) {  // over the link: edges masked in the stream
        GappedHostDesc h;
        static_cast<GappedDesc &>(h) = GappedDesc{(uint64_t)(uintptr_t)d_base, stride, len};
        return launch<GappedHostDesc, false>(h, n, len, d_out, flags, (hipStream_t)stream);
    }
    if (stride != len) {  // gaps between the packets (device memory)
        GappedDesc d{(uint64_t)(uintptr_t)d_base, stride, len};
        return launch_gapped(d, n, d_out, flags, (hipStream_t)stream);
    }
    if (!host_bytes && gm == 0) {
        GappedDesc d{(uint64_t)(uintptr_t)d_base, stride, len};
        return launch<GappedDesc, false>(d, n, len, d_out, flags, (hipStream_t)stream);
    }
    StridedDesc d{(uint64_t)(uintptr_t)d_base, stride, len};
    if (!host_bytes && gm != -1 && len >= 64u)
        return launch_short_runs<StridedDesc, false>(d, n, len, d_out, flags, (hipStream_t)stream);
    return launch<StridedDesc, false>(d, n, len, d_out, flags, (hipStream_t)stream);
}

int batch_csr_from(const void *d_base, const uint64_t *d_offsets, uint64_t n, uint16_t *d_out,
                   uint32_t flags, void *stream, bool host_bytes) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_offsets || !d_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    // CSR packets are back to back: short runs (round 5; config C 236.8 us against 241.7 for
    // the round-4 gathered stream, tools/ab.py, profiles/r05/driver2), except for bytes read
    // over the link from host memory (C end to end 48.9 vs 44.9 GiB/s in stream mode) or with
    // tunable "gather" 0 (gathered) / -1 (stream mode, 64-packet chunks).
    const int gm = tuning().gather.load(std::memory_order_relaxed);
    if (!host_bytes && gm >= 1) {  // short runs (launch_short_runs), 16-packet chunks at ~760 B
        CsrDesc d{(uint64_t)(uintptr_t)d_base, d_offsets};
        return launch_short_runs<CsrDesc, false>(d, n, 768u, d_out, flags, (hipStream_t)stream);
    }
    if (!host_bytes && gm != -1) {
        GatheredCsrDesc d;
        d.base = (uint64_t)(uintptr_t)d_base;
        d.offsets = d_offsets;
        return launch<GatheredCsrDesc, false>(d, n, 1500u, d_out, flags, (hipStream_t)stream);
    }
    CsrDesc d{(uint64_t)(uintptr_t)d_base, d_offsets};
    return launch<CsrDesc, false>(d, n, 1500u, d_out, flags, (hipStream_t)stream);
}

}  // namespace aipstack_amd

extern "C" int aipstack_chksum_batch_strided(const void *d_base, uint64_t stride, uint32_t len,
                                             uint64_t n, uint16_t *d_out, uint32_t flags,
                                             void *stream) {
    return batch_strided_from(d_base, stride, len, n, d_out, flags, stream, false);
}

namespace aipstack_amd {

int batch_slotted_from(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                       uint64_t n, uint16_t *d_out, uint32_t flags, void *stream,
                       bool host_bytes) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_base || !d_len || !d_out || slot_stride == 0 || n > (1ull << 40))
        return AIPSTACK_CHKSUM_EINVAL;
    SlottedDesc d;
    d.base = (uint64_t)(uintptr_t)d_base;
    d.stride = slot_stride;
    d.lens = d_len;
    d.cap = (uint32_t)(slot_stride < AIPSTACK_CHKSUM_MAX_LEN ? slot_stride : AIPSTACK_CHKSUM_MAX_LEN);
    // U from the typical packet (<= ~2 KiB: one group of 2 segments per lane), not the
    // slot: C2K (64-1500 B in 2048-B slots) U = 1 / 2 / 3: 286 / 277 / 328 us
    // (profiles/r03/slots/sweep_C2K.jsonl); longer packets loop over further groups
    const uint32_t max_len = d.cap < 2000u ? d.cap : 2000u;
    if (host_bytes) {  // read over the link: edges masked in the stream (SlottedHostDesc)
        SlottedHostDesc h;
        static_cast<SlottedDesc &>(h) = d;
        return launch<SlottedHostDesc, false>(h, n, max_len, d_out, flags, (hipStream_t)stream);
    }
    return launch<SlottedDesc, false>(d, n, max_len, d_out, flags, (hipStream_t)stream);
}

}  // namespace aipstack_amd

extern "C" int aipstack_chksum_batch_slotted(const void *d_base, uint64_t slot_stride,
                                             const uint32_t *d_len, uint64_t n, uint16_t *d_out,
                                             uint32_t flags, void *stream) {
    return batch_slotted_from(d_base, slot_stride, d_len, n, d_out, flags, stream, false);
}

extern "C" int aipstack_chksum_batch_csr(const void *d_base, const uint64_t *d_offsets,
                                         uint64_t n, uint16_t *d_out, uint32_t flags,
                                         void *stream) {
    return batch_csr_from(d_base, d_offsets, n, d_out, flags, stream, false);
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
    // sweep-only tunables: their non-default values need a -DAIPSTACK_ALL_VARIANTS build
    else if (!std::strcmp(key, "unroll") && (kAllVariants || value == 0)) t.unroll = value;
    else if (!std::strcmp(key, "packets") && (kAllVariants || value == 0)) t.packets = value;
    else if (!std::strcmp(key, "nontemporal") && (kAllVariants || value == 1)) t.nontemporal = value;
    else if (!std::strcmp(key, "frames") && (kAllVariants || value == 0 || value == 4))
        t.frames = value;
    else if (!std::strcmp(key, "stream")) t.stream = value;
    else if (!std::strcmp(key, "chunk_packets")) t.chunk_packets = value;
    else if (!std::strcmp(key, "tx_gather")) t.tx_gather = value;
    else if (!std::strcmp(key, "tx_store")) t.tx_store = value;
    else if (!std::strcmp(key, "chain_short")) t.chain_short = value;
    else if (!std::strcmp(key, "gather")) t.gather = value;
    else if (!std::strcmp(key, "lds_pad")) t.lds_pad = value;
    else if (!std::strcmp(key, "short_loads")) t.short_loads = value;
    else if (!std::strcmp(key, "slot_windows")) t.slot_windows = value;
    else if (!std::strcmp(key, "engine_zero_copy")) t.engine_zero_copy = value;
    else if (!std::strcmp(key, "engine_zero_copy_small")) t.engine_zero_copy_small = value;
    else if (!std::strcmp(key, "engine_pageable_rows")) t.engine_pageable_rows = value;
    else return AIPSTACK_CHKSUM_EINVAL;
    return AIPSTACK_CHKSUM_OK;
}

extern "C" int aipstack_chksum_launch_shape(uint64_t n, int cus, int csr,
                                            uint32_t *chunk_packets, int *stream_windows) {
    if (!chunk_packets || !stream_windows || cus <= 0) return AIPSTACK_CHKSUM_EINVAL;
    const Shape sh = pick_shape(n, cus);
    *chunk_packets = sh.chunk_packets;
    *stream_windows = pick_stream_for(csr != 0, sh);
    return AIPSTACK_CHKSUM_OK;
}

namespace {
int chain_batch(const uint64_t *d_chunk_addr, const uint32_t *d_chunk_len,
                const uint64_t *d_chunk_index, const uint32_t *d_states,
                const uint64_t *d_fields, uint64_t n, uint16_t *d_out, uint32_t flags,
                void *stream) {
    // SU: gathered-stream windows per group ("stream" tunable: 2 or 4; off and 8 map to
    // 2 -- every chunk goes through the gathered stream, and 8 windows spill registers).
    // Measured on CHAIN (profiles/r02/bench_CHAIN_cleaned_sweep.jsonl): 2 windows, 73 VGPRs,
    // 6 waves per SIMD, 286-291 us; 4 windows, 96 VGPRs, 5 waves, 300-302 us.
#define AIPSTACK_LAUNCH_CHAIN(NT, SU)                                                       \
    return launch_chain<NT, SU>(d_chunk_addr, d_chunk_len, d_chunk_index, d_states, d_fields, \
                                n, d_out, flags, (hipStream_t)stream)
    if constexpr (kAllVariants)
        if (!tuning().nontemporal.load(std::memory_order_relaxed)) AIPSTACK_LAUNCH_CHAIN(false, 2);
    // 4 windows in flight (round 4, once the SU = 4 kernel no longer spilled): CHAIN 242.0-242.4
    // against 248.3-248.4 us with 2, alternating processes (profiles/r04/calib)
    if (tuning_stream_windows(4) == 2) AIPSTACK_LAUNCH_CHAIN(true, 2);
    AIPSTACK_LAUNCH_CHAIN(true, 4);
#undef AIPSTACK_LAUNCH_CHAIN
}
}  // namespace

extern "C" int aipstack_chksum_batch_chain(const uint64_t *d_chunk_addr,
                                           const uint32_t *d_chunk_len,
                                           const uint64_t *d_chunk_index,
                                           const uint32_t *d_states, uint64_t n,
                                           uint16_t *d_out, uint32_t flags, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_chunk_addr || !d_chunk_len || !d_chunk_index || !d_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    return chain_batch(d_chunk_addr, d_chunk_len, d_chunk_index, d_states, nullptr, n, d_out,
                       flags & (AIPSTACK_CHKSUM_FINAL | AIPSTACK_CHKSUM_JUST_WRITTEN), stream);
}

extern "C" int aipstack_chksum_batch_chain_fill(const uint64_t *d_chunk_addr,
                                                const uint32_t *d_chunk_len,
                                                const uint64_t *d_chunk_index,
                                                const uint32_t *d_states,
                                                const uint64_t *d_field_addr, uint64_t n,
                                                uint16_t *d_out, uint32_t flags, void *stream) {
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!d_chunk_addr || !d_chunk_len || !d_chunk_index || !d_field_addr || !d_out)
        return AIPSTACK_CHKSUM_EINVAL;
    if (n > (1ull << 40)) return AIPSTACK_CHKSUM_EINVAL;
    return chain_batch(d_chunk_addr, d_chunk_len, d_chunk_index, d_states, d_field_addr, n,
                       d_out, AIPSTACK_CHKSUM_FINAL |
                                  (flags & (AIPSTACK_CHKSUM_ZERO_AS_FFFF | AIPSTACK_CHKSUM_JUST_WRITTEN)),
                       stream);
}
