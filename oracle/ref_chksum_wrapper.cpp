// TEST INFRASTRUCTURE ONLY -- builds the REFERENCE's own checksum code into
// oracle/_ref/libref_chksum.so (git-ignored; built only where /root/reference exists,
// then shipped to the GPU box as a prebuilt .so together with the snapshot).
//
// Nothing from the reference is copied here: this file #includes the reference header
// <aipstack/infra/Chksum.h> from /root/reference/src (see oracle/Makefile) and exports
// thin extern "C" entry points so that Python (ctypes) can
//   * generate the golden vectors under tests/golden/ (tests/golden/make_golden.py), and
//   * time the reference's scalar path as bench.py's cpu_baseline (kind "reference").
//
// Compiled with the reference's own flags: -std=c++17 -O2 (default.nix:7).

#include <aipstack/infra/Chksum.h>

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

using AIpStack::IpBufNode;
using AIpStack::IpBufRef;
using AIpStack::IpChksumAccumulator;

extern "C" {

// Reference IpChksumInverted (Chksum.h:77-99).
std::uint16_t ref_chksum_inverted(const char *data, std::size_t len)
{
    return IpChksumInverted(data, len);
}

// Reference IpChksum(ptr,len) (Chksum.h:122-125).
std::uint16_t ref_chksum(const char *data, std::size_t len)
{
    return AIpStack::IpChksum(data, len);
}

// Reference IpChksumAccumulator(State{state}).getChksum(IpBufRef{chain}) over a chain
// of `nchunks` IpBufNodes (Chksum.h:171-174, 263-315; Buf.h:68-251), starting at byte
// `offset` of the first node and covering `tot_len` bytes.
std::uint16_t ref_chksum_chain(std::uint32_t state, char *const *ptrs,
                               const std::size_t *lens, std::size_t nchunks,
                               std::size_t offset, std::size_t tot_len)
{
    std::vector<IpBufNode> nodes(nchunks ? nchunks : 1);
    for (std::size_t i = 0; i < nchunks; i++) {
        nodes[i].ptr = ptrs[i];
        nodes[i].len = lens[i];
        nodes[i].next = (i + 1 < nchunks) ? &nodes[i + 1] : nullptr;
    }
    IpChksumAccumulator acc{IpChksumAccumulator::State(state)};
    return acc.getChksum(IpBufRef{nodes.data(), offset, tot_len});
}

// Reference IpChksumAccumulator header-word API (Chksum.h:191-235) followed by
// getChksum(IpBufRef) over one flat buffer: state after addWord16 x n16,
// addWord32 x n32, addEvenBytes(hdr, hdr_len), then the payload.
std::uint16_t ref_accumulate(const std::uint16_t *w16, std::size_t n16,
                             const std::uint32_t *w32, std::size_t n32,
                             const char *hdr, std::size_t hdr_len,
                             char *payload, std::size_t payload_len,
                             std::uint32_t *state_out)
{
    IpChksumAccumulator acc;
    for (std::size_t i = 0; i < n16; i++)
        acc.addWord(AIpStack::WrapType<std::uint16_t>(), w16[i]);
    for (std::size_t i = 0; i < n32; i++)
        acc.addWord(AIpStack::WrapType<std::uint32_t>(), w32[i]);
    acc.addEvenBytes(hdr, hdr_len);
    if (state_out)
        *state_out = static_cast<std::uint32_t>(acc.getState());
    IpBufNode node{payload, payload_len, nullptr};
    return acc.getChksum(IpBufRef{&node, 0, payload_len});
}

// CPU baseline: the reference's scalar IpChksumInverted over a strided or CSR batch,
// on `threads` std::threads over disjoint packet ranges. Runs `reps` timed passes
// (after one untimed warm-up pass) and returns the MEDIAN pass time in seconds.
static double time_batch(int threads, int reps, std::uint64_t n,
                         const char *base, std::uint64_t stride, std::uint32_t len,
                         const std::uint64_t *offsets, std::uint16_t *out)
{
    if (threads < 1)
        threads = 1;
    auto pass = [&]() {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; t++) {
            std::uint64_t lo = n * std::uint64_t(t) / std::uint64_t(threads);
            std::uint64_t hi = n * std::uint64_t(t + 1) / std::uint64_t(threads);
            pool.emplace_back([=]() {
                for (std::uint64_t i = lo; i < hi; i++) {
                    if (offsets)
                        out[i] = IpChksumInverted(base + offsets[i],
                                                  std::size_t(offsets[i + 1] - offsets[i]));
                    else
                        out[i] = IpChksumInverted(base + i * stride, len);
                }
            });
        }
        for (auto &th : pool)
            th.join();
    };
    pass();
    std::vector<double> times;
    for (int r = 0; r < reps; r++) {
        auto t0 = std::chrono::steady_clock::now();
        pass();
        auto t1 = std::chrono::steady_clock::now();
        times.push_back(std::chrono::duration<double>(t1 - t0).count());
    }
    std::sort(times.begin(), times.end());
    return times.empty() ? 0.0 : times[times.size() / 2];
}

double ref_time_batch_strided(int threads, int reps, const char *base,
                              std::uint64_t stride, std::uint32_t len,
                              std::uint64_t n, std::uint16_t *out)
{
    return time_batch(threads, reps, n, base, stride, len, nullptr, out);
}

double ref_time_batch_csr(int threads, int reps, const char *base,
                          const std::uint64_t *offsets, std::uint64_t n,
                          std::uint16_t *out)
{
    return time_batch(threads, reps, n, base, 0, 0, offsets, out);
}

// CPU baseline for chains: chain i = chunks [index[i], index[i+1]) of the table (device
// addresses addr[k] - addr_bias = host addresses), linked as IpBufNodes once, outside the
// timing, as the stack holds them (a TCP header node + send-ring nodes). Each timed pass
// computes IpChksumAccumulator(State(states[i])).getChksum(IpBufRef{chain i}) for every
// chain (Chksum.h:171-174, 263-336), `threads` std::threads over disjoint chain ranges.
double ref_time_batch_chain(int threads, int reps, std::uint64_t addr_bias,
                            const std::uint64_t *addr, const std::uint32_t *len,
                            const std::uint64_t *index, const std::uint32_t *states,
                            std::uint64_t n, std::uint16_t *out)
{
    if (threads < 1)
        threads = 1;
    const std::uint64_t nchunks = index[n];
    std::vector<IpBufNode> nodes(nchunks ? nchunks : 1);
    std::vector<std::size_t> tot(n);
    for (std::uint64_t i = 0; i < n; i++) {
        std::size_t t = 0;
        for (std::uint64_t k = index[i]; k < index[i + 1]; k++) {
            nodes[k].ptr = reinterpret_cast<char *>(addr[k] - addr_bias);
            nodes[k].len = len[k];
            nodes[k].next = k + 1 < index[i + 1] ? &nodes[k + 1] : nullptr;
            t += len[k];
        }
        tot[i] = t;
    }
    auto pass = [&]() {
        std::vector<std::thread> pool;
        for (int th = 0; th < threads; th++) {
            std::uint64_t lo = n * std::uint64_t(th) / std::uint64_t(threads);
            std::uint64_t hi = n * std::uint64_t(th + 1) / std::uint64_t(threads);
            pool.emplace_back([&, lo, hi]() {
                for (std::uint64_t i = lo; i < hi; i++) {
                    IpChksumAccumulator acc{IpChksumAccumulator::State(states[i])};
                    out[i] = index[i + 1] > index[i]
                                 ? acc.getChksum(IpBufRef{&nodes[index[i]], 0, tot[i]})
                                 : acc.getChksum();
                }
            });
        }
        for (auto &t : pool)
            t.join();
    };
    pass();
    std::vector<double> times;
    for (int r = 0; r < reps; r++) {
        auto t0 = std::chrono::steady_clock::now();
        pass();
        auto t1 = std::chrono::steady_clock::now();
        times.push_back(std::chrono::duration<double>(t1 - t0).count());
    }
    std::sort(times.begin(), times.end());
    return times.empty() ? 0.0 : times[times.size() / 2];
}

} // extern "C"

// The reference stack's checksum call sequences (tests/cpp/call_sites.inc, shared text with
// tests/cpp/hpp_shim.cpp), compiled against the reference's AIpStack:: types as ref_cs_*.
using AIpStack::IpChksum;
using AIpStack::WrapType;
#define CS_NAME(x) ref_cs_##x
#define CS_PROCESS_BYTES(buf, len, fn) \
    AIpStack::ipBufProcessBytes(buf, len, AIpStack::makeTypedFunction(fn))
#include "call_sites.inc"
