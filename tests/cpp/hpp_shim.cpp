// Test shim: exposes the C++ header surface (include/aipstack_amd/Chksum.hpp) through
// extern "C" so the Python tests can check it against the reference's golden vectors:
// the accumulator/chain entry points below, and the reference stack's call sequences of
// call_sites.inc (hpp_cs_*), the same text the reference wrapper compiles as ref_cs_*.
#include <cstddef>
#include <cstdint>
#include <vector>

#include "aipstack_amd/Chksum.hpp"

using namespace AIpStackAmd;

extern "C" std::uint16_t hpp_chksum_chain(std::uint32_t state, char *const *ptrs,
                                          const std::size_t *lens, std::size_t nchunks,
                                          std::size_t offset, std::size_t tot_len) {
    std::vector<IpBufNode> nodes(nchunks ? nchunks : 1);
    for (std::size_t i = 0; i < nchunks; i++)
        nodes[i] = IpBufNode{ptrs[i], lens[i], i + 1 < nchunks ? &nodes[i + 1] : nullptr};
    IpChksumAccumulator acc{IpChksumAccumulator::State(state)};
    return acc.getChksum(IpBufRef{nodes.data(), offset, tot_len});
}

extern "C" std::uint16_t hpp_accumulate(const std::uint16_t *w16, std::size_t n16,
                                        const std::uint32_t *w32, std::size_t n32,
                                        const char *hdr, std::size_t hdr_len, char *payload,
                                        std::size_t payload_len, std::uint32_t *state_out) {
    IpChksumAccumulator acc;
    for (std::size_t i = 0; i < n16; i++) acc.addWord(WrapType<std::uint16_t>(), w16[i]);
    for (std::size_t i = 0; i < n32; i++) acc.addWord(WrapType<std::uint32_t>(), w32[i]);
    acc.addEvenBytes(hdr, hdr_len);
    if (state_out) *state_out = std::uint32_t(acc.getState());
    IpBufNode node{payload, payload_len, nullptr};
    return acc.getChksum(IpBufRef{&node, 0, payload_len});
}

extern "C" std::uint16_t hpp_chksum(const char *p, std::size_t n) { return IpChksum(p, n); }

#define CS_NAME(x) hpp_cs_##x
#define CS_PROCESS_BYTES(buf, len, fn) ipBufProcessBytes(buf, len, fn)
#include "call_sites.inc"
