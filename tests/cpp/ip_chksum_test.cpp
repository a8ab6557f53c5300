// Counterpart of the reference's tests/ip_chksum_test.cpp, run against this repo's C++
// surface (include/aipstack_amd/Chksum.hpp) and the host hook IpChksumInverted of
// libaipstack_chksum.so. Deterministic (fixed seed) instead of std::random_device.
//   1. Known answer (reference :33-62): 1023 x 0xFF as a 512-node chain (255 x 2 B,
//      1 x 1 B, 256 x 2 B) -> IpChksum == 0x00FF, chain == flat.
//   2. Property (reference :64-106): for random 101-byte buffers, the chained checksum
//      equals the flat one for every 2/3/4-chunk split at {33, 34, 50, 51}.
//   3. Extra: the same property with random states (pseudo-header seeds), scatter chains
//      whose chunks are not adjacent in memory, and odd chunk starts.
// Exit status 0 = pass; a failure prints and aborts (like AIPSTACK_ASSERT_FORCE).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "aipstack_amd/Chksum.hpp"

using namespace AIpStackAmd;

#define CHECK(cond)                                                                 \
    do {                                                                            \
        if (!(cond)) {                                                              \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            std::abort();                                                           \
        }                                                                           \
    } while (0)

int main(int argc, char **argv) {
    long iterations = argc > 1 ? std::atol(argv[1]) : 1000000;
    std::mt19937_64 rng(12345);

    {
        char data[1023];
        std::memset(data, 0xFF, sizeof(data));
        const int num_nodes = 512;
        IpBufNode node[num_nodes];
        for (int i = 0; i < num_nodes; i++) {
            std::size_t sz = (i == 255) ? 1 : 2;
            node[i] = IpBufNode{data, sz, (i == num_nodes - 1) ? nullptr : &node[i + 1]};
        }
        std::uint16_t chain = IpChksum(IpBufRef{&node[0], 0, 1023});
        std::uint16_t flat = IpChksum(data, 1023);
        CHECK(chain == flat);
        CHECK(chain == 0xFF);
    }

    const std::size_t buf_size = 101;
    char buf[buf_size];
    const std::size_t brk[4] = {buf_size / 3, buf_size / 3 + 1, buf_size / 2, buf_size / 2 + 1};
    for (long it = 0; it < iterations; it++) {
        for (std::size_t i = 0; i < buf_size; i++) buf[i] = char(rng() & 0xFF);
        const std::uint16_t good = IpChksum(buf, buf_size);
        IpBufNode node[4];
        for (int b1 = 0; b1 < 4; b1++) {
            node[0] = {buf, brk[b1], &node[1]};
            node[1] = {buf + brk[b1], buf_size - brk[b1], nullptr};
            CHECK(IpChksum(IpBufRef{&node[0], 0, buf_size}) == good);
            for (int b2 = b1 + 1; b2 < 4; b2++) {
                node[0] = {buf, brk[b1], &node[1]};
                node[1] = {buf + brk[b1], brk[b2] - brk[b1], &node[2]};
                node[2] = {buf + brk[b2], buf_size - brk[b2], nullptr};
                CHECK(IpChksum(IpBufRef{&node[0], 0, buf_size}) == good);
                for (int b3 = b2 + 1; b3 < 4; b3++) {
                    node[0] = {buf, brk[b1], &node[1]};
                    node[1] = {buf + brk[b1], brk[b2] - brk[b1], &node[2]};
                    node[2] = {buf + brk[b2], brk[b3] - brk[b2], &node[3]};
                    node[3] = {buf + brk[b3], buf_size - brk[b3], nullptr};
                    CHECK(IpChksum(IpBufRef{&node[0], 0, buf_size}) == good);
                }
            }
        }
    }

    // Scatter chains with states: compare against the flat concatenation.
    std::vector<char> pool(1 << 16), flat;
    for (auto &c : pool) c = char(rng() & 0xFF);
    for (long it = 0; it < iterations / 10 + 1; it++) {
        int nch = 1 + int(rng() % 6);
        std::vector<IpBufNode> nodes(nch);
        flat.clear();
        for (int i = 0; i < nch; i++) {
            std::size_t len = rng() % 4 == 0 ? rng() % 4 : rng() % 1600;
            std::size_t off = rng() % (pool.size() - len);
            nodes[i] = IpBufNode{pool.data() + off, len, i + 1 < nch ? &nodes[i + 1] : nullptr};
            flat.insert(flat.end(), pool.begin() + off, pool.begin() + off + len);
        }
        std::uint32_t state = std::uint32_t(rng());
        IpChksumAccumulator a{IpChksumAccumulator::State(state)};
        IpChksumAccumulator b{IpChksumAccumulator::State(state)};
        IpBufNode one{flat.data(), flat.size(), nullptr};
        CHECK(a.getChksum(IpBufRef{&nodes[0], 0, flat.size()}) ==
              b.getChksum(IpBufRef{&one, 0, flat.size()}));
    }

    std::printf("ip_chksum_test: OK (%ld iterations)\n", iterations);
    return 0;
}
