// Host hook throughput per body (tools only): IpChksumInverted variants of host_hook.cc on
// cache-resident packets of several sizes, one core. Prints one JSON line per size.
//   make -C tools build/hook_bench
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <vector>

extern "C" uint16_t aipstack_chksum_host_variant(int variant, const char *data, size_t len);

int main() {
    std::vector<char> buf(1 << 16);
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (char)(i * 2654435761u >> 13);
    const size_t sizes[] = {64, 576, 1500, 9000, 65535};
    const char *names[] = {"portable", "sse2", "avx2", "avx512"};
    for (size_t len : sizes) {
        std::printf("{\"len\": %zu", len);
        for (int v = 0; v < 4; ++v) {
            const size_t iters = (size_t)(2e9 / (double)len);
            unsigned acc = 0;
            const auto t0 = std::chrono::steady_clock::now();
            for (size_t k = 0; k < iters; ++k)
                acc += aipstack_chksum_host_variant(v, buf.data() + (k & 7), len);
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            std::printf(", \"%s_GiBps\": %.2f", names[v], (double)iters * len / s / (1 << 30));
            if (acc == 0xFFFFFFFFu) std::printf(" ");
        }
        std::printf("}\n");
    }
    return 0;
}
