// Timing harness of the repo's drop-in per-packet hook (tools only, loaded by bench.py's
// cpu_baseline leg): IpChksumInverted from libaipstack_chksum_hook.so -- the symbol the stack
// links under -DAIPSTACK_EXTERNAL_CHKSUM (reference src/aipstack/infra/Chksum.h:46-51) -- over
// a strided or CSR batch in host memory, on `threads` std::threads over disjoint packet
// ranges, the same way bench.py times the reference's own loop (oracle/ref_chksum_wrapper.cpp).
// Returns the MEDIAN of `reps` timed passes (after one untimed warm-up pass), in seconds.
//   make -C tools build/libhook_time.so
#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <thread>
#include <vector>

extern "C" uint16_t IpChksumInverted(const char *data, size_t len);

namespace {
double time_batch(int threads, int reps, uint64_t n, const char *base, uint64_t stride,
                  uint32_t len, const uint64_t *offsets, uint16_t *out) {
    if (threads < 1) threads = 1;
    auto pass = [&]() {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) {
            const uint64_t lo = n * (uint64_t)t / (uint64_t)threads;
            const uint64_t hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
            pool.emplace_back([=]() {
                for (uint64_t i = lo; i < hi; ++i)
                    out[i] = offsets ? IpChksumInverted(base + offsets[i],
                                                        (size_t)(offsets[i + 1] - offsets[i]))
                                     : IpChksumInverted(base + i * stride, len);
            });
        }
        for (std::thread &th : pool) th.join();
    };
    pass();
    std::vector<double> times;
    for (int r = 0; r < reps; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        pass();
        times.push_back(
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(times.begin(), times.end());
    return times.empty() ? 0.0 : times[times.size() / 2];
}
}  // namespace

extern "C" double hook_time_batch_strided(int threads, int reps, const char *base,
                                          uint64_t stride, uint32_t len, uint64_t n,
                                          uint16_t *out) {
    return time_batch(threads, reps, n, base, stride, len, nullptr, out);
}

extern "C" double hook_time_batch_csr(int threads, int reps, const char *base,
                                      const uint64_t *offsets, uint64_t n, uint16_t *out) {
    return time_batch(threads, reps, n, base, 0, 0, offsets, out);
}
