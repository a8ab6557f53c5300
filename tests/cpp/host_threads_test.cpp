// The engines' host-thread layer (aipstack_amd/csrc/host_threads.{h,cpp}) on the CPU: the sysfs
// CPU-list parser, and HostPool -- every part of every run() done exactly once, also with
// several threads running jobs on one pool at once (the engine's submitting thread stages while
// its applier applies), a pool without workers, and stop() with nothing queued. Run by
// tests/test_host_cpp.py (plain and ASan/UBSan builds). Exit 0 = pass.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "host_threads.h"

using aipstack_amd::HostPool;
using aipstack_amd::parse_cpu_list;

static int failures = 0;
#define EXPECT(c, ...)                                           \
    do {                                                         \
        if (!(c)) {                                              \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);                   \
            std::fprintf(stderr, "\n");                          \
            ++failures;                                          \
        }                                                        \
    } while (0)

int main() {
    EXPECT((parse_cpu_list("0-3,8,10-11\n") == std::vector<int>{0, 1, 2, 3, 8, 10, 11}), "list");
    EXPECT((parse_cpu_list("5") == std::vector<int>{5}), "single");
    EXPECT(parse_cpu_list("").empty() && parse_cpu_list("3-1").empty() &&
               parse_cpu_list("a").empty() && parse_cpu_list("1-").empty(),
           "malformed lists give nothing");

    for (unsigned workers : {0u, 1u, 3u, 7u}) {
        HostPool pool;
        pool.start(workers, {});
        EXPECT(pool.workers() == workers, "workers");
        for (unsigned parts : {1u, 2u, 5u, 64u, 300u}) {
            std::vector<std::atomic<int>> hit(parts);
            pool.run(parts, [&](unsigned p) { hit[p].fetch_add(1); });
            bool ok = true;
            for (auto &h : hit) ok &= h.load() == 1;
            EXPECT(ok, "every part once (%u workers, %u parts)", workers, parts);
        }
        {  // a named callable (F deduces to an lvalue reference), and a const one
            std::vector<std::atomic<int>> hit(9);
            auto named = [&](unsigned p) { hit[p].fetch_add(1); };
            pool.run(9, named);
            const auto cnamed = [&](unsigned p) { hit[p].fetch_add(1); };
            pool.run(9, cnamed);
            bool ok = true;
            for (auto &h : hit) ok &= h.load() == 2;
            EXPECT(ok, "lvalue callables (%u workers)", workers);
        }
        // several callers at once, many rounds
        std::vector<std::thread> callers;
        std::atomic<long> total{0};
        for (int c = 0; c < 4; ++c)
            callers.emplace_back([&, c] {
                for (int round = 0; round < 200; ++round) {
                    const unsigned parts = 1u + (unsigned)((c * 7 + round) % 17);
                    std::vector<int> hit(parts, 0);
                    pool.run(parts, [&](unsigned p) { ++hit[p]; });
                    for (int h : hit)
                        if (h != 1) total.fetch_add(1000000);
                    total.fetch_add((long)parts);
                }
            });
        long want = 0;
        for (int c = 0; c < 4; ++c)
            for (int round = 0; round < 200; ++round) want += 1 + (c * 7 + round) % 17;
        for (auto &t : callers) t.join();
        EXPECT(total.load() == want, "concurrent runs (%u workers): %ld vs %ld", workers,
               total.load(), want);
        pool.stop();
        pool.stop();  // idempotent
    }
    if (failures) std::fprintf(stderr, "%d failures\n", failures);
    else std::printf("host_threads_test: OK\n");
    return failures ? 1 : 0;
}
