// Small-batch latency through the C-ABI from C++ (no Python wrappers): batches of N packets
// of 1500 B (config A's layout) from a ring of R slots, one aipstack_chksum_batch_strided
// launch per batch, timed with HIP events over K batches, eagerly and as replays of one
// hipGraph holding the R launches (stream capture). The last batch of each form is checked
// against the library's host hook (IpChksumInverted, itself pinned to the reference by the
// CPU suite). Prints one JSON line per N.
//
//   tools/build/latency_capi [N ...]        (default N = 1 64 256 1024 4096 16384)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "aipstack_amd/chksum.h"
#include "aipstack_amd/synth.h"

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

static int run(uint64_t n) {
    const uint32_t len = 1500;
    const int R = 64;
    const int K = 4096;
    const uint64_t slot = n * len;
    char *d_buf = nullptr;
    uint16_t *d_out = nullptr;
    CHECK(hipMalloc(&d_buf, slot * R));
    CHECK(hipMalloc(&d_out, n * sizeof(uint16_t) * R));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (aipstack_synth_fill_device(d_buf, slot * R, 42, 0, s) != 0) return 1;
    auto launch = [&](int r) {
        return aipstack_chksum_batch_strided(d_buf + r * slot, len, len, n, d_out + r * n, 0, s);
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto check = [&](int r) {
        std::vector<char> h(slot);
        std::vector<uint16_t> got(n);
        CHECK(hipMemcpy(h.data(), d_buf + r * slot, slot, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(got.data(), d_out + r * n, n * 2, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n; ++i)
            if (got[i] != IpChksumInverted(h.data() + i * len, len)) return false;
        return true;
    };
    // eager
    for (int k = 0; k < K; ++k)
        if (launch(k % R) != 0) return 1;
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(e0, s));
    for (int k = 0; k < K; ++k)
        if (launch(k % R) != 0) return 1;
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms_eager = 0;
    CHECK(hipEventElapsedTime(&ms_eager, e0, e1));
    const bool ok_e = check((K - 1) % R);
    // graph: R launches captured once, replayed K / R times
    CHECK(hipMemsetAsync(d_out, 0, n * sizeof(uint16_t) * R, s));
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < R; ++r)
        if (launch(r) != 0) return 1;
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int k = 0; k < K / R; ++k) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(e0, s));
    for (int k = 0; k < K / R; ++k) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms_graph = 0;
    CHECK(hipEventElapsedTime(&ms_graph, e0, e1));
    const bool ok_g = check(R - 1);
    const double us_e = ms_eager * 1e3 / K, us_g = ms_graph * 1e3 / K;
    std::printf("{\"metric\": \"small batches through the C-ABI from C++ (%llu x 1500 B per batch)\", "
                "\"eager_us\": %.3f, \"graph_us\": %.3f, \"eager_GiB_s\": %.2f, "
                "\"graph_GiB_s\": %.2f, \"batches\": %d, \"ring_slots\": %d, \"parity\": \"%s\"}\n",
                (unsigned long long)n, us_e, us_g, slot / (us_e * 1e-6) / (1ull << 30),
                slot / (us_g * 1e-6) / (1ull << 30), K, R, ok_e && ok_g ? "bit-exact" : "MISMATCH");
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    CHECK(hipStreamDestroy(s));
    CHECK(hipFree(d_buf));
    CHECK(hipFree(d_out));
    return ok_e && ok_g ? 0 : 2;
}

int main(int argc, char **argv) {
    std::vector<uint64_t> ns = {1, 64, 256, 1024, 4096, 16384};
    if (argc > 1) {
        ns.clear();
        for (int i = 1; i < argc; ++i) ns.push_back(std::strtoull(argv[i], nullptr, 10));
    }
    int rc = 0;
    for (uint64_t n : ns) rc |= run(n);
    return rc;
}
