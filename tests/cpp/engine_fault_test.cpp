// The host-memory engine's error and teardown semantics (chksum_engine.cpp), with batch
// pieces made to fail on purpose: this program links an engine compiled with
// -DAIPSTACK_ENGINE_FAULT_INJECTION (test builds only; make -C tests/cpp engine_fault), whose
// aipstack_chksum_engine_test_inject(launch_mask, completion_mask) fails piece k (numbered
// from 1 per engine) at its launch or its completion as a HIP error would.
//
//   1. two failing batches in flight: _wait of the FIRST (whose failure was seen while the
//      second was being submitted) still returns < 0, once; a clean batch after them is exact
//   2. a launch failure part-way: _submit returns < 0 with the ticket set, _wait returns it
//   3. a failed piece of the batch being submitted stops its enqueue (status propagated)
//   4. destroy with a Tx fill batch pending: the frames end up filled (as the oracle fills)
//   5. unregister while a batch on the region is in flight: the batch completes first
//   6. _wait does not hold the engine while it waits: _poll from another thread returns
// Needs a GPU (exit 3 without one). Exit 0 = pass.
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <algorithm>
#include <vector>

#include "aipstack_amd/chksum.h"
#include "aipstack_amd/synth.h"
#include "frame_oracle.h"

extern "C" void aipstack_chksum_engine_test_inject(uint64_t fail_at_launch,
                                                    uint64_t fail_at_completion);
extern "C" void aipstack_chksum_engine_test_wait_delay(uint64_t us);

static int failures = 0;
#define EXPECT(cond, ...)                        \
    do {                                         \
        if (!(cond)) {                           \
            std::fprintf(stderr, "FAIL: ");      \
            std::fprintf(stderr, __VA_ARGS__);   \
            std::fprintf(stderr, "\n");          \
            ++failures;                          \
        }                                        \
    } while (0)

namespace {

constexpr uint32_t kLen = 1500;
constexpr uint64_t kChunk = 1u << 17;                     // 128 KiB pieces
constexpr uint64_t kPerPiece = (kChunk - kLen) / kLen + 1;  // 87 packets of 1500 B
constexpr int kStreams = 4;

uint64_t bit(int piece) { return 1ull << (piece - 1); }

std::vector<uint16_t> host_sums(const std::vector<unsigned char> &buf, uint64_t n) {
    std::vector<uint16_t> r(n);
    for (uint64_t i = 0; i < n; ++i)
        r[i] = IpChksumInverted(reinterpret_cast<const char *>(buf.data() + i * kLen), kLen);
    return r;
}

aipstack_chksum_engine *make_engine(uint64_t chunk = kChunk, int streams = kStreams) {
    aipstack_chksum_engine *e = nullptr;
    const int st = aipstack_chksum_engine_create(0, chunk, streams, &e);
    if (st != AIPSTACK_CHKSUM_OK) {
        std::fprintf(stderr, "engine create failed: %d\n", st);
        std::exit(2);
    }
    return e;
}

void two_failing_batches() {
    aipstack_chksum_engine *e = make_engine();
    const uint64_t n = 4 * kPerPiece;  // 4 pieces per batch, one per stream
    std::vector<unsigned char> a(n * kLen), b(n * kLen), c(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 1, 0);
    aipstack_synth_fill_host(b.data(), b.size(), 2, 0);
    aipstack_synth_fill_host(c.data(), c.size(), 3, 0);
    std::vector<uint16_t> oa(n), ob(n), oc(n);
    // A = pieces 1-4, B = pieces 5-8: B's submit completes A's pieces (back-pressure) and
    // sees piece 1 fail; piece 5 (B's first) fails when B is waited
    aipstack_chksum_engine_test_inject(0, bit(1) | bit(5));
    uint64_t ta = 0, tb = 0, tc = 0;
    EXPECT(aipstack_chksum_engine_submit_strided(e, a.data(), kLen, kLen, n, oa.data(), 0, &ta) == 0,
           "submit A");
    EXPECT(aipstack_chksum_engine_submit_strided(e, b.data(), kLen, kLen, n, ob.data(), 0, &tb) == 0,
           "submit B (A's failed piece belongs to A, not B)");
    EXPECT(aipstack_chksum_engine_wait(e, tb) < 0, "wait(B) must report B's failed piece");
    EXPECT(aipstack_chksum_engine_wait(e, ta) < 0,
           "wait(A) must report A's failed piece after B failed too");
    EXPECT(aipstack_chksum_engine_wait(e, ta) == 0, "a failure is reported once");
    EXPECT(aipstack_chksum_engine_poll(e, tb) == 0, "B's failure was consumed by wait");
    // pieces 2-4 of A completed fine: their results are in place
    const std::vector<uint16_t> wa = host_sums(a, n);
    EXPECT(std::equal(oa.begin() + kPerPiece, oa.end(), wa.begin() + kPerPiece),
           "A's good pieces must hold their results");
    aipstack_chksum_engine_test_inject(0, 0);
    EXPECT(aipstack_chksum_engine_submit_strided(e, c.data(), kLen, kLen, n, oc.data(), 0, &tc) == 0,
           "submit C");
    EXPECT(aipstack_chksum_engine_wait(e, tc) == 0 && oc == host_sums(c, n), "clean batch C");
    aipstack_chksum_engine_destroy(e);
}

void launch_failure_part_way() {
    aipstack_chksum_engine *e = make_engine();
    const uint64_t n = 3 * kPerPiece;
    std::vector<unsigned char> a(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 4, 0);
    std::vector<uint16_t> oa(n, 0);
    aipstack_chksum_engine_test_inject(bit(2), 0);  // the batch's second piece
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_submit_strided(e, a.data(), kLen, kLen, n, oa.data(), 0, &t);
    EXPECT(st < 0 && t != 0, "submit must fail at piece 2 with the ticket set (st %d)", st);
    EXPECT(aipstack_chksum_engine_wait(e, t) < 0, "wait of the part-enqueued batch reports it");
    const std::vector<uint16_t> w = host_sums(a, n);
    EXPECT(std::equal(oa.begin(), oa.begin() + kPerPiece, w.begin()),
           "the piece enqueued before the failure completes with its results");
    aipstack_chksum_engine_test_inject(0, 0);
    aipstack_chksum_engine_destroy(e);
}

void own_piece_failure_stops_enqueue() {
    aipstack_chksum_engine *e = make_engine();
    const uint64_t n = 8 * kPerPiece;  // wraps the 4 streams: piece 5 completes piece 1
    std::vector<unsigned char> a(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 5, 0);
    std::vector<uint16_t> oa(n);
    aipstack_chksum_engine_test_inject(0, bit(1));
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_submit_strided(e, a.data(), kLen, kLen, n, oa.data(), 0, &t);
    EXPECT(st < 0, "submit must return its own failed piece's status (got %d)", st);
    EXPECT(aipstack_chksum_engine_wait(e, t) < 0, "and wait reports it too");
    aipstack_chksum_engine_test_inject(0, 0);
    aipstack_chksum_engine_destroy(e);
}

void destroy_completes_tx() {
    const uint64_t nf = 20000;
    std::vector<uint64_t> off(nf + 1);
    const uint64_t bytes = aipstack_synth_frames_host(nullptr, off.data(), nf, 9, 1460);
    std::vector<unsigned char> fr(bytes), want(bytes);
    aipstack_synth_frames_host(fr.data(), off.data(), nf, 9, 1460);
    want = fr;
    std::vector<uint8_t> st(nf, 0xEE), want_st(nf);
    oracle_tx_fill_batch(want.data(), off.data(), nf, want_st.data());
    EXPECT(fr != want, "the synthetic frames must need filling");
    aipstack_chksum_engine *e = make_engine(1u << 20, 2);  // ~23 pieces
    uint64_t t = 0;
    EXPECT(aipstack_chksum_engine_submit_tx_fill(e, fr.data(), off.data(), nf, st.data(), &t) == 0,
           "submit tx fill");
    aipstack_chksum_engine_destroy(e);  // no wait: destroy completes the batch
    EXPECT(fr == want && st == want_st, "destroy must apply the pending Tx records");
}

void unregister_in_flight() {
    aipstack_chksum_engine *e = make_engine();
    const uint64_t n = 4 * kPerPiece;
    std::vector<unsigned char> a(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 6, 0);
    std::vector<uint16_t> oa(n);
    EXPECT(aipstack_chksum_engine_register(e, a.data(), a.size()) == 0, "register");
    uint64_t t = 0;
    EXPECT(aipstack_chksum_engine_submit_strided(e, a.data(), kLen, kLen, n, oa.data(), 0, &t) == 0,
           "submit on the registered region");
    EXPECT(aipstack_chksum_engine_unregister(e, a.data()) == 0, "unregister");
    EXPECT(oa == host_sums(a, n), "unregister completes the batch in flight first");
    EXPECT(aipstack_chksum_engine_wait(e, t) == 0, "and its ticket then completes with 0");
    aipstack_chksum_engine_destroy(e);
}

void wait_does_not_hold_the_engine() {
    // _wait stays 300 ms in its GPU wait (test hook: a sleep where it would block on the
    // batch's events, outside the engine lock); a _poll from another thread meanwhile must
    // return at once, not behind the waiter.
    aipstack_chksum_engine *e = make_engine();
    const uint64_t n = 4 * kPerPiece;
    std::vector<unsigned char> a(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 8, 0);
    std::vector<uint16_t> oa(n);
    uint64_t t = 0;
    EXPECT(aipstack_chksum_engine_submit_strided(e, a.data(), kLen, kLen, n, oa.data(), 0, &t) == 0,
           "submit");
    aipstack_chksum_engine_test_wait_delay(300000);
    std::atomic<bool> waited{false};
    int wst = -100;
    std::thread waiter([&] {
        wst = aipstack_chksum_engine_wait(e, t);
        waited = true;
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const auto p0 = std::chrono::steady_clock::now();
    const int p = aipstack_chksum_engine_poll(e, t);
    const double poll_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p0).count();
    const bool done_before = waited.load();
    waiter.join();
    aipstack_chksum_engine_test_wait_delay(0);
    EXPECT(!done_before && poll_ms < 100.0 && (p == 0 || p == 1),
           "poll must return while wait is waiting (poll %d after %.1f ms, waiter done %d)", p,
           poll_ms, (int)done_before);
    EXPECT(wst == 0, "wait");
    EXPECT(oa == host_sums(a, n), "results");
    aipstack_chksum_engine_destroy(e);
}

}  // namespace

int main() {
    if (aipstack_chksum_device_check(0) != AIPSTACK_CHKSUM_OK) {
        std::fprintf(stderr, "device 0 is not a usable gfx950 device\n");
        return 3;
    }
    two_failing_batches();
    launch_failure_part_way();
    own_piece_failure_stops_enqueue();
    destroy_completes_tx();
    unregister_in_flight();
    wait_does_not_hold_the_engine();
    if (failures) std::fprintf(stderr, "%d failures\n", failures);
    else std::printf("engine_fault_test: OK\n");
    std::fflush(nullptr);
    // Every engine was destroyed above. The HIP runtime's own exit-time teardown is skipped:
    // under ASan it frees through the sanitizer's device allocator after the HSA runtime has
    // unloaded ("dev_runtime_unloaded_" CHECK in libhsa-runtime64's __cxa_finalize path).
    std::_Exit(failures ? 1 : 0);
}
