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
//   7. a submit waiting for a busy slot (back-pressure) does not hold the engine either: _poll
//      of an earlier batch from another thread answers at once (round 4)
//   8. an engine group (two engines: on devices 0 and 0, or on the devices listed in
//      AIPSTACK_FAULT_GROUP_DEVICES, e.g. "0,1" on a box with two GPUs): a group ticket with one
//      failing device reports that device's failure (dev_status) and the other's results are
//      exact; group tickets in flight completed out of order; the group's own destroy with a
//      batch pending
//   9. the same group, _wait and _poll of one failing ticket from two threads: while the wait
//      owns the ticket the poll answers "pending", and the failure is reported once, by the
//      wait
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
extern "C" void aipstack_chksum_engine_test_inject_only(const aipstack_chksum_engine *e);

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

void poll_answers_while_submit_is_back_pressured() {
    // One stream: batch B's submit must first complete batch A's piece on it. The test hook
    // makes that back-pressure wait 300 ms long (outside the engine lock); a _poll of A from
    // another thread meanwhile must answer at once.
    aipstack_chksum_engine *e = make_engine(kChunk, 1);
    const uint64_t n = kPerPiece;
    std::vector<unsigned char> a(n * kLen), b(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 11, 0);
    aipstack_synth_fill_host(b.data(), b.size(), 12, 0);
    std::vector<uint16_t> oa(n), ob(n);
    uint64_t ta = 0, tb = 0;
    EXPECT(aipstack_chksum_engine_submit_strided(e, a.data(), kLen, kLen, n, oa.data(), 0, &ta) == 0,
           "submit A");
    aipstack_chksum_engine_test_wait_delay(300000);
    std::atomic<bool> submitted{false};
    int sst = -100;
    std::thread submitter([&] {
        sst = aipstack_chksum_engine_submit_strided(e, b.data(), kLen, kLen, n, ob.data(), 0, &tb);
        submitted = true;
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    const auto p0 = std::chrono::steady_clock::now();
    const int p = aipstack_chksum_engine_poll(e, ta);
    const double poll_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p0).count();
    const bool done_before = submitted.load();
    submitter.join();
    aipstack_chksum_engine_test_wait_delay(0);
    EXPECT(!done_before && poll_ms < 100.0 && (p == 0 || p == 1),
           "poll must answer while a submit is back-pressured (poll %d after %.1f ms, submit "
           "done %d)", p, poll_ms, (int)done_before);
    EXPECT(sst == 0 && aipstack_chksum_engine_wait(e, tb) == 0, "submit / wait B");
    EXPECT(aipstack_chksum_engine_wait(e, ta) == 0, "wait A");
    EXPECT(oa == host_sums(a, n) && ob == host_sums(b, n), "results of A and B");
    aipstack_chksum_engine_destroy(e);
}

// The group's two devices: AIPSTACK_FAULT_GROUP_DEVICES ("a,b"), else device 0 twice.
void group_devices(int (&devs)[2]) {
    devs[0] = devs[1] = 0;
    if (const char *s = std::getenv("AIPSTACK_FAULT_GROUP_DEVICES"))
        if (std::sscanf(s, "%d,%d", &devs[0], &devs[1]) != 2) devs[0] = devs[1] = 0;
}

void group_ticket_with_one_failing_device() {
    int devs[2];
    group_devices(devs);
    aipstack_chksum_engine_group *g = nullptr;
    EXPECT(aipstack_chksum_engine_group_create(devs, 2, kChunk, kStreams, &g) == 0, "group create");
    if (!g) return;
    // 12 MB: split over both engines (>= 4 MiB each)
    const uint64_t n = 8000;
    std::vector<unsigned char> a(n * kLen), b(n * kLen), c(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 21, 0);
    aipstack_synth_fill_host(b.data(), b.size(), 22, 0);
    aipstack_synth_fill_host(c.data(), c.size(), 23, 0);
    std::vector<uint16_t> oa(n), ob(n), oc(n);
    aipstack_chksum_engine *e1 = aipstack_chksum_engine_group_engine(g, 1);
    EXPECT(e1 != nullptr && aipstack_chksum_engine_group_engine(g, 2) == nullptr, "group engines");
    aipstack_chksum_engine_test_inject_only(e1);
    aipstack_chksum_engine_test_inject(0, bit(1));  // engine 1's first piece fails
    uint64_t ta = 0, tb = 0, tc = 0;
    EXPECT(aipstack_chksum_engine_group_submit_strided(g, a.data(), kLen, kLen, n, oa.data(), 0,
                                                       &ta) == 0, "group submit A");
    int ds[2] = {-100, -100};
    const int wa = aipstack_chksum_engine_group_wait(g, ta, ds);
    EXPECT(wa < 0 && ds[0] == 0 && ds[1] < 0,
           "group wait A: device 1's failure (got %d, dev %d / %d)", wa, ds[0], ds[1]);
    const std::vector<uint16_t> want_a = host_sums(a, n);
    EXPECT(std::equal(oa.begin(), oa.begin() + 100, want_a.begin()),
           "device 0's range holds its results");
    EXPECT(aipstack_chksum_engine_group_wait(g, ta, nullptr) == 0, "a group failure is reported once");
    aipstack_chksum_engine_test_inject(0, 0);
    aipstack_chksum_engine_test_inject_only(nullptr);
    // two clean tickets in flight, completed out of order
    EXPECT(aipstack_chksum_engine_group_submit_strided(g, b.data(), kLen, kLen, n, ob.data(), 0,
                                                       &tb) == 0, "group submit B");
    EXPECT(aipstack_chksum_engine_group_submit_strided(g, c.data(), kLen, kLen, n, oc.data(), 0,
                                                       &tc) == 0, "group submit C");
    EXPECT(aipstack_chksum_engine_group_wait(g, tc, ds) == 0 && ds[0] == 0 && ds[1] == 0, "wait C");
    int pb = 1;
    for (int i = 0; i < 100000 && pb == 1; ++i) pb = aipstack_chksum_engine_group_poll(g, tb, ds);
    EXPECT(pb == 0, "poll B completes (%d)", pb);
    EXPECT(ob == host_sums(b, n) && oc == host_sums(c, n), "results of B and C");
    // destroy with a batch pending completes it
    std::vector<uint16_t> oa2(n);
    EXPECT(aipstack_chksum_engine_group_submit_strided(g, a.data(), kLen, kLen, n, oa2.data(), 0,
                                                       &ta) == 0, "group submit A again");
    aipstack_chksum_engine_group_destroy(g);
    EXPECT(oa2 == want_a, "group destroy completes the pending batch");
}

void group_wait_and_poll_of_one_ticket() {
    int devs[2];
    group_devices(devs);
    aipstack_chksum_engine_group *g = nullptr;
    EXPECT(aipstack_chksum_engine_group_create(devs, 2, kChunk, kStreams, &g) == 0, "group create");
    if (!g) return;
    const uint64_t n = 8000;  // 12 MB: split over both engines
    std::vector<unsigned char> a(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 24, 0);
    std::vector<uint16_t> oa(n);
    aipstack_chksum_engine_test_inject_only(aipstack_chksum_engine_group_engine(g, 1));
    aipstack_chksum_engine_test_inject(0, bit(1));  // engine 1's first piece fails
    aipstack_chksum_engine_test_wait_delay(200000);  // the wait sleeps 200 ms before it waits
    uint64_t t = 0;
    EXPECT(aipstack_chksum_engine_group_submit_strided(g, a.data(), kLen, kLen, n, oa.data(), 0,
                                                       &t) == 0, "group submit");
    int ds_w[2] = {-100, -100};
    std::atomic<int> w{1};
    std::thread waiter([&] { w = aipstack_chksum_engine_group_wait(g, t, ds_w); });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    int ds_p[2] = {-100, -100};
    const int p_during = aipstack_chksum_engine_group_poll(g, t, ds_p);
    waiter.join();
    const int p_after = aipstack_chksum_engine_group_poll(g, t, ds_p);
    aipstack_chksum_engine_test_wait_delay(0);
    aipstack_chksum_engine_test_inject(0, 0);
    aipstack_chksum_engine_test_inject_only(nullptr);
    EXPECT(p_during == 1, "a poll while the wait owns the ticket answers pending (%d)", p_during);
    EXPECT(w.load() < 0 && ds_w[0] == 0 && ds_w[1] < 0,
           "the wait reports device 1's failure (%d; %d / %d)", w.load(), ds_w[0], ds_w[1]);
    EXPECT(p_after == 0, "the completed ticket polls OK afterwards (%d)", p_after);
    aipstack_chksum_engine_group_destroy(g);
}

// Two waits of one ticket, both blocked when it completes with a failure: each returns the
// failure and every device's status (the second once returned OK, its
// dev_status untouched). A wait after the completion returns OK.
void group_two_waits_of_one_ticket() {
    int devs[2];
    group_devices(devs);
    aipstack_chksum_engine_group *g = nullptr;
    EXPECT(aipstack_chksum_engine_group_create(devs, 2, kChunk, kStreams, &g) == 0, "group create");
    if (!g) return;
    const uint64_t n = 8000;  // 12 MB: split over both engines
    std::vector<unsigned char> a(n * kLen);
    aipstack_synth_fill_host(a.data(), a.size(), 25, 0);
    std::vector<uint16_t> oa(n);
    aipstack_chksum_engine_test_inject_only(aipstack_chksum_engine_group_engine(g, 1));
    aipstack_chksum_engine_test_inject(0, bit(1));  // engine 1's first piece fails
    aipstack_chksum_engine_test_wait_delay(200000);  // the owning wait sleeps 200 ms first
    uint64_t t = 0;
    EXPECT(aipstack_chksum_engine_group_submit_strided(g, a.data(), kLen, kLen, n, oa.data(), 0,
                                                       &t) == 0, "group submit");
    int ds1[2] = {-100, -100}, ds2[2] = {-100, -100};
    std::atomic<int> w1{1}, w2{1};
    std::thread first([&] { w1 = aipstack_chksum_engine_group_wait(g, t, ds1); });
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    std::thread second([&] { w2 = aipstack_chksum_engine_group_wait(g, t, ds2); });
    first.join();
    second.join();
    int ds3[2] = {-100, -100};
    const int w3 = aipstack_chksum_engine_group_wait(g, t, ds3);
    aipstack_chksum_engine_test_wait_delay(0);
    aipstack_chksum_engine_test_inject(0, 0);
    aipstack_chksum_engine_test_inject_only(nullptr);
    EXPECT(w1.load() < 0 && ds1[0] == 0 && ds1[1] < 0,
           "the first wait reports device 1's failure (%d; %d / %d)", w1.load(), ds1[0], ds1[1]);
    EXPECT(w2.load() == w1.load() && ds2[0] == 0 && ds2[1] == ds1[1],
           "the second wait reports the same (%d; %d / %d)", w2.load(), ds2[0], ds2[1]);
    EXPECT(w3 == 0, "a wait after the completion returns OK (%d)", w3);
    aipstack_chksum_engine_group_destroy(g);
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
    poll_answers_while_submit_is_back_pressured();
    group_ticket_with_one_failing_device();
    group_wait_and_poll_of_one_ticket();
    group_two_waits_of_one_ticket();
    if (failures) std::fprintf(stderr, "%d failures\n", failures);
    else std::printf("engine_fault_test: OK\n");
    std::fflush(nullptr);
    // Every engine was destroyed above. The HIP runtime's own exit-time teardown is skipped:
    // under ASan it frees through the sanitizer's device allocator after the HSA runtime has
    // unloaded ("dev_runtime_unloaded_" CHECK in libhsa-runtime64's __cxa_finalize path).
    std::_Exit(failures ? 1 : 0);
}
