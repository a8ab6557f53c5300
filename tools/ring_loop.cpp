// A TAP-style receive loop through the host engine, from C++ (tools only): a registered ring
// of R regions x B slots of 2048 B holding raw frames (the RX mix of the bench, Tx-filled so
// that most verify), driven the way a receive loop would drive it -- region r is submitted
// for Rx verify (aipstack_chksum_engine_submit_rx_verify_slotted) and only waited for when the
// loop comes back to r, so R - 1 batches stay in flight. Times K batches per batch size B and
// checks the verdicts of every region of the last lap against the frame oracle. Prints one
// JSON line per B: batches/s, frames/s, GiB/s of frame bytes, us per batch.
//
//   tools/build/ring_loop [-r R] [B ...]   (default R = 8, B = 256 1024 4096 16384 65536;
//                                         R = 1: one batch at a time, the round-trip latency)
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aipstack_amd/chksum.h"
#include "aipstack_amd/synth.h"
#include "frame_oracle.h"

static int run(uint64_t B, uint64_t R) {
    const uint64_t slot = 2048;
    const uint64_t nfr = R * B;
    // frames: the RX mix, filled as a sender would, laid one per slot
    std::vector<uint64_t> off(nfr + 1);
    const uint64_t bytes = aipstack_synth_frames_host(nullptr, off.data(), nfr, 42, 1460);
    std::vector<unsigned char> compact(bytes);
    aipstack_synth_frames_host(compact.data(), off.data(), nfr, 42, 1460);
    std::vector<uint8_t> st(nfr);
    oracle_tx_fill_batch(compact.data(), off.data(), nfr, st.data());
    std::vector<unsigned char> ring(nfr * slot, 0x5A);
    std::vector<uint32_t> len(nfr);
    uint64_t frame_bytes = 0;
    for (uint64_t i = 0; i < nfr; ++i) {
        len[i] = (uint32_t)(off[i + 1] - off[i]);
        std::memcpy(ring.data() + i * slot, compact.data() + off[i], len[i]);
        frame_bytes += len[i];
    }
    std::vector<uint8_t> verdict(nfr, 0xEE), want(nfr);
    oracle_rx_verify_slotted(ring.data(), slot, len.data(), nfr, want.data());

    aipstack_chksum_engine *eng = nullptr;
    if (aipstack_chksum_engine_create(0, 64ull << 20, 4, &eng) != 0) return 1;
    if (aipstack_chksum_engine_register(eng, ring.data(), ring.size()) != 0) return 1;
    std::vector<uint64_t> ticket(R, 0);
    auto lap = [&](uint64_t laps) {
        for (uint64_t k = 0; k < laps * R; ++k) {
            const uint64_t r = k % R;
            if (ticket[r] && aipstack_chksum_engine_wait(eng, ticket[r]) != 0) return false;
            if (aipstack_chksum_engine_submit_rx_verify_slotted(
                    eng, ring.data() + r * B * slot, slot, len.data() + r * B, B,
                    verdict.data() + r * B, &ticket[r]) != 0)
                return false;
        }
        return true;
    };
    auto drain = [&]() {
        for (uint64_t r = 0; r < R; ++r)
            if (ticket[r] && aipstack_chksum_engine_wait(eng, ticket[r]) != 0) return false;
        return true;
    };
    // warm-up, then K batches (at least 2 GiB of frames or 4096 batches, whichever is less)
    if (!lap(2) || !drain()) return 1;
    uint64_t laps = (uint64_t)(2.0 * (1ull << 30) / (double)frame_bytes) + 1;
    if (laps * R > 4096) laps = 4096 / R;
    if (laps < 2) laps = 2;
    const auto t0 = std::chrono::steady_clock::now();
    if (!lap(laps) || !drain()) return 1;
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const bool ok = verdict == want;
    const double batches = (double)(laps * R);
    std::printf("{\"slots_per_batch\": %llu, \"regions_in_flight\": %llu, \"batches\": %.0f, "
                "\"us_per_batch\": %.2f, \"Mframes_per_s\": %.2f, \"GiBps_frames\": %.2f, "
                "\"parity\": \"%s\"}\n",
                (unsigned long long)B, (unsigned long long)R - 1, batches, s / batches * 1e6,
                batches * (double)B / s / 1e6, batches * (double)frame_bytes / R / s / (1 << 30),
                ok ? "bit-exact (last lap, every region vs frame oracle)" : "MISMATCH");
    aipstack_chksum_engine_unregister(eng, ring.data());
    aipstack_chksum_engine_destroy(eng);
    return ok ? 0 : 2;
}

int main(int argc, char **argv) {
    std::vector<uint64_t> sizes;
    uint64_t regions = 8;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "-r") && i + 1 < argc) {
            regions = std::strtoull(argv[++i], nullptr, 10);
            if (regions < 1) regions = 1;
            continue;
        }
        sizes.push_back(std::strtoull(argv[i], nullptr, 10));
    }
    if (sizes.empty()) sizes = {256, 1024, 4096, 16384, 65536};
    int rc = 0;
    for (uint64_t b : sizes) rc |= run(b, regions);
    return rc;
}
