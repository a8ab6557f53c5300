// A TAP-style receive loop through the host engine, from C++ (tools only).
//
// Ring mode (default): a registered ring of R regions x B slots of 2048 B holding raw frames
// (the RX mix of the bench, Tx-filled so that most verify), driven the way a receive loop would
// drive it -- region r is submitted for Rx verify (..._submit_rx_verify_slotted) and only waited
// for when the loop comes back to r, so R - 1 batches stay in flight. Times K batches per batch
// size B and checks the verdicts of every region of the last lap against the frame oracle.
//
// Socket mode (-s, round 4): the frames move through file descriptors, as the TAP driver moves
// them (reference tap/linux/TapDeviceLinux.cpp:142-186 reads one frame per read() into its
// receive buffer; :109-127 write()s one frame per send):
//   * a producer thread write()s the RX mix, one frame per write(), into a
//     socketpair(AF_UNIX, SOCK_SEQPACKET); the loop read()s one frame per 2048-B slot of a
//     registered receive ring and submits Rx verify for each region of B frames; a region's
//     verdicts are checked against the frame oracle when the loop comes back to it;
//   * the send side builds B raw frames per region of a registered send ring (copied from the
//     frame templates, as the stack writes its headers), submits the Tx fill, and when the loop
//     comes back to the region write()s each filled frame into a second socketpair, where a
//     consumer thread read()s them and compares each with the oracle's fill.
// Every syscall is inside the timed loop: us per batch = one Rx batch + one Tx batch of B frames.
//
// -g N: the same through an engine group of N engines on device 0 (group tickets).
//
//   tools/build/ring_loop [-r R] [-g N] [-s] [B ...]  (default R = 8, B = 256 1024 4096 16384
//                                                     65536; R = 1: one batch at a time)
// Prints one JSON line per B.
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "aipstack_amd/chksum.h"
#include "aipstack_amd/synth.h"
#include "frame_oracle.h"

namespace {

constexpr uint64_t kSlot = 2048;

// One engine or an engine group behind the same three calls.
struct Driver {
    aipstack_chksum_engine *eng = nullptr;
    aipstack_chksum_engine_group *grp = nullptr;

    bool open(int engines) {
        if (engines <= 0) return aipstack_chksum_engine_create(0, 64ull << 20, 4, &eng) == 0;
        std::vector<int> devs((size_t)engines, 0);
        return aipstack_chksum_engine_group_create(devs.data(), engines, 64ull << 20, 4, &grp) == 0;
    }
    void close() {
        if (eng) aipstack_chksum_engine_destroy(eng);
        if (grp) aipstack_chksum_engine_group_destroy(grp);
    }
    int reg(void *p, uint64_t n) {
        return eng ? aipstack_chksum_engine_register(eng, p, n)
                   : aipstack_chksum_engine_group_register(grp, p, n);
    }
    int unreg(void *p) {
        return eng ? aipstack_chksum_engine_unregister(eng, p)
                   : aipstack_chksum_engine_group_unregister(grp, p);
    }
    int rx(const void *base, const uint32_t *len, uint64_t n, uint8_t *out, uint64_t *t) {
        return eng ? aipstack_chksum_engine_submit_rx_verify_slotted(eng, base, kSlot, len, n, out, t)
                   : aipstack_chksum_engine_group_submit_rx_verify_slotted(grp, base, kSlot, len, n,
                                                                           out, t);
    }
    int tx(void *base, const uint32_t *len, uint64_t n, uint8_t *st, uint64_t *t) {
        return eng ? aipstack_chksum_engine_submit_tx_fill_slotted(eng, base, kSlot, len, n, st, t)
                   : aipstack_chksum_engine_group_submit_tx_fill_slotted(grp, base, kSlot, len, n,
                                                                         st, t);
    }
    int wait(uint64_t t) {
        return eng ? aipstack_chksum_engine_wait(eng, t)
                   : aipstack_chksum_engine_group_wait(grp, t, nullptr);
    }
};

// The RX mix: nfr frames, raw (as a sender builds them) and Tx-filled (as they arrive).
struct Frames {
    std::vector<uint64_t> off;
    std::vector<unsigned char> raw, filled;
    std::vector<uint8_t> verdict;  // the oracle's Rx verdict of each filled frame
    uint64_t bytes = 0;
    explicit Frames(uint64_t nfr) : off(nfr + 1), verdict(nfr) {
        bytes = aipstack_synth_frames_host(nullptr, off.data(), nfr, 42, 1460);
        raw.resize(bytes);
        aipstack_synth_frames_host(raw.data(), off.data(), nfr, 42, 1460);
        filled = raw;
        std::vector<uint8_t> st(nfr);
        oracle_tx_fill_batch(filled.data(), off.data(), nfr, st.data());
        oracle_rx_verify_batch(filled.data(), off.data(), nfr, verdict.data());
    }
    uint32_t len(uint64_t i) const { return (uint32_t)(off[i + 1] - off[i]); }
};

const char *mode_name(int engines) { return engines > 0 ? "group" : "engine"; }

int run_ring(uint64_t B, uint64_t R, int engines) {
    const uint64_t nfr = R * B;
    Frames fr(nfr);
    std::vector<unsigned char> ring(nfr * kSlot, 0x5A);
    std::vector<uint32_t> len(nfr);
    for (uint64_t i = 0; i < nfr; ++i) {
        len[i] = fr.len(i);
        std::memcpy(ring.data() + i * kSlot, fr.filled.data() + fr.off[i], len[i]);
    }
    std::vector<uint8_t> verdict(nfr, 0xEE);
    Driver d;
    if (!d.open(engines) || d.reg(ring.data(), ring.size()) != 0) return 1;
    std::vector<uint64_t> ticket(R, 0);
    auto lap = [&](uint64_t laps) {
        for (uint64_t k = 0; k < laps * R; ++k) {
            const uint64_t r = k % R;
            if (ticket[r] && d.wait(ticket[r]) != 0) return false;
            if (d.rx(ring.data() + r * B * kSlot, len.data() + r * B, B, verdict.data() + r * B,
                     &ticket[r]) != 0)
                return false;
        }
        return true;
    };
    auto drain = [&]() {
        for (uint64_t r = 0; r < R; ++r)
            if (ticket[r] && d.wait(ticket[r]) != 0) return false;
        return true;
    };
    // warm-up, then K batches (at least 2 GiB of frames or 4096 batches, whichever is less)
    if (!lap(2) || !drain()) return 1;
    uint64_t laps = (uint64_t)(2.0 * (1ull << 30) / (double)fr.bytes) + 1;
    if (laps * R > 4096) laps = 4096 / R;
    if (laps < 2) laps = 2;
    const auto t0 = std::chrono::steady_clock::now();
    if (!lap(laps) || !drain()) return 1;
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const bool ok = verdict == fr.verdict;
    const double batches = (double)(laps * R);
    std::printf("{\"mode\": \"ring\", \"driver\": \"%s\", \"engines\": %d, \"slots_per_batch\": %llu, "
                "\"regions_in_flight\": %llu, \"batches\": %.0f, \"us_per_batch\": %.2f, "
                "\"Mframes_per_s\": %.2f, \"GiBps_frames\": %.2f, \"parity\": \"%s\"}\n",
                mode_name(engines), engines > 0 ? engines : 1, (unsigned long long)B,
                (unsigned long long)R - 1, batches, s / batches * 1e6,
                batches * (double)B / s / 1e6, batches * (double)fr.bytes / R / s / (1 << 30),
                ok ? "bit-exact (last lap, every region vs frame oracle)" : "MISMATCH");
    d.unreg(ring.data());
    d.close();
    return ok ? 0 : 2;
}

// Socket mode: see the file comment.
int run_socket(uint64_t B, uint64_t R, int engines) {
    const uint64_t nfr = R * B;  // frame templates, cycled
    Frames fr(nfr);
    int rxp[2], txp[2];
    if (socketpair(AF_UNIX, SOCK_SEQPACKET, 0, rxp) != 0 ||
        socketpair(AF_UNIX, SOCK_SEQPACKET, 0, txp) != 0) {
        std::perror("socketpair");
        return 1;
    }
    uint64_t laps = (uint64_t)(1.0 * (1ull << 30) / (double)fr.bytes) + 1;
    if (laps * R > 2048) laps = 2048 / R;
    if (laps < 3) laps = 3;
    const uint64_t total = laps * R * B;  // frames each way
    // producer: the wire side of the receive path, one frame per write()
    std::thread producer([&] {
        for (uint64_t i = 0; i < total; ++i) {
            const uint64_t f = i % nfr;
            if (write(rxp[1], fr.filled.data() + fr.off[f], fr.len(f)) != (ssize_t)fr.len(f)) {
                std::perror("producer write");
                return;
            }
        }
    });
    // consumer: the wire side of the send path, one frame per read(), checked against the fill
    std::atomic<uint64_t> tx_bad{0}, tx_seen{0};
    std::thread consumer([&] {
        std::vector<unsigned char> buf(kSlot);
        for (uint64_t i = 0; i < total; ++i) {
            const ssize_t got = read(txp[0], buf.data(), buf.size());
            const uint64_t f = i % nfr;
            if (got != (ssize_t)fr.len(f) ||
                std::memcmp(buf.data(), fr.filled.data() + fr.off[f], fr.len(f)) != 0)
                tx_bad.fetch_add(1);
            tx_seen.fetch_add(1);
        }
    });
    std::vector<unsigned char> rx_ring(R * B * kSlot, 0x5A), tx_ring(R * B * kSlot, 0xA5);
    std::vector<uint32_t> rx_len(R * B), tx_len(R * B);
    std::vector<uint8_t> verdict(R * B), status(R * B);
    std::vector<uint64_t> rx_first(R, 0), tx_first(R, 0);  // first frame id in each region
    std::vector<uint64_t> rx_t(R, 0), tx_t(R, 0);
    uint64_t rx_bad = 0, rx_next = 0, tx_next = 0;
    bool fail = false;
    Driver d;
    if (!d.open(engines) || d.reg(rx_ring.data(), rx_ring.size()) != 0 ||
        d.reg(tx_ring.data(), tx_ring.size()) != 0)
        return 1;
    auto step = [&](uint64_t r) {
        unsigned char *rxr = rx_ring.data() + r * B * kSlot;
        unsigned char *txr = tx_ring.data() + r * B * kSlot;
        // receive: the region's previous batch done -> check its verdicts, refill it by read()
        if (rx_t[r]) {
            if (d.wait(rx_t[r]) != 0) fail = true;
            for (uint64_t j = 0; j < B; ++j)
                rx_bad += verdict[r * B + j] != fr.verdict[(rx_first[r] + j) % nfr];
        }
        rx_first[r] = rx_next;
        for (uint64_t j = 0; j < B; ++j) {
            const ssize_t got = read(rxp[0], rxr + j * kSlot, kSlot);
            if (got < 0) fail = true;
            rx_len[r * B + j] = got > 0 ? (uint32_t)got : 0u;
        }
        rx_next += B;
        if (d.rx(rxr, rx_len.data() + r * B, B, verdict.data() + r * B, &rx_t[r]) != 0) fail = true;
        // send: the region's previous batch filled -> write() its frames, build the next ones
        if (tx_t[r]) {
            if (d.wait(tx_t[r]) != 0) fail = true;
            for (uint64_t j = 0; j < B; ++j)
                if (write(txp[1], txr + j * kSlot, tx_len[r * B + j]) != (ssize_t)tx_len[r * B + j])
                    fail = true;
        }
        tx_first[r] = tx_next;
        for (uint64_t j = 0; j < B; ++j) {
            const uint64_t f = (tx_next + j) % nfr;
            tx_len[r * B + j] = fr.len(f);
            std::memcpy(txr + j * kSlot, fr.raw.data() + fr.off[f], fr.len(f));
        }
        tx_next += B;
        if (d.tx(txr, tx_len.data() + r * B, B, status.data() + r * B, &tx_t[r]) != 0) fail = true;
    };
    const uint64_t steps = laps * R;
    const uint64_t warm = R;  // the first lap fills the pipeline, untimed
    std::chrono::steady_clock::time_point t0;
    for (uint64_t k = 0; k < steps && !fail; ++k) {
        if (k == warm) t0 = std::chrono::steady_clock::now();
        step(k % R);
    }
    // the last lap's batches: verdicts checked, filled frames sent
    for (uint64_t r = 0; r < R && !fail; ++r) {
        if (d.wait(rx_t[r]) != 0) fail = true;
        for (uint64_t j = 0; j < B; ++j)
            rx_bad += verdict[r * B + j] != fr.verdict[(rx_first[r] + j) % nfr];
        if (d.wait(tx_t[r]) != 0) fail = true;
        for (uint64_t j = 0; j < B; ++j)
            (void)!write(txp[1], tx_ring.data() + (r * B + j) * kSlot, tx_len[r * B + j]);
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    producer.join();
    consumer.join();
    const bool ok = !fail && rx_bad == 0 && tx_bad == 0 && tx_seen == total;
    const double batches = (double)(steps - warm);
    std::printf("{\"mode\": \"socket\", \"driver\": \"%s\", \"engines\": %d, \"frames_per_batch\": "
                "%llu, \"regions\": %llu, \"batches\": %.0f, \"us_per_batch_rx_plus_tx\": %.2f, "
                "\"Mframes_per_s_each_way\": %.3f, \"GiBps_frames_each_way\": %.3f, \"rx_bad\": %llu, "
                "\"tx_bad\": %llu, \"parity\": \"%s\"}\n",
                mode_name(engines), engines > 0 ? engines : 1, (unsigned long long)B,
                (unsigned long long)R, batches, s / batches * 1e6, batches * (double)B / s / 1e6,
                batches * (double)fr.bytes / (double)R / s / (1 << 30), (unsigned long long)rx_bad,
                (unsigned long long)tx_bad.load(),
                ok ? "bit-exact (every Rx verdict and every sent frame vs frame oracle)" : "MISMATCH");
    d.unreg(rx_ring.data());
    d.unreg(tx_ring.data());
    d.close();
    for (int fd : {rxp[0], rxp[1], txp[0], txp[1]}) ::close(fd);
    return ok ? 0 : 2;
}

}  // namespace

int main(int argc, char **argv) {
    std::vector<uint64_t> sizes;
    uint64_t regions = 8;
    int engines = 0;
    bool socket = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "-r") && i + 1 < argc) {
            regions = std::strtoull(argv[++i], nullptr, 10);
            if (regions < 1) regions = 1;
            continue;
        }
        if (!std::strcmp(argv[i], "-g") && i + 1 < argc) {
            engines = std::atoi(argv[++i]);
            continue;
        }
        if (!std::strcmp(argv[i], "-s")) {
            socket = true;
            continue;
        }
        sizes.push_back(std::strtoull(argv[i], nullptr, 10));
    }
    if (sizes.empty()) sizes = socket ? std::vector<uint64_t>{64, 256, 1024, 4096}
                                      : std::vector<uint64_t>{256, 1024, 4096, 16384, 65536};
    int rc = 0;
    for (uint64_t b : sizes) rc |= socket ? run_socket(b, regions, engines) : run_ring(b, regions, engines);
    return rc;
}
