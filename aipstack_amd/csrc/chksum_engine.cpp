// aipstack_amd -- host-memory streaming engine.
//
// The reference's packet path starts and ends in host memory: a TAP read() fills one host
// buffer per frame (reference tap/linux/TapDeviceLinux.cpp:156-178) and write() sends one
// (:122-127). This engine checksums batches that live in HOST memory and returns the
// results to HOST memory, overlapping the PCIe transfers with the kernels:
//
//   chunk i (a run of whole packets, <= chunk_bytes) on stream i % nstreams:
//     registered input:  batch kernel reading the caller's page-locked bytes over the link
//                        (offsets / lengths and results in the slot's pinned staging)
//     pageable input:    CPU copy into pinned staging -> H2D -> batch kernel -> D2H
//
// Host buffers registered with aipstack_chksum_engine_register() (page-locked via
// hipHostRegister, as a TAP/socket ring would be once at start-up) are read in place by the
// kernels (round 3: as fast as a DMA for back-to-back packets, ~1.85x for ring slots, whose
// slack never crosses the link, and two DMA operations fewer per small batch; the DMA path
// stays behind tuning "engine_zero_copy" = 0). Other host memory is first copied on the CPU
// into pinned staging (the "pageable" path).
//
// Batches are submitted (aipstack_chksum_engine_submit_*: enqueue and return a ticket) and
// completed (_poll: non-blocking, _wait: blocking); the synchronous calls are submit +
// wait. A receive loop can therefore read() the next frames into its ring while the GPU
// works on the previous batch. Each slot (stream + staging) carries the ticket of the
// batch piece it holds; a submit that needs a busy slot first completes that slot's piece
// (back-pressure after nstreams pieces in flight).
//
// Errors are kept per ticket: a piece that fails (at enqueue or at completion, whichever
// call completes it) records its status against its own batch's ticket until that ticket
// is completed by _poll / _wait, so a failure is never reported for, nor hidden from,
// another batch. Destroy completes every piece still in flight as _wait would (results
// delivered, Tx fields applied) before it frees anything.
//
// Locking (round 4): `submit_mu` serialises the submits (and register / unregister, which
// change what a submit reads); `mu` guards the slots' bookkeeping, the failure records and
// the ticket counter, and is only ever held for short bookkeeping -- never while the host
// waits for a GPU piece (a back-pressured submit, _wait), copies pageable input into staging
// or waits for the Tx applier. So _poll from the receive loop's other thread always answers
// at once.
//
// Host threads (round 4): a persistent pool per engine (host_threads.h), pinned with the
// applier thread to the CPUs next to the device; the pinned staging is allocated from those
// CPUs too, so that its pages sit on the device's NUMA node.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "aipstack_amd/chksum.h"
#include "chksum_internal.h"
#include "host_threads.h"

using namespace aipstack_amd;

namespace {

struct Slot {
    hipStream_t stream = nullptr;
    void *d_bytes = nullptr;       // device staging for packet bytes
    uint64_t *d_off = nullptr;     // device staging for CSR offsets
    uint16_t *d_out = nullptr;     // device results (up to 8 bytes per packet)
    void *h_stage = nullptr;       // pinned host staging (pageable inputs)
    uint64_t *h_off = nullptr;     // pinned host staging for rebased offsets
    uint16_t *h_out = nullptr;     // pinned host results
    uint64_t *dh_off = nullptr;    // device addresses of h_off / h_out (mapped pinned memory)
    uint16_t *dh_out = nullptr;
    // What this piece's kernel reads its offsets / lengths from and writes its results to:
    // d_off / d_out (copied H2D / D2H around the kernel), or, for a small piece, the pinned
    // staging itself through dh_off / dh_out (no copies: fewer DMA ops per small batch)
    uint64_t *k_off = nullptr;
    uint16_t *k_out = nullptr;
    void *k_bytes = nullptr;  // the packet bytes as the kernel reads them: d_bytes, or the
                              // caller's registered memory itself (zero-copy pieces), or the
                              // pinned staging (pageable ring slots, frame bytes only)
    char *dh_stage = nullptr;  // device address of h_stage
    bool zero_copy = false;
    bool host_bytes = false;  // k_bytes is page-locked host memory the kernel reads over the link
    hipEvent_t done = nullptr;
    bool busy = false;
    void *user_out = nullptr;      // where h_out goes once the slot completes
    uint64_t count = 0;
    uint32_t out_elem = 2;         // bytes per result: 2 (checksums), 1 (Rx verdicts), 8 (Tx)
    // Tx fill: instead of copying the results out, apply the piece's records to the
    // caller's frames in host memory (frames + offs[i], i < count) and statuses
    char *tx_frames = nullptr;
    const uint64_t *tx_offs = nullptr;  // frame i at tx_frames + tx_offs[i] (CSR), or
    uint64_t tx_stride = 0;             // at tx_frames + i * tx_stride (ring slots)
    uint8_t *tx_status = nullptr;
    uint64_t ticket = 0;           // batch this slot's piece belongs to
    uint64_t seq = 0;              // piece number within the engine (1, 2, ...)
};

struct Region {
    const char *p;
    uint64_t bytes;
    bool owned = true;  // registered by this engine (unregistered by it); else adopted
    const char *dev = nullptr;  // the region as the device addresses it (mapped), or null
};

// A completed Tx piece's records, applied to the caller's frames by the engine's applier
// thread while the slot already carries the next piece.
struct ApplyJob {
    std::vector<uint64_t> rec;
    char *frames;
    const uint64_t *offs;
    uint64_t stride;
    uint8_t *status;
    uint64_t ticket;
};

// One background thread per engine (started with the first Tx piece): the host-side record
// apply of a Tx piece (up to ~0.3 ms for 64 MiB of frames) used to run on the submitting
// thread, inside the drain that frees a slot for the next piece, and stalled the pipeline.
struct Applier {
    std::mutex mu;
    std::condition_variable work, done;
    std::deque<ApplyJob> queue;
    std::map<uint64_t, int> pending;  // ticket -> pieces queued or being applied
    bool stop = false;
    std::thread thread;
    std::atomic<uint64_t> *busy_ns = nullptr;  // engine stats (AIPSTACK_ENGINE_STATS), or null
};

// Where an engine's host time goes (AIPSTACK_ENGINE_STATS=1: one JSON line on stderr at
// destroy; the counters cost nothing otherwise). Nanoseconds, summed over the engine's life.
struct Stats {
    bool on = false;
    std::atomic<uint64_t> enqueue{0};     // inside the submit calls
    std::atomic<uint64_t> slot_wait{0};   // of which: waiting for a slot's previous piece
    std::atomic<uint64_t> rec_copy{0};    // of which: Tx records copied out of a slot
    std::atomic<uint64_t> stage{0};       // of which: pageable input staged by the CPU
    std::atomic<uint64_t> apply{0};       // applier thread: Tx records applied
    std::atomic<uint64_t> apply_wait{0};  // completion calls waiting for the applier
    std::atomic<uint64_t> complete{0};    // inside the poll / wait calls
    uint64_t created = 0;
    std::atomic<uint64_t> pieces{0};
};

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Adds the time since construction to a counter, when stats are on.
struct Span_ns {
    std::atomic<uint64_t> *to;
    uint64_t t0;
    Span_ns(const Stats &st, std::atomic<uint64_t> &c) : to(st.on ? &c : nullptr), t0(to ? now_ns() : 0) {}
    ~Span_ns() {
        if (to) to->fetch_add(now_ns() - t0, std::memory_order_relaxed);
    }
};

}  // namespace

struct aipstack_chksum_engine {
    int device = 0;
    uint64_t chunk_bytes = 0;
    uint64_t chunk_packets = 0;
    bool slot_rows = true;  // ring slots: copy each slot's used prefix only (2-D copy)
    // Zero copy (round 3): a kernel reads registered input where it lies, over the
    // link, instead of a DMA into d_bytes first -- the same rate for back-to-back packets,
    // ~1.85x for ring slots (only the frames' bytes cross, not the slack), and two fewer DMA
    // operations per small batch. Offsets / lengths and results then stay in the pinned
    // staging too; so they do for small pieces of pageable input.
    bool zero_copy_bytes = true;
    uint64_t zero_copy_max = 65536;  // metadata in pinned staging for pieces up to this
    bool pageable_rows = true;  // pageable ring slots: frame bytes staged, read in place
    std::vector<Slot> slots;
    std::vector<Region> registered;  // changed under submit_mu (and mu)
    size_t next_slot = 0;      // round robin over the slots, across batches (submit_mu)
    uint64_t next_ticket = 1;  // tickets are never 0 (mu)
    uint64_t submitting = 0;   // the ticket whose submit is running (mu): not complete yet
    uint64_t pieces = 0;       // pieces enqueued so far (Slot::seq; submit_mu)
    // tickets with a failed piece -> the first failure's status, until the ticket is
    // completed (poll / wait) or the engine is destroyed
    std::map<uint64_t, int> failed;
    std::mutex submit_mu;  // serialises the submits, register and unregister
    std::mutex mu;         // the slots' bookkeeping, failures, tickets: short sections only
    std::unique_ptr<Applier> applier;  // Tx record apply, off the submitting thread
    DeviceLocality loc;    // the device's NUMA node and local CPUs
    HostPool pool;         // pinned host workers: staging copies, Tx record applies
    Stats stats;
};

namespace {

const Region *find_registered(const aipstack_chksum_engine *e, const void *p, uint64_t bytes) {
    const char *c = static_cast<const char *>(p);
    for (const Region &r : e->registered)
        if (c >= r.p && c + bytes <= r.p + r.bytes) return &r;
    return nullptr;
}

// The device address of a page-locked host region (null if the runtime gives none).
const char *mapped_address(const void *host_ptr) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<void *>(host_ptr), 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<const char *>(d);
}

#ifdef AIPSTACK_ENGINE_FAULT_INJECTION
// Test builds only (tests/cpp): make chosen pieces fail, at their launch or at their
// completion, as a HIP error would. Bit k-1 of a mask = piece k (Slot::seq), k <= 64.
std::atomic<uint64_t> g_fail_at_launch{0}, g_fail_at_completion{0};
std::atomic<uint64_t> g_wait_delay_us{0};  // _wait and a back-pressured submit sleep this
                                           // long outside the engine lock
std::atomic<const aipstack_chksum_engine *> g_fail_engine{nullptr};  // null: every engine
bool injected(const aipstack_chksum_engine *e, const std::atomic<uint64_t> &mask, uint64_t seq) {
    const aipstack_chksum_engine *only = g_fail_engine.load();
    return (!only || only == e) && seq >= 1 && seq <= 64 && ((mask.load() >> (seq - 1)) & 1u);
}
#endif

void record_failure(aipstack_chksum_engine *e, uint64_t ticket, int status) {
    e->failed.emplace(ticket, status);  // the first failure of a batch is kept
}

void stop_applier(aipstack_chksum_engine *e);

void release(aipstack_chksum_engine *e) {
    stop_applier(e);  // after every queued apply (destroy drains first)
    for (Slot &s : e->slots) {
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (s.d_bytes) (void)hipFree(s.d_bytes);
        if (s.d_off) (void)hipFree(s.d_off);
        if (s.d_out) (void)hipFree(s.d_out);
        if (s.h_stage) (void)hipHostFree(s.h_stage);
        if (s.h_off) (void)hipHostFree(s.h_off);
        if (s.h_out) (void)hipHostFree(s.h_out);
        if (s.done) (void)hipEventDestroy(s.done);
        if (s.stream) (void)hipStreamDestroy(s.stream);
    }
    for (const Region &r : e->registered)
        if (r.owned) (void)hipHostUnregister(const_cast<char *>(r.p));
}

// Host threads the engine uses for one piece's Tx records / pageable staging copy, the caller
// included (AIPSTACK_ENGINE_HOST_THREADS, default 8; read once): the pool holds one fewer.
unsigned host_threads_cap() {
    static const unsigned cap = [] {
        const char *v = std::getenv("AIPSTACK_ENGINE_HOST_THREADS");
        const int t = v ? std::atoi(v) : 8;
        return (unsigned)std::min(std::max(t, 1), 64);
    }();
    return cap;
}

// Parts a piece's host work is split into: one per `per_part_min` units, at most the pool's
// threads plus the caller.
unsigned host_parts(const HostPool &pool, uint64_t units, uint64_t per_part_min) {
    return (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>(units / per_part_min, pool.workers() + 1u));
}

// Pageable input into pinned staging: one core copies ~20 GB/s, below the PCIe link the
// DMA then feeds, so large pieces are copied by the pool over disjoint 4 KiB-aligned
// ranges (the previous piece's DMA runs meanwhile).
void stage_copy(HostPool &pool, void *dst, const void *src, uint64_t bytes) {
    const unsigned nt = host_parts(pool, bytes, 4ull << 20);
    const uint64_t per = ((bytes + nt - 1) / nt + 4095) & ~4095ull;
    pool.run(nt, [=](unsigned t) {
        const uint64_t lo = std::min((uint64_t)t * per, bytes);
        const uint64_t len = std::min(per, bytes - lo);
        std::memcpy(static_cast<char *>(dst) + lo, static_cast<const char *>(src) + lo, len);
    });
}

// Tx fill from host memory: write the checksum fields (big-endian) of frames [lo, hi) of a
// completed piece into the caller's frames, and their statuses (record layout: chksum.h,
// aipstack_chksum_tx_fill_records).
void apply_tx_range(const uint64_t *rec, char *frames, const uint64_t *offs, uint64_t stride,
                    uint8_t *status, uint64_t lo, uint64_t hi) {
    // every frame's field line is a cache miss (the device read the frames, not this core):
    // the lines a few frames ahead are requested while this one is written
    constexpr uint64_t kAhead = 16;
    for (uint64_t i = lo; i < hi; ++i) {
        if (i + kAhead < hi) {
            const char *g = frames + (offs ? offs[i + kAhead] : (i + kAhead) * stride);
            __builtin_prefetch(g + 24, 1, 0);  // the IPv4 checksum
            __builtin_prefetch(g + 51, 1, 0);  // TCP's (UDP's and ICMP's share a line with one)
        }
        const uint64_t x = rec[i];
        char *f = frames + (offs ? offs[i] : i * stride);
        status[i] = (uint8_t)(x >> 48);
        if ((x >> 40) & 1u) {
            f[24] = (char)((x >> 8) & 0xFFu);
            f[25] = (char)(x & 0xFFu);
        }
        if ((x >> 41) & 1u) {
            const uint32_t fo = (uint32_t)(x >> 32) & 0xFFu;
            f[fo] = (char)((x >> 24) & 0xFFu);
            f[fo + 1] = (char)((x >> 16) & 0xFFu);
        }
    }
}

// A piece's frames are spread over up to 64 MiB of host memory: every frame is a cache miss,
// so a large piece is applied by the pool (16 Ki frames and more per part).
void apply_tx_records(HostPool &pool, const uint64_t *rec, char *frames, const uint64_t *offs,
                      uint64_t stride, uint8_t *status, uint64_t count) {
    const unsigned nt = host_parts(pool, count, 16384);
    const uint64_t per = (count + nt - 1) / nt;
    pool.run(nt, [=](unsigned t) {
        const uint64_t lo = std::min((uint64_t)t * per, count);
        apply_tx_range(rec, frames, offs, stride, status, lo, std::min(count, lo + per));
    });
}

void applier_loop(Applier *a, HostPool *pool, const std::vector<int> *cpus) {
    pin_current_thread(*cpus);
    std::unique_lock<std::mutex> lock(a->mu);
    for (;;) {
        a->work.wait(lock, [a] { return a->stop || !a->queue.empty(); });
        if (a->queue.empty()) return;  // stop, and nothing left to apply
        ApplyJob job = std::move(a->queue.front());
        a->queue.pop_front();
        lock.unlock();
        const uint64_t t0 = a->busy_ns ? now_ns() : 0;
        apply_tx_records(*pool, job.rec.data(), job.frames, job.offs, job.stride, job.status,
                         job.rec.size());
        if (a->busy_ns) a->busy_ns->fetch_add(now_ns() - t0, std::memory_order_relaxed);
        lock.lock();
        if (--a->pending[job.ticket] == 0) a->pending.erase(job.ticket);
        a->done.notify_all();
    }
}

// The applier starts with the engine (its thread pinned beside the pool's).
void start_applier(aipstack_chksum_engine *e) {
    e->applier.reset(new Applier);
    if (e->stats.on) e->applier->busy_ns = &e->stats.apply;
    e->applier->thread = std::thread(applier_loop, e->applier.get(), &e->pool, &e->loc.cpus);
}

void queue_apply(aipstack_chksum_engine *e, ApplyJob &&job) {
    Applier *a = e->applier.get();
    std::lock_guard<std::mutex> lock(a->mu);
    ++a->pending[job.ticket];
    a->queue.push_back(std::move(job));
    a->work.notify_one();
}

// Whether ticket's records (every ticket's for 0) are still being applied; with `blocking`,
// waits until they are not (callers hold no engine lock then: the applier may take ~0.3 ms
// per queued 64 MiB piece).
bool applies_pending(aipstack_chksum_engine *e, uint64_t ticket, bool blocking) {
    Applier *a = e->applier.get();
    if (!a) return false;
    Span_ns timed(e->stats, e->stats.apply_wait);
    std::unique_lock<std::mutex> lock(a->mu);
    auto busy = [a, ticket] {
        return ticket == 0 ? !a->pending.empty() : a->pending.count(ticket) != 0;
    };
    if (blocking) a->done.wait(lock, [&] { return !busy(); });
    return busy();
}

void stop_applier(aipstack_chksum_engine *e) {
    Applier *a = e->applier.get();
    if (!a) return;
    {
        std::lock_guard<std::mutex> lock(a->mu);
        a->stop = true;
        a->work.notify_one();
    }
    a->thread.join();
    e->applier.reset();
}

// Complete slot s: wait for it (blocking) or only if it is done (non-blocking: returns
// 1 while it is still running), then hand its results to the caller. A HIP error is
// recorded against the slot's ticket.
int drain(aipstack_chksum_engine *e, Slot &s, bool blocking = true) {
    if (!s.busy) return AIPSTACK_CHKSUM_OK;
    hipError_t r;
    if (blocking) {
        Span_ns timed(e->stats, e->stats.slot_wait);
        r = hipEventSynchronize(s.done);
    } else {
        r = hipEventQuery(s.done);
        if (r == hipErrorNotReady) return 1;
    }
#ifdef AIPSTACK_ENGINE_FAULT_INJECTION
    if (r == hipSuccess && injected(e, g_fail_at_completion, s.seq)) r = hipErrorLaunchFailure;
#endif
    const int st = check_hip(r);
    if (st == AIPSTACK_CHKSUM_OK && s.tx_frames) {
        // the records leave the slot (copied), the applier writes the fields
        const uint64_t *rec = reinterpret_cast<const uint64_t *>(s.h_out);
        Span_ns timed(e->stats, e->stats.rec_copy);
        queue_apply(e, ApplyJob{std::vector<uint64_t>(rec, rec + s.count), s.tx_frames,
                                s.tx_offs, s.tx_stride, s.tx_status, s.ticket});
    } else if (st == AIPSTACK_CHKSUM_OK) {
        std::memcpy(s.user_out, s.h_out, s.count * s.out_elem);
    } else {
        record_failure(e, s.ticket, st);
    }
    s.busy = false;
    return st;
}

// A piece's host bytes: `bytes` from `src`, or -- when width is set and the bytes are
// registered -- rows of `pitch` bytes of which only the first `width` travel (ring slots:
// the slack after the longest frame of the piece stays behind; the device copy keeps the
// slot layout). Pageable rows are staged and sent whole: a per-row CPU copy runs slower
// than the bulk one, and the bulk copy already keeps up with the link.
struct Span {
    const char *src = nullptr;
    uint64_t bytes = 0;
    uint64_t pitch = 0, width = 0;
    const uint32_t *row_len = nullptr;  // ring slots: each row's frame length
};

// Pageable ring slots into pinned staging: each slot's frame bytes only (row r's first
// row_len[r] bytes, at the same pitch), by up to host_threads_cap() threads; the kernel then
// reads the staging in place, so neither the CPU nor the link moves any slack.
void stage_copy_frames(HostPool &pool, void *dst, const void *src, uint64_t pitch,
                       const uint32_t *row_len, uint64_t rows) {
    const unsigned nt = host_parts(pool, rows, 2048);
    const uint64_t per = (rows + nt - 1) / nt;
    pool.run(nt, [=](unsigned t) {
        const uint64_t hi = std::min(rows, (uint64_t)(t + 1) * per);
        for (uint64_t r = (uint64_t)t * per; r < hi; ++r)
            std::memcpy(static_cast<char *>(dst) + r * pitch,
                        static_cast<const char *>(src) + r * pitch, row_len[r]);
    });
}

// Enqueue one batch as chunks over the slots. chunker(i0, &i1, &span) describes chunk
// [i0, i1) of packets and its bytes in host memory; launch(slot, i0, i1) enqueues its
// kernel, whose results (elem bytes per packet) land in the slot's d_out. Returns the
// status of the enqueue; *ticket identifies the batch.
//
// Called with submit_mu held and mu NOT held. A slot whose previous piece is still running
// is waited for without mu (so _poll / _wait from other threads go on), then drained under it;
// a slot taken by this submit is not busy, so nothing else touches it while its piece is
// staged and launched without mu, and only its hand-over (busy, ticket, results) is under mu.
template <class Chunker, class Launch>
int enqueue(aipstack_chksum_engine *e, uint64_t n, void *h_out, uint32_t elem, Chunker chunker,
            Launch launch, uint64_t *ticket) {
    Span_ns timed(e->stats, e->stats.enqueue);
    DeviceGuard dg(e->device);
    if (!dg.ok) return AIPSTACK_CHKSUM_ENODEV;
    uint64_t t;
    {
        std::lock_guard<std::mutex> lock(e->mu);
        t = e->next_ticket++;
        e->submitting = t;
    }
    *ticket = t;
    int status = AIPSTACK_CHKSUM_OK;
    uint64_t i0 = 0;
    while (i0 < n && status == AIPSTACK_CHKSUM_OK) {
        Slot &s = e->slots[e->next_slot];
        e->next_slot = (e->next_slot + 1) % e->slots.size();
        // An earlier piece (this batch's or an older one's) completes; its failure is
        // recorded against its own ticket. One of this batch's own pieces failing ends
        // the enqueue (the rest would be wasted work).
        hipEvent_t ev = nullptr;
        uint64_t prev = 0, prev_seq = 0;
        {
            std::lock_guard<std::mutex> lock(e->mu);
            if (s.busy) {
                ev = s.done;
                prev = s.ticket;
                prev_seq = s.seq;
            }
        }
#ifdef AIPSTACK_ENGINE_FAULT_INJECTION
        if (ev) {  // a long back-pressure wait, made deterministic (test builds)
            if (const uint64_t us = g_wait_delay_us.load())
                std::this_thread::sleep_for(std::chrono::microseconds(us));
        }
#endif
        if (ev && hipEventQuery(ev) == hipErrorNotReady) {  // back-pressure, without mu
            Span_ns waited(e->stats, e->stats.slot_wait);
            (void)hipEventSynchronize(ev);
        } else if (ev) {
            (void)hipGetLastError();
        }
        int ds = AIPSTACK_CHKSUM_OK;
        if (ev) {
            std::lock_guard<std::mutex> lock(e->mu);
            // a _poll / _wait may have completed it meanwhile (its failure, if any, is then
            // recorded against its ticket already)
            if (s.busy && s.seq == prev_seq) ds = drain(e, s);
            else if (prev == t) {
                const auto it = e->failed.find(t);
                if (it != e->failed.end()) ds = it->second;
            }
        }
        if (ds < 0 && prev == t) {
            status = ds;
            break;
        }
        s.tx_frames = nullptr;  // a Tx fill's launch sets it again
        uint64_t i1 = 0;
        Span sp;
        chunker(i0, &i1, &sp);
        const uint64_t cnt = i1 - i0;
        const Region *reg = sp.bytes ? find_registered(e, sp.src, sp.bytes) : nullptr;
        const bool registered = reg != nullptr;
        const bool in_place = e->zero_copy_bytes && registered && reg->dev;
        const bool staged_rows = !registered && sp.bytes && sp.row_len && e->pageable_rows;
        s.zero_copy = in_place || staged_rows || cnt <= e->zero_copy_max;
        s.k_off = s.zero_copy ? s.dh_off : s.d_off;
        s.k_out = s.zero_copy ? s.dh_out : s.d_out;
        const bool rows = registered && sp.width != 0 && sp.width < sp.pitch;
        const void *h_src = sp.src;
        s.k_bytes = s.d_bytes;
        s.host_bytes = in_place || staged_rows;
        if (in_place) {
            // the kernel reads the caller's page-locked bytes over the link itself
            s.k_bytes = const_cast<char *>(reg->dev + (sp.src - reg->p));
        } else if (staged_rows) {
            // the frames' bytes into pinned staging, read there by the kernel
            Span_ns staged(e->stats, e->stats.stage);
            stage_copy_frames(e->pool, s.h_stage, sp.src, sp.pitch, sp.row_len, sp.bytes / sp.pitch);
            s.k_bytes = s.dh_stage;
        } else if (sp.bytes && !registered) {  // pageable: CPU copy into pinned staging
            Span_ns staged(e->stats, e->stats.stage);
            stage_copy(e->pool, s.h_stage, sp.src, sp.bytes);
            h_src = s.h_stage;
        }
        const bool copy = sp.bytes && s.k_bytes == s.d_bytes;
        if (copy && rows)
            status = check_hip(hipMemcpy2DAsync(s.d_bytes, sp.pitch, h_src, sp.pitch, sp.width,
                                                sp.bytes / sp.pitch, hipMemcpyHostToDevice,
                                                s.stream));
        else if (copy)
            status = check_hip(hipMemcpyAsync(s.d_bytes, h_src, sp.bytes, hipMemcpyHostToDevice,
                                              s.stream));
        s.seq = ++e->pieces;
        e->stats.pieces.fetch_add(1, std::memory_order_relaxed);
#ifdef AIPSTACK_ENGINE_FAULT_INJECTION
        if (status == AIPSTACK_CHKSUM_OK && injected(e, g_fail_at_launch, s.seq))
            status = AIPSTACK_CHKSUM_EHIP;
#endif
        if (status == AIPSTACK_CHKSUM_OK) status = launch(s, i0, i1);
        if (status == AIPSTACK_CHKSUM_OK && !s.zero_copy)
            status = check_hip(hipMemcpyAsync(s.h_out, s.d_out, cnt * elem,
                                              hipMemcpyDeviceToHost, s.stream));
        if (status == AIPSTACK_CHKSUM_OK) status = check_hip(hipEventRecord(s.done, s.stream));
        {
            std::lock_guard<std::mutex> lock(e->mu);
            s.user_out = static_cast<char *>(h_out) + i0 * elem;
            s.count = cnt;
            s.out_elem = elem;
            s.ticket = t;
            s.busy = status == AIPSTACK_CHKSUM_OK;
        }
        i0 = i1;
    }
    std::lock_guard<std::mutex> lock(e->mu);
    if (status != AIPSTACK_CHKSUM_OK) record_failure(e, t, status);
    e->submitting = 0;
    return status;
}

// Complete batch `ticket` (with mu held): 0 = done (results in place), 1 = still running
// (a piece, or its Tx records in the applier), < 0 = it failed (its first failure; the
// record is consumed). `blocking` waits for its pieces (whose events the caller has already
// waited for without mu), never for the applier: _wait does that outside mu.
int complete(aipstack_chksum_engine *e, uint64_t ticket, bool blocking) {
    if (ticket == 0 || ticket >= e->next_ticket) return AIPSTACK_CHKSUM_EINVAL;
    if (ticket == e->submitting) return 1;
    Span_ns timed(e->stats, e->stats.complete);
    DeviceGuard dg(e->device);
    if (!dg.ok) return AIPSTACK_CHKSUM_ENODEV;
    int pending = 0;
    for (Slot &s : e->slots) {
        if (!s.busy || s.ticket != ticket) continue;
        const int st = drain(e, s, blocking);
        if (st == 1) pending = 1;
    }
    if (pending) return 1;
    if (applies_pending(e, ticket, false)) return 1;
    const auto it = e->failed.find(ticket);
    if (it == e->failed.end()) return AIPSTACK_CHKSUM_OK;
    const int st = it->second;
    e->failed.erase(it);
    return st;
}

// Every piece in flight, completed as _wait completes it (results delivered, Tx records
// applied); failures stay recorded. Called with mu held, only where no submit can run
// (destroy; unregister holds submit_mu): the applier then only holds pieces queued before.
void drain_all(aipstack_chksum_engine *e) {
    for (Slot &s : e->slots) (void)drain(e, s, true);
    (void)applies_pending(e, 0, true);
}

}  // namespace

extern "C" int aipstack_chksum_engine_create(int device, uint64_t chunk_bytes, int nstreams,
                                             aipstack_chksum_engine **out) {
    if (!out || nstreams < 1 || nstreams > 16) return AIPSTACK_CHKSUM_EINVAL;
    *out = nullptr;
    if (chunk_bytes == 0) chunk_bytes = 64ull << 20;
    if (chunk_bytes < (1u << 17)) chunk_bytes = 1u << 17;  // >= 2 max-size packets
    const int dc = aipstack_chksum_device_check(device);
    if (dc != AIPSTACK_CHKSUM_OK) return dc;
    DeviceGuard dg(device);
    if (!dg.ok) return AIPSTACK_CHKSUM_ENODEV;
    auto *e = new (std::nothrow) aipstack_chksum_engine;
    if (!e) return AIPSTACK_CHKSUM_EINVAL;
    e->device = device;
    e->chunk_bytes = chunk_bytes;
    // results/offsets staging sized for the smallest packets (64 B, the Ethernet minimum)
    e->chunk_packets = chunk_bytes / 64 + 1;
    // experiments: AIPSTACK_ENGINE_SLOT_ROWS=0 copies whole slots (one 1-D span per piece)
    if (const char *v = std::getenv("AIPSTACK_ENGINE_SLOT_ROWS")) e->slot_rows = std::atoi(v) != 0;
    e->zero_copy_bytes = tuning_engine_zero_copy() != 0;
    e->zero_copy_max = (uint64_t)std::max(tuning_engine_zero_copy_small(), 0);
    e->pageable_rows = tuning_engine_pageable_rows() != 0;
    if (const char *v = std::getenv("AIPSTACK_ENGINE_STATS")) e->stats.on = std::atoi(v) != 0;
    e->stats.created = now_ns();
    // host threads next to the device: the pool and the applier pinned to its local CPUs,
    // and the pinned staging allocated from them (its pages on the device's NUMA node)
    e->loc = device_locality(device);
    e->pool.start(host_threads_cap() - 1u, e->loc.cpus);
    start_applier(e);
    ScopedAffinity near_device(e->loc.cpus);
    e->slots.resize((size_t)nstreams);
    int st = AIPSTACK_CHKSUM_OK;
    for (Slot &s : e->slots) {
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipMalloc(&s.d_bytes, chunk_bytes));
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipMalloc(reinterpret_cast<void **>(&s.d_off), (e->chunk_packets + 1) * 8));
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipMalloc(reinterpret_cast<void **>(&s.d_out), e->chunk_packets * 8));
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipHostMalloc(&s.h_stage, chunk_bytes, hipHostMallocDefault));
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipHostMalloc(reinterpret_cast<void **>(&s.h_off), (e->chunk_packets + 1) * 8, hipHostMallocDefault));
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipHostMalloc(reinterpret_cast<void **>(&s.h_out), e->chunk_packets * 8, hipHostMallocDefault));
        if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        if (st == AIPSTACK_CHKSUM_OK)
            st = check_hip(hipHostGetDevicePointer(reinterpret_cast<void **>(&s.dh_off), s.h_off, 0));
        if (st == AIPSTACK_CHKSUM_OK)
            st = check_hip(hipHostGetDevicePointer(reinterpret_cast<void **>(&s.dh_out), s.h_out, 0));
        if (st == AIPSTACK_CHKSUM_OK)
            st = check_hip(hipHostGetDevicePointer(reinterpret_cast<void **>(&s.dh_stage), s.h_stage, 0));
    }
    if (st != AIPSTACK_CHKSUM_OK) {
        release(e);
        delete e;
        return st;
    }
    *out = e;
    return AIPSTACK_CHKSUM_OK;
}

extern "C" void aipstack_chksum_engine_destroy(aipstack_chksum_engine *e) {
    if (!e) return;
    {
        std::lock_guard<std::mutex> sub(e->submit_mu);
        std::lock_guard<std::mutex> lock(e->mu);
        DeviceGuard dg(e->device);
        drain_all(e);  // pieces in flight complete: results written, Tx fields applied
    }
    release(e);
    e->pool.stop();
    if (e->stats.on) {
        const Stats &t = e->stats;
        auto ms = [](const std::atomic<uint64_t> &v) { return (double)v.load() / 1e6; };
        std::fprintf(stderr,
                     "{\"engine_stats\": {\"device\": %d, \"pieces\": %llu, \"life_ms\": %.3f, "
                     "\"enqueue_ms\": %.3f, \"slot_wait_ms\": %.3f, \"rec_copy_ms\": %.3f, "
                     "\"stage_ms\": %.3f, \"complete_ms\": %.3f, \"apply_wait_ms\": %.3f, "
                     "\"applier_busy_ms\": %.3f}}\n",
                     e->device, (unsigned long long)t.pieces.load(),
                     (double)(now_ns() - t.created) / 1e6, ms(t.enqueue), ms(t.slot_wait),
                     ms(t.rec_copy), ms(t.stage), ms(t.complete), ms(t.apply_wait), ms(t.apply));
    }
    delete e;
}

namespace aipstack_amd {
// For the engine group (chksum_engine_group.cpp): a region page-locked once for every
// device (hipHostRegisterPortable) becomes DMA-direct input of this engine too; removing it
// first completes the pieces in flight (they may still read it).
bool engine_adopt_region(aipstack_chksum_engine *e, const void *p, uint64_t bytes) {
    std::lock_guard<std::mutex> sub(e->submit_mu);
    std::lock_guard<std::mutex> lock(e->mu);
    DeviceGuard dg(e->device);
    const char *dev = mapped_address(p);
    e->registered.push_back(Region{static_cast<const char *>(p), bytes, false, dev});
    return dev != nullptr;
}
void engine_drop_region(aipstack_chksum_engine *e, const void *p) {
    std::lock_guard<std::mutex> sub(e->submit_mu);
    std::lock_guard<std::mutex> lock(e->mu);
    for (size_t i = 0; i < e->registered.size(); ++i) {
        if (e->registered[i].p == p) {
            DeviceGuard dg(e->device);
            drain_all(e);
            e->registered.erase(e->registered.begin() + (long)i);
            return;
        }
    }
}
}  // namespace aipstack_amd

extern "C" int aipstack_chksum_engine_register(aipstack_chksum_engine *e, void *host_ptr,
                                               uint64_t bytes) {
    if (!e || !host_ptr || bytes == 0) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> sub(e->submit_mu);
    std::lock_guard<std::mutex> lock(e->mu);
    DeviceGuard dg(e->device);
    if (!dg.ok) return AIPSTACK_CHKSUM_ENODEV;
    const int st = check_hip(hipHostRegister(host_ptr, bytes, hipHostRegisterMapped));
    if (st == AIPSTACK_CHKSUM_OK)
        e->registered.push_back(Region{static_cast<char *>(host_ptr), bytes, true,
                                       mapped_address(host_ptr)});
    return st;
}

extern "C" int aipstack_chksum_engine_unregister(aipstack_chksum_engine *e, void *host_ptr) {
    if (!e || !host_ptr) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> sub(e->submit_mu);
    std::lock_guard<std::mutex> lock(e->mu);
    for (size_t i = 0; i < e->registered.size(); ++i) {
        if (e->registered[i].p == host_ptr) {
            DeviceGuard dg(e->device);
            // pieces in flight may still DMA from (or, Tx, complete into) the region
            drain_all(e);
            const int st = e->registered[i].owned ? check_hip(hipHostUnregister(host_ptr))
                                                  : AIPSTACK_CHKSUM_OK;
            e->registered.erase(e->registered.begin() + (long)i);
            return st;
        }
    }
    return AIPSTACK_CHKSUM_EINVAL;
}

extern "C" int aipstack_chksum_engine_submit_strided(aipstack_chksum_engine *e,
                                                     const void *h_base, uint64_t stride,
                                                     uint32_t len, uint64_t n, uint16_t *h_out,
                                                     uint32_t flags, uint64_t *ticket) {
    if (!e || !h_base || !h_out || !ticket || len > AIPSTACK_CHKSUM_MAX_LEN)
        return AIPSTACK_CHKSUM_EINVAL;
    // packets per chunk: the chunk's byte span (i1-i0-1)*stride + len must fit
    uint64_t per = stride ? (e->chunk_bytes - len) / stride + 1 : e->chunk_packets;
    per = std::min<uint64_t>(std::max<uint64_t>(per, 1), e->chunk_packets);
    if ((per - 1) * stride + len > e->chunk_bytes) return AIPSTACK_CHKSUM_EINVAL;
    const char *base = static_cast<const char *>(h_base);
    auto chunker = [&](uint64_t i0, uint64_t *i1, Span *sp) {
        *i1 = std::min(n, i0 + per);
        sp->src = base + i0 * stride;
        sp->bytes = (*i1 - i0 - 1) * stride + len;
    };
    auto launch = [&](Slot &s, uint64_t i0, uint64_t i1) {
        return batch_strided_from(s.k_bytes, stride, len, i1 - i0, s.k_out, flags, s.stream,
                                  s.host_bytes);
    };
    std::lock_guard<std::mutex> lock(e->submit_mu);
    return enqueue(e, n, h_out, 2, chunker, launch, ticket);
}

namespace {
// CSR batches (checksums or Rx verdicts): whole packets per chunk while they fit, offsets
// rebased into the slot's staging.
template <class Kernel>
int submit_csr_like(aipstack_chksum_engine *e, const void *h_base, const uint64_t *h_offsets,
                    uint64_t n, void *h_out, uint32_t elem, Kernel kernel, uint64_t *ticket) {
    for (uint64_t i = 0; i < n; ++i)  // contract check: non-decreasing, each <= 65535
        if (h_offsets[i + 1] < h_offsets[i] || h_offsets[i + 1] - h_offsets[i] > AIPSTACK_CHKSUM_MAX_LEN)
            return AIPSTACK_CHKSUM_EINVAL;
    const char *base = static_cast<const char *>(h_base);
    auto chunker = [&](uint64_t i0, uint64_t *i1, Span *sp) {
        // whole packets while they fit the chunk (binary search on the offsets)
        const uint64_t limit = h_offsets[i0] + e->chunk_bytes;
        const uint64_t *hi = std::upper_bound(h_offsets + i0 + 1,
                                              h_offsets + std::min(n, i0 + e->chunk_packets) + 1,
                                              limit);
        uint64_t j = (uint64_t)(hi - h_offsets) - 1;  // last offset <= limit
        if (j <= i0) j = i0 + 1;
        *i1 = j;
        sp->src = base + h_offsets[i0];
        sp->bytes = h_offsets[j] - h_offsets[i0];
    };
    auto launch = [&](Slot &s, uint64_t i0, uint64_t i1) {
        const uint64_t cnt = i1 - i0;
        const uint64_t b0 = h_offsets[i0];
        for (uint64_t i = 0; i <= cnt; ++i) s.h_off[i] = h_offsets[i0 + i] - b0;  // rebased
        if (!s.zero_copy) {
            const int st = check_hip(hipMemcpyAsync(s.d_off, s.h_off, (cnt + 1) * 8,
                                                    hipMemcpyHostToDevice, s.stream));
            if (st != AIPSTACK_CHKSUM_OK) return st;
        }
        return kernel(s, i0, cnt);
    };
    std::lock_guard<std::mutex> lock(e->submit_mu);
    return enqueue(e, n, h_out, elem, chunker, launch, ticket);
}
}  // namespace

extern "C" int aipstack_chksum_engine_submit_rx_verify(aipstack_chksum_engine *e,
                                                       const void *h_base,
                                                       const uint64_t *h_offsets, uint64_t n,
                                                       uint8_t *h_verdicts, uint64_t *ticket) {
    if (!e || !h_base || !h_offsets || !h_verdicts || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    return submit_csr_like(e, h_base, h_offsets, n, h_verdicts, 1,
                           [&](Slot &s, uint64_t, uint64_t cnt) {
                               return aipstack_chksum_rx_verify(s.k_bytes, s.k_off, cnt,
                                                                reinterpret_cast<uint8_t *>(s.k_out),
                                                                s.stream);
                           },
                           ticket);
}

extern "C" int aipstack_chksum_engine_submit_tx_fill(aipstack_chksum_engine *e, void *h_base,
                                                     const uint64_t *h_offsets, uint64_t n,
                                                     uint8_t *h_status, uint64_t *ticket) {
    if (!e || !h_base || !h_offsets || !h_status || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    char *frames = static_cast<char *>(h_base);
    return submit_csr_like(e, h_base, h_offsets, n, h_status, 8,
                           [&](Slot &s, uint64_t i0, uint64_t cnt) {
                               s.tx_frames = frames;  // applied on completion (drain)
                               s.tx_offs = h_offsets + i0;
                               s.tx_stride = 0;
                               s.tx_status = h_status + i0;
                               return aipstack_chksum_tx_fill_records(
                                   s.k_bytes, s.k_off, cnt, reinterpret_cast<uint64_t *>(s.k_out),
                                   s.stream);
                           },
                           ticket);
}

extern "C" int aipstack_chksum_engine_host_tx_fill(aipstack_chksum_engine *e, void *h_base,
                                                   const uint64_t *h_offsets, uint64_t n,
                                                   uint8_t *h_status) {
    if (!e || !h_base || !h_offsets || !h_status) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_submit_tx_fill(e, h_base, h_offsets, n, h_status, &t);
    if (st != AIPSTACK_CHKSUM_OK) {
        if (t) (void)aipstack_chksum_engine_wait(e, t);
        return st;
    }
    return aipstack_chksum_engine_wait(e, t);
}

extern "C" int aipstack_chksum_engine_host_rx_verify(aipstack_chksum_engine *e, const void *h_base,
                                                     const uint64_t *h_offsets, uint64_t n,
                                                     uint8_t *h_verdicts) {
    if (!e || !h_base || !h_offsets || !h_verdicts) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_submit_rx_verify(e, h_base, h_offsets, n, h_verdicts, &t);
    if (st != AIPSTACK_CHKSUM_OK) {
        if (t) (void)aipstack_chksum_engine_wait(e, t);
        return st;
    }
    return aipstack_chksum_engine_wait(e, t);
}

extern "C" int aipstack_chksum_engine_submit_csr(aipstack_chksum_engine *e, const void *h_base,
                                                 const uint64_t *h_offsets, uint64_t n,
                                                 uint16_t *h_out, uint32_t flags,
                                                 uint64_t *ticket) {
    if (!e || !h_base || !h_offsets || !h_out || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    return submit_csr_like(e, h_base, h_offsets, n, h_out, 2,
                           [&](Slot &s, uint64_t, uint64_t cnt) {
                               return batch_csr_from(s.k_bytes, s.k_off, cnt, s.k_out, flags,
                                                     s.stream, s.host_bytes);
                           },
                           ticket);
}

namespace {
// Ring-slot batches: whole slots per chunk, lengths staged beside them. From registered
// memory only the piece's longest frame's length (rounded up to 64 bytes) of each slot
// crosses PCIe, as one 2-D copy that keeps the slot layout on the device: a 2048-byte ring
// of Ethernet frames (<= 1514 B) moves <= 1536 bytes per slot instead of 2048. Every length is checked first:
// <= min(slot_stride, 65535), else _EINVAL before any work.
template <class Kernel>
int submit_slotted_like(aipstack_chksum_engine *e, const void *h_base, uint64_t slot_stride,
                        const uint32_t *h_len, uint64_t n, void *h_out, uint32_t elem,
                        Kernel kernel, uint64_t *ticket) {
    if (slot_stride == 0 || slot_stride > e->chunk_bytes) return AIPSTACK_CHKSUM_EINVAL;
    const uint64_t cap = std::min<uint64_t>(slot_stride, AIPSTACK_CHKSUM_MAX_LEN);
    for (uint64_t i = 0; i < n; ++i)
        if (h_len[i] > cap) return AIPSTACK_CHKSUM_EINVAL;
    const uint64_t per = std::min<uint64_t>(e->chunk_bytes / slot_stride, e->chunk_packets);
    const char *base = static_cast<const char *>(h_base);
    auto chunker = [&](uint64_t i0, uint64_t *i1, Span *sp) {
        *i1 = std::min(n, i0 + per);
        sp->src = base + i0 * slot_stride;
        sp->bytes = (*i1 - i0) * slot_stride;
        sp->pitch = slot_stride;
        sp->row_len = h_len + i0;
        if (!e->slot_rows) return;
        uint32_t longest = 0;
        for (uint64_t i = i0; i < *i1; ++i) longest = std::max(longest, h_len[i]);
        sp->width = std::min<uint64_t>(((uint64_t)longest + 63u) & ~63ull, slot_stride);
        if (longest == 0) sp->bytes = 0;  // every frame empty: nothing to copy
    };
    auto launch = [&](Slot &s, uint64_t i0, uint64_t i1) {
        const uint64_t cnt = i1 - i0;
        std::memcpy(s.h_off, h_len + i0, cnt * sizeof(uint32_t));  // lengths -> pinned staging
        if (!s.zero_copy) {
            const int st = check_hip(hipMemcpyAsync(s.d_off, s.h_off, cnt * sizeof(uint32_t),
                                                    hipMemcpyHostToDevice, s.stream));
            if (st != AIPSTACK_CHKSUM_OK) return st;
        }
        return kernel(s, i0, cnt, reinterpret_cast<const uint32_t *>(s.k_off));
    };
    std::lock_guard<std::mutex> lock(e->submit_mu);
    return enqueue(e, n, h_out, elem, chunker, launch, ticket);
}
}  // namespace

extern "C" int aipstack_chksum_engine_submit_slotted(aipstack_chksum_engine *e, const void *h_base,
                                                     uint64_t slot_stride, const uint32_t *h_len,
                                                     uint64_t n, uint16_t *h_out, uint32_t flags,
                                                     uint64_t *ticket) {
    if (!e || !h_base || !h_len || !h_out || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    return submit_slotted_like(e, h_base, slot_stride, h_len, n, h_out, 2,
                               [&](Slot &s, uint64_t, uint64_t cnt, const uint32_t *d_len) {
                                   return batch_slotted_from(s.k_bytes, slot_stride, d_len, cnt,
                                                             s.k_out, flags, s.stream,
                                                             s.host_bytes);
                               },
                               ticket);
}

extern "C" int aipstack_chksum_engine_submit_rx_verify_slotted(
    aipstack_chksum_engine *e, const void *h_base, uint64_t slot_stride, const uint32_t *h_len,
    uint64_t n, uint8_t *h_verdicts, uint64_t *ticket) {
    if (!e || !h_base || !h_len || !h_verdicts || !ticket ||
        slot_stride > AIPSTACK_CHKSUM_MAX_SLOT_STRIDE)
        return AIPSTACK_CHKSUM_EINVAL;
    return submit_slotted_like(e, h_base, slot_stride, h_len, n, h_verdicts, 1,
                               [&](Slot &s, uint64_t, uint64_t cnt, const uint32_t *d_len) {
                                   return rx_verify_slotted_from(
                                       s.k_bytes, slot_stride, d_len, cnt,
                                       reinterpret_cast<uint8_t *>(s.k_out), s.stream,
                                       s.host_bytes);
                               },
                               ticket);
}

extern "C" int aipstack_chksum_engine_submit_tx_fill_slotted(
    aipstack_chksum_engine *e, void *h_base, uint64_t slot_stride, const uint32_t *h_len,
    uint64_t n, uint8_t *h_status, uint64_t *ticket) {
    if (!e || !h_base || !h_len || !h_status || !ticket ||
        slot_stride > AIPSTACK_CHKSUM_MAX_SLOT_STRIDE)
        return AIPSTACK_CHKSUM_EINVAL;
    char *frames = static_cast<char *>(h_base);
    return submit_slotted_like(e, h_base, slot_stride, h_len, n, h_status, 8,
                               [&](Slot &s, uint64_t i0, uint64_t cnt, const uint32_t *d_len) {
                                   s.tx_frames = frames + i0 * slot_stride;
                                   s.tx_offs = nullptr;
                                   s.tx_stride = slot_stride;
                                   s.tx_status = h_status + i0;
                                   return tx_fill_records_slotted_from(
                                       s.k_bytes, slot_stride, d_len, cnt,
                                       reinterpret_cast<uint64_t *>(s.k_out), s.stream,
                                       s.host_bytes);
                               },
                               ticket);
}

namespace {
// The synchronous calls: submit, then wait (also for the pieces a failed submit enqueued).
int finish_sync(aipstack_chksum_engine *e, int st, uint64_t t) {
    if (st != AIPSTACK_CHKSUM_OK) {
        if (t) (void)aipstack_chksum_engine_wait(e, t);
        return st;
    }
    return aipstack_chksum_engine_wait(e, t);
}
}  // namespace

extern "C" int aipstack_chksum_engine_host_slotted(aipstack_chksum_engine *e, const void *h_base,
                                                   uint64_t slot_stride, const uint32_t *h_len,
                                                   uint64_t n, uint16_t *h_out, uint32_t flags) {
    if (!e || !h_base || !h_len || !h_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    return finish_sync(e, aipstack_chksum_engine_submit_slotted(e, h_base, slot_stride, h_len, n,
                                                               h_out, flags, &t), t);
}

extern "C" int aipstack_chksum_engine_host_rx_verify_slotted(aipstack_chksum_engine *e,
                                                             const void *h_base,
                                                             uint64_t slot_stride,
                                                             const uint32_t *h_len, uint64_t n,
                                                             uint8_t *h_verdicts) {
    if (!e || !h_base || !h_len || !h_verdicts) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    return finish_sync(e, aipstack_chksum_engine_submit_rx_verify_slotted(
                              e, h_base, slot_stride, h_len, n, h_verdicts, &t), t);
}

extern "C" int aipstack_chksum_engine_host_tx_fill_slotted(aipstack_chksum_engine *e, void *h_base,
                                                           uint64_t slot_stride,
                                                           const uint32_t *h_len, uint64_t n,
                                                           uint8_t *h_status) {
    if (!e || !h_base || !h_len || !h_status) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    return finish_sync(e, aipstack_chksum_engine_submit_tx_fill_slotted(
                              e, h_base, slot_stride, h_len, n, h_status, &t), t);
}

extern "C" int aipstack_chksum_engine_poll(aipstack_chksum_engine *e, uint64_t ticket) {
    if (!e) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(e->mu);
    return complete(e, ticket, false);
}

extern "C" int aipstack_chksum_engine_wait(aipstack_chksum_engine *e, uint64_t ticket) {
    if (!e) return AIPSTACK_CHKSUM_EINVAL;
    // The long part -- the GPU finishing the batch -- is waited for without the engine
    // lock, so _poll and _submit from other threads go on meanwhile. A slot drained (and
    // re-used) by another thread in between has delivered its piece already; its event then
    // only makes this wait a little longer.
    std::vector<hipEvent_t> events;
    {
        std::lock_guard<std::mutex> lock(e->mu);
        if (ticket == 0 || ticket >= e->next_ticket) return AIPSTACK_CHKSUM_EINVAL;
        for (const Slot &s : e->slots)
            if (s.busy && s.ticket == ticket) events.push_back(s.done);
    }
#ifdef AIPSTACK_ENGINE_FAULT_INJECTION
    if (const uint64_t us = g_wait_delay_us.load())  // a long GPU wait, made deterministic
        std::this_thread::sleep_for(std::chrono::microseconds(us));
#endif
    for (hipEvent_t ev : events) (void)hipEventSynchronize(ev);
    for (;;) {
        {
            std::lock_guard<std::mutex> lock(e->mu);
            const int st = complete(e, ticket, true);
            if (st != 1) return st;
        }
        // its Tx records are still queued in the applier: wait for them without mu
        // (ADVICE round 3), then collect the ticket's status (a ticket whose submit is still
        // running on another thread -- it cannot have been returned yet -- yields meanwhile)
        if (!applies_pending(e, ticket, true)) std::this_thread::yield();
    }
}

#ifdef AIPSTACK_ENGINE_FAULT_INJECTION
// Test builds only: pieces (engine-wide numbering from 1) that fail at launch / completion.
extern "C" void aipstack_chksum_engine_test_inject(uint64_t fail_at_launch,
                                                    uint64_t fail_at_completion) {
    g_fail_at_launch = fail_at_launch;
    g_fail_at_completion = fail_at_completion;
}
extern "C" void aipstack_chksum_engine_test_wait_delay(uint64_t us) { g_wait_delay_us = us; }
// Restricts the injected failures to one engine (null: every engine), e.g. one engine of a
// group (aipstack_chksum_engine_group_engine).
extern "C" void aipstack_chksum_engine_test_inject_only(const aipstack_chksum_engine *e) {
    g_fail_engine = e;
}
#endif

extern "C" int aipstack_chksum_engine_locality(const aipstack_chksum_engine *e, int *numa_node,
                                               int *pinned_cpus) {
    if (!e) return AIPSTACK_CHKSUM_EINVAL;
    if (numa_node) *numa_node = e->loc.numa_node;
    if (pinned_cpus) *pinned_cpus = (int)e->loc.cpus.size();
    return AIPSTACK_CHKSUM_OK;
}

extern "C" int aipstack_chksum_engine_region_mapped(aipstack_chksum_engine *e, const void *host_ptr) {
    if (!e || !host_ptr) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(e->mu);
    const Region *r = find_registered(e, host_ptr, 1);
    if (!r) return AIPSTACK_CHKSUM_EINVAL;
    return r->dev && e->zero_copy_bytes ? 1 : 0;
}

extern "C" int aipstack_chksum_engine_host_strided(aipstack_chksum_engine *e, const void *h_base,
                                                   uint64_t stride, uint32_t len, uint64_t n,
                                                   uint16_t *h_out, uint32_t flags) {
    if (!e || !h_base || !h_out || len > AIPSTACK_CHKSUM_MAX_LEN) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_submit_strided(e, h_base, stride, len, n, h_out, flags, &t);
    if (st != AIPSTACK_CHKSUM_OK) {
        if (t) (void)aipstack_chksum_engine_wait(e, t);  // pieces already in flight
        return st;
    }
    return aipstack_chksum_engine_wait(e, t);
}

extern "C" int aipstack_chksum_engine_host_csr(aipstack_chksum_engine *e, const void *h_base,
                                               const uint64_t *h_offsets, uint64_t n,
                                               uint16_t *h_out, uint32_t flags) {
    if (!e || !h_base || !h_offsets || !h_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_submit_csr(e, h_base, h_offsets, n, h_out, flags, &t);
    if (st != AIPSTACK_CHKSUM_OK) {
        if (t) (void)aipstack_chksum_engine_wait(e, t);
        return st;
    }
    return aipstack_chksum_engine_wait(e, t);
}
