// aipstack_amd -- several devices behind one host-memory batch, in ONE process.
//
// The reference stack runs in one process on one event-loop thread (reference
// event_loop/event_loop.dox:48-50), so it cannot use the one-process-per-GPU launch the bench
// uses for device-resident shards. A host batch that arrives through host memory is PCIe-bound
// (~50 GiB/s per device link); spreading it over several devices' links is how the
// engine outruns the host's own cores on host-resident data. The group owns one engine per
// device (each with its own streams, pinned staging and host threads next to its device),
// splits a batch into disjoint contiguous ranges of about equal bytes, and runs each range on
// its engine. There is no data exchange between the devices: each range is an independent
// batch (disjoint packet ranges, no collective).
//
// Asynchronous (round 4): a batch is submitted and gets ONE group ticket over the per-device
// engine tickets; _poll / _wait complete it, with each device's status and the first failure
// (by device order) as the result -- so the event loop keeps filling its next batch while
// every device works, as it can with a single engine. Where a range is submitted:
//   * on the calling thread, when that is cheap: the batch lies in a region registered with the
//     group (the engines' kernels read it in place; a submit only launches) or is small;
//   * else on the range's device worker: one persistent thread per device, pinned to the CPUs
//     next to it, which runs the engine submit (the pageable staging copy, on the device's NUMA
//     node) while the caller returns at once.
// A batch smaller than kSplitMin bytes per device goes to fewer devices (round robin), whole:
// a 64-frame burst is one engine's batch, as fast as on a single engine.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
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

constexpr uint64_t kSplitMin = 4ull << 20;   // bytes per device before a batch is split
constexpr uint64_t kInlineMax = 1ull << 20;  // pageable batches up to this submit inline

// One device's share of a group batch.
struct Part {
    uint64_t i0 = 0, i1 = 0;
    bool used = false;        // the device has a range of this batch
    bool submitted = false;   // its engine submit has returned
    int submit_status = AIPSTACK_CHKSUM_OK;
    uint64_t eng_ticket = 0;  // the engine's ticket (0: nothing was enqueued)
    bool done = false;
    bool waiting = false;     // a group _wait owns its engine ticket: _poll leaves it alone
    int status = AIPSTACK_CHKSUM_OK;
};

struct Batch {
    std::vector<Part> parts;  // one per engine
    int waiters = 0;          // _wait calls blocked on this ticket (not the one that owns it)
};

// The outcome of a batch that completed while other _wait calls were blocked on it: each of
// them returns it too (then it is dropped). Calls made after the completion return OK.
struct Finished {
    int result = AIPSTACK_CHKSUM_OK;
    std::vector<int> dev_status;
    int waiters = 0;
};

// A persistent thread per device: runs the engine submits of its device's ranges, in order.
struct DevWorker {
    std::thread thread;
    std::deque<std::function<void()>> jobs;
    std::condition_variable cv;
    std::vector<int> cpus;
};

struct Region {
    const char *p;
    uint64_t bytes;
};

}  // namespace

struct aipstack_chksum_engine_group {
    std::vector<aipstack_chksum_engine *> engines;
    std::vector<int> devices;
    std::vector<Region> regions;  // page-locked by the group (portable, mapped)
    std::vector<std::unique_ptr<DevWorker>> workers;
    std::map<uint64_t, Batch> batches;  // tickets not yet completed
    std::map<uint64_t, Finished> finished;  // completed with waits still blocked on them
    uint64_t next_ticket = 1;
    size_t rr = 0;                      // first device of the next batch that uses fewer
    std::mutex mu;                      // the state above; never held across an engine wait
    std::condition_variable submitted;  // a part's submit returned
    bool stop = false;
};

namespace {

// Packet ranges [cut[k], cut[k+1]) over `parts` parts, about equal bytes each: `bytes_before(i)`
// is the byte position of packet i (non-decreasing, bytes_before(n) = total).
template <class BytesBefore>
std::vector<uint64_t> split(uint64_t n, size_t parts, BytesBefore bytes_before) {
    std::vector<uint64_t> cut(parts + 1, n);
    cut[0] = 0;
    const uint64_t total = bytes_before(n);
    for (size_t k = 1; k < parts; ++k) {
        const uint64_t target = (uint64_t)((__uint128_t)total * k / parts);
        uint64_t lo = cut[k - 1], hi = n;  // first packet whose start is >= target
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo) / 2;
            if (bytes_before(mid) < target) lo = mid + 1;
            else hi = mid;
        }
        cut[k] = lo;
    }
    return cut;
}

bool in_group_region(const aipstack_chksum_engine_group *g, const void *p, uint64_t bytes) {
    const char *c = static_cast<const char *>(p);
    for (const Region &r : g->regions)
        if (c >= r.p && c + bytes <= r.p + r.bytes) return true;
    return false;
}

void worker_loop(aipstack_chksum_engine_group *g, DevWorker *w) {
    pin_current_thread(w->cpus);
    std::unique_lock<std::mutex> lock(g->mu);
    for (;;) {
        w->cv.wait(lock, [&] { return g->stop || !w->jobs.empty(); });
        if (w->jobs.empty()) return;  // stop, and nothing queued
        std::function<void()> job = std::move(w->jobs.front());
        w->jobs.pop_front();
        lock.unlock();
        job();
        lock.lock();
    }
}

// Records part k of batch t as submitted (with g->mu held).
void mark_submitted(aipstack_chksum_engine_group *g, uint64_t t, size_t k, int st, uint64_t et) {
    const auto it = g->batches.find(t);
    if (it == g->batches.end()) return;
    Part &p = it->second.parts[k];
    p.submitted = true;
    p.submit_status = st;
    p.eng_ticket = et;
    g->submitted.notify_all();
}

// Submits a batch of n packets whose bytes lie in [span_p, span_p + span_bytes): splits it
// (bytes_before as for split()), and runs submit_part(k, i0, i1, &engine_ticket) for every
// range, inline or on the ranges' device workers. Returns the first inline failure, else _OK.
template <class BytesBefore, class SubmitPart>
int group_submit(aipstack_chksum_engine_group *g, uint64_t n, const void *span_p,
                 uint64_t span_bytes, BytesBefore bytes_before, SubmitPart submit_part,
                 uint64_t *ticket) {
    const size_t m = g->engines.size();
    const size_t parts = (size_t)std::max<uint64_t>(
        1, std::min<uint64_t>(m, span_bytes / kSplitMin));
    const std::vector<uint64_t> cut = split(n, parts, bytes_before);
    bool inline_submit;
    uint64_t t;
    std::vector<size_t> dev(parts);
    {
        std::lock_guard<std::mutex> lock(g->mu);  // (regions change under it)
        inline_submit = span_bytes <= kInlineMax || in_group_region(g, span_p, span_bytes);
        t = g->next_ticket++;
        Batch &b = g->batches[t];
        b.parts.resize(m);
        const size_t first = parts < m ? g->rr : 0;
        if (parts < m) g->rr = (g->rr + parts) % m;
        for (size_t j = 0; j < parts; ++j) {
            dev[j] = (first + j) % m;
            Part &p = b.parts[dev[j]];
            p.i0 = cut[j];
            p.i1 = cut[j + 1];
            p.used = p.i1 > p.i0;
        }
    }
    *ticket = t;
    int first_fail = AIPSTACK_CHKSUM_OK;
    for (size_t j = 0; j < parts; ++j) {
        const size_t k = dev[j];
        const uint64_t i0 = cut[j], i1 = cut[j + 1];
        if (i1 == i0) continue;
        if (inline_submit) {
            uint64_t et = 0;
            const int st = submit_part(k, i0, i1, &et);
            if (first_fail == AIPSTACK_CHKSUM_OK && st != AIPSTACK_CHKSUM_OK) first_fail = st;
            std::lock_guard<std::mutex> lock(g->mu);
            mark_submitted(g, t, k, st, et);
        } else {
            std::lock_guard<std::mutex> lock(g->mu);
            DevWorker *w = g->workers[k].get();
            w->jobs.push_back([g, t, k, i0, i1, submit_part] {
                uint64_t et = 0;
                const int st = submit_part(k, i0, i1, &et);
                std::lock_guard<std::mutex> l(g->mu);
                mark_submitted(g, t, k, st, et);
            });
            w->cv.notify_one();
        }
    }
    return first_fail;
}

// The result of a finished batch (with g->mu held): every device's status into dev_status,
// the first failure by device order as the return value; the batch record is dropped.
// Waits still blocked on the ticket get the same outcome (g->finished).
int finish_batch(aipstack_chksum_engine_group *g, std::map<uint64_t, Batch>::iterator it,
                 int *dev_status) {
    int first = AIPSTACK_CHKSUM_OK;
    const std::vector<Part> &parts = it->second.parts;
    std::vector<int> st(parts.size());
    for (size_t k = 0; k < parts.size(); ++k) {
        st[k] = parts[k].used ? parts[k].status : AIPSTACK_CHKSUM_OK;
        if (dev_status) dev_status[k] = st[k];
        if (first == AIPSTACK_CHKSUM_OK && st[k] != AIPSTACK_CHKSUM_OK) first = st[k];
    }
    if (it->second.waiters > 0)
        g->finished[it->first] = Finished{first, std::move(st), it->second.waiters};
    g->batches.erase(it);
    return first;
}

// A part's outcome once its engine ticket is complete: the submit's failure if it had one,
// else the ticket's.
void settle(Part &p, int engine_result) {
    p.done = true;
    p.status = p.submit_status != AIPSTACK_CHKSUM_OK ? p.submit_status : engine_result;
}

bool csr_ok(const uint64_t *off, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > AIPSTACK_CHKSUM_MAX_LEN) return false;
    return true;
}

// Ring slots (frame i = h_len[i] bytes at h_base + i * slot_stride): every length is checked
// before any device starts.
bool slots_ok(uint64_t slot_stride, const uint32_t *h_len, uint64_t n) {
    if (slot_stride == 0) return false;
    const uint64_t cap = std::min<uint64_t>(slot_stride, AIPSTACK_CHKSUM_MAX_LEN);
    for (uint64_t i = 0; i < n; ++i)
        if (h_len[i] > cap) return false;
    return true;
}

// The synchronous calls: submit, then wait (also after a failed submit: its other ranges).
int sync_call(aipstack_chksum_engine_group *g, int st, uint64_t t, int *dev_status) {
    const int w = t ? aipstack_chksum_engine_group_wait(g, t, dev_status) : st;
    return st != AIPSTACK_CHKSUM_OK ? st : w;
}

}  // namespace

extern "C" int aipstack_chksum_engine_group_create(const int *devices, int n_devices,
                                                   uint64_t chunk_bytes, int nstreams,
                                                   aipstack_chksum_engine_group **out) {
    if (!out || !devices || n_devices < 1 || n_devices > 64) return AIPSTACK_CHKSUM_EINVAL;
    *out = nullptr;
    auto *g = new (std::nothrow) aipstack_chksum_engine_group;
    if (!g) return AIPSTACK_CHKSUM_EINVAL;
    int st = AIPSTACK_CHKSUM_OK;
    for (int k = 0; k < n_devices && st == AIPSTACK_CHKSUM_OK; ++k) {
        aipstack_chksum_engine *e = nullptr;
        st = aipstack_chksum_engine_create(devices[k], chunk_bytes, nstreams, &e);
        if (st == AIPSTACK_CHKSUM_OK) {
            g->engines.push_back(e);
            g->devices.push_back(devices[k]);
        }
    }
    if (st != AIPSTACK_CHKSUM_OK) {
        for (aipstack_chksum_engine *e : g->engines) aipstack_chksum_engine_destroy(e);
        delete g;
        return st;
    }
    for (int k = 0; k < n_devices; ++k) {
        g->workers.emplace_back(new DevWorker);
        g->workers.back()->cpus = device_locality(devices[k]).cpus;
    }
    for (auto &w : g->workers) w->thread = std::thread(worker_loop, g, w.get());
    *out = g;
    return AIPSTACK_CHKSUM_OK;
}

extern "C" void aipstack_chksum_engine_group_destroy(aipstack_chksum_engine_group *g) {
    if (!g) return;
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->stop = true;  // the workers run what is queued, then exit
        for (auto &w : g->workers) w->cv.notify_one();
    }
    for (auto &w : g->workers) w->thread.join();
    // every range is submitted now; destroying an engine completes its pieces in flight
    for (aipstack_chksum_engine *e : g->engines) aipstack_chksum_engine_destroy(e);
    for (const Region &r : g->regions) (void)hipHostUnregister(const_cast<char *>(r.p));
    delete g;
}

extern "C" int aipstack_chksum_engine_group_size(const aipstack_chksum_engine_group *g) {
    return g ? (int)g->engines.size() : AIPSTACK_CHKSUM_EINVAL;
}

extern "C" aipstack_chksum_engine *aipstack_chksum_engine_group_engine(
    aipstack_chksum_engine_group *g, int k) {
    if (!g || k < 0 || (size_t)k >= g->engines.size()) return nullptr;
    return g->engines[(size_t)k];
}

extern "C" int aipstack_chksum_engine_group_register(aipstack_chksum_engine_group *g,
                                                     void *host_ptr, uint64_t bytes) {
    if (!g || !host_ptr || bytes == 0) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard dg(g->devices[0]);
    if (!dg.ok) return AIPSTACK_CHKSUM_ENODEV;
    // portable: page-locked for every device; mapped: each device's kernels can read it in
    // place (engine_adopt_region looks up each device's own address of it)
    const int st = check_hip(
        hipHostRegister(host_ptr, bytes, hipHostRegisterPortable | hipHostRegisterMapped));
    if (st != AIPSTACK_CHKSUM_OK) return st;
    g->regions.push_back(Region{static_cast<const char *>(host_ptr), bytes});
    for (aipstack_chksum_engine *e : g->engines) (void)engine_adopt_region(e, host_ptr, bytes);
    return AIPSTACK_CHKSUM_OK;
}

extern "C" int aipstack_chksum_engine_group_region_mapped(aipstack_chksum_engine_group *g,
                                                          const void *host_ptr) {
    if (!g || !host_ptr) return AIPSTACK_CHKSUM_EINVAL;
    int all = 1;
    for (aipstack_chksum_engine *e : g->engines) {
        const int r = aipstack_chksum_engine_region_mapped(e, host_ptr);
        if (r < 0) return r;
        all &= r;
    }
    return all;
}

extern "C" int aipstack_chksum_engine_group_unregister(aipstack_chksum_engine_group *g,
                                                       void *host_ptr) {
    if (!g || !host_ptr) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto it = std::find_if(g->regions.begin(), g->regions.end(),
                                 [&](const Region &r) { return r.p == host_ptr; });
    if (it == g->regions.end()) return AIPSTACK_CHKSUM_EINVAL;
    // (ranges queued on a worker still submit after this: the caller must have completed every
    // batch on the region first, as with a single engine)
    for (aipstack_chksum_engine *e : g->engines) engine_drop_region(e, host_ptr);
    g->regions.erase(it);
    return check_hip(hipHostUnregister(host_ptr));
}

extern "C" int aipstack_chksum_engine_group_poll(aipstack_chksum_engine_group *g, uint64_t ticket,
                                                 int *dev_status) {
    if (!g) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto it = g->batches.find(ticket);
    if (it == g->batches.end())
        return ticket != 0 && ticket < g->next_ticket ? AIPSTACK_CHKSUM_OK : AIPSTACK_CHKSUM_EINVAL;
    bool pending = false;
    for (size_t k = 0; k < it->second.parts.size(); ++k) {
        Part &p = it->second.parts[k];
        if (!p.used || p.done) continue;
        if (!p.submitted || p.waiting) {  // (a wait consumes that engine ticket's result)
            pending = true;
            continue;
        }
        const int r = p.eng_ticket ? aipstack_chksum_engine_poll(g->engines[k], p.eng_ticket)
                                   : AIPSTACK_CHKSUM_OK;
        if (r == 1) pending = true;
        else settle(p, r);
    }
    if (pending) return 1;
    return finish_batch(g, it, dev_status);
}

extern "C" int aipstack_chksum_engine_group_wait(aipstack_chksum_engine_group *g, uint64_t ticket,
                                                 int *dev_status) {
    if (!g) return AIPSTACK_CHKSUM_EINVAL;
    std::vector<std::pair<size_t, uint64_t>> todo;
    {
        std::unique_lock<std::mutex> lock(g->mu);
        auto it = g->batches.find(ticket);
        if (it == g->batches.end())
            return ticket != 0 && ticket < g->next_ticket ? AIPSTACK_CHKSUM_OK
                                                          : AIPSTACK_CHKSUM_EINVAL;
        // every range submitted, and none owned by another thread's wait
        ++it->second.waiters;
        g->submitted.wait(lock, [&] {
            it = g->batches.find(ticket);
            if (it == g->batches.end()) return true;
            for (const Part &p : it->second.parts)
                if (p.used && (!p.submitted || (p.waiting && !p.done))) return false;
            return true;
        });
        if (it == g->batches.end()) {  // completed by another thread meanwhile: its outcome
            const auto f = g->finished.find(ticket);
            if (f == g->finished.end()) return AIPSTACK_CHKSUM_OK;  // (not reachable)
            const int r = f->second.result;
            if (dev_status)
                std::copy(f->second.dev_status.begin(), f->second.dev_status.end(), dev_status);
            if (--f->second.waiters == 0) g->finished.erase(f);
            return r;
        }
        --it->second.waiters;
        // this wait owns the open parts: a concurrent _poll treats them as pending, so an
        // engine failure this wait consumes is reported here, once
        for (size_t k = 0; k < it->second.parts.size(); ++k) {
            Part &p = it->second.parts[k];
            if (p.used && !p.done) {
                p.waiting = true;
                todo.emplace_back(k, p.eng_ticket);
            }
        }
    }
    std::vector<int> res(todo.size(), AIPSTACK_CHKSUM_OK);
    for (size_t j = 0; j < todo.size(); ++j)  // the engines' waits, without the group lock
        if (todo[j].second)
            res[j] = aipstack_chksum_engine_wait(g->engines[todo[j].first], todo[j].second);
    std::lock_guard<std::mutex> lock(g->mu);
    // still there if this wait owns a part (no one else settles it); with nothing owned (every
    // part already done), a concurrent poll may have completed it meanwhile
    const auto it = g->batches.find(ticket);
    if (it == g->batches.end()) return AIPSTACK_CHKSUM_OK;
    for (size_t j = 0; j < todo.size(); ++j) {
        Part &p = it->second.parts[todo[j].first];
        if (!p.done) settle(p, res[j]);
    }
    const int r = finish_batch(g, it, dev_status);
    g->submitted.notify_all();  // other waits of this ticket: it is gone now
    return r;
}

// ---- submits ----------------------------------------------------------------------------

extern "C" int aipstack_chksum_engine_group_submit_strided(aipstack_chksum_engine_group *g,
                                                           const void *h_base, uint64_t stride,
                                                           uint32_t len, uint64_t n,
                                                           uint16_t *h_out, uint32_t flags,
                                                           uint64_t *ticket) {
    if (!g || !h_base || !h_out || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    *ticket = 0;
    if (len > AIPSTACK_CHKSUM_MAX_LEN) return AIPSTACK_CHKSUM_EINVAL;
    const char *b = static_cast<const char *>(h_base);
    const uint64_t span = n ? (n - 1) * stride + len : 0;
    return group_submit(g, n, b, span, [=](uint64_t i) { return i * stride; },
                        [=](size_t k, uint64_t i0, uint64_t i1, uint64_t *et) {
                            return aipstack_chksum_engine_submit_strided(
                                g->engines[k], b + i0 * stride, stride, len, i1 - i0, h_out + i0,
                                flags, et);
                        },
                        ticket);
}

namespace {
// CSR batches (checksums, Rx verdicts, Tx fills): ranges of about equal bytes.
template <class Submit>
int submit_csr_like(aipstack_chksum_engine_group *g, const void *h_base, const uint64_t *h_offsets,
                    uint64_t n, Submit submit, uint64_t *ticket) {
    *ticket = 0;
    if (!csr_ok(h_offsets, n)) return AIPSTACK_CHKSUM_EINVAL;
    const char *b = static_cast<const char *>(h_base);
    return group_submit(g, n, b + h_offsets[0], h_offsets[n] - h_offsets[0],
                        [=](uint64_t i) { return h_offsets[i] - h_offsets[0]; },
                        [=](size_t k, uint64_t i0, uint64_t i1, uint64_t *et) {
                            return submit(g->engines[k], i0, i1, et);
                        },
                        ticket);
}
}  // namespace

extern "C" int aipstack_chksum_engine_group_submit_csr(aipstack_chksum_engine_group *g,
                                                       const void *h_base,
                                                       const uint64_t *h_offsets, uint64_t n,
                                                       uint16_t *h_out, uint32_t flags,
                                                       uint64_t *ticket) {
    if (!g || !h_base || !h_offsets || !h_out || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    return submit_csr_like(g, h_base, h_offsets, n,
                           [=](aipstack_chksum_engine *e, uint64_t i0, uint64_t i1, uint64_t *et) {
                               return aipstack_chksum_engine_submit_csr(
                                   e, h_base, h_offsets + i0, i1 - i0, h_out + i0, flags, et);
                           },
                           ticket);
}

extern "C" int aipstack_chksum_engine_group_submit_rx_verify(aipstack_chksum_engine_group *g,
                                                             const void *h_base,
                                                             const uint64_t *h_offsets, uint64_t n,
                                                             uint8_t *h_verdicts, uint64_t *ticket) {
    if (!g || !h_base || !h_offsets || !h_verdicts || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    return submit_csr_like(g, h_base, h_offsets, n,
                           [=](aipstack_chksum_engine *e, uint64_t i0, uint64_t i1, uint64_t *et) {
                               return aipstack_chksum_engine_submit_rx_verify(
                                   e, h_base, h_offsets + i0, i1 - i0, h_verdicts + i0, et);
                           },
                           ticket);
}

extern "C" int aipstack_chksum_engine_group_submit_tx_fill(aipstack_chksum_engine_group *g,
                                                           void *h_base, const uint64_t *h_offsets,
                                                           uint64_t n, uint8_t *h_status,
                                                           uint64_t *ticket) {
    if (!g || !h_base || !h_offsets || !h_status || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    return submit_csr_like(g, h_base, h_offsets, n,
                           [=](aipstack_chksum_engine *e, uint64_t i0, uint64_t i1, uint64_t *et) {
                               return aipstack_chksum_engine_submit_tx_fill(
                                   e, h_base, h_offsets + i0, i1 - i0, h_status + i0, et);
                           },
                           ticket);
}

namespace {
// Ring slots: contiguous runs of about equal slot counts.
template <class Submit>
int submit_slotted_like(aipstack_chksum_engine_group *g, const void *h_base, uint64_t slot_stride,
                        const uint32_t *h_len, uint64_t n, Submit submit, uint64_t *ticket) {
    *ticket = 0;
    if (!slots_ok(slot_stride, h_len, n)) return AIPSTACK_CHKSUM_EINVAL;
    return group_submit(g, n, h_base, n * slot_stride, [=](uint64_t i) { return i * slot_stride; },
                        [=](size_t k, uint64_t i0, uint64_t i1, uint64_t *et) {
                            return submit(g->engines[k], i0, i1, et);
                        },
                        ticket);
}
}  // namespace

extern "C" int aipstack_chksum_engine_group_submit_slotted(aipstack_chksum_engine_group *g,
                                                           const void *h_base, uint64_t slot_stride,
                                                           const uint32_t *h_len, uint64_t n,
                                                           uint16_t *h_out, uint32_t flags,
                                                           uint64_t *ticket) {
    if (!g || !h_base || !h_len || !h_out || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    const char *b = static_cast<const char *>(h_base);
    return submit_slotted_like(
        g, h_base, slot_stride, h_len, n,
        [=](aipstack_chksum_engine *e, uint64_t i0, uint64_t i1, uint64_t *et) {
            return aipstack_chksum_engine_submit_slotted(e, b + i0 * slot_stride, slot_stride,
                                                         h_len + i0, i1 - i0, h_out + i0, flags,
                                                         et);
        },
        ticket);
}

extern "C" int aipstack_chksum_engine_group_submit_rx_verify_slotted(
    aipstack_chksum_engine_group *g, const void *h_base, uint64_t slot_stride,
    const uint32_t *h_len, uint64_t n, uint8_t *h_verdicts, uint64_t *ticket) {
    if (!g || !h_base || !h_len || !h_verdicts || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    *ticket = 0;
    if (slot_stride > AIPSTACK_CHKSUM_MAX_SLOT_STRIDE)
        return AIPSTACK_CHKSUM_EINVAL;
    const char *b = static_cast<const char *>(h_base);
    return submit_slotted_like(
        g, h_base, slot_stride, h_len, n,
        [=](aipstack_chksum_engine *e, uint64_t i0, uint64_t i1, uint64_t *et) {
            return aipstack_chksum_engine_submit_rx_verify_slotted(
                e, b + i0 * slot_stride, slot_stride, h_len + i0, i1 - i0, h_verdicts + i0, et);
        },
        ticket);
}

extern "C" int aipstack_chksum_engine_group_submit_tx_fill_slotted(
    aipstack_chksum_engine_group *g, void *h_base, uint64_t slot_stride, const uint32_t *h_len,
    uint64_t n, uint8_t *h_status, uint64_t *ticket) {
    if (!g || !h_base || !h_len || !h_status || !ticket) return AIPSTACK_CHKSUM_EINVAL;
    *ticket = 0;
    if (slot_stride > AIPSTACK_CHKSUM_MAX_SLOT_STRIDE)
        return AIPSTACK_CHKSUM_EINVAL;
    char *b = static_cast<char *>(h_base);
    return submit_slotted_like(
        g, h_base, slot_stride, h_len, n,
        [=](aipstack_chksum_engine *e, uint64_t i0, uint64_t i1, uint64_t *et) {
            return aipstack_chksum_engine_submit_tx_fill_slotted(
                e, b + i0 * slot_stride, slot_stride, h_len + i0, i1 - i0, h_status + i0, et);
        },
        ticket);
}

// ---- synchronous forms: submit + wait ----------------------------------------------------

extern "C" int aipstack_chksum_engine_group_host_strided(aipstack_chksum_engine_group *g,
                                                         const void *h_base, uint64_t stride,
                                                         uint32_t len, uint64_t n, uint16_t *h_out,
                                                         uint32_t flags, int *dev_status) {
    if (!g || !h_base || !h_out || len > AIPSTACK_CHKSUM_MAX_LEN) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_group_submit_strided(g, h_base, stride, len, n, h_out,
                                                               flags, &t);
    return sync_call(g, st, t, dev_status);
}

extern "C" int aipstack_chksum_engine_group_host_csr(aipstack_chksum_engine_group *g,
                                                     const void *h_base, const uint64_t *h_offsets,
                                                     uint64_t n, uint16_t *h_out, uint32_t flags,
                                                     int *dev_status) {
    if (!g || !h_base || !h_offsets || !h_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_group_submit_csr(g, h_base, h_offsets, n, h_out, flags, &t);
    return sync_call(g, st, t, dev_status);
}

extern "C" int aipstack_chksum_engine_group_host_rx_verify(aipstack_chksum_engine_group *g,
                                                           const void *h_base,
                                                           const uint64_t *h_offsets, uint64_t n,
                                                           uint8_t *h_verdicts, int *dev_status) {
    if (!g || !h_base || !h_offsets || !h_verdicts) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_group_submit_rx_verify(g, h_base, h_offsets, n,
                                                                 h_verdicts, &t);
    return sync_call(g, st, t, dev_status);
}

extern "C" int aipstack_chksum_engine_group_host_tx_fill(aipstack_chksum_engine_group *g,
                                                         void *h_base, const uint64_t *h_offsets,
                                                         uint64_t n, uint8_t *h_status,
                                                         int *dev_status) {
    if (!g || !h_base || !h_offsets || !h_status) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_group_submit_tx_fill(g, h_base, h_offsets, n, h_status, &t);
    return sync_call(g, st, t, dev_status);
}

extern "C" int aipstack_chksum_engine_group_host_slotted(aipstack_chksum_engine_group *g,
                                                         const void *h_base, uint64_t slot_stride,
                                                         const uint32_t *h_len, uint64_t n,
                                                         uint16_t *h_out, uint32_t flags,
                                                         int *dev_status) {
    if (!g || !h_base || !h_len || !h_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_group_submit_slotted(g, h_base, slot_stride, h_len, n,
                                                               h_out, flags, &t);
    return sync_call(g, st, t, dev_status);
}

extern "C" int aipstack_chksum_engine_group_host_rx_verify_slotted(
    aipstack_chksum_engine_group *g, const void *h_base, uint64_t slot_stride,
    const uint32_t *h_len, uint64_t n, uint8_t *h_verdicts, int *dev_status) {
    if (!g || !h_base || !h_len || !h_verdicts) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_group_submit_rx_verify_slotted(g, h_base, slot_stride,
                                                                         h_len, n, h_verdicts, &t);
    return sync_call(g, st, t, dev_status);
}

extern "C" int aipstack_chksum_engine_group_host_tx_fill_slotted(
    aipstack_chksum_engine_group *g, void *h_base, uint64_t slot_stride, const uint32_t *h_len,
    uint64_t n, uint8_t *h_status, int *dev_status) {
    if (!g || !h_base || !h_len || !h_status) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    uint64_t t = 0;
    const int st = aipstack_chksum_engine_group_submit_tx_fill_slotted(g, h_base, slot_stride,
                                                                       h_len, n, h_status, &t);
    return sync_call(g, st, t, dev_status);
}
