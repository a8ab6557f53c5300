// aipstack_amd -- several devices behind one host-memory batch, in ONE process.
//
// The reference stack runs in one process on one event-loop thread (reference
// event_loop/event_loop.dox:48-50), so it cannot use the one-process-per-GPU launch the bench
// uses for device-resident shards. A host batch that arrives through host memory is PCIe-bound
// (~52 GiB/s per device link); spreading it over several devices' links is how the
// engine outruns the host's own cores on host-resident data. The group owns one engine per
// device (each with its own streams and pinned staging), splits every batch into disjoint
// contiguous ranges of about equal bytes, runs each range on its engine from its own host
// thread, and joins, reporting each device's status.
//
// There is no data exchange between the devices: each range is an independent batch (SURVEY
// 8(e): disjoint packet ranges, no collective).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "aipstack_amd/chksum.h"
#include "chksum_internal.h"

using namespace aipstack_amd;

struct aipstack_chksum_engine_group {
    std::vector<aipstack_chksum_engine *> engines;
    std::vector<int> devices;
    std::vector<const void *> regions;  // page-locked by the group (portable)
    std::mutex mu;                      // serialises the group's calls
};

namespace {

// Packet ranges [cut[k], cut[k+1]) per engine, about equal bytes each: `bytes_before(i)` is the
// byte position of packet i (non-decreasing, bytes_before(n) = total).
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

// Runs run(k, i0, i1) for every engine's range on its own thread; joins; per-engine status
// into dev_status (if given); returns the first failure, else _OK.
template <class Run>
int fan_out(aipstack_chksum_engine_group *g, const std::vector<uint64_t> &cut, int *dev_status,
            Run run) {
    const size_t m = g->engines.size();
    std::vector<int> st(m, AIPSTACK_CHKSUM_OK);
    std::vector<std::thread> pool;
    pool.reserve(m);
    for (size_t k = 0; k < m; ++k) {
        if (cut[k + 1] == cut[k]) continue;  // nothing for this device
        pool.emplace_back([&, k] { st[k] = run(k, cut[k], cut[k + 1]); });
    }
    for (std::thread &t : pool) t.join();
    int first = AIPSTACK_CHKSUM_OK;
    for (size_t k = 0; k < m; ++k) {
        if (dev_status) dev_status[k] = st[k];
        if (first == AIPSTACK_CHKSUM_OK && st[k] != AIPSTACK_CHKSUM_OK) first = st[k];
    }
    return first;
}

bool csr_ok(const uint64_t *off, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > AIPSTACK_CHKSUM_MAX_LEN) return false;
    return true;
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
    *out = g;
    return AIPSTACK_CHKSUM_OK;
}

extern "C" void aipstack_chksum_engine_group_destroy(aipstack_chksum_engine_group *g) {
    if (!g) return;
    {
        std::lock_guard<std::mutex> lock(g->mu);
        for (aipstack_chksum_engine *e : g->engines) aipstack_chksum_engine_destroy(e);
        for (const void *p : g->regions) (void)hipHostUnregister(const_cast<void *>(p));
        g->regions.clear();
        g->engines.clear();
    }
    delete g;  // after the lock is released (its mutex is a member)
}

extern "C" int aipstack_chksum_engine_group_size(const aipstack_chksum_engine_group *g) {
    return g ? (int)g->engines.size() : AIPSTACK_CHKSUM_EINVAL;
}

extern "C" int aipstack_chksum_engine_group_register(aipstack_chksum_engine_group *g,
                                                     void *host_ptr, uint64_t bytes) {
    if (!g || !host_ptr || bytes == 0) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard dg(g->devices[0]);
    if (!dg.ok) return AIPSTACK_CHKSUM_ENODEV;
    const int st = check_hip(hipHostRegister(host_ptr, bytes, hipHostRegisterPortable));
    if (st != AIPSTACK_CHKSUM_OK) return st;
    g->regions.push_back(host_ptr);
    for (aipstack_chksum_engine *e : g->engines) engine_adopt_region(e, host_ptr, bytes);
    return AIPSTACK_CHKSUM_OK;
}

extern "C" int aipstack_chksum_engine_group_unregister(aipstack_chksum_engine_group *g,
                                                       void *host_ptr) {
    if (!g || !host_ptr) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto it = std::find(g->regions.begin(), g->regions.end(), host_ptr);
    if (it == g->regions.end()) return AIPSTACK_CHKSUM_EINVAL;
    for (aipstack_chksum_engine *e : g->engines) engine_drop_region(e, host_ptr);
    g->regions.erase(it);
    return check_hip(hipHostUnregister(host_ptr));
}

extern "C" int aipstack_chksum_engine_group_host_strided(aipstack_chksum_engine_group *g,
                                                         const void *h_base, uint64_t stride,
                                                         uint32_t len, uint64_t n, uint16_t *h_out,
                                                         uint32_t flags, int *dev_status) {
    if (!g || !h_base || !h_out || len > AIPSTACK_CHKSUM_MAX_LEN) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto cut = split(n, g->engines.size(), [&](uint64_t i) { return i * stride; });
    const char *b = static_cast<const char *>(h_base);
    return fan_out(g, cut, dev_status, [&](size_t k, uint64_t i0, uint64_t i1) {
        return aipstack_chksum_engine_host_strided(g->engines[k], b + i0 * stride, stride, len,
                                                   i1 - i0, h_out + i0, flags);
    });
}

extern "C" int aipstack_chksum_engine_group_host_csr(aipstack_chksum_engine_group *g,
                                                     const void *h_base, const uint64_t *h_offsets,
                                                     uint64_t n, uint16_t *h_out, uint32_t flags,
                                                     int *dev_status) {
    if (!g || !h_base || !h_offsets || !h_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!csr_ok(h_offsets, n)) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto cut = split(n, g->engines.size(), [&](uint64_t i) { return h_offsets[i]; });
    return fan_out(g, cut, dev_status, [&](size_t k, uint64_t i0, uint64_t i1) {
        return aipstack_chksum_engine_host_csr(g->engines[k], h_base, h_offsets + i0, i1 - i0,
                                               h_out + i0, flags);
    });
}

extern "C" int aipstack_chksum_engine_group_host_rx_verify(aipstack_chksum_engine_group *g,
                                                           const void *h_base,
                                                           const uint64_t *h_offsets, uint64_t n,
                                                           uint8_t *h_verdicts, int *dev_status) {
    if (!g || !h_base || !h_offsets || !h_verdicts) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!csr_ok(h_offsets, n)) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto cut = split(n, g->engines.size(), [&](uint64_t i) { return h_offsets[i]; });
    return fan_out(g, cut, dev_status, [&](size_t k, uint64_t i0, uint64_t i1) {
        return aipstack_chksum_engine_host_rx_verify(g->engines[k], h_base, h_offsets + i0,
                                                     i1 - i0, h_verdicts + i0);
    });
}

extern "C" int aipstack_chksum_engine_group_host_tx_fill(aipstack_chksum_engine_group *g,
                                                         void *h_base, const uint64_t *h_offsets,
                                                         uint64_t n, uint8_t *h_status,
                                                         int *dev_status) {
    if (!g || !h_base || !h_offsets || !h_status) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!csr_ok(h_offsets, n)) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto cut = split(n, g->engines.size(), [&](uint64_t i) { return h_offsets[i]; });
    return fan_out(g, cut, dev_status, [&](size_t k, uint64_t i0, uint64_t i1) {
        return aipstack_chksum_engine_host_tx_fill(g->engines[k], h_base, h_offsets + i0, i1 - i0,
                                                   h_status + i0);
    });
}

// Ring slots (frame i = h_len[i] bytes at h_base + i * slot_stride): contiguous runs of slots
// per device, about equal slot counts. Every length is checked before any device starts.
namespace {
bool slots_ok(uint64_t slot_stride, const uint32_t *h_len, uint64_t n) {
    if (slot_stride == 0) return false;
    const uint64_t cap = std::min<uint64_t>(slot_stride, AIPSTACK_CHKSUM_MAX_LEN);
    for (uint64_t i = 0; i < n; ++i)
        if (h_len[i] > cap) return false;
    return true;
}
}  // namespace

extern "C" int aipstack_chksum_engine_group_host_slotted(aipstack_chksum_engine_group *g,
                                                         const void *h_base, uint64_t slot_stride,
                                                         const uint32_t *h_len, uint64_t n,
                                                         uint16_t *h_out, uint32_t flags,
                                                         int *dev_status) {
    if (!g || !h_base || !h_len || !h_out) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!slots_ok(slot_stride, h_len, n)) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto cut = split(n, g->engines.size(), [&](uint64_t i) { return i * slot_stride; });
    const char *b = static_cast<const char *>(h_base);
    return fan_out(g, cut, dev_status, [&](size_t k, uint64_t i0, uint64_t i1) {
        return aipstack_chksum_engine_host_slotted(g->engines[k], b + i0 * slot_stride,
                                                   slot_stride, h_len + i0, i1 - i0, h_out + i0,
                                                   flags);
    });
}

extern "C" int aipstack_chksum_engine_group_host_rx_verify_slotted(
    aipstack_chksum_engine_group *g, const void *h_base, uint64_t slot_stride,
    const uint32_t *h_len, uint64_t n, uint8_t *h_verdicts, int *dev_status) {
    if (!g || !h_base || !h_len || !h_verdicts) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!slots_ok(slot_stride, h_len, n)) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto cut = split(n, g->engines.size(), [&](uint64_t i) { return i * slot_stride; });
    const char *b = static_cast<const char *>(h_base);
    return fan_out(g, cut, dev_status, [&](size_t k, uint64_t i0, uint64_t i1) {
        return aipstack_chksum_engine_host_rx_verify_slotted(g->engines[k], b + i0 * slot_stride,
                                                             slot_stride, h_len + i0, i1 - i0,
                                                             h_verdicts + i0);
    });
}

extern "C" int aipstack_chksum_engine_group_host_tx_fill_slotted(
    aipstack_chksum_engine_group *g, void *h_base, uint64_t slot_stride, const uint32_t *h_len,
    uint64_t n, uint8_t *h_status, int *dev_status) {
    if (!g || !h_base || !h_len || !h_status) return AIPSTACK_CHKSUM_EINVAL;
    if (n == 0) return AIPSTACK_CHKSUM_OK;
    if (!slots_ok(slot_stride, h_len, n)) return AIPSTACK_CHKSUM_EINVAL;
    std::lock_guard<std::mutex> lock(g->mu);
    const auto cut = split(n, g->engines.size(), [&](uint64_t i) { return i * slot_stride; });
    char *b = static_cast<char *>(h_base);
    return fan_out(g, cut, dev_status, [&](size_t k, uint64_t i0, uint64_t i1) {
        return aipstack_chksum_engine_host_tx_fill_slotted(g->engines[k], b + i0 * slot_stride,
                                                           slot_stride, h_len + i0, i1 - i0,
                                                           h_status + i0);
    });
}
