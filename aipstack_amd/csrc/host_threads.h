// aipstack_amd -- the host threads of the engines: device locality (which CPUs and NUMA node sit
// next to a GPU) and a persistent pool of pinned worker threads.
//
// The engine's host work -- pageable input copied into pinned staging, Tx records applied to
// the caller's frames -- touches tens of MiB per piece and is memory-bound on the host; it runs
// best on the cores of the NUMA node the device hangs off (its staging is allocated there), on
// threads that live as long as the engine instead of being spawned per piece.
#ifndef AIPSTACK_AMD_HOST_THREADS_H
#define AIPSTACK_AMD_HOST_THREADS_H

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <thread>
#include <memory>
#include <type_traits>
#include <vector>

namespace aipstack_amd {

// Where a device sits: its PCI address, the NUMA node the kernel reports for it (-1 unknown)
// and its local CPUs (sysfs local_cpulist) that this process may run on (empty: unknown, or
// none allowed -- then nothing is pinned).
struct DeviceLocality {
    char pci[32] = {0};
    int numa_node = -1;
    std::vector<int> cpus;
};
DeviceLocality device_locality(int device);

// Parses a sysfs CPU list ("0-15,128-143"); empty on a malformed list.
std::vector<int> parse_cpu_list(const char *s);

// Pins the calling thread to `cpus` (no-op for an empty list); returns whether it did.
bool pin_current_thread(const std::vector<int> &cpus);

// Runs the scope on `cpus` and restores the thread's previous affinity afterwards (the
// engine allocates its pinned staging inside one, so that its pages come from the device's
// node under the default first-touch policy).
class ScopedAffinity {
public:
    explicit ScopedAffinity(const std::vector<int> &cpus);
    ~ScopedAffinity();
    ScopedAffinity(const ScopedAffinity &) = delete;
    ScopedAffinity &operator=(const ScopedAffinity &) = delete;

private:
    std::vector<unsigned char> saved_;  // the previous cpu_set_t, if it was changed
};

// A fixed set of worker threads, started once (pinned to `cpus` when given). run(parts, fn)
// calls fn(0) .. fn(parts - 1) and returns when all are done: the caller runs parts itself too
// (so a busy pool never stalls it), the workers take the others. Several threads may run()
// on one pool at once (the engine's submitting thread stages while its applier applies).
class HostPool {
public:
    HostPool() = default;
    ~HostPool() { stop(); }
    HostPool(const HostPool &) = delete;
    HostPool &operator=(const HostPool &) = delete;

    void start(unsigned workers, const std::vector<int> &cpus);
    void stop();
    unsigned workers() const { return (unsigned)threads_.size(); }

    template <class F>
    void run(unsigned parts, F &&fn) {
        if (parts == 0) return;
        if (parts == 1 || threads_.empty()) {
            for (unsigned p = 0; p < parts; ++p) fn(p);
            return;
        }
        // (F may deduce to an lvalue reference, possibly const: point at the object itself)
        using Fn = std::remove_reference_t<F>;
        Job job{[](void *f, unsigned p) { (*static_cast<Fn *>(f))(p); },
                const_cast<void *>(static_cast<const void *>(std::addressof(fn))), parts - 1};
        {
            std::lock_guard<std::mutex> lock(mu_);
            for (unsigned p = 1; p < parts; ++p) tasks_.push_back(Task{&job, p});
        }
        work_.notify_all();
        fn(0);
        help_until_done(job);
    }

private:
    struct Job {
        void (*call)(void *, unsigned);
        void *fn;
        unsigned left;  // parts not yet finished (guarded by mu_)
    };
    struct Task {
        Job *job;
        unsigned part;
    };
    void help_until_done(Job &job);
    void worker_loop();
    void finish(Task t);

    std::mutex mu_;
    std::condition_variable work_, done_;
    std::deque<Task> tasks_;
    std::vector<std::thread> threads_;
    std::vector<int> cpus_;
    bool stop_ = false;
};

}  // namespace aipstack_amd

#endif
