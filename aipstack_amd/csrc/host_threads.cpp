// aipstack_amd -- device locality and the engines' persistent host worker pool (host_threads.h).
#include "host_threads.h"

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace aipstack_amd {

std::vector<int> parse_cpu_list(const char *s) {
    std::vector<int> cpus;
    while (s && *s && *s != '\n') {
        char *end = nullptr;
        const long a = std::strtol(s, &end, 10);
        if (end == s || a < 0) return {};
        long b = a;
        s = end;
        if (*s == '-') {
            b = std::strtol(s + 1, &end, 10);
            if (end == s + 1 || b < a) return {};
            s = end;
        }
        if (b >= CPU_SETSIZE) return {};
        for (long c = a; c <= b; ++c) cpus.push_back((int)c);
        if (*s == ',') ++s;
        else if (*s && *s != '\n') return {};
    }
    return cpus;
}

namespace {
bool read_line(const char *path, char *buf, size_t n) {
    FILE *f = std::fopen(path, "r");
    if (!f) return false;
    const bool ok = std::fgets(buf, (int)n, f) != nullptr;
    std::fclose(f);
    return ok;
}
}  // namespace

DeviceLocality device_locality(int device) {
    DeviceLocality loc;
    if (hipDeviceGetPCIBusId(loc.pci, (int)sizeof(loc.pci), device) != hipSuccess) {
        (void)hipGetLastError();
        loc.pci[0] = 0;
        return loc;
    }
    for (char *c = loc.pci; *c; ++c) *c = (char)std::tolower((unsigned char)*c);
    char path[128], line[4096];
    std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", loc.pci);
    if (read_line(path, line, sizeof(line))) loc.numa_node = std::atoi(line);
    if (loc.numa_node < 0) loc.numa_node = -1;
    std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/local_cpulist", loc.pci);
    if (!read_line(path, line, sizeof(line))) return loc;
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return loc;
    for (int c : parse_cpu_list(line))
        if (CPU_ISSET(c, &allowed)) loc.cpus.push_back(c);
    return loc;
}

bool pin_current_thread(const std::vector<int> &cpus) {
    if (cpus.empty()) return false;
    cpu_set_t set;
    CPU_ZERO(&set);
    for (int c : cpus) CPU_SET(c, &set);
    return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

ScopedAffinity::ScopedAffinity(const std::vector<int> &cpus) {
    if (cpus.empty()) return;
    cpu_set_t prev;
    CPU_ZERO(&prev);
    if (pthread_getaffinity_np(pthread_self(), sizeof(prev), &prev) != 0) return;
    if (!pin_current_thread(cpus)) return;
    saved_.resize(sizeof(prev));
    std::memcpy(saved_.data(), &prev, sizeof(prev));
}

ScopedAffinity::~ScopedAffinity() {
    if (saved_.empty()) return;
    cpu_set_t prev;
    std::memcpy(&prev, saved_.data(), sizeof(prev));
    (void)pthread_setaffinity_np(pthread_self(), sizeof(prev), &prev);
}

void HostPool::start(unsigned workers, const std::vector<int> &cpus) {
    cpus_ = cpus;
    stop_ = false;
    for (unsigned i = 0; i < workers; ++i) threads_.emplace_back([this] { worker_loop(); });
}

void HostPool::stop() {
    {
        std::lock_guard<std::mutex> lock(mu_);
        stop_ = true;
    }
    work_.notify_all();
    for (std::thread &t : threads_) t.join();
    threads_.clear();
}

void HostPool::finish(Task t) {
    std::lock_guard<std::mutex> lock(mu_);
    if (--t.job->left == 0) done_.notify_all();
}

void HostPool::worker_loop() {
    pin_current_thread(cpus_);
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
        work_.wait(lock, [this] { return stop_ || !tasks_.empty(); });
        if (tasks_.empty()) return;  // stop, and nothing queued
        const Task t = tasks_.front();
        tasks_.pop_front();
        lock.unlock();
        t.job->call(t.job->fn, t.part);
        finish(t);
        lock.lock();
    }
}

// The caller of run(): takes queued parts (its own or another run's) while its job is not
// done, so it never just sleeps behind workers busy with someone else's parts.
void HostPool::help_until_done(Job &job) {
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
        if (job.left == 0) return;
        if (!tasks_.empty()) {
            const Task t = tasks_.front();
            tasks_.pop_front();
            lock.unlock();
            t.job->call(t.job->fn, t.part);
            finish(t);
            lock.lock();
            continue;
        }
        done_.wait(lock, [&] { return job.left == 0 || !tasks_.empty(); });
    }
}

}  // namespace aipstack_amd
