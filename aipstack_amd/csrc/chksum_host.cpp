// aipstack_amd -- host runtime of libaipstack_chksum.so:
//   * status / diagnostics entry points of include/aipstack_amd/chksum.h,
//   * the device-property cache used by the kernel launchers.
// (The per-packet host hook IpChksumInverted is in host_hook.cc, compiled as plain C++.)

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "aipstack_amd/chksum.h"
#include "chksum_internal.h"

namespace aipstack_amd {

namespace {
thread_local int g_last_hip_error = 0;
}  // namespace

int check_hip(hipError_t e) {
    if (e == hipSuccess) return AIPSTACK_CHKSUM_OK;
    g_last_hip_error = (int)e;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu)
        return AIPSTACK_CHKSUM_ENODEV;
    return AIPSTACK_CHKSUM_EHIP;
}

int device_cu_count(hipStream_t stream) {
    // Keyed by the device the launch stream belongs to (a stream of device 1 launched
    // while device 0 is current sizes its grid for device 1). Any thread may launch, so
    // the cache entries are atomics; two threads filling one entry store the same value.
    constexpr int kMaxDev = 64;
    static std::atomic<int> cache[kMaxDev];
    hipDevice_t dev = -1;
    if (stream != nullptr) {
        if (hipStreamGetDevice(stream, &dev) != hipSuccess) return -1;
    } else if (hipGetDevice(&dev) != hipSuccess) {
        return -1;
    }
    if (dev < 0) return -1;
    if (dev < kMaxDev) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0) return c;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -1;
    if (dev < kMaxDev) cache[dev].store(cus, std::memory_order_relaxed);
    return cus;
}

}  // namespace aipstack_amd

using namespace aipstack_amd;

extern "C" const char *aipstack_chksum_strerror(int status) {
    switch (status) {
        case AIPSTACK_CHKSUM_OK: return "ok";
        case AIPSTACK_CHKSUM_EINVAL: return "invalid argument";
        case AIPSTACK_CHKSUM_EHIP: return "HIP runtime error";
        case AIPSTACK_CHKSUM_ENODEV: return "no usable gfx950 device";
        default: return "unknown status";
    }
}

extern "C" int aipstack_chksum_last_hip_error(void) { return g_last_hip_error; }

extern "C" int aipstack_chksum_abi_version(void) { return AIPSTACK_CHKSUM_ABI_VERSION; }

// Generated at build time from the library's sources (Makefile: build/source_digest.h).
#include "build/source_digest.h"
extern "C" const char *aipstack_chksum_source_digest(void) { return AIPSTACK_SOURCE_DIGEST; }

extern "C" int aipstack_chksum_device_check(int device) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess) return check_hip(e);
    if (device < 0 || device >= count) return AIPSTACK_CHKSUM_ENODEV;
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return check_hip(e);
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return AIPSTACK_CHKSUM_ENODEV;
    return AIPSTACK_CHKSUM_OK;
}

extern "C" int aipstack_chksum_contract_violations(int device, uint32_t *mask, int clear) {
    if (!mask) return AIPSTACK_CHKSUM_EINVAL;
    const int dc = aipstack_chksum_device_check(device);
    if (dc != AIPSTACK_CHKSUM_OK) return dc;
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) prev = device;
    int st = check_hip(hipSetDevice(device));
    if (st == AIPSTACK_CHKSUM_OK) st = check_hip(hipDeviceSynchronize());
    uint32_t m = 0;
    if (st == AIPSTACK_CHKSUM_OK) st = take_violations_batch(&m, clear != 0);
    if (st == AIPSTACK_CHKSUM_OK) st = take_violations_frames(&m, clear != 0);
    (void)hipSetDevice(prev);
    if (st == AIPSTACK_CHKSUM_OK) *mask = m;
    return st;
}
