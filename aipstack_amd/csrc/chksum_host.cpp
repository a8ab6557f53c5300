// aipstack_amd -- host runtime of libaipstack_chksum.so:
//   * status / diagnostics entry points of include/aipstack_amd/chksum.h,
//   * the device-property cache used by the kernel launchers.
// (The per-packet host hook IpChksumInverted is in host_hook.cc, compiled as plain C++.)

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <mutex>

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

int device_cu_count() {
    constexpr int kMaxDev = 64;
    static int cache[kMaxDev] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return -1;
    if (dev < kMaxDev && cache[dev] > 0) return cache[dev];
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return -1;
    if (dev < kMaxDev) cache[dev] = cus;
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
