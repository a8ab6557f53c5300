// aipstack_amd -- host runtime of libaipstack_chksum.so:
//   * the per-packet link-time hook IpChksumInverted (reference Chksum.h:50-51, 77-99),
//   * status / diagnostics entry points of include/aipstack_amd/chksum.h,
//   * the device-property cache used by the kernel launchers.
//
// IpChksumInverted here is the HOST implementation of the hook (a GPU launch costs more
// than one packet's scalar sum). It is not a fallback for the batch entry points: those
// only ever run the HIP kernels.

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

inline uint64_t load_le64(const unsigned char *p) {
    uint64_t v;
    std::memcpy(&v, p, 8);  // x86-64 / little-endian host
    return v;
}
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

// Inverted Internet checksum of data[0..len), host side.
// Sums little-endian 32-bit words taken from `data` into a 64-bit accumulator (len <=
// 65535 gives < 2^46, far from overflow), then folds to 16 bits and byte-swaps: words
// paired little-endian from `data` put data[2i] in the LOW byte, where the reference's
// big-endian pairing (Chksum.h:85-88) puts it in the HIGH byte, and the swap is exactly
// multiplication by 256 mod 0xFFFF. A trailing partial word is zero-padded, which is
// the reference's odd-tail rule (Chksum.h:90-93). Folding keeps nonzero sums nonzero, so
// 0 is returned only for all-zero input, as by the reference.
extern "C" uint16_t IpChksumInverted(const char *data, size_t len) {
    const unsigned char *p = reinterpret_cast<const unsigned char *>(data);
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    size_t i = 0;
    for (; i + 32 <= len; i += 32) {
        const uint64_t w0 = load_le64(p + i), w1 = load_le64(p + i + 8);
        const uint64_t w2 = load_le64(p + i + 16), w3 = load_le64(p + i + 24);
        a0 += (w0 & 0xFFFFFFFFu) + (w0 >> 32);
        a1 += (w1 & 0xFFFFFFFFu) + (w1 >> 32);
        a2 += (w2 & 0xFFFFFFFFu) + (w2 >> 32);
        a3 += (w3 & 0xFFFFFFFFu) + (w3 >> 32);
    }
    for (; i + 8 <= len; i += 8) {
        const uint64_t w = load_le64(p + i);
        a0 += (w & 0xFFFFFFFFu) + (w >> 32);
    }
    if (i < len) {
        unsigned char tail[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        std::memcpy(tail, p + i, len - i);
        const uint64_t w = load_le64(tail);
        a1 += (w & 0xFFFFFFFFu) + (w >> 32);
    }
    uint64_t s = a0 + a1 + a2 + a3;
    s = (s & 0xFFFFFFFFu) + (s >> 32);
    s = (s & 0xFFFFFFFFu) + (s >> 32);
    uint32_t t = (uint32_t)s;
    t = (t & 0xFFFFu) + (t >> 16);
    t = (t & 0xFFFFu) + (t >> 16);
    return (uint16_t)(((t & 0xFFu) << 8) | (t >> 8));
}

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
