// FETCH_SIZE calibration by access width (tools only). MI355X_MICROARCH.md
// calibrates FETCH_SIZE for wide coalesced streaming reads only: it reports half their bytes,
// hence the x2 in tools/pmc_summary.py. The batch kernels also read their CSR offsets, chunk
// tables and chain states with 4- and 8-byte coalesced loads, and the chain bench's 20-byte
// header nodes as 32-byte pieces of 128-byte lines. Each kernel below reads a 1 GiB buffer
// (four times the Infinity Cache) once, one pattern per kernel:
//   w4 / w8 / w16    every byte, 4 / 8 / 16 bytes per lane, coalesced
//   s32 / s64        one 32- / 64-byte piece of every 128-byte line (16 B per lane)
// Run under rocprofv3 --kernel-trace --pmc FETCH_SIZE and compare FETCH_SIZE x 1024 with the
// bytes each kernel prints.
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/width_calib tools/width_calib.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr uint64_t kBytes = 1ull << 30;

template <int W>
__global__ __launch_bounds__(256) void dense_kernel(const uint8_t *__restrict__ p, uint32_t *out) {
    const uint64_t n = kBytes / W;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        if constexpr (W == 4) acc ^= reinterpret_cast<const uint32_t *>(p)[i];
        if constexpr (W == 8) { const u32x2 v = reinterpret_cast<const u32x2 *>(p)[i]; acc ^= v[0] ^ v[1]; }
        if constexpr (W == 16) { const u32x4 v = reinterpret_cast<const u32x4 *>(p)[i]; acc ^= v[0] ^ v[1] ^ v[2] ^ v[3]; }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// PIECE bytes (32 or 64) at the start of every 128-byte line, 16 B per lane.
template <int PIECE>
__global__ __launch_bounds__(256) void sparse_kernel(const uint8_t *__restrict__ p, uint32_t *out) {
    constexpr int kLanesPerLine = PIECE / 16;
    const uint64_t n = kBytes / 128 * kLanesPerLine;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t line = i / kLanesPerLine, k = i % kLanesPerLine;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(p + line * 128 + k * 16);
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <class K>
int run(const char *name, K kernel, const uint8_t *d, uint32_t *out, uint64_t bytes) {
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(kernel, dim3(8192), dim3(256), 0, 0, d, out);
        CK(hipGetLastError());
    }
    CK(hipDeviceSynchronize());
    printf("{\"kernel\": \"%s\", \"bytes_read\": %llu}\n", name, (unsigned long long)bytes);
    return 0;
}

int main() {
    uint8_t *d; uint32_t *out;
    CK(hipMalloc(&d, kBytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(d, 1, kBytes));
    CK(hipDeviceSynchronize());
    if (run("w4", dense_kernel<4>, d, out, kBytes)) return 1;
    if (run("w8", dense_kernel<8>, d, out, kBytes)) return 1;
    if (run("w16", dense_kernel<16>, d, out, kBytes)) return 1;
    if (run("s32", sparse_kernel<32>, d, out, kBytes / 4)) return 1;
    if (run("s64", sparse_kernel<64>, d, out, kBytes / 2)) return 1;
    return 0;
}
