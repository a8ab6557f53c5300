// Writers and a pure reader for the fresh-data experiments (tools/fresh.py):
// what does the first read of a batch cost right after something wrote it, and which
// writer / which reader pays? Not part of the product. Built as a shared library that
// tools/fresh.py loads with ctypes (every entry point is stream-ordered, no allocation).
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/build/libfresh_probe.so tools/fresh_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {

// Pure read in the column-run kernel's shape: one 12 KiB run per wave, 8 windows of 16-byte
// buffer loads in flight, folded into one word (stored only on a practically impossible
// value, so the loads stay live). MODE 0: nontemporal stream; 1: the stream at the default
// cache policy; 2: nontemporal stream plus, before it, 9 default-policy segment loads per
// wave (lanes 0..8, segments 85 apart: the column runs' boundary loads); 3: the same 9 loads
// nontemporal; 4: the 9 default-policy loads issued after the stream.
template <int MODE>
__global__ __launch_bounds__(256) void read_kernel(const u32x4 *__restrict__ p, uint64_t n16,
                                                   uint32_t *out) {
    constexpr uint64_t kPerWave = 768;
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t i = wave * kPerWave;
    if (i >= n16) return;
    const uint64_t end = min(i + kPerWave, n16);
    uint32_t acc = 0;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(p + i), (short)0,
                                                                 (int)((end - i) * 16), 0x00020000);
    u32x4 b = {0u, 0u, 0u, 0u};
    if (MODE == 2 && lane < 9) b = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 85 * 16, 0, 0);
    if (MODE == 3 && lane < 9) b = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 85 * 16, 0, 2);
    for (uint32_t off = 0; i + off < end; off += 64 * 8) {
        u32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (lane + u * 64) * 16, off * 16,
                                                         MODE == 1 ? 0 : 2);
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= v[u][0] + v[u][1] + v[u][2] + v[u][3];
    }
    if (MODE == 4 && lane < 9) b = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 85 * 16, 0, 0);
    acc += b[0] ^ b[3];
    if (acc == 0x9E3779B9u) out[wave & 0xFFFF] = acc;
}

// Rewrite one dword every `step` bytes with its own value (a real store: the line is written
// and dirtied, the data unchanged). Grid-stride.
__global__ __launch_bounds__(256) void touch_kernel(uint32_t *__restrict__ p, uint64_t ndw,
                                                    uint64_t step_dw) {
    const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t * step_dw < ndw; t += nt) {
        volatile uint32_t *q = p + t * step_dw;
        *q = *q;
    }
}

// Copy 16 bytes per thread (dst and src 16-aligned, n16 segments); nt = nontemporal stores.
template <bool NT>
__global__ __launch_bounds__(256) void copy_kernel(u32x4 *__restrict__ dst,
                                                   const u32x4 *__restrict__ src, uint64_t n16) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n16) return;
    const u32x4 v = __builtin_nontemporal_load(src + t);
    if (NT)
        __builtin_nontemporal_store(v, dst + t);
    else
        dst[t] = v;
}

unsigned blocks_for(uint64_t threads) { return (unsigned)((threads + 255) / 256); }

}  // namespace

extern "C" int fp_read(const void *buf, uint64_t nbytes, void *scratch, int mode, void *stream) {
    const uint64_t n16 = nbytes / 16;
    const uint64_t waves = (n16 + 767) / 768;
    const dim3 grid((unsigned)((waves + 3) / 4));
    const hipStream_t s = (hipStream_t)stream;
    const u32x4 *b = (const u32x4 *)buf;
    uint32_t *o = (uint32_t *)scratch;
    switch (mode) {
    case 0: hipLaunchKernelGGL(read_kernel<0>, grid, dim3(256), 0, s, b, n16, o); break;
    case 1: hipLaunchKernelGGL(read_kernel<1>, grid, dim3(256), 0, s, b, n16, o); break;
    case 2: hipLaunchKernelGGL(read_kernel<2>, grid, dim3(256), 0, s, b, n16, o); break;
    case 3: hipLaunchKernelGGL(read_kernel<3>, grid, dim3(256), 0, s, b, n16, o); break;
    case 4: hipLaunchKernelGGL(read_kernel<4>, grid, dim3(256), 0, s, b, n16, o); break;
    default: return -1;
    }
    return (int)hipGetLastError();
}

extern "C" int fp_touch(void *buf, uint64_t nbytes, uint64_t step_bytes, void *stream) {
    if (step_bytes < 4 || step_bytes % 4) return -1;
    const uint64_t ndw = nbytes / 4, step_dw = step_bytes / 4;
    const uint64_t threads = (ndw + step_dw - 1) / step_dw;
    const uint64_t b = blocks_for(threads);
    hipLaunchKernelGGL(touch_kernel, dim3((unsigned)(b < 65536 ? b : 65536)), dim3(256), 0,
                       (hipStream_t)stream, (uint32_t *)buf, ndw, step_dw);
    return (int)hipGetLastError();
}

extern "C" int fp_copy(void *dst, const void *src, uint64_t nbytes, int nontemporal, void *stream) {
    if ((((uintptr_t)dst | (uintptr_t)src | nbytes) & 15) != 0) return -1;
    const uint64_t n16 = nbytes / 16;
    if (nontemporal)
        hipLaunchKernelGGL(copy_kernel<true>, dim3(blocks_for(n16)), dim3(256), 0,
                           (hipStream_t)stream, (u32x4 *)dst, (const u32x4 *)src, n16);
    else
        hipLaunchKernelGGL(copy_kernel<false>, dim3(blocks_for(n16)), dim3(256), 0,
                           (hipStream_t)stream, (u32x4 *)dst, (const u32x4 *)src, n16);
    return (int)hipGetLastError();
}
