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

// The in-place Tx fills' access pattern without their arithmetic (the
// fill's own ceiling). CSR frames back to back (TX): a wave takes 32 frames and streams their
// bytes as one run (16-byte nontemporal buffer loads, 64 per window, 8 windows per group),
// then lane j writes two bytes at frame j's bytes 24 and 50 (the IPv4 and, behind a 20-byte
// header, the L4 checksum field) when its frame index is a multiple of `density`. STORE: 0
// none (the pure read), 1 ordinary 2-byte stores (the product's), 2 nontemporal; 3 / 4: no
// field store, an 8-byte record per frame to a separate array instead (the records pass's
// output, coalesced: 256 B per wave), ordinary / nontemporal.
template <int STORE>
__global__ __launch_bounds__(256) void fill_csr_kernel(uint8_t *__restrict__ base,
                                                       const uint64_t *__restrict__ off,
                                                       uint64_t n, uint32_t density,
                                                       uint32_t *out, uint64_t *rec) {
    constexpr int kFr = 32, U = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t p0 = wave * kFr;
    if (p0 >= n) return;
    const int cnt = (int)min((uint64_t)kFr, n - p0);
    const uint64_t S = off[p0 + (uint64_t)min(lane, cnt)];  // lane cnt: the run's end
    const uint64_t X1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(S >> 32), cnt) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)S, cnt);
    const uint64_t S0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(S >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)S);
    const uint64_t A = S0 & ~(uint64_t)15;
    const uint32_t nseg = (uint32_t)((X1 - A + 15u) >> 4);
    const uint32_t nwin = (nseg + 63u) >> 6;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(base + A), (short)0,
                                                                 (int)(nseg * 16u), 0x00020000);
    uint32_t acc = 0;
    for (uint32_t w = 0; w < nwin; w += U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)lane * 16u, (w + u) * 1024u, 2);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u][0] + v[u][1] + v[u][2] + v[u][3];
    }
    if (STORE >= 3 && lane < cnt) {
        const uint64_t r = (uint64_t)acc << 32 | (uint32_t)S;
        if (STORE == 4)
            __builtin_nontemporal_store(r, rec + p0 + lane);
        else
            rec[p0 + lane] = r;
    }
    if ((STORE == 1 || STORE == 2) && lane < cnt && (p0 + (uint64_t)lane) % density == 0) {
        uint16_t *f0 = reinterpret_cast<uint16_t *>(base + S + 24);
        uint16_t *f1 = reinterpret_cast<uint16_t *>(base + S + 50);
        if (STORE == 2) {
            __builtin_nontemporal_store((uint16_t)acc, f0);
            __builtin_nontemporal_store((uint16_t)(acc >> 16), f1);
        } else {
            *f0 = (uint16_t)acc;
            *f1 = (uint16_t)(acc >> 16);
        }
    }
    if (acc == 0x9E3779B9u) out[wave & 0xFFFF] = acc;
}

// The same for a send ring (TX2K): frame i is lens[i] bytes at base + i * stride, read one
// frame per wave instruction pair (segments lane and lane + 64 of the frame, ranged to it), 8
// frames in flight, 32 frames per wave; then the two field stores as above.
template <int STORE>
__global__ __launch_bounds__(256) void fill_slots_kernel(uint8_t *__restrict__ base,
                                                         uint64_t stride,
                                                         const uint32_t *__restrict__ lens,
                                                         uint64_t n, uint32_t density,
                                                         uint32_t *out) {
    constexpr int kFr = 32, P = 8;
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t p0 = wave * kFr;
    if (p0 >= n) return;
    const uint64_t end = min(p0 + (uint64_t)kFr, n);
    uint32_t acc = 0;
    for (uint64_t i = p0; i < end; i += P) {
        u32x4 v[P][2];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const uint64_t k = min(i + q, end - 1);
            const uint32_t len = __builtin_amdgcn_readfirstlane(lens[k]);
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(base + k * stride), (short)0, (int)((len + 15) & ~15u), 0x00020000);
            v[q][0] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 0, 2);
            v[q][1] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 1024, 2);
        }
#pragma unroll
        for (int q = 0; q < P; ++q) acc ^= v[q][0][0] + v[q][0][1] + v[q][1][2] + v[q][1][3];
    }
    const uint64_t j = p0 + (uint64_t)lane;
    if (STORE != 0 && lane < kFr && j < n && j % density == 0 && lens[j] >= 52u) {
        uint16_t *f0 = reinterpret_cast<uint16_t *>(base + j * stride + 24);
        uint16_t *f1 = reinterpret_cast<uint16_t *>(base + j * stride + 50);
        if (STORE == 2) {
            __builtin_nontemporal_store((uint16_t)acc, f0);
            __builtin_nontemporal_store((uint16_t)(acc >> 16), f1);
        } else {
            *f0 = (uint16_t)acc;
            *f1 = (uint16_t)(acc >> 16);
        }
    }
    if (acc == 0x9E3779B9u) out[wave & 0xFFFF] = acc;
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

// fill probes: d_off = n + 1 CSR offsets (TX), or d_lens + stride (TX2K; d_off null);
// store 3 / 4 (CSR only): 8-byte records to d_rec (n entries) instead of field stores
extern "C" int fp_fill_rec(void *buf, const uint64_t *d_off, uint64_t stride,
                           const uint32_t *d_lens, uint64_t n, uint32_t density, int store,
                           void *scratch, uint64_t *d_rec, void *stream) {
    if (n == 0 || density == 0 || store < 0 || store > 4) return -1;
    if (store >= 3 && (!d_off || !d_rec)) return -1;
    const uint64_t waves = (n + 31) / 32;
    const dim3 grid((unsigned)((waves + 3) / 4));
    const hipStream_t s = (hipStream_t)stream;
    uint8_t *b = (uint8_t *)buf;
    uint32_t *o = (uint32_t *)scratch;
    if (d_off) {
        switch (store) {
        case 0: hipLaunchKernelGGL(fill_csr_kernel<0>, grid, dim3(256), 0, s, b, d_off, n, density, o, d_rec); break;
        case 1: hipLaunchKernelGGL(fill_csr_kernel<1>, grid, dim3(256), 0, s, b, d_off, n, density, o, d_rec); break;
        case 2: hipLaunchKernelGGL(fill_csr_kernel<2>, grid, dim3(256), 0, s, b, d_off, n, density, o, d_rec); break;
        case 3: hipLaunchKernelGGL(fill_csr_kernel<3>, grid, dim3(256), 0, s, b, d_off, n, density, o, d_rec); break;
        default: hipLaunchKernelGGL(fill_csr_kernel<4>, grid, dim3(256), 0, s, b, d_off, n, density, o, d_rec); break;
        }
    } else {
        if (!d_lens || stride == 0) return -1;
        switch (store) {
        case 0: hipLaunchKernelGGL(fill_slots_kernel<0>, grid, dim3(256), 0, s, b, stride, d_lens, n, density, o); break;
        case 1: hipLaunchKernelGGL(fill_slots_kernel<1>, grid, dim3(256), 0, s, b, stride, d_lens, n, density, o); break;
        default: hipLaunchKernelGGL(fill_slots_kernel<2>, grid, dim3(256), 0, s, b, stride, d_lens, n, density, o); break;
        }
    }
    return (int)hipGetLastError();
}

extern "C" int fp_fill(void *buf, const uint64_t *d_off, uint64_t stride, const uint32_t *d_lens,
                       uint64_t n, uint32_t density, int store, void *scratch, void *stream) {
    if (store > 2) return -1;
    return fp_fill_rec(buf, d_off, stride, d_lens, n, density, store, scratch, nullptr, stream);
}
