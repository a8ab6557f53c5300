// Streaming-read ceiling of this MI355X: read a large buffer once with 16-byte loads,
// fold it into one word per wave (so nothing is dead-code-eliminated), in the same
// style and grid shapes as the checksum kernel. Reports GB/s per variant (median of
// reps, HIP events). Not part of the product; it calibrates roofline.frac.
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/hbm_peak tools/hbm_peak.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const u32x4 *__restrict__ p, uint64_t n16,
                                                   uint64_t per_wave, uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t i = wave * per_wave;
    const uint64_t end = min(i + per_wave, n16);
    uint32_t acc = 0;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(p + i), (short)0,
                                                                 (int)((end - i) * 16), 0x00020000);
    for (uint32_t off = 0; i + off < end; off += 64 * UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (lane + u * 64) * 16, off * 16, NT ? 2 : 0);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u][0] + v[u][1] + v[u][2] + v[u][3];
    }
    if (acc == 0x12345678u) out[wave] = acc;  // practically never: keeps loads live
}

// The same read with LS contiguous segments per lane: in each group of 64 * LS segments lane
// l loads segments l * LS .. l * LS + LS - 1 (one wave instruction per segment index, lanes
// LS * 16 bytes apart), so a wave-wide prefix scan covers LS KiB instead of one.
template <int UNROLL, int LS>
__global__ __launch_bounds__(256) void read_kernel_ls(const u32x4 *__restrict__ p, uint64_t n16,
                                                      uint64_t per_wave, uint32_t *out) {
    static_assert(UNROLL % LS == 0, "whole groups");
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t i = wave * per_wave;
    const uint64_t end = min(i + per_wave, n16);
    uint32_t acc = 0;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(p + i), (short)0,
                                                                 (int)((end - i) * 16), 0x00020000);
    for (uint32_t off = 0; i + off < end; off += 64 * UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            v[u] = __builtin_amdgcn_raw_buffer_load_b128(
                r, ((u / LS) * 64 * LS + lane * LS + u % LS) * 16, off * 16, 2);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u][0] + v[u][1] + v[u][2] + v[u][3];
    }
    if (acc == 0x12345678u) out[wave] = acc;
}

// The same read through global_load_dwordx4 with a 64-bit address per lane (the gathered
// checksum loader's form) instead of a buffer descriptor.
template <int UNROLL>
__global__ __launch_bounds__(256) void read_kernel_global(const u32x4 *__restrict__ p, uint64_t n16,
                                                          uint64_t per_wave, uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t i = wave * per_wave;
    const uint64_t end = min(i + per_wave, n16);
    uint32_t acc = 0;
    for (uint64_t off = 0; i + off < end; off += 64 * UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t k = min(i + off + (uint64_t)(lane + u * 64), end - 1);
            v[u] = __builtin_nontemporal_load(p + k);
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u][0] + v[u][1] + v[u][2] + v[u][3];
    }
    if (acc == 0x12345678u) out[wave] = acc;
}

// Slotted read: packets of `len` bytes at a `stride` (MTU packets in 2048-byte ring slots),
// one packet per wave instruction pair (segments lane and lane + 64 of the packet), P
// packets in flight: the access pattern of the checksum kernel's per-packet wave mode,
// without the checksum arithmetic. The gaps between packets are not read.
template <int P>
__global__ __launch_bounds__(256) void slot_read_kernel(const uint8_t *__restrict__ p, uint64_t npk,
                                                        uint32_t stride, uint32_t len,
                                                        uint64_t per_wave, uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t i = wave * per_wave;
    const uint64_t end = min(i + per_wave, npk);
    uint32_t acc = 0;
    for (; i < end; i += P) {
        u32x4 v[P][2];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const uint64_t k = min(i + q, end - 1);
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(p + k * stride), (short)0, (int)((len + 15) & ~15u), 0x00020000);
            v[q][0] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 0, 2);
            v[q][1] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 1024, 2);
        }
#pragma unroll
        for (int q = 0; q < P; ++q)
            acc ^= v[q][0][0] + v[q][0][1] + v[q][1][2] + v[q][1][3];
    }
    if (acc == 0x12345678u) out[wave] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int U, bool NT>
float run(const u32x4 *d, uint64_t n16, uint64_t per_wave, uint32_t *out, int reps) {
    uint64_t waves = (n16 + per_wave - 1) / per_wave;
    dim3 grid((unsigned)((waves + 3) / 4));
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < reps + 2; ++r) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((read_kernel<U, NT>), grid, dim3(256), 0, 0, d, n16, per_wave, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

// The ceiling bench.py puts on its line (roofline.measured_peak): R = 3 buffers of config A's
// size (1.57 GB each, 4.7 GB in all, so no launch finds the previous one's bytes in the 256 MiB
// Infinity Cache), each launch reading the next buffer once, median of 30 launches after 15.
// Shapes: long runs per wave (32 KiB, 2 or 4 windows in flight: the rounds 1-3 probe) and the
// gathered checksum loader's shape (one short run per wave, ~12 KiB, every window issued up
// front). Prints one JSON line; "GBps" is the best shape.
template <int U, bool NT, bool GLOBAL = false, int LS = 1>
float run_rot(u32x4 *const *d, int nbuf, uint64_t n16, uint64_t per_wave, uint32_t *out,
              unsigned lds_pad = 0) {
    uint64_t waves = (n16 + per_wave - 1) / per_wave;
    dim3 grid((unsigned)((waves + 3) / 4));
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < 45; ++r) {
        (void)hipEventRecord(a);
        if (GLOBAL)
            hipLaunchKernelGGL((read_kernel_global<U>), grid, dim3(256), lds_pad, 0, d[r % nbuf], n16, per_wave, out);
        else if (LS > 1)
            hipLaunchKernelGGL((read_kernel_ls<U, LS>), grid, dim3(256), lds_pad, 0, d[r % nbuf], n16, per_wave, out);
        else
            hipLaunchKernelGGL((read_kernel<U, NT>), grid, dim3(256), lds_pad, 0, d[r % nbuf], n16, per_wave, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 15) t.push_back(ms);
    }
    (void)hipEventDestroy(a); (void)hipEventDestroy(b);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int ceiling() {
    const uint64_t bytes = 1572864000ull;  // config A: 1 M x 1500 B
    const uint64_t n16 = bytes / 16;
    constexpr int R = 3;
    u32x4 *d[R]; uint32_t *out;
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&d[r], bytes));
        CK(hipMemset(d[r], 1 + r, bytes));
    }
    CK(hipMalloc(&out, 1 << 24));
    CK(hipDeviceSynchronize());
    const float t_2 = run_rot<2, true>(d, R, n16, 2048, out);
    const float t_4 = run_rot<4, true>(d, R, n16, 2048, out);
    const float t_g12 = run_rot<12, true>(d, R, n16, 768, out);   // 12 KiB per wave, up front
    const float t_g16 = run_rot<16, true>(d, R, n16, 1024, out);  // 16 KiB per wave, up front
    const float t_g8 = run_rot<8, true>(d, R, n16, 768, out);     // 12 KiB, 8 windows then 4
    const float t_gg12 = run_rot<12, true, true>(d, R, n16, 768, out);  // global loads
    const float t_gg8 = run_rot<8, true, true>(d, R, n16, 768, out);
    // the same 12 KiB runs at 3, 4 and 5 waves per SIMD (dynamic LDS per block caps the
    // blocks per CU; the bare kernel runs 8): the checksum kernels run at 4-5
    const float t_o3 = run_rot<8, true>(d, R, n16, 768, out, 41984);
    const float t_o4 = run_rot<8, true>(d, R, n16, 768, out, 33792);
    const float t_o5 = run_rot<8, true>(d, R, n16, 768, out, 27648);
    const float best = std::min(std::min(std::min(std::min(t_2, t_4), std::min(t_g12, t_g16)),
                                         std::min(t_g8, std::min(t_gg12, t_gg8))),
                                std::min(t_o3, std::min(t_o4, t_o5)));
    auto gbps = [&](float ms) { return bytes / ms / 1e6; };
    printf("{\"GBps\": %.1f, \"us\": %.2f, \"rotation\": %d, \"bytes_per_launch\": %lu, "
           "\"shapes_GBps\": {\"run32K_u2\": %.1f, \"run32K_u4\": %.1f, \"run12K_upfront\": %.1f, "
           "\"run16K_upfront\": %.1f, \"run12K_u8\": %.1f, \"run12K_upfront_global\": %.1f, "
           "\"run12K_u8_global\": %.1f, \"run12K_u8_3waves\": %.1f, \"run12K_u8_4waves\": %.1f, "
           "\"run12K_u8_5waves\": %.1f}, \"source\": \"tools/build/hbm_peak "
           "ceiling: 16-B nontemporal reads, median of 30 launches over 3 rotated 1.57 GB "
           "buffers\"}\n",
           gbps(best), best * 1e3, R, (unsigned long)bytes, gbps(t_2), gbps(t_4), gbps(t_g12),
           gbps(t_g16), gbps(t_g8), gbps(t_gg12), gbps(t_gg8), gbps(t_o3), gbps(t_o4), gbps(t_o5));
    for (int r = 0; r < R; ++r) CK(hipFree(d[r]));
    CK(hipFree(out));
    return 0;
}

// Lane-contiguous load shapes (read_kernel_ls) against the contiguous one, 12 KiB per wave,
// 8 windows then 4, at the bare kernel's 8 waves per SIMD and at 4 and 5 (lds_pad).
int lanes() {
    const uint64_t bytes = 1572864000ull;
    const uint64_t n16 = bytes / 16;
    constexpr int R = 3;
    u32x4 *d[R]; uint32_t *out;
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&d[r], bytes));
        CK(hipMemset(d[r], 1 + r, bytes));
    }
    CK(hipMalloc(&out, 1 << 24));
    CK(hipDeviceSynchronize());
    auto gbps = [&](float ms) { return bytes / ms / 1e6; };
    for (int pass = 0; pass < 2; ++pass) {
        const float a1 = run_rot<8, true>(d, R, n16, 768, out);
        const float a2 = run_rot<8, true, false, 2>(d, R, n16, 768, out);
        const float a4 = run_rot<8, true, false, 4>(d, R, n16, 768, out);
        const float b1 = run_rot<8, true>(d, R, n16, 768, out, 33792);
        const float b2 = run_rot<8, true, false, 2>(d, R, n16, 768, out, 33792);
        const float b4 = run_rot<8, true, false, 4>(d, R, n16, 768, out, 33792);
        const float c1 = run_rot<8, true>(d, R, n16, 768, out, 27648);
        const float c4 = run_rot<8, true, false, 4>(d, R, n16, 768, out, 27648);
        const float e4 = run_rot<16, true, false, 4>(d, R, n16, 1024, out, 33792);
        printf("{\"lanes_GBps\": {\"ls1\": %.1f, \"ls2\": %.1f, \"ls4\": %.1f, \"ls1_4waves\": %.1f, "
               "\"ls2_4waves\": %.1f, \"ls4_4waves\": %.1f, \"ls1_5waves\": %.1f, \"ls4_5waves\": %.1f, "
               "\"ls4_16K_4waves\": %.1f}}\n",
               gbps(a1), gbps(a2), gbps(a4), gbps(b1), gbps(b2), gbps(b4), gbps(c1), gbps(c4), gbps(e4));
    }
    for (int r = 0; r < R; ++r) CK(hipFree(d[r]));
    CK(hipFree(out));
    return 0;
}

// Per-launch times of the first 120 launches of one read shape from a cold start (3 rotated
// 1.57 GB buffers, no warm-up): does a pure read at the checksum kernels' rate show their
// clock dip ~3 ms into a run? Shape: 12 KiB per wave, 8 windows then 4 (u8).
int trace_reads(int global) {
    const uint64_t bytes = 1572864000ull;
    const uint64_t n16 = bytes / 16;
    constexpr int R = 3;
    u32x4 *d[R]; uint32_t *out;
    for (int r = 0; r < R; ++r) {
        CK(hipMalloc(&d[r], bytes));
        CK(hipMemset(d[r], 1 + r, bytes));
    }
    CK(hipMalloc(&out, 1 << 24));
    CK(hipDeviceSynchronize());
    const uint64_t per_wave = 768, waves = (n16 + per_wave - 1) / per_wave;
    dim3 grid((unsigned)((waves + 3) / 4));
    std::vector<hipEvent_t> ev(2 * 120);
    for (auto &evk : ev) CK(hipEventCreate(&evk));
    for (int k = 0; k < 120; ++k) {
        CK(hipEventRecord(ev[2 * k]));
        if (global)
            hipLaunchKernelGGL((read_kernel_global<8>), grid, dim3(256), 0, 0, d[k % R], n16, per_wave, out);
        else
            hipLaunchKernelGGL((read_kernel<8, true>), grid, dim3(256), 0, 0, d[k % R], n16, per_wave, out);
        CK(hipEventRecord(ev[2 * k + 1]));
    }
    CK(hipDeviceSynchronize());
    printf("{\"trace\": \"%s\", \"us\": [", global ? "run12K_u8_global" : "run12K_u8");
    for (int k = 0; k < 120; ++k) {
        float ms = 0;
        CK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
        printf("%s%.2f", k ? ", " : "", ms * 1e3);
    }
    printf("]}\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && std::strcmp(argv[1], "ceiling") == 0) return ceiling();
    if (argc > 1 && std::strcmp(argv[1], "lanes") == 0) return lanes();
    if (argc > 1 && std::strcmp(argv[1], "trace") == 0) return trace_reads(argc > 2 ? std::atoi(argv[2]) : 1);
    const uint64_t bytes = 2359296000ull;  // config B's payload (2.36 GB, > 256 MiB MALL)
    const uint64_t n16 = bytes / 16;
    u32x4 *d; uint32_t *out;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMemset(d, 1, bytes));
    CK(hipDeviceSynchronize());
    const uint64_t pw[] = {2048, 4096, 8192, 16384, 32768};
    for (uint64_t per_wave : pw) {
        float t1 = run<1, true>(d, n16, per_wave, out, 10);
        float t2 = run<2, true>(d, n16, per_wave, out, 10);
        float t4 = run<4, true>(d, n16, per_wave, out, 10);
        float t4d = run<4, false>(d, n16, per_wave, out, 10);
        float t8 = run<8, true>(d, n16, per_wave, out, 10);
        printf("{\"segments_per_wave\": %lu, \"GBps\": {\"u1_nt\": %.1f, \"u2_nt\": %.1f, \"u4_nt\": %.1f, \"u4_default\": %.1f, \"u8_nt\": %.1f}}\n",
               (unsigned long)per_wave, bytes / t1 / 1e6, bytes / t2 / 1e6, bytes / t4 / 1e6,
               bytes / t4d / 1e6, bytes / t8 / 1e6);
    }
    // config A2K's pattern: 1 M x 1500-byte packets in 2048-byte slots (payload GB/s)
    const uint64_t npk = 1ull << 20;
    for (uint64_t per_wave : {8ull, 16ull, 32ull, 64ull}) {
        std::vector<float> ts;
        for (int r = 0; r < 12; ++r) {
            const uint64_t waves = (npk + per_wave - 1) / per_wave;
            hipEvent_t a, b;
            (void)hipEventCreate(&a); (void)hipEventCreate(&b);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL((slot_read_kernel<8>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0,
                               (const uint8_t *)d, npk, 2048u, 1500u, per_wave, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms; (void)hipEventElapsedTime(&ms, a, b);
            if (r >= 2) ts.push_back(ms);
            (void)hipEventDestroy(a); (void)hipEventDestroy(b);
        }
        std::sort(ts.begin(), ts.end());
        const float t = ts[ts.size() / 2];
        printf("{\"slots\": \"1M x 1500B in 2048B slots, 8 packets in flight\", \"packets_per_wave\": %lu, "
               "\"us\": %.1f, \"payload_GBps\": %.1f}\n", (unsigned long)per_wave, t * 1e3,
               npk * 1500.0 / t / 1e6);
    }
    return 0;
}
