// Tx field-store price probe. Not part of the product.
// 1 M frames of 1500 B back to back (config A's layout, Tx's shape): each wave streams
// CPW chunks of 64 frames with 16-byte loads, then lane j writes frame j's two checksum
// fields (frame bytes 24 and 50, as a TCP frame with a 20-byte IPv4 header). Variants
// price the stores by their granule:
//   read          stream only (no stores)
//   short         two 2-byte stores per frame (what frame_kernel<TX> does)
//   g32/g64/g128  the aligned 32/64/128-byte granule holding each field, written whole
//                 (one or two granules per frame: a shared one is written once)
//   scatter_*     the same stores with no read stream (a separate scatter pass)
// Output bytes are junk; only times matter. GB/s are over the 1.5 GB read.
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/tx_store_probe tools/tx_store_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16_any_align __attribute__((aligned(1)));

constexpr uint64_t kFrame = 1500, kFrames = 1u << 20, kBytes = kFrame * kFrames;

// G: 0 no store, 1 two shorts, else the aligned G-byte granule(s) holding the fields
template <int G, bool READ>
__global__ __launch_bounds__(256) void probe_kernel(uint8_t *__restrict__ p, uint32_t cpw,
                                                    uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunks = kFrames / 64;
    uint64_t c = wave * cpw;
    const uint64_t c_end = min(c + cpw, nchunks);
    uint32_t acc = lane;
    for (; c < c_end; ++c) {
        const uint64_t b0 = c * 64 * kFrame;
        if (READ) {
            const uint32_t span = 64 * kFrame;  // 96000 B, 16-byte aligned
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p + b0, (short)0, (int)span, 0x00020000);
            for (uint32_t off = 0; off < span; off += 4 * 1024) {
                u32x4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (lane + u * 64) * 16, off, 2);
#pragma unroll
                for (int u = 0; u < 4; ++u) acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
            }
        }
        const uint64_t S = (uint64_t)(uintptr_t)p + b0 + (uint64_t)lane * kFrame;
        if constexpr (G == 1) {
            *reinterpret_cast<u16_any_align *>(S + 24) = (uint16_t)acc;
            *reinterpret_cast<u16_any_align *>(S + 50) = (uint16_t)(acc >> 16);
        } else if constexpr (G > 1) {
            const uint64_t g0 = (S + 24) & ~(uint64_t)(G - 1), g1 = (S + 50) & ~(uint64_t)(G - 1);
            const u32x4 v = {acc, acc + 1, acc + 2, acc + 3};
#pragma unroll
            for (int k = 0; k < G / 16; ++k) *reinterpret_cast<u32x4 *>(g0 + 16 * k) = v;
            if (g1 != g0) {
#pragma unroll
                for (int k = 0; k < G / 16; ++k) *reinterpret_cast<u32x4 *>(g1 + 16 * k) = v;
            }
        }
    }
    if (acc == 0x12345678u) out[wave] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int G, bool READ>
float run(uint8_t *d, uint32_t cpw, uint32_t *out, int reps) {
    const uint64_t waves = (kFrames / 64 + cpw - 1) / cpw;
    dim3 grid((unsigned)((waves + 3) / 4));
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < reps + 2; ++r) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((probe_kernel<G, READ>), grid, dim3(256), 0, 0, d, cpw, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2] * 1000.0f;  // us
}

int main() {
    uint8_t *d; uint32_t *out;
    CK(hipMalloc(&d, kBytes + 4096));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMemset(d, 1, kBytes + 4096));
    CK(hipDeviceSynchronize());
    for (uint32_t cpw : {1u, 2u, 4u}) {
        // interleave twice so clock drift shows
        for (int pass = 0; pass < 2; ++pass) {
            printf("{\"cpw\": %u, \"pass\": %d, \"us\": {\"read\": %.1f, \"short\": %.1f, \"g32\": %.1f, "
                   "\"g64\": %.1f, \"g128\": %.1f, \"scatter_short\": %.1f, \"scatter_g32\": %.1f, "
                   "\"scatter_g64\": %.1f, \"scatter_g128\": %.1f}}\n",
                   cpw, pass, run<0, true>(d, cpw, out, 10), run<1, true>(d, cpw, out, 10),
                   run<32, true>(d, cpw, out, 10), run<64, true>(d, cpw, out, 10),
                   run<128, true>(d, cpw, out, 10), run<1, false>(d, cpw, out, 10),
                   run<32, false>(d, cpw, out, 10), run<64, false>(d, cpw, out, 10),
                   run<128, false>(d, cpw, out, 10));
            fflush(stdout);
        }
    }
    return 0;
}
