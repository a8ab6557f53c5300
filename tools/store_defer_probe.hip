// Store-placement probe. Not part of the product.
// 1 M frames of 1500 B back to back, read as a stream (16-byte nontemporal buffer loads,
// 4 windows of 1 KiB in flight per wave), K chunks of 64 frames per wave. Per frame the
// kernel produces a result and stores it in one of these ways:
//   none      no store (price of the read stream alone)
//   v1        1 byte per frame, stored right after each chunk (Rx verdict today)
//   v1_end    1 byte per frame, all K chunks' stores deferred to the end of the wave
//   r8        8 bytes per frame (split Tx record) after each chunk
//   r8_end    the same deferred to the end of the wave
//   sh        two 2-byte stores into the frame (S+24, S+50) after each chunk (Tx in place)
//   sh_end    the same deferred to the end of the wave
// Output bytes are junk; only times matter.
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/store_defer_probe tools/store_defer_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16_any_align __attribute__((aligned(1)));

constexpr uint64_t kFrame = 1500, kFrames = 1u << 20, kBytes = kFrame * kFrames;
enum Mode { NONE, V1, V1_END, R8, R8_END, SH, SH_END };

template <int MODE, int K>
__global__ __launch_bounds__(256) void probe_kernel(uint8_t *__restrict__ p, uint8_t *__restrict__ res) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nchunks = kFrames / 64;
    const uint64_t c0 = wave * K;
    uint32_t keep[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t c = c0 + k;
        uint32_t acc = lane + k;
        if (c < nchunks) {
            const uint64_t b0 = c * 64 * kFrame;
            const uint32_t span = 64 * kFrame;
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
        keep[k] = acc;
        const uint64_t i = c * 64 + lane;
        if (c < nchunks) {
            if constexpr (MODE == V1) res[i] = (uint8_t)acc;
            if constexpr (MODE == R8) reinterpret_cast<uint64_t *>(res)[i] = acc * 0x100000001ull;
            if constexpr (MODE == SH) {
                const uint64_t S = (uint64_t)(uintptr_t)p + i * kFrame;
                *reinterpret_cast<u16_any_align *>(S + 24) = (uint16_t)acc;
                *reinterpret_cast<u16_any_align *>(S + 50) = (uint16_t)(acc >> 16);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t c = c0 + k;
        const uint64_t i = c * 64 + lane;
        if (c < nchunks) {
            if constexpr (MODE == V1_END) res[i] = (uint8_t)keep[k];
            if constexpr (MODE == R8_END) reinterpret_cast<uint64_t *>(res)[i] = keep[k] * 0x100000001ull;
            if constexpr (MODE == SH_END) {
                const uint64_t S = (uint64_t)(uintptr_t)p + i * kFrame;
                *reinterpret_cast<u16_any_align *>(S + 24) = (uint16_t)keep[k];
                *reinterpret_cast<u16_any_align *>(S + 50) = (uint16_t)(keep[k] >> 16);
            }
        }
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE, int K>
float run(uint8_t *d, uint8_t *res, int reps) {
    const uint64_t waves = (kFrames / 64 + K - 1) / K;
    dim3 grid((unsigned)((waves + 3) / 4));
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < reps + 2; ++r) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((probe_kernel<MODE, K>), grid, dim3(256), 0, 0, d, res);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 2) t.push_back(ms);
    }
    (void)hipEventDestroy(a); (void)hipEventDestroy(b);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2] * 1000.0f;  // us
}

template <int K>
void row(uint8_t *d, uint8_t *res, int pass) {
    printf("{\"K\": %d, \"pass\": %d, \"us\": {\"none\": %.1f, \"v1\": %.1f, \"v1_end\": %.1f, "
           "\"r8\": %.1f, \"r8_end\": %.1f, \"sh\": %.1f, \"sh_end\": %.1f}}\n", K, pass,
           run<NONE, K>(d, res, 10), run<V1, K>(d, res, 10), run<V1_END, K>(d, res, 10),
           run<R8, K>(d, res, 10), run<R8_END, K>(d, res, 10), run<SH, K>(d, res, 10),
           run<SH_END, K>(d, res, 10));
    fflush(stdout);
}

int main() {
    uint8_t *d, *res;
    CK(hipMalloc(&d, kBytes + 4096));
    CK(hipMalloc(&res, 8 * kFrames + 4096));
    CK(hipMemset(d, 1, kBytes + 4096));
    CK(hipDeviceSynchronize());
    for (int pass = 0; pass < 2; ++pass) {
        row<1>(d, res, pass);
        row<2>(d, res, pass);
        row<4>(d, res, pass);
        row<8>(d, res, pass);
    }
    return 0;
}
