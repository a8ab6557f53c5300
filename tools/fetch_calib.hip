// FETCH_SIZE calibration for the frame kernels' access pattern. Not part
// of the product. MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide coalesced
// streaming reads (it reports half their bytes); the frame kernels also issue per-lane
// header loads (lane j: 128 bytes at frame j's start, 64 frames per instruction).
// Three kernels over the same 1.5 GB of frames, each reading every byte from HBM once:
//   stream       chunks of 64 frames streamed, 16 B per lane (the calibrated pattern)
//   hdr_stream   per chunk: lane j first loads frame j's first 128 aligned bytes, then the
//                chunk is streamed (the header bytes again, now from L2): Rx's pattern
//   hdr_only     just the header loads (128 B per frame at 16-B alignment)
// Frames of 1500, 772, 300 and 100 B (4-byte multiples, as Rx's frame starts are not).
// Run under rocprofv3 --pmc FETCH_SIZE and compare 2 x FETCH_SIZE with the bytes.
//   hipcc --offload-arch=gfx950 -O3 -o tools/build/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint64_t kBytes = 1500ull << 20;  // 1.5 GB, cut into frames of `frame` bytes

template <bool HDR, bool STREAM>
__global__ __launch_bounds__(256) void calib_kernel(const uint8_t *__restrict__ p, uint32_t kFrame,
                                                    uint64_t kFrames, uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t c = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (c >= kFrames / 64) return;
    const uint64_t b0 = c * 64 * kFrame;
    const uint32_t span = 64 * kFrame;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)(p + b0), (short)0, (int)span, 0x00020000);
    uint32_t acc = lane;
    if (HDR) {
        const uint32_t h = ((uint32_t)lane * kFrame) & ~15u;
        u32x4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, h + 16 * i, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc += v[i][0] ^ v[i][1] ^ v[i][2] ^ v[i][3];
    }
    if (STREAM) {
        for (uint32_t off = 0; off < span; off += 4 * 1024) {
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (lane + u * 64) * 16, off, 2);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc += v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
        }
    }
    if (acc == 0x12345678u) out[c] = acc;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <bool HDR, bool STREAM>
int run(const char *name, const uint8_t *d, uint32_t frame, uint32_t *out) {
    const uint64_t kFrames = kBytes / frame / 256 * 256;
    const dim3 grid((unsigned)(kFrames / 64 / 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((calib_kernel<HDR, STREAM>), grid, dim3(256), 0, 0, d, frame, kFrames, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (r > 0 && ms < best) best = ms;
    }
    printf("{\"kernel\": \"%s\", \"frame\": %u, \"best_us\": %.1f, \"stream_bytes\": %llu, \"header_bytes\": %llu}\n",
           name, frame, best * 1e3, (unsigned long long)(STREAM ? kFrames * frame : 0),
           (unsigned long long)(HDR ? kFrames * 128ull : 0));
    return 0;
}

int main() {
    uint8_t *d; uint32_t *out;
    CK(hipMalloc(&d, kBytes));
    CK(hipMalloc(&out, 1 << 20));
    CK(hipMemset(d, 1, kBytes));
    CK(hipDeviceSynchronize());
    for (uint32_t frame : {1500u, 772u, 300u, 100u}) {  // Rx's mean is 769 B; short frames
        if (run<false, true>("stream", d, frame, out)) return 1;
        if (run<true, true>("hdr_stream", d, frame, out)) return 1;
        if (run<true, false>("hdr_only", d, frame, out)) return 1;
    }
    return 0;
}
