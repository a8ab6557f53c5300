// Read ceiling of a ring-slot layout: the bytes of n packets / frames, one per fixed slot
// (slot_stride apart, lengths varying per slot), read with 16-byte nontemporal loads one
// packet per wave instruction pair (segments lane and lane + 64 of the packet's slot), P
// packets in flight per wave -- the access pattern of the slotted kernels' per-packet wave
// mode without their arithmetic. The slack after each packet is not read. Not part of the
// product: it calibrates the slotted bench lines (bench.py --config RX2K / C2K reports its
// rate beside its own).
//
//   slot_peak frames N SEED MAX_PAYLOAD STRIDE   lengths of aipstack_synth_frames_host(N, SEED)
//   slot_peak mixed  N STRIDE                    lengths of config C (64-1500 B, seed 43)
//   slot_peak fixed  N LEN STRIDE                every packet LEN bytes
// Prints one JSON line: the best variant's time and payload GB/s (median of 10 reps each).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "aipstack_amd/synth.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int P>
__global__ __launch_bounds__(256) void slot_read(const uint8_t *__restrict__ p, uint64_t npk,
                                                 uint64_t stride, const uint32_t *__restrict__ lens,
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
            const uint32_t len = __builtin_amdgcn_readfirstlane(lens[k]);
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(p + k * stride), (short)0, (int)((len + 15) & ~15u), 0x00020000);
            v[q][0] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 0, 2);
            v[q][1] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, 1024, 2);
        }
#pragma unroll
        for (int q = 0; q < P; ++q) acc ^= v[q][0][0] + v[q][0][1] + v[q][1][2] + v[q][1][3];
    }
    if (acc == 0x12345678u) out[wave] = acc;  // practically never: keeps the loads live
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

template <int P>
float time_variant(const uint8_t *d, uint64_t n, uint64_t stride, const uint32_t *dl,
                   uint64_t per_wave, uint32_t *out) {
    const uint64_t waves = (n + per_wave - 1) / per_wave;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL((slot_read<P>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, 0, d, n,
                           stride, dl, per_wave, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 2) ts.push_back(ms);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: slot_peak frames N SEED MAXPAY STRIDE | mixed N STRIDE | fixed N LEN STRIDE\n");
        return 2;
    }
    const std::string mode = argv[1];
    const uint64_t n = std::strtoull(argv[2], nullptr, 10);
    uint64_t stride = 0;
    std::vector<uint32_t> lens(n);
    if (mode == "frames" && argc >= 6) {
        std::vector<uint64_t> off(n + 1);
        aipstack_synth_frames_host(nullptr, off.data(), n, std::strtoull(argv[3], nullptr, 10),
                                   (uint32_t)std::strtoul(argv[4], nullptr, 10));
        for (uint64_t i = 0; i < n; ++i) lens[i] = (uint32_t)(off[i + 1] - off[i]);
        stride = std::strtoull(argv[5], nullptr, 10);
    } else if (mode == "mixed") {
        std::vector<uint64_t> off(n + 1);
        aipstack_synth_mixed_offsets_host(off.data(), n, 43);
        for (uint64_t i = 0; i < n; ++i) lens[i] = (uint32_t)(off[i + 1] - off[i]);
        stride = std::strtoull(argv[3], nullptr, 10);
    } else if (mode == "fixed" && argc >= 5) {
        std::fill(lens.begin(), lens.end(), (uint32_t)std::strtoul(argv[3], nullptr, 10));
        stride = std::strtoull(argv[4], nullptr, 10);
    } else {
        std::fprintf(stderr, "bad arguments\n");
        return 2;
    }
    uint64_t payload = 0;
    for (uint32_t l : lens) {
        if (l > stride || l > 2048) {
            std::fprintf(stderr, "lengths must fit the slot and 2 KiB\n");
            return 2;
        }
        payload += l;
    }
    uint8_t *d;
    uint32_t *dl, *out;
    CK(hipMalloc(&d, n * stride));
    CK(hipMalloc(&dl, n * 4));
    CK(hipMalloc(&out, 1 << 24));
    CK(hipMemset(d, 1, n * stride));
    CK(hipMemcpy(dl, lens.data(), n * 4, hipMemcpyHostToDevice));
    float best = 1e30f;
    int best_p = 0;
    uint64_t best_pw = 0;
    for (uint64_t pw : {16ull, 32ull, 64ull}) {
        const float t4 = time_variant<4>(d, n, stride, dl, pw, out);
        const float t8 = time_variant<8>(d, n, stride, dl, pw, out);
        if (t4 < best) best = t4, best_p = 4, best_pw = pw;
        if (t8 < best) best = t8, best_p = 8, best_pw = pw;
    }
    std::printf("{\"pattern\": \"%s\", \"n\": %lu, \"slot_stride\": %lu, \"payload_bytes\": %lu, "
                "\"us\": %.2f, \"payload_GBps\": %.1f, \"in_flight\": %d, \"packets_per_wave\": %lu}\n",
                mode.c_str(), (unsigned long)n, (unsigned long)stride, (unsigned long)payload,
                best * 1e3, payload / best / 1e6, best_p, (unsigned long)best_pw);
    return 0;
}
