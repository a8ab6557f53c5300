// aipstack_amd -- synthetic packet batches on host and device (include/aipstack_amd/synth.h).
// Bench/test plumbing: generating 1.5 GB on the device takes milliseconds instead of a
// PCIe copy, and the host side regenerates exactly the same bytes for the CPU baseline.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "chksum_internal.h"
#include "synth_common.h"

namespace {

// Thread t writes 16 bytes: words 2t and 2t+1 of the (byte_offset-aligned) stream.
// Handles a byte_offset that is not a multiple of 8 by per-byte extraction at the edges.
__global__ __launch_bounds__(256) void synth_fill_kernel(uint8_t *__restrict__ buf,
                                                         uint64_t nbytes, uint64_t seed,
                                                         uint64_t byte_offset) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i0 = t * 16;  // first buffer byte this thread writes
    if (i0 >= nbytes) return;
    if ((byte_offset & 7) == 0 && i0 + 16 <= nbytes && (((uintptr_t)(buf + i0)) & 15) == 0) {
        const uint64_t k = (byte_offset + i0) >> 3;
        typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
        u64x2 v = {aipstack_synth_word(seed, k), aipstack_synth_word(seed, k + 1)};
        *reinterpret_cast<u64x2 *>(buf + i0) = v;
        return;
    }
    for (uint64_t i = i0; i < i0 + 16 && i < nbytes; ++i) {
        const uint64_t g = byte_offset + i;
        buf[i] = (uint8_t)(aipstack_synth_word(seed, g >> 3) >> (8 * (g & 7)));
    }
}

// One wave per packet: overwrite class-0/1/2 packets.
__global__ __launch_bounds__(256) void synth_classes_kernel(uint8_t *__restrict__ buf,
                                                            const uint64_t *__restrict__ off,
                                                            uint64_t n, uint64_t len_seed,
                                                            uint64_t first_packet) {
    const uint64_t p = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= n) return;
    const uint32_t cls = aipstack_synth_class(len_seed, first_packet + p);
    if (cls > 2) return;
    const uint64_t s = off[p], e = off[p + 1];
    for (uint64_t j = lane; j < e - s; j += 64)
        buf[s + j] = (uint8_t)aipstack_synth_class_byte(cls, j, e - s);
}

}  // namespace

extern "C" void aipstack_synth_fill_host(void *buf, uint64_t nbytes, uint64_t seed,
                                         uint64_t byte_offset) {
    uint8_t *b = static_cast<uint8_t *>(buf);
    unsigned nt = std::thread::hardware_concurrency();
    if (nt == 0) nt = 1;
    if (nt > 16) nt = 16;
    if (nbytes < (1u << 20)) nt = 1;
    auto work = [=](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi;) {
            const uint64_t g = byte_offset + i;
            const uint64_t w = aipstack_synth_word(seed, g >> 3);
            for (unsigned s = (unsigned)(g & 7); s < 8 && i < hi; ++s, ++i)
                b[i] = (uint8_t)(w >> (8 * s));
        }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t) {
        const uint64_t lo = nbytes * t / nt, hi = nbytes * (t + 1) / nt;
        pool.emplace_back(work, lo, hi);
    }
    for (auto &th : pool) th.join();
}

extern "C" uint64_t aipstack_synth_mixed_offsets_host(uint64_t *offsets, uint64_t n,
                                                      uint64_t len_seed) {
    uint64_t o = 0;
    offsets[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        o += aipstack_synth_len(len_seed, i);
        offsets[i + 1] = o;
    }
    return o;
}

extern "C" void aipstack_synth_apply_classes_host(void *buf, const uint64_t *offsets,
                                                  uint64_t n, uint64_t len_seed,
                                                  uint64_t first_packet) {
    uint8_t *b = static_cast<uint8_t *>(buf);
    for (uint64_t p = 0; p < n; ++p) {
        const uint32_t cls = aipstack_synth_class(len_seed, first_packet + p);
        if (cls > 2) continue;
        const uint64_t s = offsets[p], l = offsets[p + 1] - s;
        for (uint64_t j = 0; j < l; ++j) b[s + j] = (uint8_t)aipstack_synth_class_byte(cls, j, l);
    }
}

extern "C" int aipstack_synth_fill_device(void *d_buf, uint64_t nbytes, uint64_t seed,
                                          uint64_t byte_offset, void *stream) {
    if (nbytes == 0) return 0;
    if (!d_buf) return -1;
    const uint64_t threads = (nbytes + 15) / 16;
    const uint64_t blocks = (threads + 255) / 256;
    if (blocks > 0x7FFFFFFFull) return -1;
    hipLaunchKernelGGL(synth_fill_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, (uint8_t *)d_buf, nbytes, seed, byte_offset);
    return aipstack_amd::check_hip(hipGetLastError());
}

extern "C" int aipstack_synth_apply_classes_device(void *d_buf, const uint64_t *d_offsets,
                                                   uint64_t n, uint64_t len_seed,
                                                   uint64_t first_packet, void *stream) {
    if (n == 0) return 0;
    if (!d_buf || !d_offsets) return -1;
    const uint64_t blocks = (n + 3) / 4;
    if (blocks > 0x7FFFFFFFull) return -1;
    hipLaunchKernelGGL(synth_classes_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, (uint8_t *)d_buf, d_offsets, n, len_seed,
                       first_packet);
    return aipstack_amd::check_hip(hipGetLastError());
}
