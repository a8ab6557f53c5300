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
// Nontemporal stores: the bytes land the way the Rx path's DMA delivers them. A batch written
// by ordinary (write-back) stores reads slower the first time (config A 285-312
// us against 221-231 after DMA or nontemporal stores); bench.py --fresh measures each writer.
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
        __builtin_nontemporal_store(v, reinterpret_cast<u64x2 *>(buf + i0));
        return;
    }
    for (uint64_t i = i0; i < i0 + 16 && i < nbytes; ++i) {
        const uint64_t g = byte_offset + i;
        __builtin_nontemporal_store((uint8_t)(aipstack_synth_word(seed, g >> 3) >> (8 * (g & 7))),
                                    buf + i);
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
    for (uint64_t j = lane; j < e - s; j += 64)  // (nontemporal, as synth_fill_kernel)
        __builtin_nontemporal_store((uint8_t)aipstack_synth_class_byte(cls, j, e - s), buf + s + j);
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

namespace {

struct FrameShape {
    uint32_t kind;     // 0 TCP, 1 UDP, 2 ICMP, 3 other proto, 4 ARP, 5 fragment (TCP/UDP)
    uint32_t ihl;      // IPv4 header words
    uint32_t l4hdr;    // L4 header bytes
    uint32_t payload;  // bytes after the L4 header
    uint32_t frame;    // total frame bytes (>= 60)
};

FrameShape frame_shape(uint64_t seed, uint64_t i, uint32_t max_payload) {
    const uint64_t s = seed ^ AIPSTACK_SYNTH_FRAME_SALT;
    const uint64_t r0 = aipstack_synth_word(s, 8 * i + 0);
    const uint64_t r1 = aipstack_synth_word(s, 8 * i + 1);
    const uint64_t r2 = aipstack_synth_word(s, 8 * i + 2);
    const uint64_t r3 = aipstack_synth_word(s, 8 * i + 3);
    FrameShape f;
    const uint32_t k = (uint32_t)(r0 % 100);
    f.kind = k < 50 ? 0 : k < 78 ? 1 : k < 88 ? 2 : k < 93 ? 3 : k < 97 ? 4 : 5;
    f.ihl = (r1 % 100) < 85 ? 5u : 6u + (uint32_t)((r1 >> 8) % 10);
    f.payload = (uint32_t)(r2 % ((uint64_t)max_payload + 1));
    const uint32_t proto_kind = f.kind == 5 ? (uint32_t)((r3 >> 20) & 1) : f.kind;
    f.l4hdr = proto_kind == 0 ? 20u + 4u * ((r3 % 100) < 70 ? 0u : (uint32_t)((r3 >> 8) % 11))
            : proto_kind == 1 ? 8u : proto_kind == 2 ? 8u : 0u;
    if (f.kind == 4) {  // ARP: 28-byte body
        f.ihl = 0; f.l4hdr = 0; f.payload = 28;
    }
    uint32_t len = 14 + 4 * f.ihl + f.l4hdr + f.payload;
    f.frame = len < 60 ? 60 : len;
    return f;
}

inline void put16(uint8_t *p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

}  // namespace

extern "C" uint64_t aipstack_synth_frames_host(void *buf, uint64_t *offsets, uint64_t n,
                                               uint64_t seed, uint32_t max_payload) {
    uint64_t o = 0;
    offsets[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        o += frame_shape(seed, i, max_payload).frame;
        offsets[i + 1] = o;
    }
    if (!buf) return o;
    uint8_t *b = static_cast<uint8_t *>(buf);
    aipstack_synth_fill_host(b, o, seed, 0);  // random bytes everywhere, then the headers
    const uint64_t s = seed ^ AIPSTACK_SYNTH_FRAME_SALT;
    for (uint64_t i = 0; i < n; ++i) {
        const FrameShape f = frame_shape(seed, i, max_payload);
        uint8_t *fr = b + offsets[i];
        const uint64_t r3 = aipstack_synth_word(s, 8 * i + 3);
        const uint64_t r4 = aipstack_synth_word(s, 8 * i + 4);
        if (f.kind == 4) {
            put16(fr + 12, 0x0806);
            for (uint32_t j = 14 + 28; j < f.frame; ++j) fr[j] = 0;
            continue;
        }
        put16(fr + 12, 0x0800);
        uint8_t *ip = fr + 14;
        const uint32_t hl = 4 * f.ihl;
        const uint32_t total = hl + f.l4hdr + f.payload;
        ip[0] = (uint8_t)(0x40 | f.ihl);
        put16(ip + 2, total);
        uint32_t flags_off = (r4 & 1) ? 0x4000u : 0u;  // DF sometimes
        if (f.kind == 5)
            flags_off = (r4 & 2) ? (0x2000u | (uint32_t)((r4 >> 8) % 0x2000)) : (uint32_t)(1 + (r4 >> 8) % 0x1FFF);
        put16(ip + 6, flags_off);
        ip[8] = 64;
        const uint32_t proto_kind = f.kind == 5 ? (uint32_t)((r3 >> 20) & 1) : f.kind;
        ip[9] = proto_kind == 0 ? 6 : proto_kind == 1 ? 17 : proto_kind == 2 ? 1 : 47;
        put16(ip + 10, 0);
        uint8_t *l4 = ip + hl;
        if (proto_kind == 0) {
            l4[12] = (uint8_t)(((f.l4hdr / 4) << 4) | (l4[12] & 0x0F));
            put16(l4 + 16, 0);
        } else if (proto_kind == 1) {
            put16(l4 + 4, 8 + f.payload);
            put16(l4 + 6, 0);
        } else if (proto_kind == 2) {
            l4[0] = (uint8_t)((r4 >> 16) % 3 == 0 ? 0 : (r4 >> 16) % 3 == 1 ? 8 : 3);
            put16(l4 + 2, 0);
        }
        for (uint32_t j = 14 + total; j < f.frame; ++j) fr[j] = 0;  // Ethernet padding
    }
    return o;
}
