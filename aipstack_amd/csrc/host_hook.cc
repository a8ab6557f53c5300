// aipstack_amd -- the per-packet link-time hook IpChksumInverted (reference Chksum.h:50-51,
// 77-99), HOST code compiled as plain C++ (g++, no HIP): a GPU launch costs more than one
// packet's sum. It is the replacement the reference stack links when it is compiled with
// -DAIPSTACK_EXTERNAL_CHKSUM; it is not a fallback for the batch entry points, which only
// ever run the HIP kernels.

#include <cstddef>
#include <cstdint>
#include <cstring>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace {

inline uint64_t load_le64(const unsigned char *p) {
    uint64_t v;
    std::memcpy(&v, p, 8);  // x86-64 / little-endian host
    return v;
}

}  // namespace

// Inverted Internet checksum of data[0..len), host side.
//
// Words are paired little-endian from `data`, which puts data[2i] in the LOW byte where the
// reference's big-endian pairing (Chksum.h:85-88) puts it in the HIGH byte; the folded sum
// is therefore byte-swapped at the end (a swap is multiplication by 256 mod 0xFFFF). A
// trailing partial word is zero-padded, which is the reference's odd-tail rule
// (Chksum.h:90-93). Folding keeps nonzero sums nonzero, so 0 is returned only for all-zero
// input, as by the reference.
//
// Four bodies, chosen once at load time by CPU feature: AVX-512 (64-byte loads, a masked
// load for the tail), AVX2 (32-byte loads, 16-bit halves added into 32-bit lanes), SSE2 (the
// x86-64 baseline, 16-byte loads), and a portable 64-bit-word loop (the tail of the SSE2 and
// AVX2 bodies).

namespace {

// Portable: 32-bit words into a 64-bit accumulator (len <= 65535 gives < 2^46).
inline uint64_t sum_words64(const unsigned char *p, size_t len) {
    uint64_t a0 = 0, a1 = 0;
    size_t i = 0;
    for (; i + 16 <= len; i += 16) {
        const uint64_t w0 = load_le64(p + i), w1 = load_le64(p + i + 8);
        a0 += (w0 & 0xFFFFFFFFu) + (w0 >> 32);
        a1 += (w1 & 0xFFFFFFFFu) + (w1 >> 32);
    }
    for (; i + 8 <= len; i += 8) {
        const uint64_t w = load_le64(p + i);
        a0 += (w & 0xFFFFFFFFu) + (w >> 32);
    }
    if (i < len) {
        unsigned char tail[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        std::memcpy(tail, p + i, len - i);
        const uint64_t w = load_le64(tail);
        a1 += (w & 0xFFFFFFFFu) + (w >> 32);
    }
    return a0 + a1;
}

inline uint16_t fold_swap(uint64_t s) {
    s = (s & 0xFFFFFFFFu) + (s >> 32);
    s = (s & 0xFFFFFFFFu) + (s >> 32);
    uint32_t t = (uint32_t)s;
    t = (t & 0xFFFFu) + (t >> 16);
    t = (t & 0xFFFFu) + (t >> 16);
    return (uint16_t)(((t & 0xFFu) << 8) | (t >> 8));
}

uint16_t chksum_portable(const unsigned char *p, size_t len) {
    return fold_swap(sum_words64(p, len));
}

#if defined(__x86_64__)
// 16-bit halves of each 32-bit lane summed into 32-bit lanes: per lane at most
// 2 * 65535 per 16 bytes, so even 65535 bytes stay < 2^25 in each lane.
__attribute__((target("sse2"))) uint16_t chksum_sse2(const unsigned char *p, size_t len) {
    const __m128i lo16 = _mm_set1_epi32(0xFFFF);
    __m128i acc0 = _mm_setzero_si128(), acc1 = _mm_setzero_si128();
    size_t i = 0;
    for (; i + 32 <= len; i += 32) {
        const __m128i x0 = _mm_loadu_si128(reinterpret_cast<const __m128i *>(p + i));
        const __m128i x1 = _mm_loadu_si128(reinterpret_cast<const __m128i *>(p + i + 16));
        acc0 = _mm_add_epi32(acc0, _mm_add_epi32(_mm_and_si128(x0, lo16), _mm_srli_epi32(x0, 16)));
        acc1 = _mm_add_epi32(acc1, _mm_add_epi32(_mm_and_si128(x1, lo16), _mm_srli_epi32(x1, 16)));
    }
    alignas(16) uint32_t lanes[4];
    _mm_store_si128(reinterpret_cast<__m128i *>(lanes), _mm_add_epi32(acc0, acc1));
    const uint64_t s = (uint64_t)lanes[0] + lanes[1] + lanes[2] + lanes[3] +
                       sum_words64(p + i, len - i);
    return fold_swap(s);
}

__attribute__((target("avx2"))) uint16_t chksum_avx2(const unsigned char *p, size_t len) {
    const __m256i lo16 = _mm256_set1_epi32(0xFFFF);
    __m256i acc0 = _mm256_setzero_si256(), acc1 = _mm256_setzero_si256();
    size_t i = 0;
    for (; i + 64 <= len; i += 64) {
        const __m256i x0 = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(p + i));
        const __m256i x1 = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(p + i + 32));
        acc0 = _mm256_add_epi32(acc0, _mm256_add_epi32(_mm256_and_si256(x0, lo16),
                                                       _mm256_srli_epi32(x0, 16)));
        acc1 = _mm256_add_epi32(acc1, _mm256_add_epi32(_mm256_and_si256(x1, lo16),
                                                       _mm256_srli_epi32(x1, 16)));
    }
    alignas(32) uint32_t lanes[8];
    _mm256_store_si256(reinterpret_cast<__m256i *>(lanes), _mm256_add_epi32(acc0, acc1));
    uint64_t s = sum_words64(p + i, len - i);
    for (int k = 0; k < 8; ++k) s += lanes[k];
    return fold_swap(s);
}

// AVX-512: 64-byte loads, the same halves-into-32-bit-lanes sum (per lane < 2^28 for 65535
// bytes), and the tail (< 64 bytes) as one byte-masked load: masked-off bytes read as zero
// and are never touched, so the zero padding of an odd tail comes for free.
__attribute__((target("avx512f,avx512bw"))) uint16_t chksum_avx512(const unsigned char *p,
                                                                   size_t len) {
    const __m512i lo16 = _mm512_set1_epi32(0xFFFF);
    __m512i acc0 = _mm512_setzero_si512(), acc1 = _mm512_setzero_si512();
    size_t i = 0;
    for (; i + 128 <= len; i += 128) {
        const __m512i x0 = _mm512_loadu_si512(p + i);
        const __m512i x1 = _mm512_loadu_si512(p + i + 64);
        acc0 = _mm512_add_epi32(acc0, _mm512_add_epi32(_mm512_and_si512(x0, lo16),
                                                       _mm512_srli_epi32(x0, 16)));
        acc1 = _mm512_add_epi32(acc1, _mm512_add_epi32(_mm512_and_si512(x1, lo16),
                                                       _mm512_srli_epi32(x1, 16)));
    }
    if (i + 64 <= len) {
        const __m512i x = _mm512_loadu_si512(p + i);
        acc0 = _mm512_add_epi32(acc0, _mm512_add_epi32(_mm512_and_si512(x, lo16),
                                                       _mm512_srli_epi32(x, 16)));
        i += 64;
    }
    if (i < len) {
        const __mmask64 m = (__mmask64)((1ull << (len - i)) - 1u);  // len - i < 64
        const __m512i x = _mm512_maskz_loadu_epi8(m, p + i);
        acc1 = _mm512_add_epi32(acc1, _mm512_add_epi32(_mm512_and_si512(x, lo16),
                                                       _mm512_srli_epi32(x, 16)));
    }
    alignas(64) uint32_t lanes[16];
    _mm512_store_si512(lanes, _mm512_add_epi32(acc0, acc1));
    uint64_t s = 0;
    for (int k = 0; k < 16; ++k) s += lanes[k];
    return fold_swap(s);
}
#endif

using ChksumFn = uint16_t (*)(const unsigned char *, size_t);

ChksumFn pick_host_chksum() {
#if defined(__x86_64__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw"))
        return chksum_avx512;
    if (__builtin_cpu_supports("avx2")) return chksum_avx2;
    return chksum_sse2;
#else
    return chksum_portable;
#endif
}

const ChksumFn g_host_chksum = pick_host_chksum();

}  // namespace

extern "C" uint16_t IpChksumInverted(const char *data, size_t len) {
    return g_host_chksum(reinterpret_cast<const unsigned char *>(data), len);
}

// Forced variants for tests / benchmarks (not in the public header): 0 portable, 1 SSE2,
// 2 AVX2, 3 AVX-512 (each falls back to the next one down when the CPU lacks it).
extern "C" uint16_t aipstack_chksum_host_variant(int variant, const char *data, size_t len) {
    const unsigned char *p = reinterpret_cast<const unsigned char *>(data);
#if defined(__x86_64__)
    if (variant == 3 && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw"))
        return chksum_avx512(p, len);
    if (variant == 3) variant = 2;
    if (variant == 1) return chksum_sse2(p, len);
    if (variant == 2 && __builtin_cpu_supports("avx2")) return chksum_avx2(p, len);
    if (variant == 2) return chksum_sse2(p, len);
#endif
    (void)variant;
    return chksum_portable(p, len);
}

