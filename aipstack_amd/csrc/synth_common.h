// aipstack_amd -- the synthetic-data formulas of include/aipstack_amd/synth.h, shared by
// the host (g++/hipcc host pass) and device code.
#ifndef AIPSTACK_AMD_SYNTH_COMMON_H
#define AIPSTACK_AMD_SYNTH_COMMON_H

#include <stdint.h>

#if defined(__HIPCC__)
#define AIPSTACK_HD __host__ __device__ __forceinline__
#else
#define AIPSTACK_HD static inline
#endif

#include "aipstack_amd/synth.h"

AIPSTACK_HD uint64_t aipstack_synth_word(uint64_t seed, uint64_t k) {
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

AIPSTACK_HD uint32_t aipstack_synth_len(uint64_t len_seed, uint64_t i) {
    return AIPSTACK_SYNTH_MIN_LEN +
           (uint32_t)(aipstack_synth_word(len_seed, i) %
                      (AIPSTACK_SYNTH_MAX_LEN - AIPSTACK_SYNTH_MIN_LEN + 1));
}

AIPSTACK_HD uint32_t aipstack_synth_class(uint64_t len_seed, uint64_t i) {
    return (uint32_t)(aipstack_synth_word(len_seed ^ AIPSTACK_SYNTH_CLASS_SALT, i) % 100u);
}

// Byte j (0-based) of a class-0/1/2 packet of length len; -1 = keep the random byte.
AIPSTACK_HD int aipstack_synth_class_byte(uint32_t cls, uint64_t j, uint64_t len) {
    if (cls == 0) return 0xFF;
    if (cls == 1) return 0x00;
    if (cls == 2) return (j == 0 && (len & 1)) ? 0x00 : 0xFF;
    return -1;
}

#endif
