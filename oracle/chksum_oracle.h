/* TEST INFRASTRUCTURE ONLY -- see chksum_oracle.c. Never linked by the product. */
#ifndef AIPSTACK_AMD_CHKSUM_ORACLE_H
#define AIPSTACK_AMD_CHKSUM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

uint16_t oracle_chksum_inverted(const void *data, size_t len);
uint16_t oracle_chksum(const void *data, size_t len);
uint16_t oracle_chksum_chain(uint32_t state, const void *const *ptrs,
                             const size_t *lens, size_t nchunks);
void oracle_batch_strided(const void *base, uint64_t stride, uint32_t len,
                          uint64_t n, uint16_t *out, uint32_t flags);
void oracle_batch_slotted(const void *base, uint64_t stride, const uint32_t *lens, uint64_t n,
                          uint16_t *out, uint32_t flags);
void oracle_batch_csr(const void *base, const uint64_t *offsets, uint64_t n,
                      uint16_t *out, uint32_t flags);
void oracle_batch_seeded_csr(const void *base, const uint64_t *offsets,
                             const uint32_t *states, uint64_t n, uint16_t *out);
void oracle_batch_chain(const void *base, uint64_t addr_bias, const uint64_t *addr,
                        const uint32_t *len, const uint64_t *index, const uint32_t *states,
                        uint64_t n, uint16_t *out, uint32_t flags);

#ifdef __cplusplus
}
#endif

#endif
