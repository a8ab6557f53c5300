/* TEST INFRASTRUCTURE ONLY -- see frame_oracle.c. Verdict codes are the public ones of
 * include/aipstack_amd/chksum.h (shared vocabulary; no product code is linked). */
#ifndef AIPSTACK_AMD_FRAME_ORACLE_H
#define AIPSTACK_AMD_FRAME_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "aipstack_amd/chksum.h"

#ifdef __cplusplus
extern "C" {
#endif

int oracle_rx_verify(const void *frame, size_t len);
int oracle_tx_fill(void *frame, size_t len);
void oracle_rx_verify_batch(const void *base, const uint64_t *offsets, uint64_t n,
                            uint8_t *verdict);
void oracle_tx_fill_batch(void *base, const uint64_t *offsets, uint64_t n, uint8_t *status);
void oracle_rx_verify_slotted(const void *base, uint64_t stride, const uint32_t *lens,
                              uint64_t n, uint8_t *verdict);
void oracle_tx_fill_slotted(void *base, uint64_t stride, const uint32_t *lens, uint64_t n,
                            uint8_t *status);

#ifdef __cplusplus
}
#endif

#endif
