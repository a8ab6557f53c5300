/*
 * TEST INFRASTRUCTURE ONLY -- the CPU oracle for the Internet-checksum hot path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this file's library (oracle/build/libchksum_oracle.so). The product library
 * (aipstack_amd/libaipstack_chksum.so) never links or calls it.
 *
 * This is a scalar restatement, in plain C, of the reference's algorithm
 * (ambrop72/aipstack, src/aipstack/infra/Chksum.h). It deliberately follows the
 * reference's word-at-a-time loop and its chunk-combining rule literally, so it is
 * independent of the GPU kernels' arithmetic (aligned 16-byte little-endian loads,
 * masks, wave reductions). Parity is pinned by:
 *   - tests/golden/ fixtures: vectors produced by the reference's own Chksum.h compiled in
 *     the survey container (oracle/ref_chksum_wrapper.cpp -> oracle/_ref/), and
 *   - the reference test's known answer (tests/ip_chksum_test.cpp:45-62): 1023 x 0xFF
 *     as a 512-node chain -> IpChksum == 0x00FF.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "chksum_oracle.h"

/* Big-endian 16-bit decode: ReadSingleField<uint16_t>
 * (reference Struct.h:586-590 -> BinaryTools.h:107-125, BigEndian). */
static inline uint32_t be16(const unsigned char *p)
{
    return ((uint32_t)p[0] << 8) | (uint32_t)p[1];
}

/* IpChksumInverted (reference Chksum.h:77-99).
 * 1. sum big-endian 16-bit words below len & ~1 into a uint32 (:82-88);
 * 2. odd tail byte added as the high byte (:90-93);
 * 3. fold (s & 0xFFFF) + (s >> 16) twice (:95-96); truncate to 16 bits. */
uint16_t oracle_chksum_inverted(const void *data, size_t len)
{
    const unsigned char *p = (const unsigned char *)data;
    const unsigned char *even_end = p + (len & ~(size_t)1);
    uint32_t sum = 0;
    while (p < even_end) {
        sum += be16(p);
        p += 2;
    }
    if (len & 1)
        sum += (uint32_t)p[0] << 8;
    sum = (sum & 0xFFFFu) + (sum >> 16);
    sum = (sum & 0xFFFFu) + (sum >> 16);
    return (uint16_t)sum;
}

/* IpChksum(ptr, len) (reference Chksum.h:122-125). */
uint16_t oracle_chksum(const void *data, size_t len)
{
    return (uint16_t)~oracle_chksum_inverted(data, len);
}

/* IpChksumAccumulator::swapBytes (reference Chksum.h:277-281). */
static inline uint32_t swap_bytes32(uint32_t x)
{
    return ((x >> 8) & 0x00FF00FFu) | ((x << 8) & 0xFF00FF00u);
}

/* IpChksumAccumulator(State) + getChksum(IpBufRef) over an explicit chunk list
 * (reference Chksum.h:171-174, 263-269, 283-315; the chunk walk is
 * ipBufProcessBytes, BufUtils.h:129-178, which skips empty chunks).
 * Per chunk: add IpChksumInverted(chunk) with end-around carry (:294-300);
 * odd chunk length -> swapBytes(m_sum) and toggle `swapped` (:303-306);
 * at the end swap once more if `swapped` (:312-314);
 * getChksum(): foldOnce twice, invert (:245-250, :272-275). */
uint16_t oracle_chksum_chain(uint32_t state, const void *const *ptrs,
                             const size_t *lens, size_t nchunks)
{
    uint32_t sum = state;
    int swapped = 0;
    for (size_t i = 0; i < nchunks; i++) {
        if (lens[i] == 0)
            continue;
        uint16_t b = oracle_chksum_inverted(ptrs[i], lens[i]);
        uint32_t old = sum;
        sum += b;
        if (sum < old)
            sum++;
        if (lens[i] & 1) {
            sum = swap_bytes32(sum);
            swapped = !swapped;
        }
    }
    if (swapped)
        sum = swap_bytes32(sum);
    sum = (sum & 0xFFFFu) + (sum >> 16);
    sum = (sum & 0xFFFFu) + (sum >> 16);
    return (uint16_t)~sum;
}

/* Batch helpers: loops of the scalar routine above (for parity tests and the
 * "port" CPU baseline). flags bit 0 = write the final (~) checksum. */
void oracle_batch_strided(const void *base, uint64_t stride, uint32_t len,
                          uint64_t n, uint16_t *out, uint32_t flags)
{
    const unsigned char *b = (const unsigned char *)base;
    for (uint64_t i = 0; i < n; i++) {
        uint16_t v = oracle_chksum_inverted(b + i * stride, len);
        out[i] = (flags & 1u) ? (uint16_t)~v : v;
    }
}

void oracle_batch_csr(const void *base, const uint64_t *offsets, uint64_t n,
                      uint16_t *out, uint32_t flags)
{
    const unsigned char *b = (const unsigned char *)base;
    for (uint64_t i = 0; i < n; i++) {
        uint16_t v = oracle_chksum_inverted(b + offsets[i],
                                            (size_t)(offsets[i + 1] - offsets[i]));
        out[i] = (flags & 1u) ? (uint16_t)~v : v;
    }
}

/* Ring slots: packet i = the lens[i] bytes at base + i * stride (IpChksumInverted per packet,
 * Chksum.h:77-99, as the CSR batch). */
void oracle_batch_slotted(const void *base, uint64_t stride, const uint32_t *lens, uint64_t n,
                          uint16_t *out, uint32_t flags)
{
    const unsigned char *b = (const unsigned char *)base;
    for (uint64_t i = 0; i < n; i++) {
        uint16_t v = oracle_chksum_inverted(b + i * stride, lens[i]);
        out[i] = (flags & 1u) ? (uint16_t)~v : v;
    }
}

/* Seeded batch: IpChksumAccumulator(State{states[i]}).getChksum(IpBufRef{packet i})
 * -- one contiguous chunk per packet (reference Chksum.h:171-174, 263-269). */
void oracle_batch_seeded_csr(const void *base, const uint64_t *offsets,
                             const uint32_t *states, uint64_t n, uint16_t *out)
{
    const unsigned char *b = (const unsigned char *)base;
    for (uint64_t i = 0; i < n; i++) {
        const void *p = b + offsets[i];
        size_t l = (size_t)(offsets[i + 1] - offsets[i]);
        out[i] = oracle_chksum_chain(states[i], &p, &l, 1);
    }
}

/* n chains (the C-ABI's aipstack_chksum_batch_chain): chain i = chunks
 * [index[i], index[i+1]), chunk k = len[k] bytes at address addr[k], which is read at
 * base + (addr[k] - addr_bias) (a host copy of device memory). states == NULL: state 0.
 * flags bit 0 = the final checksum (IpChksumAccumulator::getChksum), else its NOT. */
void oracle_batch_chain(const void *base, uint64_t addr_bias, const uint64_t *addr,
                        const uint32_t *len, const uint64_t *index, const uint32_t *states,
                        uint64_t n, uint16_t *out, uint32_t flags)
{
    const unsigned char *b = (const unsigned char *)base;
    size_t cap = 0;
    const void **ptrs = NULL;
    size_t *lens = NULL;
    for (uint64_t i = 0; i < n; i++) {
        const size_t m = (size_t)(index[i + 1] - index[i]);
        if (m > cap) {
            cap = m * 2;
            ptrs = (const void **)realloc((void *)ptrs, cap * sizeof *ptrs);
            lens = (size_t *)realloc(lens, cap * sizeof *lens);
        }
        for (size_t k = 0; k < m; k++) {
            ptrs[k] = b + (addr[index[i] + k] - addr_bias);
            lens[k] = len[index[i] + k];
        }
        const uint16_t v = oracle_chksum_chain(states ? states[i] : 0u, ptrs, lens, m);
        out[i] = (flags & 1u) ? v : (uint16_t)~v;
    }
    free((void *)ptrs);
    free(lens);
}
