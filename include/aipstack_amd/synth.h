/*
 * aipstack_amd -- deterministic synthetic packet batches (bench / test plumbing).
 *
 * The byte stream is counter-based so that any slice can be produced independently on
 * the host or on the device and the two agree bit for bit:
 *
 *   word(seed, k)  = splitmix64 finaliser of (seed + (k + 1) * 0x9E3779B97F4A7C15)
 *   byte(seed, i)  = (word(seed, i >> 3) >> (8 * (i & 7))) & 0xFF
 *
 * Mixed-length batches (BASELINE config C): packet i has length
 *   64 + word(len_seed, i) % 1437            (uniform in [64, 1500])
 * packed back to back (CSR offsets, so starts can be odd), and a class
 *   word(len_seed ^ AIPSTACK_SYNTH_CLASS_SALT, i) % 100
 * 0 -> every byte 0xFF; 1 -> every byte 0x00; 2 -> a nonzero packet whose word sum is
 * = 0 (mod 0xFFFF): all bytes 0xFF, except byte 0 = 0x00 when the length is odd
 * (inverted checksum 0xFFFF); else random bytes byte(data_seed, offset).
 */
#ifndef AIPSTACK_AMD_SYNTH_H
#define AIPSTACK_AMD_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AIPSTACK_SYNTH_CLASS_SALT 0xC1A55EEDull
#define AIPSTACK_SYNTH_MIN_LEN 64u
#define AIPSTACK_SYNTH_MAX_LEN 1500u

/* Host: buf[i] = byte(seed, byte_offset + i), i < nbytes. Multi-threaded. */
void aipstack_synth_fill_host(void *buf, uint64_t nbytes, uint64_t seed, uint64_t byte_offset);

/* Host: offsets[0..n] of a mixed-length batch (offsets[0] = 0). Returns total bytes. */
uint64_t aipstack_synth_mixed_offsets_host(uint64_t *offsets, uint64_t n, uint64_t len_seed);

/* Host: apply the packet classes of a mixed batch to a buffer already filled with
 * random bytes. Local packet p is global packet first_packet + p (a shard of a larger
 * batch; offsets are local). */
void aipstack_synth_apply_classes_host(void *buf, const uint64_t *offsets, uint64_t n,
                                       uint64_t len_seed, uint64_t first_packet);

/* Device, stream-ordered: d_buf[i] = byte(seed, byte_offset + i). */
int aipstack_synth_fill_device(void *d_buf, uint64_t nbytes, uint64_t seed,
                               uint64_t byte_offset, void *stream);

/* Device, stream-ordered: the class pass of a mixed batch (d_offsets on the device). */
int aipstack_synth_apply_classes_device(void *d_buf, const uint64_t *d_offsets, uint64_t n,
                                        uint64_t len_seed, uint64_t first_packet,
                                        void *stream);

/* Host: n raw Ethernet frames with every checksum field zero (fill them with a Tx-fill
 * pass). Writes offsets[0..n] (frames back to back, first at 0) and, if buf != NULL, the
 * bytes; returns the total size. Per frame i, from word(seed ^ AIPSTACK_SYNTH_FRAME_SALT,
 * 8i + k): 50 % TCP (20-60 B header), 28 % UDP, 10 % ICMP, 5 % other IP protocol (47),
 * 4 % ARP (EtherType 0x0806), 3 % IPv4 fragments (MF / offset set); IHL 5 (85 %) or 6-15
 * with option bytes; payload 0..max_payload bytes; frames shorter than 60 B are padded
 * with zeros past the IPv4 total length (Ethernet minimum). Header fields other than
 * lengths / protocol / checksums and all payload bytes are byte(seed, .) of the stream. */
#define AIPSTACK_SYNTH_FRAME_SALT 0xF4A3E5ull
uint64_t aipstack_synth_frames_host(void *buf, uint64_t *offsets, uint64_t n, uint64_t seed,
                                    uint32_t max_payload);

#ifdef __cplusplus
}
#endif

#endif
