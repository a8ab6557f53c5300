/*
 * aipstack_amd -- MI355X (gfx950) Internet-checksum engine: the C-ABI boundary.
 *
 * Plain C, plain pointers and sizes: callable from C, C++, cgo, ctypes, JNI.
 * Implemented by libaipstack_chksum.so (aipstack_amd/lib/), which holds the host
 * C++ code and the hand-written CDNA4 HIP kernels.
 *
 * Two kinds of entry point:
 *
 * 1. The per-packet link-time hook of the reference,
 *      uint16_t IpChksumInverted(char const *data, size_t len);
 *    which replaces the inline default in reference src/aipstack/infra/Chksum.h:77-99
 *    when the consumer compiles with -DAIPSTACK_EXTERNAL_CHKSUM (declaration at
 *    Chksum.h:50-51; contract at Chksum.h:54-76). This one runs on the HOST: a GPU
 *    launch (microseconds) costs more than the whole scalar computation of one packet.
 *
 * 2. The batch entry points (aipstack_chksum_batch_*): the reference has no batch API
 *    (every caller -- IpChksum(ptr,len) Chksum.h:122-125, IpChksumAccumulator::addIpBuf
 *    Chksum.h:283-315 -- processes one packet at a time), so these are new. Each is the
 *    batched equivalent of a reference call, evaluated for many packets at once on the
 *    GPU. All pointers named d_* are DEVICE pointers (hipMalloc'd or HIP-registered);
 *    the work is enqueued on `stream` (a hipStream_t; NULL = the legacy default stream)
 *    and is complete when the stream is. Nothing here allocates or synchronises.
 *    There is no CPU fallback: on a host without a usable gfx950 device these return
 *    AIPSTACK_CHKSUM_EHIP / _ENODEV.
 *
 * Results are bit-exact with the reference for every packet whose length satisfies
 * the reference precondition len <= 65535 (Chksum.h:73-74).
 */
#ifndef AIPSTACK_AMD_CHKSUM_H
#define AIPSTACK_AMD_CHKSUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (0 = success, negative = failure) ---------------------------- */
#define AIPSTACK_CHKSUM_OK      0
#define AIPSTACK_CHKSUM_EINVAL (-1) /* bad argument: null pointer, len > 65535, n too big */
#define AIPSTACK_CHKSUM_EHIP   (-2) /* HIP runtime error (see aipstack_chksum_last_hip_error) */
#define AIPSTACK_CHKSUM_ENODEV (-3) /* no gfx950 device visible to this process */

/* Largest packet length the reference admits (Chksum.h:73-74). */
#define AIPSTACK_CHKSUM_MAX_LEN 65535u

/* Largest slot stride of the frame batches on ring slots (their 64-frame header window must
 * span at most 4 MiB); a larger one is _EINVAL. */
#define AIPSTACK_CHKSUM_MAX_SLOT_STRIDE 65536u

/* ---- flags for the batch entry points ------------------------------------------ */
/* Write IpChksum (= ~IpChksumInverted, Chksum.h:122-125) instead of the inverted sum. */
#define AIPSTACK_CHKSUM_FINAL 1u
/* Hint (results are identical with or without it): the batch's bytes were written by device
 * kernels with ordinary (write-back) stores since they were last read -- e.g. segments
 * assembled on the device just before their checksum. On gfx950 a cached read of such a line
 * costs the memory side far more than a streaming one, so the batch is then read without
 * touching any of its lines through the L2-allocating path (config A: 242-258 us against
 * 285-312 for the default form; the default form is faster on bytes that arrived by DMA or
 * streaming stores, and on bytes read before). Honoured by aipstack_chksum_batch_strided
 * (back-to-back packets of >= 1 KiB: boundary segments captured from the stream; packets at a
 * stride: their edge segments read nontemporal), aipstack_chksum_batch_slotted (edge segments
 * nontemporal) and the chain batches (payload pieces that lie back to back read as column runs
 * with their boundary segments captured from the stream, CHAIN 322.5 against 365.3 us on
 * plain-written chains; other layouts: edge segments nontemporal); ignored elsewhere. */
#define AIPSTACK_CHKSUM_JUST_WRITTEN 4u

/* ---- 1. per-packet host hook ----------------------------------------------------- */

/* Replaces reference Chksum.h:77-99 (declared at Chksum.h:51 under
 * AIPSTACK_EXTERNAL_CHKSUM). Inverted checksum (ones'-complement sum of big-endian
 * 16-bit words; odd tail byte padded with a zero low byte) of `len` bytes at `data`,
 * any alignment. data must not be null; len <= 65535. Pure, reentrant, thread-safe. */
uint16_t IpChksumInverted(const char *data, size_t len);

/* ---- 2. batch entry points (device-resident, stream-ordered) -------------------- */

/* Fixed-stride batch: packet i is the `len` bytes at d_base + i*stride, for i < n.
 * d_out[i] = IpChksumInverted(packet i)   (or IpChksum(...) with AIPSTACK_CHKSUM_FINAL).
 * Batched equivalent of n calls of reference IpChksumInverted (Chksum.h:77-99) /
 * IpChksum (Chksum.h:122-125). d_base may have any byte alignment. */
int aipstack_chksum_batch_strided(const void *d_base, uint64_t stride, uint32_t len,
                                  uint64_t n, uint16_t *d_out, uint32_t flags,
                                  void *stream);

/* CSR batch: packet i is bytes [d_offsets[i], d_offsets[i+1]) of d_base (n+1 offsets,
 * non-decreasing, each packet <= 65535 bytes; starts may be odd).
 * d_out[i] as for the strided form. */
int aipstack_chksum_batch_csr(const void *d_base, const uint64_t *d_offsets,
                              uint64_t n, uint16_t *d_out, uint32_t flags,
                              void *stream);

/* Ring-slot batch: packet i is the d_len[i] bytes at d_base + i*slot_stride -- a receive
 * ring that holds one frame per fixed-size slot with its length beside it (the TAP driver
 * reads one frame per buffer, reference tap/linux/TapDeviceLinux.cpp:156-178), checksummed
 * where it lies, without compacting it first. The buffer holds n whole slots; each
 * d_len[i] <= min(slot_stride, 65535) (a longer one is clamped to that and reported through
 * aipstack_chksum_contract_violations). d_out[i] as for the strided form. */
int aipstack_chksum_batch_slotted(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                                  uint64_t n, uint16_t *d_out, uint32_t flags, void *stream);

/* Seeded CSR batch: d_out[i] = IpChksumAccumulator(State{d_states[i]})
 *                                  .getChksum(IpBufRef{packet i})
 * i.e. a per-packet saved accumulator state (pseudo-header / header words, exported by
 * IpChksumAccumulator::getState, Chksum.h:171-184) resumed and completed over the
 * packet bytes (Chksum.h:263-269, 283-315). Writes the FINAL checksum (as getChksum
 * does). A state of 0 with no header words is the plain IpChksum(IpBufRef). */
int aipstack_chksum_batch_seeded_csr(const void *d_base, const uint64_t *d_offsets,
                                     const uint32_t *d_states, uint64_t n,
                                     uint16_t *d_out, void *stream);

/* Chained (scatter-gather) batch: chain i is the chunks [d_chunk_index[i],
 * d_chunk_index[i+1]) of the chunk table, taken in order as one logical byte sequence:
 * chunk k is the d_chunk_len[k] bytes at DEVICE address d_chunk_addr[k] (any alignment,
 * each <= 65535 bytes). This is an IpBufRef chain (reference Buf.h:68-251) flattened into
 * the non-empty chunks ipBufProcessBytes visits (BufUtils.h:129-178). With
 * AIPSTACK_CHKSUM_FINAL, d_out[i] = IpChksumAccumulator(State{s_i}).getChksum(chain i)
 * (Chksum.h:171-174, 263-315), s_i = d_states[i] or 0 when d_states is NULL; without
 * the flag, the bitwise NOT of that (the inverted sum). n+1 index entries. */
int aipstack_chksum_batch_chain(const uint64_t *d_chunk_addr, const uint32_t *d_chunk_len,
                                const uint64_t *d_chunk_index, const uint32_t *d_states,
                                uint64_t n, uint16_t *d_out, uint32_t flags, void *stream);

/* Flag of aipstack_chksum_batch_chain_fill: a computed checksum of 0 is sent as 0xFFFF
 * (UDP, reference udp/IpUdpProto.h:176-178). */
#define AIPSTACK_CHKSUM_ZERO_AS_FFFF 2u

/* The send side of the chained batch: the reference's Tx call sites sum a pseudo-header
 * State, the header node and the payload chunks, then write the checksum into the header
 * (tcp/IpTcpProto_output.h:1251-1277, udp/IpUdpProto.h:164-179, ip/IpStack.h:1184).
 * Computes the FINAL checksum of chain i into d_out[i] as aipstack_chksum_batch_chain does,
 * then (a second, stream-ordered pass) stores it big-endian at DEVICE address
 * d_field_addr[i] (any alignment; 0 = no store). As in the reference, the field's two bytes
 * must read 0 when the batch runs (they are summed), and no field may lie inside another
 * chain's bytes. Flags: AIPSTACK_CHKSUM_ZERO_AS_FFFF. */
int aipstack_chksum_batch_chain_fill(const uint64_t *d_chunk_addr, const uint32_t *d_chunk_len,
                                     const uint64_t *d_chunk_index, const uint32_t *d_states,
                                     const uint64_t *d_field_addr, uint64_t n,
                                     uint16_t *d_out, uint32_t flags, void *stream);

/* ---- frame-level batches: Rx verify / Tx fill on raw Ethernet frames ------------------ */

/* Per-frame verdicts of aipstack_chksum_rx_verify (and statuses of _tx_fill), restating the
 * reference's receive-path decisions that involve checksums or the lengths they cover:
 * eth/EthIpIface.h:367-390, ip/IpStack.h:936-1018 and :1093-1130 (ICMP),
 * tcp/IpTcpProto_input.h:68-100, udp/IpUdpProto.h:470-490 and :631-652. Checks that need
 * stack state (interface addresses, listeners, reassembly) stay with the host. */
#define AIPSTACK_RX_NOT_IP4            0 /* < 14 bytes or EtherType != 0x0800 (e.g. ARP) */
#define AIPSTACK_RX_DROP_IP_MALFORMED  1 /* IPv4 header/length checks fail (IpStack.h:938-990) */
#define AIPSTACK_RX_DROP_IP_CHKSUM     2 /* IPv4 header checksum bad (IpStack.h:1016) */
#define AIPSTACK_RX_FRAGMENT           3 /* header OK, MF or offset set: host reassembles */
#define AIPSTACK_RX_DROP_L4_MALFORMED  4 /* TCP < 20 B, UDP length bad, ICMP < 8 B */
#define AIPSTACK_RX_DROP_L4_CHKSUM     5 /* TCP/UDP/ICMP checksum bad */
#define AIPSTACK_RX_ACCEPT             6 /* every checksum present verified */
#define AIPSTACK_RX_ACCEPT_NO_CHKSUM   7 /* UDP with checksum field 0 = none (IpUdpProto.h:637) */
#define AIPSTACK_RX_ACCEPT_OTHER       8 /* IPv4 header OK; protocol other than TCP/UDP/ICMP */

/* Rx verify: frame i = bytes [d_offsets[i], d_offsets[i+1]) of d_base (an Ethernet frame,
 * as the TAP driver delivers it); d_verdict[i] = one of AIPSTACK_RX_*. Read-only.
 * Frame offsets (here and in the Tx fills) are non-decreasing (n+1 entries) and each frame
 * is at most 65535 bytes, so that 64 consecutive frames span at most 4 MiB: the kernels
 * read a 64-frame chunk's header bytes through one range-checked window over that span.
 * Offsets outside this contract give unspecified verdicts (never accesses outside the
 * chunk's span). */
int aipstack_chksum_rx_verify(const void *d_base, const uint64_t *d_offsets, uint64_t n,
                              uint8_t *d_verdict, void *stream);

/* Tx fill, IN PLACE: for each IPv4 frame, write the IPv4 header checksum (field taken as 0,
 * ip/IpStack.h:425-453) and, unless it is a fragment, the TCP / UDP (0 -> 0xFFFF) / ICMP
 * checksum (tcp/IpTcpProto_output.h:1251-1277, udp/IpUdpProto.h:164-179,
 * ip/IpStack.h:1164-1190). d_status[i]: AIPSTACK_RX_ACCEPT (filled), _ACCEPT_OTHER (IPv4
 * header only), _FRAGMENT (IPv4 header only), _NOT_IP4 / _DROP_*_MALFORMED (untouched,
 * or IPv4 header only for L4-malformed). Frames must not overlap. */
int aipstack_chksum_tx_fill(void *d_base, const uint64_t *d_offsets, uint64_t n,
                            uint8_t *d_status, void *stream);

/* Tx fill in two stream-ordered passes, same results as aipstack_chksum_tx_fill: a read pass
 * computes every frame's fields into d_workspace (8 bytes per frame, 8-byte aligned, at
 * least aipstack_chksum_tx_fill_workspace_bytes(n) bytes, owned by the caller and free
 * again once the stream passes the call), then a scatter pass stores them into the frames.
 * Round 5: no faster than the one pass at any batch size measured (1 M frames: 194.5 vs
 * 193.4 us); for callers that want the stores as a pass of their own. */
uint64_t aipstack_chksum_tx_fill_workspace_bytes(uint64_t n);
int aipstack_chksum_tx_fill_split(void *d_base, const uint64_t *d_offsets, uint64_t n,
                                  uint8_t *d_status, void *d_workspace,
                                  uint64_t workspace_bytes, void *stream);

/* The split fill's read pass alone: per frame the 8-byte record the scatter pass would
 * apply, frames untouched -- for a caller that applies the fields itself (the host-memory
 * engine's Tx fill, or a NIC path that patches headers on the way out). Record of frame i:
 * bits 0-15 the IPv4 header checksum, 16-31 the L4 checksum (the field values, big-endian
 * when stored), 32-39 the L4 field's offset from the frame start, bit 40 = write the IPv4
 * field (at offset 24), bit 41 = write the L4 field, bits 48-55 the status (AIPSTACK_RX_*).
 * d_records 8-byte aligned, n entries. */
int aipstack_chksum_tx_fill_records(const void *d_base, const uint64_t *d_offsets, uint64_t n,
                                    uint64_t *d_records, void *stream);

/* The frame batches on a ring of slots (layout as aipstack_chksum_batch_slotted: frame i is
 * the d_len[i] bytes at d_base + i*slot_stride, 0 < slot_stride <=
 * AIPSTACK_CHKSUM_MAX_SLOT_STRIDE, else _EINVAL; n whole slots): Rx verify, the one-pass
 * in-place Tx fill, the split fill (records pass + scatter pass through a caller-owned
 * workspace, as aipstack_chksum_tx_fill_split), and the Tx records. Same results per frame as
 * the CSR forms. */
int aipstack_chksum_rx_verify_slotted(const void *d_base, uint64_t slot_stride,
                                      const uint32_t *d_len, uint64_t n, uint8_t *d_verdict,
                                      void *stream);
int aipstack_chksum_tx_fill_slotted(void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                                    uint64_t n, uint8_t *d_status, void *stream);
int aipstack_chksum_tx_fill_slotted_split(void *d_base, uint64_t slot_stride,
                                          const uint32_t *d_len, uint64_t n, uint8_t *d_status,
                                          void *d_workspace, uint64_t workspace_bytes,
                                          void *stream);
int aipstack_chksum_tx_fill_records_slotted(const void *d_base, uint64_t slot_stride,
                                            const uint32_t *d_len, uint64_t n,
                                            uint64_t *d_records, void *stream);

/* ---- 3. host-memory streaming engine ----------------------------------------------- */

/* The reference's packet path starts and ends in host memory (TAP read()/write(),
 * reference tap/linux/TapDeviceLinux.cpp:122-178). An engine checksums batches held in
 * HOST memory and writes the results to HOST memory, pipelining H2D copies, kernels and
 * D2H copies over `nstreams` HIP streams in chunks of at most `chunk_bytes` (0 = 64 MiB)
 * of whole packets. Host buffers registered with aipstack_chksum_engine_register()
 * (page-locked once, e.g. a receive ring) are read by the kernels where they lie, over the
 * link (only the bytes the packets cover cross it: for ring slots not the slack); with
 * aipstack_chksum_tune("engine_zero_copy", 0) before the engine is created they are DMA'd
 * to the device first instead. Other host memory is first copied into the engine's pinned
 * staging (a ring of slots: each frame's bytes only, read there by the kernel; tune
 * "engine_pageable_rows" 0 = whole slots, DMA'd). The host_* calls are synchronous; the submit_*
 * calls enqueue a batch and return a ticket at once, so the caller can fill its next batch
 * (e.g. read() frames into its ring) while the GPU works; _poll / _wait complete it. Calls
 * on one engine from several threads are serialised, except that _wait waits for the GPU
 * without holding the engine: _poll and _submit_* from other threads proceed meanwhile (a
 * _submit_* that needs a busy stream still waits for the piece on it).
 *
 * Errors are per batch: a piece that fails records its status against its own ticket,
 * whichever call completes it, and _poll / _wait of that ticket return it (once). Destroy
 * completes every piece still in flight as _wait would -- results written, Tx fields
 * applied -- before freeing anything; so does _unregister before it unpins the region. */
typedef struct aipstack_chksum_engine aipstack_chksum_engine;

int aipstack_chksum_engine_create(int device, uint64_t chunk_bytes, int nstreams,
                                  aipstack_chksum_engine **out);
void aipstack_chksum_engine_destroy(aipstack_chksum_engine *engine);
int aipstack_chksum_engine_register(aipstack_chksum_engine *engine, void *host_ptr,
                                    uint64_t bytes);
int aipstack_chksum_engine_unregister(aipstack_chksum_engine *engine, void *host_ptr);

/* h_out[i] for packet i = h_base[i*stride .. +len) (host memory), as the strided batch. */
int aipstack_chksum_engine_host_strided(aipstack_chksum_engine *engine, const void *h_base,
                                        uint64_t stride, uint32_t len, uint64_t n,
                                        uint16_t *h_out, uint32_t flags);

/* h_out[i] for packet i = h_base[h_offsets[i] .. h_offsets[i+1]) (host memory; offsets
 * non-decreasing, each packet <= 65535 bytes, else _EINVAL before any work). */
int aipstack_chksum_engine_host_csr(aipstack_chksum_engine *engine, const void *h_base,
                                    const uint64_t *h_offsets, uint64_t n, uint16_t *h_out,
                                    uint32_t flags);

/* Asynchronous form of the two calls above: enqueue the batch and return at once with
 * *ticket set. h_out is written when the batch completes; a REGISTERED h_base must stay
 * unchanged until then (it is DMA'd while the GPU runs), pageable input is copied before
 * the call returns. At most nstreams chunks are in flight per engine: a submit that needs
 * a busy stream first completes the piece on it. Returns _OK or a negative status (a
 * failure part-way leaves the pieces already enqueued to _wait). */
int aipstack_chksum_engine_submit_strided(aipstack_chksum_engine *engine, const void *h_base,
                                          uint64_t stride, uint32_t len, uint64_t n,
                                          uint16_t *h_out, uint32_t flags, uint64_t *ticket);
int aipstack_chksum_engine_submit_csr(aipstack_chksum_engine *engine, const void *h_base,
                                      const uint64_t *h_offsets, uint64_t n, uint16_t *h_out,
                                      uint32_t flags, uint64_t *ticket);

/* Rx verify of raw Ethernet frames held in HOST memory -- the TAP receive path
 * (tap/linux/TapDeviceLinux.cpp:156-178) batched: h_verdicts[i] = the AIPSTACK_RX_* verdict
 * of frame i = h_base[h_offsets[i] .. h_offsets[i+1]), as aipstack_chksum_rx_verify
 * (offsets non-decreasing, each frame <= 65535 bytes, else _EINVAL before any work).
 * Synchronous and submit forms, as above. */
int aipstack_chksum_engine_host_rx_verify(aipstack_chksum_engine *engine, const void *h_base,
                                          const uint64_t *h_offsets, uint64_t n,
                                          uint8_t *h_verdicts);
int aipstack_chksum_engine_submit_rx_verify(aipstack_chksum_engine *engine, const void *h_base,
                                            const uint64_t *h_offsets, uint64_t n,
                                            uint8_t *h_verdicts, uint64_t *ticket);

/* Tx fill of raw Ethernet frames held in HOST memory -- the TAP send path batched
 * (tap/linux/TapDeviceLinux.cpp:122-127): the frames go to the device, the Tx fill's read
 * pass computes each frame's record (aipstack_chksum_tx_fill_records), 8 bytes per frame come
 * back, and the engine writes the IPv4 header and L4 checksum fields into the caller's
 * frames IN PLACE and h_status[i] (as aipstack_chksum_tx_fill) when the batch completes (poll
 * or wait). A submitted batch's frames, offsets and statuses must stay valid until then (or
 * until the engine is destroyed, which completes it). */
int aipstack_chksum_engine_host_tx_fill(aipstack_chksum_engine *engine, void *h_base,
                                        const uint64_t *h_offsets, uint64_t n,
                                        uint8_t *h_status);
int aipstack_chksum_engine_submit_tx_fill(aipstack_chksum_engine *engine, void *h_base,
                                          const uint64_t *h_offsets, uint64_t n,
                                          uint8_t *h_status, uint64_t *ticket);

/* The same three on a ring of slots in HOST memory (layout as aipstack_chksum_batch_slotted:
 * frame i is the h_len[i] bytes at h_base + i*slot_stride; the buffer holds n whole slots;
 * every h_len[i] <= min(slot_stride, 65535) and slot_stride <= chunk_bytes, else _EINVAL
 * before any work). Pieces are runs of whole slots, copied as they lie (slack included). */
int aipstack_chksum_engine_host_slotted(aipstack_chksum_engine *engine, const void *h_base,
                                        uint64_t slot_stride, const uint32_t *h_len, uint64_t n,
                                        uint16_t *h_out, uint32_t flags);
int aipstack_chksum_engine_submit_slotted(aipstack_chksum_engine *engine, const void *h_base,
                                          uint64_t slot_stride, const uint32_t *h_len, uint64_t n,
                                          uint16_t *h_out, uint32_t flags, uint64_t *ticket);
int aipstack_chksum_engine_host_rx_verify_slotted(aipstack_chksum_engine *engine,
                                                  const void *h_base, uint64_t slot_stride,
                                                  const uint32_t *h_len, uint64_t n,
                                                  uint8_t *h_verdicts);
int aipstack_chksum_engine_submit_rx_verify_slotted(aipstack_chksum_engine *engine,
                                                    const void *h_base, uint64_t slot_stride,
                                                    const uint32_t *h_len, uint64_t n,
                                                    uint8_t *h_verdicts, uint64_t *ticket);
int aipstack_chksum_engine_host_tx_fill_slotted(aipstack_chksum_engine *engine, void *h_base,
                                                uint64_t slot_stride, const uint32_t *h_len,
                                                uint64_t n, uint8_t *h_status);
int aipstack_chksum_engine_submit_tx_fill_slotted(aipstack_chksum_engine *engine, void *h_base,
                                                  uint64_t slot_stride, const uint32_t *h_len,
                                                  uint64_t n, uint8_t *h_status,
                                                  uint64_t *ticket);

/* Completion of a submitted batch: 0 = done (h_out holds the results), 1 = still running
 * (poll only), negative = one of its pieces failed (the first failure's status; h_out /
 * the frames of the failed pieces are not written), or _EINVAL for a ticket never issued.
 * _wait blocks. A ticket's failure is reported once; completing it again returns 0. */
int aipstack_chksum_engine_poll(aipstack_chksum_engine *engine, uint64_t ticket);
int aipstack_chksum_engine_wait(aipstack_chksum_engine *engine, uint64_t ticket);

/* Where the engine's host threads run: the NUMA node of its device (-1 unknown) and how many
 * of the CPUs next to the device (sysfs local_cpulist, within this process's affinity) its
 * host threads are pinned to (0 = not pinned). Its pinned staging is allocated from them. */
int aipstack_chksum_engine_locality(const aipstack_chksum_engine *engine, int *numa_node,
                                    int *pinned_cpus);
/* 1 if the engine's kernels read the registered region holding host_ptr in place (zero copy),
 * 0 if it is DMA'd to the device first, _EINVAL if host_ptr is in no registered region. */
int aipstack_chksum_engine_region_mapped(aipstack_chksum_engine *engine, const void *host_ptr);

/* ---- 4. several devices in one process -------------------------------------------- */

/* The reference stack is one process on one event-loop thread (event_loop/event_loop.dox:
 * 48-50); a host batch is PCIe-bound per device (~50 GiB/s). An engine group owns one engine
 * per entry of `devices` (repeats allowed) and splits a batch into contiguous ranges of about
 * equal bytes, one per device (a batch of less than 4 MiB per device goes to fewer devices,
 * round robin, whole): disjoint packet ranges, no data exchanged between the devices.
 *
 * The submit_* calls enqueue a batch and return ONE group ticket at once; _poll / _wait
 * complete it: 0 = done, 1 = still running (poll), else the first failure by device order;
 * dev_status (NULL or n_devices ints) then receives each device's status (0 for a device
 * without a range). A ticket is reported once: to the call that completes it and to every
 * _wait already blocked on it then; completing it again afterwards returns 0. Each range is
 * submitted to its engine on the calling thread when the batch lies in a region registered
 * with the group (the kernels read it in place) or is small, else by a persistent worker
 * thread of its device (pinned, like the engine's own host threads, to the CPUs next to the
 * device), so the pageable staging copies of all devices run in parallel while the caller
 * goes on. Every input, output and frame buffer of a submitted batch must stay valid, and its
 * input unchanged, until the ticket completes. A submit returns _OK or a negative status: the
 * argument checks fail before anything starts (*ticket = 0); a range whose engine submit fails
 * on the calling thread leaves *ticket set, the batch's other ranges running, and the failure
 * reported again by _poll / _wait, which must still complete the ticket (as for one engine).
 * The host_* calls are submit + wait.
 * _register page-locks a region once for all devices (portable, mapped into each device). */
typedef struct aipstack_chksum_engine_group aipstack_chksum_engine_group;

int aipstack_chksum_engine_group_create(const int *devices, int n_devices, uint64_t chunk_bytes,
                                        int nstreams, aipstack_chksum_engine_group **out);
void aipstack_chksum_engine_group_destroy(aipstack_chksum_engine_group *group);
int aipstack_chksum_engine_group_size(const aipstack_chksum_engine_group *group);
/* The engine of entry k (owned by the group, valid until it is destroyed), e.g. for
 * aipstack_chksum_engine_locality; NULL for k out of range. */
aipstack_chksum_engine *aipstack_chksum_engine_group_engine(aipstack_chksum_engine_group *group,
                                                            int k);
/* 1 if every engine of the group reads the group-registered region holding host_ptr in place,
 * 0 if some DMA it, _EINVAL if it is not registered with the group. */
int aipstack_chksum_engine_group_region_mapped(aipstack_chksum_engine_group *group,
                                               const void *host_ptr);
int aipstack_chksum_engine_group_register(aipstack_chksum_engine_group *group, void *host_ptr,
                                          uint64_t bytes);
int aipstack_chksum_engine_group_unregister(aipstack_chksum_engine_group *group, void *host_ptr);
int aipstack_chksum_engine_group_host_strided(aipstack_chksum_engine_group *group,
                                              const void *h_base, uint64_t stride, uint32_t len,
                                              uint64_t n, uint16_t *h_out, uint32_t flags,
                                              int *dev_status);
int aipstack_chksum_engine_group_host_csr(aipstack_chksum_engine_group *group, const void *h_base,
                                          const uint64_t *h_offsets, uint64_t n, uint16_t *h_out,
                                          uint32_t flags, int *dev_status);
int aipstack_chksum_engine_group_host_rx_verify(aipstack_chksum_engine_group *group,
                                                const void *h_base, const uint64_t *h_offsets,
                                                uint64_t n, uint8_t *h_verdicts, int *dev_status);
int aipstack_chksum_engine_group_host_tx_fill(aipstack_chksum_engine_group *group, void *h_base,
                                              const uint64_t *h_offsets, uint64_t n,
                                              uint8_t *h_status, int *dev_status);
/* Ring slots (frame i = h_len[i] bytes at h_base + i*slot_stride): contiguous runs of about
 * equal slot counts per device; every length is checked (<= min(slot_stride, 65535)) before
 * any device starts. */
int aipstack_chksum_engine_group_host_slotted(aipstack_chksum_engine_group *group,
                                              const void *h_base, uint64_t slot_stride,
                                              const uint32_t *h_len, uint64_t n, uint16_t *h_out,
                                              uint32_t flags, int *dev_status);
int aipstack_chksum_engine_group_host_rx_verify_slotted(aipstack_chksum_engine_group *group,
                                                        const void *h_base, uint64_t slot_stride,
                                                        const uint32_t *h_len, uint64_t n,
                                                        uint8_t *h_verdicts, int *dev_status);
int aipstack_chksum_engine_group_host_tx_fill_slotted(aipstack_chksum_engine_group *group,
                                                      void *h_base, uint64_t slot_stride,
                                                      const uint32_t *h_len, uint64_t n,
                                                      uint8_t *h_status, int *dev_status);
int aipstack_chksum_engine_group_submit_strided(aipstack_chksum_engine_group *group,
                                                const void *h_base, uint64_t stride, uint32_t len,
                                                uint64_t n, uint16_t *h_out, uint32_t flags,
                                                uint64_t *ticket);
int aipstack_chksum_engine_group_submit_csr(aipstack_chksum_engine_group *group,
                                            const void *h_base, const uint64_t *h_offsets,
                                            uint64_t n, uint16_t *h_out, uint32_t flags,
                                            uint64_t *ticket);
int aipstack_chksum_engine_group_submit_rx_verify(aipstack_chksum_engine_group *group,
                                                  const void *h_base, const uint64_t *h_offsets,
                                                  uint64_t n, uint8_t *h_verdicts, uint64_t *ticket);
int aipstack_chksum_engine_group_submit_tx_fill(aipstack_chksum_engine_group *group, void *h_base,
                                                const uint64_t *h_offsets, uint64_t n,
                                                uint8_t *h_status, uint64_t *ticket);
int aipstack_chksum_engine_group_submit_slotted(aipstack_chksum_engine_group *group,
                                                const void *h_base, uint64_t slot_stride,
                                                const uint32_t *h_len, uint64_t n, uint16_t *h_out,
                                                uint32_t flags, uint64_t *ticket);
int aipstack_chksum_engine_group_submit_rx_verify_slotted(aipstack_chksum_engine_group *group,
                                                          const void *h_base, uint64_t slot_stride,
                                                          const uint32_t *h_len, uint64_t n,
                                                          uint8_t *h_verdicts, uint64_t *ticket);
int aipstack_chksum_engine_group_submit_tx_fill_slotted(aipstack_chksum_engine_group *group,
                                                        void *h_base, uint64_t slot_stride,
                                                        const uint32_t *h_len, uint64_t n,
                                                        uint8_t *h_status, uint64_t *ticket);
int aipstack_chksum_engine_group_poll(aipstack_chksum_engine_group *group, uint64_t ticket,
                                      int *dev_status);
int aipstack_chksum_engine_group_wait(aipstack_chksum_engine_group *group, uint64_t ticket,
                                      int *dev_status);

/* ---- diagnostics ------------------------------------------------------------------ */

/* Contract violations the kernels met on a device since the last clear (sticky bits). The
 * batch calls never fault on inputs outside their contract, but their results for the
 * offending packets are unspecified; these bits say that it happened:
 *   _PACKET_LEN  a CSR packet or frame longer than 65535 bytes, or offsets decreasing (its
 *                result: the exact sum up to 2^26 bytes, else 0; frames: NOT_IP4)
 *   _CHUNK_LEN   a chain chunk longer than 65535 bytes (summed as an empty chunk)
 *   _SPAN        64 consecutive frames spanning more than 4 MiB (their headers read as 0)
 * aipstack_chksum_contract_violations synchronises the whole device (hipDeviceSynchronize:
 * every stream of every engine on it waits), then stores the bits in *mask and, if `clear` is
 * non-zero, clears them in the same atomic exchange (a bit set meanwhile is never lost). */
#define AIPSTACK_CHKSUM_VIOLATION_PACKET_LEN 1u
#define AIPSTACK_CHKSUM_VIOLATION_CHUNK_LEN  2u
#define AIPSTACK_CHKSUM_VIOLATION_SPAN       4u
int aipstack_chksum_contract_violations(int device, uint32_t *mask, int clear);

/* Static description of a status code. Never NULL. */
const char *aipstack_chksum_strerror(int status);

/* hipError_t of the most recent failing HIP call made by this library on the calling
 * thread (0 if none). */
int aipstack_chksum_last_hip_error(void);

/* AIPSTACK_CHKSUM_OK if `device` is a gfx950 device this library can launch on,
 * else _ENODEV (or _EHIP if the HIP runtime itself fails). */
int aipstack_chksum_device_check(int device);

/* Launch tunables, for benchmark sweeps (0 = automatic). Keys: "waves_per_cu",
 * "chunks_per_wave", "stream" (1 KiB windows a wave issues together in stream mode -- a
 * 64-packet or 64-frame chunk that lies back to back in memory, or chain chunks that lie close
 * together: 2, 4, 8; -1 turns stream mode off, so every packet, frame or chunk is summed on its
 * own), "chunk_packets" (packets, frames or chains per wave chunk: 1, 2, 4, ..., 64; automatic
 * = short runs of about 12 KiB, 64 for stream mode (ring slots 8, chains 32), fewer for small
 * batches so that they spread over more waves), "tx_gather" (where the Tx fills take their
 * header segments: 0 per-lane loads, 1 captured from the stream, 2 captured + the two field
 * lines touched up front; -1 = by kind of launch), "tx_store" (how the in-place Tx fills write
 * the two checksum fields: 0 = 2-byte stores, 1 = the fields' whole 32-byte sectors from the
 * header bytes the kernel holds, 2 = a send ring's (slots on the 128-byte grid) first 128-byte
 * line per frame written whole; -1 = the default, 0), "chain_short" (chained batches: chunks of
 * at most this many bytes that share no 128-byte line with their neighbours in the table are
 * read first in each 64-chunk group; 0 = the table's order, -1 = the default, 128), "gather"
 * (strided and CSR checksum batches on packets back to back: 1 = short runs, one ~12 KiB chunk
 * per wave, the default since round 5; 0 = the gathered stream of the packets' segments (round
 * 4); -1 = stream mode, one contiguous run per 64-packet chunk), "short_loads" (short runs: 0
 * stream prefixes, 1 the same through global loads, 2 column runs; -1 = by packet length, the
 * default), "lds_pad" (bytes of dynamic LDS per workgroup of the batch, chain and frame
 * kernels, which caps the workgroups per CU; -1 none, 0 the launch's own). Sweep builds only
 * (tools/build_variant.sh NAME -DAIPSTACK_ALL_VARIANTS; the product build rejects values other
 * than the default): "unroll" (segments per lane issued up front, 1..4), "packets" (packets a
 * wave keeps in flight: 1, 2, 4, 8), "nontemporal" (0/1), "frames" (frames in flight per wave
 * in Rx verify / Tx fill: 2, 4, 8). Process-wide; results never depend on them.
 * Returns _OK or _EINVAL for an unknown key or a rejected value. */
int aipstack_chksum_tune(const char *key, int value);

/* The launch shape the batch entry points pick for n packets on a device with `cus` compute
 * units (host-side query, no GPU needed; honours aipstack_chksum_tune): packets per wave
 * chunk (64, or fewer for a small batch, so that it spreads over more waves) and stream
 * windows in flight per wave, for the strided (csr = 0) or CSR (csr = 1) family.
 * Returns _OK, or _EINVAL for null outputs or cus <= 0. */
int aipstack_chksum_launch_shape(uint64_t n, int cus, int csr, uint32_t *chunk_packets,
                                 int *stream_windows);

/* ABI version of this header: bumped on any incompatible change. */
#define AIPSTACK_CHKSUM_ABI_VERSION 1
int aipstack_chksum_abi_version(void);

/* sha256 (hex) of the sources this library was built from (aipstack_amd/csrc/ *.hip, *.cpp,
 * *.cc, *.h, its Makefile, include/aipstack_amd/ *.h, concatenated in sorted path order):
 * lets a test or a deployment tell a library from a stale build. */
const char *aipstack_chksum_source_digest(void);

#ifdef __cplusplus
}
#endif

#endif /* AIPSTACK_AMD_CHKSUM_H */
