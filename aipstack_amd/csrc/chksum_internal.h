// aipstack_amd -- internal helpers shared by the host runtime and the kernel launchers.
#ifndef AIPSTACK_AMD_CHKSUM_INTERNAL_H
#define AIPSTACK_AMD_CHKSUM_INTERNAL_H

#include <hip/hip_runtime.h>

namespace aipstack_amd {

// Records `e` as this thread's last HIP error and maps it to a status code.
int check_hip(hipError_t e);

// Makes `device` current for the scope and restores the caller's device after it: the
// engine's calls must not change which device the calling thread (e.g. torch) works on.
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(device) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// Compute units of the device `stream` belongs to (the current device for the null
// stream), cached per device id; <= 0 on failure.
int device_cu_count(hipStream_t stream);

// Where a Tx frame launch takes its header segments from (frame_kernels.hip kHdr*): the
// tunable "tx_gather" (0 per-lane loads, 1 captured from the stream, 2 captured + the field
// lines touched up front), else `family_default` for the kind of launch.
int tuning_tx_header_mode(int family_default);

// How the in-place Tx fills store the checksum fields (frame_kernels.hip FieldSectors): the
// tunable "tx_store" (0 = 2-byte field stores, 1 = whole sectors), else `family_default`.
constexpr int kTxStoreFields = 0, kTxStoreSectors = 1, kTxStoreLines = 2;
int tuning_tx_store(int family_default);

// Chains: chunks of at most this many bytes are read first in a group's gathered stream
// (tunable "chain_short"; 0 = the table's order, -1 = the default, 128).
int tuning_chain_short();

// The contract-violation word of each kernel translation unit on the current device:
// OR it into *mask, clear it if `clear`.
// The strided / CSR checksum batches with the caller saying where the packet bytes are:
// host_bytes = read over the link from page-locked host memory (the engine's zero-copy
// pieces), where stream mode reads better than the gathered stream, and slots mask their
// edges in the stream rather than read them twice.
int batch_strided_from(const void *d_base, uint64_t stride, uint32_t len, uint64_t n,
                       uint16_t *d_out, uint32_t flags, void *stream, bool host_bytes);
int batch_csr_from(const void *d_base, const uint64_t *d_offsets, uint64_t n, uint16_t *d_out,
                   uint32_t flags, void *stream, bool host_bytes);
int batch_slotted_from(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                       uint64_t n, uint16_t *d_out, uint32_t flags, void *stream,
                       bool host_bytes);
int rx_verify_slotted_from(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                           uint64_t n, uint8_t *d_verdict, void *stream, bool host_bytes);
int tx_fill_records_slotted_from(const void *d_base, uint64_t slot_stride, const uint32_t *d_len,
                                 uint64_t n, uint64_t *d_records, void *stream, bool host_bytes);
int take_violations_batch(uint32_t *mask, bool clear);
int take_violations_frames(uint32_t *mask, bool clear);

// Frames a wave of the Rx-verify / Tx-fill kernels keeps in flight (tunable "frames":
// 2, 4 or 8; default 4).
int tuning_frames_in_flight();
// Frames per chunk of the frame kernels: 64, or fewer for a small batch (pick_shape).
uint32_t frames_per_chunk(uint64_t n, int cus);
// The "chunk_packets" tunable (0 = automatic).
int tuning_chunk_packets();
// Dynamic LDS per block for a launch whose own default is `family_default` bytes (tunable
// lds_pad: > 0 that many bytes, -1 none): fewer blocks fit a CU, so fewer waves run per SIMD.
unsigned tuning_lds_pad(int family_default);

// Resident-wave budget per CU the grids are sized to (tunable "waves_per_cu"; 0 = each
// kernel's default).
int tuning_waves_per_cu();

// Stream-mode windows a wave issues together (tunable "stream": 2, 4, 8; 0 = stream mode
// off), with the default of the given kernel family when the tunable is automatic.
int tuning_stream_windows(int family_default);
// Host engine: kernels read registered input in place (1) or the engine DMAs it (0); pieces of
// at most tuning_engine_zero_copy_small() packets keep offsets / results in pinned staging.
int tuning_engine_zero_copy();
int tuning_engine_zero_copy_small();
int tuning_engine_pageable_rows();  // pageable ring slots: frame bytes staged, read in place

}  // namespace aipstack_amd

struct aipstack_chksum_engine;
namespace aipstack_amd {
// Host engine internals shared with the engine group (chksum_engine.cpp).
// The region (page-locked by the group, portable) as input of this engine too; returns
// whether the engine's kernels read it in place (mapped into this device's address space).
bool engine_adopt_region(aipstack_chksum_engine *e, const void *p, uint64_t bytes);
void engine_drop_region(aipstack_chksum_engine *e, const void *p);
}  // namespace aipstack_amd

#endif
