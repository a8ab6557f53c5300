// aipstack_amd -- C++ host surface of the checksum engine.
//
// Mirrors the reference's checksum interface (ambrop72/aipstack src/aipstack/infra):
//   IpChksumInverted            Chksum.h:77-99   (the extern "C" hook, in the .so)
//   IpChksum(ptr, len)          Chksum.h:122-125
//   IpChksumAccumulator         Chksum.h:148-316
//   IpChksum(IpBufRef)          Chksum.h:332-336
//   IpBufNode / IpBufRef        Buf.h:68-83, 118-251
//   ipBufProcessBytes           BufUtils.h:129-178
// in namespace AIpStackAmd, plus BatchChksum: a thin RAII-free C++ wrapper of the GPU
// batch entry points of chksum.h, and HostChksumEngine: the host-memory engine (owning).
//
// Drop-in use inside aipstack itself needs none of this: compile the stack with
// -DAIPSTACK_EXTERNAL_CHKSUM and link libaipstack_chksum.so, whose extern "C"
// IpChksumInverted the reference header then calls (Chksum.h:50-51). This header is for
// code that wants the same calls without the reference headers, and for the batch API.
#ifndef AIPSTACK_AMD_CHKSUM_HPP
#define AIPSTACK_AMD_CHKSUM_HPP

#include <cstddef>
#include <cstdint>

#include "aipstack_amd/chksum.h"

// Assertions follow the reference's configuration (misc/Assert.h): checked only where the
// application defines AIPSTACK_CONFIG_ENABLE_ASSERTIONS; a failure calls the application's
// AIPSTACK_CONFIG_ASSERT_HANDLER(msg) if it has one, else prints the message and aborts.
#ifdef AIPSTACK_CONFIG_ENABLE_ASSERTIONS
#ifdef AIPSTACK_CONFIG_ASSERT_INCLUDE
#include AIPSTACK_CONFIG_ASSERT_INCLUDE
#endif
#include <cstdio>
#include <cstdlib>
#ifdef AIPSTACK_CONFIG_ASSERT_HANDLER
#define AIPSTACK_AMD_ASSERT_FAIL(msg) AIPSTACK_CONFIG_ASSERT_HANDLER(msg)
#else
#define AIPSTACK_AMD_ASSERT_FAIL(msg) \
    (std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, msg), std::abort())
#endif
#define AIPSTACK_AMD_ASSERT(e) \
    ((e) ? (void)0 : (void)(AIPSTACK_AMD_ASSERT_FAIL("Assertion failed: " #e), 0))
#else
#define AIPSTACK_AMD_ASSERT(e) ((void)0)
#endif

namespace AIpStackAmd {

// meta/BasicMetaUtils.h:39-42: the tag type the reference's addWord overloads take
// (IpChksumAccumulator::addWord(WrapType<std::uint16_t>, ...), Chksum.h:191, 213).
template <typename TType>
struct WrapType {
    using Type = TType;
};

// Chksum.h:122-125
inline std::uint16_t IpChksum(char const *data, std::size_t len) {
    return std::uint16_t(~IpChksumInverted(data, len));
}

// Buf.h:68-83
struct IpBufNode {
    char *ptr = nullptr;
    std::size_t len = 0;
    IpBufNode const *next = nullptr;
};

// Buf.h:118-251 (the members the checksum path and its callers use)
struct IpBufRef {
    IpBufNode const *node = nullptr;
    std::size_t offset = 0;
    std::size_t tot_len = 0;

    char *getChunkPtr() const { return node->ptr + offset; }
    std::size_t getChunkLength() const {
        std::size_t rem = node->len - offset;
        return tot_len < rem ? tot_len : rem;
    }
    // Buf.h:186-191: at least `amount` bytes in the first chunk (the Rx paths' header
    // checks, e.g. ip/IpStack.h:939, udp/IpUdpProto.h:473).
    bool hasHeader(std::size_t amount) const {
        return amount <= tot_len && amount <= node->len - offset;
    }
    IpBufRef hideHeader(std::size_t amount) const {
        return IpBufRef{node, offset + amount, tot_len - amount};
    }
    IpBufRef revealHeader(std::size_t amount) const {
        return IpBufRef{node, offset - amount, tot_len + amount};
    }
    IpBufRef subTo(std::size_t new_tot_len) const { return IpBufRef{node, offset, new_tot_len}; }
};

// BufUtils.h:129-178 (same contract): hands `fn(char *ptr, size_t len)` the non-empty
// pieces of the first process_len bytes, node by node; `fn` returns how many bytes of its
// piece it took, and taking fewer ends the walk inside that node. The returned reference
// starts after the bytes taken and keeps everything not taken (tot_len shrinks by exactly
// that count). A node that was used up is left behind even when nothing more is wanted,
// as long as it has a successor -- the reference's eager advance, which also steps over
// empty nodes.
template <typename Fn>
IpBufRef ipBufProcessBytes(IpBufRef buf, std::size_t process_len, Fn &&fn) {
    std::size_t const untouched = buf.tot_len - process_len;
    IpBufNode const *at = buf.node;
    std::size_t pos = buf.offset;  // inside *at
    std::size_t want = process_len;
    for (;;) {
        std::size_t const avail = at->len - pos;
        bool const uses_up_node = want >= avail;
        std::size_t const piece = uses_up_node ? avail : want;
        if (piece != 0) {
            std::size_t const took = fn(at->ptr + pos, piece);
            pos += took;
            want -= took;
            if (took != piece) break;  // the visitor stopped early
        }
        if (!uses_up_node || at->next == nullptr) break;
        at = at->next;
        pos = 0;
    }
    return IpBufRef{at, pos, want + untouched};
}

// Chksum.h:148-316. Same observable behaviour (State export/resume, header words added
// without carry handling, chunk sums with end-around carry, getChksum = fold twice and
// invert). Chunks are combined by their logical byte position: a chunk that starts at
// an odd position contributes its sum byte-swapped, which is what the reference's
// swap-after-odd-chunk rule amounts to (a byte swap is x*256 mod 0xFFFF, and swapping
// twice is the identity).
class IpChksumAccumulator {
public:
    enum class State : std::uint32_t {};

    IpChksumAccumulator() : m_sum(0) {}
    // Chksum.h:171: implicit, as in the reference (`IpChksumAccumulator chksum = state;`).
    IpChksumAccumulator(State state) : m_sum(std::uint32_t(state)) {}

    State getState() const { return State(m_sum); }

    // Chksum.h:191-217: the reference's tag-dispatched word adds.
    void addWord(WrapType<std::uint16_t>, std::uint16_t word) { m_sum += word; }
    void addWord(WrapType<std::uint32_t>, std::uint32_t word) {
        addWord(WrapType<std::uint16_t>(), std::uint16_t(word >> 16));
        addWord(WrapType<std::uint16_t>(), std::uint16_t(word));
    }
    void addWordOctets(std::uint8_t hi, std::uint8_t lo) {
        addWord(WrapType<std::uint16_t>(), std::uint16_t((std::uint16_t(hi) << 8) | lo));
    }
    // Chksum.h:225-235. num_bytes must be even: asserted as the reference asserts it (:227),
    // when the application enables the stack's assertions (AIPSTACK_CONFIG_ENABLE_ASSERTIONS,
    // misc/Assert.h); without them an odd trailing byte is ignored (the reference would read
    // one byte past the range).
    void addEvenBytes(char const *ptr, std::size_t num_bytes) {
        AIPSTACK_AMD_ASSERT(num_bytes % 2 == 0);
        unsigned char const *p = reinterpret_cast<unsigned char const *>(ptr);
        for (std::size_t i = 0; i + 1 < num_bytes; i += 2)
            addWord(WrapType<std::uint16_t>(), std::uint16_t((std::uint16_t(p[i]) << 8) | p[i + 1]));
    }
    // Shorthands for the two addWord overloads (not in the reference).
    void addWord16(std::uint16_t word) { addWord(WrapType<std::uint16_t>(), word); }
    void addWord32(std::uint32_t word) { addWord(WrapType<std::uint32_t>(), word); }

    std::uint16_t getChksum() {
        fold();
        return std::uint16_t(~m_sum);
    }

    std::uint16_t getChksum(IpBufRef buf) {
        if (buf.tot_len > 0) addIpBuf(buf);
        return getChksum();
    }

private:
    void fold() {
        m_sum = (m_sum & 0xFFFFu) + (m_sum >> 16);
        m_sum = (m_sum & 0xFFFFu) + (m_sum >> 16);
    }
    static std::uint32_t swap16(std::uint32_t x) { return ((x & 0xFFu) << 8) | (x >> 8); }

    void addIpBuf(IpBufRef buf) {
        std::uint64_t sum = m_sum;
        std::size_t pos = 0;  // logical position of the chunk inside the sequence
        ipBufProcessBytes(buf, buf.tot_len, [&](char *p, std::size_t n) {
            std::uint32_t b = IpChksumInverted(p, n);
            sum += (pos & 1) ? swap16(b) : b;
            pos += n;
            return n;
        });
        // end-around-carry fold to 32 bits: nonzero stays nonzero, value mod 0xFFFF kept
        sum = (sum & 0xFFFFFFFFu) + (sum >> 32);
        sum = (sum & 0xFFFFFFFFu) + (sum >> 32);
        m_sum = std::uint32_t(sum);
    }

    std::uint32_t m_sum;
};

// Chksum.h:332-336
inline std::uint16_t IpChksum(IpBufRef buf) {
    IpChksumAccumulator acc;
    return acc.getChksum(buf);
}

// Flatten an IpBufRef chain into the chunk table of aipstack_chksum_batch_chain: appends
// the non-empty chunks ipBufProcessBytes visits (BufUtils.h:129-178) as (device address,
// length) and closes the chain's index entry. `to_device(char *host_ptr)` maps a node's
// host pointer to the device address of the same byte (e.g. base_dev + (p - base_host)).
template <typename ToDevice, typename AddrVec, typename LenVec, typename IndexVec>
void appendChain(IpBufRef buf, ToDevice &&to_device, AddrVec &addr, LenVec &len,
                 IndexVec &index) {
    if (index.empty()) index.push_back(0);
    if (buf.tot_len > 0) {
        ipBufProcessBytes(buf, buf.tot_len, [&](char *p, std::size_t n) {
            addr.push_back(std::uint64_t(to_device(p)));
            len.push_back(std::uint32_t(n));
            return n;
        });
    }
    index.push_back(std::uint64_t(addr.size()));
}

// GPU batch entry points (device pointers, stream-ordered; see chksum.h).
struct BatchChksum {
    static int strided(void const *d_base, std::uint64_t stride, std::uint32_t len,
                       std::uint64_t n, std::uint16_t *d_out, bool final_chksum = false,
                       void *stream = nullptr) {
        return aipstack_chksum_batch_strided(d_base, stride, len, n, d_out,
                                             final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u, stream);
    }
    static int csr(void const *d_base, std::uint64_t const *d_offsets, std::uint64_t n,
                   std::uint16_t *d_out, bool final_chksum = false, void *stream = nullptr) {
        return aipstack_chksum_batch_csr(d_base, d_offsets, n, d_out,
                                         final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u, stream);
    }
    static int seeded(void const *d_base, std::uint64_t const *d_offsets,
                      IpChksumAccumulator::State const *d_states, std::uint64_t n,
                      std::uint16_t *d_out, void *stream = nullptr) {
        return aipstack_chksum_batch_seeded_csr(
            d_base, d_offsets, reinterpret_cast<std::uint32_t const *>(d_states), n, d_out,
            stream);
    }
    static int chain(std::uint64_t const *d_chunk_addr, std::uint32_t const *d_chunk_len,
                     std::uint64_t const *d_chunk_index,
                     IpChksumAccumulator::State const *d_states, std::uint64_t n,
                     std::uint16_t *d_out, bool final_chksum = true, void *stream = nullptr) {
        return aipstack_chksum_batch_chain(
            d_chunk_addr, d_chunk_len, d_chunk_index,
            reinterpret_cast<std::uint32_t const *>(d_states), n, d_out,
            final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u, stream);
    }
    // The Tx form: chain i's final checksum stored big-endian at d_field_addr[i] (the field
    // reading 0, as the reference sets it before summing); zeroAsFfff for UDP.
    static int chainFill(std::uint64_t const *d_chunk_addr, std::uint32_t const *d_chunk_len,
                         std::uint64_t const *d_chunk_index,
                         IpChksumAccumulator::State const *d_states,
                         std::uint64_t const *d_field_addr, std::uint64_t n,
                         std::uint16_t *d_out, bool zeroAsFfff = false,
                         void *stream = nullptr) {
        return aipstack_chksum_batch_chain_fill(
            d_chunk_addr, d_chunk_len, d_chunk_index,
            reinterpret_cast<std::uint32_t const *>(d_states), d_field_addr, n, d_out,
            zeroAsFfff ? AIPSTACK_CHKSUM_ZERO_AS_FFFF : 0u, stream);
    }
    // Raw Ethernet frames at CSR offsets: receive verdicts / send-side fill (AIPSTACK_RX_*).
    static int rxVerify(void const *d_frames, std::uint64_t const *d_offsets, std::uint64_t n,
                        std::uint8_t *d_verdict, void *stream = nullptr) {
        return aipstack_chksum_rx_verify(d_frames, d_offsets, n, d_verdict, stream);
    }
    static int txFill(void *d_frames, std::uint64_t const *d_offsets, std::uint64_t n,
                      std::uint8_t *d_status, void *stream = nullptr) {
        return aipstack_chksum_tx_fill(d_frames, d_offsets, n, d_status, stream);
    }
    static std::uint64_t txFillWorkspaceBytes(std::uint64_t n) {
        return aipstack_chksum_tx_fill_workspace_bytes(n);
    }
    static int txFillSplit(void *d_frames, std::uint64_t const *d_offsets, std::uint64_t n,
                           std::uint8_t *d_status, void *d_workspace,
                           std::uint64_t workspace_bytes, void *stream = nullptr) {
        return aipstack_chksum_tx_fill_split(d_frames, d_offsets, n, d_status, d_workspace,
                                             workspace_bytes, stream);
    }
    // The read pass alone: one 8-byte record per frame (layout in chksum.h), frames untouched.
    static int txFillRecords(void const *d_frames, std::uint64_t const *d_offsets,
                             std::uint64_t n, std::uint64_t *d_records, void *stream = nullptr) {
        return aipstack_chksum_tx_fill_records(d_frames, d_offsets, n, d_records, stream);
    }
    // A receive / send ring: frame or packet i = the d_len[i] bytes at d_base + i * slotStride.
    static int slotted(void const *d_base, std::uint64_t slot_stride, std::uint32_t const *d_len,
                       std::uint64_t n, std::uint16_t *d_out, bool final_chksum = false,
                       void *stream = nullptr) {
        return aipstack_chksum_batch_slotted(d_base, slot_stride, d_len, n, d_out,
                                             final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u, stream);
    }
    static int rxVerifySlotted(void const *d_base, std::uint64_t slot_stride,
                               std::uint32_t const *d_len, std::uint64_t n,
                               std::uint8_t *d_verdict, void *stream = nullptr) {
        return aipstack_chksum_rx_verify_slotted(d_base, slot_stride, d_len, n, d_verdict, stream);
    }
    static int txFillSlotted(void *d_base, std::uint64_t slot_stride, std::uint32_t const *d_len,
                             std::uint64_t n, std::uint8_t *d_status, void *stream = nullptr) {
        return aipstack_chksum_tx_fill_slotted(d_base, slot_stride, d_len, n, d_status, stream);
    }
    static int txFillRecordsSlotted(void const *d_base, std::uint64_t slot_stride,
                                    std::uint32_t const *d_len, std::uint64_t n,
                                    std::uint64_t *d_records, void *stream = nullptr) {
        return aipstack_chksum_tx_fill_records_slotted(d_base, slot_stride, d_len, n, d_records,
                                                       stream);
    }
};

// Host-memory batches (the TAP read()/write() path, tap/linux/TapDeviceLinux.cpp:122-127,
// 156-178) through aipstack_chksum_engine: owns the engine, move-only. Every call returns the
// C-ABI status (0 = AIPSTACK_CHKSUM_OK); a failed create leaves valid() false.
class HostChksumEngine {
public:
    explicit HostChksumEngine(int device = 0, std::uint64_t chunk_bytes = 0,
                              int nstreams = 4) {
        m_status = aipstack_chksum_engine_create(device, chunk_bytes, nstreams, &m_engine);
    }
    ~HostChksumEngine() { aipstack_chksum_engine_destroy(m_engine); }
    HostChksumEngine(HostChksumEngine &&o) noexcept : m_engine(o.m_engine), m_status(o.m_status) {
        o.m_engine = nullptr;
    }
    HostChksumEngine &operator=(HostChksumEngine &&o) noexcept {
        if (this != &o) {
            aipstack_chksum_engine_destroy(m_engine);
            m_engine = o.m_engine;
            m_status = o.m_status;
            o.m_engine = nullptr;
        }
        return *this;
    }
    HostChksumEngine(HostChksumEngine const &) = delete;
    HostChksumEngine &operator=(HostChksumEngine const &) = delete;

    bool valid() const { return m_engine != nullptr; }
    int createStatus() const { return m_status; }
    aipstack_chksum_engine *handle() const { return m_engine; }

    int registerMemory(void *ptr, std::uint64_t bytes) {
        return aipstack_chksum_engine_register(m_engine, ptr, bytes);
    }
    int unregisterMemory(void *ptr) { return aipstack_chksum_engine_unregister(m_engine, ptr); }

    int strided(void const *h_base, std::uint64_t stride, std::uint32_t len, std::uint64_t n,
                std::uint16_t *h_out, bool final_chksum = false) {
        return aipstack_chksum_engine_host_strided(m_engine, h_base, stride, len, n, h_out,
                                                   final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u);
    }
    int csr(void const *h_base, std::uint64_t const *h_offsets, std::uint64_t n,
            std::uint16_t *h_out, bool final_chksum = false) {
        return aipstack_chksum_engine_host_csr(m_engine, h_base, h_offsets, n, h_out,
                                               final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u);
    }
    int rxVerify(void const *h_frames, std::uint64_t const *h_offsets, std::uint64_t n,
                 std::uint8_t *h_verdict) {
        return aipstack_chksum_engine_host_rx_verify(m_engine, h_frames, h_offsets, n, h_verdict);
    }
    // Fills the frames IN PLACE (IPv4 header and L4 checksum fields).
    int txFill(void *h_frames, std::uint64_t const *h_offsets, std::uint64_t n,
               std::uint8_t *h_status) {
        return aipstack_chksum_engine_host_tx_fill(m_engine, h_frames, h_offsets, n, h_status);
    }

    // Asynchronous forms: the buffers must stay valid (and the input unchanged) until the
    // ticket completes (poll() == 0 or wait()).
    int submitStrided(void const *h_base, std::uint64_t stride, std::uint32_t len,
                      std::uint64_t n, std::uint16_t *h_out, bool final_chksum,
                      std::uint64_t *ticket) {
        return aipstack_chksum_engine_submit_strided(
            m_engine, h_base, stride, len, n, h_out, final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u,
            ticket);
    }
    int submitCsr(void const *h_base, std::uint64_t const *h_offsets, std::uint64_t n,
                  std::uint16_t *h_out, bool final_chksum, std::uint64_t *ticket) {
        return aipstack_chksum_engine_submit_csr(m_engine, h_base, h_offsets, n, h_out,
                                                 final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u,
                                                 ticket);
    }
    int submitRxVerify(void const *h_frames, std::uint64_t const *h_offsets, std::uint64_t n,
                       std::uint8_t *h_verdict, std::uint64_t *ticket) {
        return aipstack_chksum_engine_submit_rx_verify(m_engine, h_frames, h_offsets, n,
                                                       h_verdict, ticket);
    }
    int submitTxFill(void *h_frames, std::uint64_t const *h_offsets, std::uint64_t n,
                     std::uint8_t *h_status, std::uint64_t *ticket) {
        return aipstack_chksum_engine_submit_tx_fill(m_engine, h_frames, h_offsets, n,
                                                     h_status, ticket);
    }
    // Ring slots (the TAP ring: one frame per slot, its length beside it).
    int slotted(void const *h_base, std::uint64_t slot_stride, std::uint32_t const *h_len,
                std::uint64_t n, std::uint16_t *h_out, bool final_chksum = false) {
        return aipstack_chksum_engine_host_slotted(m_engine, h_base, slot_stride, h_len, n, h_out,
                                                   final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u);
    }
    int rxVerifySlotted(void const *h_base, std::uint64_t slot_stride, std::uint32_t const *h_len,
                        std::uint64_t n, std::uint8_t *h_verdict) {
        return aipstack_chksum_engine_host_rx_verify_slotted(m_engine, h_base, slot_stride, h_len,
                                                             n, h_verdict);
    }
    int txFillSlotted(void *h_base, std::uint64_t slot_stride, std::uint32_t const *h_len,
                      std::uint64_t n, std::uint8_t *h_status) {
        return aipstack_chksum_engine_host_tx_fill_slotted(m_engine, h_base, slot_stride, h_len, n,
                                                           h_status);
    }
    int submitSlotted(void const *h_base, std::uint64_t slot_stride, std::uint32_t const *h_len,
                      std::uint64_t n, std::uint16_t *h_out, bool final_chksum,
                      std::uint64_t *ticket) {
        return aipstack_chksum_engine_submit_slotted(m_engine, h_base, slot_stride, h_len, n, h_out,
                                                     final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u,
                                                     ticket);
    }
    int submitRxVerifySlotted(void const *h_base, std::uint64_t slot_stride,
                              std::uint32_t const *h_len, std::uint64_t n,
                              std::uint8_t *h_verdict, std::uint64_t *ticket) {
        return aipstack_chksum_engine_submit_rx_verify_slotted(m_engine, h_base, slot_stride,
                                                               h_len, n, h_verdict, ticket);
    }
    int submitTxFillSlotted(void *h_base, std::uint64_t slot_stride, std::uint32_t const *h_len,
                            std::uint64_t n, std::uint8_t *h_status, std::uint64_t *ticket) {
        return aipstack_chksum_engine_submit_tx_fill_slotted(m_engine, h_base, slot_stride, h_len,
                                                             n, h_status, ticket);
    }
    // 0 = complete, 1 = still running, < 0 = error of that batch
    int poll(std::uint64_t ticket) { return aipstack_chksum_engine_poll(m_engine, ticket); }
    int wait(std::uint64_t ticket) { return aipstack_chksum_engine_wait(m_engine, ticket); }

    // NUMA node of the device (-1 unknown) and the CPUs the engine's host threads are pinned to.
    int locality(int *numa_node, int *pinned_cpus) const {
        return aipstack_chksum_engine_locality(m_engine, numa_node, pinned_cpus);
    }

private:
    aipstack_chksum_engine *m_engine = nullptr;
    int m_status = AIPSTACK_CHKSUM_EINVAL;
};

// Several devices behind one host-memory batch, in one process (aipstack_chksum_engine_group):
// owns the group, move-only. submit* return one group ticket over the devices' ranges;
// poll / wait complete it (0 done, 1 running, < 0 the first failure) and fill devStatus (NULL
// or size() ints) with each device's status.
class HostChksumEngineGroup {
public:
    HostChksumEngineGroup(int const *devices, int n_devices, std::uint64_t chunk_bytes = 0,
                          int nstreams = 4) {
        m_status = aipstack_chksum_engine_group_create(devices, n_devices, chunk_bytes, nstreams,
                                                       &m_group);
    }
    ~HostChksumEngineGroup() { aipstack_chksum_engine_group_destroy(m_group); }
    HostChksumEngineGroup(HostChksumEngineGroup &&o) noexcept
        : m_group(o.m_group), m_status(o.m_status) {
        o.m_group = nullptr;
    }
    HostChksumEngineGroup &operator=(HostChksumEngineGroup &&o) noexcept {
        if (this != &o) {
            aipstack_chksum_engine_group_destroy(m_group);
            m_group = o.m_group;
            m_status = o.m_status;
            o.m_group = nullptr;
        }
        return *this;
    }
    HostChksumEngineGroup(HostChksumEngineGroup const &) = delete;
    HostChksumEngineGroup &operator=(HostChksumEngineGroup const &) = delete;

    bool valid() const { return m_group != nullptr; }
    int createStatus() const { return m_status; }
    int size() const { return aipstack_chksum_engine_group_size(m_group); }
    aipstack_chksum_engine_group *handle() const { return m_group; }
    aipstack_chksum_engine *engine(int k) const {
        return aipstack_chksum_engine_group_engine(m_group, k);
    }

    int registerMemory(void *ptr, std::uint64_t bytes) {
        return aipstack_chksum_engine_group_register(m_group, ptr, bytes);
    }
    int unregisterMemory(void *ptr) { return aipstack_chksum_engine_group_unregister(m_group, ptr); }

    int submitStrided(void const *h_base, std::uint64_t stride, std::uint32_t len,
                      std::uint64_t n, std::uint16_t *h_out, bool final_chksum,
                      std::uint64_t *ticket) {
        return aipstack_chksum_engine_group_submit_strided(
            m_group, h_base, stride, len, n, h_out, final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u,
            ticket);
    }
    int submitCsr(void const *h_base, std::uint64_t const *h_offsets, std::uint64_t n,
                  std::uint16_t *h_out, bool final_chksum, std::uint64_t *ticket) {
        return aipstack_chksum_engine_group_submit_csr(
            m_group, h_base, h_offsets, n, h_out, final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u,
            ticket);
    }
    int submitRxVerify(void const *h_frames, std::uint64_t const *h_offsets, std::uint64_t n,
                       std::uint8_t *h_verdict, std::uint64_t *ticket) {
        return aipstack_chksum_engine_group_submit_rx_verify(m_group, h_frames, h_offsets, n,
                                                             h_verdict, ticket);
    }
    int submitTxFill(void *h_frames, std::uint64_t const *h_offsets, std::uint64_t n,
                     std::uint8_t *h_status, std::uint64_t *ticket) {
        return aipstack_chksum_engine_group_submit_tx_fill(m_group, h_frames, h_offsets, n,
                                                           h_status, ticket);
    }
    int submitSlotted(void const *h_base, std::uint64_t slot_stride, std::uint32_t const *h_len,
                      std::uint64_t n, std::uint16_t *h_out, bool final_chksum,
                      std::uint64_t *ticket) {
        return aipstack_chksum_engine_group_submit_slotted(
            m_group, h_base, slot_stride, h_len, n, h_out,
            final_chksum ? AIPSTACK_CHKSUM_FINAL : 0u, ticket);
    }
    int submitRxVerifySlotted(void const *h_base, std::uint64_t slot_stride,
                              std::uint32_t const *h_len, std::uint64_t n,
                              std::uint8_t *h_verdict, std::uint64_t *ticket) {
        return aipstack_chksum_engine_group_submit_rx_verify_slotted(m_group, h_base, slot_stride,
                                                                     h_len, n, h_verdict, ticket);
    }
    int submitTxFillSlotted(void *h_base, std::uint64_t slot_stride, std::uint32_t const *h_len,
                            std::uint64_t n, std::uint8_t *h_status, std::uint64_t *ticket) {
        return aipstack_chksum_engine_group_submit_tx_fill_slotted(m_group, h_base, slot_stride,
                                                                   h_len, n, h_status, ticket);
    }
    int poll(std::uint64_t ticket, int *devStatus = nullptr) {
        return aipstack_chksum_engine_group_poll(m_group, ticket, devStatus);
    }
    int wait(std::uint64_t ticket, int *devStatus = nullptr) {
        return aipstack_chksum_engine_group_wait(m_group, ticket, devStatus);
    }

private:
    aipstack_chksum_engine_group *m_group = nullptr;
    int m_status = AIPSTACK_CHKSUM_EINVAL;
};

}  // namespace AIpStackAmd

#endif
