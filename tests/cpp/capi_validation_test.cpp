// Host test program: the C-ABI's argument validation (include/aipstack_amd/chksum.h) --
// every entry point rejects null pointers, oversize arguments and bad handles with
// AIPSTACK_CHKSUM_EINVAL before touching a device, accepts n == 0 as a no-op, and the
// host-memory engine fails cleanly (ENODEV / EHIP) where no gfx950 device is visible.
// Built twice: plain (make -C tests/cpp) and under AddressSanitizer + UBSan together with
// the whole library's host code (make -C tests/cpp asan). Runs on a host without a GPU;
// with one, the device-dependent expectations switch to success.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "aipstack_amd/chksum.h"

#define CHECK(cond)                                                                  \
    do {                                                                             \
        if (!(cond)) {                                                               \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            std::abort();                                                            \
        }                                                                            \
    } while (0)

int main() {
    const int EINVAL_ = AIPSTACK_CHKSUM_EINVAL;
    alignas(8) char dummy[64] = {0};
    std::uint64_t off[2] = {0, 8};
    std::uint16_t out[4];
    std::uint8_t st[4];
    std::uint32_t states[4] = {0};
    std::uint32_t lens[4] = {1, 1, 1, 1};
    std::uint64_t addrs[4] = {0};

    // n == 0 is a no-op whatever the pointers
    CHECK(aipstack_chksum_batch_strided(nullptr, 0, 0, 0, nullptr, 0, nullptr) == 0);
    CHECK(aipstack_chksum_batch_csr(nullptr, nullptr, 0, nullptr, 0, nullptr) == 0);
    CHECK(aipstack_chksum_batch_seeded_csr(nullptr, nullptr, nullptr, 0, nullptr, nullptr) == 0);
    CHECK(aipstack_chksum_batch_chain(nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr) == 0);
    CHECK(aipstack_chksum_rx_verify(nullptr, nullptr, 0, nullptr, nullptr) == 0);
    CHECK(aipstack_chksum_tx_fill(nullptr, nullptr, 0, nullptr, nullptr) == 0);
    CHECK(aipstack_chksum_tx_fill_split(nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr) == 0);

    // null pointers / bad sizes
    CHECK(aipstack_chksum_batch_strided(nullptr, 1, 1, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_strided(dummy, 1, 1, 1, nullptr, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_strided(dummy, 1, 65536, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_strided(dummy, 1, 1, (1ull << 40) + 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_csr(nullptr, off, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_csr(dummy, nullptr, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_csr(dummy, off, 1, nullptr, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_seeded_csr(dummy, off, nullptr, 1, out, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_chain(nullptr, lens, off, states, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_chain(addrs, nullptr, off, states, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_chain(addrs, lens, nullptr, states, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_batch_chain(addrs, lens, off, states, 1, nullptr, 0, nullptr) == EINVAL_);
    // chain fill: the field table and d_out are required; n == 0 is a no-op
    CHECK(aipstack_chksum_batch_chain_fill(nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, 0,
                                           nullptr) == 0);
    CHECK(aipstack_chksum_batch_chain_fill(addrs, lens, off, states, nullptr, 1, out, 0, nullptr) ==
          EINVAL_);
    CHECK(aipstack_chksum_batch_chain_fill(nullptr, lens, off, states, off, 1, out, 0, nullptr) ==
          EINVAL_);
    CHECK(aipstack_chksum_batch_chain_fill(addrs, lens, off, states, off, 1, nullptr, 0, nullptr) ==
          EINVAL_);
    CHECK(aipstack_chksum_rx_verify(dummy, off, 1, nullptr, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_tx_fill(dummy, nullptr, 1, st, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_tx_fill_records(nullptr, nullptr, 0, nullptr, nullptr) == 0);
    CHECK(aipstack_chksum_tx_fill_records(dummy, off, 1, nullptr, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_tx_fill_records(dummy, off, 1, reinterpret_cast<std::uint64_t *>(dummy + 1),
                                          nullptr) == EINVAL_);
    // split fill: workspace missing, too small, misaligned
    CHECK(aipstack_chksum_tx_fill_workspace_bytes(3) >= 24);
    CHECK(aipstack_chksum_tx_fill_split(dummy, off, 1, st, nullptr, 64, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_tx_fill_split(dummy, off, 4, st, dummy, 8, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_tx_fill_split(dummy, off, 1, st, dummy + 1, 63, nullptr) == EINVAL_);

    // tunables
    CHECK(aipstack_chksum_tune(nullptr, 1) == EINVAL_);
    CHECK(aipstack_chksum_tune("no_such_key", 1) == EINVAL_);
    CHECK(aipstack_chksum_tune("stream", 0) == 0);

    // engine: argument checks come before any device work
    aipstack_chksum_engine *e = nullptr;
    CHECK(aipstack_chksum_engine_create(0, 0, 0, &e) == EINVAL_ && e == nullptr);
    CHECK(aipstack_chksum_engine_create(0, 0, 17, &e) == EINVAL_);
    CHECK(aipstack_chksum_engine_create(0, 0, 2, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_create(-1, 0, 2, &e) == AIPSTACK_CHKSUM_ENODEV && e == nullptr);
    CHECK(aipstack_chksum_engine_register(nullptr, dummy, 64) == EINVAL_);
    CHECK(aipstack_chksum_engine_unregister(nullptr, dummy) == EINVAL_);
    CHECK(aipstack_chksum_engine_host_strided(nullptr, dummy, 1, 1, 1, out, 0) == EINVAL_);
    CHECK(aipstack_chksum_engine_host_csr(nullptr, dummy, off, 1, out, 0) == EINVAL_);
    std::uint64_t ticket = 0;
    CHECK(aipstack_chksum_engine_submit_strided(nullptr, dummy, 1, 1, 1, out, 0, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_submit_csr(nullptr, dummy, off, 1, out, 0, &ticket) == EINVAL_);
    std::uint8_t verdicts[4] = {0, 0, 0, 0};
    CHECK(aipstack_chksum_engine_host_rx_verify(nullptr, dummy, off, 1, verdicts) == EINVAL_);
    CHECK(aipstack_chksum_engine_submit_rx_verify(nullptr, dummy, off, 1, verdicts, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_host_tx_fill(nullptr, dummy, off, 1, verdicts) == EINVAL_);
    CHECK(aipstack_chksum_engine_submit_tx_fill(nullptr, dummy, off, 1, verdicts, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_poll(nullptr, 1) == EINVAL_);
    CHECK(aipstack_chksum_engine_wait(nullptr, 1) == EINVAL_);
    aipstack_chksum_engine_destroy(nullptr);  // no-op

    const int dev = aipstack_chksum_device_check(0);
    CHECK(dev == 0 || dev == AIPSTACK_CHKSUM_ENODEV || dev == AIPSTACK_CHKSUM_EHIP);
    aipstack_chksum_engine_group *grp = nullptr;
    const int devs[3] = {0, 0, 0}, bad_devs[2] = {0, -1};
    CHECK(aipstack_chksum_engine_group_create(nullptr, 1, 0, 2, &grp) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_create(devs, 0, 0, 2, &grp) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_create(devs, 3, 0, 2, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_create(bad_devs, 2, 0, 2, &grp) != 0 && grp == nullptr);
    CHECK(aipstack_chksum_engine_group_size(nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_register(nullptr, dummy, 64) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_unregister(nullptr, dummy) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_host_csr(nullptr, dummy, off, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_host_strided(nullptr, dummy, 1, 1, 1, out, 0, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_host_rx_verify(nullptr, dummy, off, 1, verdicts, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_host_tx_fill(nullptr, dummy, off, 1, verdicts, nullptr) == EINVAL_);
    std::uint32_t lens1[1] = {60};
    CHECK(aipstack_chksum_engine_group_submit_csr(nullptr, dummy, off, 1, out, 0, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_submit_strided(nullptr, dummy, 1, 1, 1, out, 0, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_submit_rx_verify(nullptr, dummy, off, 1, verdicts, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_submit_tx_fill(nullptr, dummy, off, 1, verdicts, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_submit_slotted(nullptr, dummy, 64, lens1, 1, out, 0, &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_submit_rx_verify_slotted(nullptr, dummy, 64, lens1, 1, verdicts,
                                                                &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_submit_tx_fill_slotted(nullptr, dummy, 64, lens1, 1, verdicts,
                                                              &ticket) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_poll(nullptr, 1, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_wait(nullptr, 1, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_group_engine(nullptr, 0) == nullptr);
    CHECK(aipstack_chksum_engine_group_region_mapped(nullptr, dummy) == EINVAL_);
    CHECK(aipstack_chksum_engine_locality(nullptr, nullptr, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_engine_region_mapped(nullptr, dummy) == EINVAL_);
    // the frame forms on slots reject strides over AIPSTACK_CHKSUM_MAX_SLOT_STRIDE before any
    // device work (here: no device needed)
    CHECK(aipstack_chksum_rx_verify_slotted(dummy, AIPSTACK_CHKSUM_MAX_SLOT_STRIDE + 1, lens1, 1,
                                            verdicts, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_tx_fill_slotted(dummy, AIPSTACK_CHKSUM_MAX_SLOT_STRIDE + 1, lens1, 1,
                                          verdicts, nullptr) == EINVAL_);
    CHECK(aipstack_chksum_tx_fill_slotted_split(dummy, 2048, lens1, 1, verdicts, nullptr, 8,
                                                nullptr) == EINVAL_);  // no workspace
    CHECK(aipstack_chksum_tx_fill_slotted_split(dummy, 2048, lens1, 1, verdicts, dummy, 4,
                                                nullptr) == EINVAL_);  // workspace too small
    CHECK(std::strlen(aipstack_chksum_source_digest()) == 64);
    aipstack_chksum_engine_group_destroy(nullptr);  // no-op
    std::uint32_t vmask = 0;
    CHECK(aipstack_chksum_contract_violations(0, nullptr, 1) == EINVAL_);
    CHECK(aipstack_chksum_contract_violations(-1, &vmask, 1) == AIPSTACK_CHKSUM_ENODEV);
    CHECK(aipstack_chksum_contract_violations(0, &vmask, 1) == dev);
    const int ec = aipstack_chksum_engine_create(0, 0, 2, &e);
    if (dev == 0) {
        CHECK(ec == 0 && e != nullptr);
        // engine-level contract checks (host side, before any copy)
        std::uint64_t bad_off[3] = {0, 8, 4};  // decreasing
        CHECK(aipstack_chksum_engine_host_csr(e, dummy, bad_off, 2, out, 0) == EINVAL_);
        std::uint64_t big_off[2] = {0, 65536};  // > 65535 bytes
        std::vector<char> big(65536, 0);
        CHECK(aipstack_chksum_engine_host_csr(e, big.data(), big_off, 1, out, 0) == EINVAL_);
        CHECK(aipstack_chksum_engine_host_strided(e, dummy, 1, 65536, 1, out, 0) == EINVAL_);
        CHECK(aipstack_chksum_engine_register(e, nullptr, 64) == EINVAL_);
        CHECK(aipstack_chksum_engine_register(e, dummy, 0) == EINVAL_);
        CHECK(aipstack_chksum_engine_unregister(e, dummy) == EINVAL_);  // never registered
        CHECK(aipstack_chksum_engine_submit_csr(e, dummy, bad_off, 2, out, 0, &ticket) == EINVAL_);
        CHECK(aipstack_chksum_engine_submit_csr(e, dummy, off, 1, out, 0, nullptr) == EINVAL_);
        CHECK(aipstack_chksum_engine_host_rx_verify(e, dummy, bad_off, 2, verdicts) == EINVAL_);
        CHECK(aipstack_chksum_engine_host_rx_verify(e, big.data(), big_off, 1, verdicts) == EINVAL_);
        CHECK(aipstack_chksum_engine_submit_rx_verify(e, dummy, off, 1, nullptr, &ticket) == EINVAL_);
        CHECK(aipstack_chksum_engine_host_rx_verify(e, dummy, off, 0, verdicts) == 0);  // no-op
        CHECK(aipstack_chksum_engine_host_tx_fill(e, dummy, bad_off, 2, verdicts) == EINVAL_);
        CHECK(aipstack_chksum_engine_host_tx_fill(e, big.data(), big_off, 1, verdicts) == EINVAL_);
        CHECK(aipstack_chksum_engine_submit_tx_fill(e, dummy, off, 1, nullptr, &ticket) == EINVAL_);
        CHECK(aipstack_chksum_engine_submit_tx_fill(e, dummy, off, 1, verdicts, nullptr) == EINVAL_);
        CHECK(aipstack_chksum_engine_host_tx_fill(e, dummy, off, 0, verdicts) == 0);  // no-op
        CHECK(aipstack_chksum_engine_poll(e, 0) == EINVAL_);          // never a ticket
        CHECK(aipstack_chksum_engine_wait(e, 1u << 30) == EINVAL_);   // not issued yet
        // a real batch through submit + poll/wait
        std::vector<char> pk(4 * 1500, 0x5A);
        std::uint16_t res[4] = {0, 0, 0, 0};
        CHECK(aipstack_chksum_engine_submit_strided(e, pk.data(), 1500, 1500, 4, res, 0, &ticket) == 0);
        CHECK(ticket != 0);
        while (aipstack_chksum_engine_poll(e, ticket) == 1) {
        }
        CHECK(aipstack_chksum_engine_wait(e, ticket) == 0);
        for (std::uint16_t r : res) CHECK(r == IpChksumInverted(pk.data(), 1500));
        aipstack_chksum_engine_destroy(e);
    } else {
        CHECK(ec == dev && e == nullptr);
    }

    // diagnostics
    for (int s : {0, -1, -2, -3, -99}) CHECK(aipstack_chksum_strerror(s) != nullptr);
    CHECK(aipstack_chksum_abi_version() == AIPSTACK_CHKSUM_ABI_VERSION);
    std::printf("capi_validation_test: OK (device %s)\n", dev == 0 ? "present" : "absent");
    return 0;
}
