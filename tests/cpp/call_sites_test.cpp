// Host test program: replays the reference call-site fixtures (tests/golden/
// call_site_cases.json, recorded from the reference's own Chksum.h) through this repo's
// C++ surface (Chksum.hpp + the IpChksumInverted hook), as a standalone executable so that
// it can run under AddressSanitizer / UBSan (make -C tests/cpp asan).
//
//   call_sites_test <blob.bin> <cases.txt>
//
// The pytest driver (tests/test_host_cpp.py) writes both files from the JSON fixture:
// blob.bin = the golden blob's bytes; cases.txt = one case per line:
//   site nargs a... hdr_hex|- nchunks (off len)... offset tot_len nwant w...
// Exit status 0 = every case matched.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "aipstack_amd/Chksum.hpp"

using namespace AIpStackAmd;

#define CS_NAME(x) cs_##x
#define CS_PROCESS_BYTES(buf, len, fn) ipBufProcessBytes(buf, len, fn)
#include "call_sites.inc"

namespace {

std::vector<char> read_file(const char *path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

std::vector<char> unhex(const std::string &h) {
    std::vector<char> out;
    if (h == "-") return out;
    for (std::size_t i = 0; i + 1 < h.size(); i += 2)
        out.push_back(char(std::strtoul(h.substr(i, 2).c_str(), nullptr, 16)));
    return out;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s blob.bin cases.txt\n", argv[0]);
        return 2;
    }
    std::vector<char> blob = read_file(argv[1]);
    std::ifstream cf(argv[2]);
    std::string line;
    long n = 0, bad = 0;
    while (std::getline(cf, line)) {
        if (line.empty()) continue;
        std::istringstream in(line);
        std::string site, hex;
        int nargs = 0;
        in >> site >> nargs;
        std::vector<unsigned long long> a(nargs);
        for (auto &x : a) in >> x;
        in >> hex;
        // the explicit first node lives in its own heap buffer (exact size, so ASan sees
        // any read past it), then the blob chunks
        std::vector<char> hdr = unhex(hex);
        std::vector<char *> ptrs;
        std::vector<std::size_t> lens;
        char *hbuf = nullptr;
        if (!hdr.empty()) {
            hbuf = static_cast<char *>(std::malloc(hdr.size()));
            std::memcpy(hbuf, hdr.data(), hdr.size());
            ptrs.push_back(hbuf);
            lens.push_back(hdr.size());
        }
        std::size_t nch = 0;
        in >> nch;
        for (std::size_t i = 0; i < nch; i++) {
            std::size_t o = 0, l = 0;
            in >> o >> l;
            if (o + l > blob.size()) return 3;
            ptrs.push_back(blob.data() + o);
            lens.push_back(l);
        }
        std::size_t offset = 0, tot_len = 0;
        int nwant = 0;
        in >> offset >> tot_len >> nwant;
        std::vector<long long> want(nwant);
        for (auto &w : want) in >> w;
        if (!in) return 4;
        char *const *P = ptrs.data();
        const std::size_t *L = lens.data();
        const std::size_t K = ptrs.size();
        std::vector<long long> got;
        std::uint32_t st = 0;
        std::size_t dl = 0;
        if (site == "tcp_rx") got = {cs_tcp_rx(a[0], a[1], P, L, K, offset, tot_len)};
        else if (site == "udp_tx") got = {cs_udp_tx(a[0], a[1], P, L, K, offset, tot_len)};
        else if (site == "udp_rx")
            got = {cs_udp_rx(a[0], a[1], std::uint16_t(a[2]), P, L, K, offset, tot_len)};
        else if (site == "tcp_tx") {
            long long r = cs_tcp_tx(std::uint16_t(a[0]), std::uint16_t(a[1]), a[2],
                                    std::uint16_t(a[3]), a[4], a[5], a[6], std::uint16_t(a[7]),
                                    P, L, K, offset, tot_len, &st);
            got = {r, st};
        } else if (site == "ip4_tx") {
            long long r = cs_ip4_tx(std::uint16_t(a[0]), std::uint8_t(a[1]), std::uint8_t(a[2]),
                                    a[3], a[4], std::uint16_t(a[5]), std::uint16_t(a[6]), &st);
            got = {r, st};
        } else if (site == "ip4_rx") {
            long long r = cs_ip4_rx(P, L, K, offset, tot_len, &dl);
            got = {r, (long long)dl};
        } else if (site == "icmp") got = {cs_icmp(P, L, K, offset, tot_len)};
        else return 5;
        std::free(hbuf);
        ++n;
        if (got != want) {
            if (++bad <= 10) std::fprintf(stderr, "mismatch: %s\n", line.c_str());
        }
    }
    std::printf("call_sites_test: %ld cases, %ld mismatches\n", n, bad);
    return bad == 0 && n > 0 ? 0 : 1;
}
