// Chksum.hpp's assertions follow the reference's configuration (misc/Assert.h): built with
// -DAIPSTACK_CONFIG_ENABLE_ASSERTIONS, IpChksumAccumulator::addEvenBytes with an odd count
// aborts as the reference's does (Chksum.h:227); an even count passes. Run by
// tests/test_host_cpp.py: `assert_test even` exits 0, `assert_test odd` aborts.
#include <cstdio>
#include <cstring>

#include "aipstack_amd/Chksum.hpp"

int main(int argc, char **argv) {
    const char bytes[5] = {0x12, 0x34, 0x56, 0x78, 0x40};
    AIpStackAmd::IpChksumAccumulator acc;
    const bool odd = argc > 1 && !std::strcmp(argv[1], "odd");
    acc.addEvenBytes(bytes, odd ? 5 : 4);
    std::printf("sum %04x\n", (unsigned)acc.getChksum());
    return 0;
}
