// CPU check of gx::host_pack24 (gx_host.cpp), the 24-bit column packer of the upload: every
// value round-trips, group tails (counts around 16), the range check on the 24-bit bound and on
// 64-bit values, unaligned output (scalar path).  Built and run by tests/test_host_pack.py.
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

namespace gx {
bool host_pack24(const uint64_t *in, uint64_t count, uint64_t limit, uint32_t *out);
}

static bool unpack_equal(const std::vector<uint64_t> &in, const unsigned char *b) {
    for (size_t k = 0; k < in.size(); k++) {
        const uint32_t c = b[3 * k] | (b[3 * k + 1] << 8) | (b[3 * k + 2] << 16);
        if (c != in[k]) return false;
    }
    return true;
}

int main() {
    std::mt19937_64 r(7);
    int fails = 0;
    for (uint64_t count : {0ull, 1ull, 3ull, 15ull, 16ull, 17ull, 31ull, 32ull, 33ull, 1000003ull, 4194321ull}) {
        for (int misalign = 0; misalign < 2; misalign++) {
            std::vector<uint64_t> in(count);
            for (auto &x : in) x = r() % (1u << 24);
            if (count > 2) {
                in[0] = (1u << 24) - 1;
                in[count / 2] = 0;
            }
            std::vector<uint32_t> buf((3 * count + 3) / 4 + 8, 0xdeadbeefu);
            uint32_t *out = buf.data() + (misalign ? 1 : 0);
            unsigned char *outb = reinterpret_cast<unsigned char *>(out) + (misalign ? 1 : 0);   // not 4-B aligned either
            const bool ok = gx::host_pack24(in.data(), count, 1u << 24, reinterpret_cast<uint32_t *>(outb));
            const bool same = unpack_equal(in, outb);
            bool bad_found = true;
            if (count > 20) {
                in[17] = 1u << 24;
                bad_found &= !gx::host_pack24(in.data(), count, 1u << 24, reinterpret_cast<uint32_t *>(outb));
                in[17] = 5;
                in[count - 1] = 1ull << 40;
                bad_found &= !gx::host_pack24(in.data(), count, 1u << 24, reinterpret_cast<uint32_t *>(outb));
                in[count - 1] = 3;
                bad_found &= !gx::host_pack24(in.data(), count, 100, reinterpret_cast<uint32_t *>(outb));   // limit < values
            }
            if (!ok || !same || !bad_found) {
                std::printf("FAIL count %llu misalign %d: ok %d same %d bad_found %d\n", (unsigned long long)count,
                            misalign, ok, same, bad_found);
                fails++;
            }
        }
    }
    std::printf(fails ? "pack24 FAILED\n" : "pack24 ok\n");
    return fails ? 1 : 0;
}
