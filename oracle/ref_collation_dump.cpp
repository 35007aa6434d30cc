// ref_collation_dump.cpp — test infrastructure (the collation pin, tests/golden/make_collation_pin.py).
// Linked with the reference's own dbms/src/TiDB/Collation/CollationLUT.cpp, compiled as it lies
// under /root/reference (it needs only <array> and <cstdint>), it writes the reference's weight
// tables as the compiler evaluated them: GeneralCI::weight_lut (65536 x u16, the PLANE_* / PLANE_ID
// macros expanded), UnicodeCI::weight_lut_0400 (65537 x u64) and weight_lut_0900 (0x2CEA1 x u64).
// Nothing here is shipped or linked into the product; the output lands in oracle/_ref/.
#include <array>
#include <cstdint>
#include <cstdio>

namespace TiDB::GeneralCI {
using WeightType = uint16_t;
extern const std::array<WeightType, 256 * 256> weight_lut;
}
namespace TiDB::UnicodeCI {
extern const std::array<uint64_t, 256 * 256 + 1> weight_lut_0400;
extern const std::array<uint64_t, 0x2CEA1> weight_lut_0900;
}

int main(int argc, char **argv) {
    if (argc != 2) {
        fprintf(stderr, "usage: %s <out.bin>\n", argv[0]);
        return 2;
    }
    FILE *f = fopen(argv[1], "wb");
    if (!f) return 1;
    const auto &g = TiDB::GeneralCI::weight_lut;
    const auto &a = TiDB::UnicodeCI::weight_lut_0400;
    const auto &b = TiDB::UnicodeCI::weight_lut_0900;
    bool ok = fwrite(g.data(), sizeof(g[0]), g.size(), f) == g.size();
    ok = ok && fwrite(a.data(), sizeof(a[0]), a.size(), f) == a.size();
    ok = ok && fwrite(b.data(), sizeof(b[0]), b.size(), f) == b.size();
    return fclose(f) == 0 && ok ? 0 : 1;
}
