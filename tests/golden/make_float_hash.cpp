// make_float_hash.cpp — generates tests/golden/float_weak_hash.json: the reference's weak hash
// of Float32 / Float64 key columns.  ColumnVector<Float>::updateWeakHash32
// (Columns/ColumnVector.cpp:520-529) passes the value to intHashCRC32(UInt64 x, UInt32 h)
// (Common/HashTable/Hash.h:83-94): an implicit Float -> UInt64 conversion, then _mm_crc32_u64.
// The conversion is implementation-defined outside [0, 2^64); this program pins it for the
// reference's toolchain (clang, x86-64 with SSE4.2, no AVX-512) by running that same call
// shape.  Build + run (x86 host):
//   /opt/rocm/lib/llvm/bin/clang++ -O2 -msse4.2 tests/golden/make_float_hash.cpp -o /tmp/mfh
//   /tmp/mfh > tests/golden/float_weak_hash.json
#include <nmmintrin.h>

#include <cinttypes>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

__attribute__((noinline)) static uint32_t intHashCRC32(uint64_t x, uint32_t updated_value) {
    return (uint32_t)_mm_crc32_u64(updated_value, x);
}
template <typename T> __attribute__((noinline)) static uint64_t to_u64(T x) { return x; }
template <typename T> __attribute__((noinline)) static uint32_t hash_one(T x) { return intHashCRC32(x, 0xFFFFFFFFu); }

template <typename T, typename Bits> static void emit(const char *name, const std::vector<T> &v, bool last) {
    printf("  \"%s\": [\n", name);
    for (size_t i = 0; i < v.size(); ++i) {
        Bits b;
        memcpy(&b, &v[i], sizeof(T));
        printf("    {\"bits\": \"%0*llx\", \"u64\": \"%016" PRIx64 "\", \"hash\": %u}%s\n", (int)(2 * sizeof(T)),
               (unsigned long long)b, to_u64(v[i]), hash_one(v[i]), i + 1 < v.size() ? "," : "");
    }
    printf("  ]%s\n", last ? "" : ",");
}

int main() {
    const double inf = std::numeric_limits<double>::infinity();
    std::vector<double> d = {0.0, -0.0, 1.0, 1.5, -1.5, -2.5, -0.7, 123456789.987, 4.5e15, 9007199254740993.0,
                             9223372036854775807.0, 9223372036854775808.0, 1e19, 18446744073709549568.0,
                             18446744073709551616.0, 3e19, -1e19, -9223372036854775808.0, -9223372036854777856.0,
                             inf, -inf, std::nan(""), -std::nan(""), 5e-324, -5e-324, 1e308, -1e308};
    std::mt19937_64 rng(2024);
    for (int i = 0; i < 24; ++i) { // random magnitudes across the whole range
        const double m = (double)(rng() >> 11) / 9007199254740992.0;
        const int e = (int)(rng() % 140) - 70;
        d.push_back((rng() & 1 ? -1 : 1) * std::ldexp(m, e));
    }
    std::vector<float> f;
    for (double x : d) f.push_back((float)x);
    f.push_back(16777217.0f);
    f.push_back(3.4028235e38f);
    printf("{\n  \"source\": \"intHashCRC32(UInt64(x), ~0u) per ColumnVector<Float>::updateWeakHash32, x86-64 clang -O2 -msse4.2\",\n");
    emit<double, uint64_t>("float64", d, false);
    emit<float, uint32_t>("float32", f, true);
    printf("}\n");
}
