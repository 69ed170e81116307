// Host build of frt::splat_fixed (csrc/frt_mlt.hpp) against the fp64 expression
// the PSS-MLT splat used until round 6: llrint((double)x * 2^36) with the
// same validity range [0, 2^63).  Compiled and run by tests/test_mlt_splat_fix.py.
// Round-6 development run: every one of the 2^32 float bit patterns, 0 differ.
#include "frt_mlt.hpp"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

int main(int argc, char **argv)
{
    const uint64_t stride = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 257;
    long bad = 0, n = 0;
    auto check = [&](float x) {
        unsigned long long a = 0;
        const bool ok = frt::splat_fixed<36>(x, a);
        const double v = (double)x * (double)(1ull << 36);
        const bool ok2 = v >= 0.0 && v < 9.2233720368547758e18;
        const unsigned long long b = ok2 ? (unsigned long long)std::llrint(v) : 0ull;
        ++n;
        if (ok != ok2 || (ok && a != b)) {
            if (bad < 10) std::printf("x=%a ok=%d/%d got=%llu want=%llu\n", x, ok, ok2, a, b);
            ++bad;
        }
    };
    for (uint64_t bits = 0; bits <= 0xffffffffull; bits += stride) {
        const uint32_t b32 = (uint32_t)bits;
        float x;
        std::memcpy(&x, &b32, 4);
        check(x);
    }
    // rounding ties and the boundaries: quanta halves, the largest valid value
    for (int e = -160; e < 30; ++e) {
        check(std::ldexp(1.0f, e));
        check(std::ldexp(1.5f, e));
        check(std::ldexp(1.0f, e) + std::ldexp(1.0f, e - 23));
        check(std::ldexp(1.0f, e) * 3.0f);
    }
    std::mt19937 g(1);
    for (int i = 0; i < 1000000; ++i) {
        const uint32_t b32 = (uint32_t)g();
        float x;
        std::memcpy(&x, &b32, 4);
        check(std::fabs(x));
    }
    check(-0.0f); check(0.0f); check(NAN); check(INFINITY); check(134217728.0f); check(std::nextafter(134217728.0f, 0.0f));
    std::printf("%ld of %ld differ\n", bad, n);
    return bad != 0;
}
