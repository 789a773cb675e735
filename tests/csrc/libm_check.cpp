// Host check of scheme-raytrace_amd/csrc/rt_libm.h against this machine's C
// library (tests/test_libm.py): the device sin / cos must be the reference
// runtime's libm bit for bit.  Arguments: the random-cosine-direction angles
// (2 pi u, u = (2k+1) 2^-53 as the path RNG draws them: util.scm:37-44), a
// wide range of both signs (marble's sin(scale z + 10 turb), texture.scm:30-34),
// and edge values.  Prints "N sin_mismatches cos_mismatches".
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "../../scheme-raytrace_amd/csrc/rt_libm.h"

static bool same(const double a, const double b) { return a == b || (std::isnan(a) && std::isnan(b)); }

// sin_full / cos_full (what the kernels call: the restatement inside its range, the platform's function
// beyond); inside the range also sin_ / cos_ themselves
static long check(const double x, long& bs, long& bc) {
    const bool in = rtlibm::in_range(x);
    if (!same(rtlibm::sin_full(x), std::sin(x)) || (in && !same(rtlibm::sin_(x), std::sin(x)))) {
        if (bs < 3) std::printf("sin(%a): %a vs libm %a\n", x, rtlibm::sin_full(x), std::sin(x));
        ++bs;
    }
    if (!same(rtlibm::cos_full(x), std::cos(x)) || (in && !same(rtlibm::cos_(x), std::cos(x)))) {
        if (bc < 3) std::printf("cos(%a): %a vs libm %a\n", x, rtlibm::cos_full(x), std::cos(x));
        ++bc;
    }
    return 1;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 4000000;
    const double kPi = 3.141592653589793;
    unsigned long long st = 0x9E3779B97F4A7C15ull;
    long bs = 0, bc = 0, total = 0;
    const double edges[] = {0.0, -0.0, 1e-300, 0x1p-27, 0x1p-26, 0.126, 0.855469, 0.8554687500000001, 2.426265,
                            kPi / 2, -kPi / 2, kPi, 2 * kPi, 1e5, -1e5, 1e8, 105414349.0, 0.5, -0.5, 1.0,
                            // the range boundary (high word 0x419921FB) and beyond: the fallback
                            0x1.921faffffffffp+26, 0x1.921fbp+26, -0x1.921fbp+26, 0x1.921fb54442d18p+26, 105414351.0,
                            1e12, -1e12, 1e300, -1e300, HUGE_VAL, -HUGE_VAL, NAN};
    for (double e : edges) total += check(e, bs, bc);
    const double bound[] = {0x1.921faffffffffp+26, 0x1.921fbp+26};   // the last value inside, the first outside
    if (!rtlibm::in_range(bound[0]) || rtlibm::in_range(bound[1])) { std::printf("in_range boundary wrong\n"); ++bs; }
    for (long i = 0; i < n; ++i) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        const double u = (double)(2 * (st >> 12) + 1) * 0x1p-53;
        total += check((2.0 * kPi) * u, bs, bc);
        total += check((u - 0.5) * 800.0, bs, bc);
        total += check((u - 0.5) * 1e6, bs, bc);
    }
    std::printf("%ld %ld %ld\n", total, bs, bc);
    return 0;
}
