// CPU check of slam-maskrcnn_amd/csrc/semtsdf_libm.h against the host C library's logf/expf
// (test infrastructure, tests/test_libm_port.py).  Prints "<name> <checked> <mismatches>".
#include "../../slam-maskrcnn_amd/csrc/semtsdf_libm.h"
#include <cmath>
#include <cstdio>
#include <cstdlib>

using semtsdf::glibc::f2u;
using semtsdf::glibc::u2f;

int main(int argc, char** argv) {
    const float eps = argc > 1 ? strtof(argv[1], nullptr) : 0.05f;
    const unsigned stride = argc > 2 ? (unsigned)atoi(argv[2]) : 1u;
    long n = 0, bad = 0;
    // logf over the association's domain [eps, 1] (tsdf.cu:318,329: log(max(q, eps)), q <= 1)
    for (uint32_t u = f2u(eps); u <= f2u(1.0f); ++u, ++n)
        if (f2u(semtsdf::glibc::logf(u2f(u))) != f2u(::logf(u2f(u)))) ++bad;
    printf("logf %ld %ld\n", n, bad);
    // expf over [logf(eps), 0] (tsdf.cu:343: exp of an average of those logs), every stride-th float
    n = bad = 0;
    const uint32_t lo = f2u(::logf(eps));
    for (uint32_t u = 0x80000000u; u <= lo; u += stride, ++n)
        if (f2u(semtsdf::glibc::expf(u2f(u))) != f2u(::expf(u2f(u)))) ++bad;
    printf("expf %ld %ld\n", n, bad);
    // outside the domain: spot checks over all finite inputs the functions are meant for
    n = bad = 0;
    for (uint32_t u = 0x00800000u; u < 0x7f800000u; u += 4099u, ++n)
        if (f2u(semtsdf::glibc::logf(u2f(u))) != f2u(::logf(u2f(u)))) ++bad;
    for (uint32_t u = 0; u < 0xff800000u; u += 4099u) {
        const float x = u2f(u);
        if (!(std::fabs(x) < 80.0f)) continue;
        ++n;
        if (f2u(semtsdf::glibc::expf(x)) != f2u(::expf(x))) ++bad;
    }
    printf("spot %ld %ld\n", n, bad);
    return 0;
}
