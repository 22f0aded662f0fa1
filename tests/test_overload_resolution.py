"""Which log/exp the reference's filter_overlaps calls.

src/SfM_CUDA/tsdf.cu:318,329 write `log(max(probs[...] / n_obs_, prior))` and :343
`exp(assignments[i][j] / cnts[i][j])` in host code: probs and assignments are float, n_obs_ and
cnts uint32_t (tsdf.cuh:46, tsdf.cu:310) and the prior a float (configuration.h:4), so every
argument is a float.  nvcc hands host code to the host compiler with cuda_runtime.h included
first (its crt/math_functions.h pulls in <math.h> and <cmath>), and OpenCV's headers include
<cmath> too (tsdf.cuh:2).  With libstdc++ the C++ <math.h> exports std::log(float) /
std::exp(float) into the global namespace, and an unqualified call on a float takes that exact
match over the promotion to ::log(double): logf/expf of the host C library, the functions
semtsdf_libm.h restates.  This test compiles the same call shapes with the host g++ and checks
both the selected overload (static_assert on the result type) and its values (bit-equal to
logf/expf, and different from the double functions rounded to float on some inputs, so the
distinction is observable).
"""
import os
import shutil
import subprocess

import pytest

SRC = r"""
#include <cmath>
#include <math.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <type_traits>
static float fmax_(float a, float b) { return a > b ? a : b; }  /* max(float, float) -> float */
int main() {
    const float prior = 0.05f;     /* Configuration::prior_mrcnn_err_rate, a float */
    const uint32_t n_obs = 7u;     /* TSDF::n_obs_, a uint32_t */
    float probs[1] = {3.0f};
    static_assert(std::is_same<decltype(probs[0] / n_obs), float>::value, "float / uint32_t is float");
    static_assert(std::is_same<decltype(log(fmax_(probs[0] / n_obs, prior))), float>::value, "log(float) is logf");
    const uint32_t cnt = 3u;
    float acc = -1.0f;
    static_assert(std::is_same<decltype(exp(acc / cnt)), float>::value, "exp(float) is expf");
    long same_f = 0, diff_d = 0, n = 0;
    for (uint32_t u = 0x3d4ccccdu; u <= 0x3f800000u; u += 997u) {  /* [0.05, 1] */
        float x;
        memcpy(&x, &u, 4);
        const float a = log(x), b = logf(x), c = (float)log((double)x);
        same_f += memcmp(&a, &b, 4) == 0;
        diff_d += memcmp(&a, &c, 4) != 0;
        ++n;
    }
    for (uint32_t u = 0xc0400000u; u >= 0x80000001u && u <= 0xc0400000u; u -= 1009u) {  /* [-3, 0) */
        float x;
        memcpy(&x, &u, 4);
        const float a = exp(x), b = expf(x), c = (float)exp((double)x);
        same_f += memcmp(&a, &b, 4) == 0;
        diff_d += memcmp(&a, &c, 4) != 0;
        ++n;
    }
    printf("%ld %ld %ld\n", n, same_f, diff_d);
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_float_arguments_select_logf_and_expf(tmp_path):
    src = tmp_path / "overload.cpp"
    src.write_text(SRC)
    exe = tmp_path / "overload"
    # -O0 -fno-builtin: the library calls themselves, as the reference's host code makes them
    subprocess.run(["g++", "-std=c++14", "-O0", "-fno-builtin", "-ffp-contract=off", str(src), "-o", str(exe), "-lm"],
                   check=True, capture_output=True, timeout=120)
    n, same_f, diff_d = map(int, subprocess.run([str(exe)], check=True, capture_output=True, text=True,
                                                timeout=120).stdout.split())
    assert n > 1000 and same_f == n  # every value is logf's / expf's
    assert diff_d > 0  # and the double functions rounded to float would differ somewhere
    os.remove(exe)
