"""The scalar Phong term's pow, pinned for every input it can take.

DrawModel's Phong path computes PhongTerm = pow(PhongTerm, 16) in double and
stores it to a float (projekt.cpp:478; SURVEY.md: double pow); PhongTerm is
clamped to [0, 1] just before (477).  k_pix (prk_kernels.hip, "pow((double)Ph, 16.0) ... four exact-range
double squarings") computes it as ((x^2)^2)^2)^2 in double: x^2 is exact (a
float's 24-bit significand squared fits a double), the three later squarings
round, so the double is within 3.5 ulp of x^16.  The oracle calls the host
libm's pow (oracle/prk_oracle.c).

This test walks all 1,065,353,217 floats in [0, 1] (8 threads, ~10 s) and
checks, in one loop:
  * the kernel's squarings, cast to float, equal (float)pow(x, 16.0) -- the
    oracle's expression -- bit for bit;
  * exact x^16 (double-double, ~2^-100 relative) lies at least MARGIN double
    ulps from every float rounding boundary, so ANY pow within MARGIN ulp of
    exact (a faithful libm: glibc, the reference's MSVC CRT) rounds to the
    same float.  The scalar Phong colours are therefore exact, not +-1 LSB.
The C program repeats k_pix's op order; device f64 mul is IEEE
round-to-nearest like the host's, and the GPU parity tests compare the
scalar Phong frames bit for bit.
"""
import os
import subprocess

import pytest

MARGIN = 8.0  # double ulps (measured minimum: 9.17, at x = 0x1.3fb41cp-8)

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static float kpix_pow16(float x) {  /* k_pix's op order */
    double ph = (double)x;
    ph = ph * ph; ph = ph * ph; ph = ph * ph; ph = ph * ph;
    return (float)ph;
}
int main(void) {
    const uint32_t lim = 0x3F800000u; /* 1.0f */
    long bad = 0;
    double best = 1e300;
    uint32_t bestb = 0;
#pragma omp parallel
    {
        double lb = 1e300;
        uint32_t lbb = 0;
#pragma omp for reduction(+ : bad) schedule(static, 65536)
        for (long i = 0; i <= (long)lim; ++i) {
            const uint32_t b = (uint32_t)i;
            float x;
            memcpy(&x, &b, 4);
            const float want = (float)pow((double)x, 16.0), got = kpix_pow16(x);
            if (memcmp(&want, &got, 4) != 0) ++bad;
            /* exact x^16 as h + l */
            double h = (double)x * (double)x, l = 0.0;
            for (int k = 0; k < 3; ++k) {
                const double p = h * h;
                double e = fma(h, h, -p);
                e = fma(2.0 * h, l, e);
                h = p + e;
                l = e - (h - p);
            }
            if (h < 0x1p-151) continue; /* rounds to +0 under any faithful pow */
            const float f = (float)h;
            const double up = 0.5 * ((double)f + (double)nextafterf(f, INFINITY));
            const double dn = 0.5 * ((double)f + (double)nextafterf(f, 0.0f));
            const double ulp = nextafter(h, INFINITY) - h;
            const double d1 = fabs((h - up) + l) / ulp, d2 = fabs((h - dn) + l) / ulp;
            const double d = d1 < d2 ? d1 : d2;
            if (d < lb) { lb = d; lbb = b; }
        }
#pragma omp critical
        if (lb < best) { best = lb; bestb = lbb; }
    }
    printf("%ld %.6f %08x\n", bad, best, bestb);
    return 0;
}
"""


def test_scalar_phong_pow_exhaustive(tmp_path):
    src = tmp_path / "pow16.c"
    src.write_text(SRC)
    exe = tmp_path / "pow16"
    r = subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", str(src), "-o", str(exe), "-lm"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("gcc -fopenmp unavailable: " + r.stderr[-200:])
    env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr
    bad, dist, where = r.stdout.split()
    assert int(bad) == 0, "k_pix's squarings differ from (float)pow(x, 16.0) for %s floats" % bad
    assert float(dist) >= MARGIN, "x^16 comes %s double ulps from a float boundary (x bits %s)" % (dist, where)
