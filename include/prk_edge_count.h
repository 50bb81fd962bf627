/* prk_edge_count.h — the visible-edge count of one triangle, as the
 * reference's FillEdgeTable returns it (projekt.cpp:3882-4121), header-only.
 *
 * libprk_hip.so's prk_fill_edge_count loops over it, and the drop-in header
 * (projekt.h) calls it inline on the vertices it snapshots, so the count and
 * the copy read each vertex once.  One definition, bit for bit the same float
 * operations in both: IEEE single precision, every product rounded before
 * its sum (prk_ec_mul keeps a caller's compiler from fusing them into FMAs
 * whatever its -ffp-contract / -march: the drop-in is built by the caller).
 */
#ifndef PRK_EDGE_COUNT_H
#define PRK_EDGE_COUNT_H

#include <math.h>
#include <stdint.h>

#include "prk.h"

/* a * b, rounded: the empty asm hands the product over in a register, so it
 * cannot be contracted into a following add. */
static inline float prk_ec_mul(float a, float b) {
    float r = a * b;
#if defined(__x86_64__) || defined(__i386__)
    __asm__("" : "+x"(r));
#elif defined(__aarch64__)
    __asm__("" : "+w"(r));
#endif
    return r;
}

/* Project (3905-3925): the reference's perspective of one camera-space point
 * (object P already added, 3898-3903); points at or behind the near plane
 * (DistanceAboveTarget - z <= 0.2) keep the zero vector. */
static inline void prk_ec_project(float cx, float cy, float cz, const prk_transform *T, float r[3]) {
    r[0] = r[1] = r[2] = 0.0f;
    const float d = T->DistanceAboveTarget - cz;
    if (d > 0.2f) {
        const float k = prk_ec_mul(1.0f / d, T->FocalLength);
        const float px = prk_ec_mul(k, cx), py = prk_ec_mul(k, cy);
        r[0] = T->ScreenCenter[0] + prk_ec_mul(T->MetersToPixels, px);
        r[1] = T->ScreenCenter[1] + prk_ec_mul(T->MetersToPixels, py);
        r[2] = d + prk_ec_mul(T->MetersToPixels, 0.0f);
    }
}

static inline void prk_ec_normalize(float *x, float *y, float *z) {
    const float s = 1.0f / sqrtf((prk_ec_mul(*x, *x) + prk_ec_mul(*y, *y)) + prk_ec_mul(*z, *z));
    *x = s * *x;
    *y = s * *y;
    *z = s * *z;
}

static inline float prk_ec_max3abs(float a, float b, float c) {
    a = fabsf(a);
    b = fabsf(b);
    c = fabsf(c);
    const float m = b > c ? b : c;
    return a > m ? a : m;
}

/* Back-face test (3926-3943) of the screen-space edge vectors A = p1 - p0,
 * B = p2 - p0: Inner((0,0,-1), Cross(Normalize(A), Normalize(B))) > 0, i.e.
 * cz = a.x*b.y - a.y*b.x < 0 of the normalised a, b.  Their components carry
 * a relative error of at most ~5 ulp and are at most 1, so the rounded cz
 * lies within ~2^-19 of the exact (Ax*By - Ay*Bx) / (|A||B|): when that
 * exceeds 2^-16 in magnitude (computed in double from the same float A, B:
 * products exact), its sign is the test's, and the two normalisations are
 * skipped.  Other cases (near-degenerate, tiny / huge / non-finite) take the
 * float ops. */
static inline int prk_ec_front(float ax, float ay, float az, float bx, float by, float bz) {
    const float ma = prk_ec_max3abs(ax, ay, az), mb = prk_ec_max3abs(bx, by, bz);
    const double D = (double)ax * by - (double)ay * bx;
    const double A2 = ((double)ax * ax + (double)ay * ay) + (double)az * az;
    const double B2 = ((double)bx * bx + (double)by * by) + (double)bz * bz;
    if (ma >= 0x1p-40f && ma <= 0x1p40f && mb >= 0x1p-40f && mb <= 0x1p40f && D * D > 0x1p-32 * A2 * B2)
        return D < 0.0;
    prk_ec_normalize(&ax, &ay, &az);
    prk_ec_normalize(&bx, &by, &bz);
    const float cz = prk_ec_mul(ax, by) - prk_ec_mul(ay, bx);
    const float cx = prk_ec_mul(ay, bz) - prk_ec_mul(az, by), cy = prk_ec_mul(az, bx) - prk_ec_mul(ax, bz);
    return (0.0f * cx + 0.0f * cy) + (-1.0f) * cz > 0.0f; /* 3943 (products exact: fusing changes nothing) */
}

/* The edges FillEdgeTable writes for the triangle v[0..8] (three xyz
 * vertices) of an object at P: 0 when it faces away (3926-3943), else its
 * edges that are not horizontal and reach below row 0 (3957-3968, 4066). */
static inline uint32_t prk_tri_edge_count(const float *v, float p0, float p1, float p2, const prk_transform *T) {
    float pr[3][3];
    for (int k = 0; k < 3; ++k) prk_ec_project(v[3 * k] + p0, v[3 * k + 1] + p1, v[3 * k + 2] + p2, T, pr[k]);
    const int front = prk_ec_front(pr[1][0] - pr[0][0], pr[1][1] - pr[0][1], pr[1][2] - pr[0][2],
                                   pr[2][0] - pr[0][0], pr[2][1] - pr[0][1], pr[2][2] - pr[0][2]);
    uint32_t ne = 0; /* (branch-free: the facing of a triangle soup is a coin toss) */
    for (int e = 0; e < 3; ++e) {
        const float y0 = pr[e][1], y1 = pr[(e + 1) % 3][1];
        const float mn = y0 > y1 ? y1 : y0, mx = y0 > y1 ? y0 : y1; /* 3957-3966 */
        ne += (uint32_t)((mx > 0) & (mn - mx != 0));                 /* 3968, 4066 */
    }
    return front ? ne : 0u;
}

#if defined(__SSE2__)
#include <emmintrin.h>
#define PRK_EC_SSE 1
static inline __m128 prk_ec_mul4(__m128 a, __m128 b) {
    __m128 r = _mm_mul_ps(a, b);
    __asm__("" : "+x"(r));
    return r;
}
/* prk_tri_edge_count of the triangle loaded as q0 = v[0..3], q1 = v[4..7],
 * q2 = (v[8], ...): the three vertices projected side by side in SSE lanes
 * (the same IEEE single operations per lane), the facing test as above.
 * The drop-in stores the same registers as its vertex snapshot. */
static inline uint32_t prk_tri_edge_count_sse(__m128 q0, __m128 q1, __m128 q2, float p0, float p1, float p2,
                                              const prk_transform *T) {
    const __m128 x = _mm_shuffle_ps(q0, q1, _MM_SHUFFLE(3, 2, 3, 0));             /* v0 v3 v6 . */
    const __m128 ty = _mm_shuffle_ps(q0, q1, _MM_SHUFFLE(3, 0, 1, 1));            /* v1 . v4 v7 */
    const __m128 y = _mm_shuffle_ps(ty, ty, _MM_SHUFFLE(3, 3, 2, 0));             /* v1 v4 v7 . */
    const __m128 tz = _mm_shuffle_ps(q0, q1, _MM_SHUFFLE(1, 1, 2, 2));            /* v2 . v5 . */
    const __m128 z = _mm_shuffle_ps(tz, q2, _MM_SHUFFLE(0, 0, 2, 0));             /* v2 v5 v8 . */
    const __m128 cx = _mm_add_ps(x, _mm_set1_ps(p0)), cy = _mm_add_ps(y, _mm_set1_ps(p1));
    const __m128 cz = _mm_add_ps(z, _mm_set1_ps(p2));
    const __m128 d = _mm_sub_ps(_mm_set1_ps(T->DistanceAboveTarget), cz);
    const __m128 near_ok = _mm_cmpgt_ps(d, _mm_set1_ps(0.2f));
    const __m128 k = prk_ec_mul4(_mm_div_ps(_mm_set1_ps(1.0f), d), _mm_set1_ps(T->FocalLength));
    const __m128 m2p = _mm_set1_ps(T->MetersToPixels);
    const __m128 rx = _mm_and_ps(near_ok, _mm_add_ps(_mm_set1_ps(T->ScreenCenter[0]), prk_ec_mul4(m2p, prk_ec_mul4(k, cx))));
    const __m128 ry = _mm_and_ps(near_ok, _mm_add_ps(_mm_set1_ps(T->ScreenCenter[1]), prk_ec_mul4(m2p, prk_ec_mul4(k, cy))));
    const __m128 rz = _mm_and_ps(near_ok, _mm_add_ps(d, prk_ec_mul4(m2p, _mm_setzero_ps())));
    /* lanes 1, 2: p1 - p0, p2 - p0 */
    const __m128 dx = _mm_sub_ps(rx, _mm_shuffle_ps(rx, rx, 0));
    const __m128 dy = _mm_sub_ps(ry, _mm_shuffle_ps(ry, ry, 0));
    const __m128 dz = _mm_sub_ps(rz, _mm_shuffle_ps(rz, rz, 0));
    /* prk_ec_front's fast test on (A, B) in double lanes: X = (ax, bx) ... */
    const __m128d X = _mm_cvtps_pd(_mm_shuffle_ps(dx, dx, _MM_SHUFFLE(3, 3, 2, 1)));
    const __m128d Y = _mm_cvtps_pd(_mm_shuffle_ps(dy, dy, _MM_SHUFFLE(3, 3, 2, 1)));
    const __m128d Z = _mm_cvtps_pd(_mm_shuffle_ps(dz, dz, _MM_SHUFFLE(3, 3, 2, 1)));
    const __m128d XYs = _mm_mul_pd(X, _mm_shuffle_pd(Y, Y, 1));           /* (ax*by, bx*ay): exact */
    const __m128d D = _mm_sub_sd(XYs, _mm_unpackhi_pd(XYs, XYs));          /* ax*by - ay*bx */
    const __m128d S2 = _mm_add_pd(_mm_add_pd(_mm_mul_pd(X, X), _mm_mul_pd(Y, Y)), _mm_mul_pd(Z, Z)); /* (A2, B2) */
    const __m128d rhs = _mm_mul_sd(_mm_mul_sd(_mm_set_sd(0x1p-32), S2), _mm_unpackhi_pd(S2, S2));
    /* max |component| of A and B (lanes 1, 2) within [2^-40, 2^40]; a NaN
     * fails the compares, as it fails prk_ec_front's */
    const __m128 ab = _mm_castsi128_ps(_mm_set1_epi32(0x7FFFFFFF));
    const __m128 mm = _mm_max_ps(_mm_max_ps(_mm_and_ps(dx, ab), _mm_and_ps(dy, ab)), _mm_and_ps(dz, ab));
    const int inr = _mm_movemask_ps(_mm_and_ps(_mm_cmpge_ps(mm, _mm_set1_ps(0x1p-40f)),
                                               _mm_cmple_ps(mm, _mm_set1_ps(0x1p40f))));
    int front;
    if ((inr & 6) == 6 && _mm_comigt_sd(_mm_mul_sd(D, D), rhs)) {
        front = _mm_comilt_sd(D, _mm_setzero_pd());
    } else {
        float ex[4], ey[4], ez[4];
        _mm_storeu_ps(ex, dx);
        _mm_storeu_ps(ey, dy);
        _mm_storeu_ps(ez, dz);
        front = prk_ec_front(ex[1], ey[1], ez[1], ex[2], ey[2], ez[2]);
    }
    /* edges (y0,y1) (y1,y2) (y2,y0): min and max as the scalar selects */
    const __m128 yn = _mm_shuffle_ps(ry, ry, _MM_SHUFFLE(3, 0, 2, 1));
    const __m128 mn = _mm_min_ps(yn, ry), mx = _mm_max_ps(ry, yn);
    const __m128 ok = _mm_and_ps(_mm_cmpgt_ps(mx, _mm_setzero_ps()), _mm_cmpneq_ps(_mm_sub_ps(mn, mx), _mm_setzero_ps()));
    const int m = _mm_movemask_ps(ok) & 7;
    const uint32_t ne = (uint32_t)((m & 1) + ((m >> 1) & 1) + (m >> 2));
    return front ? ne : 0u;
}
#endif

#endif /* PRK_EDGE_COUNT_H */
