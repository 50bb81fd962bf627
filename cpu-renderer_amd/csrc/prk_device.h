// prk_device.h — device-side restatement of the reference hot path for gfx950.
//
// Every function here reproduces a piece of projekt.cpp bit for bit: it must
// be compiled with -ffp-contract=off (no FMA contraction) and
// with IEEE division / square root (hipcc's default,
// -fhip-fp32-correctly-rounded-divide-sqrt).  Pins for the reference's absent
// math header follow SURVEY §8(c): RoundR32ToS32 = (s32)roundf,
// Normalize(a) = (1/sqrtf(Inner(a,a)))*a, Inner = (ax*bx + ay*by) + az*bz.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Diagnostic builds only (prk_kernels.hip lists the bits); never set in a product build.
#ifndef PRK_DIAG
#define PRK_DIAG 0
#endif

namespace prk {

constexpr int kMaxLights = 8;

// Span-kernel flavours.  AVX = FillLineOptimized (projekt.cpp:1492-2320) with
// texture + Phong (the only AVX configuration with defined output);
// SC_* = scalar DrawModel (projekt.cpp:162-601).
enum Mode : int {
    MODE_AVX = 0,
    MODE_SC_GOURAUD = 1,      // untextured, vertex-lit colour
    MODE_SC_GOURAUD_TEX = 2,  // texel replaces colour, no lighting
    MODE_SC_PHONG = 3,        // untextured Phong
    MODE_SC_PHONG_TEX = 4,    // textured Phong
    MODE_COUNT = 5
};

struct DrawRec {
    const float *V, *C, *N, *UV;  // geometry base pointers (SoA, non-indexed)
    uint32_t geom_tri0;           // first triangle of this draw inside the geometry
    uint32_t first_global;        // global (submission-order) index of its first triangle
    uint32_t tri_count;
    int32_t mode;                 // Mode
    int32_t tex;                  // texture index or -1
    float P[3];                   // object offset (render_entry_3d_object::P)
    uint32_t flags;               // DRAW_ST: single-thread DrawModelOptimized(Buffer,...) quirks
    uint32_t obj_tris;            // triangles per render_entry_3d_object (1: per-triangle AETs;
                                  // > 1: one AET per object, drawn through the span path)
    uint32_t src_kind;            // 0: geometry; 1: a caller's edge list; 2: caller spans (span path)
    uint32_t src_off, src_n;      // kind 1/2: range of the flush's edge / span input
    int32_t geom;                 // host: the geometry handle (draw coalescing, geometry updates)
};

// Draw flags.  DRAW_ST: the single-thread overload DrawModelOptimized(Buffer,
// ...) (projekt.cpp:2350-3358), whose span body differs from FillLineOptimized
// in exactly two places: a left-clipped span sets XOffset = -XOffset (= -0.0f,
// 2508) instead of -L.X, and the z-test is predicate 29, GE_OQ (3205):
// z >= zbuf, so among equal z the LATEST fragment wins (and it beats an equal
// prior z).
// DRAW_RAWCOL / DRAW_WHITELIT: what FillEdgeTable left in MinColor for an
// untextured non-Phong DrawModel (MODE_SC_GOURAUD), which depends on
// FillEdgeTable's own inputs, not on the draw's: PhongShading != 0 stores the
// raw vertex colours (projekt.cpp:4012-4019, so DrawModel interpolates them
// unlit); PhongShading == 0 lights them per vertex (4020-4063), from a white
// base when Object->Bitmap is set (4034-4054, DRAW_WHITELIT), else from the
// vertex colour.  Every other mode's output does not depend on them.
enum : uint32_t { DRAW_ST = 1u, DRAW_RAWCOL = 2u, DRAW_WHITELIT = 4u };
// Span path (whole-object AETs): SpanPos flags of a DrawModel (scalar) span,
// whose mode sits at bits 8..15, and the first word of its FillLineOptimized
// record slot (no AVX record has bit 31 set: texture indices are < 2^15).
constexpr uint32_t SPAN_SCALAR = 2u;
constexpr uint32_t kScalarSpan = 0x80000000u;

// Visibility key low words.  Keys are max-reduced: a
// fragment's key is (ordered z << 32) | tag.  Queue-semantics pairs (strict
// '>', earliest wins on equal z) take 0x7FFFFFFE - j, the prior z-buffer
// 0x7FFFFFFF, single-thread pairs (>=, latest wins and beats the prior)
// 0x80000000 + j, where j is the pair's submission-order index: this ordering
// reproduces any interleaving of the two tie rules in one frame.
constexpr uint32_t kTagPrior = 0x7FFFFFFFu;
constexpr uint32_t kMaxPairs = 0x7FFFFFFFu;  // j < kMaxPairs
__device__ __forceinline__ uint32_t pair_tag(uint32_t j, bool ge) { return ge ? 0x80000000u + j : 0x7FFFFFFEu - j; }
// The winning pair of a key low word; false for the prior z (0x7FFFFFFF) and
// for a NaN prior z, whose key is all ones and blocks the pixel.
__device__ __forceinline__ bool tag_pair(uint32_t low, uint32_t &j) {
    if (low == kTagPrior || low == 0xFFFFFFFFu) return false;
    j = low < kTagPrior ? 0x7FFFFFFEu - low : low - 0x80000000u;
    return true;
}

struct TexRec {
    const uint8_t *mem;  // (h+1) rows, last one the zeroed guard row
    int32_t w, h, pitch;
    int32_t filter;      // PRK_FILTER_* (bilinear: AVX semantics only, an extension)
};

// Per-triangle setup record of an AVX-semantics frame, written once per
// frame by the binning pass (k_bin_count) and read by every bin entry of the
// triangle in k_vis and by k_walk: FillEdgeTable (projekt.cpp:3882-4121) +
// MergeSort (2-72) + the AET insertions of the triangle's first row
// (3654-3713), so no raster kernel repeats the ~30 divisions of the setup.
// TriRec holds what the visibility sweep reads (160 B) plus, for the shading
// walk, which vertices each sorted edge joins: k_walk rebuilds the edges'
// normals (4014-4019, 4103-4108: no top clip) from the triangle's three vertex
// normals, which costs it a 36-B read instead of an 80-B record per triangle.
struct TriRec {
    float e[3][10];      // sorted edge k: X, G, Z, ZG, W, WG, U, UG, V, VG
    int32_t ymin[3];     // YMin | Left << 31 (YMin >= 0: Maximum(0, .), 3999)
    int32_t ymax[3];
    uint32_t head;       // n | ord << 4 | cnt << 12 | (pend + 1) << 16 | anomaly << 20 | st << 24
    uint32_t vtx;        // sorted edge k's Vtx (mi | ma << 2) at bits 4k
    uint32_t pad[2];
};
static_assert(sizeof(TriRec) == 160, "TriRec is ten dwordx4");

// The camera and lights a span is shaded with: UnprojectVertex(_8x) and the
// Phong loop read Commands->Transform / LightData when the span runs
// (DrawModel 452-458, FillLineOptimized 2042-2046, the single-thread overload
// 3030-3034), which need not be what FillEdgeTable saw (prk_set_shade_camera).
struct ShadeCam {
    float D, F, Cx, Cy, InvM2P;
    float InvF;       // 1/F, exact when f_pow2
    int32_t f_pow2;   // F = 2^k (k in [-125,126]): d/F == d*InvF bit for bit
    uint32_t light_count;
    float amb[4];
    float lp[kMaxLights][3];
    float li[kMaxLights][4];
};

struct FrameParams {
    // projective_transform and light_data of the setup (FillEdgeTable:
    // ProjectVertex 3906-3910, Gouraud lighting 4020-4063)
    float D, F, M2P, Cx, Cy, InvM2P;
    float InvF;
    int32_t f_pow2;
    uint32_t light_count;
    float amb[4];
    float lp[kMaxLights][3];
    float li[kMaxLights][4];
    // ... and of the span shading
    ShadeCam sh;
    // target band: frame rows [row0,row1) of a W x H frame
    int32_t W, H, row0, row1;
    int32_t pitch;   // colour pitch in bytes
    uint32_t *color; // points at frame row row0
    float *zbuf;     // points at frame row row0 (row stride W floats)
    int32_t *winners;// optional (debug): per pixel winning triangle, -1 none
    uint32_t win_base; // winner ids of this pass start here (frames drawn in several passes)
    // fused clear (prk_target_clear_on_flush): prior contents are (clear_color, clear_z)
    int32_t clear_fused;
    uint32_t clear_color;
    float clear_z;
    unsigned long long *prof;  // 16 phase-cycle counters (PRK_PROF builds only write them)
    // span-record frames with z_in_vis (prk_set_early_z): k_vis writes z, k_pix
    // the colour (and a -0.0 z, which the visibility key stores as +0.0,
    // counted in negz for the download); else k_pix writes both
    int32_t z_in_vis;
    uint32_t *negz;
    // tiling
    int32_t tile_w, tile_h, tiles_x, tiles_y;
    int32_t tile_w_log2;  // tile_w is a power of two
    // geometry
    uint32_t tri_count;
    uint32_t ndraws;
    const DrawRec *draws;
    const uint32_t *tri_draw;  // nullptr when ndraws == 1
    const TexRec *texs;
    // Single-draw frames (k_raster<M, true>): the draw and its texture as
    // kernel arguments, i.e. wave-uniform scalar registers.
    DrawRec draw0;
    TexRec tex0;
    // Setup records (all-AVX frames; nullptr otherwise): written by
    // k_bin_count for every binned triangle, read by k_vis / k_walk.
    TriRec *trec;
};

// d / FocalLength of UnprojectVertex(_8x) (projekt.cpp:141-142, 157).  When
// F is a power of two the quotient is the single rounding of d*2^-k, which
// the multiply by the exact 1/F also produces.  (fp is uniform: a scalar
// branch, no divergence.)
__device__ __forceinline__ float div_focal(const FrameParams &fp, float d);  // (below DivBy)

// (float)k / 255.0f for an integer k in [0, 255], bit for bit: k * RN(1/255)
// plus one FMA residual correction is the correctly rounded quotient for
// every such k (exhaustive check: tests/test_oracle.py::test_u8_unit_exact).
__device__ __forceinline__ float u8_unit(uint32_t k) {
    const float c = 0x1.010102p-8f;  // RN(1/255)
    const float kf = (float)k, q0 = kf * c;
    const float rem = __builtin_fmaf(-255.0f, q0, kf);  // exact residual
    return __builtin_fmaf(rem, c, q0);
}

// Tiles a triangle may touch: the rectangle [tx0..tx1] x [ty0..ty1], plus
// for scalar semantics the column-0 tiles of rows [oty0..oty1] that receive
// DrawModel's one-past-the-row store (see span_setup_scalar).
// pad0 / pad1: the triangle's band rows [r0, r1) (prk_bin.hip: row classes)
struct TileRange { uint16_t tx0, ty0, tx1, ty1, oty0, oty1, pad0, pad1; };

// ---------------------------------------------------------------------------
// Conversions with x86 semantics (the reference runs on x86).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int32_t cvtt_s32(float f) {
    // cvttss2si / cvttps2dq: NaN and out-of-range give INT_MIN.
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int32_t)f : INT32_MIN;
}
__device__ __forceinline__ int32_t round_s32(float f) { return cvtt_s32(roundf(f)); }
__device__ __forceinline__ uint32_t round_u32(float f) {
    // x86-64 (u32)float: 64-bit cvttss2si, keep the low 32 bits.
    float r = roundf(f);
    return (r >= -9223372036854775808.0f && r < 9223372036854775808.0f)
               ? (uint32_t)(uint64_t)(int64_t)r
               : 0u;
}
__device__ __forceinline__ int32_t cvt_rne_s32(float f) {
    // _mm256_cvtps_epi32 with the default MXCSR: round to nearest even.
    return (f >= -2147483648.0f && f < 2147483648.0f) ? (int32_t)__builtin_rintf(f) : INT32_MIN;
}
__device__ __forceinline__ float maxps(float a, float b) { return a > b ? a : b; }  // MAXPS
__device__ __forceinline__ float minps(float a, float b) { return a < b ? a : b; }  // MINPS
__device__ __forceinline__ float clamp01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }

// FillLineOptimized's span ends (projekt.cpp:1545-1592): LeftX / RightX
// clamped to [0, W-1], MinX = round(LeftX), MaxX = round(RightX), and XDiff =
// round(R.X) - round(L.X) on the unclamped ends (1568-1570).  A clamped end
// is 0 or W - 1, which round to themselves, so two roundings serve all four
// (PRK_SPAN_ROUND2; 0: the literal four).  False for a NaN end (pinned: the
// span draws nothing).  st: the single-thread overload's left-clip XOffset
// (2508).
#ifndef PRK_SPAN_ROUND2
#define PRK_SPAN_ROUND2 1
#endif
__device__ __forceinline__ bool span_ends(float LX, float RX, int32_t W, bool st, int32_t &MinX, int32_t &MaxX,
                                          int32_t &XDiff, float &XOffset) {
    XOffset = 0.0f;
    if (LX != LX || RX != RX) return false;
    const bool lneg = LX < 0, lbig = LX >= W, rneg = RX < 0, rbig = RX >= W;
    if (lneg) XOffset = st ? -XOffset : -LX;  // 1545-1565
    if (PRK_SPAN_ROUND2) {
        const int32_t rl = round_s32(LX), rr = round_s32(RX);
        XDiff = (int32_t)((uint32_t)rr - (uint32_t)rl);
        MinX = lneg ? 0 : (lbig ? W - 1 : rl);
        MaxX = rneg ? 0 : (rbig ? W - 1 : rr);
    } else {
        XDiff = (int32_t)((uint32_t)round_s32(RX) - (uint32_t)round_s32(LX));
        MinX = round_s32(lneg ? 0.0f : (lbig ? (float)W - 1 : LX));
        MaxX = round_s32(rneg ? 0.0f : (rbig ? (float)W - 1 : RX));
    }
    return true;
}

// Normalize (pinned scalar form) — used by the AET edge step and DrawModel.
__device__ __forceinline__ void normalize_rcp(float &x, float &y, float &z) {
    float s = 1.0f / sqrtf((x * x + y * y) + z * z);
    x = s * x;
    y = s * y;
    z = s * z;
}
// ---- quotients sharing one divisor ------------------------------------------
// `x / d` (f32, IEEE division, denormals on) compiles on gfx950 to: v_div_scale
// of d and of x, v_rcp of the scaled d, two Newton FMAs refining the
// reciprocal, the quotient, two residual FMAs, v_div_fmas and v_div_fixup.
// When |d| lies in [2^-32, 2^32] and |x| in [2^-80, 2^32], v_div_scale returns
// its operands unchanged (no extreme exponent gap, no denormal operand,
// reciprocal or quotient) and v_div_fixup passes the finite quotient through,
// so the sequence is exactly the FMA chain of div_fast — whose reciprocal half
// (div_by) depends on d alone.  Several quotients over one d (a
// normalisation, a span's or an edge's increments) share it: one v_rcp and
// two FMAs instead of one v_rcp, two v_div_scale, v_div_fmas and v_div_fixup
// per quotient.  div_all takes that path when every lane of the wave is in
// range (a wave-uniform branch, so the quotients stay one straight-line,
// interleaved block) and the plain divisions otherwise: every quotient is the
// correctly rounded x / d, bit for bit (prk_selftest_div,
// tests/test_gpu_parity.py::test_shared_divisor_exact).
#ifndef PRK_SHARED_DIV
#define PRK_SHARED_DIV 1
#endif
struct DivBy {
    float nd, r;
};
__device__ __forceinline__ DivBy div_by(float d) {
    DivBy s;
    s.nd = -d;
    const float r0 = __builtin_amdgcn_rcpf(d);
    const float e = __builtin_fmaf(s.nd, r0, 1.0f);
    s.r = __builtin_fmaf(e, r0, r0);
    return s;
}
__device__ __forceinline__ float div_fast(const DivBy &s, float x) {
    const float m = x * s.r;
    const float f2 = __builtin_fmaf(s.nd, m, x);
    const float m1 = __builtin_fmaf(f2, s.r, m);
    const float f4 = __builtin_fmaf(s.nd, m1, x);
    return __builtin_fmaf(f4, s.r, m1);
}
// x[k] / d for every k.
template <int K>
__device__ __forceinline__ void div_all(float d, float (&x)[K]) {
    if (PRK_SHARED_DIV) {
        // NaN / inf / large numerators fail the sum, zero and tiny ones the min
        float sum = fabsf(x[0]), mn = fabsf(x[0]);
#pragma unroll
        for (int k = 1; k < K; ++k) {
            sum = sum + fabsf(x[k]);
            mn = fminf(mn, fabsf(x[k]));
        }
        const float ad = fabsf(d);
        const bool ok = ad >= 0x1p-32f && ad <= 0x1p32f && sum <= 0x1p32f && mn >= 0x1p-80f;
        if (__builtin_expect(__all(ok), 1)) {
            const DivBy s = div_by(d);
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = div_fast(s, x[k]);
            return;
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = x[k] / d;
}

// d / F (the focal length divide of UnprojectVertex); F is uniform, so its
// reciprocal half can be hoisted out of a thread's pixel loop.
__device__ __forceinline__ float div_focal(const FrameParams &fp, float d) {
    if (fp.sh.f_pow2) return d * fp.sh.InvF;
    float q[1] = {d};
    div_all(fp.sh.F, q);
    return q[0];
}

// sqrtf for x in [2^-96, FLT_MAX]: the compiler's correctly rounded f32
// sqrt (denormals on) is v_sqrt_f32 plus a one-ulp correction from the two
// neighbours' residuals, wrapped in a 2^32 pre-scale for x < 2^-96 and a
// zero / +inf pass-through; in this range both wrappers are identities, so
// this is the same value bit for bit (prk_selftest_div checks it).
__device__ __forceinline__ float sqrt_mid(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __int_as_float(__float_as_int(s) - 1), up = __int_as_float(__float_as_int(s) + 1);
    const float vp = __builtin_fmaf(-dn, s, x), vs = __builtin_fmaf(-up, s, x);
    float r = vp <= 0.0f ? dn : s;
    r = vs > 0.0f ? up : r;
    return r;
}

// NormalizeVector_8x (projekt.cpp:603-620), one lane: division form (three
// quotients over one length).  Fast path (wave-uniform, as div_all): the
// squared length in [2^-64, 2^62] puts the length in [2^-32, 2^31] (sqrt is
// correctly rounded and monotone) and every |component| below 2^32, so the
// sqrt wrappers and the division's scale / fixup steps are identities.
#ifndef PRK_FAST_NORM
#define PRK_FAST_NORM 1
#endif
__device__ __forceinline__ void normalize_div(float &x, float &y, float &z) {
    const float d = (x * x + y * y) + z * z;
    if (PRK_SHARED_DIV && PRK_FAST_NORM) {
        const float mn = fminf(fminf(fabsf(x), fabsf(y)), fabsf(z));
        const bool ok = d >= 0x1p-64f && d <= 0x1p62f && mn >= 0x1p-80f;
        if (__builtin_expect(__all(ok), 1)) {
            const DivBy s = div_by(sqrt_mid(d));
            x = div_fast(s, x);
            y = div_fast(s, y);
            z = div_fast(s, z);
            return;
        }
    }
    const float len = sqrtf(d);
    float q[3] = {x, y, z};
    div_all(len, q);
    x = q[0];
    y = q[1];
    z = q[2];
}

// _mm_mullo_epi16/_mm_mulhi_epi16 pitch multiply (projekt.cpp:1916-1920).
__device__ __forceinline__ int32_t mul16_trick(int32_t y, int32_t p) {
    uint32_t ylo = (uint32_t)y & 0xFFFFu, yhi = (uint32_t)y >> 16;
    uint32_t plo = (uint32_t)p & 0xFFFFu, phi = (uint32_t)p >> 16;
    uint32_t lo = (ylo * plo) & 0xFFFFu;
    uint32_t hi_mullo = (yhi * phi) & 0xFFFFu;
    int32_t sprod = (int32_t)(int16_t)ylo * (int32_t)(int16_t)plo;
    uint32_t hi_mulhi = ((uint32_t)sprod >> 16) & 0xFFFFu;
    return (int32_t)(lo | ((hi_mullo | hi_mulhi) << 16));
}

// Texel read with the P2/P4 clamp: offsets outside [0, Pitch*(Th+1)-4] read
// offset 0.  The texture holds its zeroed guard row.
__device__ __forceinline__ uint32_t texel_at(const TexRec &t, int32_t off) {
    int64_t limit = (int64_t)t.pitch * (t.h + 1) - 4;
    if (off < 0 || (int64_t)off > limit) off = 0;
    const uint8_t *p = t.mem + off;
    if ((off & 3) == 0) return *(const uint32_t *)p;
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// The wave's LDS writes are visible to all its lanes (no workgroup barrier).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Ordered 32-bit key of a float z for the visibility max (strict '>' with
// submission order == max z, earliest triangle on ties).
// +0 and -0 compare equal in the reference, so both map to one key.
__device__ __forceinline__ uint32_t zkey(float z) {
    uint32_t b = __float_as_uint(z);
    if (z == 0.0f) b = 0u;
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
// The z of a key's high word (-0.0 comes back as +0.0: zkey merges them).
__device__ __forceinline__ float zkey_z(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// ---------------------------------------------------------------------------
// Edge record (edge_info, projekt.h:17-37) as registers.
// ---------------------------------------------------------------------------
struct Edge {
    float X, G, Z, ZG, W, WG, U, UG, V, VG;
    float N0, N1, N2, NG0, NG1, NG2;
    float C0, C1, C2, C3, CG0, CG1, CG2, CG3;
    int32_t YMin, YMax, Left;
    int32_t Vtx;  // the edge's (Min, Max) vertex of its triangle: mi | ma << 2 (setup records)
};

__device__ __forceinline__ Edge sel(bool c, const Edge &a, const Edge &b) {
    Edge r;
    r.X = c ? a.X : b.X; r.G = c ? a.G : b.G; r.Z = c ? a.Z : b.Z; r.ZG = c ? a.ZG : b.ZG;
    r.W = c ? a.W : b.W; r.WG = c ? a.WG : b.WG; r.U = c ? a.U : b.U; r.UG = c ? a.UG : b.UG;
    r.V = c ? a.V : b.V; r.VG = c ? a.VG : b.VG;
    r.N0 = c ? a.N0 : b.N0; r.N1 = c ? a.N1 : b.N1; r.N2 = c ? a.N2 : b.N2;
    r.NG0 = c ? a.NG0 : b.NG0; r.NG1 = c ? a.NG1 : b.NG1; r.NG2 = c ? a.NG2 : b.NG2;
    r.C0 = c ? a.C0 : b.C0; r.C1 = c ? a.C1 : b.C1; r.C2 = c ? a.C2 : b.C2; r.C3 = c ? a.C3 : b.C3;
    r.CG0 = c ? a.CG0 : b.CG0; r.CG1 = c ? a.CG1 : b.CG1; r.CG2 = c ? a.CG2 : b.CG2;
    r.CG3 = c ? a.CG3 : b.CG3;
    r.YMin = c ? a.YMin : b.YMin; r.YMax = c ? a.YMax : b.YMax; r.Left = c ? a.Left : b.Left;
    r.Vtx = c ? a.Vtx : b.Vtx;
    return r;
}

// Which edge fields a mode actually reads.  Skipping dead fields changes no
// output: the texel overwrites the AVX colour lanes (projekt.cpp:2029-2032);
// untextured objects never read U/V/(1/z); non-Phong never reads normals.
template <int M> struct ModeTraits;
template <> struct ModeTraits<MODE_AVX> { static constexpr bool tex = true, phong = true, color = false; };
template <> struct ModeTraits<MODE_SC_GOURAUD> { static constexpr bool tex = false, phong = false, color = true; };
template <> struct ModeTraits<MODE_SC_GOURAUD_TEX> { static constexpr bool tex = true, phong = false, color = false; };
template <> struct ModeTraits<MODE_SC_PHONG> { static constexpr bool tex = false, phong = true, color = true; };
template <> struct ModeTraits<MODE_SC_PHONG_TEX> { static constexpr bool tex = true, phong = true, color = false; };

struct V3 { float x, y, z; };

// x / fp.tile_h for x >= 0.  tile_h is 8 in every default configuration, so
// a uniform branch takes a shift there instead of the ~30-instruction
// integer division (the binning's tile ranges divide six times a triangle).
__device__ __forceinline__ int32_t tile_row_of(const FrameParams &fp, int32_t x) {
    const uint32_t h = (uint32_t)fp.tile_h;
    if ((h & (h - 1)) == 0) return (int32_t)((uint32_t)x >> __builtin_ctz(h));
    return (int32_t)((uint32_t)x / h);
}

// ProjectVertex (projekt.cpp:74-93).
__device__ __forceinline__ V3 project_vertex(V3 c, const FrameParams &fp) {
    V3 r = {0.0f, 0.0f, 0.0f};
    float d = fp.D - c.z;
    if (d > 0.2f) {
        float k = (1.0f / d) * fp.F;
        float px = k * c.x, py = k * c.y;
        r.x = fp.Cx + fp.M2P * px;
        r.y = fp.Cy + fp.M2P * py;
        r.z = d + fp.M2P * 0.0f;
    }
    return r;
}

__device__ __forceinline__ V3 nrm_rcp(V3 a) {
    normalize_rcp(a.x, a.y, a.z);
    return a;
}

// Back-face test of FillEdgeTable (projekt.cpp:3926-3943):
// Inner((0,0,-1), Cross(Normalize(P1-P0), Normalize(P2-P0))) > 0.
__device__ __forceinline__ bool front_facing(const V3 *p) {
    V3 a = nrm_rcp(V3{p[1].x - p[0].x, p[1].y - p[0].y, p[1].z - p[0].z});
    V3 b = nrm_rcp(V3{p[2].x - p[0].x, p[2].y - p[0].y, p[2].z - p[0].z});
    float cx = a.y * b.z - a.z * b.y;
    float cy = a.z * b.x - a.x * b.z;
    float cz = a.x * b.y - a.y * b.x;
    float inner = (0.0f * cx + 0.0f * cy) + (-1.0f) * cz;
    return inner > 0.0f;
}

struct TriVerts {
    V3 cam[3], proj[3], nrm[3];
    float col[3][4], uv[3][2];
};

__device__ __forceinline__ void resolve_draw(const FrameParams &fp, uint32_t g, const DrawRec *&d,
                                             uint32_t &gt) {
    uint32_t di = fp.ndraws == 1 ? 0u : fp.tri_draw[g];
    d = fp.draws + di;
    gt = d->geom_tri0 + (g - d->first_global);
}

// Camera + projected positions only (binning pass).
__device__ __forceinline__ void load_positions(const DrawRec &d, uint32_t gt, const FrameParams &fp,
                                               V3 *cam, V3 *proj) {
    const float *v = d.V + 9 * (size_t)gt;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        cam[k] = V3{v[3 * k + 0] + d.P[0], v[3 * k + 1] + d.P[1], v[3 * k + 2] + d.P[2]};
        proj[k] = project_vertex(cam[k], fp);
    }
}

// The vertex attributes one triangle's setup reads (per mode), loaded
// separately so a sweep can fetch the next triangle while it walks this one.
template <int M>
struct TriRaw {
    float v[9], n[9], c[12], uv[6];
};

template <int M>
__device__ __forceinline__ void load_tri(const DrawRec &d, uint32_t gt, TriRaw<M> &r) {
    using TR = ModeTraits<M>;
    const float *v = d.V + 9 * (size_t)gt;
#pragma unroll
    for (int k = 0; k < 9; ++k) r.v[k] = v[k];
#pragma unroll
    for (int k = 0; k < 9; ++k) r.n[k] = 0.0f;
#pragma unroll
    for (int k = 0; k < 12; ++k) r.c[k] = 0.0f;
#pragma unroll
    for (int k = 0; k < 6; ++k) r.uv[k] = 0.0f;
    if (TR::phong || !TR::tex) {  // Phong normals, or Gouraud lighting's normals
        const float *n = d.N + 9 * (size_t)gt;
#pragma unroll
        for (int k = 0; k < 9; ++k) r.n[k] = n[k];
    }
    if (TR::color && d.C) {
        const float *c = d.C + 12 * (size_t)gt;
#pragma unroll
        for (int k = 0; k < 12; ++k) r.c[k] = c[k];
    }
    if (TR::tex) {
        const float *u = d.UV + 6 * (size_t)gt;
#pragma unroll
        for (int k = 0; k < 6; ++k) r.uv[k] = u[k];
    }
}

// FillEdgeTable (projekt.cpp:3882-4121) for ONE binned (front-facing)
// triangle: its three edges {0,1},{1,2},{2,0} and which of them are visible
// (3968, 4066), in edge order, unsorted.
template <int M>
__device__ __forceinline__ void tri_edges(const TriRaw<M> &r, const DrawRec &d, const FrameParams &fp, Edge &e0,
                                          Edge &e1, Edge &e2, bool *vis) {
    using TR = ModeTraits<M>;
    constexpr bool kTex = TR::tex;
    constexpr bool kPhong = TR::phong;
    constexpr bool kColor = TR::color;
    V3 cam[3], proj[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // camera vertex = vertex + Object->P (3898-3903), ProjectVertex
        cam[k] = V3{r.v[3 * k + 0] + d.P[0], r.v[3 * k + 1] + d.P[1], r.v[3 * k + 2] + d.P[2]};
        proj[k] = project_vertex(cam[k], fp);
    }
    // Back-face cull (3926-3943): every triangle reaching a raster kernel
    // passed the identical test in k_bin_count (prk_bin.hip), so it is not
    // repeated per bin entry.

    V3 nrm[3];
    float col[3][4], uv[3][2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        nrm[k] = V3{r.n[3 * k + 0], r.n[3 * k + 1], r.n[3 * k + 2]};
        col[k][0] = r.c[4 * k + 0]; col[k][1] = r.c[4 * k + 1];
        col[k][2] = r.c[4 * k + 2]; col[k][3] = r.c[4 * k + 3];
        uv[k][0] = r.uv[2 * k + 0]; uv[k][1] = r.uv[2 * k + 1];
    }

#pragma unroll
    for (int ei = 0; ei < 3; ++ei) {
        const int i0 = ei, i1 = (ei + 1) % 3;  // Indices {0,1},{1,2},{2,0}
        const bool sw = proj[i0].y > proj[i1].y;  // 3957-3966
        const int mi = sw ? i1 : i0, ma = sw ? i0 : i1;
        V3 MinV = sw ? proj[i1] : proj[i0];
        V3 MaxV = sw ? proj[i0] : proj[i1];
        V3 FirstCam = sw ? cam[i1] : cam[i0];
        V3 SecondCam = sw ? cam[i0] : cam[i1];
        Edge E;
        E.YMax = round_s32(MaxV.y);  // 3988
        float ClippedY = 0.0f, t = 0.0f;
        if (MinV.y < 0.0f) {  // 3993-3997
            ClippedY = -MinV.y;
            t = (-MinV.y) / (MaxV.y - MinV.y);
        }
        {
            float r = (float)round_s32(MinV.y);
            E.YMin = (int32_t)(0.0f > r ? 0.0f : r);  // Maximum(0, .) 3999
        }
        E.X = MinV.x;
        E.Z = FirstCam.z;
        E.U = E.V = E.W = E.UG = E.VG = E.WG = 0.0f;
        E.N0 = E.N1 = E.N2 = E.NG0 = E.NG1 = E.NG2 = 0.0f;
        E.C0 = E.C1 = E.C2 = E.C3 = E.CG0 = E.CG1 = E.CG2 = E.CG3 = 0.0f;
        float FirstUV0 = 0, FirstUV1 = 0, SecondUV0 = 0, SecondUV1 = 0;
        if (kTex) {
            FirstUV0 = uv[mi][0]; FirstUV1 = uv[mi][1];
            SecondUV0 = uv[ma][0]; SecondUV1 = uv[ma][1];
            E.U = FirstUV0 / MinV.z;
            E.V = FirstUV1 / MinV.z;
            E.W = 1.0f / MinV.z;
            float s2 = 1.0f / MaxV.z;  // 4010
            SecondUV0 *= s2; SecondUV1 *= s2;
            float s1 = 1.0f / MinV.z;  // 4012
            FirstUV0 *= s1; FirstUV1 *= s1;
        }
        float MaxC[4] = {0, 0, 0, 0}, MinC[4] = {0, 0, 0, 0};
        float MaxN[3] = {0, 0, 0};
        if (kPhong) {  // 4014-4019
            if (kColor) {
#pragma unroll
                for (int c = 0; c < 4; ++c) { MinC[c] = col[mi][c]; MaxC[c] = col[ma][c]; }
            }
            E.N0 = nrm[mi].x; E.N1 = nrm[mi].y; E.N2 = nrm[mi].z;
            MaxN[0] = nrm[ma].x; MaxN[1] = nrm[ma].y; MaxN[2] = nrm[ma].z;
        } else if (!kTex && (d.flags & DRAW_RAWCOL)) {  // FillEdgeTable(..., Phong = 1): raw colours (4014-4015)
#pragma unroll
            for (int c = 0; c < 4; ++c) { MinC[c] = col[mi][c]; MaxC[c] = col[ma][c]; }
        } else if (!kTex) {  // Gouraud vertex lighting 4020-4063 (untextured only reaches output)
            // Object->Bitmap set: Hadamard(V4(1,1,1,1), .) replaces the vertex
            // colour (4034-4054); 1.0f * x == x, so a white base is exact
            const bool white = (d.flags & DRAW_WHITELIT) != 0;
            float cmi[4], cma[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                cmi[c] = white ? 1.0f : col[mi][c];
                cma[c] = white ? 1.0f : col[ma][c];
            }
            for (uint32_t li = 0; li < fp.light_count; ++li) {
                V3 LP = V3{fp.lp[li][0], fp.lp[li][1], fp.lp[li][2]};
                V3 FVL = nrm_rcp(V3{LP.x - FirstCam.x, LP.y - FirstCam.y, LP.z - FirstCam.z});
                V3 SVL = nrm_rcp(V3{LP.x - SecondCam.x, LP.y - SecondCam.y, LP.z - SecondCam.z});
                if (li == 0) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        MinC[c] = cmi[c] * fp.amb[c];
                        MaxC[c] = cma[c] * fp.amb[c];
                    }
                }
                float FD = clamp01((FVL.x * nrm[mi].x + FVL.y * nrm[mi].y) + FVL.z * nrm[mi].z);
                float SD = clamp01((SVL.x * nrm[ma].x + SVL.y * nrm[ma].y) + SVL.z * nrm[ma].z);
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    MinC[c] = clamp01(MinC[c] + FD * (cmi[c] * fp.li[li][c]));
                    MaxC[c] = clamp01(MaxC[c] + SD * (cma[c] * fp.li[li][c]));
                }
            }
        }
        // Textured, non-Phong: the vertex colour is replaced by the texel in
        // the span (projekt.cpp:445), so the lit colour never reaches output.
        vis[ei] = (MaxV.y > 0) && (MinV.y - MaxV.y != 0);  // 3968, 4066
        float YDiff = (float)E.YMax - (float)E.YMin;
        E.ZG = (SecondCam.z - FirstCam.z) / YDiff;
        E.G = (MaxV.x - MinV.x) / (MaxV.y - MinV.y);
        E.X += ClippedY * E.G;
        E.Z += ClippedY * E.ZG;
        if (kTex) {  // 4078-4089
            E.UG = (SecondUV0 - FirstUV0) / YDiff;
            E.VG = (SecondUV1 - FirstUV1) / YDiff;
            E.U += ClippedY * E.UG;
            E.V += ClippedY * E.VG;
            E.WG = ((1.0f / MaxV.z) - E.W) / YDiff;
            E.W += ClippedY * E.WG;
        }
        if (kColor) {  // 4091, 4095-4101
#pragma unroll
            for (int c = 0; c < 4; ++c) MinC[c] = (1.0f - t) * MinC[c] + t * MaxC[c];
            E.C0 = MinC[0]; E.C1 = MinC[1]; E.C2 = MinC[2]; E.C3 = MinC[3];
            E.CG0 = (MaxC[0] - MinC[0]) / YDiff;
            E.CG1 = (MaxC[1] - MinC[1]) / YDiff;
            E.CG2 = (MaxC[2] - MinC[2]) / YDiff;
            E.CG3 = (MaxC[3] - MinC[3]) / YDiff;
        }
        if (kPhong) {  // 4103-4108
            E.NG0 = (MaxN[0] - E.N0) / YDiff;
            E.NG1 = (MaxN[1] - E.N1) / YDiff;
            E.NG2 = (MaxN[2] - E.N2) / YDiff;
        }
        E.Left = (E.YMin == round_s32(proj[i0].y)) ? 1 : 0;  // 4093
        E.Vtx = mi | (ma << 2);
        if (ei == 0) e0 = E; else if (ei == 1) e1 = E; else e2 = E;
    }
}

// FillEdgeTable for ONE triangle followed by MergeSort (2-72) of its <= 3
// visible edges (the per-triangle AET).  Returns the edge count.
template <int M>
__device__ __forceinline__ int setup_from_raw(const TriRaw<M> &r, const DrawRec &d, const FrameParams &fp,
                                              Edge &s0, Edge &s1, Edge &s2) {
    Edge e0, e1, e2;
    bool vis[3];
    tri_edges<M>(r, d, fp, e0, e1, e2, vis);
    // Compact visible edges in edge order, then MergeSort (projekt.cpp:2-72).
    const int n = (int)vis[0] + (int)vis[1] + (int)vis[2];
    const Edge a0 = sel(vis[0], e0, sel(vis[1], e1, e2));
    const Edge a1 = sel(vis[0] && vis[1], e1, e2);
    const Edge &a2 = e2;
    // n == 2: swap if YMin descending.  n == 3: Half0 = [a0],
    // Half1 = sort2([a1, a2]); the merge takes Half0 only on strict '<'.
    const bool sw12 = a1.YMin > a2.YMin;
    const Edge b1 = sel(sw12, a2, a1), b2 = sel(sw12, a1, a2);
    const bool two_sw = a0.YMin > a1.YMin;
    const bool h0_first = a0.YMin < b1.YMin;   // n == 3: a0 leads
    const bool h0_second = a0.YMin < b2.YMin;  // n == 3, b1 leads: a0 second?
    if (n == 3) {
        s0 = sel(h0_first, a0, b1);
        s1 = sel(h0_first, b1, sel(h0_second, a0, b2));
        s2 = sel(h0_first, b2, sel(h0_second, b2, a0));
    } else {
        s0 = sel(n == 2 && two_sw, a1, a0);
        s1 = sel(two_sw, a0, a1);
        s2 = a2;
    }
    return n;
}

template <int M>
__device__ __forceinline__ int setup_triangle(const DrawRec &d, uint32_t gt, const FrameParams &fp,
                                              Edge &s0, Edge &s1, Edge &s2) {
    TriRaw<M> r;
    load_tri<M>(d, gt, r);
    return setup_from_raw<M>(r, d, fp, s0, s1, s2);
}

// ---- setup records ---------------------------------------------------------
__device__ __forceinline__ void rec_edge_out(const Edge &E, float *f, int32_t &ymin, int32_t &ymax) {
    f[0] = E.X; f[1] = E.G; f[2] = E.Z; f[3] = E.ZG; f[4] = E.W;
    f[5] = E.WG; f[6] = E.U; f[7] = E.UG; f[8] = E.V; f[9] = E.VG;
    ymin = (int32_t)((uint32_t)E.YMin | ((uint32_t)(E.Left != 0) << 31));
    ymax = E.YMax;
}
__device__ __forceinline__ Edge rec_edge_in(const float *f, int32_t ymin, int32_t ymax) {
    Edge E;
    E.X = f[0]; E.G = f[1]; E.Z = f[2]; E.ZG = f[3]; E.W = f[4];
    E.WG = f[5]; E.U = f[6]; E.UG = f[7]; E.V = f[8]; E.VG = f[9];
    E.N0 = E.N1 = E.N2 = E.NG0 = E.NG1 = E.NG2 = 0.0f;
    E.C0 = E.C1 = E.C2 = E.C3 = E.CG0 = E.CG1 = E.CG2 = E.CG3 = 0.0f;
    E.YMin = (int32_t)((uint32_t)ymin & 0x7FFFFFFFu);
    E.Left = (int32_t)((uint32_t)ymin >> 31);
    E.YMax = ymax;
    return E;
}
// The normals of a sorted edge from its triangle's vertex normals n[9]
// (FillEdgeTable 4014-4019, 4103-4108: MinNormal = the Min vertex's normal,
// no top clip; NormalGradient = (MaxNormal - MinNormal) / YDiff).
__device__ __forceinline__ void nrm_edge_from(Edge &E, uint32_t vtx, const float *n) {
    const int mi = (int)(vtx & 3u), ma = (int)((vtx >> 2) & 3u);
    E.N0 = n[3 * mi + 0]; E.N1 = n[3 * mi + 1]; E.N2 = n[3 * mi + 2];
    float g[3] = {n[3 * ma + 0] - E.N0, n[3 * ma + 1] - E.N1, n[3 * ma + 2] - E.N2};
    div_all((float)E.YMax - (float)E.YMin, g);  // / YDiff
    E.NG0 = g[0]; E.NG1 = g[1]; E.NG2 = g[2];
}

// AET edge step (projekt.cpp:3811-3829), only the fields mode M reads
// (normals only when NRM: the visibility sweep never reads them).
template <int M, bool NRM>
__device__ __forceinline__ void step_edge(Edge &E) {
    using TR = ModeTraits<M>;
    E.X += E.G;
    E.Z += E.ZG;
    if (TR::color && NRM) { E.C0 += E.CG0; E.C1 += E.CG1; E.C2 += E.CG2; E.C3 += E.CG3; }
    if (TR::phong && NRM) {
        float x = E.N0 + E.NG0, y = E.N1 + E.NG1, z = E.N2 + E.NG2;
        normalize_rcp(x, y, z);
        E.N0 = x; E.N1 = y; E.N2 = z;
    }
    if (TR::tex) { E.U += E.UG; E.V += E.VG; E.W += E.WG; }
}

// The list-order fields of an edge alone (X, its gradient and the keys of
// insertion/expiry): Walker<M, NRM, EdgeX> replays only the AET order.
struct EdgeX {
    float X, G;
    int32_t YMin, YMax, Left;
};

__device__ __forceinline__ EdgeX edge_x(const Edge &E, float X) { return EdgeX{X, E.G, E.YMin, E.YMax, E.Left}; }

__device__ __forceinline__ EdgeX sel(bool c, const EdgeX &a, const EdgeX &b) {
    return EdgeX{c ? a.X : b.X, c ? a.G : b.G, c ? a.YMin : b.YMin, c ? a.YMax : b.YMax, c ? a.Left : b.Left};
}

template <int M, bool NRM>
__device__ __forceinline__ void step_edge(EdgeX &E) {
    E.X += E.G;
}

// AET insertion order (projekt.cpp:3663-3667).
// (bitwise & / | : the comparisons have no side effects, and short-circuit
// && / || compiled to a branch per term)
__device__ __forceinline__ bool insert_before(const Edge &A, const Edge &B) {
    return (A.X < B.X) | ((A.X == B.X) & ((A.G < B.G) | ((A.G == B.G) & (A.Left < B.Left))));
}

// Per-triangle active edge table of DrawModelOptimized(RenderQueue,...)
// (projekt.cpp:3615-3871, with the P3 head/tail fix; DrawModel's AET,
// 168-598, is the same list logic) as a row-by-row state machine.
//
// The three sorted setup edges stay in fixed registers E0..E2; the list is a
// permutation `ord` (2 bits per list slot, head first) plus a count, so
// insertion, expiry and the crossing swap move only a few integer bits.
// For ONE triangle the two sorted edges with the smallest YMin always share
// it, so all insertions of FirstRow happen in init() and at
// most one edge is still pending afterwards; `anomaly` counts triangles
// violating that (never observed; reported by the host).
template <int M, bool NRM, typename EdgeT = Edge>
struct Walker {
    EdgeT E0, E1, E2;
    uint32_t ord;     // list slot j holds edge (ord >> 2j) & 3
    int cnt;          // list length
    int pend;         // index of the pending edge, or -1
    int32_t FirstRow, MaxY, Row;

    __device__ __forceinline__ int slot(int j) const { return (int)((ord >> (2 * j)) & 3u); }
    __device__ __forceinline__ EdgeT get(int k) const { return sel(k == 0, E0, sel(k == 1, E1, E2)); }
    // (value selects: a conditional over lvalues would become a pointer select
    // and push the walker to scratch memory)
    template <typename T>
    __device__ __forceinline__ static T pick(int k, T a, T b, T c) { return k == 0 ? a : (k == 1 ? b : c); }
    __device__ __forceinline__ float X(int k) const { return pick<float>(k, E0.X, E1.X, E2.X); }
    __device__ __forceinline__ float G(int k) const { return pick<float>(k, E0.G, E1.G, E2.G); }
    __device__ __forceinline__ int32_t Lf(int k) const { return pick<int32_t>(k, E0.Left, E1.Left, E2.Left); }
    __device__ __forceinline__ int32_t YMax(int k) const { return pick<int32_t>(k, E0.YMax, E1.YMax, E2.YMax); }

    // AET insertion order (projekt.cpp:3663-3667) of edge a before edge b.
    __device__ __forceinline__ bool before(int a, int b) const {
        const float xa = X(a), xb = X(b), ga = G(a), gb = G(b);
        return (xa < xb) | ((xa == xb) & ((ga < gb) | ((ga == gb) & (Lf(a) < Lf(b)))));
    }

    __device__ __forceinline__ void insert(int k) {  // 3654-3713
        int pos = cnt;
        if (cnt > 1 && before(k, slot(1))) pos = 1;
        if (cnt > 0 && before(k, slot(0))) pos = 0;
        const uint32_t lowmask = (1u << (2 * pos)) - 1u;
        ord = (ord & lowmask) | ((uint32_t)k << (2 * pos)) | ((ord & ~lowmask) << 2);
        ord &= 0x3Fu;
        ++cnt;
    }

    __device__ __forceinline__ void init(int n, const EdgeT &s0, const EdgeT &s1, const EdgeT &s2, int32_t H,
                                         int32_t row_end, uint32_t &anomaly) {
        E0 = s0; E1 = s1; E2 = s2;
        FirstRow = s0.YMin;
        int32_t MaxRow = s0.YMax;
        if (n > 1 && MaxRow < s1.YMax) MaxRow = s1.YMax;
        if (n > 2 && MaxRow < s2.YMax) MaxRow = s2.YMax;
        MaxY = min(min(MaxRow, H), row_end);
        Row = FirstRow;
        ord = 0u;
        cnt = 1;
        pend = -1;
        if (n > 1) {
            if (s1.YMin == FirstRow) insert(1);
            else ++anomaly;
        }
        if (n > 2) {
            if (s2.YMin == FirstRow) insert(2);
            else pend = 2;
        }
    }

    // The same state from a setup record: the insertions of FirstRow were
    // replayed once per triangle by the binning pass (head word of TriRec).
    __device__ __forceinline__ void init_rec(int n, const EdgeT &s0, const EdgeT &s1, const EdgeT &s2, int32_t H,
                                             int32_t row_end, uint32_t head) {
        E0 = s0; E1 = s1; E2 = s2;
        FirstRow = s0.YMin;
        int32_t MaxRow = s0.YMax;
        if (n > 1 && MaxRow < s1.YMax) MaxRow = s1.YMax;
        if (n > 2 && MaxRow < s2.YMax) MaxRow = s2.YMax;
        MaxY = min(min(MaxRow, H), row_end);
        Row = FirstRow;
        ord = (head >> 4) & 0xFFu;
        cnt = (int)((head >> 12) & 0xFu);
        pend = (int)((head >> 16) & 0xFu) - 1;
    }

    // Insertion + expiry of this->Row; true when a pair is emitted: the left
    // edge is slot(0), the right edge slot(1).
    __device__ __forceinline__ bool begin_row() {
        if (pend >= 0 && E2.YMin == Row) {
            insert(2);
            pend = -1;
        }
        // Expiry (3715-3749): drop every entry with YMax <= Row, keep order.
        uint32_t o = 0u;
        int c = 0;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int k = slot(j);
            if (j < cnt && !(YMax(k) <= Row)) {
                o |= (uint32_t)k << (2 * c);
                ++c;
            }
        }
        ord = o;
        cnt = c;
        // Pairing (3751-3869): one pair; a third entry is left unpaired and
        // unstepped, as in the reference.
        return cnt >= 2;
    }

    // Edge step of the emitted pair (3811-3829) and the crossing swap
    // (3831-3841 + P3), then move to the next row.
    __device__ __forceinline__ void end_row(bool paired) {
        if (paired) {
            const int a = slot(0), b = slot(1);
            EdgeT t0 = E0, t1 = E1, t2 = E2;
            step_edge<M, NRM>(t0);
            step_edge<M, NRM>(t1);
            step_edge<M, NRM>(t2);
            E0 = sel(a == 0 || b == 0, t0, E0);
            E1 = sel(a == 1 || b == 1, t1, E1);
            E2 = sel(a == 2 || b == 2, t2, E2);
            if (X(a) > X(b)) ord = (ord & ~0xFu) | ((uint32_t)a << 2) | (uint32_t)b;
        }
        ++Row;
    }

    // Rows [Row, min(ystart, MaxY)) above the tile, straight after init(n, ...):
    // the same edge state and list order as begin_row/end_row row by row, at
    // a few adds per edge and row.  Within one triangle the active set of a
    // row follows from the edges' [YMin, YMax) alone; when exactly two edges
    // are active on every replayed row, each edge is stepped on every row of
    // its interval and the DDAs run independently.  The order entering row
    // `stop` is then the strict X order of the last pair (the crossing swap,
    // 3831-3841); an X tie (or NaN) leaves the order to history, which is
    // replayed on X alone (returns 1).  Returns -1, changing nothing, when the
    // rows are irregular (a row with fewer or more than two active edges): the
    // caller then replays row by row.  0: replayed by the edge DDAs alone.
    __device__ __forceinline__ int fast_replay(int32_t ystart, int n) {
        if (MaxY <= ystart) {  // the triangle ends above the tile: nothing to draw
            Row = max(Row, MaxY);
            return 0;
        }
        const int32_t stop = ystart;
        if (Row >= stop) return 0;
#if defined(PRK_DIAG) && (PRK_DIAG & 32)
        Row = stop;  // diagnostic builds only: no replay (wrong output, timing ablation)
        return 0;
#endif
        if (n < 2 || E1.YMin != FirstRow || cnt < 2 || Row != FirstRow) return -1;
        const int32_t h0 = min(E0.YMax, stop), h1 = min(E1.YMax, stop);
        const int32_t i2 = n > 2 ? E2.YMin : stop, h2 = n > 2 ? min(E2.YMax, stop) : stop;
        const int32_t l0 = max(0, h0 - FirstRow), l1 = max(0, h1 - FirstRow), l2 = max(0, h2 - i2);
        const bool three = n > 2 && i2 < min(min(h0, h1), h2);
        if (three || l0 + l1 + l2 != 2 * (stop - FirstRow)) return -1;
        const float ox0 = E0.X, ox1 = E1.X, ox2 = E2.X;
#pragma unroll 4
        for (int32_t k = 0; k < l0; ++k) step_edge<M, NRM>(E0);
#pragma unroll 4
        for (int32_t k = 0; k < l1; ++k) step_edge<M, NRM>(E1);
#pragma unroll 4
        for (int32_t k = 0; k < l2; ++k) step_edge<M, NRM>(E2);
        // The pair of row stop-1 (exactly two of these hold).
        const bool act0 = E0.YMax >= stop, act1 = E1.YMax >= stop;
        const int a = act0 ? 0 : 1, b = (act0 && act1) ? 1 : 2;
        const float xa = X(a), xb = X(b);
        int slow = 0;
        if (xa < xb) ord = (uint32_t)a | ((uint32_t)b << 2);
        else if (xa > xb) ord = (uint32_t)b | ((uint32_t)a << 2);
        else {
            Walker<M, NRM, EdgeX> w;
            uint32_t unused = 0;
            w.init(n, edge_x(E0, ox0), edge_x(E1, ox1), edge_x(E2, ox2), 0x7fffffff, MaxY, unused);
            w.MaxY = MaxY;
            while (w.Row < stop) w.end_row(w.begin_row());
            ord = w.ord;
            slow = 1;
        }
        cnt = 2;
        pend = (n > 2 && i2 >= stop) ? 2 : -1;
        Row = stop;
        return slow;
    }
};

// The same active edge table with the list held physically: S0, S1, S2 are
// list slots 0..2 (a pending third edge waits in S2).  The emitted pair is
// always (S0, S1), so the per-row edge step touches two edges and needs no
// selects; edges move only on the rare rows of an insertion, an expiry or a
// crossing swap.  Built from a Walker after its setup / fast replay.
template <int M, bool NRM>
struct RowWalker {
    Edge S0, S1, S2;
    int cnt;
    bool pend;
    int32_t MaxY, Row;

    __device__ __forceinline__ void from(const Walker<M, NRM> &w) {
        S0 = w.get(w.slot(0));
        S1 = w.get(w.slot(1));
        S2 = w.pend >= 0 ? w.E2 : w.get(w.slot(2));
        cnt = w.cnt;
        pend = w.pend >= 0;
        MaxY = w.MaxY;
        Row = w.Row;
    }

    // Insertion + expiry of this->Row; true when the pair (S0, S1) is emitted.
    // (Edges move by value selects: a conditional struct copy would become a
    // pointer select and push the walker to scratch memory.)
    __device__ __forceinline__ bool begin_row() {
        if (pend && S2.YMin == Row) {  // insertion (3654-3713)
            const bool b0 = cnt > 0 && insert_before(S2, S0);
            const bool b1 = cnt > 1 && insert_before(S2, S1);
            // b0: [S2 S0 S1]  b1: [S0 S2 S1]  else: S2 appended at slot cnt
            const Edge n0 = sel(b0 || cnt == 0, S2, S0);
            const Edge n1 = sel(b0, S0, sel(b1 || cnt == 1, S2, S1));
            const Edge n2 = sel(b0 || b1, S1, S2);
            S0 = n0; S1 = n1; S2 = n2;
            ++cnt;
            pend = false;
        }
        // Expiry (3715-3749): drop every entry with YMax <= Row, keep order.
        // (While an edge is pending cnt <= 2, so S2 is never read as a slot.)
        const bool k0 = cnt > 0 && !(S0.YMax <= Row);
        const bool k1 = cnt > 1 && !(S1.YMax <= Row);
        const bool k2 = cnt > 2 && !(S2.YMax <= Row);
        if ((!k0 && (k1 || k2)) || (!k1 && k2)) {  // a kept entry moves down
            const Edge n0 = sel(k0, S0, sel(k1, S1, S2));
            const Edge n1 = sel(k0 && k1, S1, S2);
            S0 = n0; S1 = n1;
        }
        cnt = (int)k0 + (int)k1 + (int)k2;
        // Pairing (3751-3869): one pair; a third entry stays unpaired.
        return cnt >= 2;
    }

    // Edge step of the pair (3811-3829) and the crossing swap (3831-3841 + P3).
    __device__ __forceinline__ void end_row(bool paired) {
        if (paired) {
            step_edge<M, NRM>(S0);
            step_edge<M, NRM>(S1);
            const bool sw = S0.X > S1.X;
            if (sw) {
                const Edge a = sel(sw, S1, S0), b = sel(sw, S0, S1);
                S0 = a; S1 = b;
            }
        }
        ++Row;
    }
};

// The chunked walk of large objects (prk_spans.hip k_pr_*): its pass-wide
// buffers and sizes, set by flush_spans (prk_api.hip).
struct PrWalkArgs {
    const void *objs;           // ObjDesc[]
    const void *pro;            // PrObj[npr]
    uint32_t npr;               // objects
    uint32_t warmup;            // chunks start one chunk early (0: from their own first row)
    uint32_t nchunks;           // their chunks
    uint32_t max_edges;         // most edges of one object
    const uint32_t *escan, *total0p;
    const void *work;           // the walk's working copy (ObjEdge[])
    void *prrow;                // PrRow[npr]
    uint32_t *cnt, *eoff, *fge; // per row: rows + 1 per object
    uint32_t *ccur;             // per chunk: its first row's entries
    void *key;                  // float4 per entry (chunk j of an object: ent_off + j * most)
    void *est, *sst, *eend;     // ObjEdge per entry: arrival order / canonical list / a walk's end list
    uint32_t *eend_m, *match;   // per chunk
    uint32_t *sidx, *s_m;       // per entry / per chunk: a chunk's list at its first row (edge indices)
    uint32_t *prstat;           // per object of the pass
    const unsigned long long *soff;
    void *raw, *pos;            // PairRaw / SpanPos per span slot
    uint32_t *span_tri, *err;
};
}  // namespace prk
