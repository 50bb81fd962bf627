/*
 * prk_oracle.c — CPU restatement of the reference rasterizer hot path.
 *
 *   TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 *   bench.py's cpu_baseline leg may load this library, and only as the
 *   checker / the timed CPU baseline.  The product (libprk_hip.so) never
 *   links, loads or calls it.
 *
 *   PARITY UNPINNED: the reference (MacSpain/cpu-renderer, /root/reference)
 *   has no tests, no fixtures and no golden images, and it cannot be built
 *   here without writing stand-ins for its absent platform/math headers
 *   (v3, loaded_bitmap, game_render_commands, RoundR32ToS32, ...), which this
 *   round's rules forbid.  This file is a restatement written from reading
 *   projekt.cpp; every function cites the lines it follows.  SURVEY.md
 *   records that the same semantic description (its Appendix A/B) matched a
 *   shimmed build of the reference bit-exactly during the survey; that check
 *   is not reproducible under this round's rules, so it is cited, not relied
 *   on.  Pins for the absent helpers follow SURVEY §8(c)/App. C/D:
 *     RoundR32ToS32(x) = (s32)roundf(x)     (half away from zero)
 *     RoundR32ToU32(x) = (u32)roundf(x)
 *     Normalize(a)     = (1/sqrtf(Inner(a,a))) * a
 *     Inner(a,b)       = (a.x*b.x + a.y*b.y) + a.z*b.z
 *     Clamp01(x)       = x<0 ? 0 : (x>1 ? 1 : x)
 *   Harness fixes where the reference crashes:
 *     P1 MergeSort(Count==0) returns; DrawModel* with 0 edges draws nothing.
 *     P2/P4 texel byte offsets outside [0, Pitch*(Th+1)-4] read offset 0.
 *     P3 the AET first-pair swap updates ListHead / ListTail.
 *     An AET that empties mid-walk skips the row instead of dereferencing NULL.
 *   x86 conversion semantics are restated explicitly (cvttss2si returns
 *   INT_MIN for NaN / out of range; MINPS/MAXPS return the 2nd operand on
 *   NaN) so results do not depend on this compiler's UB choices.
 *
 *   Build: see oracle/Makefile (gcc -O2 -ffp-contract=off, no -ffast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <float.h>

#include "../include/prk.h"

/* ------------------------------------------------------------------ */
/* Helpers: the absent math header, pinned.    */
/* ------------------------------------------------------------------ */

typedef struct { float x, y, z; } or_v3;

static inline int32_t or_cvtt_s32(float f)
{
    /* x86 cvttss2si: truncation; NaN / out of range -> INT_MIN. */
    if (f >= -2147483648.0f && f < 2147483648.0f) return (int32_t)f;
    return INT32_MIN;
}
static inline int32_t or_round_s32(float f) { return or_cvtt_s32(roundf(f)); }
static inline uint32_t or_round_u32(float f)
{
    /* x86-64 gcc (u32)float: cvttss2si into a 64-bit register, keep low 32. */
    float r = roundf(f);
    if (r >= -9223372036854775808.0f && r < 9223372036854775808.0f)
        return (uint32_t)(uint64_t)(int64_t)r;
    return 0u;
}
static inline int32_t or_cvt_rne_s32(float f)
{
    /* _mm256_cvtps_epi32 under the default MXCSR (round to nearest even). */
    if (f >= -2147483648.0f && f < 2147483648.0f) return (int32_t)nearbyintf(f);
    return INT32_MIN;
}
static inline float or_maxps(float a, float b) { return a > b ? a : b; } /* MAXPS */
static inline float or_minps(float a, float b) { return a < b ? a : b; } /* MINPS */
static inline float or_clamp01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }

static inline or_v3 or_v3make(float x, float y, float z) { or_v3 r = {x, y, z}; return r; }
static inline or_v3 or_sub(or_v3 a, or_v3 b) { return or_v3make(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline or_v3 or_add(or_v3 a, or_v3 b) { return or_v3make(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline or_v3 or_scale(float s, or_v3 a) { return or_v3make(s * a.x, s * a.y, s * a.z); }
static inline float or_inner(or_v3 a, or_v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline or_v3 or_cross(or_v3 a, or_v3 b)
{
    return or_v3make(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline or_v3 or_normalize(or_v3 a) { return or_scale(1.0f / sqrtf(or_inner(a, a)), a); }

/* NormalizeVector_8x, one lane (projekt.cpp:603-620): division form. */
static inline void or_normalize_div(float *x, float *y, float *z)
{
    float len = sqrtf((*x * *x + *y * *y) + *z * *z);
    *x = *x / len;
    *y = *y / len;
    *z = *z / len;
}

/* _mm_mullo_epi16 / _mm_mulhi_epi16 pitch multiply (projekt.cpp:1916-1920). */
static inline int32_t or_mul16_trick(int32_t y, int32_t p)
{
    uint32_t ylo = (uint32_t)y & 0xFFFFu, yhi = (uint32_t)y >> 16;
    uint32_t plo = (uint32_t)p & 0xFFFFu, phi = (uint32_t)p >> 16;
    uint32_t lo = (ylo * plo) & 0xFFFFu;
    uint32_t hi_mullo = (yhi * phi) & 0xFFFFu;
    int32_t sprod = (int32_t)(int16_t)ylo * (int32_t)(int16_t)plo;
    uint32_t hi_mulhi = ((uint32_t)sprod >> 16) & 0xFFFFu;
    return (int32_t)(lo | ((hi_mullo | hi_mulhi) << 16));
}

/* ------------------------------------------------------------------ */
/* Data model (projekt.h:17-37).                                       */
/* ------------------------------------------------------------------ */

typedef struct or_edge {
    int32_t YMax;
    float XMin, ZMin, OneOverZMin, Gradient, ZGradient, OneOverZGradient;
    int32_t YMin;
    float UMin, VMin, UGradient, VGradient;
    int32_t Left;
    float MinColor[4], ColorGradient[4];
    float MinNormal[3], NormalGradient[3];
    struct or_edge *Next;
} or_edge;

typedef struct or_ctx {
    const prk_transform *T;
    const prk_light_data *Lights;
    const prk_bitmap *Bitmap;  /* NULL: untextured */
    uint32_t *Color;
    int32_t Pitch;             /* bytes */
    float *Z;
    int32_t Width, Height;
    int32_t *Winners;          /* optional */
    int32_t TriIndex;          /* winner id for the current object */
    int32_t RowLo, RowHi;      /* band filter [RowLo, RowHi) */
    int32_t BandH, BandMod, BandRem; /* interleaved bands: draw row r iff (r/BandH)%BandMod==BandRem */
    int Phong;
    int Filter;                /* PRK_FILTER_*: texture sampling of the AVX span */
    int St;                    /* the single-thread overload DrawModelOptimized(Buffer,...) */
    uint64_t Spans, SpanPixels, Writes;
} or_ctx;

/* Does this call draw frame row r?  (band filter used by the threaded driver) */
static inline int or_owns(const or_ctx *X_, int32_t r)
{
    return r >= X_->RowLo && r < X_->RowHi && (r / X_->BandH) % X_->BandMod == X_->BandRem;
}

/* ------------------------------------------------------------------ */
/* ProjectVertex (projekt.cpp:74-93).                                  */
/* ------------------------------------------------------------------ */
static or_v3 or_project_vertex(or_v3 cam, const prk_transform *T)
{
    or_v3 r = {0.0f, 0.0f, 0.0f};
    float d = T->DistanceAboveTarget - cam.z;
    if (d > 0.2f) {
        float k = (1.0f / d) * T->FocalLength;
        float px = k * cam.x, py = k * cam.y;
        r.x = T->ScreenCenter[0] + T->MetersToPixels * px;
        r.y = T->ScreenCenter[1] + T->MetersToPixels * py;
        r.z = d + T->MetersToPixels * 0.0f;
    }
    return r;
}

/* ------------------------------------------------------------------ */
/* MergeSort on YMin (projekt.cpp:2-72), with P1 (Count == 0).         */
/* ------------------------------------------------------------------ */
static void or_merge_sort(uint32_t Count, or_edge *First, or_edge *Temp)
{
    if (Count == 0 || Count == 1) return;
    if (Count == 2) {
        if (First[0].YMin > First[1].YMin) {
            or_edge t = First[0];
            First[0] = First[1];
            First[1] = t;
        }
        return;
    }
    uint32_t Half0 = Count / 2, Half1 = Count - Half0;
    or_edge *InHalf1 = First + Half0, *End = First + Count;
    or_merge_sort(Half0, First, Temp);
    or_merge_sort(Half1, InHalf1, Temp);
    or_edge *R0 = First, *R1 = InHalf1, *Out = Temp;
    for (uint32_t i = 0; i < Count; ++i) {
        if (R0 == InHalf1) *Out++ = *R1++;
        else if (R1 == End) *Out++ = *R0++;
        else if (R0->YMin < R1->YMin) *Out++ = *R0++;
        else *Out++ = *R1++;
    }
    for (uint32_t i = 0; i < Count; ++i) First[i] = Temp[i];
}

/* ------------------------------------------------------------------ */
/* FillEdgeTable (projekt.cpp:3882-4121) for `tri_count` triangles.    */
/* Writes at most 3*tri_count edges; returns the visible edge count.   */
/* ------------------------------------------------------------------ */
static uint32_t or_fill_edge_table(const float *V, const float *C, const float *N,
                                   const float *UV, uint32_t tri0, uint32_t tri_count,
                                   const float P[3], int Textured, int Phong,
                                   const prk_transform *T, const prk_light_data *Lights,
                                   or_edge *Edges, or_edge *Sort)
{
    const or_v3 Eye = {0.0f, 0.0f, -1.0f};
    uint32_t Visible = 0;
    static const uint32_t Indices[3][2] = {{0, 1}, {1, 2}, {2, 0}};
    for (uint32_t t = tri0; t < tri0 + tri_count; ++t) {
        or_v3 Cam[3], Proj[3], Nrm[3];
        float Col[3][4], Uv[3][2];
        for (int k = 0; k < 3; ++k) {
            const float *v = V + 9 * (size_t)t + 3 * k;
            Cam[k] = or_v3make(v[0] + P[0], v[1] + P[1], v[2] + P[2]);
        }
        for (int k = 0; k < 3; ++k) Proj[k] = or_project_vertex(Cam[k], T);
        for (int k = 0; k < 3; ++k) {
            for (int c = 0; c < 4; ++c) Col[k][c] = C ? C[12 * (size_t)t + 4 * k + c] : 0.0f;
            for (int c = 0; c < 2; ++c) Uv[k][c] = UV ? UV[6 * (size_t)t + 2 * k + c] : 0.0f;
            const float *n = N ? N + 9 * (size_t)t + 3 * k : NULL;
            Nrm[k] = n ? or_v3make(n[0], n[1], n[2]) : or_v3make(0, 0, 0);
        }
        or_v3 FirstVN = or_normalize(or_sub(Proj[1], Proj[0]));
        or_v3 SecondVN = or_normalize(or_sub(Proj[2], Proj[0]));
        if (!(or_inner(Eye, or_cross(FirstVN, SecondVN)) > 0.0f)) continue; /* 3926-3943 */

        for (uint32_t e = 0; e < 3; ++e) {
            uint32_t MinI = Indices[e][0], MaxI = Indices[e][1];
            or_v3 MinV = Proj[MinI], MaxV = Proj[MaxI];
            if (MinV.y > MaxV.y) { /* 3957-3966 */
                or_v3 tv = MinV; MinV = MaxV; MaxV = tv;
                uint32_t ti = MinI; MinI = MaxI; MaxI = ti;
            }
            if (!(MaxV.y > 0)) continue; /* 3968 */
            or_edge *E = Edges + Visible;
            memset(E, 0, sizeof(*E)); /* pin: uninitialised fields read as 0 */
            or_v3 FirstCam = Cam[MinI], SecondCam = Cam[MaxI];
            or_v3 FirstN = Nrm[MinI], SecondN = Nrm[MaxI];
            float FirstC[4], SecondC[4], MaxColor[4] = {0, 0, 0, 0}, MaxNormal[3] = {0, 0, 0};
            memcpy(FirstC, Col[MinI], sizeof FirstC);
            memcpy(SecondC, Col[MaxI], sizeof SecondC);
            float FirstUV[2] = {Uv[MinI][0], Uv[MinI][1]};
            float SecondUV[2] = {Uv[MaxI][0], Uv[MaxI][1]};

            E->YMax = or_round_s32(MaxV.y); /* 3988 */
            float ClippedY = 0.0f, t_ = 0.0f;
            if (MinV.y < 0.0f) { /* 3993-3997 */
                ClippedY = -MinV.y;
                t_ = (-MinV.y) / (MaxV.y - MinV.y);
            }
            {
                float r = (float)or_round_s32(MinV.y);
                E->YMin = (int32_t)(0.0f > r ? 0.0f : r); /* Maximum(0, .) 3999 */
            }
            E->XMin = MinV.x;
            E->ZMin = FirstCam.z;
            E->UMin = FirstUV[0] / MinV.z;
            E->VMin = FirstUV[1] / MinV.z;
            E->OneOverZMin = 1.0f / MinV.z;
            { float s = 1.0f / MaxV.z; SecondUV[0] *= s; SecondUV[1] *= s; } /* 4010 */
            { float s = 1.0f / MinV.z; FirstUV[0] *= s; FirstUV[1] *= s; }   /* 4012 */

            if (Phong) { /* 4014-4019 */
                memcpy(E->MinColor, FirstC, sizeof FirstC);
                memcpy(MaxColor, SecondC, sizeof SecondC);
                E->MinNormal[0] = FirstN.x; E->MinNormal[1] = FirstN.y; E->MinNormal[2] = FirstN.z;
                MaxNormal[0] = SecondN.x; MaxNormal[1] = SecondN.y; MaxNormal[2] = SecondN.z;
            } else { /* Gouraud vertex lighting 4020-4063 */
                for (uint32_t li = 0; li < Lights->LightCount; ++li) {
                    const prk_light_info *L = &Lights->Lights[li];
                    or_v3 LP = or_v3make(L->P[0], L->P[1], L->P[2]);
                    or_v3 FirstVL = or_normalize(or_sub(LP, FirstCam));
                    or_v3 SecondVL = or_normalize(or_sub(LP, SecondCam));
                    if (li == 0) {
                        for (int c = 0; c < 4; ++c) {
                            if (Textured) {
                                E->MinColor[c] = 1.0f * Lights->AmbientIntensity[c];
                                MaxColor[c] = 1.0f * Lights->AmbientIntensity[c];
                            } else {
                                E->MinColor[c] = FirstC[c] * Lights->AmbientIntensity[c];
                                MaxColor[c] = SecondC[c] * Lights->AmbientIntensity[c];
                            }
                        }
                    }
                    float FirstDot = or_clamp01(or_inner(FirstVL, FirstN));
                    float SecondDot = or_clamp01(or_inner(SecondVL, SecondN));
                    for (int c = 0; c < 4; ++c) {
                        float a = Textured ? 1.0f * L->Intensity[c] : FirstC[c] * L->Intensity[c];
                        float b = Textured ? 1.0f * L->Intensity[c] : SecondC[c] * L->Intensity[c];
                        E->MinColor[c] = or_clamp01(E->MinColor[c] + FirstDot * a);
                        MaxColor[c] = or_clamp01(MaxColor[c] + SecondDot * b);
                    }
                }
            }

            if (MinV.y - MaxV.y != 0) { /* 4066 */
                ++Visible;
                float YDiff = (float)E->YMax - (float)E->YMin;
                E->ZGradient = (SecondCam.z - FirstCam.z) / YDiff;
                E->Gradient = (MaxV.x - MinV.x) / (MaxV.y - MinV.y);
                E->XMin += ClippedY * E->Gradient;
                E->ZMin += ClippedY * E->ZGradient;
                if (Textured) { /* 4078-4089 */
                    E->UGradient = (SecondUV[0] - FirstUV[0]) / YDiff;
                    E->VGradient = (SecondUV[1] - FirstUV[1]) / YDiff;
                    E->UMin += ClippedY * E->UGradient;
                    E->VMin += ClippedY * E->VGradient;
                    E->OneOverZGradient = ((1.0f / MaxV.z) - E->OneOverZMin) / YDiff;
                    E->OneOverZMin += ClippedY * E->OneOverZGradient;
                }
                for (int c = 0; c < 4; ++c) /* 4091 */
                    E->MinColor[c] = (1.0f - t_) * E->MinColor[c] + t_ * MaxColor[c];
                E->Left = (E->YMin == or_round_s32(Proj[Indices[e][0]].y)) ? 1 : 0; /* 4093 */
                E->Next = NULL;
                for (int c = 0; c < 4; ++c)
                    E->ColorGradient[c] = (MaxColor[c] - E->MinColor[c]) / YDiff;
                for (int c = 0; c < 3; ++c)
                    E->NormalGradient[c] = (MaxNormal[c] - E->MinNormal[c]) / YDiff;
            }
        }
    }
    or_merge_sort(Visible, Edges, Sort); /* 4117 */
    return Visible;
}

/* ------------------------------------------------------------------ */
/* Texel fetch with the P2/P4 clamp (projekt.cpp:1936-1967, 436-440).  */
/* ------------------------------------------------------------------ */
static inline uint32_t or_texel(const prk_bitmap *B, int32_t off)
{
    int64_t limit = (int64_t)B->Pitch * (B->Height + 1) - 4;
    if (off < 0 || (int64_t)off > limit) off = 0;
    uint32_t t;
    memcpy(&t, (const uint8_t *)B->Memory + off, 4);
    return t;
}

/* ------------------------------------------------------------------ */
/* Bilinear texture sampling — an EXTENSION of this build (BASELINE    */
/* config 4 asks for it; the reference samples nearest texels only,    */
/* projekt.cpp:1881-2032), so it has no reference to match: this is    */
/* its definition, restated op for op by the GPU kernel.  Texel        */
/* centres at +0.5, clamp to the edge, fp32, no FMA contraction.        */
/* ------------------------------------------------------------------ */
static inline float or_u8(uint32_t t, int sh) { return (float)((t >> sh) & 0xFF) / 255.0f; }

static void or_bilinear(const prk_bitmap *B, float FU, float FV, float *CA, float *CR, float *CG, float *CB)
{
    const float x = (float)B->Width * FU - 0.5f, y = (float)B->Height * FV - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    const float ax = x - fx, ay = y - fy;
    int32_t x0 = (int32_t)fx, y0 = (int32_t)fy, x1 = x0 + 1, y1 = y0 + 1;
    const int32_t wm = B->Width - 1, hm = B->Height - 1;
    x0 = x0 < 0 ? 0 : (x0 > wm ? wm : x0); x1 = x1 < 0 ? 0 : (x1 > wm ? wm : x1);
    y0 = y0 < 0 ? 0 : (y0 > hm ? hm : y0); y1 = y1 < 0 ? 0 : (y1 > hm ? hm : y1);
    const uint8_t *m = (const uint8_t *)B->Memory;
    uint32_t t00, t10, t01, t11;
    memcpy(&t00, m + (size_t)y0 * B->Pitch + 4 * (size_t)x0, 4);
    memcpy(&t10, m + (size_t)y0 * B->Pitch + 4 * (size_t)x1, 4);
    memcpy(&t01, m + (size_t)y1 * B->Pitch + 4 * (size_t)x0, 4);
    memcpy(&t11, m + (size_t)y1 * B->Pitch + 4 * (size_t)x1, 4);
    const float bx = 1.0f - ax, by = 1.0f - ay;
    float out[4];
    const int sh[4] = {24, 16, 8, 0}; /* A R G B */
    for (int c = 0; c < 4; ++c) {
        const float top = bx * or_u8(t00, sh[c]) + ax * or_u8(t10, sh[c]);
        const float bot = bx * or_u8(t01, sh[c]) + ax * or_u8(t11, sh[c]);
        out[c] = by * top + ay * bot;
    }
    *CA = out[0]; *CR = out[1]; *CG = out[2]; *CB = out[3];
}

/* ------------------------------------------------------------------ */
/* FillLineOptimized (projekt.cpp:1492-2320), one lane at a time.      */
/* The non-Phong branch (2285-2316) is out of scope (prk rejects it).  */
/* X_->St: the span body of the single-thread overload                */
/* DrawModelOptimized(Buffer,...) (2350-3358), identical but for the   */
/* left-clip XOffset = -XOffset (2508, i.e. -0.0f) and the GE_OQ z-test */
/* (predicate 29, 3205); its unlocked aligned stores (3235-3236) store  */
/* the same values.                                                     */
/* ------------------------------------------------------------------ */
static void or_fill_line_optimized(or_ctx *X_, const or_edge *L, const or_edge *R, int32_t Row)
{
    if (!or_owns(X_, Row)) return;
    const prk_bitmap *Bm = X_->Bitmap;
    const prk_transform *T = X_->T;
    const int32_t W = X_->Width;
    float XOffset = 0.0f;
    if (Row < 0) return;

    float LeftX = L->XMin; /* 1545-1565 */
    if (LeftX < 0) { XOffset = X_->St ? -XOffset /* 2508 */ : -L->XMin; LeftX = 0; }
    else if (LeftX >= W) LeftX = (float)W - 1;
    float RightX = R->XMin;
    if (RightX < 0) RightX = 0;
    else if (RightX >= W) RightX = (float)W - 1;
    if (LeftX != LeftX || RightX != RightX) return; /* pin: NaN edge X draws nothing */

    int32_t CLP = or_round_s32(L->XMin), CRP = or_round_s32(R->XMin); /* 1568-1570 */
    int32_t XDiff = (int32_t)((uint32_t)CRP - (uint32_t)CLP);
    LeftX = (float)or_round_s32(LeftX); /* 1588-1592 */
    RightX = (float)or_round_s32(RightX);
    int32_t MinX = (int32_t)LeftX, MaxX = (int32_t)RightX;

    int Start[8], End[8], Clip[8];
    for (int i = 0; i < 8; ++i) Start[i] = End[i] = 1;
    if (MinX & 7) { /* 1594-1609 */
        for (int i = 0; i < 8; ++i) Start[i] = i >= (MinX & 7);
        LeftX = (float)(MinX & ~7);
        XOffset -= (float)(MinX & 7) * 1.0f;
    }
    if (MaxX & 7) { /* 1611-1624 */
        for (int i = 0; i < 8; ++i) End[i] = i < (MaxX & 7);
        RightX = (float)((MaxX & ~7) + 8);
    }
    if ((LeftX + 8) >= RightX) /* 1627-1664 */
        for (int i = 0; i < 8; ++i) Start[i] = Start[i] & End[i];

    if (MaxX > MinX) X_->SpanPixels += (uint64_t)(MaxX - MinX);
    X_->Spans++;

    /* Increments and lane init (1666-1835). */
    float fXD = (float)XDiff;
    float IncW = 0, IncU = 0, IncV = 0, IncN[3] = {0, 0, 0}, IncZ = 0;
    if (XDiff != 0) {
        IncW = (R->OneOverZMin - L->OneOverZMin) / fXD;
        IncU = (R->UMin - L->UMin) / fXD;
        IncV = (R->VMin - L->VMin) / fXD;
        for (int c = 0; c < 3; ++c) IncN[c] = (R->MinNormal[c] - L->MinNormal[c]) / fXD;
        IncZ = (R->ZMin - L->ZMin) / fXD;
    }
    float Wl[8], Ul[8], Vl[8], Nx[8], Ny[8], Nz[8], Zl[8];
    for (int i = 0; i < 8; ++i) {
        float o = XOffset + (float)i;
        Wl[i] = L->OneOverZMin + o * IncW;
        Ul[i] = L->UMin + o * IncU;
        Vl[i] = L->VMin + o * IncV;
        Nx[i] = L->MinNormal[0] + o * IncN[0];
        Ny[i] = L->MinNormal[1] + o * IncN[1];
        Nz[i] = L->MinNormal[2] + o * IncN[2];
        or_normalize_div(&Nx[i], &Ny[i], &Nz[i]); /* 1754 */
        Zl[i] = L->ZMin + o * IncZ;
    }
    /* Colour lanes (1777-1811) are dead: the texel overwrites them (2029-2032). */
    const float IncW8 = IncW * 8.0f, IncU8 = IncU * 8.0f, IncV8 = IncV * 8.0f;
    const float IncN8[3] = {IncN[0] * 8.0f, IncN[1] * 8.0f, IncN[2] * 8.0f};
    const float IncZ8 = 8.0f * IncZ;

    const float Tw = (float)Bm->Width, Th = (float)Bm->Height;
    const float InvM2P = 1.0f / T->MetersToPixels;
    for (int i = 0; i < 8; ++i) Clip[i] = Start[i];

    const int32_t X0 = (int32_t)LeftX, X1 = (int32_t)RightX;
    for (int32_t X = X0; X < X1; X += 8) { /* 1858 */
        for (int i = 0; i < 8; ++i) {
            float IW = 1.0f / Wl[i];
            float FU = IW * Ul[i], FV = IW * Vl[i];
            float TCX = Tw * FU, TCY = Th * FV;
            int Mask = (FU >= 0.0f) && (FU <= 1.0f) && (FV >= 0.0f) && (FV <= 1.0f) && Clip[i];
            if (!Mask) continue;
            float zb = X_->Z[(size_t)Row * W + X + i];
            float CA, CR, CG, CB;
            if (X_->Filter == PRK_FILTER_BILINEAR) {
                or_bilinear(Bm, FU, FV, &CA, &CR, &CG, &CB);
            } else {
                int32_t FX = (int32_t)((uint32_t)or_cvtt_s32(TCX) << 2);
                int32_t FY = or_mul16_trick(or_cvtt_s32(TCY), Bm->Pitch);
                int32_t Off = (int32_t)((uint32_t)FX + (uint32_t)FY);
                uint32_t Tx = or_texel(Bm, Off);
                CA = (float)((Tx >> 24) & 0xFF) / 255.0f;
                CR = (float)((Tx >> 16) & 0xFF) / 255.0f;
                CG = (float)((Tx >> 8) & 0xFF) / 255.0f;
                CB = (float)((Tx >> 0) & 0xFF) / 255.0f;
            }

            /* Phong (2040-2128) with UnprojectVertex_8x (102-145). */
            float d = T->DistanceAboveTarget - Zl[i];
            float Xf = (float)X + (float)i, Yf = (float)Row + 0.0f;
            float AX = (Xf - T->ScreenCenter[0]) * InvM2P;
            float AY = (Yf - T->ScreenCenter[1]) * InvM2P;
            float PX = (d / T->FocalLength) * AX, PY = (d / T->FocalLength) * AY, PZ = Zl[i];
            float Fr = 0, Fg = 0, Fb = 0, Fa = 0;
            for (uint32_t li = 0; li < X_->Lights->LightCount; ++li) {
                const prk_light_info *Lt = &X_->Lights->Lights[li];
                if (li == 0) {
                    Fr = CR * X_->Lights->AmbientIntensity[0];
                    Fg = CG * X_->Lights->AmbientIntensity[1];
                    Fb = CB * X_->Lights->AmbientIntensity[2];
                    Fa = CA * X_->Lights->AmbientIntensity[3];
                }
                float Lx = Lt->P[0] - PX, Ly = Lt->P[1] - PY, Lz = Lt->P[2] - PZ;
                or_normalize_div(&Lx, &Ly, &Lz);
                float Cos = or_minps(1.0f, or_maxps(0.0f, (Nx[i] * Lx + Ny[i] * Ly) + Nz[i] * Lz));
                float Vx = 0.0f - PX, Vy = 0.0f - PY, Vz = 0.0f - PZ;
                or_normalize_div(&Vx, &Vy, &Vz);
                float Hx = Lx + Vx, Hy = Ly + Vy, Hz = Lz + Vz;
                or_normalize_div(&Hx, &Hy, &Hz);
                float Ph = or_minps(1.0f, or_maxps(0.0f, (Nx[i] * Hx + Ny[i] * Hy) + Nz[i] * Hz));
                for (int f = 0; f < 4; ++f) Ph = Ph * Ph;
                Fr = Fr + ((Cos * (CR * Lt->Intensity[0])) + (Ph * (1.0f * Lt->Intensity[0])));
                Fg = Fg + ((Cos * (CG * Lt->Intensity[1])) + (Ph * (1.0f * Lt->Intensity[1])));
                Fb = Fb + ((Cos * (CB * Lt->Intensity[2])) + (Ph * (1.0f * Lt->Intensity[2])));
                Fa = Fa + ((Cos * (CA * Lt->Intensity[3])) + (Ph * (1.0f * Lt->Intensity[3])));
            }
            Fr = or_maxps(or_minps(Fr, 1.0f), 0.0f);
            Fg = or_maxps(or_minps(Fg, 1.0f), 0.0f);
            Fb = or_maxps(or_minps(Fb, 1.0f), 0.0f);
            Fa = or_maxps(or_minps(Fa, 1.0f), 0.0f);
            uint32_t Packed = ((uint32_t)or_cvt_rne_s32(Fr * 255.0f) << 16) |
                              ((uint32_t)or_cvt_rne_s32(Fg * 255.0f) << 8) |
                              ((uint32_t)or_cvt_rne_s32(Fb * 255.0f) << 0) |
                              ((uint32_t)or_cvt_rne_s32(Fa * 255.0f) << 24);
            /* z-test, predicate 30 = GT_OQ (2217-2233); single-thread
             * overload: predicate 29 = GE_OQ (3205). */
            if (X_->St ? (Zl[i] >= zb) : (Zl[i] > zb)) {
                size_t px = (size_t)Row * W + X + i;
                X_->Z[px] = Zl[i];
                uint32_t *row = (uint32_t *)((uint8_t *)X_->Color + (size_t)Row * X_->Pitch);
                row[X + i] = Packed;
                if (X_->Winners) X_->Winners[px] = X_->TriIndex;
                X_->Writes++;
            }
        }
        /* Next clip mask (2241-2256), then the block step (2262-2282). */
        for (int i = 0; i < 8; ++i) Clip[i] = ((X + 16) < RightX) ? 1 : End[i];
        for (int i = 0; i < 8; ++i) {
            float a = Nx[i] + IncN8[0], b = Ny[i] + IncN8[1], c = Nz[i] + IncN8[2];
            or_normalize_div(&a, &b, &c);
            Nx[i] = a; Ny[i] = b; Nz[i] = c;
            Zl[i] = Zl[i] + IncZ8;
            Wl[i] = Wl[i] + IncW8;
            Ul[i] = Ul[i] + IncU8;
            Vl[i] = Vl[i] + IncV8;
        }
    }
}

/* ------------------------------------------------------------------ */
/* DrawModel span body (projekt.cpp:298-538), scalar semantics.        */
/* ------------------------------------------------------------------ */
static void or_fill_line_scalar(or_ctx *X_, const or_edge *L, const or_edge *R, int32_t Row)
{
    const prk_transform *T = X_->T;
    const prk_bitmap *Bm = X_->Bitmap;
    const int32_t W = X_->Width;
    float XOffset = 0.0f;
    if (Row < 0) return;
    float XDiff = roundf(R->XMin - L->XMin); /* 311-312 */
    float IncW = 0, IncU = 0, IncV = 0, IncN[3] = {0, 0, 0}, IncC[4] = {0, 0, 0, 0}, IncZ = 0;
    if (XDiff != 0.0f) { /* 329-360 */
        IncW = (R->OneOverZMin - L->OneOverZMin) / XDiff;
        IncU = (R->UMin - L->UMin) / XDiff;
        IncV = (R->VMin - L->VMin) / XDiff;
        for (int c = 0; c < 3; ++c) IncN[c] = (R->MinNormal[c] - L->MinNormal[c]) / XDiff;
        for (int c = 0; c < 4; ++c) IncC[c] = (R->MinColor[c] - L->MinColor[c]) / XDiff;
        IncZ = (R->ZMin - L->ZMin) / XDiff;
    }
    float CurZ = L->ZMin, CurW = L->OneOverZMin, CurU = L->UMin, CurV = L->VMin;
    float CurN[3] = {L->MinNormal[0], L->MinNormal[1], L->MinNormal[2]};
    float CurC[4] = {L->MinColor[0], L->MinColor[1], L->MinColor[2], L->MinColor[3]};
    float LeftX = L->XMin; /* 381-400 */
    if (LeftX < 0) { XOffset = -L->XMin; LeftX = 0; }
    else if (LeftX >= W) LeftX = (float)W - 1;
    float RightX = R->XMin;
    if (RightX < 0) RightX = 0;
    else if (RightX >= W) RightX = (float)W - 1;
    if (LeftX != LeftX || RightX != RightX) return; /* pin: NaN edge X draws nothing */
    LeftX = (float)or_round_s32(LeftX);
    RightX = (float)or_round_s32(RightX);
    int32_t MinX = (int32_t)LeftX, MaxX = (int32_t)RightX;
    CurZ += XOffset * IncZ; /* 408-412 */
    CurW += XOffset * IncW;
    CurU += XOffset * IncU;
    CurV += XOffset * IncV;
    for (int c = 0; c < 3; ++c) CurN[c] += XOffset * IncN[c];
    for (int c = 0; c < 4; ++c) CurC[c] += XOffset * IncC[c];

    if (or_owns(X_, Row)) {
        if (MaxX >= MinX) X_->SpanPixels += (uint64_t)(MaxX - MinX + 1);
        X_->Spans++;
    }
    uint32_t *rowp = (uint32_t *)((uint8_t *)X_->Color + (size_t)Row * X_->Pitch);
    float *zrow = X_->Z + (size_t)Row * W;
    const float InvM2P = 1.0f / T->MetersToPixels;

    /* MaxX can round to Width (RightX in [W-0.5, W) is not clamped, 389-399),
     * so the inclusive loop stores one pixel past the row: linear index
     * Row*W + W, i.e. pixel (Row+1, 0) of the z-buffer (and of the colour
     * buffer when Pitch == 4*W).  On the last row that store lands outside
     * the buffers (undefined in the reference): pinned as dropped. */
    const int own_row = or_owns(X_, Row);
    const int own_next = Row + 1 < X_->Height && or_owns(X_, Row + 1);
    for (int32_t X = MinX; X <= MaxX; ++X) { /* 423 */
        const int draw = X < W ? own_row : own_next;
        if (Bm) { /* 427-446 */
            float s = 1.0f / CurW;
            float FU = s * CurU, FV = s * CurV;
            float TCx = FU * (float)(Bm->Width - 1), TCy = FV * (float)(Bm->Height - 1);
            int32_t TX = or_round_s32(TCx), TY = or_round_s32(TCy);
            int32_t Off = (int32_t)((uint32_t)TX * 4u + (uint32_t)TY * (uint32_t)Bm->Pitch);
            uint32_t Tx = or_texel(Bm, Off);
            CurC[3] = (float)((Tx >> 24) & 0xFF) / 255.0f;
            CurC[0] = (float)((Tx >> 16) & 0xFF) / 255.0f;
            CurC[1] = (float)((Tx >> 8) & 0xFF) / 255.0f;
            CurC[2] = (float)((Tx >> 0) & 0xFF) / 255.0f;
        }
        float F[4] = {0, 0, 0, 0};
        if (X_->Phong) { /* 448-510 */
            float d = T->DistanceAboveTarget - CurZ;
            or_v3 Pv = or_v3make(((d) / T->FocalLength) * (((float)X - T->ScreenCenter[0]) * InvM2P),
                                 ((d) / T->FocalLength) * (((float)Row - T->ScreenCenter[1]) * InvM2P),
                                 CurZ);
            or_v3 Nv = or_v3make(CurN[0], CurN[1], CurN[2]);
            for (uint32_t li = 0; li < X_->Lights->LightCount; ++li) {
                const prk_light_info *Lt = &X_->Lights->Lights[li];
                if (li == 0)
                    for (int c = 0; c < 4; ++c) F[c] = CurC[c] * X_->Lights->AmbientIntensity[c];
                or_v3 LP = or_v3make(Lt->P[0], Lt->P[1], Lt->P[2]);
                or_v3 Lv = or_normalize(or_sub(LP, Pv));
                float Cos = or_clamp01(or_inner(Nv, Lv));
                or_v3 Vv = or_normalize(or_v3make(-Pv.x, -Pv.y, -Pv.z));
                or_v3 Hv = or_normalize(or_add(Lv, Vv));
                float Ph = or_clamp01(or_inner(Nv, Hv));
                Ph = (float)pow((double)Ph, 16.0);
                for (int c = 0; c < 4; ++c)
                    F[c] = F[c] + ((Cos * (CurC[c] * Lt->Intensity[c])) + (Ph * (1.0f * Lt->Intensity[c])));
            }
            for (int c = 0; c < 4; ++c) F[c] = or_clamp01(F[c]);
        } else {
            for (int c = 0; c < 4; ++c) F[c] = CurC[c]; /* 515 (no clamp) */
        }
        uint32_t Packed = (or_round_u32(F[3] * 255.0f) << 24) | (or_round_u32(F[0] * 255.0f) << 16) |
                          (or_round_u32(F[1] * 255.0f) << 8) | (or_round_u32(F[2] * 255.0f) << 0);
        if (draw && CurZ > zrow[X]) { /* 495 / 525 */
            zrow[X] = CurZ;
            rowp[X] = Packed;
            if (X_->Winners) X_->Winners[(size_t)Row * W + X] = X_->TriIndex;
            X_->Writes++;
        }
        if (X_->Phong) { /* 504-510 */
            or_v3 n = or_normalize(or_v3make(CurN[0] + IncN[0], CurN[1] + IncN[1], CurN[2] + IncN[2]));
            CurN[0] = n.x; CurN[1] = n.y; CurN[2] = n.z;
            for (int c = 0; c < 4; ++c) CurC[c] = CurC[c] + IncC[c];
            CurZ += IncZ;
            CurW += IncW;
            CurU += IncU;
            CurV += IncV;
        } else { /* 530-535 */
            for (int c = 0; c < 4; ++c) CurC[c] = CurC[c] + IncC[c];
            CurZ += IncZ;
            CurU += IncU;
            CurV += IncV;
            CurW += IncW;
        }
    }
}

/* ------------------------------------------------------------------ */
/* Active-edge-table walk shared by DrawModel (projekt.cpp:168-598)    */
/* and DrawModelOptimized(RenderQueue,...) (3615-3871): identical list */
/* logic; the span body is the callback.  P3 applied at the swap.      */
/* ------------------------------------------------------------------ */
typedef void (*or_span_fn)(or_ctx *, const or_edge *, const or_edge *, int32_t);
#ifndef OR_AVX_SPAN
#define OR_AVX_SPAN or_fill_line_optimized
#endif

static inline int or_insert_before(const or_edge *A, const or_edge *B)
{
    return A->XMin < B->XMin ||
           (A->XMin == B->XMin &&
            (A->Gradient < B->Gradient || (A->Gradient == B->Gradient && A->Left < B->Left)));
}

static void or_step_edge(or_edge *E)
{
    E->XMin += E->Gradient;
    E->ZMin += E->ZGradient;
    for (int c = 0; c < 4; ++c) E->MinColor[c] += E->ColorGradient[c];
    or_v3 n = or_normalize(or_v3make(E->MinNormal[0] + E->NormalGradient[0],
                                     E->MinNormal[1] + E->NormalGradient[1],
                                     E->MinNormal[2] + E->NormalGradient[2]));
    E->MinNormal[0] = n.x; E->MinNormal[1] = n.y; E->MinNormal[2] = n.z;
    E->UMin += E->UGradient;
    E->VMin += E->VGradient;
    E->OneOverZMin += E->OneOverZGradient;
}

static void or_aet_walk(or_ctx *X_, or_edge *Edges, uint32_t EdgeCount, or_span_fn Span)
{
    if (EdgeCount == 0) return; /* P1 consequence */
    int32_t FirstRow = Edges[0].YMin; /* 3626 */
    int32_t MaxRow = Edges[0].YMax;
    for (uint32_t i = 1; i < EdgeCount; ++i)
        if (MaxRow < Edges[i].YMax) MaxRow = Edges[i].YMax;
    int32_t MaxY = FirstRow + (MaxRow - FirstRow);
    if (MaxY > X_->Height) MaxY = X_->Height;
    if (MaxY > X_->RowHi) MaxY = X_->RowHi; /* band filter: rows past the band are never drawn */
    or_edge *Head = NULL, *Tail = NULL;
    for (int32_t Row = FirstRow; Row < MaxY; ++Row) {
        for (uint32_t i = 0; i < EdgeCount; ++i) { /* insertion 3654-3713 */
            or_edge *Cur = Edges + i;
            if (Cur->YMin != Row) continue;
            if (Head) {
                if (or_insert_before(Cur, Head)) {
                    Cur->Next = Head;
                    Head = Cur;
                } else {
                    or_edge *Cmp = Head, *Prev = Head;
                    while (Cmp != Tail) {
                        Cmp = Cmp->Next;
                        if (or_insert_before(Cur, Cmp)) {
                            Cur->Next = Cmp;
                            Prev->Next = Cur;
                            Cmp = Tail;
                        } else {
                            Prev = Cmp;
                        }
                    }
                    if (Prev == Cmp) {
                        Tail->Next = Cur;
                        Tail = Cur;
                    }
                }
            } else {
                Head = Cur;
                Tail = Head;
            }
        }
        while (Head && Head->YMax <= Row) { /* expiry 3715-3720 */
            or_edge *Rm = Head;
            Head = Head->Next;
            Rm->Next = NULL;
        }
        if (!Head) { Tail = NULL; continue; } /* pin: the reference dereferences NULL */
        {
            or_edge *Prev = Head, *Chk = Head; /* 3722-3749 */
            while (Chk != Tail) {
                Chk = Chk->Next;
                if (Chk->YMax <= Row) {
                    if (Chk == Tail) {
                        Tail = Prev;
                        Tail->Next = NULL;
                        Chk = Tail;
                    } else {
                        Prev->Next = Chk->Next;
                        Chk = Prev;
                    }
                }
                Prev = Chk;
            }
        }
        or_edge *PrevCur = NULL, *PrevNext = NULL; /* pairing 3751-3869 */
        or_edge *Cur = Head, *Next = Cur->Next;
        while (Next) {
            if (or_owns(X_, Row) || (Span == or_fill_line_scalar && or_owns(X_, Row + 1))) {
                or_edge a = *Cur, b = *Next; /* by-value copies (3759-3807) */
                a.Next = b.Next = NULL;
                Span(X_, &a, &b, Row);
            }
            or_step_edge(Cur); /* 3811-3829 */
            or_step_edge(Next);
            if (Cur->XMin > Next->XMin) { /* 3831-3841 */
                Cur->Next = Next->Next;
                Next->Next = Cur;
                if (PrevNext) PrevNext->Next = Next;
                else Head = Next;                  /* P3 */
                if (Tail == Next) Tail = Cur;      /* P3 */
                Cur = Next;
                Next = Cur->Next;
            }
            if (PrevNext) { /* 3843-3853 */
                if (PrevNext->XMin > Cur->XMin) {
                    PrevNext->Next = Cur->Next;
                    Cur->Next = PrevNext;
                    PrevCur->Next = Cur;
                    PrevNext = Cur;
                    Cur = PrevNext->Next;
                }
            }
            PrevCur = Cur;
            PrevNext = Next;
            if (Next->Next) {
                Cur = Next->Next;
                Next = Cur->Next;
            } else {
                Next = NULL;
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* Public oracle entry points.                                         */
/* ------------------------------------------------------------------ */

typedef struct or_draw_desc {
    const float *Vertices, *Colors, *Normals, *UVs;
    uint32_t TriCount;
    uint32_t TrisPerObject;   /* 1 = per-triangle submission (the parity contract) */
    float P[3];
    int32_t Semantics;        /* PRK_SEM_* */
    int32_t Phong;
    const prk_bitmap *Bitmap; /* host memory with guard row, or NULL */
    int32_t TriIndexBase;     /* winner id of triangle 0 */
    int32_t Filter;           /* PRK_FILTER_* (AVX semantics; extension) */
    int32_t Setup;            /* FillEdgeTable's own inputs (prk.h PRK_SETUP_*): bit 0 its
                                 PhongShading, bit 1 Object->Bitmap != 0; < 0: as the draw
                                 (Phong, Bitmap != NULL) */
    /* The camera and lights FillEdgeTable saw (ProjectVertex 3906-3910, Gouraud
     * lighting 4020-4063), when the caller changed Commands between the
     * object's FillEdgeTable and its DrawModel* call; NULL: the draw's own
     * (the span shading always reads the draw's: 452-458, 2042-2046, 3030-3034). */
    const prk_transform *SetupT;
    const prk_light_data *SetupLights;
} or_draw_desc;

static inline const prk_transform *or_setup_t(const or_draw_desc *D, const prk_transform *T)
{
    return D->SetupT ? D->SetupT : T;
}
static inline const prk_light_data *or_setup_l(const or_draw_desc *D, const prk_light_data *L)
{
    return D->SetupLights ? D->SetupLights : L;
}

/* FillEdgeTable's PhongShading and Object->Bitmap of a draw (projekt.cpp:
 * 4012-4089 read them; DrawModel* reads its own Phong / Bitmap). */
static inline int or_setup_phong(const or_draw_desc *D) { return D->Setup < 0 ? D->Phong != 0 : (D->Setup & 1); }
static inline int or_setup_bitmap(const or_draw_desc *D)
{
    return D->Setup < 0 ? D->Bitmap != NULL : ((D->Setup >> 1) & 1);
}

typedef struct or_target {
    uint32_t *Color;
    int32_t Pitch;
    float *Z;
    int32_t Width, Height;
    int32_t *Winners;
} or_target;

/* Conservative row range [lo, hi) an object can draw into: spans lie on rows
 * [max(0, round(min y)), round(max y)) of its projected vertices. */
static void or_object_rows(const or_draw_desc *D, uint32_t t0, uint32_t n, const prk_transform *T,
                           int32_t *lo, int32_t *hi)
{
    float ymin = INFINITY, ymax = -INFINITY;
    for (uint32_t t = t0; t < t0 + n; ++t)
        for (int k = 0; k < 3; ++k) {
            const float *v = D->Vertices + 9 * (size_t)t + 3 * k;
            or_v3 p = or_project_vertex(or_v3make(v[0] + D->P[0], v[1] + D->P[1], v[2] + D->P[2]), T);
            if (p.y != p.y) { ymin = -INFINITY; ymax = INFINITY; continue; }
            if (p.y < ymin) ymin = p.y;
            if (p.y > ymax) ymax = p.y;
        }
    float a = floorf(ymin), b = ceilf(ymax);
    *lo = a < -1e9f ? INT32_MIN / 2 : (a > 1e9f ? INT32_MAX / 2 : (int32_t)a);
    *hi = b < -1e9f ? INT32_MIN / 2 : (b > 1e9f ? INT32_MAX / 2 : (int32_t)b);
}

static int or_draw_filtered(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                            const prk_light_data *Lights, int32_t row_lo, int32_t row_hi,
                            int32_t band_h, int32_t band_mod, int32_t band_rem, uint64_t *stats)
{
    if (!D || !Tg || !T || !Lights) return PRK_ERR_ARG;
    const int avx = D->Semantics == PRK_SEM_AVX || D->Semantics == PRK_SEM_AVX_ST;
    if (avx && (!D->Bitmap || !D->Phong)) return PRK_ERR_UNSUPPORTED;
    if (avx && (Tg->Width % 8)) return PRK_ERR_UNSUPPORTED;
    /* edge fields FillEdgeTable never wrote: MinNormal without its
     * PhongShading (4012-4064), U/V/(1/z) gradients without Object->Bitmap
     * (4078-4089) -- a draw reading them is undefined */
    if ((D->Phong && !or_setup_phong(D)) || (D->Bitmap && !or_setup_bitmap(D))) return PRK_ERR_UNSUPPORTED;
    if (Lights->LightCount > PRK_MAX_LIGHTS) return PRK_ERR_ARG;
    if (D->SetupLights && D->SetupLights->LightCount > PRK_MAX_LIGHTS) return PRK_ERR_ARG;
    uint32_t per = D->TrisPerObject ? D->TrisPerObject : 1;
    or_edge *Edges = (or_edge *)malloc(sizeof(or_edge) * 3 * per);
    or_edge *Sort = (or_edge *)malloc(sizeof(or_edge) * 3 * per);
    if (!Edges || !Sort) { free(Edges); free(Sort); return PRK_ERR_NOMEM; }
    or_ctx X_;
    memset(&X_, 0, sizeof X_);
    X_.T = T; X_.Lights = Lights; X_.Bitmap = D->Bitmap;
    X_.Color = Tg->Color; X_.Pitch = Tg->Pitch; X_.Z = Tg->Z;
    X_.Width = Tg->Width; X_.Height = Tg->Height; X_.Winners = Tg->Winners;
    X_.RowLo = row_lo; X_.RowHi = row_hi; X_.Phong = D->Phong; X_.Filter = D->Filter;
    X_.BandH = band_h; X_.BandMod = band_mod; X_.BandRem = band_rem;
    X_.St = D->Semantics == PRK_SEM_AVX_ST;
    /* OR_AVX_SPAN: the AVX2 CPU baseline (prk_cpu_avx.c) substitutes its
     * 8-wide span here; this file alone always uses the scalar restatement. */
    or_span_fn Span = D->Semantics == PRK_SEM_AVX ? OR_AVX_SPAN
                      : (D->Semantics == PRK_SEM_AVX_ST ? or_fill_line_optimized : or_fill_line_scalar);
    for (uint32_t t0 = 0; t0 < D->TriCount; t0 += per) {
        uint32_t n = D->TriCount - t0 < per ? D->TriCount - t0 : per;
        if (band_mod > 1 || row_lo > 0 || row_hi < Tg->Height) {
            /* Skip objects that cannot touch a row this call draws (a pure
             * speed-up: the walk of such an object never reaches Span). */
            int32_t lo, hi;
            or_object_rows(D, t0, n, or_setup_t(D, T), &lo, &hi);
            if (D->Semantics == PRK_SEM_SCALAR && hi < INT32_MAX / 2) hi += 1; /* row-overflow pixel */
            if (lo < row_lo) lo = row_lo;
            if (hi > row_hi) hi = row_hi;
            if (lo >= hi) continue;
            if (band_mod > 1 && (hi - lo) < band_h * band_mod) {
                int32_t b0 = lo / band_h, b1 = (hi - 1) / band_h, hit = 0;
                for (int32_t b = b0; b <= b1 && !hit; ++b) hit = (b % band_mod) == band_rem;
                if (!hit) continue;
            }
        }
        uint32_t ec = or_fill_edge_table(D->Vertices, D->Colors, D->Normals, D->UVs, t0, n, D->P,
                                         or_setup_bitmap(D), or_setup_phong(D), or_setup_t(D, T),
                                         or_setup_l(D, Lights), Edges, Sort);
        X_.TriIndex = D->TriIndexBase + (int32_t)t0;
        or_aet_walk(&X_, Edges, ec, Span);
    }
    free(Edges);
    free(Sort);
    if (stats) { stats[0] += X_.Spans; stats[1] += X_.SpanPixels; stats[2] += X_.Writes; }
    return PRK_OK;
}

/* Draw one batch of triangles restricted to frame rows [row_lo, row_hi).
 * stats (nullable): [spans, span_pixels, writes]. */
int oracle_draw_band(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                     const prk_light_data *Lights, int32_t row_lo, int32_t row_hi,
                     uint64_t *stats)
{
    return or_draw_filtered(D, Tg, T, Lights, row_lo, row_hi, 1, 1, 0, stats);
}

int oracle_draw(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                const prk_light_data *Lights, uint64_t *stats)
{
    return oracle_draw_band(D, Tg, T, Lights, 0, Tg ? Tg->Height : 0, stats);
}

/* Banded multi-threaded driver (the CPU baseline's "banded" schedule,
 * BASELINE.md §3): rows are cut into 32-row bands and thread t owns the bands
 * b with b % threads == t.  Each thread walks, in submission order, only the
 * triangles whose row range meets one of its bands and draws only its rows.
 * No locks; output identical to the single-threaded oracle. */
#define OR_BAND_H 32
typedef struct or_job {
    const or_draw_desc *D; const or_target *Tg; const prk_transform *T;
    const prk_light_data *L; int32_t mod, rem; uint64_t stats[3]; int rc, spawned;
} or_job;

static void *or_job_run(void *p)
{
    or_job *j = (or_job *)p;
    j->rc = or_draw_filtered(j->D, j->Tg, j->T, j->L, 0, j->Tg->Height, OR_BAND_H, j->mod, j->rem,
                             j->stats);
    return NULL;
}

int oracle_draw_mt(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                   const prk_light_data *Lights, int32_t threads, uint64_t *stats)
{
    if (!Tg) return PRK_ERR_ARG;
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    or_job *jobs = (or_job *)calloc((size_t)threads, sizeof(or_job));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return PRK_ERR_NOMEM; }
    for (int t = 0; t < threads; ++t) {
        memset(&jobs[t], 0, sizeof jobs[t]);
        jobs[t].D = D; jobs[t].Tg = Tg; jobs[t].T = T; jobs[t].L = Lights;
        jobs[t].mod = threads; jobs[t].rem = t;
        jobs[t].spawned = pthread_create(&th[t], NULL, or_job_run, &jobs[t]) == 0;
    }
    int rc = PRK_OK;
    for (int t = 0; t < threads; ++t) {
        /* `spawned` is written before the thread exists; `rc` belongs to the
         * thread until the join (reading it earlier raced, found by TSan). */
        if (jobs[t].spawned) pthread_join(th[t], NULL);
        else or_job_run(&jobs[t]); /* could not spawn: run inline */
        if (jobs[t].rc != PRK_OK) rc = jobs[t].rc;
        if (stats) for (int k = 0; k < 3; ++k) stats[k] += jobs[t].stats[k];
    }
    free(jobs);
    free(th);
    return rc;
}

/* Expose FillEdgeTable alone (edge-level known-answer tests).  Writes the
 * sorted visible edges of triangles [tri0, tri0+n) of D as flat records:
 * [YMax, XMin, ZMin, OneOverZMin, Gradient, ZGradient, OneOverZGradient, YMin,
 *  UMin, VMin, UGradient, VGradient, Left, MinColor[4], ColorGradient[4],
 *  MinNormal[3], NormalGradient[3]] = 27 x 4-byte words per edge. */
int oracle_fill_edge_table(const or_draw_desc *D, uint32_t tri0, uint32_t n,
                           const prk_transform *T, const prk_light_data *Lights,
                           uint32_t *out_words, uint32_t *out_count)
{
    if (!D || !T || !Lights || !out_words || !out_count) return PRK_ERR_ARG;
    or_edge *Edges = (or_edge *)calloc(3 * (size_t)n + 1, sizeof(or_edge));
    or_edge *Sort = (or_edge *)calloc(3 * (size_t)n + 1, sizeof(or_edge));
    if (!Edges || !Sort) { free(Edges); free(Sort); return PRK_ERR_NOMEM; }
    uint32_t ec = or_fill_edge_table(D->Vertices, D->Colors, D->Normals, D->UVs, tri0, n, D->P,
                                     or_setup_bitmap(D), or_setup_phong(D), T, Lights, Edges, Sort);
    for (uint32_t i = 0; i < ec; ++i) {
        uint32_t *w = out_words + 27 * (size_t)i;
        const or_edge *E = Edges + i;
        memcpy(w + 0, &E->YMax, 4); memcpy(w + 1, &E->XMin, 4); memcpy(w + 2, &E->ZMin, 4);
        memcpy(w + 3, &E->OneOverZMin, 4); memcpy(w + 4, &E->Gradient, 4);
        memcpy(w + 5, &E->ZGradient, 4); memcpy(w + 6, &E->OneOverZGradient, 4);
        memcpy(w + 7, &E->YMin, 4); memcpy(w + 8, &E->UMin, 4); memcpy(w + 9, &E->VMin, 4);
        memcpy(w + 10, &E->UGradient, 4); memcpy(w + 11, &E->VGradient, 4);
        memcpy(w + 12, &E->Left, 4); memcpy(w + 13, E->MinColor, 16);
        memcpy(w + 17, E->ColorGradient, 16); memcpy(w + 21, E->MinNormal, 12);
        memcpy(w + 24, E->NormalGradient, 12);
    }
    *out_count = ec;
    free(Edges);
    free(Sort);
    return PRK_OK;
}

uint32_t oracle_edge_words(void) { return 27u; }

/* What DrawModel* leaves in the caller's edge list (all overloads share the
 * list walk and the edge step, 3654-3869 / 542-560): the walk of
 * or_aet_walk over a frame of `height` rows with no span body.  E (27 words
 * per edge, as oracle_fill_edge_table writes them) is advanced in place;
 * next_idx[i] = the index Edges[i].Next points at, or -1 for NULL. */
static void or_no_span(or_ctx *X_, const or_edge *L, const or_edge *R, int32_t Row)
{
    (void)X_; (void)L; (void)R; (void)Row;
}

int oracle_advance_edges(uint32_t *words, uint32_t n, int32_t height, int32_t *next_idx)
{
    if ((!words || !next_idx) && n) return PRK_ERR_ARG;
    or_edge *Edges = (or_edge *)calloc((size_t)n + 1, sizeof(or_edge));
    if (!Edges) return PRK_ERR_NOMEM;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t *w = words + 27 * (size_t)i;
        or_edge *E = Edges + i;
        memcpy(&E->YMax, w + 0, 4); memcpy(&E->XMin, w + 1, 4); memcpy(&E->ZMin, w + 2, 4);
        memcpy(&E->OneOverZMin, w + 3, 4); memcpy(&E->Gradient, w + 4, 4);
        memcpy(&E->ZGradient, w + 5, 4); memcpy(&E->OneOverZGradient, w + 6, 4);
        memcpy(&E->YMin, w + 7, 4); memcpy(&E->UMin, w + 8, 4); memcpy(&E->VMin, w + 9, 4);
        memcpy(&E->UGradient, w + 10, 4); memcpy(&E->VGradient, w + 11, 4);
        memcpy(&E->Left, w + 12, 4); memcpy(E->MinColor, w + 13, 16);
        memcpy(E->ColorGradient, w + 17, 16); memcpy(E->MinNormal, w + 21, 12);
        memcpy(E->NormalGradient, w + 24, 12);
        E->Next = NULL;
    }
    or_ctx X_;
    memset(&X_, 0, sizeof X_);
    X_.Height = height; X_.RowLo = 0; X_.RowHi = height;
    X_.BandH = 1; X_.BandMod = 1; X_.BandRem = 0;
    or_aet_walk(&X_, Edges, n, or_no_span);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t *w = words + 27 * (size_t)i;
        const or_edge *E = Edges + i;
        memcpy(w + 1, &E->XMin, 4); memcpy(w + 2, &E->ZMin, 4); memcpy(w + 3, &E->OneOverZMin, 4);
        memcpy(w + 8, &E->UMin, 4); memcpy(w + 9, &E->VMin, 4);
        memcpy(w + 13, E->MinColor, 16); memcpy(w + 21, E->MinNormal, 12);
        next_idx[i] = E->Next ? (int32_t)(E->Next - Edges) : -1;
    }
    free(Edges);
    return PRK_OK;
}

/* ------------------------------------------------------------------ */
/* Draws from a caller's edge list / span list (prk_draw_edges /       */
/* prk_draw_spans): DrawModelOptimized* on a ready edge_info list      */
/* (3615-3871: no sort, the insertion scan over every edge each row)   */
/* and the work records of DoLineRenderWork / DoBufferLineRenderWork   */
/* (2336-2348: FillLineOptimized / FillLinesOptimized on a pair).      */
/* ------------------------------------------------------------------ */
static void or_ctx_for(or_ctx *X_, int32_t semantics, const prk_bitmap *Bm, int32_t phong, int32_t filter,
                       const or_target *Tg, const prk_transform *T, const prk_light_data *L)
{
    memset(X_, 0, sizeof *X_);
    X_->T = T; X_->Lights = L; X_->Bitmap = Bm;
    X_->Color = Tg->Color; X_->Pitch = Tg->Pitch; X_->Z = Tg->Z;
    X_->Width = Tg->Width; X_->Height = Tg->Height; X_->Winners = Tg->Winners;
    X_->RowLo = 0; X_->RowHi = Tg->Height; X_->Phong = phong; X_->Filter = filter;
    X_->BandH = 1; X_->BandMod = 1; X_->BandRem = 0;
    X_->St = semantics == PRK_SEM_AVX_ST;
}

int oracle_draw_edges(const prk_edge *E, uint32_t n, int32_t semantics, const prk_bitmap *Bm, int32_t phong,
                      int32_t filter, int32_t tri_index, const or_target *Tg, const prk_transform *T,
                      const prk_light_data *L, uint64_t *stats)
{
    /* DrawModelOptimized* (AVX semantics) or DrawModel (scalar, 162-601) */
    const int scalar = semantics == PRK_SEM_SCALAR;
    if (!scalar && semantics != PRK_SEM_AVX && semantics != PRK_SEM_AVX_ST) return PRK_ERR_UNSUPPORTED;
    if (!scalar && (!Bm || !phong || (Tg->Width % 8))) return PRK_ERR_UNSUPPORTED;
    or_edge *Edges = (or_edge *)calloc((size_t)n + 1, sizeof(or_edge));
    if (!Edges) return PRK_ERR_NOMEM;
    for (uint32_t i = 0; i < n; ++i) {
        or_edge *o = Edges + i;
        o->YMax = E[i].YMax; o->XMin = E[i].XMin; o->ZMin = E[i].ZMin; o->OneOverZMin = E[i].OneOverZMin;
        o->Gradient = E[i].Gradient; o->ZGradient = E[i].ZGradient; o->OneOverZGradient = E[i].OneOverZGradient;
        o->YMin = E[i].YMin; o->UMin = E[i].UMin; o->VMin = E[i].VMin; o->UGradient = E[i].UGradient;
        o->VGradient = E[i].VGradient; o->Left = E[i].Left;
        memcpy(o->MinColor, E[i].MinColor, 16); memcpy(o->ColorGradient, E[i].ColorGradient, 16);
        memcpy(o->MinNormal, E[i].MinNormal, 12); memcpy(o->NormalGradient, E[i].NormalGradient, 12);
        o->Next = NULL;
    }
    or_ctx X_;
    or_ctx_for(&X_, semantics, Bm, phong, filter, Tg, T, L);
    X_.TriIndex = tri_index;
    or_aet_walk(&X_, Edges, n, scalar ? or_fill_line_scalar : or_fill_line_optimized);
    free(Edges);
    if (stats) { stats[0] += X_.Spans; stats[1] += X_.SpanPixels; stats[2] += X_.Writes; }
    return PRK_OK;
}

int oracle_draw_spans(const prk_span *S, uint32_t n, int32_t semantics, const prk_bitmap *Bm, int32_t phong,
                      int32_t filter, int32_t tri_index_base, const or_target *Tg, const prk_transform *T,
                      const prk_light_data *L, uint64_t *stats)
{
    if (semantics != PRK_SEM_AVX && semantics != PRK_SEM_AVX_ST) return PRK_ERR_UNSUPPORTED;
    if (!Bm || !phong || (Tg->Width % 8)) return PRK_ERR_UNSUPPORTED;
    or_ctx X_;
    or_ctx_for(&X_, semantics, Bm, phong, filter, Tg, T, L);
    for (uint32_t k = 0; k < n; ++k) {
        or_edge Le, Re; /* FillLinesOptimized 648-670: the pair's end points only */
        memset(&Le, 0, sizeof Le);
        memset(&Re, 0, sizeof Re);
        const prk_span_end *a = &S[k].Left, *b = &S[k].Right;
        Le.XMin = a->XMin; Le.ZMin = a->ZMin; Le.OneOverZMin = a->OneOverZMin; Le.UMin = a->UMin; Le.VMin = a->VMin;
        memcpy(Le.MinColor, a->MinColor, 16); memcpy(Le.MinNormal, a->MinNormal, 12);
        Re.XMin = b->XMin; Re.ZMin = b->ZMin; Re.OneOverZMin = b->OneOverZMin; Re.UMin = b->UMin; Re.VMin = b->VMin;
        memcpy(Re.MinColor, b->MinColor, 16); memcpy(Re.MinNormal, b->MinNormal, 12);
        X_.TriIndex = tri_index_base + (int32_t)k;
        if (S[k].Row < Tg->Height) or_fill_line_optimized(&X_, &Le, &Re, S[k].Row);
    }
    if (stats) { stats[0] += X_.Spans; stats[1] += X_.SpanPixels; stats[2] += X_.Writes; }
    return PRK_OK;
}
