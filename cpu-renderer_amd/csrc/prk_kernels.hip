// prk_kernels.hip — gfx950 kernels of the rasterizer hot path.
//
// Pipeline per flush: binning (prk_bin.hip) lists, for every
// screen tile, its (triangle, pair) entries — pair = the triangle's index
// for that tile, numbered in submission order — and, for all-AVX frames,
// writes one setup record per triangle (FillEdgeTable + MergeSort, projekt.cpp
// 3882-4121, 2-72).  Then:
//   k_vis    one workgroup per tile, the tile's 64-bit visibility keys in
//            LDS.  Each lane takes one bin entry, walks its triangle's AET
//            (3615-3871) over the tile's rows and spreads the spans' pixels
//            over the wave (FillLineOptimized 1492-2320 / DrawModel 298-538
//            arithmetic, z and the UV mask only).  LDS atomicMax of
//            key = (ordered z << 32) | tag(pair) keeps the reference's winner
//            (strict '>' in submission order: the EARLIEST fragment of
//            maximal z) whatever order the bin is walked in.
//            Out: the winning tag of every pixel, won (pair, row) flags.
//   k_won_local + k_walk   (AVX) the triangles that won a pixel, each walked
//            once over its whole AET with normals; every won row span
//            becomes a 64-B lane-init record.
//   k_pix    (AVX) one thread per pixel: winner -> record -> lane chain ->
//            texel + Phong -> z and colour, coalesced.
//   k_shade  (scalar DrawModel frames) per tile, re-walks the entries that won
//            a pixel and shades only their winning fragments.

#include "prk_device.h"

// Diagnostic builds only (tools/diag): 1 = skip the shading sweep, 2 = skip
// work items, 4 = skip the AET rows (setup only), 8 = skip the shading sweep's
// work items, 16 = no Phong/texel (winners store a dummy colour), 32 = no
// replay of the rows above a tile.  Never set
// in a product build.
#ifndef PRK_DIAG
#define PRK_DIAG 0
#endif
#ifndef PRK_PROF
#define PRK_PROF 0  // 1: accumulate per-phase s_memtime cycles into fp.prof (diagnostic builds)
#endif
#if PRK_PROF
#define PRK_T() __builtin_amdgcn_s_memtime()
#else
#define PRK_T() 0ull
#endif
#ifndef PRK_VIS_MIN_WAVES
#define PRK_VIS_MIN_WAVES 4  // waves per SIMD k_vis is register-budgeted for (<= 128 VGPRs)
#endif
#ifndef PRK_SPAN_RECORDS
#define PRK_SPAN_RECORDS 1  // AVX frames shade through k_walk + k_pix (else k_shade)
#endif
#ifndef PRK_WALK_MIN_WAVES
#define PRK_WALK_MIN_WAVES 4  // waves per SIMD k_walk is register-budgeted for
#endif
#ifndef PRK_WALK_ON_VIS
#define PRK_WALK_ON_VIS 0  // k_walk on k_vis's stream (k_pix alone on the flush stream)
#endif
#ifndef PRK_PIX_SPLIT
#define PRK_PIX_SPLIT 2  // k_pix workgroups per tile (2: serial k_pix 0.249 -> 0.245 ms on C3b; unrolling the
                         // pixel loop instead measured no change)
#endif
#ifndef PRK_SETUP_REC
#define PRK_SETUP_REC 1  // all-AVX frames: k_vis / k_walk read the binning pass's setup records
#endif
#ifndef PRK_SHADE_MIN_WAVES
#define PRK_SHADE_MIN_WAVES 3  // waves per SIMD k_shade is register-budgeted for
#endif

namespace prk {

__global__ void k_tri_draw(const DrawRec *__restrict__ draws, uint32_t ndraws,
                           uint32_t *__restrict__ tri_draw, uint32_t tri_count) {
    uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tri_count) return;
    uint32_t lo = 0, hi = ndraws - 1;
    while (lo < hi) {  // last draw with first_global <= g
        uint32_t mid = (lo + hi + 1) >> 1;
        if (draws[mid].first_global <= g) lo = mid; else hi = mid - 1;
    }
    tri_draw[g] = lo;
}

// Tiles a triangle may touch: the rectangle [tx0..tx1] x [ty0..ty1], plus
// for scalar semantics the column-0 tiles of rows [oty0..oty1] that receive
// DrawModel's one-past-the-row store (see span_scalar).
// ---------------------------------------------------------------------------
// Tile raster.
//
// One workgroup (4 waves) per tile.  A wave takes 64 bin entries at a time,
// one triangle per lane: the lane runs FillEdgeTable for it and then all 64
// lanes walk their AETs row by row in lock step.  At each row a lane's span
// (the reference's line_render_work, projekt.cpp:3756-3809) goes to the
// wave's LDS slots, and the wave splits the row's spans into work items:
//   AVX    : item j of a span = pixels xa+j, xa+j+8, ... < xb, i.e. ONE of the
//            8 lane chains of FillLineOptimized (each chain is an independent
//            float recurrence: lane init + one step per 8-px block);
//   scalar : one item per span (DrawModel's recurrence runs pixel by pixel).
// Items are spread over the 64 lanes (prefix sum + binary search), so the
// pixel work no longer serialises on the lane that owns the triangle.
// ---------------------------------------------------------------------------
#ifndef PRK_ZPRE
#define PRK_ZPRE 1  // sweep 1: skip 1/w and the UV mask of fragments that cannot raise the key
#endif
#ifndef PRK_PREFETCH
#define PRK_PREFETCH 0  // single-draw sweeps prefetch the next chunk's triangles (costs the
                        // registers of a 4-wave-per-SIMD k_vis: measured slower)
#endif
#ifndef PRK_LANE_ROWS
#define PRK_LANE_ROWS 1  // sweeps: each lane walks its own rows (no row lock step across the wave)
#endif
#ifndef PRK_MULTI_ROWS
#define PRK_MULTI_ROWS 1  // sweeps: lanes emit up to 8 rows per iteration when few lanes hold rows
#endif
#ifndef PRK_MULTI_ROWS_AVX
#define PRK_MULTI_ROWS_AVX 4  // AVX sweeps: multi-row iterations only with at most this many active lanes
#endif
static_assert(PRK_MULTI_ROWS_AVX <= 8, "8 rows per lane for at most 8 lanes: the 64 span slots");
#ifndef PRK_VIS_GROUP
#define PRK_VIS_GROUP 2  // visibility items: G consecutive pixels each (0: one lane chain each)
#endif
#ifndef PRK_PIXEL_ITEMS
#define PRK_PIXEL_ITEMS 1  // shading sweep (AVX): one work item per won pixel, not per lane chain
#endif
#ifndef PRK_VIS_PREBIN
#define PRK_VIS_PREBIN 1  // k_vis: the next chunk's bin entries load while this chunk runs
#endif
#ifndef PRK_VIS_DYN
#define PRK_VIS_DYN 1  // k_vis waves take the bin's chunks from an LDS counter
#endif
#ifndef PRK_VIS_WAVES
// waves per k_vis tile workgroup; each takes whole 64-entry chunks of the bin.
// Four waves share one 16 KiB key array: 4 workgroups = 16 waves per CU.
#define PRK_VIS_WAVES 4
#endif
#ifndef PRK_SHADE_WAVES
#define PRK_SHADE_WAVES 2  // waves per k_shade tile workgroup
#endif
constexpr int kVisWaves = PRK_VIS_WAVES, kShadeWaves = PRK_SHADE_WAVES;
constexpr int kSpanF = 22;  // float fields per span slot
constexpr int kSpanI = 11;  // int fields per span slot
// (the visibility sweep uses the first kSpanIVis int fields only)
enum { SI_XA = 0, SI_XB, SI_LEFT, SI_PRE, SI_TAG, SI_OVF, SI_MARK, SI_ROW, SI_TEX, SI_WM0, SI_WM1 };
// AVX float slots
enum { SF_XOFF = 0, SF_LW, SF_LU, SF_LV, SF_LZ, SF_IW, SF_IU, SF_IV, SF_IZ, SF_LN0, SF_LN1, SF_LN2,
       SF_IN0, SF_IN1, SF_IN2 };
// scalar float slots
enum { SS_Z = 0, SS_IZ, SS_W, SS_U, SS_V, SS_IW, SS_IU, SS_IV, SS_N0, SS_N1, SS_N2, SS_IN0, SS_IN1, SS_IN2,
       SS_C0, SS_C1, SS_C2, SS_C3, SS_IC0, SS_IC1, SS_IC2, SS_IC3 };

template <int NF, int NI>
struct WaveSlotsT {
    float f[NF][64];
    int32_t i[NI][64];
};
constexpr int kTagPad = 16;  // k_shade: tags past the tile's last pixel (chunked reads)
constexpr int kSpanFVis = 9;  // the visibility sweep reads no normals or colours (SF_IZ + 1)
constexpr int kSpanIVis = 8;  // SI_ROW + 1
using VisSlots = WaveSlotsT<kSpanFVis, kSpanIVis>;
// (All-AVX frames could drop SI_OVF and the scan scratch: 32 KiB per 256x8
// workgroup, five workgroups per CU instead of four.  Measured no faster on
// C3b, k_vis 0.495 ms either way: it is issue-bound, not latency-bound.)
using ShadeSlots = WaveSlotsT<kSpanF, kSpanI>;

struct TileCtx {
    int32_t x0, x1, y0, y1, tw;  // tile pixel rectangle [x0,x1) x [y0,y1), LDS row stride tw
    unsigned long long *key;     // LDS (k_vis): visibility keys
    const uint32_t *tags;        // LDS (k_shade): low key word = winning entry tag per pixel
};

__device__ __forceinline__ unsigned long long make_key(float z, uint32_t tag) {
    return ((unsigned long long)zkey(z) << 32) | tag;
}

__device__ __forceinline__ bool is_winner(const TileCtx &tc, int p, uint32_t tag) {
    return tc.tags[p] == tag;
}

// The winning fragment of pixel (x, y): store its z and colour (each pixel
// has exactly one winner, so these plain stores never race).
__device__ __forceinline__ void put_winner(const FrameParams &fp, int32_t x, int32_t y, float z, uint32_t col) {
    const size_t row = (size_t)(y - fp.row0);
    fp.zbuf[row * fp.W + x] = z;
    reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(fp.color) + row * fp.pitch)[x] = col;
}
__device__ __forceinline__ void put_color(const FrameParams &fp, int32_t x, int32_t y, uint32_t col) {
    reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(fp.color) + (size_t)(y - fp.row0) * fp.pitch)[x] = col;
}

// ----- span setup --------------------------------------------------------
// FillLineOptimized span setup (projekt.cpp:1543-1835) for row Row; writes the
// lane's slot and returns its item count (pixels of [MinX, MaxX) in the tile,
// at most 8 chains).
template <bool SHADE, class WS>
__device__ __forceinline__ int span_setup_avx(const FrameParams &fp, const TileCtx &tc, WS &ws, int lane,
                                              uint32_t tag, int32_t texi, const Edge &L, const Edge &R,
                                              int32_t Row, bool st) {
    if (Row < tc.y0) return 0;
    float XOffset;
    int32_t MinX, MaxX, XDiff;
    if (!span_ends(L.X, R.X, fp.W, st, MinX, MaxX, XDiff, XOffset)) return 0;  // 1545-1592
    int32_t LeftXa = MinX;
    if (MinX & 7) {  // 1594-1609
        LeftXa = MinX & ~7;
        XOffset -= (float)(MinX & 7) * 1.0f;
    }
    // The clip masks of 1594-1664 / 2241-2256 cover exactly [MinX, MaxX).
    const int32_t xa = max(MinX, tc.x0), xb = min(MaxX, tc.x1);
    if (xa >= xb) return 0;
    const float fXD = (float)XDiff;
    float IW = 0, IU = 0, IV = 0, IZ = 0, IN0 = 0, IN1 = 0, IN2 = 0;
    if (XDiff != 0) {  // 1666-1835
        // the span's increments over XDiff (div_all: one shared reciprocal)
        if constexpr (SHADE) {
            float q[7] = {R.W - L.W, R.U - L.U, R.V - L.V, R.N0 - L.N0, R.N1 - L.N1, R.N2 - L.N2, R.Z - L.Z};
            div_all(fXD, q);
            IW = q[0]; IU = q[1]; IV = q[2]; IN0 = q[3]; IN1 = q[4]; IN2 = q[5]; IZ = q[6];
        } else {  // (visibility: plain quotients, measured 1 % faster in k_vis than div_all)
            IW = (R.W - L.W) / fXD;
            IU = (R.U - L.U) / fXD;
            IV = (R.V - L.V) / fXD;
            IZ = (R.Z - L.Z) / fXD;
        }
    }
    ws.i[SI_XA][lane] = xa;
    ws.i[SI_XB][lane] = xb;
    ws.i[SI_LEFT][lane] = LeftXa;
    ws.i[SI_TAG][lane] = (int32_t)tag;
    if constexpr (SHADE) ws.i[SI_TEX][lane] = texi;
    ws.f[SF_XOFF][lane] = XOffset;
    ws.f[SF_LW][lane] = L.W; ws.f[SF_LU][lane] = L.U; ws.f[SF_LV][lane] = L.V; ws.f[SF_LZ][lane] = L.Z;
    ws.f[SF_IW][lane] = IW; ws.f[SF_IU][lane] = IU; ws.f[SF_IV][lane] = IV; ws.f[SF_IZ][lane] = IZ;
    if constexpr (SHADE) {
        ws.f[SF_LN0][lane] = L.N0; ws.f[SF_LN1][lane] = L.N1; ws.f[SF_LN2][lane] = L.N2;
        ws.f[SF_IN0][lane] = IN0; ws.f[SF_IN1][lane] = IN1; ws.f[SF_IN2][lane] = IN2;
#if PRK_PIXEL_ITEMS
        // Shading sweep: one item per pixel this span won; the won pixels of
        // the span's first 64 columns as a bit mask.
        // Tags are read 16 at a time (4 x ds_read_b128 from 16-B aligned
        // chunks), so the loads of a chunk are in flight together.
        const int rowoff = (Row - tc.y0) * tc.tw - tc.x0;
        int won = 0;
        uint64_t wm = 0;
        for (int32_t x0 = xa & ~3; x0 < xb; x0 += 16) {
            const uint4 *q = reinterpret_cast<const uint4 *>(tc.tags + rowoff + x0);
            const uint4 c0 = q[0], c1 = q[1], c2 = q[2], c3 = q[3];
            const uint32_t tg[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                                     c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int32_t x = x0 + k;
                const bool w = tg[k] == tag && x >= xa && x < xb;
                won += w ? 1 : 0;
                const int32_t sh = x - xa;
                if (w && sh < 64) wm |= 1ull << sh;
            }
        }
        ws.i[SI_WM0][lane] = (int32_t)(uint32_t)wm;
        ws.i[SI_WM1][lane] = (int32_t)(uint32_t)(wm >> 32);
        return won;
#endif
    }
    if constexpr (!SHADE && PRK_VIS_GROUP > 0) {
        constexpr int G = PRK_VIS_GROUP > 0 ? PRK_VIS_GROUP : 1;
        return (xb - xa + G - 1) / G;
    }
    return min(8, xb - xa);
}

// DrawModel spans are split into chunks of kScChunk pixels, one work item
// each.  The span's recurrence is sequential per pixel (423-538: Current* +=
// Increment after every pixel), so a chunk replays the adds (and, Phong, the
// renormalisations) from MinX to its first pixel, then does the per-pixel work
// of its own pixels only: a 200-px span costs its lanes one 200-step add chain
// instead of one lane 200 z-tests / shades in sequence.
template <bool SHADE>
constexpr int kScChunk = SHADE ? 8 : 16;
template <bool SHADE>
__device__ __forceinline__ int scalar_chunks(int32_t xa, int32_t xb) {
    return xa < xb ? (xb - xa + kScChunk<SHADE> - 1) / kScChunk<SHADE> : 0;
}

// DrawModel span setup (projekt.cpp:298-412).  Items: the span's chunks of
// [xa, xb), plus one for the one-past-the-row pixel (SI_OVF).
template <int M, bool SHADE, class WS>
__device__ __forceinline__ int span_setup_scalar(const FrameParams &fp, const TileCtx &tc, WS &ws, int lane,
                                                 uint32_t tag, int32_t texi, const Edge &L, const Edge &R,
                                                 int32_t Row) {
    using TR = ModeTraits<M>;
    const int32_t W = fp.W;
    float XOffset = 0.0f;
    const float XDiff = roundf(R.X - L.X);  // 311-312
    float IW = 0, IU = 0, IV = 0, IZ = 0, IN0 = 0, IN1 = 0, IN2 = 0;
    float IC0 = 0, IC1 = 0, IC2 = 0, IC3 = 0;
    if (XDiff != 0.0f) {  // 329-360
        // the span's increments over XDiff (div_all: one shared reciprocal)
        constexpr bool kT = SHADE && TR::tex, kP = SHADE && TR::phong, kC = SHADE && TR::color;
        float q[1 + (kT ? 3 : 0) + (kP ? 3 : 0) + (kC ? 4 : 0)];
        int qi = 0;
        q[qi++] = R.Z - L.Z;
        if (kT) { q[qi++] = R.W - L.W; q[qi++] = R.U - L.U; q[qi++] = R.V - L.V; }
        if (kP) { q[qi++] = R.N0 - L.N0; q[qi++] = R.N1 - L.N1; q[qi++] = R.N2 - L.N2; }
        if (kC) { q[qi++] = R.C0 - L.C0; q[qi++] = R.C1 - L.C1; q[qi++] = R.C2 - L.C2; q[qi++] = R.C3 - L.C3; }
        div_all(XDiff, q);
        qi = 0;
        IZ = q[qi++];
        if (kT) { IW = q[qi++]; IU = q[qi++]; IV = q[qi++]; }
        if (kP) { IN0 = q[qi++]; IN1 = q[qi++]; IN2 = q[qi++]; }
        if (kC) { IC0 = q[qi++]; IC1 = q[qi++]; IC2 = q[qi++]; IC3 = q[qi++]; }
    }
    float LeftX = L.X;  // 381-400
    if (LeftX < 0) { XOffset = -L.X; LeftX = 0; }
    else if (LeftX >= W) LeftX = (float)W - 1;
    float RightX = R.X;
    if (RightX < 0) RightX = 0;
    else if (RightX >= W) RightX = (float)W - 1;
    if (LeftX != LeftX || RightX != RightX) return 0;
    const int32_t MinX = round_s32(LeftX), MaxX = round_s32(RightX);  // 402-406
    // Inclusive [MinX, MaxX].  RightX in [W-0.5, W) is not clamped (389-399),
    // so MaxX can be W: the reference then stores linear pixel Row*W + W,
    // i.e. (Row+1, 0), which belongs to a column-0 tile one row down; on the
    // frame's last row it would fall outside the buffers (dropped).
    const bool in_rows = Row >= tc.y0;
    const int32_t xa = in_rows ? max(MinX, tc.x0) : 0;
    const int32_t xb = in_rows ? min(MaxX + 1, tc.x1) : 0;
    const bool ovf = tc.x0 == 0 && MaxX >= W && Row + 1 >= tc.y0 && Row + 1 < tc.y1;
    if (xa >= xb && !ovf) return 0;
    const int items = scalar_chunks<SHADE>(xa, xb) + (ovf ? 1 : 0);
    ws.i[SI_XA][lane] = xa;
    ws.i[SI_XB][lane] = xb;
    ws.i[SI_LEFT][lane] = MinX;
    ws.i[SI_TAG][lane] = (int32_t)tag;
    ws.i[SI_OVF][lane] = ovf ? (Row + 1 - tc.y0) * tc.tw : -1;
    if constexpr (SHADE) ws.i[SI_TEX][lane] = texi;
    ws.f[SS_Z][lane] = L.Z + XOffset * IZ;  // 408-412: Current* += XOffset*Increment
    ws.f[SS_IZ][lane] = IZ;
    if constexpr (SHADE) {
        if (TR::tex) {
            ws.f[SS_W][lane] = L.W + XOffset * IW; ws.f[SS_IW][lane] = IW;
            ws.f[SS_U][lane] = L.U + XOffset * IU; ws.f[SS_IU][lane] = IU;
            ws.f[SS_V][lane] = L.V + XOffset * IV; ws.f[SS_IV][lane] = IV;
        }
        if (TR::phong) {
            ws.f[SS_N0][lane] = L.N0 + XOffset * IN0; ws.f[SS_IN0][lane] = IN0;
            ws.f[SS_N1][lane] = L.N1 + XOffset * IN1; ws.f[SS_IN1][lane] = IN1;
            ws.f[SS_N2][lane] = L.N2 + XOffset * IN2; ws.f[SS_IN2][lane] = IN2;
        }
        if (TR::color) {
            ws.f[SS_C0][lane] = L.C0 + XOffset * IC0; ws.f[SS_IC0][lane] = IC0;
            ws.f[SS_C1][lane] = L.C1 + XOffset * IC1; ws.f[SS_IC1][lane] = IC1;
            ws.f[SS_C2][lane] = L.C2 + XOffset * IC2; ws.f[SS_IC2][lane] = IC2;
            ws.f[SS_C3][lane] = L.C3 + XOffset * IC3; ws.f[SS_IC3][lane] = IC3;
        }
    }
    return items;
}

// ----- work items ----------------------------------------------------------
// Phong + texel of one FillLineOptimized lane (projekt.cpp:1865-2200).
// Texel of one FillLineOptimized lane (1881-2032): trunc, <<2, 16-bit pitch
// multiply, P2 clamp.
__device__ __forceinline__ uint32_t texel_avx(const TexRec &tex, float fu, float fv) {
    const int32_t FX = (int32_t)((uint32_t)cvtt_s32((float)tex.w * fu) << 2);
    const int32_t FY = mul16_trick(cvtt_s32((float)tex.h * fv), tex.pitch);
    return texel_at(tex, (int32_t)((uint32_t)FX + (uint32_t)FY));
}

// A texel as the span's colour lanes (2029-2032): A, R, G, B in [0, 1].
struct Texel4 { float a, r, g, b; };

__device__ __forceinline__ Texel4 texel4(uint32_t t) {
    return Texel4{u8_unit((t >> 24) & 0xFF), u8_unit((t >> 16) & 0xFF), u8_unit((t >> 8) & 0xFF), u8_unit(t & 0xFF)};
}

// Bilinear sampling: an EXTENSION (BASELINE config 4; the reference samples
// nearest texels only).  Definition = oracle/prk_oracle.c:or_bilinear, op for
// op: texel centres at +0.5, clamp to the edge, fp32, no contraction.
__device__ __forceinline__ Texel4 bilinear(const TexRec &tex, float fu, float fv) {
    const float x = (float)tex.w * fu - 0.5f, y = (float)tex.h * fv - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    const float ax = x - fx, ay = y - fy;
    const int32_t wm = tex.w - 1, hm = tex.h - 1;
    const int32_t xi = (int32_t)fx, yi = (int32_t)fy;
    const int32_t x0 = min(max(xi, 0), wm), x1 = min(max(xi + 1, 0), wm);
    const int32_t y0 = min(max(yi, 0), hm), y1 = min(max(yi + 1, 0), hm);
    const uint32_t *r0 = reinterpret_cast<const uint32_t *>(tex.mem + (size_t)y0 * tex.pitch);
    const uint32_t *r1 = reinterpret_cast<const uint32_t *>(tex.mem + (size_t)y1 * tex.pitch);
    const Texel4 c00 = texel4(r0[x0]), c10 = texel4(r0[x1]), c01 = texel4(r1[x0]), c11 = texel4(r1[x1]);
    const float bx = 1.0f - ax, by = 1.0f - ay;
    Texel4 o;
    o.a = by * (bx * c00.a + ax * c10.a) + ay * (bx * c01.a + ax * c11.a);
    o.r = by * (bx * c00.r + ax * c10.r) + ay * (bx * c01.r + ax * c11.r);
    o.g = by * (bx * c00.g + ax * c10.g) + ay * (bx * c01.g + ax * c11.g);
    o.b = by * (bx * c00.b + ax * c10.b) + ay * (bx * c01.b + ax * c11.b);
    return o;
}

__device__ __forceinline__ Texel4 sample_avx(const TexRec &tex, float fu, float fv) {
    if (tex.filter == 1) return bilinear(tex, fu, fv);
    return texel4(texel_avx(tex, fu, fv));
}

__device__ __forceinline__ uint32_t shade_avx_texel(const FrameParams &fp, const Texel4 &c4, float z, float n0,
                                                    float n1, float n2, int32_t x, int32_t i, int32_t Row) {
    const float CA = c4.a, CR = c4.r, CG = c4.g, CB = c4.b;
    // Phong (2040-2128) at UnprojectVertex_8x (102-145), with the shading camera
    // (Commands as the span reads it, 2042-2046).
    const float d = fp.sh.D - z;
    const float Xf = (float)(x - i) + (float)i, Yf = (float)Row + 0.0f;
    const float AX = (Xf - fp.sh.Cx) * fp.sh.InvM2P, AY = (Yf - fp.sh.Cy) * fp.sh.InvM2P;
    const float dF = div_focal(fp, d);
    const float PX = dF * AX, PY = dF * AY, PZ = z;
    float Fr = 0, Fg = 0, Fb = 0, Fa = 0;
    for (uint32_t li = 0; li < fp.sh.light_count; ++li) {
        if (li == 0) {
            Fr = CR * fp.sh.amb[0]; Fg = CG * fp.sh.amb[1];
            Fb = CB * fp.sh.amb[2]; Fa = CA * fp.sh.amb[3];
        }
        float Lx = fp.sh.lp[li][0] - PX, Ly = fp.sh.lp[li][1] - PY, Lz = fp.sh.lp[li][2] - PZ;
        normalize_div(Lx, Ly, Lz);
        const float Cos = minps(1.0f, maxps(0.0f, (n0 * Lx + n1 * Ly) + n2 * Lz));
        float Vx = 0.0f - PX, Vy = 0.0f - PY, Vz = 0.0f - PZ;
        normalize_div(Vx, Vy, Vz);
        float Hx = Lx + Vx, Hy = Ly + Vy, Hz = Lz + Vz;
        normalize_div(Hx, Hy, Hz);
        float Ph = minps(1.0f, maxps(0.0f, (n0 * Hx + n1 * Hy) + n2 * Hz));
        Ph = Ph * Ph; Ph = Ph * Ph; Ph = Ph * Ph; Ph = Ph * Ph;
        const float *I = fp.sh.li[li];
        Fr = Fr + ((Cos * (CR * I[0])) + (Ph * (1.0f * I[0])));
        Fg = Fg + ((Cos * (CG * I[1])) + (Ph * (1.0f * I[1])));
        Fb = Fb + ((Cos * (CB * I[2])) + (Ph * (1.0f * I[2])));
        Fa = Fa + ((Cos * (CA * I[3])) + (Ph * (1.0f * I[3])));
    }
    Fr = maxps(minps(Fr, 1.0f), 0.0f);  // 2131-2134
    Fg = maxps(minps(Fg, 1.0f), 0.0f);
    Fb = maxps(minps(Fb, 1.0f), 0.0f);
    Fa = maxps(minps(Fa, 1.0f), 0.0f);
    return ((uint32_t)cvt_rne_s32(Fr * 255.0f) << 16) | ((uint32_t)cvt_rne_s32(Fg * 255.0f) << 8) |
           ((uint32_t)cvt_rne_s32(Fb * 255.0f)) | ((uint32_t)cvt_rne_s32(Fa * 255.0f) << 24);
}

__device__ __forceinline__ uint32_t shade_avx(const FrameParams &fp, const TexRec &tex, float fu, float fv,
                                              float z, float n0, float n1, float n2, int32_t x, int32_t i,
                                              int32_t Row) {
    return shade_avx_texel(fp, sample_avx(tex, fu, fv), z, n0, n1, n2, x, i, Row);
}

// Item j of an AVX span: lane chain i = (xa + j - LeftXa) & 7 from block b.
template <bool SHADE, bool UNI, class WS>
__device__ __forceinline__ void item_avx(const FrameParams &fp, const TileCtx &tc, const WS &ws, int s,
                                         int j, int32_t Row) {
    const int32_t xa = ws.i[SI_XA][s], xb = ws.i[SI_XB][s], LeftXa = ws.i[SI_LEFT][s];
    const uint32_t tag = (uint32_t)ws.i[SI_TAG][s];
    const int rowoff = (Row - tc.y0) * tc.tw - tc.x0;
    int32_t x = xa + j;
    if (SHADE) {
        bool any = false;
        for (int32_t xx = x; xx < xb; xx += 8) any |= is_winner(tc, rowoff + xx, tag);
        if (!any) return;
    }
    // The texture of the span's draw (the item may run on any lane).
    TexRec tex;
    if constexpr (SHADE) tex = UNI ? fp.tex0 : fp.texs[ws.i[SI_TEX][s]];
    else { tex.mem = nullptr; tex.w = tex.h = tex.pitch = tex.filter = 0; }
    const int32_t rel = x - LeftXa, i = rel & 7, b = rel >> 3;
    const float IW = ws.f[SF_IW][s], IU = ws.f[SF_IU][s], IV = ws.f[SF_IV][s], IZ = ws.f[SF_IZ][s];
    const float IW8 = IW * 8.0f, IU8 = IU * 8.0f, IV8 = IV * 8.0f, IZ8 = 8.0f * IZ;
    const float o = ws.f[SF_XOFF][s] + (float)i;  // lane init (XOffset + i)*inc, 1712-1835
    float w = ws.f[SF_LW][s] + o * IW, u = ws.f[SF_LU][s] + o * IU;
    float v = ws.f[SF_LV][s] + o * IV, z = ws.f[SF_LZ][s] + o * IZ;
    float n0 = 0, n1 = 0, n2 = 0, IN08 = 0, IN18 = 0, IN28 = 0;
    if constexpr (SHADE) {
        const float IN0 = ws.f[SF_IN0][s], IN1 = ws.f[SF_IN1][s], IN2 = ws.f[SF_IN2][s];
        IN08 = IN0 * 8.0f; IN18 = IN1 * 8.0f; IN28 = IN2 * 8.0f;
        n0 = ws.f[SF_LN0][s] + o * IN0; n1 = ws.f[SF_LN1][s] + o * IN1; n2 = ws.f[SF_LN2][s] + o * IN2;
        normalize_div(n0, n1, n2);  // 1754
    }
    for (int32_t k = 0; k < b; ++k) {  // block steps 2262-2282
        if (SHADE) {
            float a = n0 + IN08, bb = n1 + IN18, c = n2 + IN28;
            normalize_div(a, bb, c);
            n0 = a; n1 = bb; n2 = c;
        }
        z = z + IZ8; w = w + IW8; u = u + IU8; v = v + IV8;
    }
    for (; x < xb; x += 8) {
        const int p = rowoff + x;
        if (!SHADE) {
            // A key not above the pixel's current maximum cannot change it,
            // whatever the UV mask says: skip the 1/w and the mask.
            const unsigned long long k = make_key(z, tag);
            if (!PRK_ZPRE || k > tc.key[p]) {
                const float iw = 1.0f / w;  // 1865-1866
                const float fu = iw * u, fv = iw * v;
                if (fu >= 0.0f && fu <= 1.0f && fv >= 0.0f && fv <= 1.0f && z == z) atomicMax(&tc.key[p], k);
            }
        } else {
            if (is_winner(tc, p, tag)) {
                const float iw = 1.0f / w;  // 1865-1866
                const float fu = iw * u, fv = iw * v;
                put_winner(fp, x, Row, z, (PRK_DIAG & 16) ? __float_as_uint(fu + fv + n0 + n1 + n2)
                                                         : shade_avx(fp, tex, fu, fv, z, n0, n1, n2, x, i, Row));
            }
            if (x + 8 < xb) {
                float a = n0 + IN08, bb = n1 + IN18, c = n2 + IN28;
                normalize_div(a, bb, c);
                n0 = a; n1 = bb; n2 = c;
            }
        }
        z = z + IZ8; w = w + IW8; u = u + IU8; v = v + IV8;
    }
}

// Visibility item j of an AVX span (PRK_VIS_GROUP = G > 0): the G consecutive
// pixels xa + G*j ... of the span, each evaluated from its own lane chain
// (lane init + b block steps, the recurrence item_avx walks), so one item's
// slot reads and item->span mapping serve G fragments.
template <class WS>
__device__ __forceinline__ void item_vis_group(const TileCtx &tc, const WS &ws, int s, int j, int32_t Row) {
    constexpr int G = PRK_VIS_GROUP > 0 ? PRK_VIS_GROUP : 1;
    const int32_t xa = ws.i[SI_XA][s], xb = ws.i[SI_XB][s], LeftXa = ws.i[SI_LEFT][s];
    const uint32_t tag = (uint32_t)ws.i[SI_TAG][s];
    const int rowoff = (Row - tc.y0) * tc.tw - tc.x0;
    const float IW = ws.f[SF_IW][s], IU = ws.f[SF_IU][s], IV = ws.f[SF_IV][s], IZ = ws.f[SF_IZ][s];
    const float IW8 = IW * 8.0f, IU8 = IU * 8.0f, IV8 = IV * 8.0f, IZ8 = 8.0f * IZ;
    const float XO = ws.f[SF_XOFF][s], LW = ws.f[SF_LW][s], LU = ws.f[SF_LU][s], LV = ws.f[SF_LV][s];
    const float LZ = ws.f[SF_LZ][s];
    const int32_t x0 = xa + G * j;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int32_t x = x0 + g;
        if (x < xb) {
            const int32_t rel = x - LeftXa, i = rel & 7, b = rel >> 3;
            const float o = XO + (float)i;  // lane init (XOffset + i)*inc, 1712-1835
            float w = LW + o * IW, u = LU + o * IU, v = LV + o * IV, z = LZ + o * IZ;
            for (int32_t k = 0; k < b; ++k) { z = z + IZ8; w = w + IW8; u = u + IU8; v = v + IV8; }  // 2262-2282
            const int p = rowoff + x;
            // A key not above the pixel's current maximum cannot change it,
            // whatever the UV mask says: skip the 1/w and the mask.
            const unsigned long long k = make_key(z, tag);
            if (!PRK_ZPRE || k > tc.key[p]) {
                const float iw = 1.0f / w;  // 1865-1866
                const float fu = iw * u, fv = iw * v;
                if (fu >= 0.0f && fu <= 1.0f && fv >= 0.0f && fv <= 1.0f && z == z) atomicMax(&tc.key[p], k);
            }
        }
    }
}

// Shading item j of an AVX span: the span's j-th won pixel.  Its lane chain
// i = (x - LeftXa) & 7 is replayed from the lane init through b block steps
// (the same recurrence item_avx walks), so every lane of the wave shades one
// winning pixel instead of one chain that may hold none.
template <bool UNI>
__device__ __forceinline__ void item_avx_pixel(const FrameParams &fp, const TileCtx &tc, const ShadeSlots &ws, int s,
                                               int j, int32_t Row) {
    const int32_t xa = ws.i[SI_XA][s], LeftXa = ws.i[SI_LEFT][s];
    const uint32_t tag = (uint32_t)ws.i[SI_TAG][s];
    int32_t x = xa;
    uint64_t wm = (uint64_t)(uint32_t)ws.i[SI_WM0][s] | ((uint64_t)(uint32_t)ws.i[SI_WM1][s] << 32);
    int k = j;
    for (; k > 0 && wm; --k) wm &= wm - 1;  // drop the j lowest won columns
    if (wm) {
        x += (int32_t)__builtin_ctzll(wm);
    } else {  // past the span's first 64 columns
        const int rowoff = (Row - tc.y0) * tc.tw - tc.x0;
        for (x = xa + 64;; ++x) {
            if (is_winner(tc, rowoff + x, tag)) {
                if (k == 0) break;
                --k;
            }
        }
    }
    const TexRec tex = UNI ? fp.tex0 : fp.texs[ws.i[SI_TEX][s]];
    const int32_t rel = x - LeftXa, i = rel & 7, b = rel >> 3;
    const float IW = ws.f[SF_IW][s], IU = ws.f[SF_IU][s], IV = ws.f[SF_IV][s], IZ = ws.f[SF_IZ][s];
    const float o = ws.f[SF_XOFF][s] + (float)i;  // lane init (XOffset + i)*inc, 1712-1835
    float w = ws.f[SF_LW][s] + o * IW, u = ws.f[SF_LU][s] + o * IU;
    float v = ws.f[SF_LV][s] + o * IV, z = ws.f[SF_LZ][s] + o * IZ;
    {
        const float IW8 = IW * 8.0f, IU8 = IU * 8.0f, IV8 = IV * 8.0f, IZ8 = 8.0f * IZ;
        for (int32_t k = 0; k < b; ++k) { z = z + IZ8; w = w + IW8; u = u + IU8; v = v + IV8; }  // 2262-2282
    }
    const float iw = 1.0f / w;  // 1865-1866
    const float fu = iw * u, fv = iw * v;
    // The texel load goes out before the normal's block steps.
    const Texel4 t = sample_avx(tex, fu, fv);
    const float IN0 = ws.f[SF_IN0][s], IN1 = ws.f[SF_IN1][s], IN2 = ws.f[SF_IN2][s];
    float n0 = ws.f[SF_LN0][s] + o * IN0, n1 = ws.f[SF_LN1][s] + o * IN1, n2 = ws.f[SF_LN2][s] + o * IN2;
    normalize_div(n0, n1, n2);  // 1754
    {
        const float IN08 = IN0 * 8.0f, IN18 = IN1 * 8.0f, IN28 = IN2 * 8.0f;
        for (int32_t k = 0; k < b; ++k) {  // block steps 2262-2282
            float a = n0 + IN08, bb = n1 + IN18, c = n2 + IN28;
            normalize_div(a, bb, c);
            n0 = a; n1 = bb; n2 = c;
        }
    }
    put_winner(fp, x, Row, z, (PRK_DIAG & 16) ? __float_as_uint(fu + fv + n0 + n1 + n2 + t.r)
                                               : shade_avx_texel(fp, t, z, n0, n1, n2, x, i, Row));
}

// Chunk j of a DrawModel span (projekt.cpp:423-538) restricted to the tile:
// pixels [xa + j*K, min(xa + (j+1)*K, xb)), or (j past the last chunk) the
// one-past-the-row pixel x == W stored at (Row + 1, 0).
template <int M, bool SHADE, bool UNI, class WS>
__device__ __forceinline__ void item_scalar(const FrameParams &fp, const TileCtx &tc, const WS &ws, int s,
                                            int j, int32_t Row) {
    using TR = ModeTraits<M>;
    constexpr int K = kScChunk<SHADE>;
    const int32_t W = fp.W;
    const int32_t xa = ws.i[SI_XA][s], xb = ws.i[SI_XB][s], MinX = ws.i[SI_LEFT][s];
    const uint32_t tag = (uint32_t)ws.i[SI_TAG][s];
    const int povf = ws.i[SI_OVF][s];
    const int rowoff = (Row - tc.y0) * tc.tw - tc.x0;
    const bool reg = j < scalar_chunks<SHADE>(xa, xb);
    const int32_t cx0 = reg ? xa + j * K : W;
    const int32_t cx1 = reg ? min(cx0 + K, xb) : W + 1;
    if (SHADE) {
        bool any = false;
        for (int32_t x = cx0; x < cx1; ++x) any |= is_winner(tc, x == W ? povf : rowoff + x, tag);
        if (!any) return;
    }
    TexRec tex;
    if constexpr (SHADE && TR::tex) tex = UNI ? fp.tex0 : fp.texs[ws.i[SI_TEX][s]];  // the span's draw, not this lane's
    else { tex.mem = nullptr; tex.w = tex.h = tex.pitch = tex.filter = 0; }
    float z = ws.f[SS_Z][s];
    const float IZ = ws.f[SS_IZ][s];
    float w = 0, u = 0, v = 0, IW = 0, IU = 0, IV = 0, n0 = 0, n1 = 0, n2 = 0, IN0 = 0, IN1 = 0, IN2 = 0;
    float c0 = 0, c1 = 0, c2 = 0, c3 = 0, IC0 = 0, IC1 = 0, IC2 = 0, IC3 = 0;
    if constexpr (SHADE) {
        if (TR::tex) {
            w = ws.f[SS_W][s]; u = ws.f[SS_U][s]; v = ws.f[SS_V][s];
            IW = ws.f[SS_IW][s]; IU = ws.f[SS_IU][s]; IV = ws.f[SS_IV][s];
        }
        if (TR::phong) {
            n0 = ws.f[SS_N0][s]; n1 = ws.f[SS_N1][s]; n2 = ws.f[SS_N2][s];
            IN0 = ws.f[SS_IN0][s]; IN1 = ws.f[SS_IN1][s]; IN2 = ws.f[SS_IN2][s];
        }
        if (TR::color) {
            c0 = ws.f[SS_C0][s]; c1 = ws.f[SS_C1][s]; c2 = ws.f[SS_C2][s]; c3 = ws.f[SS_C3][s];
            IC0 = ws.f[SS_IC0][s]; IC1 = ws.f[SS_IC1][s]; IC2 = ws.f[SS_IC2][s]; IC3 = ws.f[SS_IC3][s];
        }
    }
    // The per-pixel steps of pixels [MinX, cx0) (504-510 / 530-535): the
    // same adds in the same order as the reference's loop, nothing else.
#pragma unroll 4
    for (int32_t x = MinX; x < cx0; ++x) {
        if (SHADE) {
            if (TR::phong) {
                float a = n0 + IN0, b = n1 + IN1, c = n2 + IN2;
                normalize_rcp(a, b, c);
                n0 = a; n1 = b; n2 = c;
            }
            if (TR::color) { c0 = c0 + IC0; c1 = c1 + IC1; c2 = c2 + IC2; c3 = c3 + IC3; }
            if (TR::tex) { w += IW; u += IU; v += IV; }
        }
        z += IZ;
    }
    for (int32_t x = cx0; x < cx1; ++x) {  // 423: sequential per-pixel stepping
        {
            const int p = x == W ? povf : rowoff + x;
            if (!SHADE) {
                if (z == z) atomicMax(&tc.key[p], make_key(z, tag));
            } else if (is_winner(tc, p, tag)) {
                float C[4] = {c0, c1, c2, c3};
                if (TR::tex) {  // 427-446
                    const float sc = 1.0f / w;
                    const float FU = sc * u, FV = sc * v;
                    const int32_t TX = round_s32(FU * (float)(tex.w - 1));
                    const int32_t TY = round_s32(FV * (float)(tex.h - 1));
                    const uint32_t t =
                        texel_at(tex, (int32_t)((uint32_t)TX * 4u + (uint32_t)TY * (uint32_t)tex.pitch));
                    C[3] = u8_unit((t >> 24) & 0xFF);  // (r32)byte / 255.0f
                    C[0] = u8_unit((t >> 16) & 0xFF);
                    C[1] = u8_unit((t >> 8) & 0xFF);
                    C[2] = u8_unit(t & 0xFF);
                }
                float F[4];
                if (TR::phong) {  // 448-484 with UnprojectVertex (147-160); the shading camera (452-458)
                    const float d = fp.sh.D - z;
                    const float dF = div_focal(fp, d);
                    const float PX = dF * (((float)x - fp.sh.Cx) * fp.sh.InvM2P);
                    const float PY = dF * (((float)Row - fp.sh.Cy) * fp.sh.InvM2P);
                    const float PZ = z;
                    F[0] = F[1] = F[2] = F[3] = 0.0f;
                    for (uint32_t li = 0; li < fp.sh.light_count; ++li) {
                        if (li == 0)
                            for (int c = 0; c < 4; ++c) F[c] = C[c] * fp.sh.amb[c];
                        float Lx = fp.sh.lp[li][0] - PX, Ly = fp.sh.lp[li][1] - PY, Lz = fp.sh.lp[li][2] - PZ;
                        normalize_rcp(Lx, Ly, Lz);
                        const float Cos = clamp01((n0 * Lx + n1 * Ly) + n2 * Lz);
                        float Vx = -PX, Vy = -PY, Vz = -PZ;
                        normalize_rcp(Vx, Vy, Vz);
                        float Hx = Lx + Vx, Hy = Ly + Vy, Hz = Lz + Vz;
                        normalize_rcp(Hx, Hy, Hz);
                        float Ph = clamp01((n0 * Hx + n1 * Hy) + n2 * Hz);
                        // pow((double)Ph, 16.0) (473) as four exact-range
                        // double squarings: within 2 ulp(double) of any libm's
                        // pow, the same float after the cast except within
                        // ~2^-50 of a float rounding boundary (the ±1 LSB of
                        // the scalar Phong contract); no f64 log/exp.
                        double ph = (double)Ph;
                        ph = ph * ph; ph = ph * ph; ph = ph * ph; ph = ph * ph;
                        Ph = (float)ph;
                        for (int c = 0; c < 4; ++c)
                            F[c] = F[c] + ((Cos * (C[c] * fp.sh.li[li][c])) + (Ph * (1.0f * fp.sh.li[li][c])));
                    }
                    for (int c = 0; c < 4; ++c) F[c] = clamp01(F[c]);
                } else {
                    for (int c = 0; c < 4; ++c) F[c] = C[c];  // 515, no clamp
                }
                const uint32_t packed = (round_u32(F[3] * 255.0f) << 24) | (round_u32(F[0] * 255.0f) << 16) |
                                        (round_u32(F[1] * 255.0f) << 8) | (round_u32(F[2] * 255.0f));
                if (x == W) put_winner(fp, 0, Row + 1, z, packed);  // DrawModel's one-past-the-row store
                else put_winner(fp, x, Row, z, packed);
            }
        }
        if (SHADE) {  // per-pixel step (504-510 / 530-535)
            if (TR::phong) {
                float a = n0 + IN0, b = n1 + IN1, c = n2 + IN2;
                normalize_rcp(a, b, c);
                n0 = a; n1 = b; n2 = c;
            }
            c0 = c0 + IC0; c1 = c1 + IC1; c2 = c2 + IC2; c3 = c3 + IC3;
            w += IW; u += IU; v += IV;
        }
        z += IZ;
    }
}

// Wave64 inclusive prefix sum / max in registers (DPP row shifts + row
// broadcasts: no LDS round trips).
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
    (void)lane;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}
__device__ __forceinline__ int wave_incl_max(int v) {  // v >= 0
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));
    return v;
}


// The walker of a sweep's row loop.  PRK_VIS_PERM: the visibility sweep
// keeps the three edges in fixed registers and the list as a permutation
// (Walker): every row steps and selects a few fields (the span reads X, z,
// 1/z, u/z, v/z of its two edges), and insertion / expiry / the crossing
// swap move two bits.  RowWalker holds the list physically: a row steps two
// edges with no selects, but an insertion, expiry or swap row moves whole
// edges — and with 64 triangles per wave nearly every row has one in some
// lane (about half of the visibility row loop's VALU instructions were those
// moves).
#ifndef PRK_VIS_PERM
#define PRK_VIS_PERM 1
#endif
#ifndef PRK_WALK_PERM
#define PRK_WALK_PERM 0  // 1: k_walk walks with the permutation walker too (normals included): measured k_walk +5 % (three normalisations per row instead of two)
#endif
template <int M, bool SHADE>
using SweepWalker = typename std::conditional<PRK_VIS_PERM && !SHADE, Walker<M, SHADE>, RowWalker<M, SHADE>>::type;
template <int M, bool NRM>
__device__ __forceinline__ void wk_from(RowWalker<M, NRM> &wk, const Walker<M, NRM> &w0) { wk.from(w0); }
template <int M, bool NRM>
__device__ __forceinline__ void wk_from(Walker<M, NRM> &wk, const Walker<M, NRM> &w0) { wk = w0; }
template <int M, bool NRM>
__device__ __forceinline__ void wk_pair(const RowWalker<M, NRM> &wk, Edge &L, Edge &R) { L = wk.S0; R = wk.S1; }
template <int M, bool NRM>
__device__ __forceinline__ void wk_pair(const Walker<M, NRM> &wk, Edge &L, Edge &R) {
    L = wk.get(wk.slot(0));
    R = wk.get(wk.slot(1));
}

// One sweep over the tile's bin for mode M.  SHADE=false: visibility keys;
// SHADE=true: shade the winners.
template <int M, bool SHADE, bool UNI, bool REC = false, class WS>
__device__ __forceinline__ void sweep(const FrameParams &fp, const TileCtx &tc, WS &ws,
                                      const uint2 *__restrict__ bins, uint32_t b0, uint32_t n,
                                      const uint32_t *__restrict__ list, uint32_t *anomaly,
                                      uint32_t *chunk_ctr = nullptr) {
    // Entries [0, n) of the tile's bin, or (list != nullptr) the n entries it names.
    // chunk_ctr (LDS, zeroed): the waves take the bin's 64-entry chunks in
    // turn from this counter, each its next chunk when it finishes one,
    // instead of every nwaves-th chunk (a tile of 6-7 chunks left two of its
    // four waves idle for a chunk's time).
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool col0 = tc.x0 == 0 && M != MODE_AVX;
    const int32_t ystart = col0 ? tc.y0 - 1 : tc.y0;  // scalar: (row-1) may store into (row, 0)
    unsigned long long pt[4] = {0, 0, 0, 0};  // PRK_PROF: setup, walk, scan/map, items
    // PRK_PROF event counts (visibility sweep): chunks, row iterations, item
    // windows, items, active lanes summed over row iterations, spans with items
    unsigned long long pc[7] = {0, 0, 0, 0, 0, 0, 0};
    // Single-draw frames prefetch: the next chunk's bin entry is loaded at the
    // top of a chunk and its vertex attributes before the row walk, so both
    // loads are in flight while this chunk's setup and rows run.
    constexpr bool kPre = UNI && PRK_PREFETCH && !SHADE;  // (k_shade has no registers to spare)
    TriRaw<M> nraw;
    uint32_t ne_e = 0, ne_g = 0, ne_j = 0;
    if constexpr (kPre) {
        const uint32_t i0 = wave * 64 + lane;
        if (i0 < n) {
            ne_e = list ? list[b0 + i0] : i0;
            const uint2 be = bins[b0 + ne_e];
            ne_g = be.x;
            ne_j = be.y;
            load_tri<M>(fp.draw0, fp.draw0.geom_tri0 + (ne_g - fp.draw0.first_global), nraw);
        }
    }
    const uint32_t nwaves = blockDim.x >> 6;
    auto next_chunk = [&](uint32_t cur) -> uint32_t {
        if (kPre || !chunk_ctr) return cur + 64 * nwaves;
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(chunk_ctr, 64u);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
    };
    const uint32_t first = (kPre || !chunk_ctr) ? wave * 64 : next_chunk(0);
    // Setup-record sweeps take the next chunk when they start one and load
    // its bin entries while this chunk runs, so a chunk's first load is its
    // records (bin entry -> record were two dependent round trips).
    constexpr bool kPreBin = REC && !SHADE && !kPre && PRK_VIS_PREBIN;
    uint2 pbe = make_uint2(0u, 0u);
    if (kPreBin && !list && first + lane < n) pbe = bins[b0 + first + lane];
    for (uint32_t base = first, nb = 0; base < n; base = nb) {
        const uint2 cbe = pbe;
        nb = next_chunk(base);
        if (kPreBin && !list && nb + lane < n) pbe = bins[b0 + nb + lane];
        unsigned long long t0 = PRK_T();
        const uint32_t i = base + lane;
        bool active = i < n;
        if (PRK_PROF) pc[0] += 1;
        uint32_t e = 0, j = 0;  // bin entry, its pair index (the tie-break order)
        uint32_t st = 0;        // DRAW_ST: single-thread DrawModelOptimized(Buffer,...) semantics
        int32_t texi = 0;
        SweepWalker<M, SHADE> wk;
        uint32_t anom = 0;
        TriRaw<M> craw;
        const uint32_t inext = i + 64 * nwaves;
        if constexpr (kPre) {
            craw = nraw;
            e = ne_e;
            j = ne_j;
            if (inext < n) {
                ne_e = list ? list[b0 + inext] : inext;
                const uint2 be = bins[b0 + ne_e];
                ne_g = be.x;
                ne_j = be.y;
            }
        }
        if (active) {
            if constexpr (!kPre) {
                e = list ? list[b0 + i] : i;
                j = (kPreBin && !list) ? cbe.y : bins[b0 + e].y;
            }
            Edge s0, s1, s2;
            int ne;
            uint32_t rhead = 0;
            if constexpr (REC) {
                // Setup record of the binning pass: no per-entry FillEdgeTable.
                const uint32_t g = (kPreBin && !list) ? cbe.x : bins[b0 + e].x;
                const float4 *q = reinterpret_cast<const float4 *>(fp.trec + g);
                float4 v[10];
#pragma unroll
                for (int k = 0; k < 10; ++k) v[k] = q[k];
                const float *f = reinterpret_cast<const float *>(v);
                const int32_t *iw = reinterpret_cast<const int32_t *>(v);
                s0 = rec_edge_in(f + 0, iw[30], iw[33]);
                s1 = rec_edge_in(f + 10, iw[31], iw[34]);
                s2 = rec_edge_in(f + 20, iw[32], iw[35]);
                rhead = (uint32_t)iw[36];
                ne = (int)(rhead & 0xFu);
                anom = (rhead >> 20) & 0xFu;
                st = (rhead >> 24) & 1u;
            } else if constexpr (kPre) {
                ne = setup_from_raw<M>(craw, fp.draw0, fp, s0, s1, s2);
                texi = fp.draw0.tex;
                st = fp.draw0.flags & DRAW_ST;
            } else if constexpr (UNI) {  // one draw: its record is uniform (kernel arguments)
                const uint32_t g = bins[b0 + e].x;
                const uint32_t gt = fp.draw0.geom_tri0 + (g - fp.draw0.first_global);
                ne = setup_triangle<M>(fp.draw0, gt, fp, s0, s1, s2);
                texi = fp.draw0.tex;
                st = fp.draw0.flags & DRAW_ST;
            } else {
                const uint32_t g = bins[b0 + e].x;
                const DrawRec *d;
                uint32_t gt;
                resolve_draw(fp, g, d, gt);
                // (mixed frames sweep the bin once per mode)
                ne = d->mode == M ? setup_triangle<M>(*d, gt, fp, s0, s1, s2) : 0;
                texi = d->tex;
                st = d->flags & DRAW_ST;
            }
            active = ne >= 2;
            if (active) {
                Walker<M, SHADE> w0;
                if constexpr (REC) w0.init_rec(ne, s0, s1, s2, fp.H, tc.y1, rhead);
                else w0.init(ne, s0, s1, s2, fp.H, tc.y1, anom);
                // Replay the rows above the tile (edge DDA only); row by row
                // only for irregular edge lists.
                const int fr = w0.fast_replay(ystart, ne);
                wk_from(wk, w0);
                if (fr < 0)
                    while (wk.Row < ystart && wk.Row < wk.MaxY) wk.end_row(wk.begin_row());
                if (fr != 0 && !SHADE) atomicAdd(anomaly + 1, 1u);
                active = wk.Row < wk.MaxY;
            }
        }
        if constexpr (kPre) {
            if (inext < n) load_tri<M>(fp.draw0, fp.draw0.geom_tri0 + (ne_g - fp.draw0.first_global), nraw);
        }
        if (anom) atomicAdd(anomaly, anom);
        if (!(ModeTraits<M>::tex && active)) texi = 0;
        // Visibility tag: the pair index orders fragments of equal z exactly as
        // submission order does (pairs are numbered in triangle order, one per
        // triangle and tile), whatever order the bin lists them in.
        const uint32_t tag = pair_tag(j, st != 0);
        if (PRK_DIAG & 4) active = false;
        if (PRK_PROF) { const unsigned long long t1 = PRK_T(); pt[0] += t1 - t0; t0 = t1; }
        // PRK_LANE_ROWS: every lane walks its own next row each iteration (the
        // span's row travels in its slot); else all lanes step row r together.
        if (PRK_LANE_ROWS && active) active = wk.Row < tc.y1;
        for (int32_t r = ystart; PRK_LANE_ROWS || r < tc.y1; ++r) {
            // Rows per lane this iteration: when few lanes still hold rows, each
            // emits up to 8 of its next rows into the wave's 64 span slots
            // (slot = rank among the active lanes * k + q), so the items of
            // several rows share one window and the rows' per-pixel recurrences
            // run side by side instead of one row after another.
            int k = 1, rank = 0;
            if (PRK_PROF) { pc[1] += 1; pc[4] += (unsigned long long)__popcll(__ballot(active)); }
            if (PRK_LANE_ROWS && PRK_MULTI_ROWS) {
                const unsigned long long am = __ballot(active);
                const int A = __popcll(am);
                if (M != MODE_AVX) k = A <= 8 ? 8 : (A <= 16 ? 4 : (A <= 32 ? 2 : 1));
                else k = A <= PRK_MULTI_ROWS_AVX ? 8 : 1;  // (AVX: only near-idle waves; C3b measured 2 % slower otherwise)
                rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
            }
            const bool multi = k > 1;
            int items = 0;
            if (multi) {  // per-slot item counts go through SI_PRE (rewritten after the scan)
                ws.i[SI_PRE][lane] = 0;
                wave_lds_sync();
            }
            for (int q = 0; q < k; ++q) {
                if (active && (PRK_LANE_ROWS || wk.Row == r)) {
                    const int slot = multi ? rank * k + q : lane;
                    const int32_t row = wk.Row;
                    const bool paired = wk.begin_row();
                    if (paired) {
                        Edge L, R;
                        wk_pair(wk, L, R);
                        int ni;
                        if constexpr (M == MODE_AVX) ni = span_setup_avx<SHADE>(fp, tc, ws, slot, tag, texi, L, R, row, st != 0);
                        else ni = span_setup_scalar<M, SHADE>(fp, tc, ws, slot, tag, texi, L, R, row);
                        ws.i[SI_ROW][slot] = row;
                        if (multi) ws.i[SI_PRE][slot] = ni;
                        else items = ni;
                    }
                    wk.end_row(paired);
                    active = wk.Row < wk.MaxY && (!PRK_LANE_ROWS || wk.Row < tc.y1);
                }
            }
            if (multi) {
                wave_lds_sync();
                items = ws.i[SI_PRE][lane];
            }
            if (PRK_PROF) { const unsigned long long t1 = PRK_T(); pt[1] += t1 - t0; t0 = t1; }
            const int incl = wave_incl_scan(items, lane);
            const int total = __builtin_amdgcn_readlane(incl, 63);
            const int excl = incl - items;
            ws.i[SI_PRE][lane] = excl;
            if (PRK_PROF) {
                pc[2] += (unsigned long long)((total + 63) / 64);
                pc[3] += (unsigned long long)total;
                pc[5] += (unsigned long long)__popcll(__ballot(items > 0));
            }
            // Item -> span: the span lanes starting an item inside the window
            // mark their start position; a prefix max over the window (plus
            // the span carried over from the previous window) names the span
            // of every item.
            int carry = 0;
            if (PRK_PROF) { const unsigned long long t1 = PRK_T(); pt[2] += t1 - t0; t0 = t1; }
            for (int it0 = 0; it0 < (((PRK_DIAG & 2) || ((PRK_DIAG & 8) && SHADE)) ? 0 : total); it0 += 64) {
                ws.i[SI_MARK][lane] = 0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (items > 0 && excl >= it0 && excl < it0 + 64) ws.i[SI_MARK][excl - it0] = lane + 1;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int m = max(wave_incl_max(ws.i[SI_MARK][lane]), carry);
                carry = __builtin_amdgcn_readlane(m, 63);
                const int it = it0 + lane;
                if (it < total) {
                    const int s = m - 1, j = it - ws.i[SI_PRE][s];
                    const int32_t srow = ws.i[SI_ROW][s];
                    if constexpr (M == MODE_AVX && SHADE && PRK_PIXEL_ITEMS) item_avx_pixel<UNI>(fp, tc, ws, s, j, srow);
                    else if constexpr (M == MODE_AVX && !SHADE && PRK_VIS_GROUP > 0) item_vis_group(tc, ws, s, j, srow);
                    else if constexpr (M == MODE_AVX) item_avx<SHADE, UNI>(fp, tc, ws, s, j, srow);
                    else item_scalar<M, SHADE, UNI>(fp, tc, ws, s, j, srow);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (PRK_PROF) { const unsigned long long t1 = PRK_T(); pt[3] += t1 - t0; t0 = t1; }
            if (!__any(active)) break;
        }
    }
    if (PRK_PROF && lane == 0)
        for (int k = 0; k < 4; ++k) atomicAdd(fp.prof + (SHADE ? 4 : 0) + k, pt[k]);
    if (PRK_PROF && !SHADE && lane == 0)
        for (int k = 0; k < 7; ++k) atomicAdd(fp.prof + 8 + k, pc[k]);
}

// Workgroup-wide exclusive scan of one value per thread.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *scratch, uint32_t &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan((int)v, lane);
    if (lane == 63) scratch[wave] = (uint32_t)incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wave) before += scratch[w];
        total += scratch[w];
    }
    __syncthreads();
    return before + (uint32_t)incl - v;
}

__device__ __forceinline__ TileCtx tile_ctx(const FrameParams &fp, int t) {
    const int tx = t % fp.tiles_x, ty = t / fp.tiles_x;
    TileCtx tc;
    tc.tw = fp.tile_w;
    tc.x0 = tx * fp.tile_w;
    tc.x1 = min(fp.W, tc.x0 + fp.tile_w);
    tc.y0 = fp.row0 + ty * fp.tile_h;
    tc.y1 = min(fp.row1, tc.y0 + fp.tile_h);
    tc.key = nullptr;
    tc.tags = nullptr;
    return tc;
}

// Visibility (sweep 1), one workgroup per tile.  MODESET: a single Mode, or
// -1: any mode (a mixed frame sweeps the bin once per mode, each skipping the
// other modes' entries).  UNI: the frame is one draw (then MODESET is its mode).
// Output per tile: the winning entry tag of every pixel (wtag, tile-major),
// the list of bin entries that won at least one pixel and its length.
template <int MODESET, bool UNI, bool ZV = false>  // ZV: write the z here, k_pix the colour (fp.z_in_vis)
__global__ void __launch_bounds__(64 * kVisWaves, PRK_VIS_MIN_WAVES)
    k_vis(FrameParams fp, const uint32_t *__restrict__ offs, const uint2 *__restrict__ bins,
          uint8_t *__restrict__ won, uint32_t *__restrict__ list, uint32_t *__restrict__ nwin_out,
          uint32_t *__restrict__ wtag, const uint32_t *__restrict__ pair_tri, uint8_t *__restrict__ trwon,
          uint32_t *__restrict__ anomaly) {
    // Span-record frames (all draws AVX): k_walk + k_pix shade from the
    // winner tags; k_vis marks the won (pair, row)s and triangles for them.
    constexpr bool kRec = MODESET == MODE_AVX && PRK_SPAN_RECORDS;
    constexpr bool kZV = kRec && ZV;
    extern __shared__ unsigned long long lds[];
    const int ntile = fp.tiles_x * fp.tiles_y;
    const int t = blockIdx.x;
    if (t >= ntile) return;
    const uint32_t b0 = offs[t], b1 = offs[t + 1];
    if (b0 == b1) {  // no triangle touches this tile: leave it untouched
        if (threadIdx.x == 0) nwin_out[t] = 0;
        if (kZV && fp.clear_fused) {  // (the fused clear's z: k_pix writes its colour)
            const TileCtx tc = tile_ctx(fp, t);
            for (int p = threadIdx.x; p < fp.tile_w * fp.tile_h; p += blockDim.x) {
                const int x = tc.x0 + (p & (fp.tile_w - 1)), y = tc.y0 + (p >> fp.tile_w_log2);
                if (x < tc.x1 && y < tc.y1) fp.zbuf[(size_t)(y - fp.row0) * fp.W + x] = fp.clear_z;
            }
        }
        return;
    }
    const uint32_t n = b1 - b0;
    TileCtx tc = tile_ctx(fp, t);
    const int npx = fp.tile_w * fp.tile_h;
    tc.key = lds;
    VisSlots *slots = reinterpret_cast<VisSlots *>(lds + npx);
    VisSlots &ws = slots[threadIdx.x >> 6];
    uint32_t *scratch = reinterpret_cast<uint32_t *>(slots + kVisWaves);

    if (threadIdx.x == 0) scratch[8] = 0;  // the sweep's chunk counter (PRK_VIS_DYN)
    // Prior z of the target: a fragment must beat it strictly.
    for (int p = threadIdx.x; p < npx; p += blockDim.x) {
        const int lx = p & (fp.tile_w - 1), ly = p >> fp.tile_w_log2;
        const int x = tc.x0 + lx, y = tc.y0 + ly;
        unsigned long long k = ~0ull;
        if (x < tc.x1 && y < tc.y1) {
            const float z = fp.clear_fused ? fp.clear_z : fp.zbuf[(size_t)(y - fp.row0) * fp.W + x];
            k = (z != z) ? ~0ull : (((unsigned long long)zkey(z) << 32) | kTagPrior);
        }
        tc.key[p] = k;
    }
    __syncthreads();
    if constexpr (MODESET >= 0) {
        // all-AVX frames read the binning pass's setup records (TriRec)
        sweep<(MODESET >= 0 ? MODESET : 0), false, UNI, MODESET == MODE_AVX && PRK_SETUP_REC>(
            fp, tc, ws, bins, b0, n, nullptr, anomaly, PRK_VIS_DYN ? scratch + 8 : nullptr);
    } else {
        sweep<MODE_AVX, false, false>(fp, tc, ws, bins, b0, n, nullptr, anomaly);
        sweep<MODE_SC_GOURAUD, false, false>(fp, tc, ws, bins, b0, n, nullptr, anomaly);
        sweep<MODE_SC_GOURAUD_TEX, false, false>(fp, tc, ws, bins, b0, n, nullptr, anomaly);
        sweep<MODE_SC_PHONG, false, false>(fp, tc, ws, bins, b0, n, nullptr, anomaly);
        sweep<MODE_SC_PHONG_TEX, false, false>(fp, tc, ws, bins, b0, n, nullptr, anomaly);
    }
    __syncthreads();
    // Winner tags out, and which bin entries won at least one pixel.
    uint32_t *tags_out = wtag + (size_t)t * npx;
    int anyw = 0;
    for (int p = threadIdx.x; p < npx; p += blockDim.x) {
        const uint32_t low = (uint32_t)tc.key[p];
        tags_out[p] = low;
        uint32_t j;  // the winning pair
        const bool won_px = tag_pair(low, j);
        if constexpr (kZV) {
            // the pixel's final z (the winner's, from its key, or the fused
            // clear's): k_pix writes only the colour, so z is done here and a
            // download can take it while the frame shades
            const int x = tc.x0 + (p & (fp.tile_w - 1)), y = tc.y0 + (p >> fp.tile_w_log2);
            if (x < tc.x1 && y < tc.y1 && (won_px || fp.clear_fused))
                fp.zbuf[(size_t)(y - fp.row0) * fp.W + x] =
                    won_px ? zkey_z((uint32_t)(tc.key[p] >> 32)) : fp.clear_z;
        }
        if (!won_px) continue;
        if constexpr (kRec) {  // the winner's (pair, row) and triangle (benign same-value races)
            anyw = 1;
            won[(size_t)j * fp.tile_h + (p >> fp.tile_w_log2)] = 1;
            trwon[pair_tri[j]] = 1;
        } else {
            won[j] = 1;
        }
    }
    // Debug builds also export the winning triangle map.
    if (fp.winners) {
        for (int p = threadIdx.x; p < npx; p += blockDim.x) {
            const int x = tc.x0 + (p & (fp.tile_w - 1)), y = tc.y0 + (p >> fp.tile_w_log2);
            if (x >= tc.x1 || y >= tc.y1) continue;
            uint32_t j;  // (the prior contents keep their winner: an earlier pass's, or -1)
            if (tag_pair((uint32_t)tc.key[p], j))
                fp.winners[(size_t)(y - fp.row0) * fp.W + x] = (int32_t)(fp.win_base + pair_tri[j]);
        }
    }
    if constexpr (kRec) {
        anyw = __syncthreads_or(anyw);
        if (threadIdx.x == 0) nwin_out[t] = (PRK_DIAG & 1) ? 0u : (uint32_t)anyw;
        return;
    }
    __threadfence_block();
    __syncthreads();
    // Entries that won at least one pixel of the tile (k_shade walks these).
    uint32_t nwin = 0;
    for (uint32_t base = 0; base < n; base += blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t f = (i < n && won[bins[b0 + i].y]) ? 1u : 0u;
        uint32_t tot;
        const uint32_t pos = block_excl_scan(f, scratch, tot);
        if (f) list[b0 + nwin + pos] = i;
        nwin += tot;
    }
    if (threadIdx.x == 0) nwin_out[t] = (PRK_DIAG & 1) ? 0u : nwin;
}

// Shading (sweep 2), one workgroup per tile: re-walk only the entries that
// won a pixel and shade exactly the winning fragments.  Winners store their
// z and colour; untouched pixels keep the prior contents.
template <int MODESET, bool UNI>
__global__ void __launch_bounds__(64 * kShadeWaves, PRK_SHADE_MIN_WAVES)
    k_shade(FrameParams fp, const uint32_t *__restrict__ offs, const uint2 *__restrict__ bins,
            const uint32_t *__restrict__ list, const uint32_t *__restrict__ nwin_in,
            const uint32_t *__restrict__ wtag, uint32_t *__restrict__ anomaly) {
    extern __shared__ unsigned long long lds[];
    const int ntile = fp.tiles_x * fp.tiles_y;
    const int t = blockIdx.x;
    if (t >= ntile) return;
    const uint32_t nwin = nwin_in[t];
    if (nwin == 0) return;
    const uint32_t b0 = offs[t];
    TileCtx tc = tile_ctx(fp, t);
    const int npx = fp.tile_w * fp.tile_h;
    uint32_t *tags = reinterpret_cast<uint32_t *>(lds);
    tc.tags = tags;
    ShadeSlots *slots = reinterpret_cast<ShadeSlots *>(tags + npx + kTagPad);
    ShadeSlots &ws = slots[threadIdx.x >> 6];
    const uint32_t *tags_in = wtag + (size_t)t * npx;
    for (int p = threadIdx.x; p < npx; p += blockDim.x) tags[p] = tags_in[p];
    if (threadIdx.x < kTagPad) tags[npx + threadIdx.x] = 0xFFFFFFFFu;  // chunked reads run past the end
    __syncthreads();
    if constexpr (MODESET >= 0) {
        sweep<(MODESET >= 0 ? MODESET : 0), true, UNI>(fp, tc, ws, bins, b0, nwin, list, anomaly);
    } else {
        sweep<MODE_AVX, true, false>(fp, tc, ws, bins, b0, nwin, list, anomaly);
        sweep<MODE_SC_GOURAUD, true, false>(fp, tc, ws, bins, b0, nwin, list, anomaly);
        sweep<MODE_SC_GOURAUD_TEX, true, false>(fp, tc, ws, bins, b0, nwin, list, anomaly);
        sweep<MODE_SC_PHONG, true, false>(fp, tc, ws, bins, b0, nwin, list, anomaly);
        sweep<MODE_SC_PHONG_TEX, true, false>(fp, tc, ws, bins, b0, nwin, list, anomaly);
    }
}

// ---------------------------------------------------------------------------
// AVX frames shade in two kernels instead of k_shade's in-wave work items:
//   k_walk  one thread per triangle that won a pixel: setup once, walk the
//           triangle's rows once (normals included) and, for every (pair, row)
//           k_vis marked won, write the span's FillLineOptimized lane-init
//           record (64 B) at recs[pair * tile_h + row in tile];
//   k_pix   one thread per pixel: winner tag -> bin entry -> pair -> record;
//           replays its lane chain from the record, shades (texel + Phong)
//           and stores z and colour, coalesced.
// Each triangle is set up and walked once for shading (a per-tile walk would
// set it up per tile and replay the rows above every tile), and the shading
// runs at full lane occupancy with no walker registers.
// ---------------------------------------------------------------------------
struct SpanRec {  // one won row span (FillLineOptimized span setup, 1543-1835)
    int32_t left_tex;  // LeftXa (low 16 bits) | texture index << 16
    float xoff, lw, lu, lv, lz, iw, iu, iv, iz, ln0, ln1, ln2, in0, in1, in2;
};
static_assert(sizeof(SpanRec) == 64, "span record is four dwordx4");

// k_walk: FillLineOptimized span setup (projekt.cpp:1543-1835) of one row of
// the triangle; for every tile the span crosses whose (pair, row) won a pixel
// in k_vis, write the span's record at recs[pair * tile_h + row-in-tile].
__device__ __forceinline__ void walk_record(const FrameParams &fp, const Edge &L, const Edge &R, int32_t Row,
                                            int32_t texi, const TileRange &tr, uint32_t jb, int ntx,
                                            const uint8_t *__restrict__ won, SpanRec *__restrict__ recs, bool st) {
    if (Row < fp.row0) return;
    float XOffset;
    int32_t MinX, MaxX, XDiff;
    if (!span_ends(L.X, R.X, fp.W, st, MinX, MaxX, XDiff, XOffset)) return;  // 1545-1592
    if (MinX >= MaxX) return;  // [MinX, MaxX) empty
    const int32_t rr = Row - fp.row0, ty = tile_row_of(fp, rr), ly = rr - ty * fp.tile_h;
    if (ty < (int)tr.ty0 || ty > (int)tr.ty1) return;  // (binning covers every span pixel)
    const int tx0 = max((int)tr.tx0, MinX >> fp.tile_w_log2);
    const int tx1 = min((int)tr.tx1, (MaxX - 1) >> fp.tile_w_log2);
    const uint32_t jrow = jb + (uint32_t)((ty - (int)tr.ty0) * ntx - (int)tr.tx0);
    // One tile column and at most 8 tile rows: k_walk queued this row only
    // because its won bit (loaded up front) is set, so the won flags need not
    // be read again here (a dependent load per span).
    const bool known = fp.tile_h == 8 && tr.tx0 == tr.tx1 && (int)tr.ty1 - (int)tr.ty0 < 8;
    if (!known) {
        bool any = false;
        for (int tx = tx0; tx <= tx1; ++tx) any |= won[(size_t)(jrow + tx) * fp.tile_h + ly] != 0;
        if (!any) return;
    }
    int32_t LeftXa = MinX;
    if (MinX & 7) {  // 1594-1609
        LeftXa = MinX & ~7;
        XOffset -= (float)(MinX & 7) * 1.0f;
    }
    const float fXD = (float)XDiff;
    float IW = 0, IU = 0, IV = 0, IZ = 0, IN0 = 0, IN1 = 0, IN2 = 0;
    if (XDiff != 0) {  // 1666-1835
        // the span's increments over XDiff (div_all: one shared reciprocal)
        float q[7] = {R.W - L.W, R.U - L.U, R.V - L.V, R.N0 - L.N0, R.N1 - L.N1, R.N2 - L.N2, R.Z - L.Z};
        div_all(fXD, q);
        IW = q[0]; IU = q[1]; IV = q[2]; IN0 = q[3]; IN1 = q[4]; IN2 = q[5]; IZ = q[6];
    }
    const float4 q0 = make_float4(__int_as_float((LeftXa & 0xFFFF) | (texi << 16)), XOffset, L.W, L.U);
    const float4 q1 = make_float4(L.V, L.Z, IW, IU);
    const float4 q2 = make_float4(IV, IZ, L.N0, L.N1);
    const float4 q3 = make_float4(L.N2, IN0, IN1, IN2);
    for (int tx = tx0; tx <= tx1; ++tx) {  // a span crossing a tile border: one record per won tile
        const size_t ri = (size_t)(jrow + tx) * fp.tile_h + ly;
        if (!known && !won[ri]) continue;
        float4 *q = reinterpret_cast<float4 *>(recs + ri);
        q[0] = q0; q[1] = q1; q[2] = q2; q[3] = q3;
    }
}

// Per-wave queue of won row spans between k_walk's row walk and its record
// writes: the walk finds a won row on only some lanes in a given step, so the
// span setup (7 divisions) and the stores run once 64 spans are queued, one
// per lane.  Entry: both edges' X, W, U, V, z and normal (16 floats), row |
// texture << 16, the triangle's first pair, its tile rectangle (2 words).
constexpr int kWalkWaves = 2, kWalkQ = 128;
struct WalkQueue {
    float f[16][kWalkQ];
    int32_t i[4][kWalkQ];
};

__device__ __forceinline__ void walk_flush(const FrameParams &fp, const WalkQueue &q, int slot,
                                           const uint8_t *__restrict__ won, SpanRec *__restrict__ recs) {
    Edge L, R;
    L.X = q.f[0][slot]; L.W = q.f[1][slot]; L.U = q.f[2][slot]; L.V = q.f[3][slot]; L.Z = q.f[4][slot];
    L.N0 = q.f[5][slot]; L.N1 = q.f[6][slot]; L.N2 = q.f[7][slot];
    R.X = q.f[8][slot]; R.W = q.f[9][slot]; R.U = q.f[10][slot]; R.V = q.f[11][slot]; R.Z = q.f[12][slot];
    R.N0 = q.f[13][slot]; R.N1 = q.f[14][slot]; R.N2 = q.f[15][slot];
    const int32_t rt = q.i[0][slot];
    const uint32_t jb = (uint32_t)q.i[1][slot], t0 = (uint32_t)q.i[2][slot], t1 = (uint32_t)q.i[3][slot];
    TileRange tr;
    tr.tx0 = (uint16_t)(t0 & 0xFFFF); tr.ty0 = (uint16_t)(t0 >> 16);
    tr.tx1 = (uint16_t)(t1 & 0xFFFF); tr.ty1 = (uint16_t)(t1 >> 16);
    walk_record(fp, L, R, rt & 0xFFFF, (rt >> 16) & 0x7FFF, tr, jb, (int)tr.tx1 - (int)tr.tx0 + 1, won, recs,
                (rt >> 31) != 0);
}


// k_walk: one thread per triangle that won a pixel.  FillEdgeTable +
// MergeSort once, then the triangle's whole AET walk (projekt.cpp:3615-3871,
// normals included) from its first row of the band: no per-tile setup and no
// replay of the rows above a tile.  Won rows go through the wave's queue.
template <bool UNI>
__global__ void __launch_bounds__(64 * kWalkWaves, PRK_WALK_MIN_WAVES) k_walk(FrameParams fp, const uint32_t *__restrict__ wlist,
                                              const uint32_t *__restrict__ nwlist,
                                              const uint32_t *__restrict__ tri_off,
                                              const TileRange *__restrict__ ranges, const uint8_t *__restrict__ won,
                                              SpanRec *__restrict__ recs, uint32_t *__restrict__ anomaly) {
    constexpr int M = MODE_AVX;
    __shared__ WalkQueue queues[kWalkWaves];
    const int lane = threadIdx.x & 63;
    WalkQueue &q = queues[threadIdx.x >> 6];
    const uint32_t nw = *nwlist;
    if (blockIdx.x * blockDim.x + (threadIdx.x & ~63u) >= nw) return;  // whole wave past the list
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool active = i < nw;
    const uint32_t g = active ? wlist[i] : 0u;  // the triangles that won a pixel (compacted)
    typename std::conditional<PRK_WALK_PERM, Walker<M, true>, RowWalker<M, true>>::type wk;
    int32_t texi = 0;
    uint32_t st = 0;  // DRAW_ST
    TileRange tr{};
    uint32_t jb = 0;
    uint64_t rows = ~0ull;
    int32_t rbase = 0;
    bool fast = false;
    if (active) {
        Edge s0, s1, s2;
        int ne;
        uint32_t rhead = 0;
        if constexpr (PRK_SETUP_REC) {  // the binning pass's setup record + the vertex normals
            const float4 *q = reinterpret_cast<const float4 *>(fp.trec + g);
            float4 v[10];
#pragma unroll
            for (int k = 0; k < 10; ++k) v[k] = q[k];
            const DrawRec *d = &fp.draw0;
            uint32_t gt;
            if constexpr (UNI) gt = fp.draw0.geom_tri0 + (g - fp.draw0.first_global);
            else resolve_draw(fp, g, d, gt);
            texi = d->tex;
            const float *nv = d->N + 9 * (size_t)gt;
            float n[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) n[k] = nv[k];
            const float *f = reinterpret_cast<const float *>(v);
            const int32_t *iw = reinterpret_cast<const int32_t *>(v);
            s0 = rec_edge_in(f + 0, iw[30], iw[33]);
            s1 = rec_edge_in(f + 10, iw[31], iw[34]);
            s2 = rec_edge_in(f + 20, iw[32], iw[35]);
            const uint32_t vtx = (uint32_t)iw[37];
            nrm_edge_from(s0, vtx, n);
            nrm_edge_from(s1, vtx >> 4, n);
            nrm_edge_from(s2, vtx >> 8, n);
            rhead = (uint32_t)iw[36];
            ne = (int)(rhead & 0xFu);
            st = (rhead >> 24) & 1u;
        } else if constexpr (UNI) {
            ne = setup_triangle<M>(fp.draw0, fp.draw0.geom_tri0 + (g - fp.draw0.first_global), fp, s0, s1, s2);
            texi = fp.draw0.tex;
            st = fp.draw0.flags & DRAW_ST;
        } else {
            const DrawRec *d;
            uint32_t gt;
            resolve_draw(fp, g, d, gt);
            ne = setup_triangle<M>(*d, gt, fp, s0, s1, s2);
            texi = d->tex;
            st = d->flags & DRAW_ST;
        }
        active = ne >= 2;
        if (active) {
            uint32_t anom = 0;
            Walker<M, true> w0;
            if constexpr (PRK_SETUP_REC) w0.init_rec(ne, s0, s1, s2, fp.H, fp.row1, rhead);
            else w0.init(ne, s0, s1, s2, fp.H, fp.row1, anom);
            const int fr = w0.fast_replay(fp.row0, ne);  // band above row0 (row bands only)
            wk_from(wk, w0);
            if (fr < 0)
                while (wk.Row < fp.row0 && wk.Row < wk.MaxY) wk.end_row(wk.begin_row());
            if (anom) atomicAdd(anomaly, anom);
            active = wk.Row < wk.MaxY;
            tr = ranges[g];
            jb = tri_off[g];
            const int ntx = (int)tr.tx1 - (int)tr.tx0 + 1, nty = (int)tr.ty1 - (int)tr.ty0 + 1;
            // Rows that won a pixel in any tile, as bits over the triangle's
            // tile rows (8-row tiles, <= 8 pairs): the won flags of a pair are
            // 8 consecutive bytes, loaded together up front.
            rbase = fp.row0 + (int32_t)tr.ty0 * fp.tile_h;
            fast = fp.tile_h == 8 && ntx * nty <= 8;
            if (fast) {
                uint64_t m[8];
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    m[k] = k < ntx * nty ? *reinterpret_cast<const uint64_t *>(won + (size_t)(jb + k) * 8) : 0ull;
                rows = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int ty = k / ntx;  // pair k = (ty, tx) row-major
                    rows |= ((m[k] * 0x0102040810204080ull) >> 56) << (8 * ty);  // bytes (0/1) -> bits
                }
                // the walk ends at the triangle's last won row (rows below it
                // emit nothing, and no earlier row depends on them)
                if (rows) wk.MaxY = min(wk.MaxY, rbase + 64 - (int32_t)__clzll((long long)rows));
            }
        }
    }
    const int32_t t0 = (int32_t)((uint32_t)tr.tx0 | ((uint32_t)tr.ty0 << 16));
    const int32_t t1 = (int32_t)((uint32_t)tr.tx1 | ((uint32_t)tr.ty1 << 16));
    uint32_t head = 0, cnt = 0;  // wave-uniform queue state
    while (__any(active)) {
        bool push = false, paired = false;
        int32_t Row = 0;
        if (active) {
            Row = wk.Row;
            paired = wk.begin_row();
            const int32_t rb = Row - rbase;
            const bool want = !fast || (rb >= 0 && rb < 64 && ((rows >> rb) & 1ull));
            push = paired && want && Row >= fp.row0;
        }
        const uint64_t bal = __ballot(push);
        if (push) {
            const uint32_t slot = (head + cnt + (uint32_t)__builtin_amdgcn_mbcnt_hi(
                (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))) & (kWalkQ - 1);
            Edge L, R;
            wk_pair(wk, L, R);
            q.f[0][slot] = L.X; q.f[1][slot] = L.W; q.f[2][slot] = L.U; q.f[3][slot] = L.V; q.f[4][slot] = L.Z;
            q.f[5][slot] = L.N0; q.f[6][slot] = L.N1; q.f[7][slot] = L.N2;
            q.f[8][slot] = R.X; q.f[9][slot] = R.W; q.f[10][slot] = R.U; q.f[11][slot] = R.V; q.f[12][slot] = R.Z;
            q.f[13][slot] = R.N0; q.f[14][slot] = R.N1; q.f[15][slot] = R.N2;
            q.i[0][slot] = (int32_t)((uint32_t)(Row & 0xFFFF) | ((uint32_t)texi << 16) | (st << 31));
            q.i[1][slot] = (int32_t)jb;
            q.i[2][slot] = t0;
            q.i[3][slot] = t1;
        }
        cnt += (uint32_t)__popcll(bal);
        if (active) {
            wk.end_row(paired);
            active = wk.Row < wk.MaxY;
        }
        if (cnt >= 64) {  // one queued span per lane
            wave_lds_sync();
            walk_flush(fp, q, (int)((head + lane) & (kWalkQ - 1)), won, recs);
            wave_lds_sync();
            head += 64;
            cnt -= 64;
        }
    }
    wave_lds_sync();
    if ((uint32_t)lane < cnt) walk_flush(fp, q, (int)((head + lane) & (kWalkQ - 1)), won, recs);
}

// ---------------------------------------------------------------------------
// k_walk's triangle list: the triangles that won a pixel (k_won_local, one
// launch, the count stays on the device).  Each workgroup appends the won
// triangles of its 2048 consecutive triangles as one run (one atomic), so
// neighbouring triangles — whose setup records share cache lines and whose
// span records land close together — stay together in the list.
// PRK_WON_SORT 1 groups each run by triangle height, tallest first (each
// k_walk lane walks its own triangle, so a wave runs as long as its tallest
// one); measured on C3b (serial k_walk): 0 -> 0.249 ms, 1 -> 0.278, a global
// height grouping -> 0.263, round 1's library stream compaction -> 0.256: the
// scattered record traffic costs more than the lane utilisation gains.
// The list length (kWonHistBytes of scratch) is zeroed before the launch.
// ---------------------------------------------------------------------------
#ifndef PRK_WON_SORT
#define PRK_WON_SORT 0
#endif
constexpr int kWonClasses = 64, kWonPer = 8, kWonThreads = 256;
constexpr size_t kWonHistBytes = 16;  // [0]: the list length

__device__ __forceinline__ int won_class(const TileRange &tr) {
    if (PRK_WON_SORT == 0) return 0;
    const int rows = (int)tr.pad1 - (int)tr.pad0;  // band rows [r0, r1) (k_bin_count)
    return kWonClasses - 1 - min(max(rows, 0), kWonClasses - 1);
}

// One workgroup per 2048 triangles: its won triangles (grouped by height with
// PRK_WON_SORT 1) at a run of the list reserved with one atomic on *count.
__global__ void __launch_bounds__(kWonThreads) k_won_local(uint32_t n, const uint8_t *__restrict__ trwon,
                                                           const TileRange *__restrict__ ranges,
                                                           uint32_t *__restrict__ count, uint32_t *__restrict__ wlist) {
    __shared__ uint32_t h[kWonClasses];
    __shared__ uint32_t base;
    if (threadIdx.x < kWonClasses) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t g0 = blockIdx.x * (kWonThreads * kWonPer) + threadIdx.x;
    int cls[kWonPer];
    uint32_t rank[kWonPer];
#pragma unroll
    for (int k = 0; k < kWonPer; ++k) {
        const uint32_t g = g0 + k * kWonThreads;
        cls[k] = -1;
        rank[k] = 0;
        if (g < n && trwon[g]) {
            cls[k] = won_class(ranges[g]);
            rank[k] = atomicAdd(&h[cls[k]], 1u);
        }
    }
    __syncthreads();
    if (threadIdx.x < kWonClasses) {  // one wave: class offsets inside the run, the run's start
        const uint32_t c = h[threadIdx.x];
        const uint32_t incl = (uint32_t)wave_incl_scan((int)c, (int)threadIdx.x);
        h[threadIdx.x] = incl - c;
        if (threadIdx.x == kWonClasses - 1) base = incl ? atomicAdd(count, incl) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kWonPer; ++k)
        if (cls[k] >= 0) wlist[base + h[cls[k]] + rank[k]] = g0 + k * kWonThreads;
}

// k_pix: shade the won pixels of one tile from their span records (SPAN:
// records indexed by span, the whole-object path; else by (pair, row in tile)).
template <bool UNI, bool SPAN = false, bool ZV = false>  // ZV: k_vis wrote the z (fp.z_in_vis)
__global__ void __launch_bounds__(256) k_pix(FrameParams fp, const uint32_t *__restrict__ nwin_in,
                                             const uint32_t *__restrict__ wtag, const SpanRec *__restrict__ recs) {
    // PRK_PIX_SPLIT workgroups per tile, each a contiguous share of its pixels
    const int ntile = fp.tiles_x * fp.tiles_y;
    const int t = blockIdx.x / PRK_PIX_SPLIT, part = blockIdx.x - t * PRK_PIX_SPLIT;
    if (t >= ntile) return;
    const bool any = nwin_in[t] != 0;  // (k_vis leaves the tags of a tile without entries unwritten)
    if (!any && !fp.clear_fused) return;
    const TileCtx tc = tile_ctx(fp, t);
    const int npx = fp.tile_w * fp.tile_h;
    const uint32_t *tags = wtag + (size_t)t * npx;
    const int pend = (int)(((long long)npx * (part + 1)) / PRK_PIX_SPLIT);
    for (int p = (int)(((long long)npx * part) / PRK_PIX_SPLIT) + threadIdx.x; p < pend; p += blockDim.x) {
        const uint32_t tag = any ? tags[p] : kTagPrior;
        const int ly = p >> fp.tile_w_log2;
        const int32_t x = tc.x0 + (p & (fp.tile_w - 1)), Row = tc.y0 + ly;
        uint32_t j;  // the winning pair
        if (!tag_pair(tag, j)) {  // no fragment beat the prior z
            if (fp.clear_fused && x < tc.x1 && Row < tc.y1) {
                if (!ZV) put_winner(fp, x, Row, fp.clear_z, fp.clear_color);
                else put_color(fp, x, Row, fp.clear_color);  // (k_vis wrote the z)
            }
            continue;
        }
        const float4 *q = reinterpret_cast<const float4 *>(recs + (SPAN ? (size_t)j : (size_t)j * fp.tile_h + ly));
        const float4 r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3];
        const int32_t lt = __float_as_int(r0.x);
        if (SPAN && (uint32_t)lt == kScalarSpan) continue;  // a DrawModel span won: k_span_shade
        const int32_t LeftXa = (int32_t)(int16_t)(lt & 0xFFFF);
        const TexRec tex = UNI ? fp.tex0 : fp.texs[lt >> 16];
        const int32_t rel = x - LeftXa, i = rel & 7, b = rel >> 3;
        const float IW = r1.z, IU = r1.w, IV = r2.x, IZ = r2.y;
        const float o = r0.y + (float)i;  // lane init (XOffset + i)*inc, 1712-1835
        float w = r0.z + o * IW, u = r0.w + o * IU;
        float v = r1.x + o * IV, z = r1.y + o * IZ;
        {
            const float IW8 = IW * 8.0f, IU8 = IU * 8.0f, IV8 = IV * 8.0f, IZ8 = 8.0f * IZ;
            for (int32_t k = 0; k < b; ++k) { z = z + IZ8; w = w + IW8; u = u + IU8; v = v + IV8; }  // 2262-2282
        }
        const float iw = 1.0f / w;  // 1865-1866
        const float fu = iw * u, fv = iw * v;
        const Texel4 tx = sample_avx(tex, fu, fv);
        const float IN0 = r3.y, IN1 = r3.z, IN2 = r3.w;
        float n0 = r2.z + o * IN0, n1 = r2.w + o * IN1, n2 = r3.x + o * IN2;
        normalize_div(n0, n1, n2);  // 1754
        {
            const float IN08 = IN0 * 8.0f, IN18 = IN1 * 8.0f, IN28 = IN2 * 8.0f;
            for (int32_t k = 0; k < b; ++k) {  // block steps 2262-2282
                float a = n0 + IN08, bb = n1 + IN18, c = n2 + IN28;
                normalize_div(a, bb, c);
                n0 = a; n1 = bb; n2 = c;
            }
        }
        const uint32_t col = shade_avx_texel(fp, tx, z, n0, n1, n2, x, i, Row);
        if (!ZV) {
            put_winner(fp, x, Row, z, col);
        } else {  // k_vis wrote the z, as +0.0 for a -0.0
            put_color(fp, x, Row, col);
            if (__float_as_uint(z) == 0x80000000u) {
                fp.zbuf[(size_t)(Row - fp.row0) * fp.W + x] = z;
                if (fp.negz) atomicAdd(fp.negz, 1u);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Span path (whole-object AETs, prk_spans.hip): visibility over a tile's bin
// of spans.  Every span is one pair of one row, given by its record and pixel
// range; its tag is its submission-order index.  FillLineOptimized spans
// (SpanRec) take the triangle path's visibility items (item_vis_group),
// DrawModel spans (ScSpanRec, SPAN_SCALAR) its scalar chunk items
// (item_scalar), the one-past-the-row pixel included.
// ---------------------------------------------------------------------------
struct SpanPosK { int32_t row, minx, maxx; uint32_t flags; };  // == prk_spans.hip SpanPos
struct ScSpanRec { float f[22]; int32_t tex, pad; };          // == prk_spans.hip ScSpanRecG
static_assert(sizeof(ScSpanRec) == 96, "scalar span record");
constexpr int32_t kAvxSlot = -2;  // SI_OVF of a slot holding a FillLineOptimized span

// The wave's items: every lane holds `items` work items of the span in its
// slot; f(slot, j) runs item j of that slot, spread over the lanes in windows
// of 64 (item -> slot: a prefix max over span-start marks, as in sweep()).
template <class WS, class F>
__device__ __forceinline__ void wave_items(WS &ws, int items, int lane, F &&f) {
    const int incl = wave_incl_scan(items, lane);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    const int excl = incl - items;
    ws.i[SI_PRE][lane] = excl;
    int carry = 0;
    for (int it0 = 0; it0 < total; it0 += 64) {
        ws.i[SI_MARK][lane] = 0;
        wave_lds_sync();
        if (items > 0 && excl >= it0 && excl < it0 + 64) ws.i[SI_MARK][excl - it0] = lane + 1;
        wave_lds_sync();
        const int m = max(wave_incl_max(ws.i[SI_MARK][lane]), carry);
        carry = __builtin_amdgcn_readlane(m, 63);
        const int it = it0 + lane;
        if (it < total) {
            const int sl = m - 1;
            f(sl, it - ws.i[SI_PRE][sl]);
        }
    }
    wave_lds_sync();
}

// A DrawModel span's slot for tile tc (scalar items, visibility or shading):
// the part [xa, xb) of its inclusive [MinX, MaxX] in the tile's columns of
// its row, and the one-past-the-row pixel (Row + 1, 0) when MaxX == W and
// that pixel lies in the tile (span_setup_scalar's ranges).  Returns the
// item count.
template <bool SHADE, class WS>
__device__ __forceinline__ int span_slot_scalar(const FrameParams &fp, const TileCtx &tc, WS &ws, int lane,
                                                const SpanPosK &sp, const ScSpanRec *__restrict__ srecs,
                                                uint32_t sidx) {
    const int32_t W = fp.W;
    const int32_t MinX = sp.minx, MaxX = sp.maxx - 1;
    const bool in_rows = sp.row >= tc.y0 && sp.row < tc.y1;
    const int32_t xa = in_rows ? max(MinX, tc.x0) : 0;
    const int32_t xb = in_rows ? min(MaxX + 1, tc.x1) : 0;
    const bool ovf = tc.x0 == 0 && MaxX >= W && sp.row + 1 >= tc.y0 && sp.row + 1 < tc.y1;
    if (xa >= xb && !ovf) return 0;
    const ScSpanRec &r = srecs[sidx];
    ws.i[SI_XA][lane] = xa;
    ws.i[SI_XB][lane] = xb;
    ws.i[SI_LEFT][lane] = MinX;
    ws.i[SI_TAG][lane] = (int32_t)pair_tag(sidx, false);
    ws.i[SI_OVF][lane] = ovf ? (sp.row + 1 - tc.y0) * tc.tw : -1;
    ws.i[SI_ROW][lane] = sp.row;
    if constexpr (SHADE) {
        ws.i[SI_TEX][lane] = r.tex;
#pragma unroll
        for (int k = 0; k < kSpanF; ++k) ws.f[k][lane] = r.f[k];
    } else {
        ws.f[SS_Z][lane] = r.f[SS_Z];
        ws.f[SS_IZ][lane] = r.f[SS_IZ];
    }
    return scalar_chunks<SHADE>(xa, xb) + (ovf ? 1 : 0);
}

__global__ void __launch_bounds__(64 * kVisWaves, PRK_VIS_MIN_WAVES)
    k_span_vis(FrameParams fp, const uint32_t *__restrict__ offs, const uint32_t *__restrict__ bins,
               const SpanPosK *__restrict__ pos, const SpanRec *__restrict__ recs,
               const ScSpanRec *__restrict__ srecs, const uint32_t *__restrict__ span_tri,
               uint32_t *__restrict__ nwin_out, uint32_t *__restrict__ wtag) {
    extern __shared__ unsigned long long lds[];
    const int ntile = fp.tiles_x * fp.tiles_y;
    const int t = blockIdx.x;
    if (t >= ntile) return;
    const uint32_t b0 = offs[t], b1 = offs[t + 1];
    if (b0 == b1) {
        if (threadIdx.x == 0) nwin_out[t] = 0;
        return;
    }
    const uint32_t n = b1 - b0;
    TileCtx tc = tile_ctx(fp, t);
    const int npx = fp.tile_w * fp.tile_h;
    tc.key = lds;
    VisSlots *slots = reinterpret_cast<VisSlots *>(lds + npx);
    VisSlots &ws = slots[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int p = threadIdx.x; p < npx; p += blockDim.x) {  // prior z (as k_vis)
        const int lx = p & (fp.tile_w - 1), ly = p >> fp.tile_w_log2;
        const int x = tc.x0 + lx, y = tc.y0 + ly;
        unsigned long long k = ~0ull;
        if (x < tc.x1 && y < tc.y1) {
            const float z = fp.clear_fused ? fp.clear_z : fp.zbuf[(size_t)(y - fp.row0) * fp.W + x];
            k = (z != z) ? ~0ull : (((unsigned long long)zkey(z) << 32) | kTagPrior);
        }
        tc.key[p] = k;
    }
    __syncthreads();
    constexpr int G = PRK_VIS_GROUP > 0 ? PRK_VIS_GROUP : 1;
    const uint32_t nwaves = blockDim.x >> 6;
    for (uint32_t base = wave * 64; base < n; base += 64 * nwaves) {
        const uint32_t i = base + lane;
        int items = 0;
        if (i < n) {
            const uint32_t sidx = bins[b0 + i];
            const SpanPosK sp = pos[sidx];
            if (sp.flags & SPAN_SCALAR) {
                items = span_slot_scalar<false>(fp, tc, ws, lane, sp, srecs, sidx);
            } else if (sp.row >= tc.y0 && sp.row < tc.y1) {
                const int32_t xa = max(sp.minx, tc.x0), xb = min(sp.maxx, tc.x1);
                if (xa < xb) {
                    const float4 *q = reinterpret_cast<const float4 *>(recs + sidx);
                    const float4 r0 = q[0], r1 = q[1], r2 = q[2];
                    ws.i[SI_XA][lane] = xa;
                    ws.i[SI_XB][lane] = xb;
                    ws.i[SI_LEFT][lane] = (int32_t)(int16_t)(__float_as_int(r0.x) & 0xFFFF);
                    ws.i[SI_TAG][lane] = (int32_t)pair_tag(sidx, (sp.flags & DRAW_ST) != 0);
                    ws.i[SI_ROW][lane] = sp.row;
                    ws.i[SI_OVF][lane] = kAvxSlot;
                    ws.f[SF_XOFF][lane] = r0.y;
                    ws.f[SF_LW][lane] = r0.z; ws.f[SF_LU][lane] = r0.w; ws.f[SF_LV][lane] = r1.x;
                    ws.f[SF_LZ][lane] = r1.y;
                    ws.f[SF_IW][lane] = r1.z; ws.f[SF_IU][lane] = r1.w; ws.f[SF_IV][lane] = r2.x;
                    ws.f[SF_IZ][lane] = r2.y;
                    items = (xb - xa + G - 1) / G;
                }
            }
        }
        wave_items(ws, items, lane, [&](int sl, int j) {
            if (ws.i[SI_OVF][sl] == kAvxSlot) item_vis_group(tc, ws, sl, j, ws.i[SI_ROW][sl]);
            else item_scalar<MODE_SC_GOURAUD, false, false>(fp, tc, ws, sl, j, ws.i[SI_ROW][sl]);
        });
    }
    __syncthreads();
    uint32_t *tags_out = wtag + (size_t)t * npx;
    int anyw = 0;
    for (int p = threadIdx.x; p < npx; p += blockDim.x) {
        const uint32_t low = (uint32_t)tc.key[p];
        tags_out[p] = low;
        uint32_t j;
        if (tag_pair(low, j)) anyw = 1;
        if (fp.winners) {
            const int x = tc.x0 + (p & (fp.tile_w - 1)), y = tc.y0 + (p >> fp.tile_w_log2);
            if (x < tc.x1 && y < tc.y1 && tag_pair(low, j))
                fp.winners[(size_t)(y - fp.row0) * fp.W + x] = (int32_t)(fp.win_base + span_tri[j]);
        }
    }
    anyw = __syncthreads_or(anyw);
    if (threadIdx.x == 0) nwin_out[t] = (uint32_t)anyw;
}

// Shading of the DrawModel spans of the span path, one workgroup per tile:
// every scalar span of mode M in the tile's bin shades the pixels it won
// (item_scalar, SHADE).  MODESET -1: one sweep per scalar mode.
template <int M>
__device__ __forceinline__ void span_shade_sweep(const FrameParams &fp, const TileCtx &tc, ShadeSlots &ws,
                                                 const uint32_t *__restrict__ bins, uint32_t b0, uint32_t n,
                                                 const SpanPosK *__restrict__ pos,
                                                 const ScSpanRec *__restrict__ srecs) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nwaves = blockDim.x >> 6;
    for (uint32_t base = wave * 64; base < n; base += 64 * nwaves) {
        const uint32_t i = base + lane;
        int items = 0;
        if (i < n) {
            const uint32_t sidx = bins[b0 + i];
            const SpanPosK sp = pos[sidx];
            if ((sp.flags & SPAN_SCALAR) && (int)((sp.flags >> 8) & 0xFFu) == M)
                items = span_slot_scalar<true>(fp, tc, ws, lane, sp, srecs, sidx);
        }
        wave_items(ws, items, lane,
                   [&](int sl, int j) { item_scalar<M, true, false>(fp, tc, ws, sl, j, ws.i[SI_ROW][sl]); });
    }
}

template <int MODESET>
__global__ void __launch_bounds__(64 * kShadeWaves, PRK_SHADE_MIN_WAVES)
    k_span_shade(FrameParams fp, const uint32_t *__restrict__ offs, const uint32_t *__restrict__ bins,
                 const SpanPosK *__restrict__ pos, const ScSpanRec *__restrict__ srecs,
                 const uint32_t *__restrict__ nwin_in, const uint32_t *__restrict__ wtag) {
    extern __shared__ unsigned long long lds[];
    const int ntile = fp.tiles_x * fp.tiles_y;
    const int t = blockIdx.x;
    if (t >= ntile || nwin_in[t] == 0) return;
    const uint32_t b0 = offs[t], n = offs[t + 1] - b0;
    TileCtx tc = tile_ctx(fp, t);
    const int npx = fp.tile_w * fp.tile_h;
    uint32_t *tags = reinterpret_cast<uint32_t *>(lds);
    tc.tags = tags;
    ShadeSlots *slots = reinterpret_cast<ShadeSlots *>(tags + npx + kTagPad);
    ShadeSlots &ws = slots[threadIdx.x >> 6];
    const uint32_t *tags_in = wtag + (size_t)t * npx;
    for (int p = threadIdx.x; p < npx; p += blockDim.x) tags[p] = tags_in[p];
    if (threadIdx.x < kTagPad) tags[npx + threadIdx.x] = 0xFFFFFFFFu;
    __syncthreads();
    if constexpr (MODESET >= 0) {
        span_shade_sweep<(MODESET >= 0 ? MODESET : 1)>(fp, tc, ws, bins, b0, n, pos, srecs);
    } else {
        span_shade_sweep<MODE_SC_GOURAUD>(fp, tc, ws, bins, b0, n, pos, srecs);
        span_shade_sweep<MODE_SC_GOURAUD_TEX>(fp, tc, ws, bins, b0, n, pos, srecs);
        span_shade_sweep<MODE_SC_PHONG>(fp, tc, ws, bins, b0, n, pos, srecs);
        span_shade_sweep<MODE_SC_PHONG_TEX>(fp, tc, ws, bins, b0, n, pos, srecs);
    }
}

// Explicit instantiations used by the host.
#define PRK_VIS_ARGS FrameParams, const uint32_t *, const uint2 *, uint8_t *, uint32_t *, uint32_t *, uint32_t *, \
                     const uint32_t *, uint8_t *, uint32_t *
#define PRK_SHADE_ARGS FrameParams, const uint32_t *, const uint2 *, const uint32_t *, const uint32_t *, \
                       const uint32_t *, uint32_t *
#define PRK_INST(MS, UNI)                                  \
    template __global__ void k_vis<MS, UNI>(PRK_VIS_ARGS); \
    template __global__ void k_shade<MS, UNI>(PRK_SHADE_ARGS);
template __global__ void k_vis<MODE_AVX, false, true>(PRK_VIS_ARGS);
template __global__ void k_vis<MODE_AVX, true, true>(PRK_VIS_ARGS);
#define PRK_WALK_ARGS FrameParams, const uint32_t *, const uint32_t *, const uint32_t *, const TileRange *, \
                      const uint8_t *, SpanRec *, uint32_t *
#define PRK_PIX_ARGS FrameParams, const uint32_t *, const uint32_t *, const SpanRec *
template __global__ void k_walk<false>(PRK_WALK_ARGS);
template __global__ void k_walk<true>(PRK_WALK_ARGS);
template __global__ void k_pix<false>(PRK_PIX_ARGS);
template __global__ void k_pix<true>(PRK_PIX_ARGS);
template __global__ void k_pix<false, true>(PRK_PIX_ARGS);
template __global__ void k_pix<false, false, true>(PRK_PIX_ARGS);
template __global__ void k_pix<true, false, true>(PRK_PIX_ARGS);
#define PRK_SPAN_SHADE_ARGS FrameParams, const uint32_t *, const uint32_t *, const SpanPosK *, const ScSpanRec *, \
                            const uint32_t *, const uint32_t *
template __global__ void k_span_shade<-1>(PRK_SPAN_SHADE_ARGS);
template __global__ void k_span_shade<MODE_SC_GOURAUD>(PRK_SPAN_SHADE_ARGS);
template __global__ void k_span_shade<MODE_SC_PHONG>(PRK_SPAN_SHADE_ARGS);
PRK_INST(-1, false)
PRK_INST(MODE_AVX, false)
PRK_INST(MODE_AVX, true)
PRK_INST(MODE_SC_GOURAUD, false)
PRK_INST(MODE_SC_GOURAUD, true)
PRK_INST(MODE_SC_PHONG, false)
PRK_INST(MODE_SC_PHONG, true)
#undef PRK_INST

// Self-test of the shared-divisor quotients (prk_device.h DivBy): thread i
// draws (x, d) from a hash of (seed, i) — random signs, mantissas and
// exponents in [-64, 64) (both inside and outside the fast range), every 16th
// x zero — and counts quotients and normalisations that differ in any bit
// from the compiler's own x / d.
__device__ __forceinline__ uint32_t st_hash(uint64_t v) {
    v ^= v >> 33; v *= 0xff51afd7ed558ccdull; v ^= v >> 33; v *= 0xc4ceb9fe1a85ec53ull; v ^= v >> 33;
    return (uint32_t)v;
}
__device__ __forceinline__ float st_float(uint32_t h, uint32_t e) {
    const uint32_t ex = 127u - 64u + (e & 127u);
    return __uint_as_float((h & 0x807FFFFFu) | (ex << 23));
}
__global__ void k_selftest_div(uint32_t n, uint64_t seed, unsigned long long *bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = seed * 0x9E3779B97F4A7C15ull + 4ull * i;
    const uint32_t h0 = st_hash(k), h1 = st_hash(k + 1), h2 = st_hash(k + 2), h3 = st_hash(k + 3);
    const float x = (i & 15u) == 7u ? ((h0 & 1u) ? -0.0f : 0.0f) : st_float(h0, h2);
    const float d = st_float(h1, h2 >> 8);
    const volatile float dv = d;  // the plain quotient sees an opaque divisor
    float q1[1] = {x};
    div_all(d, q1);
    const float q0 = x / dv;
    unsigned long long b = __float_as_uint(q0) != __float_as_uint(q1[0]) ? 1ull : 0ull;
    // normalisation of a vector of three draws (exponents within +-24)
    const float a0 = st_float(h0, 52u + (h3 & 47u)), a1 = st_float(h1, 52u + ((h3 >> 8) & 47u));
    const float a2 = (i & 31u) == 3u ? 0.0f : st_float(h2, 52u + ((h3 >> 16) & 47u));
    float n0 = a0, n1 = a1, n2 = a2;
    normalize_div(n0, n1, n2);
    const volatile float lv = sqrtf((a0 * a0 + a1 * a1) + a2 * a2);
    const float len = lv;
    if (__float_as_uint(n0) != __float_as_uint(a0 / len) || __float_as_uint(n1) != __float_as_uint(a1 / len) ||
        __float_as_uint(n2) != __float_as_uint(a2 / len))
        b += 1ull << 32;
    // sqrt_mid against the compiler's sqrtf on [2^-96, 2^128): counted with
    // the normalisations
    const uint32_t se = 127u - 96u + (h3 >> 24) % 224u;
    const volatile float sv = __uint_as_float((h1 & 0x007FFFFFu) | (se << 23));
    const float sx = sv;
    if (__float_as_uint(sqrt_mid(sx)) != __float_as_uint(sqrtf(sv))) b += 1ull << 32;
    if (b) atomicAdd(bad, b);
}

}  // namespace prk

// ---------------------------------------------------------------------------
// Launchers (called from prk_api.cpp).
// ---------------------------------------------------------------------------
extern "C" {

// Shared-divisor self-test: *bad = quotient mismatches | normalisation
// mismatches << 32 over n draws (device memory).
hipError_t prk_selftest_div_launch(uint32_t n, uint64_t seed, unsigned long long *bad, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_selftest_div, dim3((n + 255) / 256), dim3(256), 0, s, n, seed, bad);
    return hipGetLastError();
}

// Scratch bytes of k_walk's list build (the height-class histogram and cursors).
hipError_t prk_walk_select_bytes(uint32_t, size_t *bytes) {
    *bytes = prk::kWonHistBytes;
    return hipSuccess;
}

hipError_t prk_launch_tri_draw(const prk::DrawRec *draws, uint32_t ndraws, uint32_t *tri_draw,
                               uint32_t tri_count, hipStream_t s) {
    if (tri_count == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_tri_draw, dim3((tri_count + 255) / 256), dim3(256), 0, s, draws, ndraws,
                       tri_draw, tri_count);
    return hipGetLastError();
}

// Bytes of dynamic LDS per workgroup of k_vis / k_shade.
static size_t vis_lds(const prk::FrameParams *fp) {
    return (size_t)fp->tile_w * fp->tile_h * sizeof(unsigned long long) + prk::kVisWaves * sizeof(prk::VisSlots) +
           16 * sizeof(uint32_t);
}
static size_t shade_lds(const prk::FrameParams *fp) {
    const size_t npx = (size_t)fp->tile_w * fp->tile_h;
    return (npx + prk::kTagPad) * sizeof(uint32_t) + prk::kShadeWaves * sizeof(prk::ShadeSlots);
}

// Sweep 1 (k_vis) then the shading: k_walk + k_pix for AVX frames, k_shade
// otherwise; `mid` (optional) is recorded after k_vis, `mid2` between k_walk
// and k_pix.  won: per bin entry (k_shade frames) or per (pair, row) (AVX
// frames) won flags; trwon: per triangle; recs: span records, 64 B per
// (pair, row); tri_off / ranges: the binning's pair offsets and tile ranges.
hipError_t prk_launch_raster(const prk::FrameParams *fp, int modeset, const uint32_t *offs, const void *bins_,
                             const uint32_t *pair_tri, const uint32_t *tri_off, const void *ranges, uint8_t *won,
                             uint8_t *trwon, uint32_t *wlist, void *sel_temp, size_t sel_bytes, uint32_t *list,
                             uint32_t *nwin, uint32_t *wtag, void *recs, uint32_t *anomaly, hipEvent_t mid,
                             hipEvent_t mid2, hipStream_t svis, hipStream_t s) {
    // k_vis runs on svis, the shading on s (after k_vis: `mid` is recorded on
    // svis and waited for on s); svis == s runs the frame on one stream.
    const uint32_t ntile = (uint32_t)(fp->tiles_x * fp->tiles_y);
    if (svis != s && (!mid || (PRK_WALK_ON_VIS && modeset == prk::MODE_AVX && !mid2))) return hipErrorInvalidValue;
    if (ntile == 0) return hipSuccess;
    const size_t lv = vis_lds(fp), ls = shade_lds(fp);
    const bool uni = fp->ndraws == 1;
    prk::SpanRec *rp = reinterpret_cast<prk::SpanRec *>(recs);
    const prk::TileRange *tr = reinterpret_cast<const prk::TileRange *>(ranges);
    const uint32_t nblk = (fp->tri_count + 255) / 256;
    const uint32_t nwblk = (fp->tri_count + 64 * prk::kWalkWaves - 1) / (64 * prk::kWalkWaves);
    const uint32_t nwon = (fp->tri_count + prk::kWonThreads * prk::kWonPer - 1) / (prk::kWonThreads * prk::kWonPer);
    const uint2 *bins = reinterpret_cast<const uint2 *>(bins_);
    if (modeset == prk::MODE_AVX && PRK_SPAN_RECORDS && nblk) {
        // k_walk's list histogram, cleared before k_vis is waited for (off
        // the k_vis -> k_walk path)
        if (!sel_temp || sel_bytes < prk::kWonHistBytes) return hipErrorInvalidValue;
        const hipError_t e = hipMemsetAsync(sel_temp, 0, prk::kWonHistBytes, PRK_WALK_ON_VIS ? svis : s);
        if (e != hipSuccess) return e;
    }
#define PRK_VIS(MS, UNI)                                                                                             \
    do {                                                                                                             \
        if (MS == prk::MODE_AVX && fp->z_in_vis)                                                                   \
            hipLaunchKernelGGL((prk::k_vis<MS, UNI, true>), dim3(ntile), dim3(64 * prk::kVisWaves), lv, svis, *fp,   \
                               offs, bins, won, list, nwin, wtag, pair_tri, trwon, anomaly);                         \
        else                                                                                                         \
            hipLaunchKernelGGL((prk::k_vis<MS, UNI>), dim3(ntile), dim3(64 * prk::kVisWaves), lv, svis, *fp, offs,    \
                               bins, won, list, nwin, wtag, pair_tri, trwon, anomaly);                               \
        if (mid) (void)hipEventRecord(mid, svis);                                                                    \
        if (svis != s) (void)hipStreamWaitEvent(s, mid, 0);                                                          \
    } while (0)
#define PRK_SHADE(MS, UNI)                                                                                           \
    hipLaunchKernelGGL((prk::k_shade<MS, UNI>), dim3(ntile), dim3(64 * prk::kShadeWaves), ls, s, *fp, offs, bins, list,  \
                       nwin, wtag, anomaly)
#define PRK_SPANPIX(UNI)                                                                                             \
    do {                                                                                                             \
        /* PRK_WALK_ON_VIS: k_walk follows k_vis on svis, k_pix waits for it on s */                                 \
        hipStream_t sw = PRK_WALK_ON_VIS ? svis : s;                                                                 \
        if (nblk) {                                                                                                  \
            /* the won triangles, tallest first; the count stays on the device */                                  \
            uint32_t *nsel = wlist + fp->tri_count;                                                                  \
            uint32_t *hist_ = reinterpret_cast<uint32_t *>(sel_temp);                                                \
            nsel = hist_; /* the run counter is the list length */                                                   \
            hipLaunchKernelGGL(prk::k_won_local, dim3(nwon), dim3(prk::kWonThreads), 0, sw, fp->tri_count, trwon,     \
                               tr, hist_, wlist);                                                                    \
            hipLaunchKernelGGL((prk::k_walk<UNI>), dim3(nwblk), dim3(64 * prk::kWalkWaves), 0, sw, *fp, wlist, nsel,    \
                               tri_off, tr, won,                                                                     \
                               rp, anomaly);                                                                         \
        }                                                                                                            \
        if (mid2) (void)hipEventRecord(mid2, sw);                                                                    \
        if (sw != s) (void)hipStreamWaitEvent(s, mid2, 0);                                                           \
        if (fp->z_in_vis)                                                                                            \
            hipLaunchKernelGGL((prk::k_pix<UNI, false, true>), dim3(ntile * PRK_PIX_SPLIT), dim3(256), 0, s, *fp, nwin, \
                               wtag, rp);                                                                            \
        else                                                                                                         \
            hipLaunchKernelGGL((prk::k_pix<UNI>), dim3(ntile * PRK_PIX_SPLIT), dim3(256), 0, s, *fp, nwin, wtag, rp); \
    } while (0)
    switch (modeset) {
        case prk::MODE_AVX:
            if (uni) {
                PRK_VIS(prk::MODE_AVX, true);
                if (PRK_SPAN_RECORDS) PRK_SPANPIX(true); else PRK_SHADE(prk::MODE_AVX, true);
            } else {
                PRK_VIS(prk::MODE_AVX, false);
                if (PRK_SPAN_RECORDS) PRK_SPANPIX(false); else PRK_SHADE(prk::MODE_AVX, false);
            }
            break;
        case prk::MODE_SC_GOURAUD:
            if (uni) { PRK_VIS(prk::MODE_SC_GOURAUD, true); PRK_SHADE(prk::MODE_SC_GOURAUD, true); }
            else { PRK_VIS(prk::MODE_SC_GOURAUD, false); PRK_SHADE(prk::MODE_SC_GOURAUD, false); }
            break;
        case prk::MODE_SC_PHONG:
            if (uni) { PRK_VIS(prk::MODE_SC_PHONG, true); PRK_SHADE(prk::MODE_SC_PHONG, true); }
            else { PRK_VIS(prk::MODE_SC_PHONG, false); PRK_SHADE(prk::MODE_SC_PHONG, false); }
            break;
        default: PRK_VIS(-1, false); PRK_SHADE(-1, false); break;
    }
#undef PRK_VIS
#undef PRK_SHADE
#undef PRK_SPANPIX
    return hipGetLastError();
}

// Span path: visibility then shading of the pass's spans.  scalar_modes: bit
// m set when the pass holds DrawModel spans of mode m (srecs non-null then);
// bit MODE_AVX when it holds FillLineOptimized spans.
hipError_t prk_launch_spans(const prk::FrameParams *fp, const uint32_t *offs, const uint32_t *bins, const void *pos,
                            const void *recs, const void *srecs, uint32_t modes, const uint32_t *span_tri,
                            uint32_t *nwin, uint32_t *wtag, hipStream_t s) {
    const uint32_t ntile = (uint32_t)(fp->tiles_x * fp->tiles_y);
    if (ntile == 0) return hipSuccess;
    const uint32_t sc = modes & ~(1u << prk::MODE_AVX);
    if (sc && !srecs) return hipErrorInvalidValue;
    const size_t lv = vis_lds(fp), ls = shade_lds(fp);
    const prk::SpanPosK *P = reinterpret_cast<const prk::SpanPosK *>(pos);
    const prk::ScSpanRec *SR = reinterpret_cast<const prk::ScSpanRec *>(srecs);
    hipLaunchKernelGGL(prk::k_span_vis, dim3(ntile), dim3(64 * prk::kVisWaves), lv, s, *fp, offs, bins, P,
                       reinterpret_cast<const prk::SpanRec *>(recs), SR, span_tri, nwin, wtag);
    if ((modes & (1u << prk::MODE_AVX)) || fp->clear_fused)
        hipLaunchKernelGGL((prk::k_pix<false, true>), dim3(ntile * PRK_PIX_SPLIT), dim3(256), 0, s, *fp, nwin, wtag,
                           reinterpret_cast<const prk::SpanRec *>(recs));
#define PRK_SPAN_SHADE(MS) \
    hipLaunchKernelGGL((prk::k_span_shade<MS>), dim3(ntile), dim3(64 * prk::kShadeWaves), ls, s, *fp, offs, bins, P, \
                       SR, nwin, wtag)
    if (sc == (1u << prk::MODE_SC_GOURAUD)) PRK_SPAN_SHADE(prk::MODE_SC_GOURAUD);
    else if (sc == (1u << prk::MODE_SC_PHONG)) PRK_SPAN_SHADE(prk::MODE_SC_PHONG);
    else if (sc) PRK_SPAN_SHADE(-1);
#undef PRK_SPAN_SHADE
    return hipGetLastError();
}

}  // extern "C"
