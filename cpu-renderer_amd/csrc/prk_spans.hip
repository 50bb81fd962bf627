// prk_spans.hip — whole-object active edge tables (the span path).
//
// A render_entry_3d_object of several triangles is ONE AET in the reference:
// FillEdgeTable appends the visible edges of all its triangles to one list
// (projekt.cpp:3894-4117), MergeSort orders them by YMin (2-72), and
// DrawModelOptimized(RenderQueue,...) pairs consecutive list entries into
// spans across triangles (3654-3869).  The per-triangle kernels cannot
// express that, so objects of more than one triangle take this path:
//
//   k_objtri_count / k_objtri_emit   one thread per triangle of the pass's
//                 objects: FillEdgeTable (3894-4117) — the visible edges of
//                 every triangle, compacted in the reference's order (an
//                 exclusive scan over the per-triangle counts) — and each
//                 edge's MergeSort key.
//   sort          MergeSort (2-72) sorts by YMin with a tie order fixed by its
//                 recursion (merges take Half1 first on ties, a two-entry run
//                 keeps its order); the key (object, YMin, recursion path)
//                 reproduces it exactly under one device radix sort.
//   k_obj_walk    the AET walk with the reference's list operations (insertion
//                 scan, expiry, pairing, the two crossing swaps of 3831-3853
//                 with the P3 head/tail fix), stepping the paired edges row by
//                 row: one thread per small object or caller edge list, one
//                 wave per large object (k_obj_walk_wave: the list in LDS, the
//                 insertion scan, expiry compaction, the pairs' span setup and
//                 edge steps and both swap passes spread over the lanes).
//                 Pass 0 counts the object's emitted spans; pass 1 writes, for
//                 each span in submission order (object, row, pair), its lane-
//                 init record (FillLineOptimized SpanRec 1543-1835, or DrawModel
//                 ScSpanRec 298-412) and its pixel range.
//   k_span_tiles  span -> tile bin entries: every tile's count (wave-
//                 aggregated atomics), their scan, each span placed at its
//                 tile's offset + arrival rank (no sort: the visibility max
//                 does not depend on the order within a tile).
//   k_span_vis (prk_kernels.hip)  per-tile visibility over the spans with
//                 the 64-bit key max (tag = span index in submission order).
//   k_pix (prk_kernels.hip, span records indexed by span)  shading.
#include <atomic>

#include "prk_device.h"

namespace prk {
// Diagnostic builds (-DPRK_WPROF=1): walk_object_block accumulates its
// phases' cycles into fp.prof (prk_debug_counters): 0 insertion, 1 expiry,
// 2 pairing, 3 rows walked, 4 batches (insert_batch_b), 6 one-at-a-time
// insertions, 7 the whole walk, 8 new edges.
#ifndef PRK_WPROF
#define PRK_WPROF 0
#endif
#define PRK_WT() (PRK_WPROF ? __builtin_amdgcn_s_memtime() : 0ull)

// One object of the span path.
//   kind 0: triangles [g0, g0 + tris) of its draw's geometry: FillEdgeTable +
//           MergeSort, then the AET (render_entry_3d_object);
//   kind 1: a caller's edge_info list (edges [src, src + nsrc) of the pass's
//           edge input), drawn as DrawModelOptimized* draws it: no sort, the
//           insertion scan over every edge each row (3654-3713);
//   kind 2: one caller-given span (span input src): line_render_work /
//           buffer_line_render_work's pair of one row (2336-2348).
// g0 is the winner id (pass-local) of what it draws.
struct ObjDesc {
    uint32_t draw;
    uint32_t g0;
    uint32_t tris;
    uint32_t tri0;      // kind 0: its first triangle among the pass's object triangles
    uint32_t kind, src, nsrc;
    uint32_t k1off;     // kind 1: its first edge slot after the pass's triangle edges;
                        // bit 31 (kObjWave): walked by one wave (k_obj_walk_wave)
};
constexpr uint32_t kObjWave = 0x80000000u;
// An object's status in the parallel-rows walk (k_pr_*): 0 not taken,
// walked by rows, or failed its check (the workgroup walk takes it).
constexpr uint32_t kPrDone = 1u, kPrFailed = 2u;

// A run of objects as the host lists them (prk_api.hip ObjRun): a draw of
// kind 0 is `count` objects of `per` triangles (the last one shorter), kind 2
// one object per span, kind 1 one object; k_obj_tables expands them.
struct ObjRun {
    uint32_t kind, draw, obj0, count, per, tri_count, first_global, tri0, k0base, src_off, src_n, k1off;
};
__global__ void k_obj_tables(const ObjRun *__restrict__ runs, uint32_t nruns, uint32_t nobj, uint32_t wave_tris,
                             ObjDesc *__restrict__ objs, uint32_t *__restrict__ k0obj, uint32_t *__restrict__ k0tri0) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nobj) return;
    uint32_t lo = 0, hi = nruns;  // the last run with obj0 <= o
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (runs[mid].obj0 <= o) lo = mid;
        else hi = mid;
    }
    const ObjRun R = runs[lo];
    const uint32_t j = o - R.obj0;
    if (R.kind == 1) {
        objs[o] = ObjDesc{R.draw, R.first_global, 0u, 0u, 1u, R.src_off, R.src_n, R.k1off};
    } else if (R.kind == 2) {
        objs[o] = ObjDesc{R.draw, R.first_global + j, 0u, 0u, 2u, R.src_off + j, 1u, 0u};
    } else {
        const uint32_t t = j * R.per, n = min(R.per, R.tri_count - t);
        objs[o] = ObjDesc{R.draw, R.first_global + t, n, R.tri0 + t, 0u, 0u, 0u, n >= wave_tris ? kObjWave : 0u};
        k0obj[R.k0base + j] = o;
        k0tri0[R.k0base + j] = R.tri0 + t;
    }
}

// Caller edges (prk_edge = edge_info without Next, prk.h) and spans (prk_span).
struct EdgeIn {
    int32_t YMax;
    float XMin, ZMin, OneOverZMin, Gradient, ZGradient, OneOverZGradient;
    int32_t YMin;
    float UMin, VMin, UGradient, VGradient;
    int32_t Left;
    float MinColor[4], ColorGradient[4], MinNormal[3], NormalGradient[3];
};
struct SpanEndIn {
    float XMin, ZMin, OneOverZMin, UMin, VMin, MinColor[4], MinNormal[3];
};
struct SpanIn {
    SpanEndIn L, R;
    int32_t Row;
};

// Mutable edge_info of the object's AET (projekt.h:17-37) in global memory.
struct ObjEdge {
    float X, G, Z, ZG, W, WG, U, UG, V, VG;
    float N0, N1, N2, NG0, NG1, NG2;
    int32_t YMin, YMax, Left, Next;
    float C0, C1, C2, C3, CG0, CG1, CG2, CG3;  // MinColor / ColorGradient (DrawModel's Gouraud colour)
};
static_assert(sizeof(ObjEdge) == 112, "ObjEdge is seven dwordx4");

// Span of the span path: its row and pixel range [minx, maxx) (half-open,
// 1588-1592), DRAW_ST in flags.
struct SpanPos {
    int32_t row, minx, maxx;
    uint32_t flags;
};

struct SpanRecG {  // == SpanRec of prk_kernels.hip (FillLineOptimized lane init)
    float4 q0, q1, q2, q3;
};
// A DrawModel span (scalar semantics) of the span path: the values at MinX
// after the left clip (308-412) and the per-pixel increments, in the float
// slot order of the scalar sweeps (prk_kernels.hip SS_*), plus its texture.
// Its SpanRecG slot carries kScalarSpan in its first word, its SpanPos the
// half-open [MinX, MaxX + 1) and SPAN_SCALAR | mode << 8 (prk_device.h).
struct ScSpanRecG {
    float f[22];
    int32_t tex, pad;
};
static_assert(sizeof(ScSpanRecG) == 96, "scalar span record is six dwordx4");


__device__ __forceinline__ void obj_edge_store(ObjEdge &o, const Edge &E) {
    o.X = E.X; o.G = E.G; o.Z = E.Z; o.ZG = E.ZG; o.W = E.W; o.WG = E.WG;
    o.U = E.U; o.UG = E.UG; o.V = E.V; o.VG = E.VG;
    o.N0 = E.N0; o.N1 = E.N1; o.N2 = E.N2; o.NG0 = E.NG0; o.NG1 = E.NG1; o.NG2 = E.NG2;
    o.YMin = E.YMin; o.YMax = E.YMax; o.Left = E.Left; o.Next = -1;
    o.C0 = E.C0; o.C1 = E.C1; o.C2 = E.C2; o.C3 = E.C3;
    o.CG0 = E.CG0; o.CG1 = E.CG1; o.CG2 = E.CG2; o.CG3 = E.CG3;
}

// AET insertion order (3663-3667).
__device__ __forceinline__ bool obj_before(const ObjEdge &A, const ObjEdge &B) {
    return A.X < B.X || (A.X == B.X && (A.G < B.G || (A.G == B.G && A.Left < B.Left)));
}

// Edge step (3811-3829 / DrawModel 542-560), the fields mode M reads: AVX
// semantics X, Z, the normal, U, V, 1/z (the colour lanes are dead,
// 2029-2032); DrawModel also the colour (Gouraud) and drops what its mode
// never reads (ModeTraits).
template <int M>
__device__ __forceinline__ void obj_step(ObjEdge &E) {
    using TR = ModeTraits<M>;
    E.X += E.G;
    E.Z += E.ZG;
    if (TR::color) { E.C0 += E.CG0; E.C1 += E.CG1; E.C2 += E.CG2; E.C3 += E.CG3; }
    if (TR::phong) {
        float x = E.N0 + E.NG0, y = E.N1 + E.NG1, z = E.N2 + E.NG2;
        normalize_rcp(x, y, z);
        E.N0 = x; E.N1 = y; E.N2 = z;
    }
    if (TR::tex) {
        E.U += E.UG;
        E.V += E.VG;
        E.W += E.WG;
    }
}

// FillLineOptimized span setup (1543-1835) of the pair (L, R) at Row: the
// lane-init record and the covered range [MinX, MaxX).  False when the span
// covers nothing.
__device__ __forceinline__ bool obj_span(const FrameParams &fp, const ObjEdge &L, const ObjEdge &R, int32_t Row,
                                         int32_t texi, bool st, SpanRecG &rec, SpanPos &pos) {
    float XOffset;
    int32_t MinX, MaxX, XDiff;
    if (!span_ends(L.X, R.X, fp.W, st, MinX, MaxX, XDiff, XOffset)) return false;  // 1545-1592
    if (MinX >= MaxX) return false;
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
    rec.q0 = make_float4(__int_as_float((LeftXa & 0xFFFF) | (texi << 16)), XOffset, L.W, L.U);
    rec.q1 = make_float4(L.V, L.Z, IW, IU);
    rec.q2 = make_float4(IV, IZ, L.N0, L.N1);
    rec.q3 = make_float4(L.N2, IN0, IN1, IN2);
    pos.row = Row;
    pos.minx = MinX;
    pos.maxx = MaxX;
    pos.flags = st ? DRAW_ST : 0u;
    return true;
}

// DrawModel span setup (projekt.cpp:298-412) of the pair (L, R) at Row for
// mode M: the values at MinX (Current* += XOffset * Increment) and the
// per-pixel increments, as span_setup_scalar (prk_kernels.hip) computes them
// for the per-triangle sweeps, and the inclusive range [MinX, MaxX] (MaxX may
// be W: the one-past-the-row store into (Row + 1, 0)).  False when the span
// draws nothing (a NaN end: pinned).
template <int M>
__device__ __forceinline__ bool obj_span_scalar(const FrameParams &fp, const ObjEdge &L, const ObjEdge &R, int32_t Row,
                                                int32_t texi, ScSpanRecG &rec, SpanPos &pos) {
    using TR = ModeTraits<M>;
    const int32_t W = fp.W;
    float XOffset = 0.0f;
    const float XDiff = roundf(R.X - L.X);  // 311-312
    float IW = 0, IU = 0, IV = 0, IZ = 0, IN0 = 0, IN1 = 0, IN2 = 0;
    float IC0 = 0, IC1 = 0, IC2 = 0, IC3 = 0;
    if (XDiff != 0.0f) {  // 329-360
        constexpr bool kT = TR::tex, kP = TR::phong, kC = TR::color;
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
    if (LeftX != LeftX || RightX != RightX) return false;
    const int32_t MinX = round_s32(LeftX), MaxX = round_s32(RightX);  // 402-406
    if (MaxX < MinX) return false;
    for (int k = 0; k < 22; ++k) rec.f[k] = 0.0f;
    rec.f[0] = L.Z + XOffset * IZ;  // 408-412 (SS_Z, SS_IZ)
    rec.f[1] = IZ;
    if (TR::tex) {  // SS_W, SS_U, SS_V, SS_IW, SS_IU, SS_IV
        rec.f[2] = L.W + XOffset * IW; rec.f[5] = IW;
        rec.f[3] = L.U + XOffset * IU; rec.f[6] = IU;
        rec.f[4] = L.V + XOffset * IV; rec.f[7] = IV;
    }
    if (TR::phong) {  // SS_N0..2, SS_IN0..2
        rec.f[8] = L.N0 + XOffset * IN0; rec.f[11] = IN0;
        rec.f[9] = L.N1 + XOffset * IN1; rec.f[12] = IN1;
        rec.f[10] = L.N2 + XOffset * IN2; rec.f[13] = IN2;
    }
    if (TR::color) {  // SS_C0..3, SS_IC0..3
        rec.f[14] = L.C0 + XOffset * IC0; rec.f[18] = IC0;
        rec.f[15] = L.C1 + XOffset * IC1; rec.f[19] = IC1;
        rec.f[16] = L.C2 + XOffset * IC2; rec.f[20] = IC2;
        rec.f[17] = L.C3 + XOffset * IC3; rec.f[21] = IC3;
    }
    rec.tex = TR::tex ? texi : 0;
    rec.pad = 0;
    pos.row = Row;
    pos.minx = MinX;
    pos.maxx = MaxX + 1;
    pos.flags = SPAN_SCALAR | ((uint32_t)M << 8);
    return true;
}

// One thread per object.  pass 0: span counts -> counts[o]; pass 1: spans at
// offs[o] + k.  edges / ord / tmp: 3 slots per triangle of the pass.
__device__ __forceinline__ void obj_edge_in(ObjEdge &o, const EdgeIn &e) {
    o.X = e.XMin; o.G = e.Gradient; o.Z = e.ZMin; o.ZG = e.ZGradient; o.W = e.OneOverZMin;
    o.WG = e.OneOverZGradient; o.U = e.UMin; o.UG = e.UGradient; o.V = e.VMin; o.VG = e.VGradient;
    o.N0 = e.MinNormal[0]; o.N1 = e.MinNormal[1]; o.N2 = e.MinNormal[2];
    o.NG0 = e.NormalGradient[0]; o.NG1 = e.NormalGradient[1]; o.NG2 = e.NormalGradient[2];
    o.YMin = e.YMin; o.YMax = e.YMax; o.Left = e.Left; o.Next = -1;
    o.C0 = e.MinColor[0]; o.C1 = e.MinColor[1]; o.C2 = e.MinColor[2]; o.C3 = e.MinColor[3];
    o.CG0 = e.ColorGradient[0]; o.CG1 = e.ColorGradient[1]; o.CG2 = e.ColorGradient[2];
    o.CG3 = e.ColorGradient[3];
}
__device__ __forceinline__ ObjEdge span_end_in(const SpanEndIn &e) {  // FillLinesOptimized 648-670
    ObjEdge o;
    o.X = e.XMin; o.Z = e.ZMin; o.W = e.OneOverZMin; o.U = e.UMin; o.V = e.VMin;
    o.N0 = e.MinNormal[0]; o.N1 = e.MinNormal[1]; o.N2 = e.MinNormal[2];
    o.G = o.ZG = o.WG = o.UG = o.VG = o.NG0 = o.NG1 = o.NG2 = 0.0f;
    o.C0 = e.MinColor[0]; o.C1 = e.MinColor[1]; o.C2 = e.MinColor[2]; o.C3 = e.MinColor[3];
    o.CG0 = o.CG1 = o.CG2 = o.CG3 = 0.0f;
    o.YMin = o.YMax = o.Left = 0;
    o.Next = -1;
    return o;
}

// ---------------------------------------------------------------------------
// FillEdgeTable of the pass's objects, one thread per triangle.
// ---------------------------------------------------------------------------
// Which of a triangle's edges {0,1},{1,2},{2,0} FillEdgeTable writes (bit k):
// none unless it passes the back-face test (3926-3943), then those with
// MaxY > 0 (3968) and MinY != MaxY (4066) — tri_edges' `vis`.  rows: the
// rows [max(YMin, row_lo), min(YMax, row_hi)) its visible edges can be
// active on (YMax = round(MaxY) 3988, YMin = Maximum(0, round(MinY)) 3999),
// summed — twice the most spans they can take part in.
__device__ __forceinline__ uint32_t tri_vis_mask(const FrameParams &fp, const DrawRec &d, uint32_t gt,
                                                 int32_t row_lo, int32_t row_hi, uint32_t *rows = nullptr) {
    V3 cam[3], proj[3];
    load_positions(d, gt, fp, cam, proj);
    if (!front_facing(proj)) return 0u;
    uint32_t m = 0, r = 0;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const float y0 = proj[e].y, y1 = proj[(e + 1) % 3].y;
        const bool sw = y0 > y1;  // 3957-3966
        const float mn = sw ? y1 : y0, mx = sw ? y0 : y1;
        if (mx > 0 && mn - mx != 0) {
            m |= 1u << e;
            const float rm = (float)round_s32(mn);
            const int32_t ymin = (int32_t)(0.0f > rm ? 0.0f : rm), ymax = round_s32(mx);
            r += (uint32_t)max(0, min(ymax, row_hi) - max(ymin, row_lo));
        }
    }
    if (rows) *rows = r;
    return m;
}

// Rows a draw's spans can lie on: [row0, min(H, row1)) of the pass's band,
// from row0 - 1 for DrawModel (its one-past-the-row store, 423-538).
__device__ __forceinline__ int32_t draw_row_lo(const FrameParams &fp, const DrawRec &d) {
    return d.mode != MODE_AVX ? fp.row0 - 1 : fp.row0;
}
__device__ __forceinline__ int32_t draw_row_hi(const FrameParams &fp) { return min(fp.H, fp.row1); }

// The kind-0 object (index into the pass's kind-0 list) of object triangle s.
__device__ __forceinline__ uint32_t obj_of_tri(const uint32_t *__restrict__ k0tri0, uint32_t nk0, uint32_t s) {
    uint32_t lo = 0, hi = nk0 - 1;
    while (lo < hi) {  // last object with tri0 <= s
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (k0tri0[mid] <= s) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// MergeSort (projekt.cpp:2-72) as a sort key.  The recursion sorts by YMin;
// among equal YMin it leaves a two-entry run in its order (13: swap only on
// '>') and puts every Half1 entry before every Half0 entry (51-57: Half0 only
// on strict '<').  So entry i of n precedes entry j of equal YMin iff, at the
// recursion node that separates them, i is the first of a two-entry run or
// lies in Half1: the path of branch bits from the root (Half1 = 0, Half0 = 1,
// run position last), left-aligned in `pbits` (more than the recursion's
// depth, ceil(log2 n)), orders ties exactly.
struct SortKeyBits {
    uint32_t pbits, ybits;  // path bits, YMin bits (YMin clamped to ycap = H: rows >= H are never walked)
    int32_t ycap;
};
__device__ __forceinline__ uint64_t merge_path(uint32_t i, uint32_t n, uint32_t pbits) {
    uint32_t first = 0, count = n;
    uint64_t path = 0;
    uint32_t bits = 0;
    while (count > 2) {
        const uint32_t h0 = count / 2;  // Half0 = [first, first + h0)
        if (i < first + h0) {
            path = (path << 1) | 1u;
            count = h0;
        } else {
            path <<= 1;
            first += h0;
            count -= h0;
        }
        ++bits;
    }
    if (count == 2) {
        path = (path << 1) | (i - first);
        ++bits;
    }
    return path << (pbits - bits);
}

// Visible edge count (ecnt) and active-row count (rcnt) of every object
// triangle (ecnt[ntri] = rcnt[ntri] = 0: the scans' totals).
__global__ void k_objtri_count(FrameParams fp, const ObjDesc *__restrict__ objs, const uint32_t *__restrict__ k0obj,
                               const uint32_t *__restrict__ k0tri0, uint32_t nk0, uint32_t ntri,
                               uint32_t *__restrict__ ecnt, unsigned long long *__restrict__ rcnt) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > ntri) return;
    if (s == ntri) {
        ecnt[s] = 0;
        rcnt[s] = 0;
        return;
    }
    const ObjDesc od = objs[k0obj[obj_of_tri(k0tri0, nk0, s)]];
    const DrawRec &d = fp.draws[od.draw];
    const uint32_t g = od.g0 + (s - od.tri0);
    uint32_t rows = 0;
    ecnt[s] = (uint32_t)__popc(tri_vis_mask(fp, d, d.geom_tri0 + (g - d.first_global), draw_row_lo(fp, d),
                                            draw_row_hi(fp), &rows));
    rcnt[s] = rows;
}

// The visible edges of every object triangle (FillEdgeTable 3947-4111, in the
// reference's order: triangle by triangle, edges {0,1},{1,2},{2,0}) at
// escan[s], with their MergeSort keys (object, min(YMin, H), path); the key
// slots past the visible edges keep the all-ones padding (sorted last).
template <int M>
__device__ __forceinline__ void objtri_edges(const FrameParams &fp, const DrawRec &d, uint32_t gt, ObjEdge *out,
                                             uint32_t mask) {
    TriRaw<M> raw;
    load_tri<M>(d, gt, raw);
    Edge e[3];
    bool vis[3];
    tri_edges<M>(raw, d, fp, e[0], e[1], e[2], vis);
    uint32_t k = 0;
#pragma unroll
    for (int j = 0; j < 3; ++j)
        if ((mask >> j) & 1u) obj_edge_store(out[k++], e[j]);
}

__global__ void k_objtri_emit(FrameParams fp, const ObjDesc *__restrict__ objs, const uint32_t *__restrict__ k0obj,
                              const uint32_t *__restrict__ k0tri0, uint32_t nk0, uint32_t ntri,
                              const uint32_t *__restrict__ escan, SortKeyBits kb, ObjEdge *__restrict__ edges,
                              unsigned long long *__restrict__ keys, uint32_t *__restrict__ vals) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= ntri) return;
    const uint32_t j = obj_of_tri(k0tri0, nk0, s);
    const ObjDesc od = objs[k0obj[j]];
    const DrawRec &d = fp.draws[od.draw];
    const uint32_t g = od.g0 + (s - od.tri0);
    const uint32_t gt = d.geom_tri0 + (g - d.first_global);
    const uint32_t mask = tri_vis_mask(fp, d, gt, 0, 0);
    if (!mask) return;
    const uint32_t e0 = escan[s];
    switch (d.mode) {
        case MODE_AVX: objtri_edges<MODE_AVX>(fp, d, gt, edges + e0, mask); break;
        case MODE_SC_GOURAUD: objtri_edges<MODE_SC_GOURAUD>(fp, d, gt, edges + e0, mask); break;
        case MODE_SC_GOURAUD_TEX: objtri_edges<MODE_SC_GOURAUD_TEX>(fp, d, gt, edges + e0, mask); break;
        case MODE_SC_PHONG: objtri_edges<MODE_SC_PHONG>(fp, d, gt, edges + e0, mask); break;
        default: objtri_edges<MODE_SC_PHONG_TEX>(fp, d, gt, edges + e0, mask); break;
    }
    const uint32_t ob = escan[od.tri0], n = escan[od.tri0 + od.tris] - ob;
    const uint32_t c = (uint32_t)__popc(mask);
    for (uint32_t k = 0; k < c; ++k) {
        const uint64_t ymin = (uint64_t)min(edges[e0 + k].YMin, kb.ycap);
        keys[e0 + k] = ((uint64_t)j << (kb.ybits + kb.pbits)) | (ymin << kb.pbits) |
                       merge_path(e0 + k - ob, n, kb.pbits);
        vals[e0 + k] = e0 + k;
    }
}

// Span slots of every object: the most spans its walk can emit — a span
// pairs two entries active on its row, an entry is active on the rows
// [YMin, YMax) of its edge walked — so half its edges' active rows (kind 0:
// from the per-triangle counts; kind 1: its caller edges; kind 2: one).
__global__ void k_obj_bound(FrameParams fp, const ObjDesc *__restrict__ objs, uint32_t nobj,
                            const unsigned long long *__restrict__ rscan, const EdgeIn *__restrict__ edges_in,
                            unsigned long long *__restrict__ bound) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o > nobj) return;
    if (o == nobj) {
        bound[o] = 0;
        return;
    }
    const ObjDesc od = objs[o];
    unsigned long long b = 1;
    if (od.kind == 0) {
        b = (rscan[od.tri0 + od.tris] - rscan[od.tri0]) / 2;
    } else if (od.kind == 1) {
        const DrawRec &d = fp.draws[od.draw];
        const int32_t lo = draw_row_lo(fp, d), hi = draw_row_hi(fp);
        unsigned long long r = 0;
        for (uint32_t e = 0; e < od.nsrc; ++e) {
            const EdgeIn &E = edges_in[od.src + e];
            r += (unsigned long long)max(0, min(E.YMax, hi) - max(E.YMin, lo));
        }
        b = r / 2;
    }
    bound[o] = b;
}

// The walk's working copy of every object's edges: the triangle edges in
// MergeSort order (work[i] = edges[ord[i]], i < total0), then the caller edge
// lists (kind 1) as given.  Re-made before each walk pass (the walk steps it).
// (wy, when given: the triangle edges' (YMin, YMax), for k_obj_seg)
__global__ void k_obj_gather(const ObjEdge *__restrict__ edges, const uint32_t *__restrict__ ord,
                             const uint32_t *__restrict__ total0p, const EdgeIn *__restrict__ edges_in,
                             const uint32_t *__restrict__ k1src, uint32_t nk1, ObjEdge *__restrict__ work,
                             int2 *__restrict__ wy) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t total0 = *total0p;
    if (i < total0) {
        if (!ord) return;  // (k_obj_sort_local placed them)
        const ObjEdge e = edges[ord[i]];
        work[i] = e;
        if (wy) wy[i] = make_int2(e.YMin, e.YMax);
    } else if (i - total0 < nk1) {
        obj_edge_in(work[i], edges_in[k1src[i - total0]]);
    }
}

// An object's edges in the working copy: [e0, e0 + n).
__device__ __forceinline__ void obj_range(const ObjDesc &od, const uint32_t *__restrict__ escan, uint32_t total0,
                                          uint32_t &e0, uint32_t &n) {
    if (od.kind == 0) {
        e0 = escan[od.tri0];
        n = escan[od.tri0 + od.tris] - e0;
    } else {
        e0 = total0 + (od.k1off & ~kObjWave);
        n = od.nsrc;
    }
}

// One span of the pair (L, R) at Row, written at span slot `at` (when `write`).
template <int M>
__device__ __forceinline__ bool emit_span(const FrameParams &fp, const ObjEdge &L, const ObjEdge &R, int32_t Row,
                                          const DrawRec &d, bool st, uint32_t g0, bool write, uint32_t at,
                                          SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                                          SpanPos *__restrict__ pos, uint32_t *__restrict__ span_tri) {
    SpanPos sp;
    if constexpr (M != MODE_AVX) {
        ScSpanRecG srec;
        if (!obj_span_scalar<M>(fp, L, R, Row, d.tex, srec, sp)) return false;
        if (write) {
            SpanRecG mark;
            mark.q0 = make_float4(__uint_as_float(kScalarSpan), 0.0f, 0.0f, 0.0f);
            mark.q1 = mark.q2 = mark.q3 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            recs[at] = mark;
            srecs[at] = srec;
        }
    } else {
        SpanRecG rec;
        if (!obj_span(fp, L, R, Row, d.tex, st, rec, sp)) return false;
        if (write) recs[at] = rec;
    }
    if (write) {
        pos[at] = sp;
        span_tri[at] = g0;
    }
    return true;
}

// The list fields of the thread walk (links, keys, row range), read and
// written through one of two stores: the working copy itself (GLinks), or
// per-thread LDS mirrors (LLinks: objects of at most kLinkCap edges), so the
// list's chains of dependent accesses (insertion scans, expiry, pairing and
// swaps) run at LDS latency; the edge records stay in device memory, read
// for a span and stepped per pair, off those chains.  LLinks steps its X
// mirror with obj_step's own add.
struct GLinks {
    ObjEdge *E;
    __device__ __forceinline__ int32_t next(int i) const { return E[i].Next; }
    __device__ __forceinline__ void set_next(int i, int32_t v) const { E[i].Next = v; }
    __device__ __forceinline__ float x(int i) const { return E[i].X; }
    __device__ __forceinline__ int32_t ymin(int i) const { return E[i].YMin; }
    __device__ __forceinline__ int32_t ymax(int i) const { return E[i].YMax; }
    __device__ __forceinline__ bool before(int a, int b) const { return obj_before(E[a], E[b]); }
    __device__ __forceinline__ void stepped(int) const {}  // (obj_step stepped E[i].X)
    static constexpr bool kCache = false;  // (the list reads the records' X and links)
};
constexpr int kLinkCap = 48;     // edges per object with LDS links (C3b as 16-triangle objects: 48)
constexpr int kLinkThreads = 64;  // k_obj_walk's workgroup
// 13 B per edge (YMax relative to the object's first row; YMin is read from
// the working copy, only where the sorted insertion scan advances), so four
// 64-thread workgroups fit a CU's LDS.
// (CAP: edges per thread; k_obj_walk_seg's segments take a smaller mirror,
// so more of its waves fit a CU)
template <int CAP>
struct LinkLdsT {
    float x[CAP * kLinkThreads], g[CAP * kLinkThreads];
    int16_t ymax[CAP * kLinkThreads];
    int16_t nxt[CAP * kLinkThreads];
    int8_t left[CAP * kLinkThreads];
};
using LinkLds = LinkLdsT<kLinkCap>;
template <int CAP>
struct LLinksT {
    LinkLdsT<CAP> *L;
    const ObjEdge *E;
    int lane;
    int32_t row0;  // the object's first row: YMax - row0 in (0, 32767]
    __device__ __forceinline__ int at(int i) const { return i * kLinkThreads + lane; }
    __device__ __forceinline__ int32_t next(int i) const { return L->nxt[at(i)]; }
    __device__ __forceinline__ void set_next(int i, int32_t v) const { L->nxt[at(i)] = (int16_t)v; }
    __device__ __forceinline__ float x(int i) const { return L->x[at(i)]; }
    __device__ __forceinline__ int32_t ymin(int i) const { return E[i].YMin; }
    __device__ __forceinline__ int32_t ymax(int i) const { return row0 + (int32_t)L->ymax[at(i)]; }
    __device__ __forceinline__ bool before(int a, int b) const {
        const float ax = x(a), bx = x(b), ag = L->g[at(a)], bg = L->g[at(b)];
        return ax < bx || (ax == bx && (ag < bg || (ag == bg && L->left[at(a)] < L->left[at(b)])));
    }
    __device__ __forceinline__ void stepped(int i) const { L->x[at(i)] += L->g[at(i)]; }  // E.X += E.G (obj_step)
#ifndef PRK_OBJ_PAIR_CACHE
#define PRK_OBJ_PAIR_CACHE 1
#endif
    static constexpr bool kCache = PRK_OBJ_PAIR_CACHE;
};
using LLinks = LLinksT<kLinkCap>;

// An edge record held in seven named float4 registers (ObjEdge's layout): a
// loop-carried ObjEdge went to scratch.
#define PRK_ER(w) float4 w##0, w##1, w##2, w##3, w##4, w##5, w##6
#define PRK_ER_ZERO(w) \
    do { w##0 = w##1 = w##2 = w##3 = w##4 = w##5 = w##6 = make_float4(0.0f, 0.0f, 0.0f, 0.0f); } while (0)
#define PRK_ER_LOAD(w, p)                                                      \
    do {                                                                       \
        const float4 *s_ = reinterpret_cast<const float4 *>(p);               \
        w##0 = s_[0]; w##1 = s_[1]; w##2 = s_[2]; w##3 = s_[3];               \
        w##4 = s_[4]; w##5 = s_[5]; w##6 = s_[6];                             \
    } while (0)
#define PRK_ER_STORE(p, w)                                                     \
    do {                                                                       \
        float4 *d_ = reinterpret_cast<float4 *>(p);                           \
        d_[0] = w##0; d_[1] = w##1; d_[2] = w##2; d_[3] = w##3;               \
        d_[4] = w##4; d_[5] = w##5; d_[6] = w##6;                             \
    } while (0)
#define PRK_ER_SWAP(a, b)                                                                 \
    do {                                                                                  \
        float4 t_;                                                                        \
        t_ = a##0; a##0 = b##0; b##0 = t_; t_ = a##1; a##1 = b##1; b##1 = t_;             \
        t_ = a##2; a##2 = b##2; b##2 = t_; t_ = a##3; a##3 = b##3; b##3 = t_;             \
        t_ = a##4; a##4 = b##4; b##4 = t_; t_ = a##5; a##5 = b##5; b##5 = t_;             \
        t_ = a##6; a##6 = b##6; b##6 = t_;                                                \
    } while (0)
__device__ __forceinline__ ObjEdge er_edge(float4 q0, float4 q1, float4 q2, float4 q3, float4 q4, float4 q5,
                                           float4 q6) {
    ObjEdge e;
    e.X = q0.x; e.G = q0.y; e.Z = q0.z; e.ZG = q0.w;
    e.W = q1.x; e.WG = q1.y; e.U = q1.z; e.UG = q1.w;
    e.V = q2.x; e.VG = q2.y; e.N0 = q2.z; e.N1 = q2.w;
    e.N2 = q3.x; e.NG0 = q3.y; e.NG1 = q3.z; e.NG2 = q3.w;
    e.YMin = __float_as_int(q4.x); e.YMax = __float_as_int(q4.y); e.Left = __float_as_int(q4.z);
    e.Next = __float_as_int(q4.w);
    e.C0 = q5.x; e.C1 = q5.y; e.C2 = q5.z; e.C3 = q5.w;
    e.CG0 = q6.x; e.CG1 = q6.y; e.CG2 = q6.z; e.CG3 = q6.w;
    return e;
}
#define PRK_ER_EDGE(w) er_edge(w##0, w##1, w##2, w##3, w##4, w##5, w##6)
#define PRK_ER_FROM(w, e)                                                                              \
    do {                                                                                               \
        w##0 = make_float4((e).X, (e).G, (e).Z, (e).ZG);                                               \
        w##1 = make_float4((e).W, (e).WG, (e).U, (e).UG);                                              \
        w##2 = make_float4((e).V, (e).VG, (e).N0, (e).N1);                                             \
        w##3 = make_float4((e).N2, (e).NG0, (e).NG1, (e).NG2);                                         \
        w##5 = make_float4((e).C0, (e).C1, (e).C2, (e).C3);                                            \
    } while (0)  /* (q4, q6: row range, link, colour gradient — not stepped) */

// MergeSort of objects of at most 64 edges without the device radix sort:
// one wave per object, lane i ranks edge i's key (object, min(YMin, H),
// recursion path: unique within the object) among the object's keys and
// copies the edge to the working copy at that rank -- the order the sort +
// k_obj_gather give (their cost on C3b as 16-triangle objects: 0.46 ms).
constexpr int kLocalSortEdges = 64;
__global__ void __launch_bounds__(256) k_obj_sort_local(const ObjDesc *__restrict__ objs,
                                                        const uint32_t *__restrict__ k0obj, uint32_t nk0,
                                                        const uint32_t *__restrict__ escan,
                                                        const unsigned long long *__restrict__ keys,
                                                        const ObjEdge *__restrict__ edges, ObjEdge *__restrict__ work,
                                                        int2 *__restrict__ wy, uint32_t *__restrict__ err) {
    const uint32_t j = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int lane = (int)(threadIdx.x & 63);
    if (j >= nk0) return;
    const ObjDesc od = objs[k0obj[j]];
    const uint32_t ob = escan[od.tri0], n = escan[od.tri0 + od.tris] - ob;
    if (n > (uint32_t)kLocalSortEdges) {  // (never: the host takes this path only for such objects)
        if (lane == 0) atomicOr(err, 4u);
        return;
    }
    const unsigned long long k = lane < (int)n ? keys[ob + lane] : ~0ull;
    const uint32_t klo = (uint32_t)k, khi = (uint32_t)(k >> 32);
    uint32_t rank = 0;
    for (uint32_t q = 0; q < n; ++q) {
        const uint32_t qlo = (uint32_t)__builtin_amdgcn_readlane((int)klo, (int)q);
        const uint32_t qhi = (uint32_t)__builtin_amdgcn_readlane((int)khi, (int)q);
        rank += (qhi < khi || (qhi == khi && qlo < klo)) ? 1u : 0u;
    }
    if (lane < (int)n) {
        PRK_ER(w);
        PRK_ER_LOAD(w, &edges[ob + lane]);
        PRK_ER_STORE(&work[ob + rank], w);
        if (wy) wy[ob + rank] = make_int2(__float_as_int(w4.x), __float_as_int(w4.y));
    }
}

// The AET walk of one object by one thread (small objects, caller edge
// lists): E = its n edges, sorted (kind 0) or as given (kind 1).  Its spans
// go to slots [base, base + bound) in emission order.
template <int M, class LK>
__device__ void walk_object(const FrameParams &fp, const ObjDesc &od, const DrawRec &d, ObjEdge *__restrict__ E,
                            uint32_t n, uint32_t base, uint32_t bound, SpanRecG *__restrict__ recs,
                            ScSpanRecG *__restrict__ srecs, SpanPos *__restrict__ pos,
                            uint32_t *__restrict__ span_tri, uint32_t *__restrict__ err, const LK lk) {
    constexpr bool kScalar = M != MODE_AVX;
    const bool st = (d.flags & DRAW_ST) != 0;
    const bool given = od.kind == 1;  // a caller's edge list: scanned whole every row
    uint32_t emitted = 0;
    // The slots the walk leaves unused (spans that cover nothing take none)
    // are marked row -1 at the end, binned nowhere: frames without large
    // objects skip the memset of every slot (prk_api.hip).
    if (n == 0) {
        for (uint32_t q = 0; q < bound; ++q) pos[base + q] = SpanPos{-1, 0, 0, 0u};
        return;
    }
    // The AET walk of DrawModelOptimized(RenderQueue,...) (3626-3869) /
    // DrawModel (173-598): the same list logic.
    const int32_t FirstRow = lk.ymin(0);
    int32_t MaxRow = lk.ymax(0);
    for (uint32_t i = 1; i < n; ++i) MaxRow = max(MaxRow, lk.ymax((int)i));
    const int32_t MaxY = min(min(MaxRow, fp.H), fp.row1);
    // DrawModel's span of row row0-1 can store its one-past-the-row pixel
    // into (row0, 0)
    const int32_t RowLo = kScalar ? fp.row0 - 1 : fp.row0;
    for (uint32_t i = 0; i < n; ++i) lk.set_next((int)i, -1);
    int32_t Head = -1, Tail = -1;
    uint32_t ins = 0;  // next sorted edge to insert (sorted by YMin)
    int32_t nym = FirstRow;  // its YMin (INT32_MAX past the end)
    // (LK::kCache) the last pair's records, stepped in registers, written back
    // when another pair needs the registers (the list fields live in LK, so
    // nothing reads a record's stale copy meanwhile; the working copy is not
    // read after the walk)
    PRK_ER(ca);
    PRK_ER(cb);
    PRK_ER_ZERO(ca);
    PRK_ER_ZERO(cb);
    int32_t ia = -1, ib = -1;
    for (int32_t Row = FirstRow; Row < MaxY; ++Row) {
        // insertion (3654-3713): the edges with YMin == Row, in array
        // order.  Sorted lists (MergeSort) hold them contiguously; a
        // caller's list is scanned whole, as the reference does.
        uint32_t i0 = 0, i1 = n;
        if (!given) {
            while (ins < n && nym < Row) nym = ++ins < n ? lk.ymin((int)ins) : INT32_MAX;
            i0 = ins;
            while (ins < n && nym == Row) nym = ++ins < n ? lk.ymin((int)ins) : INT32_MAX;
            i1 = ins;
        }
        for (uint32_t ii = i0; ii < i1; ++ii) {
            if (given && lk.ymin((int)ii) != Row) continue;  // (sorted: all of [i0, i1) start here)
            const int32_t c = (int32_t)ii;
            if (Head >= 0) {
                if (lk.before(c, Head)) {
                    lk.set_next(c, Head);
                    Head = c;
                } else {
                    int32_t Cmp = Head, Prev = Head;
                    while (Cmp != Tail) {
                        Cmp = lk.next(Cmp);
                        if (lk.before(c, Cmp)) {
                            lk.set_next(c, Cmp);
                            lk.set_next(Prev, c);
                            Cmp = Tail;
                        } else {
                            Prev = Cmp;
                        }
                    }
                    if (Prev == Cmp) {
                        lk.set_next(Tail, c);
                        Tail = c;
                    }
                }
            } else {
                Head = c;
                Tail = c;
            }
        }
        while (Head >= 0 && lk.ymax(Head) <= Row) {  // expiry 3715-3720
            const int32_t Rm = Head;
            Head = lk.next(Head);
            lk.set_next(Rm, -1);
        }
        if (Head < 0) {  // pin: the reference dereferences NULL
            Tail = -1;
            // nothing happens on the rows before the next insertion: go there
            if (!given) {
                if (ins >= n) break;
                Row = max(Row, nym - 1);
            }
            continue;
        }
        {
            int32_t Prev = Head, Chk = Head;  // 3722-3749
            while (Chk != Tail) {
                Chk = lk.next(Chk);
                if (lk.ymax(Chk) <= Row) {
                    if (Chk == Tail) {
                        Tail = Prev;
                        lk.set_next(Tail, -1);
                        Chk = Tail;
                    } else {
                        lk.set_next(Prev, lk.next(Chk));
                        Chk = Prev;
                    }
                }
                Prev = Chk;
            }
        }
        int32_t PrevCur = -1, PrevNext = -1;  // pairing 3751-3869
        int32_t Cur = Head, Next = lk.next(Cur);
        while (Next >= 0) {
            if constexpr (LK::kCache) {
                // the pair's records: in registers while the same two edges
                // pair row after row (either order), else written back and
                // the new pair's loaded
                if (!(Cur == ia && Next == ib)) {
                    if (Cur == ib && Next == ia) {
                        PRK_ER_SWAP(ca, cb);
                        ib = ia;
                        ia = Cur;
                    } else {
                        if (ia >= 0) {
                            PRK_ER_STORE(&E[ia], ca);
                            PRK_ER_STORE(&E[ib], cb);
                        }
                        PRK_ER_LOAD(ca, &E[Cur]);
                        PRK_ER_LOAD(cb, &E[Next]);
                        ia = Cur;
                        ib = Next;
                    }
                }
                ObjEdge eA = PRK_ER_EDGE(ca), eB = PRK_ER_EDGE(cb);
                if (Row >= RowLo &&  // a span of this pass's rows (3759-3809 / 298-538)
                    emit_span<M>(fp, eA, eB, Row, d, st, od.g0, emitted < bound, base + emitted, recs, srecs, pos,
                                 span_tri)) {
                    if (emitted >= bound) atomicOr(err, 2u);  // (never: the bound holds every span)
                    ++emitted;
                }
                obj_step<M>(eA);  // 3811-3829
                obj_step<M>(eB);
                PRK_ER_FROM(ca, eA);
                PRK_ER_FROM(cb, eB);
            } else {
                if (Row >= RowLo &&
                    emit_span<M>(fp, E[Cur], E[Next], Row, d, st, od.g0, emitted < bound, base + emitted, recs,
                                 srecs, pos, span_tri)) {
                    if (emitted >= bound) atomicOr(err, 2u);
                    ++emitted;
                }
                obj_step<M>(E[Cur]);
                obj_step<M>(E[Next]);
            }
            lk.stepped(Cur);
            lk.stepped(Next);
            if (lk.x(Cur) > lk.x(Next)) {  // 3831-3841
                lk.set_next(Cur, lk.next(Next));
                lk.set_next(Next, Cur);
                if (PrevNext >= 0) lk.set_next(PrevNext, Next);
                else Head = Next;               // P3
                if (Tail == Next) Tail = Cur;   // P3
                Cur = Next;
                Next = lk.next(Cur);
            }
            if (PrevNext >= 0) {  // 3843-3853
                if (lk.x(PrevNext) > lk.x(Cur)) {
                    lk.set_next(PrevNext, lk.next(Cur));
                    lk.set_next(Cur, PrevNext);
                    lk.set_next(PrevCur, Cur);
                    PrevNext = Cur;
                    Cur = lk.next(PrevNext);
                }
            }
            PrevCur = Cur;
            PrevNext = Next;
            if (lk.next(Next) >= 0) {
                Cur = lk.next(Next);
                Next = lk.next(Cur);
            } else {
                Next = -1;
            }
        }
    }
    for (uint32_t q = emitted; q < bound; ++q) pos[base + q] = SpanPos{-1, 0, 0, 0u};
}

#ifndef PRK_OBJ_LDS_LINKS
#define PRK_OBJ_LDS_LINKS 1
#endif
// LINKS: the launch holds triangle objects small enough for LDS links (the
// 40-KB mirror is allocated only then: it limits a CU to four workgroups).
template <bool LINKS>
__global__ void __launch_bounds__(kLinkThreads, 1) k_obj_walk(FrameParams fp, const ObjDesc *__restrict__ objs, uint32_t nobj,
                                                 const uint32_t *__restrict__ escan,
                                                 const uint32_t *__restrict__ total0p, ObjEdge *__restrict__ work,
                                                 const unsigned long long *__restrict__ soff,
                                                 SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                                                 SpanPos *__restrict__ pos, uint32_t *__restrict__ span_tri,
                                                 const SpanIn *__restrict__ spans_in, uint32_t *__restrict__ err,
                                                 uint32_t segmented) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nobj) return;
    const ObjDesc od = objs[o];
    if (od.kind != 2 && (od.k1off & kObjWave)) return;  // k_obj_walk_wave's
    if (od.kind == 0 && segmented) return;             // k_obj_walk_seg's
    const DrawRec &d = fp.draws[od.draw];
    const bool st = (d.flags & DRAW_ST) != 0;
    const uint32_t base = (uint32_t)soff[o], bound = (uint32_t)(soff[o + 1] - soff[o]);
    if (od.kind == 2) {  // one caller-given span (DoLineRenderWork / DoBufferLineRenderWork)
        const SpanIn sp = spans_in[od.src];
        uint32_t used = 0;
        if (sp.Row >= fp.row0 && sp.Row < fp.row1 && sp.Row < fp.H && bound)
            used = emit_span<MODE_AVX>(fp, span_end_in(sp.L), span_end_in(sp.R), sp.Row, d, st, od.g0, true, base,
                                       recs, srecs, pos, span_tri) ? 1u : 0u;
        for (uint32_t q = used; q < bound; ++q) pos[base + q] = SpanPos{-1, 0, 0, 0u};  // (as walk_object's)
        return;
    }
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    ObjEdge *E = work + e0;
    __shared__ typename std::conditional<LINKS, LinkLds, char>::type lds_;
    LinkLds &lds = *reinterpret_cast<LinkLds *>(&lds_);
    // (triangle edges only: their Left is 0 / 1, a caller's edge_info.Left any b32)
    bool in_lds = LINKS && od.kind == 0 && n > 0 && n <= (uint32_t)kLinkCap;
    const int32_t row0 = n ? E[0].YMin : 0;  // (sorted: the smallest YMin)
    if (in_lds) {
        int32_t hi = row0;
        for (uint32_t i = 0; i < n; ++i) hi = max(hi, E[i].YMax);
        in_lds = hi - row0 <= 32767;
    }
    if (in_lds) {  // the list fields' mirrors
        const int lane = (int)threadIdx.x;
        for (uint32_t i = 0; i < n; ++i) {
            const int a = (int)i * kLinkThreads + lane;
            lds.x[a] = E[i].X;
            lds.g[a] = E[i].G;
            lds.ymax[a] = (int16_t)(E[i].YMax - row0);
            lds.left[a] = (int8_t)E[i].Left;
        }
    }
    switch (d.mode) {
#define PRK_WALK_OBJ(MM)                                                                                 \
    case MM:                                                                                             \
        if (in_lds)                                                                                      \
            walk_object<MM>(fp, od, d, E, n, base, bound, recs, srecs, pos, span_tri, err,               \
                            LLinks{&lds, E, (int)threadIdx.x, row0});                                    \
        else                                                                                             \
            walk_object<MM>(fp, od, d, E, n, base, bound, recs, srecs, pos, span_tri, err, GLinks{E});   \
        break;
        PRK_WALK_OBJ(MODE_AVX)
        PRK_WALK_OBJ(MODE_SC_GOURAUD)
        PRK_WALK_OBJ(MODE_SC_GOURAUD_TEX)
        PRK_WALK_OBJ(MODE_SC_PHONG)
        PRK_WALK_OBJ(MODE_SC_PHONG_TEX)
#undef PRK_WALK_OBJ
        default:  // (no such mode: its slots binned nowhere)
            for (uint32_t q = 0; q < bound; ++q) pos[base + q] = SpanPos{-1, 0, 0, 0u};
            break;
    }
}

// Segments of the small triangle objects (k_obj_walk's thread walk): an
// object's sorted edges split where the list runs empty -- before edge i when
// every earlier edge has expired by i's first row (YMin[i] >= their YMax) --
// and every segment walked by a thread of its own (k_obj_walk_seg), from an
// empty list as the sequential walk is there: new edges inserted in one row
// end up in their sorted order whatever expiring entries they scan past, so
// the list after that row's expiry is the same.  The segments' spans keep
// the walk's order: segment k takes the slots after segments 0..k-1's bounds
// (half their edges' active rows, as k_obj_bound's), a slot a segment leaves
// unused stays row -1.  Random scattered triangles grouped 16 at a time
// (C3b as 16-triangle objects) make ~12 segments of a few edges per object.
struct ObjSeg {
    uint32_t o;      // object
    uint32_t e0, n;  // its sorted edges [e0, e0 + n) (object-relative)
    uint32_t base, bound;  // span slots
    uint32_t pad;
};
// One thread per object: the segments' count (WRITE false; segcnt[nobj] = 0)
// or descriptors (at segoff[o]), in object order.  (Ordering them by length
// instead, so a wave's segments end together, made the walk slower.)
template <bool WRITE>
__global__ void k_obj_seg(FrameParams fp, const ObjDesc *__restrict__ objs, uint32_t nobj,
                          const uint32_t *__restrict__ escan, const uint32_t *__restrict__ total0p,
                          const int2 *__restrict__ wy, const unsigned long long *__restrict__ soff,
                          uint32_t *__restrict__ segcnt, const uint32_t *__restrict__ segoff,
                          ObjSeg *__restrict__ segs, SpanPos *__restrict__ pos) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o > nobj) return;
    if (o == nobj) {
        if (!WRITE) segcnt[o] = 0;
        return;
    }
    const ObjDesc od = objs[o];
    uint32_t k = 0;
    if (od.kind == 0 && !(od.k1off & kObjWave)) {
        uint32_t e0, n;
        obj_range(od, escan, *total0p, e0, n);
        const int2 *Y = wy + e0;
        const DrawRec &d = fp.draws[od.draw];
        const int32_t lo = draw_row_lo(fp, d), hi = draw_row_hi(fp);
        uint32_t at = (uint32_t)soff[o], rows = 0, first = 0;
        int32_t runmax = INT32_MIN;
        for (uint32_t i = 0; i < n; ++i) {
            const int2 yy = Y[i];
            if (i > 0 && yy.x >= runmax) {  // the list is empty at YMin[i]: edges [first, i) are a segment
                if (WRITE) segs[segoff[o] + k] = ObjSeg{o, first, i - first, at, rows / 2, 0u};
                at += rows / 2;
                rows = 0;
                first = i;
                ++k;
            }
            runmax = max(runmax, yy.y);
            rows += (uint32_t)max(0, min(yy.y, hi) - max(yy.x, lo));
        }
        if (n) {
            if (WRITE) segs[segoff[o] + k] = ObjSeg{o, first, n - first, at, rows / 2, 0u};
            at += rows / 2;
            ++k;
        }
        // the object's slots past its segments' (each segment's bound rounds
        // its half down): row -1, as the walk marks its own unused ones
        if (WRITE)
            for (uint32_t q = at; q < (uint32_t)soff[o + 1]; ++q) pos[q] = SpanPos{-1, 0, 0, 0u};
    }
    if (!WRITE) segcnt[o] = k;
}

#ifndef PRK_SEG_LINK_CAP
#define PRK_SEG_LINK_CAP 16
#endif
constexpr int kSegLinkCap = PRK_SEG_LINK_CAP;  // edges per segment with LDS links (k_obj_walk_seg)
__global__ void __launch_bounds__(kLinkThreads) k_obj_walk_seg(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                  const ObjSeg *__restrict__ segs,
                                                  const uint32_t *__restrict__ nsegp,
                                                  const uint32_t *__restrict__ escan,
                                                  const uint32_t *__restrict__ total0p, ObjEdge *__restrict__ work,
                                                  SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                                                  SpanPos *__restrict__ pos, uint32_t *__restrict__ span_tri,
                                                  uint32_t *__restrict__ err) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= *nsegp) return;
    const ObjSeg sg = segs[q];
    const ObjDesc od = objs[sg.o];
    const DrawRec &d = fp.draws[od.draw];
    uint32_t e0, n0;
    obj_range(od, escan, *total0p, e0, n0);
    ObjEdge *E = work + e0 + sg.e0;
    const uint32_t n = sg.n;
    __shared__ LinkLdsT<kSegLinkCap> lds;
    bool in_lds = n > 0 && n <= (uint32_t)kSegLinkCap;
    const int32_t row0 = n ? E[0].YMin : 0;
    if (in_lds) {
        int32_t hi = row0;
        for (uint32_t i = 0; i < n; ++i) hi = max(hi, E[i].YMax);
        in_lds = hi - row0 <= 32767;
    }
    if (in_lds) {
        const int lane = (int)threadIdx.x;
        for (uint32_t i = 0; i < n; ++i) {
            const int a = (int)i * kLinkThreads + lane;
            lds.x[a] = E[i].X;
            lds.g[a] = E[i].G;
            lds.ymax[a] = (int16_t)(E[i].YMax - row0);
            lds.left[a] = (int8_t)E[i].Left;
        }
    }
    switch (d.mode) {
#define PRK_WALK_SEG(MM)                                                                                     \
    case MM:                                                                                                 \
        if (in_lds)                                                                                          \
            walk_object<MM>(fp, od, d, E, n, sg.base, sg.bound, recs, srecs, pos, span_tri, err,             \
                            LLinksT<kSegLinkCap>{&lds, E, (int)threadIdx.x, row0});                          \
        else                                                                                                 \
            walk_object<MM>(fp, od, d, E, n, sg.base, sg.bound, recs, srecs, pos, span_tri, err, GLinks{E}); \
        break;
        PRK_WALK_SEG(MODE_AVX)
        PRK_WALK_SEG(MODE_SC_GOURAUD)
        PRK_WALK_SEG(MODE_SC_GOURAUD_TEX)
        PRK_WALK_SEG(MODE_SC_PHONG)
        PRK_WALK_SEG(MODE_SC_PHONG_TEX)
#undef PRK_WALK_SEG
        default:
            for (uint32_t q = 0; q < sg.bound; ++q) pos[sg.base + q] = SpanPos{-1, 0, 0, 0u};
            break;
    }
}

// ---------------------------------------------------------------------------
// The AET walk of one large object by one wave.  The list is an array in
// list order (position p = the p-th edge from ListHead) holding, beside each
// edge index, the fields the list operations read (X, Gradient, Left, YMax);
// the edges themselves stay in the working copy.  It lives in LDS when the
// object's most simultaneously listed edges (k_obj_maxact) fit `lcap`, and
// in device memory (a slice of a pool sized by the object's edge count)
// beyond that: the list has no length limit, as the
// reference's pointer list has none.  Per row, exactly the reference's
// operations (P3 included), as array operations:
//   insertion (3654-3713)  each new edge goes before the first entry it sorts
//                          before (by X, Gradient, Left), else to the tail —
//                          see insert_batch for doing a row's insertions at
//                          once; one or two (or any with a NaN key) one at a
//                          time, by a ballot over the list and a shift;
//   expiry (3715-3749)     entries with YMax <= Row leave, order kept (a
//                          ballot compaction);
//   pairing (3751-3869)    entries (2k, 2k+1) pair: span, then both edges
//                          step; then every pair swaps if Cur.X > Next.X
//                          (3831-3841), then every boundary (2k-1, 2k) swaps
//                          if PrevNext.X > Cur.X (3843-3853).  Pair k's second
//                          swap reads entry 2k-1 as pair k-1's first swap left
//                          it and entry 2k as its own first swap left it, and
//                          pairs touch disjoint entries, so the reference's
//                          left-to-right sequence equals the two parallel
//                          passes.  An odd last entry neither pairs nor steps.
// ---------------------------------------------------------------------------
constexpr int kWaveListArrays = 9;   // int32 arrays of cap + 2 entries each
constexpr uint32_t kSlotCapLds = 1022;  // walk_object_block's largest LDS capacity (listed edges; 1024 threads)
struct WaveList {
    int32_t *idx;
    float *x, *g;
    int32_t *left, *ymax;
    int32_t *aux;  // prefix-max positions, then the row's gap histogram and its exclusive scan
    int32_t *nb;   // per new edge of the row: its gap
    int32_t *bk;   // per new edge: its arrival slot in its gap, then its final position
    int32_t *bk2;  // the row's new edges grouped by gap
    __device__ __forceinline__ void carve(int32_t *base, uint32_t cap) {
        const size_t s = (size_t)cap + 2;
        idx = base;
        x = reinterpret_cast<float *>(base + s);
        g = reinterpret_cast<float *>(base + 2 * s);
        left = base + 3 * s;
        ymax = base + 4 * s;
        aux = base + 5 * s;
        nb = base + 6 * s;
        bk = base + 7 * s;
        bk2 = base + 8 * s;
        static_assert(kWaveListArrays == 9, "carve cuts kWaveListArrays arrays");
    }
};

// The wave's list writes visible to all its lanes: LDS needs no more than the
// wave's own order; a list in device memory waits for its stores
// (workgroup scope: the wave is the workgroup, one CU, one L1).
template <bool GL>
__device__ __forceinline__ void list_sync() {
    if (GL) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        wave_lds_sync();
    }
}

// Lane moves without the LDS (DPP, GFX9): row_shr:n inside each 16-lane row,
// row_bcast:15 / row_bcast:31 across rows; a lane without a source keeps
// `old`.  (__shfl* go through
// ds_bpermute: an LDS round trip each, the one-wave walks' critical path.)
template <int CTRL, int ROW = 0xf>
__device__ __forceinline__ int32_t dpp_i(int32_t old, int32_t v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW, 0xf, false);
}
template <int CTRL, int ROW = 0xf>
__device__ __forceinline__ float dpp_f(float old, float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROW, 0xf, false));
}
constexpr int kDppShr1 = 0x111, kDppShr2 = 0x112, kDppShr4 = 0x114, kDppShr8 = 0x118;
constexpr int kDppBcast15 = 0x142, kDppBcast31 = 0x143;
__device__ __forceinline__ int32_t wave_incl_sum_i32(int32_t v) {
    v += dpp_i<kDppShr1>(0, v);
    v += dpp_i<kDppShr2>(0, v);
    v += dpp_i<kDppShr4>(0, v);
    v += dpp_i<kDppShr8>(0, v);
    v += dpp_i<kDppBcast15, 0xa>(0, v);
    v += dpp_i<kDppBcast31, 0xc>(0, v);
    return v;
}
__device__ __forceinline__ int32_t wave_incl_max_i32(int32_t v) {
    v = max(v, dpp_i<kDppShr1>(INT32_MIN, v));
    v = max(v, dpp_i<kDppShr2>(INT32_MIN, v));
    v = max(v, dpp_i<kDppShr4>(INT32_MIN, v));
    v = max(v, dpp_i<kDppShr8>(INT32_MIN, v));
    v = max(v, dpp_i<kDppBcast15, 0xa>(INT32_MIN, v));
    v = max(v, dpp_i<kDppBcast31, 0xc>(INT32_MIN, v));
    return v;
}
__device__ __forceinline__ int32_t readlane_i(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int wave_max_i32(int v) { return readlane_i(wave_incl_max_i32(v), 63); }
__device__ __forceinline__ int32_t lane_rank(unsigned long long bal) {
    return (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

// The insertion order as a key.  "Cur sorts before E" (3663-3667) is
// key(E) > key(Cur) for keys compared (X, Gradient, Left) lexicographically
// with float compares, once NaNs are mapped out: an entry with a NaN X never
// compares greater than a new edge (lowest key), one with a NaN Gradient only
// by X (lowest Gradient and Left).  (New edges with a NaN in their key take
// the one-at-a-time insertion.)  +0 and -0 compare equal, as in the reference.
struct LKey {
    float x, g;
    int32_t l;
};
__device__ __forceinline__ LKey entry_key(float x, float g, int32_t l) {
    if (x != x) return LKey{-INFINITY, -INFINITY, INT32_MIN};
    if (g != g) return LKey{x, -INFINITY, INT32_MIN};
    return LKey{x, g, l};
}
__device__ __forceinline__ bool key_gt(const LKey &a, const LKey &b) {
    return a.x > b.x || (a.x == b.x && (a.g > b.g || (a.g == b.g && a.l > b.l)));
}
// Inclusive prefix maximum of the lanes' keys (lane order), with the lane
// position of a maximum as payload.
template <int CTRL, int ROW = 0xf>
__device__ __forceinline__ void key_max_step(LKey &k, int32_t &p) {
    const LKey o{dpp_f<CTRL, ROW>(-INFINITY, k.x), dpp_f<CTRL, ROW>(-INFINITY, k.g), dpp_i<CTRL, ROW>(INT32_MIN, k.l)};
    const int32_t op = dpp_i<CTRL, ROW>(-1, p);
    if (key_gt(o, k)) { k = o; p = op; }
}
__device__ __forceinline__ void wave_key_prefix_max(LKey &k, int32_t &p) {
    key_max_step<kDppShr1>(k, p);
    key_max_step<kDppShr2>(k, p);
    key_max_step<kDppShr4>(k, p);
    key_max_step<kDppShr8>(k, p);
    key_max_step<kDppBcast15, 0xa>(k, p);
    key_max_step<kDppBcast31, 0xc>(k, p);
}

// One new edge E[c] inserted as the reference does (3654-3713): before the
// first entry it sorts before, else at the tail.
template <bool GL>
__device__ __forceinline__ void insert_one(const WaveList &L, int &m, float cx, float cg, int32_t cl, int32_t cy,
                                           int32_t c) {
    const int lane = threadIdx.x & 63;
    int p = m;
    for (int c0 = 0; c0 < m; c0 += 64) {
        const int q = c0 + lane;
        bool b = false;
        if (q < m) {
            const float x = L.x[q], g = L.g[q];
            b = cx < x || (cx == x && (cg < g || (cg == g && cl < L.left[q])));
        }
        const unsigned long long bal = __ballot(b);
        if (bal) {
            p = c0 + (int)__builtin_ctzll(bal);
            break;
        }
    }
    for (int top = m; top > p; top -= 64) {  // entries [p, m) move up one, top chunk first
        const int q = top - 1 - lane;
        int32_t vi = 0, vl = 0, vy = 0;
        float vx = 0, vg = 0;
        if (q >= p) { vi = L.idx[q]; vx = L.x[q]; vg = L.g[q]; vl = L.left[q]; vy = L.ymax[q]; }
        list_sync<GL>();
        if (q >= p) { L.idx[q + 1] = vi; L.x[q + 1] = vx; L.g[q + 1] = vg; L.left[q + 1] = vl; L.ymax[q + 1] = vy; }
        list_sync<GL>();
    }
    if (lane == 0) { L.idx[p] = c; L.x[p] = cx; L.g[p] = cg; L.left[p] = cl; L.ymax[p] = cy; }
    list_sync<GL>();
    ++m;
}

// The k new edges of a row (E[c0, c0 + k), in insertion order, no NaN key)
// inserted at once, with the result of inserting them one by one.  With
// PM(q) = the maximum key of entries [0, q], the first entry a new edge c
// sorts before is the first q with PM(q) > key(c), and inserting c there
// inserts key(c) into the non-decreasing PM sequence at that point (every
// entry before it is <= key(c), every one after > key(c)): one insertion is an
// upper-bound insertion into a sorted sequence.  So the final list is the
// stable merge of the list (its entries weighted by PM) and the new edges
// ordered by (key, insertion order): new edge c lands at
//     gap(c) + #{new edges of gap < gap(c)} + #{new edges of its gap ordered before it},
// gap(c) = the first q with PM(q) > key(c) (m: none), and entry q moves up by
// #{new edges of gap <= q}.  O(m/64 + k/64) wave steps and a binary search per
// new edge, instead of a list scan and a shift per new edge.
template <bool GL>
__device__ void insert_batch(const WaveList &L, int &m, const ObjEdge *__restrict__ E, uint32_t c0, int k,
                             float rx, float rg, int32_t rl, int32_t ry) {
    // (k <= 64: new edge t = lane's key fields arrive in registers rx, rg, rl, ry)
    const int lane = threadIdx.x & 63;
    const bool reg = k <= 64;
    // 1. aux[q] = position of a maximal key of entries [0, q]
    {
        LKey ck{-INFINITY, -INFINITY, INT32_MIN};
        int32_t cp = -1;  // carry: the running maximum (none yet)
        for (int b0 = 0; b0 < m; b0 += 64) {
            const int q = b0 + lane;
            LKey kk{-INFINITY, -INFINITY, INT32_MIN};
            int32_t kp = q;
            if (q < m) kk = entry_key(L.x[q], L.g[q], L.left[q]);
            wave_key_prefix_max(kk, kp);
            if (cp >= 0 && key_gt(ck, kk)) { kk = ck; kp = cp; }
            if (q < m) L.aux[q] = kp;
            const int last = min(63, m - 1 - b0);
            ck.x = readlane_f(kk.x, last);
            ck.g = readlane_f(kk.g, last);
            ck.l = readlane_i(kk.l, last);
            cp = readlane_i(kp, last);
        }
    }
    list_sync<GL>();
    // 2. nb[t] = gap of new edge t: a binary search over the non-decreasing PM
    for (int t = lane; t < k; t += 64) {
        const LKey kc = reg ? LKey{rx, rg, rl} : LKey{E[c0 + t].X, E[c0 + t].G, E[c0 + t].Left};
        int lo = 0, hi = m;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const int32_t pq = L.aux[mid];
            if (key_gt(entry_key(L.x[pq], L.g[pq], L.left[pq]), kc)) hi = mid;
            else lo = mid + 1;
        }
        L.nb[t] = lo;
    }
    list_sync<GL>();
    // 3. gap histogram (aux[0, m + 2)), each new edge's arrival slot in its gap
    for (int q = lane; q < m + 2; q += 64) L.aux[q] = 0;
    list_sync<GL>();
    for (int t = lane; t < k; t += 64) L.bk[t] = atomicAdd(&L.aux[L.nb[t]], 1);
    list_sync<GL>();
    // 4. exclusive scan: aux[g] = new edges of gaps < g (aux[m + 1] = k)
    {
        int32_t carry = 0;
        for (int b0 = 0; b0 < m + 2; b0 += 64) {
            const int q = b0 + lane;
            const int32_t v = q < m + 2 ? L.aux[q] : 0;
            const int32_t inc = wave_incl_sum_i32(v);
            if (q < m + 2) L.aux[q] = carry + inc - v;
            carry += readlane_i(inc, 63);
        }
    }
    list_sync<GL>();
    // 5. the new edges grouped by gap
    for (int t = lane; t < k; t += 64) L.bk2[L.aux[L.nb[t]] + L.bk[t]] = t;
    list_sync<GL>();
    // 6. final positions: gap + new edges of earlier gaps + those of its gap
    //    ordered before it (smaller key, or an equal key inserted earlier)
    for (int t = lane; t < k; t += 64) {
        const LKey kc = reg ? LKey{rx, rg, rl} : LKey{E[c0 + t].X, E[c0 + t].G, E[c0 + t].Left};
        const int gq = L.nb[t];
        const int32_t s0 = L.aux[gq], h = L.aux[gq + 1] - s0;
        int32_t r = 0;
        for (int32_t j = 0; j < h; ++j) {
            const int32_t u = L.bk2[s0 + j];
            if (u == t) continue;
            const ObjEdge &U = E[c0 + u];
            const LKey ku{U.X, U.G, U.Left};
            r += (key_gt(kc, ku) || (!key_gt(ku, kc) && u < t)) ? 1 : 0;
        }
        L.bk[t] = gq + s0 + r;
    }
    list_sync<GL>();
    // 7. entries move up by the new edges of gaps <= their position, top
    //    chunk first (an entry only moves up, into slots already read)
    for (int top = m; top > 0; top -= 64) {
        const int q = top - 1 - lane;
        int32_t vi = 0, vl = 0, vy = 0, to = 0;
        float vx = 0, vg = 0;
        if (q >= 0) {
            to = q + L.aux[q + 1];
            vi = L.idx[q]; vx = L.x[q]; vg = L.g[q]; vl = L.left[q]; vy = L.ymax[q];
        }
        list_sync<GL>();
        if (q >= 0 && to != q) { L.idx[to] = vi; L.x[to] = vx; L.g[to] = vg; L.left[to] = vl; L.ymax[to] = vy; }
        list_sync<GL>();
    }
    // 8. the new edges into the free slots
    for (int t = lane; t < k; t += 64) {
        const int32_t at = L.bk[t];
        if (reg) {
            L.idx[at] = (int32_t)(c0 + t); L.x[at] = rx; L.g[at] = rg; L.left[at] = rl; L.ymax[at] = ry;
        } else {
            const ObjEdge &C = E[c0 + t];
            L.idx[at] = (int32_t)(c0 + t); L.x[at] = C.X; L.g[at] = C.G; L.left[at] = C.Left; L.ymax[at] = C.YMax;
        }
    }
    list_sync<GL>();
    m += k;
}

// Emits the wave's spans of one pairing chunk at base + emitted (in list
// order); a span past the object's bound sets err (the bound is the object's
// active edge rows / 2, which no walk exceeds).
template <int M, bool GL>
__device__ void walk_object_wave(const FrameParams &fp, const ObjDesc &od, const DrawRec &d,
                                 ObjEdge *__restrict__ E, uint32_t n, uint32_t base, uint32_t bound,
                                 const WaveList &L, SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                                 SpanPos *__restrict__ pos, uint32_t *__restrict__ span_tri,
                                 uint32_t *__restrict__ err) {
    constexpr bool kScalar = M != MODE_AVX;
    const int lane = threadIdx.x & 63;
    const bool st = (d.flags & DRAW_ST) != 0;
    if (n == 0) return;
    int32_t mr = INT32_MIN;
    for (uint32_t i = lane; i < n; i += 64) mr = max(mr, E[i].YMax);
    const int32_t MaxRow = wave_max_i32(mr);
    const int32_t FirstRow = E[0].YMin;
    const int32_t MaxY = min(min(MaxRow, fp.H), fp.row1);
    const int32_t RowLo = kScalar ? fp.row0 - 1 : fp.row0;
    uint32_t emitted = 0;
    int m = 0;         // list length (wave-uniform)
    uint32_t ins = 0;  // next sorted edge to insert
    for (int32_t Row = FirstRow; Row < MaxY; ++Row) {
        // The row's new edges E[ins, ins + k): YMin == Row, contiguous in the
        // MergeSort order (entries below Row: none past the first row).
        // One load per 64 edges: lane t of the first chunk keeps new edge
        // ins + t's key fields for the insertion.
        int k = 0;
        bool nan = false;
        float rx = 0.0f, rg = 0.0f;
        int32_t rl = 0, ry = 0;
        for (;;) {
            const uint32_t i = ins + (uint32_t)k + (uint32_t)lane;
            int32_t y = INT32_MAX;
            float x = 0.0f, g = 0.0f;
            int32_t l = 0, ym = 0;
            if (i < n) {
                const ObjEdge &C = E[i];
                y = C.YMin; x = C.X; g = C.G; l = C.Left; ym = C.YMax;
            }
            const unsigned long long lt = __ballot(y < Row);
            if (lt) {  // (never past the first row of a sorted list: entries below the row are skipped)
                ins += (uint32_t)__popcll(lt);
                continue;
            }
            const bool eq = y == Row;
            const unsigned long long b = __ballot(eq);
            if (k == 0) { rx = x; rg = g; rl = l; ry = ym; }
            nan |= eq && (x != x || g != g);
            k += __popcll(b);
            if (b != ~0ull) break;
        }
        if (k > 0) {
            if (k <= 2 || __any(nan)) {  // insertion 3654-3713, one edge at a time in sorted order
                for (int t = 0; t < k; ++t) {
                    if (t < 64) {
                        insert_one<GL>(L, m, __shfl(rx, t), __shfl(rg, t), __shfl(rl, t), __shfl(ry, t),
                                       (int32_t)(ins + t));
                    } else {
                        const ObjEdge &C = E[ins + t];
                        insert_one<GL>(L, m, C.X, C.G, C.Left, C.YMax, (int32_t)(ins + t));
                    }
                }
            } else {
                insert_batch<GL>(L, m, E, ins, k, rx, rg, rl, ry);
            }
            ins += (uint32_t)k;
        }
        {  // expiry 3715-3749: keep entries with YMax > Row, in order
            int out = 0;
            for (int c0 = 0; c0 < m; c0 += 64) {
                const int q = c0 + lane;
                const bool keep = q < m && !(L.ymax[q] <= Row);
                int32_t vi = 0, vl = 0, vy = 0;
                float vx = 0, vg = 0;
                if (keep) { vi = L.idx[q]; vx = L.x[q]; vg = L.g[q]; vl = L.left[q]; vy = L.ymax[q]; }
                const unsigned long long bal = __ballot(keep);
                const int at = out + lane_rank(bal);
                list_sync<GL>();
                if (keep) { L.idx[at] = vi; L.x[at] = vx; L.g[at] = vg; L.left[at] = vl; L.ymax[at] = vy; }
                list_sync<GL>();
                out += __popcll(bal);
            }
            m = out;
        }
        if (m == 0) {  // nothing happens on the rows before the next insertion: go there
            if (ins >= n) break;
            Row = max(Row, E[ins].YMin - 1);
            continue;
        }
        const int P = m / 2;  // pairing 3751-3869
        for (int k0 = 0; k0 < P; k0 += 64) {
            const int kk = k0 + lane;
            const bool valid = kk < P;
            bool em = false;
            int32_t ia = 0, ib = 0;
            SpanPos sp;
            SpanRecG rec;
            ScSpanRecG srec;
            if (valid) {
                ia = L.idx[2 * kk];
                ib = L.idx[2 * kk + 1];
            }
            ObjEdge a = E[ia], b = E[ib];  // (edge 0 for lanes past the pairs: unused)
            if (valid) {
                if (Row >= RowLo) {
                    if constexpr (kScalar) em = obj_span_scalar<M>(fp, a, b, Row, d.tex, srec, sp);
                    else em = obj_span(fp, a, b, Row, d.tex, st, rec, sp);
                }
            }
            const unsigned long long bal = __ballot(em);
            if (em) {
                const uint32_t j = emitted + (uint32_t)lane_rank(bal);
                if (j < bound) {
                    const uint32_t at = base + j;
                    if constexpr (kScalar) {
                        SpanRecG mark;
                        mark.q0 = make_float4(__uint_as_float(kScalarSpan), 0.0f, 0.0f, 0.0f);
                        mark.q1 = mark.q2 = mark.q3 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                        recs[at] = mark;
                        srecs[at] = srec;
                    } else {
                        recs[at] = rec;
                    }
                    pos[at] = sp;
                    span_tri[at] = od.g0;
                } else {
                    atomicOr(err, 2u);  // (never: the bound holds every span)
                }
            }
            emitted += (uint32_t)__popcll(bal);
            if (valid) {  // 3811-3829
                obj_step<M>(a);
                obj_step<M>(b);
                E[ia] = a;
                E[ib] = b;
                L.x[2 * kk] = a.X;
                L.x[2 * kk + 1] = b.X;
            }
        }
        list_sync<GL>();
        for (int pass_sw = 0; pass_sw < 2; ++pass_sw) {  // 3831-3841, then 3843-3853
            for (int k0 = pass_sw; k0 < P; k0 += 64) {
                const int kk = k0 + lane;
                const int q = pass_sw == 0 ? 2 * kk : 2 * kk - 1;  // swap entries q, q + 1
                bool sw = false;
                int32_t i0 = 0, i1 = 0, l0 = 0, l1 = 0, y0 = 0, y1 = 0;
                float x0 = 0, x1 = 0, g0 = 0, g1 = 0;
                if (kk < P) {
                    x0 = L.x[q];
                    x1 = L.x[q + 1];
                    sw = x0 > x1;
                    if (sw) {
                        i0 = L.idx[q]; i1 = L.idx[q + 1]; g0 = L.g[q]; g1 = L.g[q + 1];
                        l0 = L.left[q]; l1 = L.left[q + 1]; y0 = L.ymax[q]; y1 = L.ymax[q + 1];
                    }
                }
                list_sync<GL>();
                if (sw) {
                    L.idx[q] = i1; L.idx[q + 1] = i0; L.x[q] = x1; L.x[q + 1] = x0; L.g[q] = g1; L.g[q + 1] = g0;
                    L.left[q] = l1; L.left[q + 1] = l0; L.ymax[q] = y1; L.ymax[q + 1] = y0;
                }
                list_sync<GL>();
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The same walk by a whole workgroup, everything in LDS (objects whose most
// active edges fit the launch's capacity C <= 1022): the listed edges'
// mutable state in C slots (a free-slot stack), and the list as an array of
// slot numbers only — its operations move one int per entry and read the
// keys (X, Gradient, Left, YMax) from the slots.  The workgroup has NT >= C + 2
// threads, so every list operation is one step: thread q holds entry q, the
// scans and searches are workgroup scans (a DPP wave scan plus the waves'
// totals through LDS).  A lone wave walking a long list in 64-entry chunks
// ran each row's chain of dependent steps chunk after chunk (C2 as one
// object: ~80 k clocks a row); here a row is ~20 barriers.  A row touches
// device memory only for the sorted edges it inserts (read ahead NT at a
// time, one per thread) and the pairs it writes.  Pairing: thread k holds
// pair k, does its first swap (3831-3841) itself and its second (3843-3853)
// against pair k-1's second entry through LDS.
// ---------------------------------------------------------------------------
constexpr int kSlotListArrays = 5;  // int arrays of cap + 2: idx (slots), aux, nb, bk, bk2
constexpr uint32_t kSlotMaxThreads = 1024;
__host__ __device__ constexpr uint32_t slot_threads(uint32_t cap) {  // NT: >= cap + 2, a multiple of 64
    return ((cap + 2 + 63) / 64) * 64 > kSlotMaxThreads ? kSlotMaxThreads : ((cap + 2 + 63) / 64) * 64;
}
struct SlotLds {
    int32_t *idx;  // the list: slot of each entry, in list order
    int32_t *aux, *nb, *bk, *bk2;  // insertion / pairing scratch
    float *nkx, *nkg;              // the batch's new edges: keys (x, g, l) and slots, NT each
    int32_t *nkl, *nks;
    int32_t *fs;   // free slots: fs[0, top)
    ObjEdge *st;   // edge state per slot
    __device__ __forceinline__ void carve(int32_t *base, uint32_t cap, uint32_t nt) {
        const size_t s = (size_t)cap + 2;
        idx = base;
        aux = base + s;
        nb = base + 2 * s;
        bk = base + 3 * s;
        bk2 = base + 4 * s;
        int32_t *k = base + kSlotListArrays * s;
        nkx = reinterpret_cast<float *>(k);
        nkg = reinterpret_cast<float *>(k + nt);
        nkl = k + 2 * nt;
        nks = k + 3 * nt;
        fs = k + 4 * nt;
        const size_t off = ((size_t)kSlotListArrays * s + 4 * (size_t)nt + cap) * 4;
        st = reinterpret_cast<ObjEdge *>(reinterpret_cast<char *>(base) + ((off + 15) & ~(size_t)15));
    }
    __device__ __forceinline__ LKey key(int32_t sl) const {
        return entry_key(st[sl].X, st[sl].G, st[sl].Left);
    }
};
__host__ __device__ constexpr size_t slot_lds_bytes(uint32_t cap) {
    return ((((size_t)kSlotListArrays * (cap + 2) + 4 * (size_t)slot_threads(cap) + cap) * 4 + 15) & ~(size_t)15) +
           (size_t)cap * sizeof(ObjEdge);
}

// Workgroup reductions and scans over thread order (R: the waves' partials;
// every caller reaches them with the whole workgroup).
struct BlockRed {
    int32_t a[16], b[16], c[16];
    float x[16], g[16];
};
// A workgroup barrier; LO: ordering LDS only (no wait for the workgroup's
// outstanding device-memory accesses -- for walks whose threads share only
// LDS, with device-memory stores that nobody in the workgroup reads back).
template <bool LO = false>
__device__ __forceinline__ void blk_sync() {
    if (LO) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    } else {
        __syncthreads();
    }
}
template <bool LO = false>
__device__ __forceinline__ int32_t blk_excl_sum(BlockRed &R, int32_t v, int32_t &tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int32_t inc = wave_incl_sum_i32(v);
    if (lane == 63) R.a[w] = inc;
    blk_sync<LO>();
    int32_t before = 0, t = 0;
    for (int i = 0; i < nw; ++i) {
        const int32_t x = R.a[i];
        before += i < w ? x : 0;
        t += x;
    }
    blk_sync<LO>();
    tot = t;
    return before + inc - v;
}
// Two exclusive scans at once (one barrier pair).
template <bool LO = false>
__device__ __forceinline__ void blk_excl_sum2(BlockRed &R, int32_t v1, int32_t v2, int32_t &e1, int32_t &e2,
                                              int32_t &t1, int32_t &t2) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int32_t i1 = wave_incl_sum_i32(v1), i2 = wave_incl_sum_i32(v2);
    if (lane == 63) { R.a[w] = i1; R.b[w] = i2; }
    blk_sync<LO>();
    int32_t b1 = 0, b2 = 0, s1 = 0, s2 = 0;
    for (int i = 0; i < nw; ++i) {
        const int32_t x = R.a[i], y = R.b[i];
        b1 += i < w ? x : 0;
        b2 += i < w ? y : 0;
        s1 += x;
        s2 += y;
    }
    blk_sync<LO>();
    e1 = b1 + i1 - v1;
    e2 = b2 + i2 - v2;
    t1 = s1;
    t2 = s2;
}
// Three sums.
template <bool LO = false>
__device__ __forceinline__ void blk_sum3(BlockRed &R, int32_t v1, int32_t v2, int32_t v3, int32_t &t1, int32_t &t2,
                                         int32_t &t3) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int32_t s1 = readlane_i(wave_incl_sum_i32(v1), 63), s2 = readlane_i(wave_incl_sum_i32(v2), 63),
                  s3 = readlane_i(wave_incl_sum_i32(v3), 63);
    if ((threadIdx.x & 63) == 0) { R.a[w] = s1; R.b[w] = s2; R.c[w] = s3; }
    blk_sync<LO>();
    t1 = t2 = t3 = 0;
    for (int i = 0; i < nw; ++i) { t1 += R.a[i]; t2 += R.b[i]; t3 += R.c[i]; }
    blk_sync<LO>();
}
template <bool LO = false>
__device__ __forceinline__ int32_t blk_max(BlockRed &R, int32_t v) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int32_t m = wave_max_i32(v);
    if ((threadIdx.x & 63) == 0) R.a[w] = m;
    blk_sync<LO>();
    int32_t r = INT32_MIN;
    for (int i = 0; i < nw; ++i) r = max(r, R.a[i]);
    blk_sync<LO>();
    return r;
}
// The first thread with b (INT32_MAX: none).
__device__ __forceinline__ int32_t blk_first(BlockRed &R, bool b) {
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const unsigned long long bal = __ballot(b);
    if ((threadIdx.x & 63) == 0) R.a[w] = bal ? w * 64 + (int)__builtin_ctzll(bal) : INT32_MAX;
    __syncthreads();
    int32_t r = INT32_MAX;
    for (int i = 0; i < nw; ++i) r = min(r, R.a[i]);
    __syncthreads();
    return r;
}
// Inclusive prefix maximum of the threads' keys.
template <bool LO = false>
__device__ __forceinline__ void blk_key_prefix_max(BlockRed &R, LKey &k) {
    const int w = threadIdx.x >> 6;
    int32_t p = 0;
    wave_key_prefix_max(k, p);
    if ((threadIdx.x & 63) == 63) { R.x[w] = k.x; R.g[w] = k.g; R.a[w] = k.l; }
    blk_sync<LO>();
    LKey c{-INFINITY, -INFINITY, INT32_MIN};
    for (int i = 0; i < w; ++i) {
        const LKey o{R.x[i], R.g[i], R.a[i]};
        if (key_gt(o, c)) c = o;
    }
    if (key_gt(c, k)) k = c;
    blk_sync<LO>();
}

// One new edge (key c, slot sl) before the first entry it sorts before
// (3663-3667), else at the tail (thread q: entry q).
__device__ void insert_one_b(const SlotLds &S, BlockRed &R, int &m, const LKey &c, int32_t sl) {
    const int q = threadIdx.x;
    bool b = false;
    if (q < m) {
        const int32_t e = S.idx[q];
        const float x = S.st[e].X, g = S.st[e].G;
        b = c.x < x || (c.x == x && (c.g < g || (c.g == g && c.l < S.st[e].Left)));
    }
    const int p = min(blk_first(R, b), m);
    const bool mv = q >= p && q < m;  // entries [p, m) move up one
    const int32_t v = mv ? S.idx[q] : 0;
    __syncthreads();
    if (mv) S.idx[q + 1] = v;
    if (q == 0) S.idx[p] = sl;
    __syncthreads();
    ++m;
}

// The k new edges of the batch (S.nk*[0, k), in insertion order, no NaN key)
// inserted at once with the result of inserting them one by one (see
// insert_batch: each new edge lands at its gap + the new edges of earlier
// gaps + those of its gap ordered before it; entry q moves up by the new
// edges of gaps <= q).  Thread q: entry q and new edge q.
__device__ void insert_batch_b(const SlotLds &S, BlockRed &R, int &m, int k) {
    const int q = threadIdx.x;
    const bool mine = q < k;
    // 1. PM(q) = the maximum key of entries [0, q], its (x, g, l) in (nb, bk, aux)
    float *pmx = reinterpret_cast<float *>(S.nb), *pmg = reinterpret_cast<float *>(S.bk);
    {
        LKey kk{-INFINITY, -INFINITY, INT32_MIN};
        if (q < m) kk = S.key(S.idx[q]);
        blk_key_prefix_max(R, kk);
        if (q < m) { pmx[q] = kk.x; pmg[q] = kk.g; S.aux[q] = kk.l; }
    }
    __syncthreads();
    // 2. the gap of new edge q: binary search over the non-decreasing PM
    LKey kc{0.0f, 0.0f, 0};
    int32_t rs = 0, gq = 0;
    if (mine) {
        kc = LKey{S.nkx[q], S.nkg[q], S.nkl[q]};
        rs = S.nks[q];
        int lo = 0, hi = m;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (key_gt(LKey{pmx[mid], pmg[mid], S.aux[mid]}, kc)) hi = mid;
            else lo = mid + 1;
        }
        gq = lo;
    }
    __syncthreads();
    // 3. gap histogram (aux[0, m + 2)), each new edge's arrival slot in its gap
    if (q < m + 2) S.aux[q] = 0;
    __syncthreads();
    int32_t arr = 0;
    if (mine) arr = atomicAdd(&S.aux[gq], 1);
    __syncthreads();
    {  // 4. exclusive scan: aux[g] = new edges of gaps < g
        const int32_t v = q < m + 2 ? S.aux[q] : 0;
        int32_t tot;
        const int32_t ex = blk_excl_sum(R, v, tot);
        if (q < m + 2) S.aux[q] = ex;
    }
    __syncthreads();
    int32_t s0 = 0, h = 0;
    if (mine) {  // 5. the new edges grouped by gap
        s0 = S.aux[gq];
        h = S.aux[gq + 1] - s0;
        S.bk2[s0 + arr] = q;
    }
    __syncthreads();
    // 6. final positions: gap + new edges of earlier gaps + those of its gap
    //    ordered before it (smaller key, or an equal key inserted earlier)
    //    (a per-thread loop: no barrier inside)
    int32_t r = 0;
    for (int32_t j = 0; j < h; ++j) {
        const int32_t u = S.bk2[s0 + j];
        if (u != q) {
            const LKey ku{S.nkx[u], S.nkg[u], S.nkl[u]};
            r += (key_gt(kc, ku) || (!key_gt(ku, kc) && u < q)) ? 1 : 0;
        }
    }
    // 7. entries move up by the new edges of gaps <= their position; 8. the new edges
    int32_t v = 0, to = 0;
    if (q < m) {
        to = q + S.aux[q + 1];
        v = S.idx[q];
    }
    __syncthreads();
    if (q < m) S.idx[to] = v;
    if (mine) S.idx[gq + s0 + r] = rs;
    __syncthreads();
    m += k;
}

// A pair of the slot walk, before its span setup: both edges' values at the
// row (the fields obj_span / obj_span_scalar read), written by the walk; its
// SpanPos holds the row, the draw (in minx) and SPAN_RAW until k_span_finish
// turns it into the span's record (or row -1 when it covers nothing).  The
// setup's ~300 instructions per span leave the walk's row-serial path.
constexpr uint32_t SPAN_RAW = 0x40000000u;
struct PairRaw {
    float4 l0, l1, l2, r0, r1, r2;  // X Z W U | V N0 N1 N2 | C0 C1 C2 C3, left then right edge
};
static_assert(sizeof(PairRaw) == 96, "six dwordx4");
__device__ __forceinline__ void pair_raw_out(const ObjEdge &a, const ObjEdge &b, PairRaw &o) {
    o.l0 = make_float4(a.X, a.Z, a.W, a.U);
    o.l1 = make_float4(a.V, a.N0, a.N1, a.N2);
    o.l2 = make_float4(a.C0, a.C1, a.C2, a.C3);
    o.r0 = make_float4(b.X, b.Z, b.W, b.U);
    o.r1 = make_float4(b.V, b.N0, b.N1, b.N2);
    o.r2 = make_float4(b.C0, b.C1, b.C2, b.C3);
}
__device__ __forceinline__ ObjEdge pair_raw_in(const float4 &q0, const float4 &q1, const float4 &q2) {
    ObjEdge e = ObjEdge{};
    e.X = q0.x; e.Z = q0.y; e.W = q0.z; e.U = q0.w;
    e.V = q1.x; e.N0 = q1.y; e.N1 = q1.z; e.N2 = q1.w;
    e.C0 = q2.x; e.C1 = q2.y; e.C2 = q2.z; e.C3 = q2.w;
    return e;
}
__global__ void k_span_finish(FrameParams fp, const PairRaw *__restrict__ raw, uint32_t nslot,
                              SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                              SpanPos *__restrict__ pos) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslot) return;
    SpanPos p = pos[s];
    if (p.flags != SPAN_RAW) return;  // (unused slots: all ones)
    const PairRaw r = raw[s];
    const ObjEdge L = pair_raw_in(r.l0, r.l1, r.l2), R = pair_raw_in(r.r0, r.r1, r.r2);
    const DrawRec &d = fp.draws[p.minx];
    const int32_t Row = p.row;
    bool em = false;
    switch (d.mode) {
        case MODE_AVX: {
            SpanRecG rec;
            em = obj_span(fp, L, R, Row, d.tex, (d.flags & DRAW_ST) != 0, rec, p);
            if (em) recs[s] = rec;
            break;
        }
#define PRK_FINISH_SC(MM)                                                          \
    case MM: {                                                                     \
        ScSpanRecG srec;                                                           \
        em = obj_span_scalar<MM>(fp, L, R, Row, d.tex, srec, p);                   \
        if (em) {                                                                  \
            SpanRecG mark;                                                         \
            mark.q0 = make_float4(__uint_as_float(kScalarSpan), 0.0f, 0.0f, 0.0f); \
            mark.q1 = mark.q2 = mark.q3 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);     \
            recs[s] = mark;                                                        \
            srecs[s] = srec;                                                       \
        }                                                                          \
        break;                                                                     \
    }
        PRK_FINISH_SC(MODE_SC_GOURAUD)
        PRK_FINISH_SC(MODE_SC_GOURAUD_TEX)
        PRK_FINISH_SC(MODE_SC_PHONG)
        PRK_FINISH_SC(MODE_SC_PHONG_TEX)
#undef PRK_FINISH_SC
        default: break;
    }
    if (!em) p = SpanPos{-1, 0, 0, 0u};  // covers nothing: binned nowhere
    pos[s] = p;
}

// Read-ahead window of sorted edges as seven dwordx4 (ObjEdge's layout: X, G
// in q0.xy, YMin, YMax, Left in q4.xyz), named registers (an ObjEdge copy in
// a loop-carried variable went to scratch).
#define PRK_WIN(w) float4 w##0, w##1, w##2, w##3, w##4, w##5, w##6
#define PRK_WIN_LOAD(w, E, i, n)                                                      \
    do {                                                                              \
        const float4 *s_ = reinterpret_cast<const float4 *>((E) + min((i), (n) - 1)); \
        w##0 = s_[0]; w##1 = s_[1]; w##2 = s_[2]; w##3 = s_[3];                       \
        w##4 = s_[4]; w##5 = s_[5]; w##6 = s_[6];                                     \
        if ((i) >= (n)) (w##4).x = __int_as_float(INT32_MAX);  /* past the end */     \
    } while (0)
// The window's loads complete right where they are issued (s_waitcnt
// vmcnt(0), once per 64 edges), and the registers are redefined by an empty
// asm, so no later use waits on the load again: a window register still in
// flight across the row loop's back edge made the compiler wait for every
// outstanding access (the previous row's stores included) at the top of
// every row.
#define PRK_WIN_WAIT() __builtin_amdgcn_s_waitcnt(0x0F70)  // vmcnt(0) expcnt(7) lgkmcnt(15)
#define PRK_Q4(q) "+v"(q.x), "+v"(q.y), "+v"(q.z), "+v"(q.w)
#define PRK_WIN_LAUNDER(w)                                      \
    do {                                                        \
        asm volatile("" : PRK_Q4(w##0), PRK_Q4(w##1));          \
        asm volatile("" : PRK_Q4(w##2), PRK_Q4(w##3));          \
        asm volatile("" : PRK_Q4(w##4), PRK_Q4(w##5));          \
        asm volatile("" : PRK_Q4(w##6));                        \
    } while (0)
#define PRK_WIN_COPY(d, w) \
    do { d##0 = w##0; d##1 = w##1; d##2 = w##2; d##3 = w##3; d##4 = w##4; d##5 = w##5; d##6 = w##6; } while (0)
#define PRK_WIN_STORE(dst, w)                                                          \
    do {                                                                               \
        float4 *d_ = reinterpret_cast<float4 *>(dst);                                  \
        d_[0] = w##0; d_[1] = w##1; d_[2] = w##2; d_[3] = w##3;                        \
        d_[4] = w##4; d_[5] = w##5; d_[6] = w##6;                                      \
    } while (0)

template <int M>
__device__ void walk_object_block(const FrameParams &fp, const ObjDesc &od, const ObjEdge *__restrict__ E,
                                  uint32_t n, int32_t MaxY, uint32_t base, uint32_t bound, const SlotLds &S,
                                  BlockRed &R, uint32_t cap, PairRaw *__restrict__ raw, SpanPos *__restrict__ pos,
                                  uint32_t *__restrict__ span_tri, uint32_t *__restrict__ err) {
    constexpr bool kScalar = M != MODE_AVX;
    const int tid = threadIdx.x;
    const uint32_t NT = blockDim.x;
    const int32_t RowLo = kScalar ? fp.row0 - 1 : fp.row0;
    unsigned long long wp[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const unsigned long long wt0 = PRK_WT();
    for (uint32_t q = tid; q < cap; q += NT) S.fs[q] = (int32_t)q;
    int top = (int)cap;  // free slots (the same value in every thread, as every uniform below)
    // read-ahead window: thread t holds sorted edge wb + t
    uint32_t wb = 0;
    PRK_WIN(wa);
    PRK_WIN_LOAD(wa, E, (uint32_t)tid, n);
    PRK_WIN_WAIT();
    PRK_WIN_LAUNDER(wa);
    uint32_t emitted = 0;
    int m = 0;
    uint32_t ins = 0;
    __syncthreads();
    for (int32_t Row = E[0].YMin; Row < MaxY; ++Row) {
        unsigned long long t0 = PRK_WT();
        if (PRK_WPROF) wp[3] += 1;
        // insertion (3654-3713): the edges with YMin == Row, in sorted order,
        // a window at a time (batches in order == one at a time)
        for (;;) {
            if (ins == wb + NT) {
                wb += NT;
                PRK_WIN_LOAD(wa, E, wb + tid, n);
                PRK_WIN_WAIT();
                PRK_WIN_LAUNDER(wa);
            }
            const float wx = wa0.x, wg = wa0.y;
            const int32_t wymin = __float_as_int(wa4.x), wl = __float_as_int(wa4.z);
            const int rel = tid - (int)(ins - wb);
            const bool eqr = rel >= 0 && wymin == Row;
            int32_t lt, k, nanc;
            blk_sum3(R, (rel >= 0 && wymin < Row) ? 1 : 0, eqr ? 1 : 0, (eqr && (wx != wx || wg != wg)) ? 1 : 0, lt,
                     k, nanc);
            if (lt) {  // (never past the first row: entries below the row are skipped)
                ins += (uint32_t)lt;
                continue;
            }
            if (k == 0) break;
            if (rel >= 0 && rel < k) {  // the row's new edges take slots; their keys go to nk*
                const int32_t slot = S.fs[top - 1 - rel];
                PRK_WIN_STORE(&S.st[slot], wa);
                S.nkx[rel] = wx;
                S.nkg[rel] = wg;
                S.nkl[rel] = wl;
                S.nks[rel] = slot;
            }
            top -= k;
            __syncthreads();
            if (PRK_WPROF) {
                wp[8] += (unsigned long long)k;
                wp[(k <= 2 || nanc) ? 6 : 4] += 1;
            }
            if (k <= 2 || nanc) {  // one at a time (any NaN key), 3654-3713
                for (int t = 0; t < k; ++t)
                    insert_one_b(S, R, m, LKey{S.nkx[t], S.nkg[t], S.nkl[t]}, S.nks[t]);
            } else {
                insert_batch_b(S, R, m, k);
            }
            ins += (uint32_t)k;
            if (ins < wb + NT) break;  // the row's edges end inside the window
        }
        if (PRK_WPROF) { const unsigned long long t1 = PRK_WT(); wp[0] += t1 - t0; t0 = t1; }
        {  // expiry 3715-3749: keep entries with YMax > Row, in order; free the others' slots
            int32_t e = 0;
            bool keep = false;
            if (tid < m) {
                e = S.idx[tid];
                keep = !(S.st[e].YMax <= Row);
            }
            const bool gone = tid < m && !keep;
            int32_t kp, gp, kt, gt;
            blk_excl_sum2(R, keep ? 1 : 0, gone ? 1 : 0, kp, gp, kt, gt);
            if (keep) S.idx[kp] = e;
            if (gone) S.fs[top + gp] = e;
            m = kt;
            top += gt;
            __syncthreads();
        }
        if (PRK_WPROF) { const unsigned long long t1 = PRK_WT(); wp[1] += t1 - t0; t0 = t1; }
        if (m == 0) {  // nothing happens on the rows before the next insertion: go there
            if (ins >= n) break;
            Row = max(Row, E[ins].YMin - 1);
            continue;
        }
        const int P = m / 2;  // pairing 3751-3869: thread k holds pair k
        const bool valid = tid < P;
        const bool emit = Row >= RowLo;  // every pair of the pass's rows takes a slot (k_span_finish sets it up)
        int32_t i0 = 0, i1 = 0;
        float x0 = 0.0f, x1 = 0.0f;
        if (valid) {
            i0 = S.idx[2 * tid];
            i1 = S.idx[2 * tid + 1];
            const uint32_t j = emitted + (uint32_t)tid;
            const bool w = emit && j < bound;
            if (emit && j >= bound) atomicOr(err, 2u);  // (never: the bound holds every pair)
            const uint32_t at = base + j;
            ObjEdge a = S.st[i0];  // left edge: its values at the row, then its step (3811-3829)
            if (w) {
                raw[at].l0 = make_float4(a.X, a.Z, a.W, a.U);
                raw[at].l1 = make_float4(a.V, a.N0, a.N1, a.N2);
                raw[at].l2 = make_float4(a.C0, a.C1, a.C2, a.C3);
            }
            obj_step<M>(a);
            S.st[i0] = a;
            x0 = a.X;
            ObjEdge b = S.st[i1];  // right edge
            if (w) {
                raw[at].r0 = make_float4(b.X, b.Z, b.W, b.U);
                raw[at].r1 = make_float4(b.V, b.N0, b.N1, b.N2);
                raw[at].r2 = make_float4(b.C0, b.C1, b.C2, b.C3);
                pos[at] = SpanPos{Row, (int32_t)od.draw, 0, SPAN_RAW};
                span_tri[at] = od.g0;
            }
            obj_step<M>(b);
            S.st[i1] = b;
            x1 = b.X;
            if (x0 > x1) {  // 3831-3841
                const int32_t t = i0; i0 = i1; i1 = t;
                const float f = x0; x0 = x1; x1 = f;
            }
            // pair k's entries after its first swap, for its neighbours
            S.nb[tid] = i0;
            S.bk[tid] = __float_as_int(x0);
            S.aux[tid] = i1;
            S.bk2[tid] = __float_as_int(x1);
        }
        __syncthreads();
        if (valid) {  // 3843-3853: pair k's first entry against pair k-1's second
            const bool sw = tid >= 1 && __int_as_float(S.bk2[tid - 1]) > x0;
            const bool swn = tid + 1 < P && x1 > __int_as_float(S.bk[tid + 1]);  // pair k+1's swap takes my second
            const int32_t nf = sw ? S.aux[tid - 1] : i0, ns = swn ? S.nb[tid + 1] : i1;
            i0 = nf;
            i1 = ns;
        }
        __syncthreads();
        if (valid) {
            S.idx[2 * tid] = i0;
            S.idx[2 * tid + 1] = i1;
        }
        if (emit) emitted += (uint32_t)P;
        __syncthreads();
        if (PRK_WPROF) wp[2] += PRK_WT() - t0;
    }
    if (PRK_WPROF && tid == 0) {
        wp[7] = PRK_WT() - wt0;
        for (int k = 0; k < 14; ++k) atomicAdd(fp.prof + k, wp[k]);
    }
}

// The most entries each large object's list holds at once (thread block
// per object, a difference histogram of its listed edges over up to
// kMaxactRows rows; more rows: INT32_MAX, its list goes to device memory).
// The host reads them back with the span slot total and launches each
// object's walk with a workgroup just large enough (slot_threads).
constexpr int32_t kMaxactRows = 16000;  // (the histogram is static LDS: < 64 KiB)
// (most[nbig + b]: the rows its walk visits, MaxY - FirstRow (0 when none,
// INT32_MAX past the histogram); most[2 * nbig + b]: its list entries over
// them, the sum over its edges of their rows [YMin, min(YMax, MaxY)),
// saturated at INT32_MAX: the sizes of the parallel-rows walk, k_pr_*.)
__global__ void __launch_bounds__(kSlotMaxThreads) k_obj_maxact(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                               const uint32_t *__restrict__ big, uint32_t nbig,
                                                               const uint32_t *__restrict__ escan,
                                                               const uint32_t *__restrict__ total0p,
                                                               const ObjEdge *__restrict__ work,
                                                               int32_t *__restrict__ most, uint32_t huge_min) {
    __shared__ int32_t h[kMaxactRows + 1];
    __shared__ BlockRed R;
    __shared__ unsigned long long ents;
    const ObjDesc od = objs[big[blockIdx.x]];
    if (huge_min && od.kind == 0 && 3ull * od.tris >= huge_min) return;  // (k_maxact_huge_*)
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const ObjEdge *E = work + e0;
    const int tid = threadIdx.x, NT = blockDim.x;
    if (n == 0) {
        if (tid == 0) most[blockIdx.x] = most[nbig + blockIdx.x] = most[2 * nbig + blockIdx.x] = 0;
        return;
    }
    int32_t mr = INT32_MIN;
    for (uint32_t i = tid; i < n; i += NT) mr = max(mr, E[i].YMax);
    const int32_t MaxY = min(min(blk_max(R, mr), fp.H), fp.row1), FirstRow = E[0].YMin;
    const int64_t rows = (int64_t)MaxY - FirstRow;
    if (rows <= 0 || rows + 1 > kMaxactRows) {
        if (tid == 0) {
            most[blockIdx.x] = most[nbig + blockIdx.x] = rows <= 0 ? 0 : INT32_MAX;
            most[2 * nbig + blockIdx.x] = 0;
        }
        return;
    }
    const int Rn = (int)rows;
    for (int q = tid; q <= Rn; q += NT) h[q] = 0;
    if (tid == 0) ents = 0;
    __syncthreads();
    unsigned long long mine = 0;
    for (uint32_t i = tid; i < n; i += NT) {  // an edge is listed on rows [YMin, max(YMin, YMax)]
        const int32_t y0 = E[i].YMin, y1 = E[i].YMax;
        if (y0 >= MaxY) continue;  // never inserted
        atomicAdd(&h[y0 - FirstRow], 1);
        atomicAdd(&h[min(max(y0, y1), MaxY - 1) - FirstRow + 1], -1);
        mine += (unsigned long long)max(0, min(y1, MaxY) - y0);
    }
    if (mine) atomicAdd(&ents, mine);
    __syncthreads();
    if (tid == 0) {
        most[nbig + blockIdx.x] = Rn;
        most[2 * nbig + blockIdx.x] = (int32_t)min(ents, (unsigned long long)INT32_MAX);
    }
    int32_t carry = 0, best = 0;
    for (int b0 = 0; b0 < Rn; b0 += NT) {
        const int q = b0 + tid;
        const int32_t v = q < Rn ? h[q] : 0;
        int32_t tot;
        const int32_t ex = blk_excl_sum(R, v, tot);
        if (q < Rn) best = max(best, carry + ex + v);
        carry += tot;
    }
    best = blk_max(R, best);
    if (tid == 0) most[blockIdx.x] = best;
}

// The same sizes for one huge object (big[b]: 3 * tris >= huge_min edges),
// its edges spread over many workgroups: the difference histogram in device
// memory (hist: kMaxactRows + 2 zeroed ints; acc: 3 zeroed words -- the
// most YMax, the entries, an overflow flag), clipped at min(H, row1) instead
// of MaxY (what lands past MaxY - FirstRow is never scanned), then
// k_maxact_huge_fin scans it.
constexpr uint32_t kMaxactChunk = 8 * kSlotMaxThreads;  // edges per workgroup
__global__ void __launch_bounds__(kSlotMaxThreads) k_maxact_huge_part(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                                     const uint32_t *__restrict__ big, uint32_t b,
                                                                     const uint32_t *__restrict__ escan,
                                                                     const uint32_t *__restrict__ total0p,
                                                                     const ObjEdge *__restrict__ work,
                                                                     int32_t *__restrict__ hist,
                                                                     unsigned long long *__restrict__ acc) {
    __shared__ BlockRed R;
    __shared__ unsigned long long ents;
    const ObjDesc od = objs[big[b]];
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const uint32_t i0 = blockIdx.x * kMaxactChunk;
    if (n == 0 || i0 >= n) return;
    const ObjEdge *E = work + e0;
    const int32_t FirstRow = E[0].YMin, Hc = min(fp.H, fp.row1);
    if ((int64_t)Hc - FirstRow + 1 > kMaxactRows) {
        if (threadIdx.x == 0) atomicOr(acc + 2, 1ull);
        return;
    }
    if (threadIdx.x == 0) ents = 0;
    __syncthreads();
    int32_t mr = INT32_MIN;
    unsigned long long mine = 0;
    for (uint32_t i = i0 + threadIdx.x; i < min(n, i0 + kMaxactChunk); i += kSlotMaxThreads) {
        const int32_t y0 = E[i].YMin, y1 = E[i].YMax;
        mr = max(mr, y1);
        if (y0 >= Hc) continue;
        atomicAdd(&hist[y0 - FirstRow], 1);
        atomicAdd(&hist[min(max(y0, y1), Hc - 1) - FirstRow + 1], -1);
        mine += (unsigned long long)max(0, min(y1, Hc) - y0);
    }
    if (mine) atomicAdd(&ents, mine);
    mr = blk_max(R, mr);  // (its barriers also order the LDS sum)
    if (threadIdx.x == 0) {
        atomicMax(acc, (unsigned long long)((int64_t)mr - (int64_t)INT32_MIN));  // (biased: unsigned max)
        if (ents) atomicAdd(acc + 1, ents);
    }
}
__global__ void __launch_bounds__(kSlotMaxThreads) k_maxact_huge_fin(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                                    const uint32_t *__restrict__ big, uint32_t b,
                                                                    uint32_t nbig, const uint32_t *__restrict__ escan,
                                                                    const uint32_t *__restrict__ total0p,
                                                                    const ObjEdge *__restrict__ work,
                                                                    const int32_t *__restrict__ hist,
                                                                    const unsigned long long *__restrict__ acc,
                                                                    int32_t *__restrict__ most) {
    __shared__ BlockRed R;
    const ObjDesc od = objs[big[b]];
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const int tid = threadIdx.x, NT = blockDim.x;
    if (n == 0) {
        if (tid == 0) most[b] = most[nbig + b] = most[2 * nbig + b] = 0;
        return;
    }
    const int32_t FirstRow = work[e0].YMin;
    const int32_t MaxYMax = (int32_t)((int64_t)acc[0] + (int64_t)INT32_MIN);
    const int32_t MaxY = min(min(MaxYMax, fp.H), fp.row1);
    const int64_t rows = (int64_t)MaxY - FirstRow;
    if (rows <= 0 || rows + 1 > kMaxactRows || acc[2]) {
        if (tid == 0) {
            most[b] = most[nbig + b] = rows <= 0 ? 0 : INT32_MAX;
            most[2 * nbig + b] = 0;
        }
        return;
    }
    const int Rn = (int)rows;
    if (tid == 0) {
        most[nbig + b] = Rn;
        most[2 * nbig + b] = (int32_t)min(acc[1], (unsigned long long)INT32_MAX);
    }
    int32_t carry = 0, best = 0;
    for (int b0 = 0; b0 < Rn; b0 += NT) {
        const int q = b0 + tid;
        const int32_t v = q < Rn ? hist[q] : 0;
        int32_t tot;
        const int32_t ex = blk_excl_sum(R, v, tot);
        if (q < Rn) best = max(best, carry + ex + v);
        carry += tot;
    }
    best = blk_max(R, best);
    if (tid == 0) most[b] = best;
}

// One workgroup per large object: lcap > 0, everything in LDS
// (walk_object_block, lcap slots, slot_threads(lcap) threads); lcap == 0, the
// list in the object's pool slice pool + big_off[blockIdx.x]
// (kWaveListArrays arrays of big_cap[blockIdx.x] + 2 ints, big_cap >= its
// edge count), walked by one wave (64 threads).
template <int M>
__global__ void __launch_bounds__(kSlotMaxThreads) k_obj_walk_wave(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                      const uint32_t *__restrict__ big,
                                                      const unsigned long long *__restrict__ big_off,
                                                      const uint32_t *__restrict__ big_cap, int32_t *__restrict__ pool,
                                                      uint32_t lcap, const uint32_t *__restrict__ escan,
                                                      const uint32_t *__restrict__ total0p, ObjEdge *__restrict__ work,
                                                      const unsigned long long *__restrict__ soff,
                                                      SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                                                      PairRaw *__restrict__ raw, SpanPos *__restrict__ pos,
                                                      uint32_t *__restrict__ span_tri, uint32_t *__restrict__ err,
                                                      const uint32_t *__restrict__ prstat) {
    extern __shared__ int32_t lds_list[];
    __shared__ BlockRed R;
    const uint32_t o = big[blockIdx.x];
    if (prstat && prstat[o] == kPrDone) return;  // walked by rows (k_pr_*)
    const ObjDesc od = objs[o];
    const DrawRec &d = fp.draws[od.draw];
    const uint32_t base = (uint32_t)soff[o], bound = (uint32_t)(soff[o + 1] - soff[o]);
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    ObjEdge *E = work + e0;
    if (n == 0) return;  // (the whole workgroup)
    if (lcap == 0) {  // the list in device memory, one wave
        if (threadIdx.x >= 64) return;
        if (n > big_cap[blockIdx.x]) {  // (the host sizes every slice by the object's edges)
            if (threadIdx.x == 0) atomicOr(err, 1u);
            return;
        }
        WaveList L;
        L.carve(pool + big_off[blockIdx.x], big_cap[blockIdx.x]);
        walk_object_wave<M, true>(fp, od, d, E, n, base, bound, L, recs, srecs, pos, span_tri, err);
        return;
    }
    int32_t mr = INT32_MIN;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) mr = max(mr, E[i].YMax);
    const int32_t MaxY = min(min(blk_max(R, mr), fp.H), fp.row1);
    SlotLds S;
    S.carve(lds_list, lcap, blockDim.x);
    walk_object_block<M>(fp, od, E, n, MaxY, base, bound, S, R, lcap, raw, pos, span_tri, err);
}

// ---------------------------------------------------------------------------
// The walk of huge objects (objects whose most active edges exceed the
// workgroup walk's LDS list, up to kBigMaxM of them; C3b as ONE object holds
// ~16 k edges a row).  One workgroup of kBigThreads walks the object's rows
// in order (3615-3869) with its list in device memory: two SoA buffers of
// (X, Gradient, Left, YMax, edge index) in list order, each list operation a
// few workgroup-wide passes (entry q of a pass: thread q % kBigThreads, tile
// q / kBigThreads), every scan a DPP wave scan + the waves' totals in LDS:
//   insertion + expiry (3654-3749), one scan: a batch of new edges (<=
//     kBigThreads, MergeSort order, no NaN key) lands where inserting them one
//     at a time puts them (insert_batch's argument).  New edge c's gap is the
//     first entry whose key is greater (found through the entries' per-16
//     maxima, prefix-maxed in LDS, then those 16 entries), and
//        c lands at  #kept entries before gap(c) + #kept new edges of smaller
//                    gap + those of its gap ordered before it (key, arrival),
//        a kept entry q at  #kept entries before q + #kept new edges of gap <= q:
//     the new edges counted per gap, one scan of (keep flag, count) over the
//     entries, then each gap's few new edges rank themselves.  (A batch with
//     a NaN key goes one edge at a time; the row's last batch also drops the
//     expired entries.)
//   pairing (3751-3869), one pass: thread k steps pair k's X and its
//     neighbours' (X += Gradient, obj_step's first line), does its first swap
//     (3831-3841) and both boundary swaps (3843-3853; the neighbours' fields
//     through lane shuffles, from memory at wave edges), and writes its two
//     entries' final places.
// The walk sets up no span.  Per row it leaves the list it pairs (the edges'
// indices in list order, `ids`), the row's first slot (or "not emitted":
// rows above the band) and its unpaired odd last entry, if any (not stepped).
// k_big_replay then sets up every pair of every row at once, a thread per
// pair: both edges replayed from their FillEdgeTable state, stepped on every
// row they were listed on before this one but the unpaired ones (obj_step,
// 3811-3829), into the pair's PairRaw; k_span_finish sets the spans up as it
// does the chunked walk's.  The pairing also leaves the next row's per-16 key
// maxima in LDS, so a row's insertion reads the list once.
// ---------------------------------------------------------------------------
constexpr int kBigThreads = 1024;
constexpr int kBigWaves = kBigThreads / 64;
constexpr int kBigMaxTiles = 64;
constexpr uint32_t kBigMaxM = (uint32_t)kBigMaxTiles * kBigThreads - 2;  // list entries (and the pool stride - 2)
constexpr int kBigSamp = kBigMaxTiles * kBigThreads / 16;                // per-16 maxima
constexpr int kBigU = 8;                                                 // tiles a pass keeps in registers
constexpr int kBigListArrays = 12;  // 2 x (x, g, left, ymax, ei) + d + base, big_stride(cap) int32 each
constexpr uint32_t kBigNoEmit = 0xFFFFFFFEu;  // a row above the band: paired, no spans

// Each array of a huge object's pool slice: cap + 2 ints, rounded up to 16 B
// (the slice itself starts 16-B aligned: vector loads of 4 / 2 entries).
__host__ __device__ constexpr size_t big_stride(uint32_t cap) { return ((size_t)cap + 2 + 3) & ~(size_t)3; }
struct BigBuf {  // one list buffer, in list order
    float *x, *g;
    int32_t *left, *ymax, *ei;  // (ei: the edge's index in the object's sorted edges)
};
// A huge object's pool slice: the list buffers, d and base (kBigListArrays
// arrays of big_stride(cap) ints), a header (FirstRow, rows), per row
// (off, m, j0, unp): its list's place in ids, its length, its first slot
// (kBigNoEmit: none) and its unpaired entry (-1: none), then ids.
__host__ __device__ constexpr uint64_t big_slice_ints(uint32_t cap, uint32_t rows, uint32_t ents) {
    return ((uint64_t)kBigListArrays * big_stride(cap) + 4 + 4ull * rows + ents + 3) & ~3ull;
}
struct BigList {
    BigBuf b0, b1;
    int32_t *d;     // the batch's kept new edges per gap
    int32_t *base;  // where each gap's new edges begin
    int32_t *hdr, *ri, *ids;
    __device__ __forceinline__ void carve(int32_t *p0, uint32_t cap, uint32_t rows) {
        const size_t s = big_stride(cap);
        int32_t *p = p0;
        b0 = BigBuf{reinterpret_cast<float *>(p), reinterpret_cast<float *>(p + s), p + 2 * s, p + 3 * s, p + 4 * s};
        p = p0 + 5 * s;
        b1 = BigBuf{reinterpret_cast<float *>(p), reinterpret_cast<float *>(p + s), p + 2 * s, p + 3 * s, p + 4 * s};
        d = p0 + 10 * s;
        base = p0 + 11 * s;
        hdr = p0 + (size_t)kBigListArrays * s;
        ri = hdr + 4;
        ids = ri + 4 * (size_t)rows;
        static_assert(kBigListArrays == 12, "carve cuts kBigListArrays arrays");
    }
    // (selects, not an indexed pair: an indexed pointer array went to scratch)
    __device__ __forceinline__ BigBuf buf(int c) const {
        return BigBuf{c ? b1.x : b0.x, c ? b1.g : b0.g, c ? b1.left : b0.left, c ? b1.ymax : b0.ymax,
                      c ? b1.ei : b0.ei};
    }
};
struct BigLds {
    float sx[kBigSamp], sg[kBigSamp];  // per-16 key maxima, then their prefix maxima
    int32_t sl[kBigSamp];
    int32_t ts[kBigMaxTiles * kBigWaves], tm[kBigMaxTiles * kBigWaves];  // wave totals: keep and count sums
    float px[kBigThreads], pg[kBigThreads];  // per-thread key maxima (the sample scan)
    int32_t pl[kBigThreads];
    float nkx[kBigThreads], nkg[kBigThreads];  // the row's new edges (a window of kBigThreads)
    int32_t nkl[kBigThreads], nky[kBigThreads], nke[kBigThreads];
    int32_t collide;  // two new edges of the batch share a gap
};

// Insertion of the new edges S.nk*[c0, c0 + kb) into the list (buffer cur,
// m entries) and, when `expire`, expiry of every entry with YMax <= Row: the
// result into buffer cur ^ 1.  Returns the new length.
#define PRK_BIG_T(k, t)                                    \
    do {                                                   \
        if (PRK_WPROF) {                                   \
            const unsigned long long t_ = PRK_WT();        \
            if (wp) wp[k] += t_ - (t);                     \
            (t) = t_;                                      \
        }                                                  \
    } while (0)
__device__ __forceinline__ int big_insert_expire(const BigList &L, BigLds &S, BlockRed &R, int cur, int m, int c0, int kb,
                                                 bool expire, int32_t Row, bool samples_ready,
                                                 unsigned long long *wp = nullptr) {
    unsigned long long tw0 = PRK_WT();
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int T = (m + kBigThreads - 1) / kBigThreads;
    const BigBuf A = L.buf(cur), B = L.buf(cur ^ 1);
    const float *X = A.x, *G = A.g;
    const int32_t *LF = A.left, *YM = A.ymax, *EI = A.ei;
    int32_t gapc = 0, kr = 0;
    bool keptc = false;
    if (tid == 0) S.collide = 0;
    if (kb > 0) {
        if (tid == 0) L.d[m] = 0;
        if (m > 0) {
            // 1. the entries' keys: per-16 maxima (a 16-lane row each); d zeroed
            //    (samples_ready: big_pair left both)
            for (int t0 = 0; !samples_ready && t0 < T; t0 += kBigU) {
                float kx[kBigU], kg[kBigU];
                int32_t kl[kBigU];
#pragma unroll
                for (int u = 0; u < kBigU; ++u) {
                    const int q = (t0 + u) * kBigThreads + tid;
                    kx[u] = -INFINITY; kg[u] = -INFINITY; kl[u] = INT32_MIN;
                    if (t0 + u < T && q < m) { kx[u] = X[q]; kg[u] = G[q]; kl[u] = LF[q]; }
                }
#pragma unroll
                for (int u = 0; u < kBigU; ++u) {
                    if (t0 + u >= T) break;
                    const int q = (t0 + u) * kBigThreads + tid;
                    LKey k = q < m ? entry_key(kx[u], kg[u], kl[u]) : LKey{-INFINITY, -INFINITY, INT32_MIN};
                    int32_t p = 0;
                    key_max_step<kDppShr1>(k, p);
                    key_max_step<kDppShr2>(k, p);
                    key_max_step<kDppShr4>(k, p);
                    key_max_step<kDppShr8>(k, p);
                    if ((lane & 15) == 15 && (q >> 4) < kBigSamp) {
                        S.sx[q >> 4] = k.x; S.sg[q >> 4] = k.g; S.sl[q >> 4] = k.l;
                    }
                    if (q < m) L.d[q] = 0;
                }
            }
            __syncthreads();
            PRK_BIG_T(9, tw0);
            // 2. prefix maxima of the samples (4 a thread)
            const int ns = (m + 15) >> 4;
            LKey run{-INFINITY, -INFINITY, INT32_MIN};
            for (int j = 4 * tid; j < min(4 * tid + 4, ns); ++j) {
                const LKey s{S.sx[j], S.sg[j], S.sl[j]};
                if (key_gt(s, run)) run = s;
            }
            LKey inc = run;
            blk_key_prefix_max(R, inc);
            S.px[tid] = inc.x; S.pg[tid] = inc.g; S.pl[tid] = inc.l;
            __syncthreads();
            LKey carry = tid ? LKey{S.px[tid - 1], S.pg[tid - 1], S.pl[tid - 1]} : LKey{-INFINITY, -INFINITY, INT32_MIN};
            for (int j = 4 * tid; j < min(4 * tid + 4, ns); ++j) {
                const LKey s{S.sx[j], S.sg[j], S.sl[j]};
                if (key_gt(s, carry)) carry = s;
                S.sx[j] = carry.x; S.sg[j] = carry.g; S.sl[j] = carry.l;
            }
            __syncthreads();
            PRK_BIG_T(10, tw0);
            // 3. gap of new edge tid: the first sample block whose prefix max
            //    exceeds its key, then the first entry of that block that does
            if (tid < kb) {
                const LKey kc{S.nkx[c0 + tid], S.nkg[c0 + tid], S.nkl[c0 + tid]};
                int lo = 0, hi = ns;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (key_gt(LKey{S.sx[mid], S.sg[mid], S.sl[mid]}, kc)) hi = mid;
                    else lo = mid + 1;
                }
                gapc = m;
                if (lo < ns) {
                    // the block's X (four 16-B loads: the arrays have room past
                    // m), each entry's full key only where X ties
                    const int q0 = lo << 4, qn = min(16, m - q0);
                    const float4 *X4 = reinterpret_cast<const float4 *>(X + q0);
                    const float4 v0 = X4[0], v1 = X4[1], v2 = X4[2], v3 = X4[3];
                    const float bx[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                                          v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
                    int f = qn;
                    for (int u = 0; u < qn; ++u) {
                        if (bx[u] > kc.x) { f = u; break; }  // (a NaN X never: its key is the lowest)
                        if (bx[u] == kc.x && key_gt(entry_key(bx[u], G[q0 + u], LF[q0 + u]), kc)) { f = u; break; }
                    }
                    gapc = q0 + f;  // (f < qn: the block's maximum exceeds kc)
                }
            }
        }
        __syncthreads();
        PRK_BIG_T(11, tw0);
        // 4. the kept new edges counted per gap (d), each with its arrival
        if (tid < kb) {
            keptc = !expire || !(S.nky[c0 + tid] <= Row);
            if (keptc) kr = atomicAdd(&L.d[gapc], 1);
            if (kr > 0) S.collide = 1;
        }
        __syncthreads();
        PRK_BIG_T(12, tw0);
    }
    // 5. one scan over the entries q <= m (q = m: the tail gap): keep(q) and
    //    d(q) sums; a kept entry q moves to  #kept before q + #new of gap <= q,
    //    and gap q's new edges start at  base[q] = #kept before q + #new of gap < q
    const bool cnt = kb > 0;
    const int ns = m + (cnt ? 1 : 0), Ts = (ns + kBigThreads - 1) / kBigThreads;
    int32_t vk[kBigU], vd[kBigU];
    const bool regs = Ts <= kBigU;
    auto load = [&](int t0) {
#pragma unroll
        for (int u = 0; u < kBigU; ++u) {
            const int q = (t0 + u) * kBigThreads + tid;
            vk[u] = 0;
            vd[u] = 0;
            if (t0 + u < Ts && q < ns) {
                if (q < m) vk[u] = (!expire || !(YM[q] <= Row)) ? 1 : 0;
                if (cnt) vd[u] = L.d[q];
            }
        }
    };
    if (regs) load(0);
    for (int t0 = 0; t0 < Ts; t0 += kBigU) {
        if (!regs) load(t0);
#pragma unroll
        for (int u = 0; u < kBigU; ++u) {
            if (t0 + u >= Ts) break;
            const int32_t sk = wave_incl_sum_i32(vk[u]), sd = wave_incl_sum_i32(vd[u]);
            if (lane == 63) {
                S.ts[(t0 + u) * kBigWaves + w] = sk;
                S.tm[(t0 + u) * kBigWaves + w] = sd;
            }
        }
    }
    __syncthreads();
    int32_t kept_old = 0, kept_new = 0;
    {
        const bool mine = tid < Ts * kBigWaves;
        const int32_t a = mine ? S.ts[tid] : 0, b = mine ? S.tm[tid] : 0;
        int32_t ea, eb;
        blk_excl_sum2(R, a, b, ea, eb, kept_old, kept_new);
        if (mine) { S.ts[tid] = ea; S.tm[tid] = eb; }
    }
    __syncthreads();
    for (int t0 = 0; t0 < Ts; t0 += kBigU) {
        if (!regs) load(t0);
#pragma unroll
        for (int u0 = 0; u0 < kBigU; u0 += 4) {
            if (t0 + u0 >= Ts) break;
            // the entries' fields, four tiles' loads in flight at once
            float fx[4], fg[4];
            int32_t fl[4], fy[4], fw[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int q = min((t0 + u0 + v) * kBigThreads + tid, m - 1);
                fx[v] = fg[v] = 0.0f;
                fl[v] = fy[v] = fw[v] = 0;
                if (m > 0) { fx[v] = X[q]; fg[v] = G[q]; fl[v] = LF[q]; fy[v] = YM[q]; fw[v] = EI[q]; }
            }
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int u = u0 + v;
                if (t0 + u >= Ts) break;
                const int q = (t0 + u) * kBigThreads + tid;
                const int32_t sk = wave_incl_sum_i32(vk[u]), sd = wave_incl_sum_i32(vd[u]);
                const int32_t before = S.ts[(t0 + u) * kBigWaves + w] + sk - vk[u];  // kept entries before q
                const int32_t nex = S.tm[(t0 + u) * kBigWaves + w] + sd - vd[u];     // new edges of gap < q
                if (q < m && vk[u]) {
                    const int32_t to = before + nex + vd[u];
                    B.x[to] = fx[v]; B.g[to] = fg[v]; B.left[to] = fl[v]; B.ymax[to] = fy[v]; B.ei[to] = fw[v];
                }
                if (cnt && q < ns) L.base[q] = before + nex;
            }
        }
    }
    __syncthreads();
    PRK_BIG_T(13, tw0);
    // 6. the kept new edges into their places: gap(c)'s block [base, base +
    //    d) holds its new edges ordered by (key, arrival) -- the members meet
    //    in that block (arrival slots), rank themselves, then move
    if (cnt && !S.collide) {  // one new edge a gap: no ranking
        if (tid < kb && keptc) {
            const int32_t to = L.base[gapc];
            B.x[to] = S.nkx[c0 + tid]; B.g[to] = S.nkg[c0 + tid]; B.left[to] = S.nkl[c0 + tid];
            B.ymax[to] = S.nky[c0 + tid]; B.ei[to] = S.nke[c0 + tid];
        }
    } else if (cnt) {
        int32_t bs = 0, h = 0;
        if (tid < kb && keptc) {
            bs = L.base[gapc];
            h = L.d[gapc];
            B.ei[bs + kr] = tid;
        }
        __syncthreads();
        int32_t r = 0;
        if (tid < kb && keptc) {
            const LKey kc{S.nkx[c0 + tid], S.nkg[c0 + tid], S.nkl[c0 + tid]};
            for (int32_t j = 0; j < h; ++j) {
                const int32_t u = B.ei[bs + j];
                if (u == tid) continue;
                const LKey k{S.nkx[c0 + u], S.nkg[c0 + u], S.nkl[c0 + u]};
                r += (key_gt(kc, k) || (!key_gt(k, kc) && u < tid)) ? 1 : 0;
            }
        }
        __syncthreads();
        if (tid < kb && keptc) {
            const int32_t to = bs + r;
            B.x[to] = S.nkx[c0 + tid]; B.g[to] = S.nkg[c0 + tid]; B.left[to] = S.nkl[c0 + tid];
            B.ymax[to] = S.nky[c0 + tid]; B.ei[to] = S.nke[c0 + tid];
        }
    }
    __syncthreads();
    PRK_BIG_T(14, tw0);
    return kept_old + kept_new;
}

// Pairing (3751-3869) of the list in buffer cur (m >= 1 entries) into buffer
// cur ^ 1, one pass: thread k loads pairs k - 1, k and k + 1, steps them (X
// += Gradient), does their first swaps (3831-3841) and the boundary swaps on
// either side of pair k (3843-3853: boundaries (2k - 1, 2k) are disjoint, and
// each reads what the first swaps left), and writes entries 2k, 2k + 1.  It
// also leaves the row's list in ids[off, off + m) (the pairs' edges, before
// the step), the row's record ri = (off, m, j0 or kBigNoEmit, the unpaired
// odd last entry or -1), the per-16 key maxima of the result in S.s* and d
// zeroed -- the next row's insertion starts from them.
__device__ __forceinline__ void big_pair(const BigList &L, BigLds &S, int cur, int m, int32_t r, bool emit,
                                         uint32_t j0, uint32_t off) {
    constexpr int PB = 1;  // tiles whose loads are in flight at once (2: spills)
    const int tid = threadIdx.x, lane = tid & 63;
    const int P = m >> 1, items = P + (m & 1);
    const BigBuf A = L.buf(cur), B = L.buf(cur ^ 1);
    int32_t *ids = L.ids + off;
    if (tid == 0) {
        int32_t *q = L.ri + 4 * (size_t)r;
        q[0] = (int32_t)off;
        q[1] = m;
        q[2] = emit ? (int32_t)j0 : (int32_t)kBigNoEmit;
        if (!(m & 1)) q[3] = -1;
    }
    for (int k0 = 0; k0 < items; k0 += PB * kBigThreads) {
        // pairs k - 1, k, k + 1 (clamped; the odd last entry's pair reads past m: in the slice)
        float2 px[PB][3], pg[PB][3];
        int2 pl[PB][3], py[PB][3], pi[PB][3];
#pragma unroll
        for (int v = 0; v < PB; ++v) {
            const int k = min(k0 + v * kBigThreads + tid, items - 1);
#pragma unroll
            for (int h = 0; h < 3; ++h) {
                const int e = 2 * min(max(k - 1 + h, 0), items - 1);
                px[v][h] = *reinterpret_cast<const float2 *>(A.x + e);
                pg[v][h] = *reinterpret_cast<const float2 *>(A.g + e);
                pl[v][h] = *reinterpret_cast<const int2 *>(A.left + e);
                py[v][h] = *reinterpret_cast<const int2 *>(A.ymax + e);
                pi[v][h] = *reinterpret_cast<const int2 *>(A.ei + e);
            }
        }
#pragma unroll
        for (int v = 0; v < PB; ++v) {
            if (k0 + v * kBigThreads >= items) break;  // (uniform: every lane of a live tile takes the maxima)
            const int k = k0 + v * kBigThreads + tid;
            const int e = 2 * k;
            LKey ka{-INFINITY, -INFINITY, INT32_MIN}, kb2{-INFINITY, -INFINITY, INT32_MIN};
            if (k < items) {
                const float2 x1 = px[v][1], g1 = pg[v][1];
                const int2 l1 = pl[v][1], y1 = py[v][1], i1 = pi[v][1];
                ids[e] = i1.x;
                if (k == P) {  // the odd last entry: not paired, not stepped
                    B.x[e] = x1.x; B.g[e] = g1.x; B.left[e] = l1.x; B.ymax[e] = y1.x; B.ei[e] = i1.x;
                    L.d[e] = 0;
                    L.ri[4 * (size_t)r + 3] = i1.x;
                    ka = entry_key(x1.x, g1.x, l1.x);
                } else {
                    ids[e + 1] = i1.y;
                    // stepped (3811-3829), then each pair's first swap: f / s = its first / second
                    bool sidx[3];  // (per pair: its entries swapped)
                    float sx[3][2];
#pragma unroll
                    for (int h = 0; h < 3; ++h) {
                        const float a = px[v][h].x + pg[v][h].x, b = px[v][h].y + pg[v][h].y;
                        sidx[h] = a > b;
                        sx[h][0] = sidx[h] ? b : a;  // first
                        sx[h][1] = sidx[h] ? a : b;  // second
                    }
                    const bool lo = k >= 1 && sx[0][1] > sx[1][0];      // boundary k: pair k - 1's second comes down
                    const bool hi = k + 1 < P && sx[1][1] > sx[2][0];   // boundary k + 1: pair k + 1's first comes up
                    // entry 2k: pair k - 1's second (its .x if it swapped, else .y) or pair k's first;
                    // entry 2k + 1: pair k + 1's first or pair k's second (selects: no indexed registers)
                    const bool f0y = lo ? !sidx[0] : sidx[1], f1y = hi ? sidx[2] : !sidx[1];
                    const float ox0 = lo ? sx[0][1] : sx[1][0], ox1 = hi ? sx[2][0] : sx[1][1];
                    const float2 G0 = lo ? pg[v][0] : pg[v][1], G1 = hi ? pg[v][2] : pg[v][1];
                    const int2 L0 = lo ? pl[v][0] : pl[v][1], L1 = hi ? pl[v][2] : pl[v][1];
                    const int2 Y0 = lo ? py[v][0] : py[v][1], Y1 = hi ? py[v][2] : py[v][1];
                    const int2 I0 = lo ? pi[v][0] : pi[v][1], I1 = hi ? pi[v][2] : pi[v][1];
                    const float og0 = f0y ? G0.y : G0.x, og1 = f1y ? G1.y : G1.x;
                    const int32_t ol0 = f0y ? L0.y : L0.x, ol1 = f1y ? L1.y : L1.x;
                    const int32_t oy0 = f0y ? Y0.y : Y0.x, oy1 = f1y ? Y1.y : Y1.x;
                    const int32_t oi0 = f0y ? I0.y : I0.x, oi1 = f1y ? I1.y : I1.x;
                    *reinterpret_cast<float2 *>(B.x + e) = make_float2(ox0, ox1);
                    *reinterpret_cast<float2 *>(B.g + e) = make_float2(og0, og1);
                    *reinterpret_cast<int2 *>(B.left + e) = make_int2(ol0, ol1);
                    *reinterpret_cast<int2 *>(B.ymax + e) = make_int2(oy0, oy1);
                    *reinterpret_cast<int2 *>(B.ei + e) = make_int2(oi0, oi1);
                    *reinterpret_cast<int2 *>(L.d + e) = make_int2(0, 0);
                    ka = entry_key(ox0, og0, ol0);
                    kb2 = entry_key(ox1, og1, ol1);
                }
            }
            LKey kk = key_gt(kb2, ka) ? kb2 : ka;  // the maximum of the 16 entries of 8 lanes
            int32_t p = 0;
            key_max_step<kDppShr1>(kk, p);
            key_max_step<kDppShr2>(kk, p);
            key_max_step<kDppShr4>(kk, p);
            if ((lane & 7) == 7 && (k >> 3) < kBigSamp) {
                S.sx[k >> 3] = kk.x; S.sg[k >> 3] = kk.g; S.sl[k >> 3] = kk.l;
            }
        }
    }
    __syncthreads();
}

// One workgroup per huge object: its list in the pool slice at big_off
// (big_slice_ints(big_cap, meta rows, meta ents); big_cap >= its most active
// entries; big_meta[2b], big_meta[2b + 1]: its rows MaxY - FirstRow and list
// entries over them, k_obj_maxact's sizes).
__global__ void __launch_bounds__(kBigThreads) k_obj_walk_big(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                             const uint32_t *__restrict__ big,
                                                             const unsigned long long *__restrict__ big_off,
                                                             const uint32_t *__restrict__ big_cap,
                                                             const uint32_t *__restrict__ big_meta,
                                                             int32_t *__restrict__ pool,
                                                             const uint32_t *__restrict__ escan,
                                                             const uint32_t *__restrict__ total0p,
                                                             const ObjEdge *__restrict__ work,
                                                             const unsigned long long *__restrict__ soff,
                                                             uint32_t *__restrict__ err,
                                                             const uint32_t *__restrict__ prstat) {
    __shared__ BigLds S;
    __shared__ BlockRed R;
    const uint32_t o = big[blockIdx.x];
    if (prstat && prstat[o] == kPrDone) return;  // walked by rows (k_pr_*)
    const ObjDesc od = objs[o];
    const uint32_t bound = (uint32_t)(soff[o + 1] - soff[o]);
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const uint32_t cap = min(big_cap[blockIdx.x], kBigMaxM), rows_cap = big_meta[2 * blockIdx.x],
                   ents = big_meta[2 * blockIdx.x + 1];
    BigList L;
    L.carve(pool + big_off[blockIdx.x], cap, rows_cap);
    const int tid = threadIdx.x;
    for (uint32_t q = tid; q < 4 * rows_cap; q += kBigThreads) L.ri[q] = q % 4 == 3 ? -1 : 0;  // (rows not walked: m = 0)
    if (n == 0) {
        if (tid == 0) { L.hdr[0] = 0; L.hdr[1] = 0; }
        return;
    }
    const ObjEdge *E = work + e0;
    int32_t mr = INT32_MIN;
    for (uint32_t i = tid; i < n; i += kBigThreads) mr = max(mr, E[i].YMax);
    const int32_t MaxY = min(min(blk_max(R, mr), fp.H), fp.row1);
    const int32_t FirstRow = E[0].YMin;
    const int32_t RowLo = fp.draws[od.draw].mode != MODE_AVX ? fp.row0 - 1 : fp.row0;
    const bool fits = (int64_t)MaxY - FirstRow <= (int64_t)rows_cap;
    if (tid == 0) {
        L.hdr[0] = FirstRow;
        L.hdr[1] = fits ? max(0, MaxY - FirstRow) : 0;
        if (!fits) atomicOr(err, 1u);  // (never: k_obj_maxact sized it)
    }
    if (!fits) return;
    int cur = 0, m = 0;
    uint32_t ins = 0, emitted = 0, off = 0;
    bool bad = false, samples = false;
    unsigned long long wpa[16] = {}, *wp = PRK_WPROF && tid == 0 ? wpa : nullptr;
    unsigned long long tw0 = PRK_WT(), twall = tw0;
    // the window of sorted edges at `pf` (loaded a row ahead, while the
    // previous row pairs)
    uint32_t pf = UINT32_MAX;
    int32_t y = INT32_MAX, l = 0, ym = 0;
    float x = 0.0f, g = 0.0f;
    auto fetch = [&](uint32_t at) {
        const uint32_t i = at + (uint32_t)tid;
        y = INT32_MAX; x = g = 0.0f; l = ym = 0;
        if (i < n) {
            const ObjEdge &C = E[i];
            y = C.YMin; x = C.X; g = C.G; l = C.Left; ym = C.YMax;
        }
        pf = at;
    };
    for (int32_t Row = FirstRow; Row < MaxY; ++Row) {
        bool expired = false;
        if (PRK_WPROF && wp) wp[3] += 1;
        for (;;) {  // the row's new edges, a window of kBigThreads at a time (3654-3713)
            if (pf != ins) fetch(ins);
            int32_t lt, kb, nanc;
            blk_sum3(R, y < Row ? 1 : 0, y == Row ? 1 : 0, (y == Row && (x != x || g != g)) ? 1 : 0, lt, kb, nanc);
            if (lt) {  // (never past the first row of a sorted list)
                ins += (uint32_t)lt;
                continue;
            }
            if (kb == 0) break;
            if ((uint32_t)(m + kb) > cap) {  // (never: cap >= the most listed entries)
                bad = true;
                break;
            }
            if (tid < kb) {
                S.nkx[tid] = x; S.nkg[tid] = g; S.nkl[tid] = l; S.nky[tid] = ym; S.nke[tid] = (int32_t)(ins + tid);
            }
            __syncthreads();
            PRK_BIG_T(0, tw0);
            if (PRK_WPROF && wp) { wp[4] += 1; wp[8] += (unsigned)kb; }
            const bool last = kb < kBigThreads;
            if (nanc) {  // one edge at a time (no total order on a batch with a NaN key)
                for (int t = 0; t < kb; ++t) {
                    const bool ex = last && t + 1 == kb;
                    m = big_insert_expire(L, S, R, cur, m, t, 1, ex, Row, samples, wp);
                    cur ^= 1;
                    samples = false;
                }
            } else {
                m = big_insert_expire(L, S, R, cur, m, 0, kb, last, Row, samples, wp);
                cur ^= 1;
                samples = false;
            }
            PRK_BIG_T(1, tw0);
            expired = last;
            ins += (uint32_t)kb;
            if (last) break;
        }
        if (bad) break;
        if (pf != ins && ins < n) fetch(ins);  // (the next row's window, in flight through this row's pairing)
        if (!expired && m > 0) {  // expiry 3715-3749 alone
            m = big_insert_expire(L, S, R, cur, m, 0, 0, true, Row, false, wp);
            cur ^= 1;
            samples = false;
        }
        PRK_BIG_T(2, tw0);
        if (m == 0) {  // nothing happens on the rows before the next insertion: go there
            if (ins >= n) break;
            Row = max(Row, E[ins].YMin - 1);
            continue;
        }
        const bool emit = Row >= RowLo;
        const uint32_t P = (uint32_t)(m >> 1);
        if ((emit && emitted + P > bound) || (uint64_t)off + (uint32_t)m > ents) {  // (never: sized by the bounds)
            bad = true;
            break;
        }
        big_pair(L, S, cur, m, Row - FirstRow, emit, emitted, off);
        cur ^= 1;
        samples = true;
        off += (uint32_t)m;
        if (emit) emitted += P;
        PRK_BIG_T(5, tw0);
        if (PRK_WPROF && wp) wp[6] += (unsigned)m;
    }
    if (bad && tid == 0) atomicOr(err, 1u);
    if (PRK_WPROF && wp) {
        wp[7] += PRK_WT() - twall;
        for (int k = 0; k < 16; ++k) atomicAdd(fp.prof + k, wp[k]);
    }
}

// ---------------------------------------------------------------------------
// The huge-object walk with the whole list in LDS (objects of at most
// kLdsCap most active edges -- C3b as ONE object: 8898): the same rows, the
// same list operations and the same output (hdr, ri, ids: k_big_replay sets
// the spans up) as k_obj_walk_big, but every list access an LDS access, so a
// row is a chain of LDS passes and workgroup barriers instead of device-
// memory round trips.  An entry is 14 bytes: X, Gradient, its edge index and
// (min(YMax, MaxY) - FirstRow) << 1 | Left (FillEdgeTable's Left is 0 / 1).
// The list is updated in place: a pass reads what it moves into registers,
// a barrier, then writes.
//   insertion + expiry (3654-3749): each new edge's gap as k_obj_walk_big
//     finds it (per-16 key maxima, prefix-maxed, then 16 entries); the kept
//     new edges ranked by (gap, key, arrival) through coarse bins of 16 gaps
//     (counts, scan, each bin's few members compared); thread t owns old
//     entries [9t, 9t + 9): a kept entry q goes to  #kept before q + #kept new
//     of gap <= q  (a binary search once, then a walk), a kept new edge to
//     #kept before its gap + its rank.
//   pairing (3751-3869): thread k reads pairs k - 1, k, k + 1, steps and
//     swaps them as big_pair does, writes entries 2k, 2k + 1 after a barrier,
//     with the next row's per-16 key maxima.
// ---------------------------------------------------------------------------
#ifndef PRK_LDS_WINCOUNT
#define PRK_LDS_WINCOUNT 1  // the LDS walk counts the next row's window in the pairing pass
#endif
constexpr int kLdsCap = 9200;                      // list entries (< 577 * 16: 576 coarse bins)
constexpr int kLdsPer = (kLdsCap + kBigThreads - 1) / kBigThreads;  // old entries a thread owns (9)
constexpr int kLdsSamp = 576;                      // per-16 maxima (>= kLdsCap / 16)
constexpr int kLdsPairs = (kLdsCap / 2 + kBigThreads - 1) / kBigThreads;  // pairs a thread owns (5)
static_assert(kLdsCap <= kLdsSamp * 16 && kLdsPer * kBigThreads >= kLdsCap, "LDS walk sizes");
struct alignas(16) LdsWalk {  // (aligned: the pairing reads a pair's fields as one 8-B access)
    float x[kLdsCap], g[kLdsCap];
    int32_t e[kLdsCap];
    uint16_t y[kLdsCap];                 // (min(YMax, MaxY) - FirstRow) << 1 | Left
    float sx[kLdsSamp], sg[kLdsSamp];   // per-16 key maxima; then (insertion) the coarse bins' counts / cursors
    int32_t sl[kLdsSamp];               // (... and the bins' members, uint16)
    float nx[kBigThreads], ng[kBigThreads];  // the batch's new edges
    int32_t ne[kBigThreads];
    uint16_t ny[kBigThreads], ngap[kBigThreads];
    uint16_t sgap[kBigThreads];          // the kept new edges' gaps in (gap, key, arrival) order
    uint16_t kbase[kBigThreads];         // kept old entries before thread t's nine
    int4 wc[kBigThreads / 64];           // the next row's window counts per wave (lds_pair: lt, kb, NaN keys)
};
__device__ __forceinline__ LKey lds_key(const LdsWalk &W, int q) { return entry_key(W.x[q], W.g[q], W.y[q] & 1); }
struct LdsE {  // an entry in registers
    float x, g;
    int32_t yp, e;  // packed row | Left, edge index
};
__device__ __forceinline__ LdsE lds_entry(const LdsWalk &W, int q) { return LdsE{W.x[q], W.g[q], W.y[q], W.e[q]}; }
// A pair stepped (X += Gradient, 3811-3829) and first-swapped (3831-3841):
// a its first entry, b its second.
__device__ __forceinline__ void lds_first_swap(LdsE &a, LdsE &b) {
    a.x += a.g;
    b.x += b.g;
    if (a.x > b.x) {
        const LdsE t = a;
        a = b;
        b = t;
    }
}
__device__ __forceinline__ uint16_t lds_ypack(int32_t ymax, int32_t left, int32_t FirstRow, int32_t MaxY) {
    return (uint16_t)(((min(max(ymax, FirstRow), MaxY) - FirstRow) << 1) | (left & 1));
}

// Insertion of the batch's new edges W.n*[c0, c0 + kb) and, when `expire`,
// expiry at row FirstRow + rrel (an entry leaves when YMax <= Row: its packed
// row <= rrel); returns the new length.  samples_ok: W.s* hold the list's
// per-16 key maxima (the pairing left them).
__device__ __forceinline__ int lds_insert(LdsWalk &W, BlockRed &R, int m, int c0, int kb, bool expire,
                                          int32_t rrel, bool samples_ok, unsigned long long *wp = nullptr) {
    unsigned long long tw0 = PRK_WT();
    const int tid = threadIdx.x;
    const bool mine = tid < kb;
    int32_t gapc = 0;
    bool keptc = false;
    if (kb > 0) {
        if (m > 0) {
            const int ns = (m + 15) >> 4;
            if (!samples_ok) {
                for (int j = tid; j < ns; j += kBigThreads) {
                    LKey mx{-INFINITY, -INFINITY, INT32_MIN};
                    for (int u = 0; u < 16 && 16 * j + u < m; ++u) {
                        const LKey k = lds_key(W, 16 * j + u);
                        if (key_gt(k, mx)) mx = k;
                    }
                    W.sx[j] = mx.x; W.sg[j] = mx.g; W.sl[j] = mx.l;
                }
                blk_sync<true>();
            }
            LKey pk = tid < ns ? LKey{W.sx[tid], W.sg[tid], W.sl[tid]} : LKey{-INFINITY, -INFINITY, INT32_MIN};
            blk_key_prefix_max<true>(R, pk);
            if (tid < ns) { W.sx[tid] = pk.x; W.sg[tid] = pk.g; W.sl[tid] = pk.l; }
            blk_sync<true>();
            PRK_BIG_T(9, tw0);
            if (mine) {  // the first entry whose key exceeds the new edge's (3663-3667)
                const LKey kc{W.nx[c0 + tid], W.ng[c0 + tid], (int32_t)(W.ny[c0 + tid] & 1)};
                int lo = 0, hi = ns;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (key_gt(LKey{W.sx[mid], W.sg[mid], W.sl[mid]}, kc)) hi = mid;
                    else lo = mid + 1;
                }
                gapc = m;
                if (lo < ns) {
                    const int q0 = lo << 4, qn = min(16, m - q0);
                    for (int u = 0; u < qn; ++u)
                        if (key_gt(lds_key(W, q0 + u), kc)) { gapc = q0 + u; break; }
                }
            }
            blk_sync<true>();  // (the sample arrays hold the bins below)
            PRK_BIG_T(10, tw0);
        }
        if (mine) {
            keptc = !expire || (int32_t)(W.ny[c0 + tid] >> 1) > rrel;
            W.ngap[tid] = (uint16_t)gapc;
        }
    }
    // the kept new edges ranked by (gap, key, arrival), through coarse bins of 16 gaps
    int kn = 0;
    int32_t srank = 0;
    if (kb > 0) {
        int32_t *bcnt = reinterpret_cast<int32_t *>(W.sx), *bcur = reinterpret_cast<int32_t *>(W.sg);
        uint16_t *bmem = reinterpret_cast<uint16_t *>(W.sl);
        const int nb = (m >> 4) + 1;  // (<= 576)
        if (tid < nb) bcnt[tid] = 0;
        blk_sync<true>();
        const int bin = gapc >> 4;
        if (mine && keptc) atomicAdd(&bcnt[bin], 1);
        blk_sync<true>();
        const int32_t cv = tid < nb ? bcnt[tid] : 0;
        int32_t tot;
        const int32_t ex = blk_excl_sum<true>(R, cv, tot);
        kn = tot;
        if (tid < nb) { bcnt[tid] = ex; bcur[tid] = ex; }
        blk_sync<true>();
        if (mine && keptc) bmem[atomicAdd(&bcur[bin], 1)] = (uint16_t)tid;
        blk_sync<true>();
        if (mine && keptc) {
            const LKey kc{W.nx[c0 + tid], W.ng[c0 + tid], (int32_t)(W.ny[c0 + tid] & 1)};
            const int32_t b0 = bcnt[bin], b1 = bin + 1 < nb ? bcnt[bin + 1] : kn;
            int32_t r = 0;
            for (int32_t s = b0; s < b1; ++s) {
                const int u = bmem[s];
                if (u == tid) continue;
                const int32_t gu = W.ngap[u];
                const LKey ku{W.nx[c0 + u], W.ng[c0 + u], (int32_t)(W.ny[c0 + u] & 1)};
                r += (gu < gapc || (gu == gapc && (key_gt(kc, ku) || (!key_gt(ku, kc) && u < tid)))) ? 1 : 0;
            }
            srank = b0 + r;
            W.sgap[srank] = (uint16_t)gapc;
        }
        PRK_BIG_T(11, tw0);
    }
    // the old entries (thread t: [9t, 9t + 9)), their kept counts
    const int q0 = kLdsPer * tid;
    float ox[kLdsPer], og[kLdsPer];
    int32_t oe[kLdsPer];
    uint16_t oy[kLdsPer];
    uint32_t keep = 0;
    int32_t kc_t = 0;
#pragma unroll
    for (int u = 0; u < kLdsPer; ++u) {
        const int q = q0 + u;
        ox[u] = og[u] = 0.0f;
        oe[u] = 0;
        oy[u] = 0;
        if (q < m) {
            ox[u] = W.x[q]; og[u] = W.g[q]; oe[u] = W.e[q]; oy[u] = W.y[q];
            const bool k = !expire || (int32_t)(oy[u] >> 1) > rrel;
            keep |= (k ? 1u : 0u) << u;
            kc_t += k ? 1 : 0;
        }
    }
    int32_t kept_old;
    const int32_t kbt = blk_excl_sum<true>(R, kc_t, kept_old);  // (its barriers also publish sgap)
    W.kbase[tid] = (uint16_t)kbt;
    blk_sync<true>();
    PRK_BIG_T(12, tw0);
    // places: a kept old entry q at #kept before q + #kept new of gap <= q
    int32_t opos[kLdsPer];
    {
        int lo = 0, hi = kn;  // #kept new with gap < q0... (the first with gap > q0 - 1)
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((int)W.sgap[mid] < q0) lo = mid + 1;
            else hi = mid;
        }
        int p = lo;
        int32_t kb_run = kbt;
#pragma unroll
        for (int u = 0; u < kLdsPer; ++u) {
            const int q = q0 + u;
            while (p < kn && (int)W.sgap[p] <= q) ++p;
            opos[u] = kb_run + p;
            kb_run += (keep >> u) & 1u;
        }
    }
    // a kept new edge at #kept before its gap + its rank
    int32_t npos = 0;
    if (kb > 0 && mine && keptc) {
        int32_t before = kept_old;
        if (gapc < m) {
            const int t = gapc / kLdsPer;
            before = W.kbase[t];
            for (int q = kLdsPer * t; q < gapc; ++q) before += (!expire || (int32_t)(W.y[q] >> 1) > rrel) ? 1 : 0;
        }
        npos = before + srank;
    }
    blk_sync<true>();  // (every read of the old list is done)
    PRK_BIG_T(13, tw0);
#pragma unroll
    for (int u = 0; u < kLdsPer; ++u)
        if ((keep >> u) & 1u) {
            const int32_t to = opos[u];
            W.x[to] = ox[u]; W.g[to] = og[u]; W.e[to] = oe[u]; W.y[to] = oy[u];
        }
    if (kb > 0 && mine && keptc) {
        W.x[npos] = W.nx[c0 + tid]; W.g[npos] = W.ng[c0 + tid]; W.e[npos] = W.ne[c0 + tid]; W.y[npos] = W.ny[c0 + tid];
    }
    blk_sync<true>();
    PRK_BIG_T(14, tw0);
    return kept_old + kn;
}

// Pairing (3751-3869) in place, as big_pair: the row's record and list out
// (ri, ids), every pair stepped and swapped, the next row's per-16 key maxima
// in W.s*.
// (nrow != INT32_MIN: also the next row's window counts from the thread's
// prefetched window edge (YMin y, key x, g), per wave into W.wc, so the next
// row's first window needs no workgroup reduction of its own)
__device__ __forceinline__ void lds_pair(LdsWalk &W, const BigList &L, int m, int32_t r, bool emit, uint32_t j0,
                                         uint32_t off, int32_t nrow, int32_t y, float x, float g,
                                         unsigned long long *wp = nullptr) {
    unsigned long long tw0 = PRK_WT();
    const int tid = threadIdx.x, lane = tid & 63;
    const int P = m >> 1, items = P + (m & 1);
    int32_t *ids = L.ids + off;
    if (tid == 0) {
        int32_t *q = L.ri + 4 * (size_t)r;
        q[0] = (int32_t)off;
        q[1] = m;
        q[2] = emit ? (int32_t)j0 : (int32_t)kBigNoEmit;
        q[3] = (m & 1) ? W.e[m - 1] : -1;
    }
    LdsE o0[kLdsPairs], o1[kLdsPairs];
#pragma unroll
    for (int i = 0; i < kLdsPairs; ++i) {
        const int k = tid + i * kBigThreads;
        o0[i] = o1[i] = LdsE{0.0f, 0.0f, 0, 0};
        if (k < items) {
            const int e = 2 * k;
            ids[e] = W.e[e];
            if (k == P) {  // the odd last entry: not paired, not stepped, stays
                o0[i] = lds_entry(W, e);
                continue;
            }
            ids[e + 1] = W.e[e + 1];
            // pairs k - 1, k, k + 1 stepped and first-swapped
            LdsE a[3], b[3];
#pragma unroll
            for (int h = 0; h < 3; ++h) {  // (a pair's entries as one 8-B read a field, y as one 4-B read)
                const int ea = 2 * min(max(k - 1 + h, 0), P - 1);
                const float2 px = *reinterpret_cast<const float2 *>(W.x + ea);
                const float2 pg = *reinterpret_cast<const float2 *>(W.g + ea);
                const int2 pe = *reinterpret_cast<const int2 *>(W.e + ea);
                const uint32_t py = *reinterpret_cast<const uint32_t *>(W.y + ea);
                a[h] = LdsE{px.x, pg.x, (int32_t)(py & 0xFFFFu), pe.x};
                b[h] = LdsE{px.y, pg.y, (int32_t)(py >> 16), pe.y};
                lds_first_swap(a[h], b[h]);
            }
            const bool lo = k >= 1 && b[0].x > a[1].x;      // boundary k (3843-3853)
            const bool hi = k + 1 < P && b[1].x > a[2].x;   // boundary k + 1
            o0[i] = lo ? b[0] : a[1];
            o1[i] = hi ? a[2] : b[1];
        }
    }
    blk_sync<true>();  // (every read of the list is done)
    PRK_BIG_T(15, tw0);
#pragma unroll
    for (int i = 0; i < kLdsPairs; ++i) {
        if (i * kBigThreads >= items) break;  // (uniform)
        const int k = tid + i * kBigThreads;
        const int e = 2 * k;
        LKey ka{-INFINITY, -INFINITY, INT32_MIN}, kb2{-INFINITY, -INFINITY, INT32_MIN};
        if (k < P) {
            *reinterpret_cast<float2 *>(W.x + e) = make_float2(o0[i].x, o1[i].x);
            *reinterpret_cast<float2 *>(W.g + e) = make_float2(o0[i].g, o1[i].g);
            *reinterpret_cast<int2 *>(W.e + e) = make_int2(o0[i].e, o1[i].e);
            *reinterpret_cast<uint32_t *>(W.y + e) = (uint32_t)(o0[i].yp & 0xFFFF) | ((uint32_t)o1[i].yp << 16);
            ka = entry_key(o0[i].x, o0[i].g, o0[i].yp & 1);
            kb2 = entry_key(o1[i].x, o1[i].g, o1[i].yp & 1);
        } else if (k == P) {
            ka = entry_key(o0[i].x, o0[i].g, o0[i].yp & 1);
        }
        LKey kk = key_gt(kb2, ka) ? kb2 : ka;  // the maximum of the 16 entries of 8 lanes
        int32_t p = 0;
        key_max_step<kDppShr1>(kk, p);
        key_max_step<kDppShr2>(kk, p);
        key_max_step<kDppShr4>(kk, p);
        if ((lane & 7) == 7 && (k >> 3) < kLdsSamp) {
            W.sx[k >> 3] = kk.x; W.sg[k >> 3] = kk.g; W.sl[k >> 3] = kk.l;
        }
    }
    if (nrow != INT32_MIN) {  // (uniform)
        const unsigned long long blt = __ballot(y < nrow), bkb = __ballot(y == nrow),
                                 bnan = __ballot(y == nrow && (x != x || g != g));
        if (lane == 0) W.wc[tid >> 6] = make_int4(__popcll(blt), __popcll(bkb), __popcll(bnan), 0);
    }
    blk_sync<true>();
}

// One workgroup per huge object whose most active edges fit kLdsCap (the
// pool slice, meta and outputs as k_obj_walk_big's).
__global__ void __launch_bounds__(kBigThreads) k_obj_walk_lds(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                             const uint32_t *__restrict__ big,
                                                             const unsigned long long *__restrict__ big_off,
                                                             const uint32_t *__restrict__ big_cap,
                                                             const uint32_t *__restrict__ big_meta,
                                                             int32_t *__restrict__ pool,
                                                             const uint32_t *__restrict__ escan,
                                                             const uint32_t *__restrict__ total0p,
                                                             const ObjEdge *__restrict__ work,
                                                             const unsigned long long *__restrict__ soff,
                                                             uint32_t *__restrict__ err,
                                                             const uint32_t *__restrict__ prstat) {
    __shared__ LdsWalk W;
    __shared__ BlockRed R;
    const uint32_t o = big[blockIdx.x];
    if (prstat && prstat[o] == kPrDone) return;  // walked by rows (k_pr_*)
    const ObjDesc od = objs[o];
    const uint32_t bound = (uint32_t)(soff[o + 1] - soff[o]);
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const uint32_t cap = min(big_cap[blockIdx.x], kBigMaxM), rows_cap = big_meta[2 * blockIdx.x],
                   ents = big_meta[2 * blockIdx.x + 1];
    BigList L;
    L.carve(pool + big_off[blockIdx.x], cap, rows_cap);
    const int tid = threadIdx.x;
    for (uint32_t q = tid; q < 4 * rows_cap; q += kBigThreads) L.ri[q] = q % 4 == 3 ? -1 : 0;  // (rows not walked: m = 0)
    if (n == 0) {
        if (tid == 0) { L.hdr[0] = 0; L.hdr[1] = 0; }
        return;
    }
    const ObjEdge *E = work + e0;
    int32_t mr = INT32_MIN;
    for (uint32_t i = tid; i < n; i += kBigThreads) mr = max(mr, E[i].YMax);
    const int32_t MaxY = min(min(blk_max(R, mr), fp.H), fp.row1);
    const int32_t FirstRow = E[0].YMin;
    const int32_t RowLo = fp.draws[od.draw].mode != MODE_AVX ? fp.row0 - 1 : fp.row0;
    const bool fits = (int64_t)MaxY - FirstRow <= (int64_t)rows_cap && (int64_t)MaxY - FirstRow < 16000;
    if (tid == 0) {
        L.hdr[0] = FirstRow;
        L.hdr[1] = fits ? max(0, MaxY - FirstRow) : 0;
        if (!fits) atomicOr(err, 1u);  // (never: k_obj_maxact sized it)
    }
    if (!fits) return;
    int m = 0;
    uint32_t ins = 0, emitted = 0, off = 0;
    bool bad = false, samples = false;
    unsigned long long wpa[16] = {}, *wp = PRK_WPROF && tid == 0 ? wpa : nullptr;
    unsigned long long tw0 = PRK_WT(), twall = tw0;
    uint32_t pf = UINT32_MAX;  // the window of sorted edges at pf, loaded a row ahead
    int32_t pre_row = INT32_MIN;  // PRK_LDS_WINCOUNT: W.wc holds row pre_row's counts of the window at pre_pf
    uint32_t pre_pf = UINT32_MAX;
    int32_t y = INT32_MAX, l = 0, ym = 0;
    float x = 0.0f, g = 0.0f;
    auto fetch = [&](uint32_t at) {
        const uint32_t i = at + (uint32_t)tid;
        y = INT32_MAX; x = g = 0.0f; l = ym = 0;
        if (i < n) {
            const ObjEdge &C = E[i];
            y = C.YMin; x = C.X; g = C.G; l = C.Left; ym = C.YMax;
        }
        pf = at;
    };
    for (int32_t Row = FirstRow; Row < MaxY; ++Row) {
        const int32_t rrel = Row - FirstRow;
        bool expired = false;
        if (PRK_WPROF && wp) wp[3] += 1;
        for (;;) {  // the row's new edges, a window of kBigThreads at a time (3654-3713)
            if (pf != ins) fetch(ins);
            int32_t lt, kb, nanc;
            if (PRK_LDS_WINCOUNT && pre_row == Row && pre_pf == pf) {  // (counted by the last row's pairing)
                lt = kb = nanc = 0;
#pragma unroll
                for (int w = 0; w < kBigThreads / 64; ++w) {
                    const int4 c = W.wc[w];
                    lt += c.x; kb += c.y; nanc += c.z;
                }
                pre_row = INT32_MIN;
            } else {
                blk_sum3<true>(R, y < Row ? 1 : 0, y == Row ? 1 : 0, (y == Row && (x != x || g != g)) ? 1 : 0, lt, kb,
                               nanc);
            }
            if (lt) {  // (never past the first row of a sorted list)
                ins += (uint32_t)lt;
                continue;
            }
            if (kb == 0) break;
            if (m + kb > kLdsCap || (uint32_t)(m + kb) > cap) {  // (never: cap >= the most listed entries)
                bad = true;
                break;
            }
            if (tid < kb) {
                W.nx[tid] = x; W.ng[tid] = g; W.ne[tid] = (int32_t)(ins + tid);
                W.ny[tid] = lds_ypack(ym, l, FirstRow, MaxY);
            }
            blk_sync<true>();
            PRK_BIG_T(0, tw0);
            if (PRK_WPROF && wp) { wp[4] += 1; wp[8] += (unsigned)kb; }
            const bool last = kb < kBigThreads;
            if (nanc) {  // one edge at a time (no total order on a batch with a NaN key)
                for (int t = 0; t < kb; ++t) {
                    m = lds_insert(W, R, m, t, 1, last && t + 1 == kb, rrel, samples, wp);
                    samples = false;
                }
            } else {
                m = lds_insert(W, R, m, 0, kb, last, rrel, samples, wp);
                samples = false;
            }
            PRK_BIG_T(1, tw0);
            expired = last;
            ins += (uint32_t)kb;
            if (last) break;
        }
        if (bad) break;
        if (pf != ins && ins < n) fetch(ins);  // (the next row's window, in flight through this row's pairing)
        if (!expired && m > 0) {  // expiry 3715-3749 alone
            m = lds_insert(W, R, m, 0, 0, true, rrel, false, wp);
            samples = false;
        }
        PRK_BIG_T(2, tw0);
        if (m == 0) {  // nothing happens on the rows before the next insertion: go there
            if (ins >= n) break;
            Row = max(Row, E[ins].YMin - 1);
            continue;
        }
        const bool emit = Row >= RowLo;
        const uint32_t P = (uint32_t)(m >> 1);
        if ((emit && emitted + P > bound) || (uint64_t)off + (uint32_t)m > ents) {  // (never: sized by the bounds)
            bad = true;
            break;
        }
        const bool pre = PRK_LDS_WINCOUNT && Row + 1 < MaxY;
        lds_pair(W, L, m, rrel, emit, emitted, off, pre ? Row + 1 : INT32_MIN, y, x, g, wp);
        if (pre) {
            pre_row = Row + 1;
            pre_pf = pf;
        }
        samples = true;
        off += (uint32_t)m;
        if (emit) emitted += P;
        PRK_BIG_T(5, tw0);
        if (PRK_WPROF && wp) wp[6] += (unsigned)m;
    }
    if (bad && tid == 0) atomicOr(err, 1u);
    if (PRK_WPROF && wp) {
        wp[7] += PRK_WT() - twall;
        for (int k = 0; k < 16; ++k) atomicAdd(fp.prof + k, wp[k]);
    }
}

// Every pair of every row of the huge objects, a thread each (grid: (rows,
// objects), a workgroup per row): both edges' states at the row -- the edge
// from FillEdgeTable stepped on each row it was listed on before this one,
// but its unpaired ones (3811-3829, as the walk stepped it) -- into the pair's
// PairRaw slot, its SpanPos and winner id beside it.
template <int M>
__global__ void __launch_bounds__(256) k_big_replay(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                    const uint32_t *__restrict__ big,
                                                    const unsigned long long *__restrict__ big_off,
                                                    const uint32_t *__restrict__ big_cap,
                                                    const uint32_t *__restrict__ big_meta,
                                                    const int32_t *__restrict__ pool,
                                                    const uint32_t *__restrict__ escan,
                                                    const uint32_t *__restrict__ total0p,
                                                    const ObjEdge *__restrict__ work,
                                                    const unsigned long long *__restrict__ soff,
                                                    PairRaw *__restrict__ raw, SpanPos *__restrict__ pos,
                                                    uint32_t *__restrict__ span_tri, const uint32_t *__restrict__ prstat) {
    const uint32_t o = big[blockIdx.y];
    if (prstat && prstat[o] == kPrDone) return;
    const ObjDesc od = objs[o];
    if (fp.draws[od.draw].mode != M) return;
    BigList L;
    L.carve(const_cast<int32_t *>(pool) + big_off[blockIdx.y], min(big_cap[blockIdx.y], kBigMaxM),
            big_meta[2 * blockIdx.y]);
    const int32_t FirstRow = L.hdr[0], rows = L.hdr[1];
    const int32_t r = (int32_t)blockIdx.x;
    if (r >= rows) return;
    const int32_t off = L.ri[4 * r], m = L.ri[4 * r + 1], j0 = L.ri[4 * r + 2];
    if ((uint32_t)j0 == kBigNoEmit || m < 2) return;
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const ObjEdge *E = work + e0;
    const uint32_t base = (uint32_t)soff[o], bound = (uint32_t)(soff[o + 1] - soff[o]);
    const int32_t Row = FirstRow + r;
    const int32_t *ids = L.ids + off;
    for (int k = threadIdx.x; k < m / 2; k += blockDim.x) {
        const uint32_t j = (uint32_t)j0 + (uint32_t)k;
        if (j >= bound) break;
        ObjEdge st[2];
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const int32_t ei = ids[2 * k + side];
            ObjEdge e = E[ei];
            for (int32_t q = e.YMin; q < Row; ++q)
                if (L.ri[4 * (q - FirstRow) + 3] != ei) obj_step<M>(e);
            st[side] = e;
        }
        PairRaw pr;
        pair_raw_out(st[0], st[1], pr);
        raw[base + j] = pr;
        pos[base + j] = SpanPos{Row, (int32_t)od.draw, 0, SPAN_RAW};
        span_tri[base + j] = od.g0;
    }
}

// ---------------------------------------------------------------------------
// The chunked walk of large objects (objects of kObjWaveTris triangles or
// more whose rows and lists fit: k_obj_maxact's sizes, host-checked).
//
// The walk is serial in rows: the list at row r is a function of the list at
// r - 1.  But that dependence fades: entries expire, crossings swap back, so
// a walk started a few rows early from a plausible list -- the row's active
// edges sorted by the insertion key (X, Gradient, Left), ties in MergeSort
// order, which is what a batch inserted into an empty list is -- usually
// reaches the true list.  So the object's rows are cut into chunks of
// kPrChunk rows and every chunk is walked at once by the workgroup walk's
// own list operations (walk_chunk = walk_object_block from a given list over
// a given row range): chunk j > 0 from the sorted list of chunk j - 1's first
// row, walking chunk j - 1's rows as a warm-up (stepping, no spans), then its
// own rows (spans).  Exactness is checked, not assumed: chunk j's list at its
// first row must equal the list chunk j - 1 ended with (k_pr_cmp); chunk 0
// starts from the true list; a chunk whose predecessor walked from the true
// list and ended on its start list walked from the true list too; any other
// chunk is walked again, in order, from its predecessor's true end list
// (k_pr_fix: one workgroup per object, chunk after chunk, walking only
// those; C2 and ConstructSphere need none).  The spans of a chunk go to the
// slots its rows take in the sequential walk -- every row pairs all its
// entries (objects with an odd row are left to k_obj_walk_wave), so a row's
// pairs are its entries / 2 whatever their order -- in the same order.
//   k_pr_hist   workgroup per object: its rows' entry counts and their scan
//               (the span slots), the first sorted edge of every row
//   k_pr_fill   thread per edge: stepped row by row as the walk steps it
//               (obj_step), its state and key at every chunk's first row
//   k_pr_start  workgroup per chunk: the sorted list of its first row (rank
//               sort), as edge states
//   k_pr_chunk  workgroup per chunk: the warm-up and the chunk's walk
//   k_pr_cmp    workgroup per chunk: its end list against the next chunk's
//               start list
//   k_pr_fix    workgroup per object: the chunks that did not walk from the
//               true list, walked again in order
// ---------------------------------------------------------------------------
#ifndef PRK_PR_CHUNK
#define PRK_PR_CHUNK 8
#endif
constexpr int32_t kPrChunk = PRK_PR_CHUNK;  // rows per chunk
constexpr int32_t kPrMaxM = 1022;           // most entries of a list (the workgroup walk's largest LDS list)
struct PrObj {                              // per object of the walk (host: flush_spans)
    uint32_t o;                             // object index
    uint32_t row_off;                       // its first row in the pass's row arrays (rows + 1 each)
    uint32_t rows;                          // MaxY - FirstRow (k_obj_maxact)
    uint32_t chunk_off;                     // its first chunk in the pass's chunk arrays
    uint32_t most;                          // k_obj_maxact's most entries (the list stride per chunk)
    uint32_t ent_off;                       // its first list entry: chunk j's lists at ent_off + j * most
    uint32_t pad0, pad1;
};
struct PrRow {                              // per object, set by k_pr_hist
    int32_t first_row, max_y;
};
__device__ __forceinline__ uint32_t pr_chunks(const PrObj &P) { return (P.rows + kPrChunk - 1) / kPrChunk; }
__device__ __forceinline__ bool pr_key_lt(float ax, float ag, int32_t al, uint32_t ai, float bx, float bg, int32_t bl,
                                          uint32_t bi) {
    return ax < bx || (ax == bx && (ag < bg || (ag == bg && (al < bl || (al == bl && ai < bi)))));
}

// cnt[row_off + j]: entries of row first_row + j; eoff: their exclusive scan
// (row + 1 values: eoff[rows] = the total); fge[row_off + j]: the first sorted
// edge with YMin >= first_row + j (j <= rows).
__global__ void __launch_bounds__(kSlotMaxThreads) k_pr_hist(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                            const PrObj *__restrict__ pro,
                                                            const uint32_t *__restrict__ escan,
                                                            const uint32_t *__restrict__ total0p,
                                                            const ObjEdge *__restrict__ work, PrRow *__restrict__ prrow,
                                                            uint32_t *__restrict__ cnt, uint32_t *__restrict__ eoff,
                                                            uint32_t *__restrict__ fge, uint32_t *__restrict__ prstat) {
    __shared__ int32_t h[kMaxactRows + 1];
    __shared__ BlockRed R;
    const PrObj P = pro[blockIdx.x];
    const ObjDesc od = objs[P.o];
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const ObjEdge *E = work + e0;
    const int tid = threadIdx.x, NT = blockDim.x;
    int32_t mr = INT32_MIN;
    for (uint32_t i = tid; i < n; i += NT) mr = max(mr, E[i].YMax);
    const int32_t MaxY = min(min(blk_max(R, mr), fp.H), fp.row1), FirstRow = n ? E[0].YMin : 0;
    const int Rn = (int)P.rows;
    if (n == 0 || (int64_t)MaxY - FirstRow != (int64_t)Rn || Rn + 1 > kMaxactRows) {  // (never: k_obj_maxact sized it)
        if (tid == 0) prstat[P.o] = kPrFailed;
        return;
    }
    for (int q = tid; q <= Rn; q += NT) h[q] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < n; i += NT) {  // active on rows [YMin, min(YMax, MaxY))
        const int32_t y0 = E[i].YMin, y1 = min(E[i].YMax, MaxY);
        // the first edge of rows (YMin[i - 1], YMin[i]] (sorted by YMin)
        const int32_t lo = i ? E[i - 1].YMin : FirstRow - 1, hi = min(y0, MaxY);
        for (int32_t r = max(lo + 1, FirstRow); r <= hi; ++r) fge[P.row_off + (uint32_t)(r - FirstRow)] = i;
        if (i + 1 == n)
            for (int32_t r = max(y0 + 1, FirstRow); r <= MaxY; ++r) fge[P.row_off + (uint32_t)(r - FirstRow)] = n;
        if (y0 >= y1) continue;
        atomicAdd(&h[y0 - FirstRow], 1);
        atomicAdd(&h[y1 - FirstRow], -1);
    }
    __syncthreads();
    int32_t carry = 0, carry_e = 0, odd = 0;
    for (int b0 = 0; b0 < Rn; b0 += NT) {
        const int q = b0 + tid;
        const int32_t v = q < Rn ? h[q] : 0;
        int32_t tot;
        const int32_t m = carry + blk_excl_sum(R, v, tot) + v;  // entries of row q
        const int32_t mm = q < Rn ? m : 0;
        int32_t tot_e;
        const int32_t ex = blk_excl_sum(R, mm, tot_e);
        if (q < Rn) {
            cnt[P.row_off + q] = (uint32_t)m;
            eoff[P.row_off + q] = (uint32_t)(carry_e + ex);
            odd |= m & 1;
        }
        carry += tot;
        carry_e += tot_e;
    }
    odd = blk_max(R, odd);
    if (tid == 0) {
        eoff[P.row_off + Rn] = (uint32_t)carry_e;
        prrow[blockIdx.x] = PrRow{FirstRow, MaxY};
        prstat[P.o] = odd ? kPrFailed : kPrDone;  // every row pairs all its entries
    }
}

// Each edge's state at its chunks' first rows (stepped every row: every
// entry is paired every row, k_pr_hist), into the chunk's entry block at
// ent_off + j * most, in arrival order (k_pr_start sorts them).
template <int M>
__device__ __forceinline__ void pr_fill_edge(ObjEdge e, int32_t r1, uint32_t idx, const PrObj &P, int32_t first_row,
                                             uint32_t *__restrict__ ccur, float4 *__restrict__ key,
                                             ObjEdge *__restrict__ est) {
    for (int32_t r = e.YMin; r < r1; ++r) {
        const int32_t j = r - first_row;
        if (j % kPrChunk == 0) {
            const uint32_t c = (uint32_t)(j / kPrChunk);
            const uint32_t at = atomicAdd(&ccur[P.chunk_off + c], 1u);
            if (at < P.most) {  // (always: most bounds every row's list)
                const uint32_t g = P.ent_off + c * P.most + at;
                key[g] = make_float4(e.X, e.G, __int_as_float(e.Left), __uint_as_float(idx));
                ObjEdge s = e;
                s.Next = (int32_t)idx;
                est[g] = s;
            }
        }
        obj_step<M>(e);  // 3811-3829
    }
}
__global__ void k_pr_fill(FrameParams fp, const ObjDesc *__restrict__ objs, const PrObj *__restrict__ pro,
                          const PrRow *__restrict__ prrow, const uint32_t *__restrict__ escan,
                          const uint32_t *__restrict__ total0p, const ObjEdge *__restrict__ work,
                          uint32_t *__restrict__ ccur, float4 *__restrict__ key, ObjEdge *__restrict__ est,
                          const uint32_t *__restrict__ prstat) {
    const PrObj P = pro[blockIdx.y];
    if (prstat[P.o] != kPrDone) return;
    const ObjDesc od = objs[P.o];
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PrRow pr = prrow[blockIdx.y];
    const ObjEdge e = work[e0 + i];
    const int32_t r1 = min(e.YMax, pr.max_y);
    if (e.YMin >= r1) return;
    switch (fp.draws[od.draw].mode) {
#define PRK_PR_FILL(MM)                                                                  \
    case MM:                                                                             \
        pr_fill_edge<MM>(e, r1, i, P, pr.first_row, ccur, key, est);                     \
        break;
        PRK_PR_FILL(MODE_AVX)
        PRK_PR_FILL(MODE_SC_GOURAUD)
        PRK_PR_FILL(MODE_SC_GOURAUD_TEX)
        PRK_PR_FILL(MODE_SC_PHONG)
        PRK_PR_FILL(MODE_SC_PHONG_TEX)
#undef PRK_PR_FILL
        default: break;
    }
}

// The object of chunk c of the pass (the last with chunk_off <= c).
__device__ __forceinline__ uint32_t pr_obj_of_chunk(const PrObj *__restrict__ pro, uint32_t npr, uint32_t c) {
    uint32_t lo = 0, hi = npr;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pro[mid].chunk_off <= c) lo = mid; else hi = mid;
    }
    return lo;
}

// The canonical list of every chunk's first row: its entries ranked by
// (X, Gradient, Left, MergeSort index), their states (est, arrival order)
// into sst in list order.
constexpr int kPrStartThreads = 256;
__global__ void __launch_bounds__(kPrStartThreads) k_pr_start(const PrObj *__restrict__ pro, uint32_t npr,
                                                              const uint32_t *__restrict__ ccur,
                                                              const float4 *__restrict__ key,
                                                              const ObjEdge *__restrict__ est,
                                                              ObjEdge *__restrict__ sst, uint32_t *__restrict__ prstat) {
    __shared__ float sx[kPrMaxM], sg[kPrMaxM];
    __shared__ int32_t sl[kPrMaxM];
    __shared__ uint32_t si[kPrMaxM];
    __shared__ uint32_t st0;
    const uint32_t c = blockIdx.x;
    const PrObj P = pro[pr_obj_of_chunk(pro, npr, c)];
    const int tid = threadIdx.x;
    if (tid == 0) st0 = prstat[P.o];
    __syncthreads();
    if (st0 != kPrDone) return;
    const uint32_t j = c - P.chunk_off;
    const int m = (int)ccur[c];
    if (m > (int)P.most || m > kPrMaxM) {  // (never: most bounds every row's list)
        if (tid == 0) atomicMax(&prstat[P.o], kPrFailed);
        return;
    }
    const uint32_t g0 = P.ent_off + j * P.most;
    bool bad = false;
    for (int q = tid; q < m; q += kPrStartThreads) {
        const float4 k = key[g0 + q];
        sx[q] = k.x;
        sg[q] = k.y;
        sl[q] = __float_as_int(k.z);
        si[q] = __float_as_uint(k.w);
        bad |= k.x != k.x || k.y != k.y;  // a NaN key: no canonical order (the walk takes the object)
    }
    __syncthreads();
    for (int q = tid; q < m; q += kPrStartThreads) {
        const float x = sx[q], g = sg[q];
        const int32_t l = sl[q];
        const uint32_t i = si[q];
        int rank = 0;
        for (int p = 0; p < m; ++p) rank += pr_key_lt(sx[p], sg[p], sl[p], si[p], x, g, l, i) ? 1 : 0;
        sst[g0 + rank] = est[g0 + q];
    }
    if (__any(bad) && (tid & 63) == 0) atomicMax(&prstat[P.o], kPrFailed);
}

// walk_object_block over the rows [r0, r1) of an object, from the list
// start[0, m0) at row r0 (states at r0, their sorted edge index in Next; the
// row's insertion and expiry done); its spans from row re >= r0 on (the rows
// before: a warm-up, walked and stepped but not emitted), from slot base +
// emitted0.  sidx: the list at re (its sorted edge indices) goes to
// sidx[] / *s_m.  r1 < MaxY: the list after r1's insertion and expiry goes to
// end[] / *end_m, and the return value says whether its edges are
// cmp[0, mc) in order (cmp null: false).  Every thread returns the same.
template <int M>
__device__ bool walk_chunk(const FrameParams &fp, const ObjDesc &od, const ObjEdge *__restrict__ E, uint32_t n,
                           int32_t MaxY, uint32_t base, uint32_t bound, const SlotLds &S, BlockRed &R, uint32_t cap,
                           int32_t r0, int32_t re, int32_t r1, uint32_t ins0, const ObjEdge *__restrict__ start, int m0,
                           uint32_t emitted0, uint32_t *__restrict__ sidx, uint32_t *__restrict__ s_m,
                           const uint32_t *__restrict__ cmp, int mc, ObjEdge *__restrict__ end,
                           uint32_t *__restrict__ end_m, PairRaw *__restrict__ raw, SpanPos *__restrict__ pos,
                           uint32_t *__restrict__ span_tri, uint32_t *__restrict__ err) {
    constexpr bool kScalar = M != MODE_AVX;
    const int tid = threadIdx.x;
    const uint32_t NT = blockDim.x;
    const int32_t RowLo = kScalar ? fp.row0 - 1 : fp.row0;
    // the start list in slots [0, m0), the free slots above
    for (int q = tid; q < m0; q += (int)NT) {
        S.st[q] = start[q];
        S.idx[q] = q;
    }
    for (uint32_t q = tid; q + m0 < cap; q += NT) S.fs[q] = (int32_t)(q + m0);
    int top = (int)cap - m0;
    int m = m0;
    uint32_t ins = ins0;  // the first sorted edge with YMin > r0
    uint32_t wb = ins;
    PRK_WIN(wa);
    PRK_WIN_LOAD(wa, E, wb + (uint32_t)tid, n);
    PRK_WIN_WAIT();
    PRK_WIN_LAUNDER(wa);
    uint32_t emitted = emitted0;
    __syncthreads();
    for (int32_t Row = r0;; ++Row) {
        if (Row != r0) {
            if (Row >= MaxY) break;  // (the last chunk: no list after it)
            // insertion (3654-3713), as walk_object_block
            for (;;) {
                if (ins == wb + NT) {
                    wb += NT;
                    PRK_WIN_LOAD(wa, E, wb + tid, n);
                    PRK_WIN_WAIT();
                    PRK_WIN_LAUNDER(wa);
                }
                const float wx = wa0.x, wg = wa0.y;
                const int32_t wymin = __float_as_int(wa4.x), wl = __float_as_int(wa4.z);
                const int rel = tid - (int)(ins - wb);
                const bool eqr = rel >= 0 && wymin == Row;
                int32_t lt, k, nanc;
                blk_sum3(R, (rel >= 0 && wymin < Row) ? 1 : 0, eqr ? 1 : 0, (eqr && (wx != wx || wg != wg)) ? 1 : 0,
                         lt, k, nanc);
                if (lt) {
                    ins += (uint32_t)lt;
                    continue;
                }
                if (k == 0) break;
                if (k > top) {  // (never: cap >= the most listed edges)
                    if (tid == 0) atomicOr(err, 1u);
                    return false;
                }
                if (rel >= 0 && rel < k) {
                    const int32_t slot = S.fs[top - 1 - rel];
                    PRK_WIN_STORE(&S.st[slot], wa);
                    S.st[slot].Next = (int32_t)(ins + (uint32_t)rel);  // (its sorted index)
                    S.nkx[rel] = wx;
                    S.nkg[rel] = wg;
                    S.nkl[rel] = wl;
                    S.nks[rel] = slot;
                }
                top -= k;
                __syncthreads();
                if (k <= 2 || nanc) {
                    for (int t = 0; t < k; ++t)
                        insert_one_b(S, R, m, LKey{S.nkx[t], S.nkg[t], S.nkl[t]}, S.nks[t]);
                } else {
                    insert_batch_b(S, R, m, k);
                }
                ins += (uint32_t)k;
                if (ins < wb + NT) break;
            }
            {  // expiry 3715-3749
                int32_t e = 0;
                bool keep = false;
                if (tid < m) {
                    e = S.idx[tid];
                    keep = !(S.st[e].YMax <= Row);
                }
                const bool gone = tid < m && !keep;
                int32_t kp, gp, kt, gt;
                blk_excl_sum2(R, keep ? 1 : 0, gone ? 1 : 0, kp, gp, kt, gt);
                if (keep) S.idx[kp] = e;
                if (gone) S.fs[top + gp] = e;
                m = kt;
                top += gt;
                __syncthreads();
            }
        }
        if (Row >= r1) break;
        if (Row == re && sidx) {  // the list where the spans begin
            for (int q = tid; q < m; q += (int)NT) sidx[q] = (uint32_t)S.st[S.idx[q]].Next;
            if (tid == 0) *s_m = (uint32_t)m;
        }
        if (m == 0) {  // nothing happens on the rows before the next insertion (or re, r1): go there
            const int32_t nx = ins < n ? E[ins].YMin : INT32_MAX;
            Row = max(Row, min(nx, Row < re ? re : r1) - 1);
            continue;
        }
        const int P = m / 2;  // pairing 3751-3869, as walk_object_block
        const bool valid = tid < P;
        const bool emit = Row >= RowLo && Row >= re;
        int32_t i0 = 0, i1 = 0;
        float x0 = 0.0f, x1 = 0.0f;
        if (valid) {
            i0 = S.idx[2 * tid];
            i1 = S.idx[2 * tid + 1];
            const uint32_t j = emitted + (uint32_t)tid;
            const bool w = emit && j < bound;
            if (emit && j >= bound) atomicOr(err, 2u);
            const uint32_t at = base + j;
            ObjEdge a = S.st[i0];
            if (w) {
                raw[at].l0 = make_float4(a.X, a.Z, a.W, a.U);
                raw[at].l1 = make_float4(a.V, a.N0, a.N1, a.N2);
                raw[at].l2 = make_float4(a.C0, a.C1, a.C2, a.C3);
            }
            obj_step<M>(a);
            S.st[i0] = a;
            x0 = a.X;
            ObjEdge b = S.st[i1];
            if (w) {
                raw[at].r0 = make_float4(b.X, b.Z, b.W, b.U);
                raw[at].r1 = make_float4(b.V, b.N0, b.N1, b.N2);
                raw[at].r2 = make_float4(b.C0, b.C1, b.C2, b.C3);
                pos[at] = SpanPos{Row, (int32_t)od.draw, 0, SPAN_RAW};
                span_tri[at] = od.g0;
            }
            obj_step<M>(b);
            S.st[i1] = b;
            x1 = b.X;
            if (x0 > x1) {
                const int32_t t = i0; i0 = i1; i1 = t;
                const float f = x0; x0 = x1; x1 = f;
            }
            S.nb[tid] = i0;
            S.bk[tid] = __float_as_int(x0);
            S.aux[tid] = i1;
            S.bk2[tid] = __float_as_int(x1);
        }
        __syncthreads();
        if (valid) {
            const bool sw = tid >= 1 && __int_as_float(S.bk2[tid - 1]) > x0;
            const bool swn = tid + 1 < P && x1 > __int_as_float(S.bk[tid + 1]);
            const int32_t nf = sw ? S.aux[tid - 1] : i0, ns = swn ? S.nb[tid + 1] : i1;
            i0 = nf;
            i1 = ns;
        }
        __syncthreads();
        if (valid) {
            S.idx[2 * tid] = i0;
            S.idx[2 * tid + 1] = i1;
        }
        if (emit) emitted += (uint32_t)P;
        __syncthreads();
    }
    if (r1 >= MaxY) return true;
    // the list at r1: out, and against cmp
    bool same = cmp != nullptr && m == mc;
    for (int q = tid; q < m; q += (int)NT) {
        const ObjEdge &e = S.st[S.idx[q]];
        end[q] = e;
        if (cmp && q < mc) same = same && (uint32_t)e.Next == cmp[q];
    }
    if (tid == 0) *end_m = (uint32_t)m;
    return blk_max(R, same ? 0 : 1) == 0;
}

// Chunk j of the objects of one mode (pro[pi], pi in group [0, ngroup)):
// grid (chunks of the group's longest object, ngroup).  Chunk j > 0 starts
// one chunk early, from the sorted list of chunk j - 1's first row, and
// walks those rows as a warm-up (the list's order converges on the true one
// as entries expire and neighbours swap), then its own rows; its list at its
// first row goes to sidx (k_pr_cmp compares it with chunk j - 1's end).
template <int M>
__global__ void __launch_bounds__(kSlotMaxThreads) k_pr_chunk(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                            const PrObj *__restrict__ pro, const uint32_t *__restrict__ grp,
                                                            uint32_t cap, const PrRow *__restrict__ prrow,
                                                            const uint32_t *__restrict__ cnt,
                                                            const uint32_t *__restrict__ eoff,
                                                            const uint32_t *__restrict__ fge,
                                                            const uint32_t *__restrict__ escan,
                                                            const uint32_t *__restrict__ total0p,
                                                            const ObjEdge *__restrict__ work,
                                                            const unsigned long long *__restrict__ soff,
                                                            const ObjEdge *__restrict__ sst, ObjEdge *__restrict__ eend,
                                                            uint32_t *__restrict__ eend_m, uint32_t *__restrict__ sidx,
                                                            uint32_t *__restrict__ s_m,
                                                            const uint32_t *__restrict__ prstat, PairRaw *__restrict__ raw,
                                                            SpanPos *__restrict__ pos, uint32_t *__restrict__ span_tri,
                                                            uint32_t *__restrict__ err, uint32_t warmup) {
    extern __shared__ int32_t lds_list[];
    __shared__ BlockRed R;
    const uint32_t pi = grp[blockIdx.y];
    const PrObj P = pro[pi];
    const uint32_t j = blockIdx.x;
    if (j >= pr_chunks(P) || prstat[P.o] != kPrDone) return;  // (prstat is final here: k_pr_start ran)
    const ObjDesc od = objs[P.o];
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const ObjEdge *E = work + e0;
    const PrRow pr = prrow[pi];
    const int32_t re = pr.first_row + (int32_t)(j * kPrChunk), r1 = min(re + kPrChunk, pr.max_y);
    const uint32_t js = j && warmup ? j - 1 : j;  // the chunk whose first row it starts from
    const int32_t r0 = pr.first_row + (int32_t)(js * kPrChunk);
    const uint32_t jr0 = js * kPrChunk, jre = j * kPrChunk;
    const int32_t RowLo = fp.draws[od.draw].mode != MODE_AVX ? fp.row0 - 1 : fp.row0;
    const uint32_t jlo = (uint32_t)min(max(0, RowLo - pr.first_row), (int32_t)P.rows);
    const uint32_t emitted0 = (eoff[P.row_off + max(jre, jlo)] - eoff[P.row_off + jlo]) / 2;
    const uint32_t base = (uint32_t)soff[P.o], bound = (uint32_t)(soff[P.o + 1] - soff[P.o]);
    SlotLds S;
    S.carve(lds_list, cap, blockDim.x);
    const uint32_t c = P.chunk_off + j;
    const uint32_t gs = P.ent_off + js * P.most, ge = P.ent_off + j * P.most, g1 = ge + P.most;
    const bool last = r1 >= pr.max_y;
    (void)walk_chunk<M>(fp, od, E, n, pr.max_y, base, bound, S, R, cap, r0, re, r1, fge[P.row_off + jr0 + 1],
                        sst + gs, (int)cnt[P.row_off + jr0], emitted0, sidx + ge, s_m + c, nullptr, 0,
                        last ? nullptr : eend + g1, eend_m + c, raw, pos, span_tri, err);
}

// match[c] = chunk c's end list (eend) is chunk c + 1's list at its first
// row (sidx): then chunk c + 1 walked its rows from the true list whenever
// chunk c did.  Workgroup per chunk.
__global__ void k_pr_cmp(const PrObj *__restrict__ pro, uint32_t npr, const uint32_t *__restrict__ prstat,
                         const ObjEdge *__restrict__ eend, const uint32_t *__restrict__ eend_m,
                         const uint32_t *__restrict__ sidx, const uint32_t *__restrict__ s_m,
                         uint32_t *__restrict__ match) {
    __shared__ int32_t diff;
    const uint32_t c = blockIdx.x;
    const PrObj P = pro[pr_obj_of_chunk(pro, npr, c)];
    const uint32_t j = c - P.chunk_off;
    if (j + 1 >= pr_chunks(P) || prstat[P.o] != kPrDone) return;
    if (threadIdx.x == 0) diff = eend_m[c] != s_m[c + 1];
    __syncthreads();
    const uint32_t g1 = P.ent_off + (j + 1) * P.most, m = eend_m[c];
    if (!diff)
        for (uint32_t q = threadIdx.x; q < m; q += blockDim.x)
            if ((uint32_t)eend[g1 + q].Next != sidx[g1 + q]) diff = 1;
    __syncthreads();
    if (threadIdx.x == 0) match[c] = diff ? 0u : 1u;
}

// Per object of the group: the chunks whose start list was not the true one,
// walked again in order from their predecessor's true end list.
template <int M>
__global__ void __launch_bounds__(kSlotMaxThreads) k_pr_fix(FrameParams fp, const ObjDesc *__restrict__ objs,
                                                          const PrObj *__restrict__ pro, const uint32_t *__restrict__ grp,
                                                          uint32_t cap, const PrRow *__restrict__ prrow,
                                                          const uint32_t *__restrict__ cnt,
                                                          const uint32_t *__restrict__ eoff,
                                                          const uint32_t *__restrict__ fge,
                                                          const uint32_t *__restrict__ escan,
                                                          const uint32_t *__restrict__ total0p,
                                                          const ObjEdge *__restrict__ work,
                                                          const unsigned long long *__restrict__ soff,
                                                          ObjEdge *__restrict__ eend, uint32_t *__restrict__ eend_m,
                                                          const uint32_t *__restrict__ sidx,
                                                          const uint32_t *__restrict__ s_m,
                                                          const uint32_t *__restrict__ match,
                                                          const uint32_t *__restrict__ prstat,
                                                          PairRaw *__restrict__ raw, SpanPos *__restrict__ pos,
                                                          uint32_t *__restrict__ span_tri, uint32_t *__restrict__ err) {
    extern __shared__ int32_t lds_list[];
    __shared__ BlockRed R;
    const uint32_t pi = grp[blockIdx.x];
    const PrObj P = pro[pi];
    if (prstat[P.o] != kPrDone) return;
    const ObjDesc od = objs[P.o];
    uint32_t e0, n;
    obj_range(od, escan, *total0p, e0, n);
    const ObjEdge *E = work + e0;
    const PrRow pr = prrow[pi];
    const int32_t RowLo = fp.draws[od.draw].mode != MODE_AVX ? fp.row0 - 1 : fp.row0;
    const uint32_t jlo = (uint32_t)min(max(0, RowLo - pr.first_row), (int32_t)P.rows);
    const uint32_t base = (uint32_t)soff[P.o], bound = (uint32_t)(soff[P.o + 1] - soff[P.o]);
    SlotLds S;
    S.carve(lds_list, cap, blockDim.x);
    const uint32_t nch = pr_chunks(P);
    bool prev_true = true;  // chunk j walked its rows from the true list (chunk 0: from the first row)
    for (uint32_t j = 0; j < nch; ++j) {
        const uint32_t c = P.chunk_off + j;
        if (prev_true) {  // its speculative walk started from the true list: keep it
            prev_true = match[c] != 0;
            continue;
        }
        // walk it again from the true list: chunk j - 1's end (eend at its entry block)
        if (threadIdx.x == 0) atomicAdd(&err[3], 1u);  // (the pass's re-walked chunks)
        const int32_t r0 = pr.first_row + (int32_t)(j * kPrChunk), r1 = min(r0 + kPrChunk, pr.max_y);
        const uint32_t jr0 = j * kPrChunk, jr1 = (uint32_t)(r1 - pr.first_row);
        const uint32_t emitted0 = (eoff[P.row_off + max(jr0, jlo)] - eoff[P.row_off + jlo]) / 2;
        const uint32_t g0 = P.ent_off + j * P.most, g1 = g0 + P.most;
        const bool last = r1 >= pr.max_y;
        __syncthreads();  // (the previous walk's LDS and eend writes)
        prev_true = walk_chunk<M>(fp, od, E, n, pr.max_y, base, bound, S, R, cap, r0, r0, r1, fge[P.row_off + jr0 + 1],
                                  eend + g0, (int)eend_m[c - 1], emitted0, nullptr, nullptr,
                                  last ? nullptr : sidx + g1, last ? 0 : (int)s_m[c + 1],
                                  last ? nullptr : eend + g1, eend_m + c, raw, pos, span_tri, err);
        (void)jr1;
    }
}

// The walk's outcome: err[1] += objects done, err[2] += objects failed
// (err[3]: chunks walked again, k_pr_fix).
__global__ void k_pr_tally(const PrObj *__restrict__ pro, uint32_t npr, const uint32_t *__restrict__ prstat,
                           uint32_t *__restrict__ err) {
    uint32_t done = 0, failed = 0;
    for (uint32_t i = threadIdx.x; i < npr; i += blockDim.x) {
        const uint32_t st = prstat[pro[i].o];
        done += st == kPrDone;
        failed += st == kPrFailed;
    }
    if (done) atomicAdd(&err[1], done);
    if (failed) atomicAdd(&err[2], failed);
}

// The tiles of a span: those of its row its [minx, min(maxx, W)) crosses and,
// for a DrawModel span whose inclusive MaxX reached W, the column-0 tile of
// row + 1 that receives its one-past-the-row store (projekt.cpp:423-538).
struct SpanTiles {
    int ty, tx0, tx1;  // own row's tiles (tx0 > tx1: none)
    int oty;           // overflow tile row (-1: none, or already among the own tiles)
};
__device__ __forceinline__ SpanTiles span_tiles(const FrameParams &fp, const SpanPos &p) {
    SpanTiles t{0, 1, 0, -1};
    const int32_t xe = min(p.maxx, fp.W);
    if (p.row >= fp.row0 && p.row < fp.row1 && p.minx < xe) {
        t.ty = tile_row_of(fp, p.row - fp.row0);
        t.tx0 = p.minx >> fp.tile_w_log2;
        t.tx1 = (xe - 1) >> fp.tile_w_log2;
    }
    if ((p.flags & SPAN_SCALAR) && p.maxx > fp.W && p.row + 1 >= fp.row0 && p.row + 1 < fp.row1 &&
        p.row + 1 < fp.H) {
        const int oty = tile_row_of(fp, p.row + 1 - fp.row0);
        if (!(t.tx0 == 0 && t.tx0 <= t.tx1 && t.ty == oty)) t.oty = oty;
    }
    return t;
}

// Span -> tile bin entries by counting, no sort: pass 0 (PLACE false)
// counts every tile's entries into ctr, pass 1 puts span s at offs[tile] +
// its arrival rank (ctr zeroed again: the tiles' cursors).  The lanes of a
// wave that hit one tile take their ranks from one atomic (the spans of an
// object's consecutive rows mostly share a tile).  Within a tile the entries
// are in arrival order, not span order: k_span_vis keeps the 64-bit maximum
// of (z, span index) per pixel and the shading tests the winner's tag, so
// neither depends on it.
template <bool PLACE>
__global__ void k_span_tiles(FrameParams fp, const SpanPos *__restrict__ pos, uint32_t nspan,
                             uint32_t *__restrict__ ctr, const uint32_t *__restrict__ offs,
                             uint32_t *__restrict__ bins) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = (int)(threadIdx.x & 63);
    SpanTiles t{0, 1, 0, -1};
    if (s < nspan) t = span_tiles(fp, pos[s]);
    const int own = max(0, t.tx1 - t.tx0 + 1), cnt = own + (t.oty >= 0 ? 1 : 0);
    const int kmax = wave_max_i32(cnt);
    for (int k = 0; k < kmax; ++k) {
        const bool act = k < cnt;
        const uint32_t tile = !act ? 0u : (uint32_t)(k < own ? t.ty * fp.tiles_x + t.tx0 + k : t.oty * fp.tiles_x);
        // the wave's lanes grouped by tile (ballots only), then one atomic per
        // group, all groups' at once (their leads), and each lane's rank from
        // its lead's return (a per-group atomic-and-wait loop serialised the
        // returns: the placement pass took 2.3x the count pass)
        unsigned long long pending = __ballot(act);
        int lead_of = lane;
        uint32_t below = 0, gsize = 0;  // lanes of my group before me; (lead) my group's size
        while (pending) {
            const int lead = (int)__builtin_ctzll(pending);
            const uint32_t lt = (uint32_t)readlane_i((int32_t)tile, lead);
            const unsigned long long m = __ballot(act && tile == lt) & pending;
            if ((m >> lane) & 1ull) {
                lead_of = lead;
                below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            }
            if (lane == lead) gsize = (uint32_t)__popcll(m);
            pending &= ~m;
        }
        uint32_t b = 0;
        if (act && lane == lead_of) b = atomicAdd(&ctr[tile], gsize);
        if (PLACE) {
            b = (uint32_t)__shfl((int32_t)b, lead_of);
            if (act) bins[offs[tile] + b + below] = s;
        }
    }
}

}  // namespace prk

extern "C" {

// The pass's objects (ObjDesc) and kind-0 object tables from the host's runs.
hipError_t prk_obj_tables(const void *runs, uint32_t nruns, uint32_t nobj, uint32_t wave_tris, void *objs,
                          uint32_t *k0obj, uint32_t *k0tri0, hipStream_t s) {
    if (nobj == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_obj_tables, dim3((nobj + 255) / 256), dim3(256), 0, s,
                       reinterpret_cast<const prk::ObjRun *>(runs), nruns, nobj, wave_tris,
                       reinterpret_cast<prk::ObjDesc *>(objs), k0obj, k0tri0);
    return hipGetLastError();
}
// FillEdgeTable of the pass's object triangles: per-triangle edge and
// active-row counts (ntri + 1 values each, the last 0) ...
hipError_t prk_objtri_count(const prk::FrameParams *fp, const void *objs, const uint32_t *k0obj,
                            const uint32_t *k0tri0, uint32_t nk0, uint32_t ntri, uint32_t *ecnt,
                            unsigned long long *rcnt, hipStream_t s) {
    hipLaunchKernelGGL(prk::k_objtri_count, dim3((ntri + 1 + 255) / 256), dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::ObjDesc *>(objs), k0obj, k0tri0, nk0, ntri, ecnt, rcnt);
    return hipGetLastError();
}
// ... then the edges at their exclusive scan, with their MergeSort keys
// (keys: 3 * ntri slots, those past the visible edges all ones).
hipError_t prk_objtri_emit(const prk::FrameParams *fp, const void *objs, const uint32_t *k0obj,
                           const uint32_t *k0tri0, uint32_t nk0, uint32_t ntri, const uint32_t *escan,
                           uint32_t pbits, uint32_t ybits, int32_t ycap, void *edges, void *keys, uint32_t *vals,
                           int pad, hipStream_t s) {
    if (ntri == 0) return hipSuccess;
    if (pad) {  // (the radix sort reads every slot; k_obj_sort_local only the visible edges')
        const hipError_t e = hipMemsetAsync(keys, 0xFF, (size_t)3 * ntri * 8, s);
        if (e != hipSuccess) return e;
    }
    const prk::SortKeyBits kb{pbits, ybits, ycap};
    hipLaunchKernelGGL(prk::k_objtri_emit, dim3((ntri + 255) / 256), dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::ObjDesc *>(objs), k0obj, k0tri0, nk0, ntri, escan, kb,
                       reinterpret_cast<prk::ObjEdge *>(edges), reinterpret_cast<unsigned long long *>(keys), vals);
    return hipGetLastError();
}
// The walk's working copy (n slots: total0 triangle edges, then nk1 caller edges).
// (wy: null, or the triangle edges' (YMin, YMax) as int2, for prk_obj_seg)
hipError_t prk_obj_gather(const void *edges, const uint32_t *ord, const uint32_t *total0p, const void *edges_in,
                          const uint32_t *k1src, uint32_t nk1, void *work, uint32_t n, void *wy, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_obj_gather, dim3((n + 255) / 256), dim3(256), 0, s,
                       reinterpret_cast<const prk::ObjEdge *>(edges), ord, total0p,
                       reinterpret_cast<const prk::EdgeIn *>(edges_in), k1src, nk1,
                       reinterpret_cast<prk::ObjEdge *>(work), reinterpret_cast<int2 *>(wy));
    return hipGetLastError();
}

// MergeSort + gather of objects of at most 64 edges (k_obj_sort_local).
hipError_t prk_obj_sort_local(const void *objs, const uint32_t *k0obj, uint32_t nk0, const uint32_t *escan,
                              const void *keys, const void *edges, void *work, void *wy, uint32_t *err,
                              hipStream_t s) {
    if (nk0 == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_obj_sort_local, dim3((nk0 + 3) / 4), dim3(256), 0, s,
                       reinterpret_cast<const prk::ObjDesc *>(objs), k0obj, nk0, escan,
                       reinterpret_cast<const unsigned long long *>(keys),
                       reinterpret_cast<const prk::ObjEdge *>(edges), reinterpret_cast<prk::ObjEdge *>(work),
                       reinterpret_cast<int2 *>(wy), err);
    return hipGetLastError();
}
// Span slots per object (nobj + 1 values, the last 0; exclusive-scanned by
// the caller into each object's first slot).
hipError_t prk_obj_bound(const prk::FrameParams *fp, const void *objs, uint32_t nobj, const unsigned long long *rscan,
                         const void *edges_in, unsigned long long *bound, hipStream_t s) {
    hipLaunchKernelGGL(prk::k_obj_bound, dim3((nobj + 1 + 255) / 256), dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::ObjDesc *>(objs), nobj, rscan,
                       reinterpret_cast<const prk::EdgeIn *>(edges_in), bound);
    return hipGetLastError();
}
// The LDS capacity of the workgroup walk on the current device (listed edges;
// 0: every walk keeps its list in device memory): the largest of 1022, 510,
// 254 whose slot_lds_bytes the device grants as dynamic LDS.
uint32_t prk_obj_walk_lcap(void) {
    static std::atomic<int> cap[64];  // per device: 0 unknown, else cap + 1
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int c = cap[dev].load();
    if (c == 0) {
        c = 1;
        for (uint32_t k = prk::kSlotCapLds; k >= 254; k = (k + 2) / 2 - 2) {
            const size_t bytes = prk::slot_lds_bytes(k);
            const void *fn[prk::MODE_COUNT] = {
                reinterpret_cast<const void *>(&prk::k_obj_walk_wave<prk::MODE_AVX>),
                reinterpret_cast<const void *>(&prk::k_obj_walk_wave<prk::MODE_SC_GOURAUD>),
                reinterpret_cast<const void *>(&prk::k_obj_walk_wave<prk::MODE_SC_GOURAUD_TEX>),
                reinterpret_cast<const void *>(&prk::k_obj_walk_wave<prk::MODE_SC_PHONG>),
                reinterpret_cast<const void *>(&prk::k_obj_walk_wave<prk::MODE_SC_PHONG_TEX>)};
            const void *fc[2 * prk::MODE_COUNT] = {  // (the chunked walk's kernels: the same slot lists)
                reinterpret_cast<const void *>(&prk::k_pr_chunk<prk::MODE_AVX>),
                reinterpret_cast<const void *>(&prk::k_pr_chunk<prk::MODE_SC_GOURAUD>),
                reinterpret_cast<const void *>(&prk::k_pr_chunk<prk::MODE_SC_GOURAUD_TEX>),
                reinterpret_cast<const void *>(&prk::k_pr_chunk<prk::MODE_SC_PHONG>),
                reinterpret_cast<const void *>(&prk::k_pr_chunk<prk::MODE_SC_PHONG_TEX>),
                reinterpret_cast<const void *>(&prk::k_pr_fix<prk::MODE_AVX>),
                reinterpret_cast<const void *>(&prk::k_pr_fix<prk::MODE_SC_GOURAUD>),
                reinterpret_cast<const void *>(&prk::k_pr_fix<prk::MODE_SC_GOURAUD_TEX>),
                reinterpret_cast<const void *>(&prk::k_pr_fix<prk::MODE_SC_PHONG>),
                reinterpret_cast<const void *>(&prk::k_pr_fix<prk::MODE_SC_PHONG_TEX>)};
            bool ok = true;
            for (int mo = 0; mo < prk::MODE_COUNT && ok; ++mo)
                ok = hipFuncSetAttribute(fn[mo], hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess;
            for (int q = 0; q < 2 * prk::MODE_COUNT && ok; ++q)
                ok = hipFuncSetAttribute(fc[q], hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) == hipSuccess;
            if (ok) {
                c = (int)k + 1;
                break;
            }
            (void)hipGetLastError();
        }
        cap[dev].store(c);
    }
    return (uint32_t)(c - 1);
}
// The object walk: a thread per small object or caller edge list ...
// (segs: the small triangle objects' segments, prk_obj_seg, walked a thread
// each; null: a thread per object)
hipError_t prk_obj_walk(const prk::FrameParams *fp, const void *objs, uint32_t nobj, const uint32_t *escan,
                        const uint32_t *total0p, void *work, const unsigned long long *soff, void *recs, void *srecs,
                        void *pos, uint32_t *span_tri, const void *spans_in, uint32_t *err, int links,
                        const void *segs, const uint32_t *nsegp, uint32_t max_segs, hipStream_t s) {
    if (nobj == 0) return hipSuccess;
    const uint32_t segmented = segs ? 1u : 0u;
    if (segs && max_segs) {
        hipLaunchKernelGGL(prk::k_obj_walk_seg, dim3((max_segs + prk::kLinkThreads - 1) / prk::kLinkThreads),
                           dim3(prk::kLinkThreads), 0, s, *fp, reinterpret_cast<const prk::ObjDesc *>(objs),
                           reinterpret_cast<const prk::ObjSeg *>(segs), nsegp, escan, total0p,
                           reinterpret_cast<prk::ObjEdge *>(work), reinterpret_cast<prk::SpanRecG *>(recs),
                           reinterpret_cast<prk::ScSpanRecG *>(srecs), reinterpret_cast<prk::SpanPos *>(pos), span_tri,
                           err);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
#define PRK_OBJ_WALK_LAUNCH(LK)                                                                                    \
    hipLaunchKernelGGL(prk::k_obj_walk<LK>, dim3((nobj + prk::kLinkThreads - 1) / prk::kLinkThreads),              \
                       dim3(prk::kLinkThreads), 0, s, *fp, reinterpret_cast<const prk::ObjDesc *>(objs), nobj, escan, \
                       total0p, reinterpret_cast<prk::ObjEdge *>(work), soff,                                      \
                       reinterpret_cast<prk::SpanRecG *>(recs), reinterpret_cast<prk::ScSpanRecG *>(srecs),        \
                       reinterpret_cast<prk::SpanPos *>(pos), span_tri,                                            \
                       reinterpret_cast<const prk::SpanIn *>(spans_in), err, segmented)
    if (links && PRK_OBJ_LDS_LINKS) PRK_OBJ_WALK_LAUNCH(true);
    else PRK_OBJ_WALK_LAUNCH(false);
#undef PRK_OBJ_WALK_LAUNCH
    return hipGetLastError();
}
uint32_t prk_obj_link_cap(void) { return (uint32_t)prk::kLinkCap; }
// The small triangle objects' segments (k_obj_seg): counts (nobj + 1 values,
// the last 0) when segs is null, else the descriptors at segoff[o].
// With the descriptors it also marks each object's slots past its segments'
// row -1 (pos).
hipError_t prk_obj_seg(const prk::FrameParams *fp, const void *objs, uint32_t nobj, const uint32_t *escan,
                       const uint32_t *total0p, const void *wy, const unsigned long long *soff, uint32_t *segcnt,
                       const uint32_t *segoff, void *segs, void *pos, hipStream_t s) {
    const dim3 g((nobj + 1 + 255) / 256), b(256);
    const prk::ObjDesc *O = reinterpret_cast<const prk::ObjDesc *>(objs);
    const int2 *W = reinterpret_cast<const int2 *>(wy);
    if (!segs)
        hipLaunchKernelGGL(prk::k_obj_seg<false>, g, b, 0, s, *fp, O, nobj, escan, total0p, W, soff, segcnt, segoff,
                           nullptr, nullptr);
    else
        hipLaunchKernelGGL(prk::k_obj_seg<true>, g, b, 0, s, *fp, O, nobj, escan, total0p, W, soff, segcnt, segoff,
                           reinterpret_cast<prk::ObjSeg *>(segs), reinterpret_cast<prk::SpanPos *>(pos));
    return hipGetLastError();
}
// ... the most active entries of the large ones (big[0, nbig)) ...
// (most: 3 * nbig values, see k_obj_maxact)
hipError_t prk_obj_maxact(const prk::FrameParams *fp, const void *objs, const uint32_t *big, uint32_t nbig,
                          const uint32_t *escan, const uint32_t *total0p, const void *work, int32_t *most,
                          uint32_t huge_min, hipStream_t s) {
    if (nbig == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_obj_maxact, dim3(nbig), dim3(prk::kSlotMaxThreads), 0, s, *fp,
                       reinterpret_cast<const prk::ObjDesc *>(objs), big, nbig, escan, total0p,
                       reinterpret_cast<const prk::ObjEdge *>(work), most, huge_min);
    return hipGetLastError();
}
// ... and those of the huge object big[b] (3 * tris >= huge_min, at most
// `edges` edges) over many workgroups: scratch = (kMaxactRows + 2) ints + 3
// words (prk_maxact_huge_scratch bytes), zeroed here.
size_t prk_maxact_huge_scratch(void) { return (size_t)(prk::kMaxactRows + 2) * 4 + 3 * 8; }
hipError_t prk_obj_maxact_huge(const prk::FrameParams *fp, const void *objs, const uint32_t *big, uint32_t b,
                               uint32_t nbig, uint32_t edges, const uint32_t *escan, const uint32_t *total0p,
                               const void *work, int32_t *most, void *scratch, hipStream_t s) {
    if (edges == 0) return hipSuccess;
    const size_t hb = (size_t)(prk::kMaxactRows + 2) * 4;
    hipError_t e = hipMemsetAsync(scratch, 0, prk_maxact_huge_scratch(), s);
    if (e != hipSuccess) return e;
    int32_t *hist = static_cast<int32_t *>(scratch);
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(static_cast<char *>(scratch) + hb);
    const prk::ObjDesc *O = reinterpret_cast<const prk::ObjDesc *>(objs);
    const prk::ObjEdge *W = reinterpret_cast<const prk::ObjEdge *>(work);
    hipLaunchKernelGGL(prk::k_maxact_huge_part, dim3((edges + prk::kMaxactChunk - 1) / prk::kMaxactChunk),
                       dim3(prk::kSlotMaxThreads), 0, s, *fp, O, big, b, escan, total0p, W, hist, acc);
    hipLaunchKernelGGL(prk::k_maxact_huge_fin, dim3(1), dim3(prk::kSlotMaxThreads), 0, s, *fp, O, big, b, nbig,
                       escan, total0p, W, hist, acc, most);
    return hipGetLastError();
}
// ... and a workgroup per large object of mode `mode` (big[0, nbig)): lcap > 0
// (<= prk_obj_walk_lcap()), slot_threads(lcap) threads, the list in LDS; lcap
// == 0, one wave, the list in the pool at big_off, big_cap edges.  Spans go to
// slots soff[o] + k.  err: bit 0 a pool slice smaller than its object, bit 1
// an object emitted past its bound (neither can happen).
uint32_t prk_obj_walk_threads(uint32_t lcap) { return lcap ? prk::slot_threads(lcap) : 64u; }
hipError_t prk_obj_walk_group(const prk::FrameParams *fp, int32_t mode, uint32_t lcap, const void *objs,
                              const uint32_t *big, const unsigned long long *big_off, const uint32_t *big_cap,
                              uint32_t nbig, int32_t *pool, const uint32_t *escan, const uint32_t *total0p,
                              void *work, const unsigned long long *soff, void *recs, void *srecs, void *raw,
                              void *pos, uint32_t *span_tri, uint32_t *err, const uint32_t *prstat,
                              hipStream_t s) {
    if (nbig == 0) return hipSuccess;
    const size_t bytes = lcap ? prk::slot_lds_bytes(lcap) : 0;
    const uint32_t nt = prk_obj_walk_threads(lcap);
    switch (mode) {
#define PRK_WALK_WAVE(MM)                                                                                           \
    case MM:                                                                                                        \
        hipLaunchKernelGGL(prk::k_obj_walk_wave<MM>, dim3(nbig), dim3(nt), bytes, s, *fp,                          \
                           reinterpret_cast<const prk::ObjDesc *>(objs), big, big_off, big_cap, pool, lcap, escan,  \
                           total0p, reinterpret_cast<prk::ObjEdge *>(work), soff,                                   \
                           reinterpret_cast<prk::SpanRecG *>(recs), reinterpret_cast<prk::ScSpanRecG *>(srecs),     \
                           reinterpret_cast<prk::PairRaw *>(raw), reinterpret_cast<prk::SpanPos *>(pos), span_tri,  \
                           err, prstat);                                                                            \
        break;
        PRK_WALK_WAVE(prk::MODE_AVX)
        PRK_WALK_WAVE(prk::MODE_SC_GOURAUD)
        PRK_WALK_WAVE(prk::MODE_SC_GOURAUD_TEX)
        PRK_WALK_WAVE(prk::MODE_SC_PHONG)
        PRK_WALK_WAVE(prk::MODE_SC_PHONG_TEX)
#undef PRK_WALK_WAVE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
// The huge-object walk (lds: k_obj_walk_lds, else k_obj_walk_big) of the
// objects big[0, nbig) of mode `mode`: their pool slices at big_off (prk_big_slice_ints(big_cap, rows,
// ents) ints each; big_meta: (rows, ents) per object, k_obj_maxact's), then
// every pair set up from a replay of its edges (k_big_replay, grid (max_rows,
// nbig)) into PairRaw slots soff[o] + j (k_span_finish sets the spans up).
uint32_t prk_big_max_entries(void) { return prk::kBigMaxM; }
uint64_t prk_big_slice_ints(uint32_t cap, uint32_t rows, uint32_t ents) { return prk::big_slice_ints(cap, rows, ents); }
uint32_t prk_big_lds_cap(void) { return (uint32_t)prk::kLdsCap; }
hipError_t prk_big_walk(const prk::FrameParams *fp, int32_t mode, int lds, const void *objs, const uint32_t *big,
                        const unsigned long long *big_off, const uint32_t *big_cap, const uint32_t *big_meta,
                        uint32_t nbig, uint32_t max_rows, int32_t *pool, const uint32_t *escan,
                        const uint32_t *total0p, const void *work, const unsigned long long *soff, void *raw,
                        void *pos, uint32_t *span_tri, uint32_t *err, const uint32_t *prstat, hipStream_t s) {
    if (nbig == 0) return hipSuccess;
    if (nbig > 65535) return hipErrorInvalidValue;
    const prk::ObjDesc *O = reinterpret_cast<const prk::ObjDesc *>(objs);
    const prk::ObjEdge *W = reinterpret_cast<const prk::ObjEdge *>(work);
    if (lds)
        hipLaunchKernelGGL(prk::k_obj_walk_lds, dim3(nbig), dim3(prk::kBigThreads), 0, s, *fp, O, big, big_off,
                           big_cap, big_meta, pool, escan, total0p, W, soff, err, prstat);
    else
        hipLaunchKernelGGL(prk::k_obj_walk_big, dim3(nbig), dim3(prk::kBigThreads), 0, s, *fp, O, big, big_off,
                           big_cap, big_meta, pool, escan, total0p, W, soff, err, prstat);
    if (max_rows == 0) return hipGetLastError();
    const dim3 g(max_rows, nbig), b(256);
    prk::PairRaw *R = reinterpret_cast<prk::PairRaw *>(raw);
    prk::SpanPos *P = reinterpret_cast<prk::SpanPos *>(pos);
    switch (mode) {
#define PRK_BIG_REPLAY(MM)                                                                                      \
    case MM:                                                                                                    \
        hipLaunchKernelGGL(prk::k_big_replay<MM>, g, b, 0, s, *fp, O, big, big_off, big_cap, big_meta, pool,    \
                           escan, total0p, W, soff, R, P, span_tri, prstat);                                    \
        break;
        PRK_BIG_REPLAY(prk::MODE_AVX)
        PRK_BIG_REPLAY(prk::MODE_SC_GOURAUD)
        PRK_BIG_REPLAY(prk::MODE_SC_GOURAUD_TEX)
        PRK_BIG_REPLAY(prk::MODE_SC_PHONG)
        PRK_BIG_REPLAY(prk::MODE_SC_PHONG_TEX)
#undef PRK_BIG_REPLAY
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
// The chunked walk of large objects (prk_spans.hip k_pr_*), in three calls:
// begin (every object: rows, chunk starts, canonical lists), a group call per
// (mode, LDS capacity) of objects (grp: indices into the PrObj table; the
// speculative chunk walks, then the walks again of chunks whose start was not
// the true list), end (the outcome into err[1], err[2]).
hipError_t prk_pr_walk_begin(const prk::FrameParams *fp, const prk::PrWalkArgs *a, hipStream_t s) {
    if (a->npr == 0) return hipSuccess;
    if (a->npr > 65535 || a->max_edges == 0) return hipErrorInvalidValue;
    const prk::PrObj *P = reinterpret_cast<const prk::PrObj *>(a->pro);
    prk::PrRow *PR = reinterpret_cast<prk::PrRow *>(a->prrow);
    const prk::ObjDesc *O = reinterpret_cast<const prk::ObjDesc *>(a->objs);
    const prk::ObjEdge *W = reinterpret_cast<const prk::ObjEdge *>(a->work);
    hipLaunchKernelGGL(prk::k_pr_hist, dim3(a->npr), dim3(prk::kSlotMaxThreads), 0, s, *fp, O, P, a->escan,
                       a->total0p, W, PR, a->cnt, a->eoff, a->fge, a->prstat);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemsetAsync(a->ccur, 0, (size_t)a->nchunks * 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(prk::k_pr_fill, dim3((a->max_edges + 255) / 256, a->npr), dim3(256), 0, s, *fp, O, P, PR,
                       a->escan, a->total0p, W, a->ccur, reinterpret_cast<float4 *>(a->key),
                       reinterpret_cast<prk::ObjEdge *>(a->est), a->prstat);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(prk::k_pr_start, dim3(a->nchunks), dim3(prk::kPrStartThreads), 0, s, P, a->npr, a->ccur,
                       reinterpret_cast<const float4 *>(a->key), reinterpret_cast<const prk::ObjEdge *>(a->est),
                       reinterpret_cast<prk::ObjEdge *>(a->sst), a->prstat);
    return hipGetLastError();
}
hipError_t prk_pr_walk_group(const prk::FrameParams *fp, const prk::PrWalkArgs *a, int32_t mode, uint32_t cap,
                             const uint32_t *grp, uint32_t ngroup, uint32_t max_chunks, hipStream_t s) {
    if (ngroup == 0 || max_chunks == 0) return hipSuccess;
    if (cap == 0 || ngroup > 65535) return hipErrorInvalidValue;
    const size_t bytes = prk::slot_lds_bytes(cap);
    const uint32_t nt = prk::slot_threads(cap);
    const prk::PrObj *P = reinterpret_cast<const prk::PrObj *>(a->pro);
    const prk::PrRow *PR = reinterpret_cast<const prk::PrRow *>(a->prrow);
    const prk::ObjDesc *O = reinterpret_cast<const prk::ObjDesc *>(a->objs);
    const prk::ObjEdge *W = reinterpret_cast<const prk::ObjEdge *>(a->work);
    const prk::ObjEdge *SST = reinterpret_cast<const prk::ObjEdge *>(a->sst);
    prk::ObjEdge *EE = reinterpret_cast<prk::ObjEdge *>(a->eend);
    prk::PairRaw *RAW = reinterpret_cast<prk::PairRaw *>(a->raw);
    prk::SpanPos *POS = reinterpret_cast<prk::SpanPos *>(a->pos);
    switch (mode) {
#define PRK_PR_GROUP(MM)                                                                                             \
    case MM:                                                                                                         \
        hipLaunchKernelGGL(prk::k_pr_chunk<MM>, dim3(max_chunks, ngroup), dim3(nt), bytes, s, *fp, O, P, grp, cap,  \
                           PR, a->cnt, a->eoff, a->fge, a->escan, a->total0p, W, a->soff, SST, EE, a->eend_m,       \
                           a->sidx, a->s_m, a->prstat, RAW, POS, a->span_tri, a->err, a->warmup);                    \
        if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;                                          \
        hipLaunchKernelGGL(prk::k_pr_cmp, dim3(a->nchunks), dim3(256), 0, s, P, a->npr, a->prstat, EE, a->eend_m,    \
                           a->sidx, a->s_m, a->match);                                                               \
        if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;                                          \
        hipLaunchKernelGGL(prk::k_pr_fix<MM>, dim3(ngroup), dim3(nt), bytes, s, *fp, O, P, grp, cap, PR, a->cnt,    \
                           a->eoff, a->fge, a->escan, a->total0p, W, a->soff, EE, a->eend_m, a->sidx, a->s_m,       \
                           a->match, a->prstat, RAW, POS, a->span_tri, a->err);                                      \
        break;
        PRK_PR_GROUP(prk::MODE_AVX)
        PRK_PR_GROUP(prk::MODE_SC_GOURAUD)
        PRK_PR_GROUP(prk::MODE_SC_GOURAUD_TEX)
        PRK_PR_GROUP(prk::MODE_SC_PHONG)
        PRK_PR_GROUP(prk::MODE_SC_PHONG_TEX)
#undef PRK_PR_GROUP
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
hipError_t prk_pr_walk_end(const prk::PrWalkArgs *a, hipStream_t s) {
    if (a->npr == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_pr_tally, dim3(1), dim3(256), 0, s, reinterpret_cast<const prk::PrObj *>(a->pro),
                       a->npr, a->prstat, a->err);
    return hipGetLastError();
}
uint32_t prk_pr_chunk_rows(void) { return (uint32_t)prk::kPrChunk; }
int32_t prk_pr_max_row_entries(void) { return prk::kPrMaxM; }
int32_t prk_pr_max_rows(void) { return prk::kMaxactRows - 1; }
// The slot walk's pairs (SPAN_RAW) into span records, one thread per slot.
hipError_t prk_span_finish(const prk::FrameParams *fp, const void *raw, uint32_t nslot, void *recs, void *srecs,
                           void *pos, hipStream_t s) {
    if (nslot == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_span_finish, dim3((nslot + 255) / 256), dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::PairRaw *>(raw), nslot, reinterpret_cast<prk::SpanRecG *>(recs),
                       reinterpret_cast<prk::ScSpanRecG *>(srecs), reinterpret_cast<prk::SpanPos *>(pos));
    return hipGetLastError();
}



// Span -> tile bin entries, pass 0: tcnt[t] = tile t's entries (ntiles + 1
// values, the last 0: the scan's total).
hipError_t prk_span_count(const prk::FrameParams *fp, const void *pos, uint32_t nspan, uint32_t *tcnt,
                          hipStream_t s) {
    const uint32_t ntiles = (uint32_t)(fp->tiles_x * fp->tiles_y);
    hipError_t e = hipMemsetAsync(tcnt, 0, ((size_t)ntiles + 1) * 4, s);
    if (e != hipSuccess || nspan == 0) return e;
    hipLaunchKernelGGL(prk::k_span_tiles<false>, dim3((nspan + 255) / 256), dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::SpanPos *>(pos), nspan, tcnt, nullptr, nullptr);
    return hipGetLastError();
}

// Pass 1: bins[offs[t] ...] = the spans of tile t (offs: the counts'
// exclusive scan; tcur: ntiles cursors, zeroed here).
hipError_t prk_span_bin(const prk::FrameParams *fp, const void *pos, uint32_t nspan, const uint32_t *offs,
                        uint32_t *tcur, uint32_t *bins, hipStream_t s) {
    const uint32_t ntiles = (uint32_t)(fp->tiles_x * fp->tiles_y);
    hipError_t e = hipMemsetAsync(tcur, 0, (size_t)ntiles * 4, s);
    if (e != hipSuccess || nspan == 0) return e;
    hipLaunchKernelGGL(prk::k_span_tiles<true>, dim3((nspan + 255) / 256), dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::SpanPos *>(pos), nspan, tcur, offs, bins);
    return hipGetLastError();
}

}  // extern "C"
