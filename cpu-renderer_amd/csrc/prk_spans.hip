// prk_spans.hip — whole-object active edge tables (the span path).
//
// A render_entry_3d_object of several triangles is ONE AET in the reference:
// FillEdgeTable appends the visible edges of all its triangles to one list
// (projekt.cpp:3894-4117), MergeSort orders them by YMin (2-72), and
// DrawModelOptimized(RenderQueue,...) pairs consecutive list entries into
// spans across triangles (3654-3869).  The per-triangle kernels cannot
// express that, so objects of more than one triangle take this path:
//
//   k_obj_walk    one thread per object: FillEdgeTable over its triangles,
//                 MergeSort with the reference's exact recursion (tie order
//                 included), then the AET walk with the reference's list
//                 operations (insertion scan, expiry, pairing, the two
//                 crossing swaps of 3831-3853 with the P3 head/tail fix),
//                 stepping the paired edges row by row.  Pass 0 counts the
//                 object's emitted spans; pass 1 writes, for each span in
//                 submission order (object, row, pair), its FillLineOptimized
//                 lane-init record (SpanRec, 1543-1835) and its pixel range.
//   k_span_count / k_span_emit   span -> (tile, span) bin entries; sorted by
//                 tile with the radix sort of the triangle path.
//   k_span_vis (prk_kernels.hip)  per-tile visibility over the spans with
//                 the 64-bit key max (tag = span index in submission order).
//   k_pix (prk_kernels.hip, span records indexed by span)  shading.
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include "prk_device.h"

namespace prk {

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
    uint32_t edge_off;  // first of its edge slots
    uint32_t kind, src, nsrc, pad;
};

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

// MergeSort (projekt.cpp:2-72) of the n edge slots named by ord[0..n), by
// YMin, with the reference's recursion: Count 2 swaps only on '>', larger
// counts split at Count/2 and merge taking Half0 only on strict '<'.  The
// tie order this produces depends on the recursion shape, so it is replayed
// (iteratively, post-order) rather than replaced by another stable sort.
__device__ void obj_merge_sort(const ObjEdge *E, uint32_t *ord, uint32_t *tmp, uint32_t n) {
    if (n < 2) return;  // P1: Count 0 returns (the reference recurses forever)
    struct Fr { uint32_t first, count, stage; };
    Fr st[64];
    int sp = 0;
    st[sp++] = Fr{0u, n, 0u};
    while (sp > 0) {
        Fr &f = st[sp - 1];
        if (f.count == 1) { --sp; continue; }
        if (f.count == 2) {
            if (E[ord[f.first]].YMin > E[ord[f.first + 1]].YMin) {
                const uint32_t t = ord[f.first];
                ord[f.first] = ord[f.first + 1];
                ord[f.first + 1] = t;
            }
            --sp;
            continue;
        }
        const uint32_t h0 = f.count / 2;
        if (f.stage == 0) { f.stage = 1; st[sp++] = Fr{f.first, h0, 0u}; continue; }
        if (f.stage == 1) { f.stage = 2; st[sp++] = Fr{f.first + h0, f.count - h0, 0u}; continue; }
        uint32_t r0 = f.first, r1 = f.first + h0;
        const uint32_t m1 = f.first + h0, end = f.first + f.count;
        for (uint32_t i = 0; i < f.count; ++i) {
            uint32_t take;
            if (r0 == m1) take = ord[r1++];
            else if (r1 == end) take = ord[r0++];
            else if (E[ord[r0]].YMin < E[ord[r1]].YMin) take = ord[r0++];
            else take = ord[r1++];
            tmp[i] = take;
        }
        for (uint32_t i = 0; i < f.count; ++i) ord[f.first + i] = tmp[i];
        --sp;
    }
}

// FillLineOptimized span setup (1543-1835) of the pair (L, R) at Row: the
// lane-init record and the covered range [MinX, MaxX).  False when the span
// covers nothing.
__device__ __forceinline__ bool obj_span(const FrameParams &fp, const ObjEdge &L, const ObjEdge &R, int32_t Row,
                                         int32_t texi, bool st, SpanRecG &rec, SpanPos &pos) {
    const int32_t W = fp.W;
    float XOffset = 0.0f;
    float LeftX = L.X;  // 1545-1565
    if (LeftX < 0) { XOffset = st ? -XOffset : -L.X; LeftX = 0; }  // single-thread: -XOffset (2508)
    else if (LeftX >= W) LeftX = (float)W - 1;
    float RightX = R.X;
    if (RightX < 0) RightX = 0;
    else if (RightX >= W) RightX = (float)W - 1;
    if (LeftX != LeftX || RightX != RightX) return false;  // pinned: NaN edge X draws nothing
    const int32_t MinX = round_s32(LeftX), MaxX = round_s32(RightX);  // 1588-1592
    if (MinX >= MaxX) return false;
    const int32_t XDiff = (int32_t)((uint32_t)round_s32(R.X) - (uint32_t)round_s32(L.X));  // 1568-1570
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

// The whole-object walk of one object of mode M (kind 0: its triangles;
// kind 1: a caller's edge list).  pass 0 counts its spans, pass 1 writes them
// at base.
template <int M>
__device__ void walk_object(const FrameParams &fp, const ObjDesc &od, const DrawRec &d, ObjEdge *__restrict__ E,
                            uint32_t *__restrict__ ord, uint32_t *__restrict__ tmp, int pass, uint32_t base,
                            uint32_t &emitted, SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                            SpanPos *__restrict__ pos, uint32_t *__restrict__ span_tri,
                            const EdgeIn *__restrict__ edges_in) {
    constexpr bool kScalar = M != MODE_AVX;
    const bool st = (d.flags & DRAW_ST) != 0;
    const bool given = od.kind == 1;  // a caller's (sorted) edge list
    uint32_t n = 0;
    if (given) {
        for (uint32_t i = 0; i < od.nsrc; ++i) {
            obj_edge_in(E[i], edges_in[od.src + i]);
            ord[i] = i;
        }
        n = od.nsrc;
    }
    // FillEdgeTable (3894-4117): visible edges of every triangle, in order.
    for (uint32_t t = 0; t < (given ? 0u : od.tris); ++t) {
        const uint32_t g = od.g0 + t;
        const uint32_t gt = d.geom_tri0 + (g - d.first_global);
        V3 cam[3], proj[3];
        load_positions(d, gt, fp, cam, proj);
        if (!front_facing(proj)) continue;  // 3926-3943
        TriRaw<M> raw;
        load_tri<M>(d, gt, raw);
        Edge e[3];
        bool vis[3];
        tri_edges<M>(raw, d, fp, e[0], e[1], e[2], vis);
        for (int k = 0; k < 3; ++k)
            if (vis[k]) {
                obj_edge_store(E[n], e[k]);
                ord[n] = n;
                ++n;
            }
    }
    if (!given) obj_merge_sort(E, ord, tmp, n);  // 4117
    if (n == 0) return;
    // The AET walk of DrawModelOptimized(RenderQueue,...) (3626-3869) /
    // DrawModel (173-598): the same list logic.
    const int32_t FirstRow = E[ord[0]].YMin;
    int32_t MaxRow = E[ord[0]].YMax;
    for (uint32_t i = 1; i < n; ++i) MaxRow = max(MaxRow, E[ord[i]].YMax);
    const int32_t MaxY = min(min(MaxRow, fp.H), fp.row1);
    // DrawModel's span of row row0-1 can store its one-past-the-row pixel
    // into (row0, 0)
    const int32_t RowLo = kScalar ? fp.row0 - 1 : fp.row0;
    int32_t Head = -1, Tail = -1;
    uint32_t ins = 0;  // next sorted edge to insert (sorted by YMin)
    for (int32_t Row = FirstRow; Row < MaxY; ++Row) {
        // insertion (3654-3713): the edges with YMin == Row, in array
        // order.  Sorted lists (our MergeSort) hold them contiguously; a
        // caller's list is scanned whole, as the reference does.
        uint32_t i0 = 0, i1 = n;
        if (!given) {
            while (ins < n && E[ord[ins]].YMin < Row) ++ins;
            i0 = ins;
            while (ins < n && E[ord[ins]].YMin == Row) ++ins;
            i1 = ins;
        }
        for (uint32_t ii = i0; ii < i1; ++ii) {
            if (E[ord[ii]].YMin != Row) continue;
            const int32_t c = (int32_t)ord[ii];
            ObjEdge &Cur = E[c];
            if (Head >= 0) {
                if (obj_before(Cur, E[Head])) {
                    Cur.Next = Head;
                    Head = c;
                } else {
                    int32_t Cmp = Head, Prev = Head;
                    while (Cmp != Tail) {
                        Cmp = E[Cmp].Next;
                        if (obj_before(Cur, E[Cmp])) {
                            Cur.Next = Cmp;
                            E[Prev].Next = c;
                            Cmp = Tail;
                        } else {
                            Prev = Cmp;
                        }
                    }
                    if (Prev == Cmp) {
                        E[Tail].Next = c;
                        Tail = c;
                    }
                }
            } else {
                Head = c;
                Tail = c;
            }
        }
        while (Head >= 0 && E[Head].YMax <= Row) {  // expiry 3715-3720
            const int32_t Rm = Head;
            Head = E[Head].Next;
            E[Rm].Next = -1;
        }
        if (Head < 0) { Tail = -1; continue; }  // pin: the reference dereferences NULL
        {
            int32_t Prev = Head, Chk = Head;  // 3722-3749
            while (Chk != Tail) {
                Chk = E[Chk].Next;
                if (E[Chk].YMax <= Row) {
                    if (Chk == Tail) {
                        Tail = Prev;
                        E[Tail].Next = -1;
                        Chk = Tail;
                    } else {
                        E[Prev].Next = E[Chk].Next;
                        Chk = Prev;
                    }
                }
                Prev = Chk;
            }
        }
        int32_t PrevCur = -1, PrevNext = -1;  // pairing 3751-3869
        int32_t Cur = Head, Next = E[Cur].Next;
        while (Next >= 0) {
            if (Row >= RowLo) {  // a span of this pass's rows (3759-3809 / 298-538)
                SpanPos sp;
                if constexpr (kScalar) {
                    ScSpanRecG srec;
                    if (obj_span_scalar<M>(fp, E[Cur], E[Next], Row, d.tex, srec, sp)) {
                        if (pass) {
                            SpanRecG mark;
                            mark.q0 = make_float4(__uint_as_float(kScalarSpan), 0.0f, 0.0f, 0.0f);
                            mark.q1 = mark.q2 = mark.q3 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                            recs[base + emitted] = mark;
                            srecs[base + emitted] = srec;
                            pos[base + emitted] = sp;
                            span_tri[base + emitted] = od.g0;
                        }
                        ++emitted;
                    }
                } else {
                    SpanRecG rec;
                    if (obj_span(fp, E[Cur], E[Next], Row, d.tex, st, rec, sp)) {
                        if (pass) {
                            recs[base + emitted] = rec;
                            pos[base + emitted] = sp;
                            span_tri[base + emitted] = od.g0;
                        }
                        ++emitted;
                    }
                }
            }
            obj_step<M>(E[Cur]);  // 3811-3829
            obj_step<M>(E[Next]);
            if (E[Cur].X > E[Next].X) {  // 3831-3841
                E[Cur].Next = E[Next].Next;
                E[Next].Next = Cur;
                if (PrevNext >= 0) E[PrevNext].Next = Next;
                else Head = Next;               // P3
                if (Tail == Next) Tail = Cur;   // P3
                Cur = Next;
                Next = E[Cur].Next;
            }
            if (PrevNext >= 0) {  // 3843-3853
                if (E[PrevNext].X > E[Cur].X) {
                    E[PrevNext].Next = E[Cur].Next;
                    E[Cur].Next = PrevNext;
                    E[PrevCur].Next = Cur;
                    PrevNext = Cur;
                    Cur = E[PrevNext].Next;
                }
            }
            PrevCur = Cur;
            PrevNext = Next;
            if (E[Next].Next >= 0) {
                Cur = E[Next].Next;
                Next = E[Cur].Next;
            } else {
                Next = -1;
            }
        }
    }
}

__global__ void __launch_bounds__(64) k_obj_walk(FrameParams fp, const ObjDesc *__restrict__ objs, uint32_t nobj,
                                                 ObjEdge *__restrict__ edges, uint32_t *__restrict__ ordbuf,
                                                 uint32_t *__restrict__ tmpbuf, int pass,
                                                 uint32_t *__restrict__ counts, const uint32_t *__restrict__ offs,
                                                 SpanRecG *__restrict__ recs, ScSpanRecG *__restrict__ srecs,
                                                 SpanPos *__restrict__ pos,
                                                 uint32_t *__restrict__ span_tri, const EdgeIn *__restrict__ edges_in,
                                                 const SpanIn *__restrict__ spans_in) {
    const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nobj) return;
    const ObjDesc od = objs[o];
    const DrawRec &d = fp.draws[od.draw];
    const bool st = (d.flags & DRAW_ST) != 0;
    const uint32_t base = pass ? offs[o] : 0u;
    uint32_t emitted = 0;
    if (od.kind == 2) {  // one caller-given span (DoLineRenderWork / DoBufferLineRenderWork)
        const SpanIn sp = spans_in[od.src];
        if (sp.Row >= fp.row0 && sp.Row < fp.row1 && sp.Row < fp.H) {
            SpanRecG rec;
            SpanPos ps;
            if (obj_span(fp, span_end_in(sp.L), span_end_in(sp.R), sp.Row, d.tex, st, rec, ps)) {
                if (pass) {
                    recs[base] = rec;
                    pos[base] = ps;
                    span_tri[base] = od.g0;
                }
                emitted = 1;
            }
        }
        if (!pass) counts[o] = emitted;
        return;
    }
    ObjEdge *E = edges + od.edge_off;
    uint32_t *ord = ordbuf + od.edge_off, *tmp = tmpbuf + od.edge_off;
    switch (d.mode) {
#define PRK_WALK_OBJ(MM)                                                                                      \
    case MM:                                                                                                  \
        walk_object<MM>(fp, od, d, E, ord, tmp, pass, base, emitted, recs, srecs, pos, span_tri, edges_in);   \
        break;
        PRK_WALK_OBJ(MODE_AVX)
        PRK_WALK_OBJ(MODE_SC_GOURAUD)
        PRK_WALK_OBJ(MODE_SC_GOURAUD_TEX)
        PRK_WALK_OBJ(MODE_SC_PHONG)
        PRK_WALK_OBJ(MODE_SC_PHONG_TEX)
#undef PRK_WALK_OBJ
        default: break;
    }
    if (!pass) counts[o] = emitted;
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
        t.ty = (p.row - fp.row0) / fp.tile_h;
        t.tx0 = p.minx >> fp.tile_w_log2;
        t.tx1 = (xe - 1) >> fp.tile_w_log2;
    }
    if ((p.flags & SPAN_SCALAR) && p.maxx > fp.W && p.row + 1 >= fp.row0 && p.row + 1 < fp.row1 &&
        p.row + 1 < fp.H) {
        const int oty = (p.row + 1 - fp.row0) / fp.tile_h;
        if (!(t.tx0 == 0 && t.tx0 <= t.tx1 && t.ty == oty)) t.oty = oty;
    }
    return t;
}

// Bin entries of every span.
__global__ void k_span_count(FrameParams fp, const SpanPos *__restrict__ pos, uint32_t nspan,
                             uint32_t *__restrict__ cnt) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > nspan) return;
    if (s == nspan) {  // sentinel: the scan's last element is the total
        cnt[s] = 0;
        return;
    }
    const SpanTiles t = span_tiles(fp, pos[s]);
    cnt[s] = (uint32_t)(max(0, t.tx1 - t.tx0 + 1) + (t.oty >= 0 ? 1 : 0));
}

__global__ void k_span_emit(FrameParams fp, const SpanPos *__restrict__ pos, uint32_t nspan,
                            const uint32_t *__restrict__ off, uint32_t *__restrict__ keys,
                            uint32_t *__restrict__ vals) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nspan) return;
    const SpanTiles t = span_tiles(fp, pos[s]);
    uint32_t o = off[s];
    for (int tx = t.tx0; tx <= t.tx1; ++tx) {
        keys[o] = (uint32_t)(t.ty * fp.tiles_x + tx);
        vals[o] = s;
        ++o;
    }
    if (t.oty >= 0) {
        keys[o] = (uint32_t)(t.oty * fp.tiles_x);
        vals[o] = s;
    }
}

__global__ void k_span_tile_offsets(const uint32_t *__restrict__ keys, uint32_t total, uint32_t ntiles,
                                    uint32_t *__restrict__ offs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    uint32_t lo = 0, hi = total;
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if (keys[mid] < t) lo = mid + 1; else hi = mid;
    }
    offs[t] = lo;
}

}  // namespace prk

extern "C" {

// Pass 0 / 1 of the object walk.
hipError_t prk_obj_walk(const prk::FrameParams *fp, const void *objs, uint32_t nobj, void *edges, uint32_t *ord,
                        uint32_t *tmp, int pass, uint32_t *counts, const uint32_t *offs, void *recs, void *srecs,
                        void *pos, uint32_t *span_tri, const void *edges_in, const void *spans_in, hipStream_t s) {
    if (nobj == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_obj_walk, dim3((nobj + 63) / 64), dim3(64), 0, s, *fp,
                       reinterpret_cast<const prk::ObjDesc *>(objs), nobj, reinterpret_cast<prk::ObjEdge *>(edges),
                       ord, tmp, pass, counts, offs, reinterpret_cast<prk::SpanRecG *>(recs),
                       reinterpret_cast<prk::ScSpanRecG *>(srecs), reinterpret_cast<prk::SpanPos *>(pos), span_tri,
                       reinterpret_cast<const prk::EdgeIn *>(edges_in), reinterpret_cast<const prk::SpanIn *>(spans_in));
    return hipGetLastError();
}

// Exclusive scan of n + 1 counts (temp == nullptr: size query).
hipError_t prk_scan_u32(const uint32_t *in, uint32_t *out, uint32_t n, void *temp, size_t *temp_bytes,
                        hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, in, out, n, s);
}

hipError_t prk_span_count(const prk::FrameParams *fp, const void *pos, uint32_t nspan, uint32_t *cnt,
                          hipStream_t s) {
    hipLaunchKernelGGL(prk::k_span_count, dim3((nspan + 1 + 255) / 256), dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::SpanPos *>(pos), nspan, cnt);
    return hipGetLastError();
}

// Emit, sort by tile (stable, span order kept) and tile offsets.
hipError_t prk_span_bin(const prk::FrameParams *fp, const void *pos, uint32_t nspan, const uint32_t *off,
                        uint32_t total, uint32_t *keys_a, uint32_t *vals_a, uint32_t *keys_b, uint32_t *vals_b,
                        uint32_t *offs, void *temp, size_t *temp_bytes, hipStream_t s) {
    const uint32_t ntiles = (uint32_t)(fp->tiles_x * fp->tiles_y);
    int bits = 1;
    while ((1u << bits) < ntiles + 1 && bits < 32) ++bits;
    if (!temp)
        return rocprim::radix_sort_pairs(nullptr, *temp_bytes, keys_a, keys_b, vals_a, vals_b, total, 0,
                                         (unsigned)bits, s);
    if (nspan)
        hipLaunchKernelGGL(prk::k_span_emit, dim3((nspan + 255) / 256), dim3(256), 0, s, *fp,
                           reinterpret_cast<const prk::SpanPos *>(pos), nspan, off, keys_a, vals_a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (total) {
        e = rocprim::radix_sort_pairs(temp, *temp_bytes, keys_a, keys_b, vals_a, vals_b, total, 0, (unsigned)bits,
                                      s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(prk::k_span_tile_offsets, dim3((ntiles + 1 + 255) / 256), dim3(256), 0, s, keys_b, total,
                       ntiles, offs);
    return hipGetLastError();
}

}  // extern "C"
