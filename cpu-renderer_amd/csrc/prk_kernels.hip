// prk_kernels.hip — gfx950 kernels of the rasterizer hot path.
//
// Pipeline per flush:
//   k_bin_count  one thread per triangle: ProjectVertex + back-face cull
//                (projekt.cpp:74-93, 3926-3943) -> conservative pixel bbox ->
//                per-tile counts.
//   k_scan       exclusive scan of the per-tile counts (one workgroup).
//   k_bin_fill   one thread per triangle: scatter its index into every tile
//                bin it overlaps (order inside a bin does not matter, see below).
//   k_raster     one workgroup per screen tile; the tile's z/colour slab lives
//                in LDS.  Each lane owns one bin entry (a triangle), re-runs
//                FillEdgeTable for it (projekt.cpp:3882-4121), walks its AET
//                (3615-3871) over the tile's rows and fills its spans with the
//                reference's exact span arithmetic (FillLineOptimized
//                1492-2320 or DrawModel 298-538).
//                Sweep 1 resolves visibility with 64-bit LDS atomicMax on
//                key = (ordered z << 32) | (0xFFFFFFFE - triangle): the
//                reference's strict z '>' in submission order keeps exactly
//                the EARLIEST fragment of maximal z, which is that max.
//                Sweep 2 re-walks and shades only the winning fragments
//                (texture + Phong), so shading runs once per pixel instead of
//                once per fragment.  A coalesced flush writes z and colour of
//                every pixel that got a winner.
#include "prk_device.h"

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

struct TileRange { uint16_t tx0, ty0, tx1, ty1; };

// Conservative tile range of a triangle's covered pixels.  Span end points
// are edge-DDA values that stay on their segment up to float error
// (DESIGN.md §4.1), so [min x, max x] of the projected vertices widened by
// that error bounds every covered pixel; rows lie in [floor(min y), ceil(max y)).
__device__ __forceinline__ bool tri_tile_range(const FrameParams &fp, uint32_t g, TileRange &tr) {
    const DrawRec *d;
    uint32_t gt;
    resolve_draw(fp, g, d, gt);
    V3 cam[3], proj[3];
    load_positions(*d, gt, fp, cam, proj);
    if (!front_facing(proj)) return false;  // also rejects every non-finite vertex
    float xmin = fminf(proj[0].x, fminf(proj[1].x, proj[2].x));
    float xmax = fmaxf(proj[0].x, fmaxf(proj[1].x, proj[2].x));
    float ymin = fminf(proj[0].y, fminf(proj[1].y, proj[2].y));
    float ymax = fmaxf(proj[0].y, fmaxf(proj[1].y, proj[2].y));
    float fr0 = floorf(ymin), fr1 = ceilf(ymax);
    int32_t r0 = fr0 < (float)fp.row0 ? fp.row0 : (fr0 >= (float)fp.row1 ? fp.row1 : (int32_t)fr0);
    int32_t r1 = fr1 > (float)fp.row1 ? fp.row1 : (fr1 <= (float)fp.row0 ? fp.row0 : (int32_t)fr1);
    if (r0 >= r1) return false;
    float maxabs = fmaxf(fabsf(xmin), fabsf(xmax));
    float slack = 2.0f + ((ymax - ymin) + 4.0f) * maxabs * (1.0f / 2097152.0f);  // 2^-21
    float fc0 = floorf(xmin - slack), fc1 = ceilf(xmax + slack) + 1.0f;
    int32_t c0 = fc0 < 0.0f ? 0 : (fc0 >= (float)fp.W ? fp.W : (int32_t)fc0);
    int32_t c1 = fc1 > (float)fp.W ? fp.W : (fc1 <= 0.0f ? 0 : (int32_t)fc1);
    if (c0 >= c1) return false;
    tr.tx0 = (uint16_t)(c0 / fp.tile_w);
    tr.tx1 = (uint16_t)((c1 - 1) / fp.tile_w);
    tr.ty0 = (uint16_t)((r0 - fp.row0) / fp.tile_h);
    tr.ty1 = (uint16_t)((r1 - 1 - fp.row0) / fp.tile_h);
    return true;
}

__global__ void k_bin_count(FrameParams fp, uint32_t *__restrict__ counts,
                            TileRange *__restrict__ ranges) {
    uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= fp.tri_count) return;
    TileRange tr;
    if (!tri_tile_range(fp, g, tr)) {
        tr.tx0 = 1; tr.tx1 = 0; tr.ty0 = 1; tr.ty1 = 0;
    } else {
        for (int ty = tr.ty0; ty <= tr.ty1; ++ty)
            for (int tx = tr.tx0; tx <= tr.tx1; ++tx)
                atomicAdd(&counts[ty * fp.tiles_x + tx], 1u);
    }
    ranges[g] = tr;
}

// Exclusive scan of n counts into offs[0..n]; offs[n] = total.  One workgroup.
__global__ void __launch_bounds__(1024) k_scan(const uint32_t *__restrict__ counts,
                                               uint32_t *__restrict__ offs, uint32_t n) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t b = t * per, e = min(n, b + per);
    uint32_t s = 0;
    for (uint32_t i = b; i < e; ++i) s += counts[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;  // exclusive prefix of this chunk
    for (uint32_t i = b; i < e; ++i) {
        offs[i] = run;
        run += counts[i];
    }
    if (t == 1023) offs[n] = part[1023];
}

__global__ void k_bin_fill(FrameParams fp, const TileRange *__restrict__ ranges,
                           const uint32_t *__restrict__ offs, uint32_t *__restrict__ cursor,
                           uint32_t *__restrict__ bins) {
    uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= fp.tri_count) return;
    TileRange tr = ranges[g];
    for (int ty = tr.ty0; ty <= tr.ty1; ++ty)
        for (int tx = tr.tx0; tx <= tr.tx1; ++tx) {
            int t = ty * fp.tiles_x + tx;
            uint32_t p = atomicAdd(&cursor[t], 1u);
            bins[offs[t] + p] = g;
        }
}

// ---------------------------------------------------------------------------
// Tile raster.
// ---------------------------------------------------------------------------
struct TileCtx {
    int32_t x0, x1, y0, y1, tw;  // tile pixel rectangle [x0,x1) x [y0,y1), LDS row stride tw
    unsigned long long *key;     // LDS: visibility keys
    uint32_t *ocol;              // LDS: winner colours
};

__device__ __forceinline__ unsigned long long make_key(float z, uint32_t tag) {
    return ((unsigned long long)zkey(z) << 32) | tag;
}

__device__ __forceinline__ bool is_winner(const TileCtx &tc, int p, uint32_t tag) {
    return (uint32_t)tc.key[p] == tag;
}

__device__ __forceinline__ void put_winner(const TileCtx &tc, int p, float z, uint32_t col) {
    tc.ocol[p] = col;
    reinterpret_cast<uint32_t *>(tc.key + p)[1] = __float_as_uint(z);  // raw z bits
}

// ----- FillLineOptimized span (projekt.cpp:1492-2320) -----------------------
template <bool SHADE>
__device__ __forceinline__ void span_avx(const FrameParams &fp, const TexRec &tex, const TileCtx &tc,
                                         uint32_t tag, const Edge &L, const Edge &R, int32_t Row) {
    const int32_t W = fp.W;
    float XOffset = 0.0f;
    if (Row < 0) return;
    float LeftX = L.X;  // 1545-1565
    if (LeftX < 0) { XOffset = -L.X; LeftX = 0; }
    else if (LeftX >= W) LeftX = (float)W - 1;
    float RightX = R.X;
    if (RightX < 0) RightX = 0;
    else if (RightX >= W) RightX = (float)W - 1;
    if (LeftX != LeftX || RightX != RightX) return;  // pinned: NaN edge X draws nothing
    const int32_t XDiff = (int32_t)((uint32_t)round_s32(R.X) - (uint32_t)round_s32(L.X));  // 1568-1570
    const int32_t MinX = round_s32(LeftX), MaxX = round_s32(RightX);  // 1588-1592
    int32_t LeftXa = MinX;
    if (MinX & 7) {  // 1594-1609
        LeftXa = MinX & ~7;
        XOffset -= (float)(MinX & 7) * 1.0f;
    }
    // Coverage of the clip masks is exactly [MinX, MaxX).
    const int32_t xa = max(MinX, tc.x0), xb = min(MaxX, tc.x1);
    if (xa >= xb) return;
    const int rowoff = (Row - tc.y0) * tc.tw - tc.x0;

    if (SHADE) {  // any winner of this triangle on this span?
        bool any = false;
        for (int32_t x = xa; x < xb; ++x) any |= is_winner(tc, rowoff + x, tag);
        if (!any) return;
    }
    const float fXD = (float)XDiff;
    float IW = 0, IU = 0, IV = 0, IZ = 0, IN0 = 0, IN1 = 0, IN2 = 0;
    if (XDiff != 0) {  // 1666-1835
        IW = (R.W - L.W) / fXD;
        IU = (R.U - L.U) / fXD;
        IV = (R.V - L.V) / fXD;
        if (SHADE) {
            IN0 = (R.N0 - L.N0) / fXD;
            IN1 = (R.N1 - L.N1) / fXD;
            IN2 = (R.N2 - L.N2) / fXD;
        }
        IZ = (R.Z - L.Z) / fXD;
    }
    const float IW8 = IW * 8.0f, IU8 = IU * 8.0f, IV8 = IV * 8.0f, IZ8 = 8.0f * IZ;
    const float IN08 = IN0 * 8.0f, IN18 = IN1 * 8.0f, IN28 = IN2 * 8.0f;
    const float Tw = (float)tex.w, Th = (float)tex.h;

    for (int i = 0; i < 8; ++i) {
        // pixels x = LeftXa + 8b + i inside [xa, xb)
        int32_t rel = xa - LeftXa - i;
        int32_t b0 = rel <= 0 ? 0 : (rel + 7) >> 3;
        int32_t x = LeftXa + 8 * b0 + i;
        if (x >= xb) continue;
        const float o = XOffset + (float)i;  // lane init (XOffset + i)*inc, 1712-1835
        float w = L.W + o * IW, u = L.U + o * IU, v = L.V + o * IV, z = L.Z + o * IZ;
        float n0 = 0, n1 = 0, n2 = 0;
        if (SHADE) {
            n0 = L.N0 + o * IN0; n1 = L.N1 + o * IN1; n2 = L.N2 + o * IN2;
            normalize_div(n0, n1, n2);  // 1754
        }
        for (int32_t k = 0; k < b0; ++k) {  // block steps 2262-2282
            if (SHADE) {
                float a = n0 + IN08, b = n1 + IN18, c = n2 + IN28;
                normalize_div(a, b, c);
                n0 = a; n1 = b; n2 = c;
            }
            z = z + IZ8; w = w + IW8; u = u + IU8; v = v + IV8;
        }
        for (; x < xb; x += 8) {
            const float iw = 1.0f / w;  // 1865-1866
            const float fu = iw * u, fv = iw * v;
            const int p = rowoff + x;
            if (!SHADE) {
                if (fu >= 0.0f && fu <= 1.0f && fv >= 0.0f && fv <= 1.0f && z == z)
                    atomicMax(&tc.key[p], make_key(z, tag));
            } else if (is_winner(tc, p, tag)) {
                // Texel (1881-2032): trunc, <<2, 16-bit pitch multiply, P2 clamp.
                const int32_t FX = (int32_t)((uint32_t)cvtt_s32(Tw * fu) << 2);
                const int32_t FY = mul16_trick(cvtt_s32(Th * fv), tex.pitch);
                const uint32_t t = texel_at(tex, (int32_t)((uint32_t)FX + (uint32_t)FY));
                const float CA = (float)((t >> 24) & 0xFF) / 255.0f;
                const float CR = (float)((t >> 16) & 0xFF) / 255.0f;
                const float CG = (float)((t >> 8) & 0xFF) / 255.0f;
                const float CB = (float)(t & 0xFF) / 255.0f;
                // Phong (2040-2128) at UnprojectVertex_8x (102-145).
                const float d = fp.D - z;
                const float Xf = (float)(x - i) + (float)i, Yf = (float)Row + 0.0f;
                const float AX = (Xf - fp.Cx) * fp.InvM2P, AY = (Yf - fp.Cy) * fp.InvM2P;
                const float PX = (d / fp.F) * AX, PY = (d / fp.F) * AY, PZ = z;
                float Fr = 0, Fg = 0, Fb = 0, Fa = 0;
                for (uint32_t li = 0; li < fp.light_count; ++li) {
                    if (li == 0) {
                        Fr = CR * fp.amb[0]; Fg = CG * fp.amb[1];
                        Fb = CB * fp.amb[2]; Fa = CA * fp.amb[3];
                    }
                    float Lx = fp.lp[li][0] - PX, Ly = fp.lp[li][1] - PY, Lz = fp.lp[li][2] - PZ;
                    normalize_div(Lx, Ly, Lz);
                    const float Cos = minps(1.0f, maxps(0.0f, (n0 * Lx + n1 * Ly) + n2 * Lz));
                    float Vx = 0.0f - PX, Vy = 0.0f - PY, Vz = 0.0f - PZ;
                    normalize_div(Vx, Vy, Vz);
                    float Hx = Lx + Vx, Hy = Ly + Vy, Hz = Lz + Vz;
                    normalize_div(Hx, Hy, Hz);
                    float Ph = minps(1.0f, maxps(0.0f, (n0 * Hx + n1 * Hy) + n2 * Hz));
                    Ph = Ph * Ph; Ph = Ph * Ph; Ph = Ph * Ph; Ph = Ph * Ph;
                    const float *I = fp.li[li];
                    Fr = Fr + ((Cos * (CR * I[0])) + (Ph * (1.0f * I[0])));
                    Fg = Fg + ((Cos * (CG * I[1])) + (Ph * (1.0f * I[1])));
                    Fb = Fb + ((Cos * (CB * I[2])) + (Ph * (1.0f * I[2])));
                    Fa = Fa + ((Cos * (CA * I[3])) + (Ph * (1.0f * I[3])));
                }
                Fr = maxps(minps(Fr, 1.0f), 0.0f);  // 2131-2134
                Fg = maxps(minps(Fg, 1.0f), 0.0f);
                Fb = maxps(minps(Fb, 1.0f), 0.0f);
                Fa = maxps(minps(Fa, 1.0f), 0.0f);
                const uint32_t packed = ((uint32_t)cvt_rne_s32(Fr * 255.0f) << 16) |
                                        ((uint32_t)cvt_rne_s32(Fg * 255.0f) << 8) |
                                        ((uint32_t)cvt_rne_s32(Fb * 255.0f)) |
                                        ((uint32_t)cvt_rne_s32(Fa * 255.0f) << 24);
                put_winner(tc, p, z, packed);
            }
            if (SHADE) {
                float a = n0 + IN08, b = n1 + IN18, c = n2 + IN28;
                normalize_div(a, b, c);
                n0 = a; n1 = b; n2 = c;
            }
            z = z + IZ8; w = w + IW8; u = u + IU8; v = v + IV8;
        }
    }
}

// ----- DrawModel span (projekt.cpp:298-538) ---------------------------------
template <int M, bool SHADE>
__device__ __forceinline__ void span_scalar(const FrameParams &fp, const TexRec &tex, const TileCtx &tc,
                                            uint32_t tag, const Edge &L, const Edge &R, int32_t Row) {
    using TR = ModeTraits<M>;
    const int32_t W = fp.W;
    float XOffset = 0.0f;
    if (Row < 0) return;
    const float XDiff = roundf(R.X - L.X);  // 311-312
    float IW = 0, IU = 0, IV = 0, IZ = 0, IN0 = 0, IN1 = 0, IN2 = 0;
    float IC0 = 0, IC1 = 0, IC2 = 0, IC3 = 0;
    if (XDiff != 0.0f) {  // 329-360
        if (TR::tex) {
            IW = (R.W - L.W) / XDiff;
            IU = (R.U - L.U) / XDiff;
            IV = (R.V - L.V) / XDiff;
        }
        if (TR::phong) {
            IN0 = (R.N0 - L.N0) / XDiff;
            IN1 = (R.N1 - L.N1) / XDiff;
            IN2 = (R.N2 - L.N2) / XDiff;
        }
        if (TR::color) {
            IC0 = (R.C0 - L.C0) / XDiff;
            IC1 = (R.C1 - L.C1) / XDiff;
            IC2 = (R.C2 - L.C2) / XDiff;
            IC3 = (R.C3 - L.C3) / XDiff;
        }
        IZ = (R.Z - L.Z) / XDiff;
    }
    float LeftX = L.X;  // 381-400
    if (LeftX < 0) { XOffset = -L.X; LeftX = 0; }
    else if (LeftX >= W) LeftX = (float)W - 1;
    float RightX = R.X;
    if (RightX < 0) RightX = 0;
    else if (RightX >= W) RightX = (float)W - 1;
    if (LeftX != LeftX || RightX != RightX) return;
    const int32_t MinX = round_s32(LeftX), MaxX = round_s32(RightX);  // 402-406
    const int32_t xa = max(MinX, tc.x0), xb = min(MaxX + 1, tc.x1);     // inclusive [MinX, MaxX]
    if (xa >= xb) return;
    const int rowoff = (Row - tc.y0) * tc.tw - tc.x0;
    if (SHADE) {
        bool any = false;
        for (int32_t x = xa; x < xb; ++x) any |= is_winner(tc, rowoff + x, tag);
        if (!any) return;
    }
    float z = L.Z + XOffset * IZ;  // 408-412 (CurrentZ += XOffset*ZIncrement)
    float w = L.W, u = L.U, v = L.V, n0 = L.N0, n1 = L.N1, n2 = L.N2;
    float c0 = L.C0, c1 = L.C1, c2 = L.C2, c3 = L.C3;
    if (SHADE) {
        w += XOffset * IW; u += XOffset * IU; v += XOffset * IV;
        n0 += XOffset * IN0; n1 += XOffset * IN1; n2 += XOffset * IN2;
        c0 += XOffset * IC0; c1 += XOffset * IC1; c2 += XOffset * IC2; c3 += XOffset * IC3;
    }
    for (int32_t x = MinX; x < xb; ++x) {  // 423: sequential per-pixel stepping
        if (x >= xa) {
            const int p = rowoff + x;
            if (!SHADE) {
                if (z == z) atomicMax(&tc.key[p], make_key(z, tag));
            } else if (is_winner(tc, p, tag)) {
                float C[4] = {c0, c1, c2, c3};
                if (TR::tex) {  // 427-446
                    const float s = 1.0f / w;
                    const float FU = s * u, FV = s * v;
                    const int32_t TX = round_s32(FU * (float)(tex.w - 1));
                    const int32_t TY = round_s32(FV * (float)(tex.h - 1));
                    const uint32_t t = texel_at(tex, (int32_t)((uint32_t)TX * 4u + (uint32_t)TY * (uint32_t)tex.pitch));
                    C[3] = (float)((t >> 24) & 0xFF) / 255.0f;
                    C[0] = (float)((t >> 16) & 0xFF) / 255.0f;
                    C[1] = (float)((t >> 8) & 0xFF) / 255.0f;
                    C[2] = (float)(t & 0xFF) / 255.0f;
                }
                float F[4];
                if (TR::phong) {  // 448-484 with UnprojectVertex (147-160)
                    const float d = fp.D - z;
                    const float PX = (d / fp.F) * (((float)x - fp.Cx) * fp.InvM2P);
                    const float PY = (d / fp.F) * (((float)Row - fp.Cy) * fp.InvM2P);
                    const float PZ = z;
                    F[0] = F[1] = F[2] = F[3] = 0.0f;
                    for (uint32_t li = 0; li < fp.light_count; ++li) {
                        if (li == 0)
                            for (int c = 0; c < 4; ++c) F[c] = C[c] * fp.amb[c];
                        float Lx = fp.lp[li][0] - PX, Ly = fp.lp[li][1] - PY, Lz = fp.lp[li][2] - PZ;
                        normalize_rcp(Lx, Ly, Lz);
                        const float Cos = clamp01((n0 * Lx + n1 * Ly) + n2 * Lz);
                        float Vx = -PX, Vy = -PY, Vz = -PZ;
                        normalize_rcp(Vx, Vy, Vz);
                        float Hx = Lx + Vx, Hy = Ly + Vy, Hz = Lz + Vz;
                        normalize_rcp(Hx, Hy, Hz);
                        float Ph = clamp01((n0 * Hx + n1 * Hy) + n2 * Hz);
                        Ph = (float)pow((double)Ph, 16.0);
                        for (int c = 0; c < 4; ++c)
                            F[c] = F[c] + ((Cos * (C[c] * fp.li[li][c])) + (Ph * (1.0f * fp.li[li][c])));
                    }
                    for (int c = 0; c < 4; ++c) F[c] = clamp01(F[c]);
                } else {
                    for (int c = 0; c < 4; ++c) F[c] = C[c];  // 515, no clamp
                }
                const uint32_t packed = (round_u32(F[3] * 255.0f) << 24) | (round_u32(F[0] * 255.0f) << 16) |
                                        (round_u32(F[1] * 255.0f) << 8) | (round_u32(F[2] * 255.0f));
                put_winner(tc, p, z, packed);
            }
        }
        // per-pixel step (504-510 / 530-535)
        if (SHADE) {
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

template <int M, bool SHADE>
__device__ __forceinline__ void raster_tri(const FrameParams &fp, const TileCtx &tc, uint32_t g) {
    const DrawRec *d;
    uint32_t gt;
    resolve_draw(fp, g, d, gt);
    Edge s0, s1, s2;
    const int n = setup_triangle<M>(*d, gt, fp, s0, s1, s2);
    if (n < 2) return;
    const uint32_t tag = 0xFFFFFFFEu - g;
    TexRec tex;
    if (ModeTraits<M>::tex) tex = fp.texs[d->tex];
    else { tex.mem = nullptr; tex.w = tex.h = tex.pitch = 0; tex.pad = 0; }
    aet_walk<M>(n, s0, s1, s2, fp.H, tc.y0, tc.y1, [&](const Edge &L, const Edge &R, int32_t Row) {
        if (M == MODE_AVX) span_avx<SHADE>(fp, tex, tc, tag, L, R, Row);
        else span_scalar<M, SHADE>(fp, tex, tc, tag, L, R, Row);
    });
}

template <bool SHADE>
__device__ __forceinline__ void raster_entry(const FrameParams &fp, const TileCtx &tc, uint32_t g) {
    const DrawRec *d;
    uint32_t gt;
    resolve_draw(fp, g, d, gt);
    switch (d->mode) {
        case MODE_AVX: raster_tri<MODE_AVX, SHADE>(fp, tc, g); break;
        case MODE_SC_GOURAUD: raster_tri<MODE_SC_GOURAUD, SHADE>(fp, tc, g); break;
        case MODE_SC_GOURAUD_TEX: raster_tri<MODE_SC_GOURAUD_TEX, SHADE>(fp, tc, g); break;
        case MODE_SC_PHONG: raster_tri<MODE_SC_PHONG, SHADE>(fp, tc, g); break;
        case MODE_SC_PHONG_TEX: raster_tri<MODE_SC_PHONG_TEX, SHADE>(fp, tc, g); break;
        default: break;
    }
}

template <int MODESET>  // MODESET: MODE_AVX..MODE_SC_PHONG_TEX (single mode) or -1 (any)
__global__ void __launch_bounds__(256) k_raster(FrameParams fp, const uint32_t *__restrict__ offs,
                                                const uint32_t *__restrict__ bins) {
    extern __shared__ unsigned long long lds[];
    const int ntile = fp.tiles_x * fp.tiles_y;
    const int t = blockIdx.x;
    if (t >= ntile) return;
    const uint32_t b0 = offs[t], b1 = offs[t + 1];
    if (b0 == b1) return;  // no triangle touches this tile: leave it untouched
    const int tx = t % fp.tiles_x, ty = t / fp.tiles_x;
    TileCtx tc;
    tc.tw = fp.tile_w;
    tc.x0 = tx * fp.tile_w;
    tc.x1 = min(fp.W, tc.x0 + fp.tile_w);
    tc.y0 = fp.row0 + ty * fp.tile_h;
    tc.y1 = min(fp.row1, tc.y0 + fp.tile_h);
    const int npx = fp.tile_w * fp.tile_h;
    tc.key = lds;
    tc.ocol = reinterpret_cast<uint32_t *>(lds + npx);

    // Prior z of the target: a fragment must beat it strictly.
    for (int p = threadIdx.x; p < npx; p += blockDim.x) {
        const int lx = p % fp.tile_w, ly = p / fp.tile_w;
        const int x = tc.x0 + lx, y = tc.y0 + ly;
        unsigned long long k = ~0ull;
        if (x < tc.x1 && y < tc.y1) {
            const float z = fp.zbuf[(size_t)(y - fp.row0) * fp.W + x];
            k = (z != z) ? ~0ull : (((unsigned long long)zkey(z) << 32) | 0xFFFFFFFFull);
        }
        tc.key[p] = k;
    }
    __syncthreads();
    for (uint32_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        if constexpr (MODESET >= 0) raster_tri<(MODESET >= 0 ? MODESET : 0), false>(fp, tc, bins[i]);
        else raster_entry<false>(fp, tc, bins[i]);
    }
    __syncthreads();
    for (uint32_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) {
        if constexpr (MODESET >= 0) raster_tri<(MODESET >= 0 ? MODESET : 0), true>(fp, tc, bins[i]);
        else raster_entry<true>(fp, tc, bins[i]);
    }
    __syncthreads();
    // Flush: every pixel with a winner gets its z and colour.
    for (int p = threadIdx.x; p < npx; p += blockDim.x) {
        const int lx = p % fp.tile_w, ly = p / fp.tile_w;
        const int x = tc.x0 + lx, y = tc.y0 + ly;
        if (x >= tc.x1 || y >= tc.y1) continue;
        const unsigned long long k = tc.key[p];
        const uint32_t low = (uint32_t)k;
        const size_t row = (size_t)(y - fp.row0);
        if (low != 0xFFFFFFFFu) {
            fp.zbuf[row * fp.W + x] = __uint_as_float((uint32_t)(k >> 32));
            reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(fp.color) + row * fp.pitch)[x] = tc.ocol[p];
        }
        if (fp.winners)
            fp.winners[row * fp.W + x] = low != 0xFFFFFFFFu ? (int32_t)(0xFFFFFFFEu - low) : -1;
    }
}

// Explicit instantiations used by the host.
template __global__ void k_raster<-1>(FrameParams, const uint32_t *, const uint32_t *);
template __global__ void k_raster<MODE_AVX>(FrameParams, const uint32_t *, const uint32_t *);
template __global__ void k_raster<MODE_SC_GOURAUD>(FrameParams, const uint32_t *, const uint32_t *);
template __global__ void k_raster<MODE_SC_PHONG>(FrameParams, const uint32_t *, const uint32_t *);

}  // namespace prk

// ---------------------------------------------------------------------------
// Launchers (called from prk_api.cpp).
// ---------------------------------------------------------------------------
extern "C" {

hipError_t prk_launch_tri_draw(const prk::DrawRec *draws, uint32_t ndraws, uint32_t *tri_draw,
                               uint32_t tri_count, hipStream_t s) {
    if (tri_count == 0) return hipSuccess;
    hipLaunchKernelGGL(prk::k_tri_draw, dim3((tri_count + 255) / 256), dim3(256), 0, s, draws, ndraws,
                       tri_draw, tri_count);
    return hipGetLastError();
}

hipError_t prk_launch_bin(const prk::FrameParams *fp, uint32_t *counts, uint32_t *offs, uint32_t *cursor,
                          void *ranges, uint32_t ntiles, hipStream_t s) {
    if (fp->tri_count == 0) return hipSuccess;
    const dim3 grid((fp->tri_count + 255) / 256);
    hipLaunchKernelGGL(prk::k_bin_count, grid, dim3(256), 0, s, *fp, counts,
                       reinterpret_cast<prk::TileRange *>(ranges));
    hipLaunchKernelGGL(prk::k_scan, dim3(1), dim3(1024), 0, s, counts, offs, ntiles);
    (void)cursor;
    return hipGetLastError();
}

hipError_t prk_launch_fill(const prk::FrameParams *fp, const void *ranges, const uint32_t *offs,
                           uint32_t *cursor, uint32_t *bins, hipStream_t s) {
    if (fp->tri_count == 0) return hipSuccess;
    const dim3 grid((fp->tri_count + 255) / 256);
    hipLaunchKernelGGL(prk::k_bin_fill, grid, dim3(256), 0, s, *fp,
                       reinterpret_cast<const prk::TileRange *>(ranges), offs, cursor, bins);
    return hipGetLastError();
}

hipError_t prk_launch_raster(const prk::FrameParams *fp, int modeset, const uint32_t *offs,
                             const uint32_t *bins, hipStream_t s) {
    const uint32_t ntile = (uint32_t)(fp->tiles_x * fp->tiles_y);
    if (ntile == 0) return hipSuccess;
    const size_t lds = (size_t)fp->tile_w * fp->tile_h * (sizeof(unsigned long long) + sizeof(uint32_t));
    switch (modeset) {
        case prk::MODE_AVX:
            hipLaunchKernelGGL(prk::k_raster<prk::MODE_AVX>, dim3(ntile), dim3(256), lds, s, *fp, offs, bins);
            break;
        case prk::MODE_SC_GOURAUD:
            hipLaunchKernelGGL(prk::k_raster<prk::MODE_SC_GOURAUD>, dim3(ntile), dim3(256), lds, s, *fp, offs,
                               bins);
            break;
        case prk::MODE_SC_PHONG:
            hipLaunchKernelGGL(prk::k_raster<prk::MODE_SC_PHONG>, dim3(ntile), dim3(256), lds, s, *fp, offs,
                               bins);
            break;
        default:
            hipLaunchKernelGGL(prk::k_raster<-1>, dim3(ntile), dim3(256), lds, s, *fp, offs, bins);
            break;
    }
    return hipGetLastError();
}

}  // extern "C"
