// prk_bin.hip — triangle -> tile binning with bins in submission order.
//
//   k_bin_count   1 thread / triangle: ProjectVertex + back-face cull
//                 (projekt.cpp:74-93, 3926-3943) -> conservative tile range ->
//                 number of (triangle, tile) entries (+ the setup records of
//                 all-AVX frames); k_bin_band the same for a row band.
//   k_cs_*        counting sort of the (triangle, pair) entries into tile
//                 bins, every size on the device (below).
//
// Pairs are numbered in triangle (= submission) order: the pair index is the
// visibility sweep's tie-break key, and k_walk / k_pix address span records
// by (pair, row).  (Scattering pairs into bins with global atomic counters
// instead of sorting measured 3x slower: device-scope atomics on 4096 hot
// counters.)
#include <algorithm>
#include <atomic>

#include "prk_device.h"

namespace prk {

// Conservative tile range of a triangle's covered pixels.  Span end points
// are edge-DDA values that stay on their segment up to float error
// (DESIGN.md §4.1), so [min x, max x] of the projected vertices widened by
// that error bounds every covered pixel; rows lie in [floor(min y), ceil(max y)).
__device__ __forceinline__ bool tri_tile_range_proj(const FrameParams &fp, const DrawRec *d, const V3 *proj,
                                                    TileRange &tr);
__device__ __forceinline__ bool tri_tile_range(const FrameParams &fp, uint32_t g, TileRange &tr) {
    const DrawRec *d;
    uint32_t gt;
    resolve_draw(fp, g, d, gt);
    V3 cam[3], proj[3];
    load_positions(*d, gt, fp, cam, proj);
    return tri_tile_range_proj(fp, d, proj, tr);
}
// The same from triangle g's nine position floats already loaded (v).
__device__ __forceinline__ bool tri_tile_range_raw(const FrameParams &fp, const DrawRec *d, const float *v,
                                                   TileRange &tr) {
    V3 proj[3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        proj[k] = project_vertex(V3{v[3 * k + 0] + d->P[0], v[3 * k + 1] + d->P[1], v[3 * k + 2] + d->P[2]}, fp);
    return tri_tile_range_proj(fp, d, proj, tr);
}
__device__ __forceinline__ bool tri_tile_range_proj(const FrameParams &fp, const DrawRec *d, const V3 *proj,
                                                    TileRange &tr) {
    const float ymin = fminf(proj[0].y, fminf(proj[1].y, proj[2].y));
    const float ymax = fmaxf(proj[0].y, fmaxf(proj[1].y, proj[2].y));
    const float fr0 = floorf(ymin), fr1 = ceilf(ymax);
    // No row of the band (nor, for scalar draws, the row-overflow store one
    // row down): no entries whatever the cull says, so skip its two
    // normalisations (row bands: most triangles lie outside a rank's band).
    if (fr1 + 1.0f <= (float)fp.row0 || fr0 >= (float)fp.row1) return false;
    if (!front_facing(proj)) return false;  // also rejects every non-finite vertex
    const float xmin = fminf(proj[0].x, fminf(proj[1].x, proj[2].x));
    const float xmax = fmaxf(proj[0].x, fmaxf(proj[1].x, proj[2].x));
    const int32_t r0 = fr0 < (float)fp.row0 ? fp.row0 : (fr0 >= (float)fp.row1 ? fp.row1 : (int32_t)fr0);
    const int32_t r1 = fr1 > (float)fp.row1 ? fp.row1 : (fr1 <= (float)fp.row0 ? fp.row0 : (int32_t)fr1);
    const float maxabs = fmaxf(fabsf(xmin), fabsf(xmax));
    const float slack = 2.0f + ((ymax - ymin) + 4.0f) * maxabs * (1.0f / 2097152.0f);  // 2^-21
    const float fc0 = floorf(xmin - slack), fc1 = ceilf(xmax + slack) + 1.0f;
    int32_t c0, c1;
    if (d->mode == MODE_AVX) {
        // Half-open [MinX, MaxX): a span clamped wholly to one side is empty.
        c0 = fc0 < 0.0f ? 0 : (fc0 >= (float)fp.W ? fp.W : (int32_t)fc0);
        c1 = fc1 > (float)fp.W ? fp.W : (fc1 <= 0.0f ? 0 : (int32_t)fc1);
    } else {
        // DrawModel's inclusive [MinX, MaxX] after clamping both ends to
        // [0, W-1] (projekt.cpp:381-425): a triangle left of the screen still
        // draws column 0, one right of it column W-1.
        c0 = fc0 < 0.0f ? 0 : (fc0 >= (float)(fp.W - 1) ? fp.W - 1 : (int32_t)fc0);
        c1 = fc1 > (float)fp.W ? fp.W : (fc1 <= 1.0f ? 1 : (int32_t)fc1);
    }
    tr.oty0 = 1;
    tr.oty1 = 0;
    tr.pad0 = (uint16_t)min(r0 - fp.row0, 65535);  // band rows [r0, r1): the bins' row classes
    tr.pad1 = (uint16_t)min(r1 - fp.row0, 65535);
    const bool rect = r0 < r1 && c0 < c1;
    if (rect) {
        tr.tx0 = (uint16_t)(c0 >> fp.tile_w_log2);
        tr.tx1 = (uint16_t)((c1 - 1) >> fp.tile_w_log2);
        tr.ty0 = (uint16_t)tile_row_of(fp, r0 - fp.row0);
        tr.ty1 = (uint16_t)tile_row_of(fp, r1 - 1 - fp.row0);
    } else {
        tr.tx0 = 1; tr.tx1 = 0; tr.ty0 = 1; tr.ty1 = 0;
    }
    if (d->mode != MODE_AVX && fc1 >= (float)fp.W) {
        // A span ending at MaxX == W stores pixel (row+1, 0): rows shift by one.
        const float lim = (float)min(fp.row1, fp.H);
        const float g0 = fr0 + 1.0f, g1 = fr1 + 1.0f;
        const int32_t o0 = g0 < (float)fp.row0 ? fp.row0 : (g0 >= lim ? (int32_t)lim : (int32_t)g0);
        const int32_t o1 = g1 > lim ? (int32_t)lim : (g1 <= (float)fp.row0 ? fp.row0 : (int32_t)g1);
        if (o0 < o1) {
            tr.oty0 = (uint16_t)tile_row_of(fp, o0 - fp.row0);
            tr.oty1 = (uint16_t)tile_row_of(fp, o1 - 1 - fp.row0);
        }
    }
    return rect || tr.oty0 <= tr.oty1;
}

// Quick band test of k_bin_band: true only when the exact test above rejects
// the triangle at its first line (no row of the band): every vertex's
// projected y, here with the hardware reciprocal in place of ProjectVertex's
// IEEE division (<= 1 ulp, so the two differ by well under 2^-18 of the
// magnitudes), lies more than that bound plus two rows outside the band on
// the same side.  A non-finite value fails every comparison: never rejected
// here.  py, pz: the draw's object position P[1], P[2].
__device__ __forceinline__ bool band_far(const FrameParams &fp, float py, float pz, const float *v) {
    bool above = true, below = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float cy = v[3 * k + 1] + py, cz = v[3 * k + 2] + pz;
        const float dd = fp.D - cz;
        float y = 0.0f, m = 0.0f;  // (project_vertex's y of a vertex with dd <= 0.2)
        if (dd > 0.2f) {
            const float t = fp.M2P * ((__builtin_amdgcn_rcpf(dd) * fp.F) * cy);
            y = fp.Cy + t;
            m = (fabsf(t) + fabsf(fp.Cy)) * 0x1p-18f;
        }
        above = above && (y + m + 2.0f < (float)fp.row0);
        below = below && (y - m >= (float)fp.row1 + 1.0f);
    }
    return above || below;
}

// Number of tiles in a range (rectangle + column-0 overflow tiles not in it).
__device__ __forceinline__ uint32_t range_entries(const TileRange &tr) {
    uint32_t n = 0;
    if (tr.tx0 <= tr.tx1 && tr.ty0 <= tr.ty1) n = (uint32_t)(tr.tx1 - tr.tx0 + 1) * (tr.ty1 - tr.ty0 + 1);
    for (int ty = tr.oty0; ty <= tr.oty1; ++ty)
        if (!(tr.tx0 == 0 && tr.tx0 <= tr.tx1 && ty >= tr.ty0 && ty <= tr.ty1)) ++n;
    return n;
}

#ifndef PRK_ROWCLASS
#define PRK_ROWCLASS 1
#endif
constexpr int kRowClassBits = 3;

// The setup record of triangle g of an all-AVX frame: FillEdgeTable +
// MergeSort + the first row's AET insertions once per triangle (TriRec,
// prk_device.h).
__device__ __forceinline__ void make_rec(const FrameParams &fp, uint32_t g, TriRec &r) {
    const DrawRec *d;
    uint32_t gt;
    resolve_draw(fp, g, d, gt);
    Edge s0, s1, s2;
    TriRaw<MODE_AVX> raw;
    load_tri<MODE_AVX>(*d, gt, raw);
    const int n = setup_from_raw<MODE_AVX>(raw, *d, fp, s0, s1, s2);
    uint32_t anom = 0;
    Walker<MODE_AVX, true> w;
    w.init(n, s0, s1, s2, fp.H, fp.H, anom);
    rec_edge_out(s0, r.e[0], r.ymin[0], r.ymax[0]);
    rec_edge_out(s1, r.e[1], r.ymin[1], r.ymax[1]);
    rec_edge_out(s2, r.e[2], r.ymin[2], r.ymax[2]);
    r.head = (uint32_t)n | (w.ord << 4) | ((uint32_t)w.cnt << 12) | ((uint32_t)(w.pend + 1) << 16) |
             (min(anom, 15u) << 20) | ((d->flags & DRAW_ST) ? (1u << 24) : 0u);
    r.vtx = (uint32_t)s0.Vtx | ((uint32_t)s1.Vtx << 4) | ((uint32_t)s2.Vtx << 8);
    r.pad[0] = r.pad[1] = 0;
}

// Records leave through LDS: a wave's 64 records are written out as
// consecutive 16-byte chunks (one coalesced store per 64 chunks when the
// wave's triangles are consecutive) instead of ten 160-byte-strided stores
// per lane.
constexpr int kCountThreads = 256;
__device__ __forceinline__ void store_recs(const FrameParams &fp, float4 *st, bool rec, const TriRec &r, uint32_t g) {
    const int lane = threadIdx.x & 63;
    const uint64_t mask = __ballot(rec);
    if (mask == 0) return;
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    if (rec) {
        const float4 *sr = reinterpret_cast<const float4 *>(&r);
#pragma unroll
        for (int k = 0; k < 10; ++k) st[lane * 10 + k] = sr[k];
    }
    wave_sync();
    for (int c = lane; c < 64 * 10; c += 64) {
        const int src = c / 10;
        const uint32_t gs = (uint32_t)__shfl((int)g, src);
        if ((mask >> src) & 1) reinterpret_cast<float4 *>(fp.trec + gs)[c - src * 10] = st[c];
    }
    wave_sync();
}

// Band test, cull, tile range and entry count of every triangle, and (recs)
// the setup records of the triangles with entries: whole-frame targets and
// the radix-sort binning.  A row band's counting-sort binning computes its
// records in k_setup_rec instead.
__global__ void __launch_bounds__(kCountThreads) k_bin_count(FrameParams fp, uint32_t *__restrict__ tri_n,
                                                              TileRange *__restrict__ ranges, bool recs) {
    __shared__ float4 stage[kCountThreads / 64][64 * 10];
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const int wv = threadIdx.x >> 6;
    bool rec = false;
    TriRec r;
    if (g < fp.tri_count) {
        TileRange tr;
        if (!tri_tile_range(fp, g, tr)) {
            tr.tx0 = 1; tr.tx1 = 0; tr.ty0 = 1; tr.ty1 = 0; tr.oty0 = 1; tr.oty1 = 0;
        }
        ranges[g] = tr;
        const uint32_t ne = range_entries(tr);
        tri_n[g] = ne;
        rec = recs && fp.trec && ne;
    } else if (g == fp.tri_count) {
        tri_n[g] = 0;  // sentinel: a scan's last element is the total
    }
    if (!recs) return;
    if (rec) make_rec(fp, g, r);
    store_recs(fp, stage[wv], rec, r, g);
}

// The setup records of the triangles with entries, one workgroup per run of
// kRecRun triangles: the run's triangles with entries are listed in LDS (in
// triangle order, a workgroup scan per 256) and set up 64 per wave, so the
// lanes stay full when few of them have entries — a row band's rank (C3b at
// N = 8: with the records computed in k_bin_count, a wave holding a few of
// the band's triangles ran the whole setup at a few lanes, 99 us of a
// 0.30 ms band frame).
constexpr uint32_t kRecRun = 2048;
#ifndef PRK_BIN_BAND
#define PRK_BIN_BAND 1  // row bands: k_bin_band (one launch) instead of k_bin_count + k_setup_rec
#endif
#ifndef PRK_WPROF
#define PRK_WPROF 0
#endif
#ifndef PRK_BAND_REC_KERNEL
#define PRK_BAND_REC_KERNEL 1  // a row band's setup records in k_band_rec (prk_band_records), not k_bin_band
#endif
#ifndef PRK_BAND_COALESCED
#define PRK_BAND_COALESCED 1  // k_bin_band: a one-draw run's positions as coalesced float4 loads through LDS
#endif
__device__ uint32_t cs_block_excl_scan(uint32_t v, uint32_t *scratch, uint32_t &total);
__global__ void __launch_bounds__(kCountThreads) k_setup_rec(FrameParams fp, const uint32_t *__restrict__ tri_n) {
    __shared__ float4 stage[kCountThreads / 64][64 * 10];
    __shared__ uint32_t list[kRecRun];
    __shared__ uint32_t scratch[kCountThreads / 64];
    const uint32_t g0 = blockIdx.x * kRecRun;
    uint32_t n = 0;
    for (uint32_t k = 0; k < kRecRun; k += kCountThreads) {
        const uint32_t g = g0 + k + threadIdx.x;
        const uint32_t f = g < fp.tri_count && tri_n[g] != 0 ? 1u : 0u;
        uint32_t tot;
        const uint32_t pos = cs_block_excl_scan(f, scratch, tot);
        if (f) list[n + pos] = g;
        n += tot;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t b = (uint32_t)wv * 64; b < n; b += kCountThreads) {
        const uint32_t i = b + lane;
        const bool rec = i < n;
        const uint32_t g = rec ? list[i] : 0u;
        TriRec r;
        if (rec) make_rec(fp, g, r);
        store_recs(fp, stage[wv], rec, r, g);
    }
}

// A row band's triangle pass: each workgroup takes a run of kRecRun
// triangles, tests every one against the band (a quick test, then the full
// tile range of the ones it keeps), writes the tile range and entry count of
// the ones with entries and lists them in triangle order
// (runlist[run * kRecRun + i], run_n[run]): the band's counting sort walks
// only those (BandRuns), and k_band_rec sets up their records (in this
// kernel, 64 per wave, with -DPRK_BAND_REC_KERNEL=0).  It clears the frame's
// won flag of every triangle of the run (trwon, span-record frames).
// (Round 2: k_bin_count + k_setup_rec, C3b at N = 8 20 + 23 us serial, each
// reading the band test's inputs of all 1 M triangles; round 5: this kernel
// with the records, 37 us; round 6: 17.7 us + k_band_rec beside the sort.)
struct BandRuns {
    const uint32_t *list;  // per run of kRecRun triangles: its triangles with entries, in order
    const uint32_t *n;     // per run: how many
    uint32_t nruns;
    uint32_t per;          // runs per counting-sort chunk
};
__global__ void __launch_bounds__(kCountThreads) k_bin_band(FrameParams fp, uint32_t *__restrict__ tri_n,
                                                             TileRange *__restrict__ ranges,
                                                             uint32_t *__restrict__ runlist,
                                                             uint32_t *__restrict__ run_n,
                                                             uint8_t *__restrict__ trwon) {
    __shared__ float4 stage[kCountThreads / 64][64 * 10];
    __shared__ uint32_t list[kRecRun];
    const uint32_t g0 = blockIdx.x * kRecRun;
    uint32_t n = 0;
    constexpr int kWaves = kCountThreads / 64;
    // -DPRK_WPROF=1: wave 0's clocks per phase (0 first half in, 1 tested, 2
    // second half in, 3 tested, 4 lists joined, 5 records) into fp.prof
    unsigned long long bt[6] = {}, bt0 = PRK_WPROF ? __builtin_amdgcn_s_memtime() : 0ull;
    const unsigned long long rt0 = PRK_WPROF ? __builtin_amdgcn_s_memrealtime() : 0ull;
#define PRK_BT(k)                                                   \
    do {                                                            \
        if (PRK_WPROF) {                                            \
            const unsigned long long t1_ = __builtin_amdgcn_s_memtime(); \
            bt[k] += t1_ - bt0;                                     \
            bt0 = t1_;                                              \
        }                                                           \
    } while (0)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // The run's positions, a half (kHalf triangles) at a time, go through LDS
    // (the record stage's space), nine floats per triangle.  One draw whose
    // run is 16-byte aligned in its geometry (the usual frame): the half's
    // 9 * kHalf floats are contiguous and come in as coalesced float4 loads (a
    // wave instruction reads 1 KiB in a row).  Otherwise each thread loads
    // its triangles' nine floats (any draw) and stores them there.
    constexpr int kHalf = kRecRun / 2;                  // triangles per LDS half
    constexpr int kPerWave = kHalf / kWaves;            // a wave's consecutive triangles per half
    constexpr int kV4 = kHalf * 9 / 4 / kCountThreads;  // float4 per thread per half
    static_assert(kHalf * 9 % (4 * kCountThreads) == 0 && kHalf * 9 * 4 <= (int)sizeof(stage), "LDS half");
    static_assert(kPerWave == kCountThreads && kPerWave % 64 == 0, "one list entry per thread and (half, wave)");
    const uint32_t gt0 = fp.draw0.geom_tri0 + (g0 - fp.draw0.first_global);
    // (gt0 % 4 == 0 makes the run's offset 16-B aligned; the base must be too:
    // prk_geometry_wrap_device takes any 4-B aligned caller pointer)
    const bool coal = PRK_BAND_COALESCED && fp.ndraws == 1 && (gt0 & 3u) == 0 &&
                      ((uintptr_t)fp.draw0.V & 15u) == 0 &&
                      g0 + (uint32_t)kRecRun <= fp.tri_count;  // (a whole run: no tail to mask)
    // Wave w takes kPerWave consecutive triangles of each half: first the
    // quick band test (band_far) over all of them, the ones it keeps listed
    // in surv[w] in order; then the full test (tri_tile_range_raw, ~500
    // instructions) over those 64 at a time, so a narrow band's rank runs it
    // at full lanes on about its share of the triangles instead of on every
    // one.  The triangles with entries go to the (half, wave) list, in list[]
    // at half * kHalf + wave * kPerWave, its length in wcnt: in triangle
    // order, so the eight lists joined in that order are the run's.
    __shared__ uint16_t surv[kWaves][kPerWave];
    __shared__ uint32_t wcnt[2][kWaves];
    float *lw = reinterpret_cast<float *>(&stage[0][0]);
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    for (int h = 0; h < 2; ++h) {
        const uint32_t hb = (uint32_t)h * kHalf;  // the half's first triangle in the run
        if (h) {
            PRK_BT(1);
            __syncthreads();  // (the previous half's reads)
        }
        if (coal) {
            const float4 *src = reinterpret_cast<const float4 *>(fp.draw0.V + 9 * ((size_t)gt0 + hb));
            float4 *lv = &stage[0][0];
#pragma unroll
            for (int kk = 0; kk < kV4; ++kk) lv[kk * kCountThreads + threadIdx.x] = src[kk * kCountThreads + threadIdx.x];
        } else {
            constexpr int kT = kHalf / kCountThreads;
            float pv[kT][9];
#pragma unroll
            for (int k = 0; k < kT; ++k) {  // (all requested before any is stored: the loads overlap)
                const uint32_t g = g0 + hb + k * kCountThreads + threadIdx.x;
                if (g < fp.tri_count) {
                    const DrawRec *d;
                    uint32_t gt;
                    resolve_draw(fp, g, d, gt);
                    const float *v = d->V + 9 * (size_t)gt;
#pragma unroll
                    for (int j = 0; j < 9; ++j) pv[k][j] = v[j];
                }
            }
#pragma unroll
            for (int k = 0; k < kT; ++k)
#pragma unroll
                for (int j = 0; j < 9; ++j) lw[9 * (k * kCountThreads + threadIdx.x) + j] = pv[k][j];
        }
        __syncthreads();
        PRK_BT(h ? 2 : 0);
        uint32_t ns = 0;  // this wave's kept triangles
#pragma unroll
        for (int k = 0; k < kPerWave / 64; ++k) {
            const uint32_t t = (uint32_t)(wv * kPerWave + k * 64 + lane), g = g0 + hb + t;
            bool keep = false;
            if (g < fp.tri_count) {
                if (trwon) trwon[g] = 0;
                float py = fp.draw0.P[1], pz = fp.draw0.P[2];
                if (!coal) {
                    const DrawRec *d;
                    uint32_t gt;
                    resolve_draw(fp, g, d, gt);
                    py = d->P[1];
                    pz = d->P[2];
                }
                keep = !band_far(fp, py, pz, lw + 9 * t);
            } else if (g == fp.tri_count) {
                tri_n[g] = 0;  // sentinel: a scan's last element is the total
            }
            const unsigned long long bal = __ballot(keep);
            const uint32_t r = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (keep) surv[wv][ns + r] = (uint16_t)t;
            ns += (uint32_t)__popcll(bal);
        }
        wave_sync();
        uint32_t wn = 0;  // this wave's list length in this half
        for (uint32_t b = 0; b < ns; b += 64) {
            const uint32_t i = b + (uint32_t)lane;
            uint32_t ne = 0, g = 0;
            if (i < ns) {
                const uint32_t t = surv[wv][i];
                g = g0 + hb + t;
                const DrawRec *d = fp.draws;
                if (!coal) {
                    uint32_t gt;
                    resolve_draw(fp, g, d, gt);
                }
                float v9[9];
#pragma unroll
                for (int j = 0; j < 9; ++j) v9[j] = lw[9 * t + j];
                TileRange tr;
                if (!tri_tile_range_raw(fp, d, v9, tr)) {
                    tr.tx0 = 1; tr.tx1 = 0; tr.ty0 = 1; tr.ty1 = 0; tr.oty0 = 1; tr.oty1 = 0;
                }
                ne = range_entries(tr);
                if (ne) {  // (only the listed triangles' are read: the band's sort, k_won_local of winners)
                    ranges[g] = tr;
                    tri_n[g] = ne;
                }
            }
            const unsigned long long bal = __ballot(ne != 0);
            const uint32_t r = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (ne) list[hb + wv * kPerWave + wn + r] = g;
            wn += (uint32_t)__popcll(bal);
        }
        if (lane == 0) wcnt[h][wv] = wn;
    }
    {
        // join the eight (half, wave) lists in order: run list out, and the
        // joined list for the records below
        PRK_BT(3);
        __syncthreads();
        uint32_t off[2][kWaves];
        n = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                off[h][w] = n;
                n += wcnt[h][w];
            }
        // (each list holds <= kHalf / kWaves = kCountThreads entries: thread t
        // moves entry t of each; every entry moves down or stays, so all are
        // read before any is written)
        static_assert(kHalf / kWaves == kCountThreads, "one entry per thread and list");
        uint32_t v[2][kWaves];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int w = 0; w < kWaves; ++w)
                v[h][w] = threadIdx.x < wcnt[h][w] ? list[h * kHalf + w * (kHalf / kWaves) + threadIdx.x] : 0u;
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int w = 0; w < kWaves; ++w)
                if (threadIdx.x < wcnt[h][w]) {
                    list[off[h][w] + threadIdx.x] = v[h][w];
                    runlist[g0 + off[h][w] + threadIdx.x] = v[h][w];
                }
    }
    if (threadIdx.x == 0) run_n[blockIdx.x] = n;
    __syncthreads();
    PRK_BT(4);
    if (fp.trec && !PRK_BAND_REC_KERNEL)
        for (uint32_t b = (uint32_t)wv * 64; b < n; b += kCountThreads) {
            const uint32_t i = b + lane;
            const bool rec = i < n;
            const uint32_t g = rec ? list[i] : 0u;
            TriRec r;
            if (rec) make_rec(fp, g, r);
            store_recs(fp, stage[wv], rec, r, g);
        }
    if (PRK_WPROF) {
        __syncthreads();
        PRK_BT(5);
        if (threadIdx.x == 0) {
            const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
            for (int k = 0; k < 6; ++k) atomicAdd(fp.prof + k, bt[k]);
            atomicAdd(fp.prof + 6, 1ull);
            atomicAdd(fp.prof + 7, (unsigned long long)n);
            atomicMax(fp.prof + 8, ~rt0);
            atomicMax(fp.prof + 9, rt1);
            atomicAdd(fp.prof + 10, rt1 - rt0);
        }
    }
}

// A row band's setup records (PRK_BAND_REC_KERNEL): k_bin_band lists each
// run's triangles with entries (runlist, run_n); workgroup (run, w), one
// wave, sets up entries [64 w, 64 w + 64) of run `run`'s list.  Inside
// k_bin_band a run's ~260 listed triangles (C3b at N = 8) took two rounds of
// its four waves, 50 k of its 80 k clocks; here every wave but a run's last
// is full, and the launch runs on the vis stream beside the band's counting
// sort (prk_api.hip), which does not read the records.
__global__ void __launch_bounds__(64) k_band_rec(FrameParams fp, const uint32_t *__restrict__ runlist,
                                                 const uint32_t *__restrict__ run_n) {
    __shared__ float4 stage[64 * 10];
    const uint32_t run = blockIdx.x, b = blockIdx.y * 64u;
    const uint32_t n = run_n[run];
    if (b >= n) return;
    const uint32_t i = b + (threadIdx.x & 63u);
    const bool rec = i < n;
    const uint32_t g = rec ? runlist[(size_t)run * kRecRun + i] : 0u;
    TriRec r;
    if (rec) make_rec(fp, g, r);
    store_recs(fp, stage, rec, r, g);
}

// Sort key = tile << kRowClassBits | row class: within a tile's bin the
// pairs are grouped by how many of the tile's rows the triangle can cover
// (bin order is free: the pair index breaks visibility ties), so the 64
// triangles a k_vis wave walks together cover similar row counts.
// It also clears the frame's won flags of its pairs (won_stride bytes per
// pair) and of its triangle (trwon, span-record frames), which k_vis sets.
__device__ __forceinline__ void clear_won(uint8_t *__restrict__ won, uint32_t stride, uint32_t o) {
    if (stride == 8) *reinterpret_cast<uint64_t *>(won + (size_t)o * 8) = 0;
    else
        for (uint32_t i = 0; i < stride; ++i) won[(size_t)o * stride + i] = 0;
}



// ---------------------------------------------------------------------------
// Counting-sort binning (the default when the frame has at most kCsMaxTiles
// tiles): no radix sort, no host round trip before the bin kernels.
//
//   k_bin_count   as above (ranges, per-triangle counts, setup records)
//   k_cs_hist     one workgroup per chunk of kCsChunk triangles: LDS histogram
//                 of the chunk's entries per tile -> ghist[chunk][tile], and
//                 the chunk's entry total
//   k_cs_colscan  per tile, exclusive prefix over the chunks (in place) and
//                 the tile's total
//   k_cs_scan     one workgroup: tile offsets (bin starts), chunk pair bases,
//                 the frame's entry count; an entry count above the scratch
//                 capacity empties every bin (the host re-runs the frame)
//   k_cs_emit     one workgroup per chunk: pair offsets of its triangles in
//                 triangle order (pair j = the tie-break key), and each entry
//                 scattered into its tile's bin through an LDS cursor
//   k_cs_class    one workgroup per tile: the bin grouped by row class (how
//                 many of the tile's rows the triangle can cover), so the 64
//                 triangles a k_vis wave walks together cover similar row
//                 counts (k_vis -13 % against no grouping, measured)
//
// The order inside a bin is free (the pair index, not the bin position,
// orders equal-z fragments), so the LDS cursors need no ordering.
// ---------------------------------------------------------------------------
constexpr int kCsThreads = 1024;
constexpr uint32_t kCsTrisPerThread = 4;
constexpr uint32_t kCsChunk = kCsThreads * kCsTrisPerThread;
constexpr uint32_t kCsMaxTiles = 32768;  // LDS: one u32 per tile (128 KiB)
#ifndef PRK_REPCLASS
#define PRK_REPCLASS 0  // 1: bins also grouped by how many tile rows of the triangle lie above the
                        // tile (its replay length); measured k_vis +6 % on C3b (0.497 -> 0.528 ms)
#endif
constexpr int kRepClassBits = PRK_REPCLASS ? 2 : 0;
constexpr int kClassBits = kRowClassBits + kRepClassBits;
constexpr uint32_t kCsClassShift = 32 - kClassBits;  // (replay, row) class in the top bits of the emitted pair index
constexpr uint32_t kCsPairMask = (1u << kCsClassShift) - 1u;
constexpr int kCsClassWindow = 2048;     // k_cs_class: entries grouped per pass

__device__ __forceinline__ uint32_t cs_wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}

// Exclusive scan over the workgroup (one value per thread); `total` = sum.
// scratch: one u32 per wave.
__device__ __forceinline__ uint32_t cs_block_excl_scan(uint32_t v, uint32_t *scratch, uint32_t &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t incl = cs_wave_incl_scan(v);
    if (lane == 63) scratch[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    total = 0;
    for (int w = 0; w < nw; ++w) {
        const uint32_t x = scratch[w];
        before += w < wave ? x : 0u;
        total += x;
    }
    __syncthreads();
    return before + incl - v;
}

// The (tile, class) of every entry of a range, in pair order: the rectangle
// row-major, then the column-0 overflow tiles not in it.  Class = the rows
// of the tile the triangle can cover (k_vis's row walk) and, above it, how
// many tile rows of the triangle lie above the tile (its replay of the rows
// above: 0, 1, 2, 3+), so the 64 entries of a k_vis wave walk and replay
// about as many rows each.
template <class F>
__device__ __forceinline__ void for_each_entry(const FrameParams &fp, const TileRange &tr, F &&f) {
    constexpr int kMaxClass = (1 << kRowClassBits) - 1;
    constexpr int kMaxRep = (1 << kRepClassBits) - 1;
    if (tr.tx0 <= tr.tx1 && tr.ty0 <= tr.ty1)
        for (int ty = tr.ty0; ty <= tr.ty1; ++ty) {
            const int y0 = ty * fp.tile_h;
            const int rows = min((int)tr.pad1, y0 + fp.tile_h) - max((int)tr.pad0, y0);
            uint32_t cls = PRK_ROWCLASS ? (uint32_t)min(kMaxClass, max(0, fp.tile_h - rows)) : 0u;
            const int rep = max(0, y0 - (int)tr.pad0);
            cls |= (uint32_t)min(kMaxRep, tile_row_of(fp, rep + fp.tile_h - 1)) << kRowClassBits;
            for (int tx = tr.tx0; tx <= tr.tx1; ++tx) f((uint32_t)(ty * fp.tiles_x + tx), cls);
        }
    for (int ty = tr.oty0; ty <= tr.oty1; ++ty)
        if (!(tr.tx0 == 0 && tr.tx0 <= tr.tx1 && ty >= tr.ty0 && ty <= tr.ty1))
            f((uint32_t)(ty * fp.tiles_x), PRK_ROWCLASS ? (uint32_t)((kMaxRep << kRowClassBits) | kMaxClass) : 0u);
}

// The triangles of counting-sort chunk c, in order, kCsThreads at a time:
// a whole frame's chunk is kCsChunk consecutive triangles; a row band's (BandRuns)
// is the listed triangles of runs [c * per, (c + 1) * per) — those with entries.
struct ChunkTris {
    uint32_t g0, count;       // whole frame: triangles [g0, g0 + count)
    const uint32_t *list;     // band: null, or the chunk's runs' lists
    uint32_t r0, nr;          // band: runs [r0, r0 + nr)
    uint32_t pre[65];         // band: prefix of the runs' counts (per <= 64)
};
constexpr uint32_t kMaxRunsPerChunk = 64;
__device__ __forceinline__ void chunk_tris(const FrameParams &fp, const BandRuns &br, uint32_t c, ChunkTris &ct) {
    if (threadIdx.x == 0) {
        ct.list = br.list;
        if (!br.list) {
            ct.g0 = c * kCsChunk;
            ct.count = ct.g0 < fp.tri_count ? min(kCsChunk, fp.tri_count - ct.g0) : 0u;
        } else {
            ct.r0 = c * br.per;
            ct.nr = min(br.per, br.nruns - ct.r0);
            uint32_t run = 0;
            for (uint32_t k = 0; k < ct.nr; ++k) {
                ct.pre[k] = run;
                run += br.n[ct.r0 + k];
            }
            ct.pre[ct.nr] = run;
            ct.count = run;
        }
    }
    __syncthreads();
}
// The p-th triangle of the chunk (p < count).
__device__ __forceinline__ uint32_t chunk_tri(const ChunkTris &ct, uint32_t p) {
    if (!ct.list) return ct.g0 + p;
    uint32_t k = 0;
    while (k + 1 < ct.nr && ct.pre[k + 1] <= p) ++k;
    return ct.list[(size_t)(ct.r0 + k) * kRecRun + (p - ct.pre[k])];
}

__global__ void __launch_bounds__(kCsThreads) k_cs_hist(FrameParams fp, const TileRange *__restrict__ ranges,
                                                         const uint32_t *__restrict__ tri_n,
                                                         uint32_t *__restrict__ ghist,
                                                         uint32_t *__restrict__ chunk_tot, uint32_t ntiles,
                                                         BandRuns br) {
    extern __shared__ uint32_t h[];
    __shared__ uint32_t scratch[kCsThreads / 64];
    __shared__ ChunkTris ct;
    for (uint32_t i = threadIdx.x; i < ntiles; i += kCsThreads) h[i] = 0;
    const uint32_t c = blockIdx.x;
    chunk_tris(fp, br, c, ct);  // (its barrier also orders the zeroed histogram)
    __syncthreads();
    uint32_t sum = 0;
    for (uint32_t p = threadIdx.x; p < ct.count; p += kCsThreads) {
        const uint32_t g = chunk_tri(ct, p);
        const uint32_t n = tri_n[g];
        if (!n) continue;
        sum += n;
        const TileRange tr = ranges[g];
        for_each_entry(fp, tr, [&](uint32_t tile, uint32_t) { atomicAdd(&h[tile], 1u); });
    }
    uint32_t tot;
    (void)cs_block_excl_scan(sum, scratch, tot);  // (its barriers also order the LDS histogram)
    if (threadIdx.x == 0) chunk_tot[c] = tot;
    uint32_t *out = ghist + (size_t)c * ntiles;
    for (uint32_t i = threadIdx.x; i < ntiles; i += kCsThreads) out[i] = h[i];
}

// 1024 threads = 64 tiles x 16 chunk segments; lane = tile, wave = segment.
constexpr int kColSegs = 16;
__global__ void __launch_bounds__(64 * kColSegs) k_cs_colscan(uint32_t *__restrict__ ghist, uint32_t nchunks,
                                                               uint32_t ntiles, uint32_t *__restrict__ tile_tot) {
    __shared__ uint32_t seg[kColSegs][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t t = blockIdx.x * 64 + lane;
    const uint32_t per = (nchunks + kColSegs - 1) / kColSegs, c0 = min(nchunks, w * per), c1 = min(nchunks, c0 + per);
    uint32_t s = 0;
    if (t < ntiles)
        for (uint32_t c = c0; c < c1; ++c) s += ghist[(size_t)c * ntiles + t];
    seg[w][lane] = s;
    __syncthreads();
    uint32_t run = 0;
    for (uint32_t k = 0; k < w; ++k) run += seg[k][lane];
    if (t < ntiles) {
        for (uint32_t c = c0; c < c1; ++c) {
            const size_t i = (size_t)c * ntiles + t;
            const uint32_t v = ghist[i];
            ghist[i] = run;
            run += v;
        }
        if (w == kColSegs - 1) tile_tot[t] = run;
    }
}

// One workgroup.  offs[0..ntiles] = exclusive scan of the tile totals (bin
// starts; offs[ntiles] = the frame's entry count), chunk_base = exclusive scan
// of the chunk totals; info[0] = entry count, info[1] = 1 if it exceeds `cap`
// (then every bin is left empty and k_cs_emit writes no pair).
// Exclusive scan of n values (n <= kCsThreads * kScanPer) by one workgroup:
// wave w scans the contiguous segment [w * kScanSeg, (w + 1) * kScanSeg),
// 64 values per load (coalesced) and one DPP wave scan per 64 with a running
// carry, then the wave totals are scanned across the workgroup.  (Round 2
// had each thread load kScanPer consecutive values: 64 cache lines per load
// instruction, and a one-workgroup kernel that waited on them — 12 us alone,
// 50-60 us when it shared its CU with k_vis / k_walk waves in a band frame.)
constexpr uint32_t kScanPer = kCsMaxTiles / kCsThreads;
constexpr uint32_t kScanSeg = kScanPer * 64;
__device__ __forceinline__ uint32_t cs_scan_small(const uint32_t *__restrict__ in, uint32_t n,
                                                  uint32_t *__restrict__ out, uint32_t *scratch, uint32_t base) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, s0 = wave * kScanSeg;
    uint32_t v[kScanPer], pre[kScanPer];
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        const uint32_t i = s0 + k * 64 + lane;
        v[k] = i < n ? in[i] : 0u;
    }
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        if (s0 + k * 64 >= n) break;  // (wave-uniform)
        const uint32_t incl = cs_wave_incl_scan(v[k]);
        pre[k] = carry + incl - v[k];
        carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    if (lane == 0) scratch[wave] = carry;
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t w = 0; w < (uint32_t)(blockDim.x >> 6); ++w) {
        const uint32_t x = scratch[w];
        before += w < wave ? x : 0u;
        tot += x;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        const uint32_t i = s0 + k * 64 + lane;
        if (s0 + k * 64 >= n) break;
        if (i < n) out[i] = base + before + pre[k];
    }
    return tot;
}

// One workgroup.  offs[0..ntiles] = exclusive scan of the tile totals (bin
// starts; offs[ntiles] = the frame's entry count), chunk_base = exclusive scan
// of the chunk totals; info[0] = entry count, info[1] = 1 if it exceeds `cap`
// (then every bin is left empty and k_cs_emit writes no pair).
__global__ void __launch_bounds__(kCsThreads) k_cs_scan(const uint32_t *__restrict__ tile_tot, uint32_t ntiles,
                                                         const uint32_t *__restrict__ chunk_tot, uint32_t nchunks,
                                                         uint32_t *__restrict__ offs,
                                                         uint32_t *__restrict__ chunk_base, uint32_t cap,
                                                         uint32_t *__restrict__ info) {
    __shared__ uint32_t scratch[kCsThreads / 64];
    const uint32_t total = cs_scan_small(tile_tot, ntiles, offs, scratch, 0u);
    const bool over = total > cap;
    uint32_t run = 0;  // chunk bases (more than one round past 128 M triangles)
    for (uint32_t b = 0; b < nchunks; b += kCsThreads * kScanPer)
        run += cs_scan_small(chunk_tot + b, min(nchunks - b, kCsThreads * kScanPer), chunk_base + b, scratch, run);
    if (over) {  // empty bins: the frame's raster draws nothing
        __syncthreads();
        for (uint32_t i = threadIdx.x; i <= ntiles; i += kCsThreads) offs[i] = 0;
    } else if (threadIdx.x == 0) {
        offs[ntiles] = total;
    }
    if (threadIdx.x == 0) {
        info[0] = total;
        info[1] = over ? 1u : 0u;
    }
}

// Workgroup b runs on XCD b % 8 (round-robin dispatch); XCD x takes the
// contiguous chunks [start(x), start(x+1)), so inside a tile's bin the
// entries one XCD writes are contiguous and its L2 merges them into whole
// lines (consecutive chunks on different XCDs left every line of a bin
// written partially by several L2s: 169 MB written for ~70 MB of data).
#ifndef PRK_CS_XCD
#define PRK_CS_XCD 1
#endif
__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t n) {
    if (!PRK_CS_XCD) return b;
    constexpr uint32_t kXcds = 8;
    const uint32_t q = n / kXcds, r = n % kXcds, x = b % kXcds;
    return x * q + min(x, r) + b / kXcds;
}

__global__ void __launch_bounds__(kCsThreads) k_cs_emit(FrameParams fp, const TileRange *__restrict__ ranges,
                                                         const uint32_t *__restrict__ tri_n,
                                                         const uint32_t *__restrict__ ghist,
                                                         const uint32_t *__restrict__ offs,
                                                         const uint32_t *__restrict__ chunk_base,
                                                         const uint32_t *__restrict__ info, uint32_t ntiles,
                                                         uint32_t *__restrict__ tri_off, uint2 *__restrict__ bins,
                                                         uint32_t *__restrict__ pair_tri, uint8_t *__restrict__ won,
                                                         uint32_t won_stride, uint8_t *__restrict__ trwon,
                                                         BandRuns br) {
    extern __shared__ uint32_t cur[];
    __shared__ uint32_t scratch[kCsThreads / 64];
    __shared__ ChunkTris ct;
    const uint32_t c = xcd_chunk(blockIdx.x, gridDim.x);
    const bool over = info[1] != 0;
    if (!over) {
        const uint32_t *gh = ghist + (size_t)c * ntiles;
        for (uint32_t i = threadIdx.x; i < ntiles; i += kCsThreads) cur[i] = offs[i] + gh[i];
    }
    chunk_tris(fp, br, c, ct);
    // (a band's run lists hold only triangles with entries; its trwon flags
    // were cleared by k_bin_band for every triangle)
    if (br.list) trwon = nullptr;
    uint32_t base = chunk_base[c];
    for (uint32_t p0 = 0; p0 < ct.count; p0 += kCsThreads) {
        const uint32_t p = p0 + threadIdx.x;
        const bool in = p < ct.count;
        const uint32_t g = in ? chunk_tri(ct, p) : 0u;
        const uint32_t n = in ? tri_n[g] : 0u;
        uint32_t tot;
        const uint32_t j0 = base + cs_block_excl_scan(n, scratch, tot);  // (also orders the cursor loads)
        base += tot;
        if (!in) continue;
        if (trwon) trwon[g] = 0;
        if (over) continue;
        tri_off[g] = j0;
        if (!n) continue;
        const TileRange tr = ranges[g];
        uint32_t j = j0;
        for_each_entry(fp, tr, [&](uint32_t tile, uint32_t cls) {
            const uint32_t pos = atomicAdd(&cur[tile], 1u);
            bins[pos] = make_uint2(g, j | (cls << kCsClassShift));
            pair_tri[j] = g;
            clear_won(won, won_stride, j);
            ++j;
        });
    }
    if (!over && c == gridDim.x - 1 && threadIdx.x == 0) tri_off[fp.tri_count] = info[0];
}

// Group every bin by row class (windows of kCsClassWindow entries) and strip
// the class bits from the pair index.
__global__ void __launch_bounds__(256) k_cs_class(const uint32_t *__restrict__ offs, uint2 *__restrict__ bins) {
    constexpr int kPer = kCsClassWindow / 256;
    constexpr int kClasses = 1 << kClassBits;
    __shared__ uint32_t cnt[kClasses];
    const uint32_t t = blockIdx.x;
    const uint32_t b0 = offs[t], n = offs[t + 1] - b0;
    if (n == 0) return;
    for (uint32_t w0 = 0; w0 < n; w0 += kCsClassWindow) {
        const uint32_t m = min((uint32_t)kCsClassWindow, n - w0);
        uint2 e[kPer];
        if (threadIdx.x < kClasses) cnt[threadIdx.x] = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t i = threadIdx.x + 256u * k;
            if (i < m) {
                e[k] = bins[b0 + w0 + i];
                atomicAdd(&cnt[e[k].y >> kCsClassShift], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
            for (int k = 0; k < kClasses; ++k) {
                const uint32_t v = cnt[k];
                cnt[k] = run;
                run += v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t i = threadIdx.x + 256u * k;
            if (i < m) {
                const uint32_t pos = atomicAdd(&cnt[e[k].y >> kCsClassShift], 1u);
                bins[b0 + w0 + pos] = make_uint2(e[k].x, e[k].y & kCsPairMask);
            }
        }
        __syncthreads();
    }
}

}  // namespace prk

extern "C" {

// Counting-sort binning (k_cs_*), after k_bin_count / k_bin_band (prk_bin_count
// below).  Every size is device-side:
// info[0] = entry count, info[1] = overflow (count > cap: bins left empty,
// no pair written; the caller re-runs the frame with more room).
// ghist: nchunks * ntiles u32; tile_tot: ntiles; chunk_tot / chunk_base: nchunks.
// All-AVX frames (fp->trec): the setup records are computed by k_setup_rec.
hipError_t prk_bin_count(const prk::FrameParams *fp, uint32_t *tri_n, void *ranges, uint32_t *runlist,
                         uint32_t *run_n, uint8_t *trwon, hipStream_t s) {
    const uint32_t n = fp->tri_count + 1;
    // A whole-frame target sets up (nearly) every triangle: inline records
    // (C3b: 76 us against 22 + 68 us split); a row band only its own.
    const bool band = fp->row0 > 0 || fp->row1 < fp->H;
    if (band && PRK_BIN_BAND && runlist) {  // (k_bin_band also writes the sentinel tri_n[tri_count])
        hipLaunchKernelGGL(prk::k_bin_band, dim3((n + prk::kRecRun - 1) / prk::kRecRun), dim3(prk::kCountThreads),
                           0, s, *fp, tri_n, reinterpret_cast<prk::TileRange *>(ranges), runlist, run_n, trwon);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(prk::k_bin_count, dim3((n + prk::kCountThreads - 1) / prk::kCountThreads),
                       dim3(prk::kCountThreads), 0, s, *fp, tri_n, reinterpret_cast<prk::TileRange *>(ranges), !band);
    if (band && fp->trec && fp->tri_count)
        hipLaunchKernelGGL(prk::k_setup_rec, dim3((fp->tri_count + prk::kRecRun - 1) / prk::kRecRun),
                           dim3(prk::kCountThreads), 0, s, *fp, tri_n);
    return hipGetLastError();
}

// A row band's setup records (k_band_rec) once k_bin_band has listed the
// runs; nothing to do unless the frame keeps records (fp->trec) and is a
// band frame with run lists.  The caller queues it on a stream of its own.
uint32_t prk_bin_runs(uint32_t tri_count);
hipError_t prk_band_records(const prk::FrameParams *fp, const uint32_t *runlist, const uint32_t *run_n,
                            hipStream_t s) {
    if (!PRK_BAND_REC_KERNEL || !fp->trec || !runlist || !fp->tri_count) return hipSuccess;
    hipLaunchKernelGGL(prk::k_band_rec, dim3(prk_bin_runs(fp->tri_count), prk::kRecRun / 64), dim3(64), 0, s, *fp,
                       runlist, run_n);
    return hipGetLastError();
}

// A row band's counting sort walks only its runs' listed triangles, `per`
// runs per chunk: about one whole-frame chunk's worth (kCsChunk) of the
// band's share of the triangles, so a narrow band has few chunks (and a
// small chunk x tile histogram).  0: not a band (whole-frame chunks).
uint32_t prk_bin_runs(uint32_t tri_count);
uint32_t prk_bin_run_len(void);
#ifndef PRK_BAND_MIN_CHUNKS
#define PRK_BAND_MIN_CHUNKS 128  // > 0: at least about this many chunks (smaller ones) per band frame
                                 // (C3b N = 8: 31 chunks of 1024 threads left the sort on 31 CUs;
                                 // serial binning 0.128 -> 0.094-0.109 ms, N = 4 0.134 -> 0.115)
#endif
uint32_t prk_cs_band_runs_per_chunk(const prk::FrameParams *fp) {
    const bool band = fp->row0 > 0 || fp->row1 < fp->H;
    if (!band || !PRK_BIN_BAND) return 0;
    const int64_t rows = std::max<int64_t>(1, (int64_t)std::min(fp->row1, fp->H) - fp->row0);
    const int64_t share = std::max<int64_t>(1, (int64_t)fp->H / rows);  // ~ triangles per band triangle
    int64_t per = (int64_t)prk::kCsChunk * share / prk::kRecRun;
    if (PRK_BAND_MIN_CHUNKS > 0) {
        const int64_t nruns = (int64_t)prk_bin_runs(fp->tri_count);
        per = std::min<int64_t>(per, nruns / std::max(1, PRK_BAND_MIN_CHUNKS));
    }
    return (uint32_t)std::min<int64_t>(prk::kMaxRunsPerChunk, std::max<int64_t>(1, per));
}
uint32_t prk_bin_runs(uint32_t tri_count) { return (tri_count + 1 + prk::kRecRun - 1) / prk::kRecRun; }
// Entries of one run of the band run list (k_bin_band writes runlist[run * this + i]).
uint32_t prk_bin_run_len(void) { return prk::kRecRun; }

// The counting sort's per-tile LDS (4 B per tile) above 64 KiB needs the
// dynamic-LDS attribute of k_cs_hist / k_cs_emit, which is per device: set
// once per device (a process may drive several GPUs), and only when a frame
// needs it.  0: not tried, 1: set, 2: refused (the caller bins with the
// radix sort instead).
static std::atomic<int> g_cs_attr[64];
int prk_cs_ready(uint32_t ntiles) {
    if (ntiles == 0 || ntiles > prk::kCsMaxTiles) return 0;
    if ((size_t)ntiles * 4 <= 65536) return 1;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int st = g_cs_attr[dev].load(std::memory_order_acquire);
    if (st == 0) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&prk::k_cs_hist),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, prk::kCsMaxTiles * 4);
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void *>(&prk::k_cs_emit),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, prk::kCsMaxTiles * 4);
        st = e == hipSuccess ? 1 : 2;
        g_cs_attr[dev].store(st, std::memory_order_release);  // (a racing setter sets the same value)
    }
    return st == 1;
}

uint32_t prk_cs_chunks(uint32_t tri_count) { return (tri_count + prk::kCsChunk - 1) / prk::kCsChunk; }
// Counting-sort chunks of a frame: whole-frame chunks, or (per > 0) a band's
// chunks of `per` runs.
uint32_t prk_cs_nchunks(uint32_t tri_count, uint32_t per) {
    if (!per) return prk_cs_chunks(tri_count);
    return (prk_bin_runs(tri_count) + per - 1) / per;
}
uint32_t prk_cs_max_tiles(void) { return prk::kCsMaxTiles; }
uint32_t prk_cs_max_pairs(void) { return prk::kCsPairMask; }

hipError_t prk_bin_cs(const prk::FrameParams *fp, const void *ranges, const uint32_t *tri_n, uint32_t *ghist,
                      uint32_t *tile_tot, uint32_t *chunk_tot, uint32_t *chunk_base, uint32_t *offs, uint32_t cap,
                      uint32_t *info, uint32_t *tri_off, void *bins, uint32_t *pair_tri, uint8_t *won,
                      uint32_t won_stride, uint8_t *trwon, const uint32_t *runlist, const uint32_t *run_n,
                      uint32_t per, hipStream_t s) {
    const uint32_t ntiles = (uint32_t)(fp->tiles_x * fp->tiles_y);
    if (ntiles > prk::kCsMaxTiles || ntiles == 0) return hipErrorInvalidValue;
    prk::BandRuns br{nullptr, nullptr, 0u, 0u};
    if (per && runlist) br = prk::BandRuns{runlist, run_n, prk_bin_runs(fp->tri_count), per};
    const uint32_t nch = prk_cs_nchunks(fp->tri_count, br.list ? per : 0u);
    const prk::TileRange *tr = reinterpret_cast<const prk::TileRange *>(ranges);
    const size_t lds = (size_t)ntiles * 4;
    if (!prk_cs_ready(ntiles)) return hipErrorNotSupported;
    if (nch) {
        hipLaunchKernelGGL(prk::k_cs_hist, dim3(nch), dim3(prk::kCsThreads), lds, s, *fp, tr, tri_n, ghist, chunk_tot,
                           ntiles, br);
        hipLaunchKernelGGL(prk::k_cs_colscan, dim3((ntiles + 63) / 64), dim3(64 * prk::kColSegs), 0, s, ghist, nch,
                           ntiles, tile_tot);
    } else {
        hipError_t e = hipMemsetAsync(tile_tot, 0, (size_t)ntiles * 4, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(prk::k_cs_scan, dim3(1), dim3(prk::kCsThreads), 0, s, tile_tot, ntiles, chunk_tot, nch, offs,
                       chunk_base, std::min(cap, prk::kCsPairMask), info);
    if (nch)
        hipLaunchKernelGGL(prk::k_cs_emit, dim3(nch), dim3(prk::kCsThreads), lds, s, *fp, tr, tri_n, ghist, offs,
                           chunk_base, info, ntiles, tri_off, reinterpret_cast<uint2 *>(bins), pair_tri, won,
                           won_stride, trwon, br);
    if (PRK_ROWCLASS)
        hipLaunchKernelGGL(prk::k_cs_class, dim3(ntiles), dim3(256), 0, s, offs, reinterpret_cast<uint2 *>(bins));
    return hipGetLastError();
}

}  // extern "C"
