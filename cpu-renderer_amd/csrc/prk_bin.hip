// prk_bin.hip — triangle -> tile binning with bins in submission order.
//
//   k_bin_count   1 thread / triangle: ProjectVertex + back-face cull
//                 (projekt.cpp:74-93, 3926-3943) -> conservative tile range ->
//                 number of (triangle, tile) entries.
//   scan          exclusive sum of the per-triangle counts (hipcub).
//   k_bin_emit    1 thread / triangle: write (tile, (triangle, pair)) at the
//                 triangle's offset, i.e. in triangle order (pair j), row-major
//                 over the triangle's tile rectangle; pair_tri[j] = triangle.
//   sort          stable LSD radix sort of the 8-byte (triangle, pair) values
//                 by tile (rocprim onesweep), so every tile's bin lists its triangles in
//                 submission order.
//   k_tile_offsets  bin start of every tile (lower_bound on the sorted tiles).
//
// Pairs are numbered in triangle (= submission) order: the pair index is the
// visibility sweep's tie-break key, and k_walk / k_pix address span records
// by (pair, row).  (Scattering pairs into bins with global atomic counters
// instead of sorting measured 3x slower: device-scope atomics on 4096 hot
// counters.)
//
// Triangle-ordered bins let k_raster name a triangle by its position in the
// tile's bin (entry order == submission order), which it uses to skip, in the
// shading sweep, every triangle that won no pixel of the tile.
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include "prk_device.h"

namespace prk {

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
        tr.tx0 = (uint16_t)(c0 / fp.tile_w);
        tr.tx1 = (uint16_t)((c1 - 1) / fp.tile_w);
        tr.ty0 = (uint16_t)((r0 - fp.row0) / fp.tile_h);
        tr.ty1 = (uint16_t)((r1 - 1 - fp.row0) / fp.tile_h);
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
            tr.oty0 = (uint16_t)((o0 - fp.row0) / fp.tile_h);
            tr.oty1 = (uint16_t)((o1 - 1 - fp.row0) / fp.tile_h);
        }
    }
    return rect || tr.oty0 <= tr.oty1;
}

// Number of tiles in a range (rectangle + column-0 overflow tiles not in it).
__device__ __forceinline__ uint32_t range_entries(const TileRange &tr) {
    uint32_t n = 0;
    if (tr.tx0 <= tr.tx1 && tr.ty0 <= tr.ty1) n = (uint32_t)(tr.tx1 - tr.tx0 + 1) * (tr.ty1 - tr.ty0 + 1);
    for (int ty = tr.oty0; ty <= tr.oty1; ++ty)
        if (!(tr.tx0 == 0 && tr.tx0 <= tr.tx1 && ty >= tr.ty0 && ty <= tr.ty1)) ++n;
    return n;
}

constexpr int kRowClassBits = 3;

__global__ void k_bin_count(FrameParams fp, uint32_t *__restrict__ tri_n, TileRange *__restrict__ ranges) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g > fp.tri_count) return;
    if (g == fp.tri_count) {  // sentinel: the scan's last element is the total
        tri_n[g] = 0;
        return;
    }
    TileRange tr;
    if (!tri_tile_range(fp, g, tr)) {
        tr.tx0 = 1; tr.tx1 = 0; tr.ty0 = 1; tr.ty1 = 0; tr.oty0 = 1; tr.oty1 = 0;
    }
    ranges[g] = tr;
    const uint32_t ne = range_entries(tr);
    tri_n[g] = ne;
    if (fp.trec && ne) {
        // All-AVX frame: FillEdgeTable + MergeSort + the first row's AET
        // insertions once per triangle (TriRec / NrmRec, prk_device.h).
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
        TriRec r;
        NrmRec q;
        rec_edge_out(s0, r.e[0], r.ymin[0], r.ymax[0]);
        rec_edge_out(s1, r.e[1], r.ymin[1], r.ymax[1]);
        rec_edge_out(s2, r.e[2], r.ymin[2], r.ymax[2]);
        r.head = (uint32_t)n | (w.ord << 4) | ((uint32_t)w.cnt << 12) | ((uint32_t)(w.pend + 1) << 16) |
                 (min(anom, 15u) << 20) | ((d->flags & DRAW_ST) ? (1u << 24) : 0u);
        r.pad[0] = r.pad[1] = r.pad[2] = 0;
        nrm_edge_out(s0, q.n[0]);
        nrm_edge_out(s1, q.n[1]);
        nrm_edge_out(s2, q.n[2]);
        q.pad[0] = q.pad[1] = 0.0f;
        float4 *dr = reinterpret_cast<float4 *>(fp.trec + g);
        const float4 *sr = reinterpret_cast<const float4 *>(&r);
#pragma unroll
        for (int k = 0; k < 10; ++k) dr[k] = sr[k];
        float4 *dq = reinterpret_cast<float4 *>(fp.nrec + g);
        const float4 *sq = reinterpret_cast<const float4 *>(&q);
#pragma unroll
        for (int k = 0; k < 5; ++k) dq[k] = sq[k];
    }
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

__global__ void k_bin_emit(FrameParams fp, const TileRange *__restrict__ ranges, const uint32_t *__restrict__ off,
                           uint32_t *__restrict__ keys, uint2 *__restrict__ vals, uint32_t *__restrict__ pair_tri,
                           uint8_t *__restrict__ won, uint32_t won_stride, uint8_t *__restrict__ trwon) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= fp.tri_count) return;
    if (trwon) trwon[g] = 0;
    const TileRange tr = ranges[g];
    uint32_t o = off[g];
    constexpr int kMaxClass = (1 << kRowClassBits) - 1;
    if (tr.tx0 <= tr.tx1 && tr.ty0 <= tr.ty1)
        for (int ty = tr.ty0; ty <= tr.ty1; ++ty) {
            const int y0 = ty * fp.tile_h;
            const int rows = min((int)tr.pad1, y0 + fp.tile_h) - max((int)tr.pad0, y0);
            const uint32_t cls = (uint32_t)min(kMaxClass, max(0, fp.tile_h - rows));
            for (int tx = tr.tx0; tx <= tr.tx1; ++tx) {
                keys[o] = ((uint32_t)(ty * fp.tiles_x + tx) << kRowClassBits) | cls;
                vals[o] = make_uint2(g, o);
                pair_tri[o] = g;
                clear_won(won, won_stride, o);
                ++o;
            }
        }
    for (int ty = tr.oty0; ty <= tr.oty1; ++ty)
        if (!(tr.tx0 == 0 && tr.tx0 <= tr.tx1 && ty >= tr.ty0 && ty <= tr.ty1)) {
            keys[o] = ((uint32_t)(ty * fp.tiles_x) << kRowClassBits) | (uint32_t)kMaxClass;
            vals[o] = make_uint2(g, o);
            pair_tri[o] = g;
            clear_won(won, won_stride, o);
            ++o;
        }
}

// offs[t] = first sorted position whose tile is >= t, for t in [0, ntiles].
// (keys carry the row class in their low kRowClassBits bits)
__global__ void k_tile_offsets(const uint32_t *__restrict__ keys, uint32_t total, uint32_t ntiles,
                               uint32_t *__restrict__ offs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    uint32_t lo = 0, hi = total;
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if ((keys[mid] >> kRowClassBits) < t) lo = mid + 1; else hi = mid;
    }
    offs[t] = lo;
}

}  // namespace prk

// Bin sort: onesweep radix at every size above one block.  rocprim's
// default switches to a block sort + merge sort below 1 M items, which is
// the band size of a 4- or 8-rank frame (C3b at N = 8: 0.4 M entries, nine
// merge passes of two launches each, 0.13 ms per frame on one MI355X against
// two onesweep passes over the band's 13-bit keys).
using BinSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                 rocprim::default_config, 0>;

extern "C" {

// Phase 1: counts + exclusive scan.  `scan_out` gets T+1 offsets; the caller
// reads scan_out[T] (the number of entries) before phase 2.
hipError_t prk_bin_phase1(const prk::FrameParams *fp, uint32_t *tri_n, uint32_t *scan_out, void *ranges,
                          void *temp, size_t *temp_bytes, hipStream_t s) {
    const uint32_t n = fp->tri_count + 1;
    if (!temp) return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, tri_n, scan_out, n, s);
    hipLaunchKernelGGL(prk::k_bin_count, dim3((n + 255) / 256), dim3(256), 0, s, *fp, tri_n,
                       reinterpret_cast<prk::TileRange *>(ranges));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, tri_n, scan_out, n, s);
}

// Phase 2: emit pairs in triangle order, stable sort of the (triangle, pair)
// values by tile, tile offsets.  keys_a / vals_a: pairs in triangle order;
// keys_b / bins: sorted by tile; pair_tri: triangle per pair; won (won_stride
// bytes per pair) and trwon (T bytes, may be null) cleared.
// With temp == nullptr only reports the temp storage the sort needs.
hipError_t prk_bin_phase2(const prk::FrameParams *fp, const void *ranges, const uint32_t *scan_out, uint32_t total,
                          uint32_t *keys_a, void *vals_a, uint32_t *keys_b, void *bins, uint32_t *pair_tri,
                          uint32_t *offs, uint8_t *won, uint32_t won_stride, uint8_t *trwon, void *temp,
                          size_t *temp_bytes, hipStream_t s) {
    const uint32_t ntiles = (uint32_t)(fp->tiles_x * fp->tiles_y);
    int bits = 1;
    while ((1u << bits) < ntiles && bits < 32) ++bits;
    bits += prk::kRowClassBits;
    uint64_t *va = reinterpret_cast<uint64_t *>(vals_a), *vb = reinterpret_cast<uint64_t *>(bins);
    if (!temp)
        return rocprim::radix_sort_pairs<BinSortConfig>(nullptr, *temp_bytes, keys_a, keys_b, va, vb, total, 0,
                                                        (unsigned)bits, s);
    if (fp->tri_count)
        hipLaunchKernelGGL(prk::k_bin_emit, dim3((fp->tri_count + 255) / 256), dim3(256), 0, s, *fp,
                           reinterpret_cast<const prk::TileRange *>(ranges), scan_out, keys_a,
                           reinterpret_cast<uint2 *>(vals_a), pair_tri, won, won_stride, trwon);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (total) {
        e = rocprim::radix_sort_pairs<BinSortConfig>(temp, *temp_bytes, keys_a, keys_b, va, vb, total, 0,
                                                     (unsigned)bits, s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(prk::k_tile_offsets, dim3((ntiles + 1 + 255) / 256), dim3(256), 0, s, keys_b, total, ntiles,
                       offs);
    return hipGetLastError();
}

}  // extern "C"
