// prk_sort.hip — the span path's device-wide exclusive scans and its stable
// radix sort of MergeSort keys, hand-written for gfx950 (wave64 DPP scans,
// LDS per-thread digit counters).  They replace the library scans and the
// library radix sort the span path used through round 5.
//
//   prk_scan_u32 / prk_scan_u64   exclusive sum of n values: up to 4096 one
//       workgroup; above, tile sums (4096 values per 256-thread workgroup),
//       then each tile scanned with its offset, which the tile adds up from
//       the earlier sums itself (two launches).
//   prk_obj_sort   LSD radix sort of (u64 key, u32 value) pairs over the key's
//       low end_bit bits, 8 bits a pass, stable (wave-ballot ranks), one
//       launch a pass with decoupled look-back between the tiles (below).  The object path's keys are (object, YMin, MergeSort
//       recursion path) of projekt.cpp:2-72 (prk_spans.hip SortKeyBits): a
//       stable order of those keys IS MergeSort's order.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace prk {
namespace {

constexpr int kScanThreads = 256, kScanItems = 16, kScanTile = kScanThreads * kScanItems;

// Wave64 inclusive prefix sum (DPP row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}
__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t v) {
    // (64-bit values: lane shifts through LDS-free permutes, six steps)
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
        const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
        if (lane >= d) v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_incl(T v);
template <>
__device__ __forceinline__ uint32_t wave_incl<uint32_t>(uint32_t v) { return wave_incl_u32(v); }
template <>
__device__ __forceinline__ uint64_t wave_incl<uint64_t>(uint64_t v) { return wave_incl_u64(v); }

// Workgroup exclusive scan of one value per thread (NT threads);
// *total = the workgroup's sum.
template <typename T, int NT = kScanThreads>
__device__ __forceinline__ T block_excl(T v, T *lds, T *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const T inc = wave_incl<T>(v);
    if (lane == 63) lds[wave] = inc;
    __syncthreads();
    T before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const T x = lds[w];
        if (w < wave) before += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return before + inc - v;
}

template <typename T>
__global__ void __launch_bounds__(kScanThreads) k_scan_tiles(const T *__restrict__ in, uint32_t n, T *__restrict__ sums) {
    __shared__ T lds[kScanThreads / 64];
    const size_t b = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    T s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (b + k < n) s += in[b + k];
    T tot;
    (void)block_excl<T>(s, lds, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// Each tile scanned with its offset: the sum of the earlier tiles' sums,
// which the workgroup adds up itself (no separate scan of the sums; a few
// thousand tiles at most, read from L2).  sums == nullptr: one tile, offset 0.
template <typename T>
__global__ void __launch_bounds__(kScanThreads) k_scan_down(const T *in, T *out, uint32_t n,
                                                            const T *__restrict__ sums) {
    __shared__ T lds[kScanThreads / 64];
    T before = 0;
    if (sums) {
        for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kScanThreads) before += sums[i];
        T tot;
        (void)block_excl<T>(before, lds, &tot);
        before = tot;
    }
    const size_t b = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    T v[kScanItems];
    T s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = b + k < n ? in[b + k] : (T)0;
        s += v[k];
    }
    T tot;
    T run = before + block_excl<T>(s, lds, &tot);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (b + k < n) {
            out[b + k] = run;
            run += v[k];
        }
}

// Exclusive scan of n values: one launch up to kScanTile values, else the
// tile sums and the tiles (two launches).
template <typename T>
hipError_t scan_excl(const T *in, T *out, uint32_t n, void *temp, size_t *temp_bytes, hipStream_t s) {
    const uint32_t tiles = (n + kScanTile - 1) / kScanTile;
    if (!temp) {
        *temp_bytes = (size_t)(tiles ? tiles : 1) * sizeof(T);
        return hipSuccess;
    }
    if (n == 0) return hipSuccess;
    if (tiles == 1) {
        hipLaunchKernelGGL(k_scan_down<T>, dim3(1), dim3(kScanThreads), 0, s, in, out, n, (const T *)nullptr);
        return hipGetLastError();
    }
    T *sums = static_cast<T *>(temp);
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3(tiles), dim3(kScanThreads), 0, s, in, n, sums);
    hipLaunchKernelGGL(k_scan_down<T>, dim3(tiles), dim3(kScanThreads), 0, s, in, out, n, (const T *)sums);
    return hipGetLastError();
}

// ---- radix sort -------------------------------------------------------------
// LSD, 8-bit digits, one launch per pass plus one histogram launch for all
// passes (the onesweep scheme):
//   k_rs_upsweep   every tile's digit counts of every pass into the global
//                  per-pass histograms (LDS, then one atomic per digit);
//   k_rs_onesweep  per pass: a tile takes the next tile number from a ticket,
//                  counts its digits, publishes them (aggregate), adds its
//                  predecessors' by decoupled look-back (one thread per digit
//                  walks back until an inclusive prefix), publishes its own
//                  inclusive prefix, and scatters: item -> the digit's global
//                  base + the earlier tiles' digit count + its place in the
//                  tile.
// Inside a tile every wave owns a contiguous segment, in rounds of 64 (item
// w * S + r * 64 + lane: coalesced, and (wave, round, lane) order = input
// order), loaded into registers once: the wave counts its digits (eight
// ballots find a lane's equal-digit peers, the lowest adds their count to the
// wave's LDS histogram), then scatters round by round at its running digit
// offsets + the lane's rank among its peers.  Equal digits keep their input
// order: the sort is stable.  Tickets make the look-back wait only on tiles
// that already run, so it cannot deadlock.
constexpr int kRsBits = 8, kRsDigits = 1 << kRsBits;
constexpr int kRsThreads = 256;
// Rounds of 64 items per wave: short tiles keep a tile's serial chain short
// (small sorts), long ones keep the look-back chains short (large sorts).
constexpr int kRsRoundsSmall = 4, kRsRoundsLarge = 16;
constexpr uint32_t kRsSmallMax = 262144;  // up to this many items: short tiles
constexpr int kRsMaxPasses = 8;
constexpr uint32_t kRsAgg = 1u << 30, kRsInc = 2u << 30, kRsVal = kRsAgg - 1u;  // look-back status word

template <int NT>
struct RsLds {
    uint32_t off[NT / 64][kRsDigits];  // per wave: its digit counts, then its running digit offsets
    uint32_t base[kRsDigits];          // the tile's first output slot of each digit
    uint32_t tmp[NT / 64];
    uint32_t ticket;
};

__device__ __forceinline__ uint64_t rs_peers(uint32_t d, bool act) {
    uint64_t m = __ballot(act);
#pragma unroll
    for (int bit = 0; bit < kRsBits; ++bit) {
        const bool x = act && ((d >> bit) & 1u);
        const uint64_t bm = __ballot(x);
        m &= ((d >> bit) & 1u) ? bm : ~bm;
    }
    return m;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The wave's digit counts of its segment (k[r], r * 64 + lane < seg_n) into L.off[w].
template <int NT, int R>
__device__ __forceinline__ void rs_count(const unsigned long long (&k)[R], uint32_t seg_n, uint32_t shift,
                                         RsLds<NT> &L) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int d = lane; d < kRsDigits; d += 64) L.off[w][d] = 0;
    wave_sync_lds();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if ((uint32_t)(r * 64) >= seg_n) break;  // (wave-uniform)
        const bool act = (uint32_t)(r * 64 + lane) < seg_n;
        const uint32_t d = (uint32_t)(k[r] >> shift) & (kRsDigits - 1);
        const uint64_t peers = rs_peers(d, act);
        if (act && (peers & lt) == 0) L.off[w][d] += (uint32_t)__popcll(peers);
        wave_sync_lds();
    }
}

// After rs_count and a barrier, with L.base set: the waves' start offsets,
// then every item to L.base[d] + the earlier waves' + its rank.
template <int NT, int R, class ST>
__device__ __forceinline__ void rs_scatter(const unsigned long long (&k)[R], const uint32_t (&v)[R], uint32_t seg_n,
                                           uint32_t shift, RsLds<NT> &L, ST &&st) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int d = threadIdx.x; d < kRsDigits; d += NT) {
        uint32_t run = L.base[d];
#pragma unroll
        for (int u = 0; u < NT / 64; ++u) {
            const uint32_t c = L.off[u][d];
            L.off[u][d] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if ((uint32_t)(r * 64) >= seg_n) break;
        const bool act = (uint32_t)(r * 64 + lane) < seg_n;
        const uint32_t d = (uint32_t)(k[r] >> shift) & (kRsDigits - 1);
        const uint64_t peers = rs_peers(d, act);
        if (act) st(L.off[w][d] + (uint32_t)__popcll(peers & lt), k[r], v[r]);
        wave_sync_lds();
        if (act && (peers & lt) == 0) L.off[w][d] += (uint32_t)__popcll(peers);
        wave_sync_lds();
    }
}

// hist[q * 256 + d] += the tile's items with digit d in pass q (all passes).
template <int R>
__global__ void __launch_bounds__(kRsThreads) k_rs_upsweep(const unsigned long long *__restrict__ keys, uint32_t n,
                                                           uint32_t passes, uint32_t *__restrict__ hist) {
    constexpr int kRsRounds = R, kRsTile = kRsThreads * R;
    __shared__ uint32_t h[kRsMaxPasses][kRsDigits];
    for (int i = threadIdx.x; i < kRsMaxPasses * kRsDigits; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const size_t t0 = (size_t)blockIdx.x * kRsTile;
    for (int r = 0; r < kRsRounds; ++r) {
        const size_t i = t0 + (size_t)r * kRsThreads + threadIdx.x;
        if (i < n) {
            const unsigned long long key = keys[i];
            for (uint32_t q = 0; q < passes; ++q) atomicAdd(&h[q][(uint32_t)(key >> (q * kRsBits)) & (kRsDigits - 1)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t q = 0; q < passes; ++q)
        for (int d = threadIdx.x; d < kRsDigits; d += kRsThreads)
            if (h[q][d]) atomicAdd(&hist[q * kRsDigits + d], h[q][d]);
}

// One pass (digit shift, its global histogram ghist[256], look-back status
// words status[tile * 256 + digit], ticket counter) of the onesweep sort.
template <int R>
__global__ void __launch_bounds__(kRsThreads) k_rs_onesweep(const unsigned long long *__restrict__ kin,
                                                            const uint32_t *__restrict__ vin, uint32_t n,
                                                            uint32_t shift, const uint32_t *__restrict__ ghist,
                                                            uint32_t *status, uint32_t *ticket,
                                                            unsigned long long *__restrict__ kout,
                                                            uint32_t *__restrict__ vout) {
    constexpr int kRsRounds = R, kRsTile = kRsThreads * R;
    __shared__ RsLds<kRsThreads> L;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) L.ticket = atomicAdd(ticket, 1u);
    // the pass's digit bases: exclusive scan of its global histogram
    const uint32_t c = t < kRsDigits ? ghist[t] : 0u;
    uint32_t tot;
    const uint32_t gbase = block_excl<uint32_t, kRsThreads>(c, L.tmp, &tot);  // (its barriers publish the ticket)
    const uint32_t b = L.ticket;
    const size_t s0 = (size_t)b * kRsTile + (size_t)w * kRsRounds * 64;
    const uint32_t seg_n = s0 >= n ? 0u : (uint32_t)min((size_t)kRsRounds * 64, n - s0);
    unsigned long long k[kRsRounds];
    uint32_t v[kRsRounds];
#pragma unroll
    for (int r = 0; r < kRsRounds; ++r) {
        const uint32_t q = (uint32_t)(r * 64 + lane);
        k[r] = q < seg_n ? kin[s0 + q] : 0ull;
        v[r] = q < seg_n ? vin[s0 + q] : 0u;
    }
    rs_count<kRsThreads, kRsRounds>(k, seg_n, shift, L);
    __syncthreads();
    if (t < kRsDigits) {  // publish, look back, publish the inclusive prefix
        uint32_t mine = 0;
#pragma unroll
        for (int u = 0; u < kRsThreads / 64; ++u) mine += L.off[u][t];
        uint32_t *st = status + (size_t)b * kRsDigits + t;
        __hip_atomic_store(st, (b == 0 ? kRsInc : kRsAgg) | mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t pre = 0;
        for (uint32_t bb = b; bb > 0;) {
            --bb;
            uint32_t x;
            do {
                x = __hip_atomic_load(status + (size_t)bb * kRsDigits + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } while ((x & ~kRsVal) == 0u);
            pre += x & kRsVal;
            if (x & kRsInc) break;
        }
        if (b > 0) __hip_atomic_store(st, kRsInc | (pre + mine), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        L.base[t] = gbase + pre;
    }
    __syncthreads();
    rs_scatter<kRsThreads, kRsRounds>(k, v, seg_n, shift, L, [&](uint32_t p, unsigned long long kk, uint32_t vv) {
        kout[p] = kk;
        vout[p] = vv;
    });
}

}  // namespace
}  // namespace prk

extern "C" {

// Exclusive scan of n values (temp == nullptr: size query).
hipError_t prk_scan_u32(const uint32_t *in, uint32_t *out, uint32_t n, void *temp, size_t *temp_bytes,
                        hipStream_t s) {
    return prk::scan_excl<uint32_t>(in, out, n, temp, temp_bytes, s);
}
hipError_t prk_scan_u64(const unsigned long long *in, unsigned long long *out, uint32_t n, void *temp,
                        size_t *temp_bytes, hipStream_t s) {
    return prk::scan_excl<uint64_t>(reinterpret_cast<const uint64_t *>(in), reinterpret_cast<uint64_t *>(out), n,
                                    temp, temp_bytes, s);
}

// Stable sort of n (key, value) pairs by the keys' low end_bit bits
// (temp == nullptr: size query).  keys_in / vals_in are not written.
hipError_t prk_obj_sort(void *keys_in, uint32_t *vals_in, void *keys_out, uint32_t *vals_out, uint32_t n,
                        uint32_t end_bit, void *temp, size_t *temp_bytes, hipStream_t s) {
    using namespace prk;
    const bool small = n <= kRsSmallMax;
    const uint32_t tile = (uint32_t)kRsThreads * (small ? kRsRoundsSmall : kRsRoundsLarge);
    const uint32_t nblk = (n + tile - 1) / tile;
    const uint32_t passes = (end_bit + kRsBits - 1) / kRsBits;
    if (passes > kRsMaxPasses || n > kRsVal) return hipErrorInvalidValue;
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    // (hist, tickets and status words are zeroed by one memset)
    const size_t ctl = (size_t)kRsMaxPasses * kRsDigits * 4 + 64 + (size_t)passes * (nblk ? nblk : 1) * kRsDigits * 4;
    const size_t need = up((size_t)n * 8) + up((size_t)n * 4) + up(ctl);
    if (!temp) {
        *temp_bytes = need;
        return hipSuccess;
    }
    if (n == 0) return hipSuccess;
    char *p = static_cast<char *>(temp);
    unsigned long long *tk = reinterpret_cast<unsigned long long *>(p);
    p += up((size_t)n * 8);
    uint32_t *tv = reinterpret_cast<uint32_t *>(p);
    p += up((size_t)n * 4);
    uint32_t *hist = reinterpret_cast<uint32_t *>(p);
    uint32_t *tickets = hist + kRsMaxPasses * kRsDigits;
    uint32_t *status = tickets + 16;
    const unsigned long long *ki = static_cast<const unsigned long long *>(keys_in);
    unsigned long long *ko = static_cast<unsigned long long *>(keys_out);
    if (passes == 0) {  // (no key bits: the identity order)
        hipError_t e = hipMemcpyAsync(ko, ki, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(vals_out, vals_in, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
        return e;
    }
    hipError_t e = hipMemsetAsync(hist, 0, ctl, s);
    if (e != hipSuccess) return e;
    if (small) hipLaunchKernelGGL(k_rs_upsweep<kRsRoundsSmall>, dim3(nblk), dim3(kRsThreads), 0, s, ki, n, passes, hist);
    else hipLaunchKernelGGL(k_rs_upsweep<kRsRoundsLarge>, dim3(nblk), dim3(kRsThreads), 0, s, ki, n, passes, hist);
    const unsigned long long *sk = ki;
    const uint32_t *sv = vals_in;
    for (uint32_t q = 0; q < passes; ++q) {
        // the last pass lands in keys_out / vals_out
        const bool to_out = ((passes - 1 - q) & 1u) == 0;
        unsigned long long *dk = to_out ? ko : tk;
        uint32_t *dv = to_out ? vals_out : tv;
        if (small)
            hipLaunchKernelGGL(k_rs_onesweep<kRsRoundsSmall>, dim3(nblk), dim3(kRsThreads), 0, s, sk, sv, n,
                               q * kRsBits, hist + q * kRsDigits, status + (size_t)q * nblk * kRsDigits, tickets + q,
                               dk, dv);
        else
            hipLaunchKernelGGL(k_rs_onesweep<kRsRoundsLarge>, dim3(nblk), dim3(kRsThreads), 0, s, sk, sv, n,
                               q * kRsBits, hist + q * kRsDigits, status + (size_t)q * nblk * kRsDigits, tickets + q,
                               dk, dv);
        sk = dk;
        sv = dv;
    }
    return hipGetLastError();
}

}  // extern "C"
