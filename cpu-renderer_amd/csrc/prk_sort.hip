// prk_sort.hip — the span path's device-wide exclusive scans and its stable
// radix sort of MergeSort keys, hand-written for gfx950 (wave64 DPP scans,
// LDS per-thread digit counters).  They replace the library scans and the
// library radix sort the span path used through round 5.
//
//   prk_scan_u32 / prk_scan_u64   exclusive sum of n values: tile sums
//       (4096 values per 256-thread workgroup), one workgroup scans the tile
//       sums, each tile scanned again with its offset.  Reads the input twice
//       and writes once; the span path scans <= a few million values per pass.
//   prk_obj_sort   LSD radix sort of (u64 key, u32 value) pairs over the key's
//       low end_bit bits, 4 bits a pass, stable: each thread owns 16
//       consecutive items, counts their digits in its own LDS column, and the
//       (digit, workgroup, thread) order of the offsets keeps equal digits in
//       input order.  The object path's keys are (object, YMin, MergeSort
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

// Workgroup exclusive scan of one value per thread (kScanThreads threads);
// *total = the workgroup's sum.
template <typename T>
__device__ __forceinline__ T block_excl(T v, T *lds, T *total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const T inc = wave_incl<T>(v);
    if (lane == 63) lds[wave] = inc;
    __syncthreads();
    T before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
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

// One workgroup: exclusive scan of the tile sums in place (each thread a
// contiguous run of ceil(m / kScanThreads) of them).
template <typename T>
__global__ void __launch_bounds__(kScanThreads) k_scan_sums(T *__restrict__ sums, uint32_t m) {
    __shared__ T lds[kScanThreads / 64];
    const uint32_t per = (m + kScanThreads - 1) / kScanThreads;
    const uint32_t a = threadIdx.x * per, e = min(m, a + per);
    T s = 0;
    for (uint32_t i = a; i < e; ++i) s += sums[i];
    T tot;
    T run = block_excl<T>(s, lds, &tot);
    for (uint32_t i = a; i < e; ++i) {
        const T x = sums[i];
        sums[i] = run;
        run += x;
    }
}

template <typename T>
__global__ void __launch_bounds__(kScanThreads) k_scan_down(const T *in, T *out, uint32_t n,
                                                            const T *__restrict__ offs) {
    __shared__ T lds[kScanThreads / 64];
    const size_t b = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    T v[kScanItems];
    T s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        v[k] = b + k < n ? in[b + k] : (T)0;
        s += v[k];
    }
    T tot;
    T run = offs[blockIdx.x] + block_excl<T>(s, lds, &tot);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (b + k < n) {
            out[b + k] = run;
            run += v[k];
        }
}

template <typename T>
hipError_t scan_excl(const T *in, T *out, uint32_t n, void *temp, size_t *temp_bytes, hipStream_t s) {
    const uint32_t tiles = (n + kScanTile - 1) / kScanTile;
    if (!temp) {
        *temp_bytes = (size_t)(tiles ? tiles : 1) * sizeof(T);
        return hipSuccess;
    }
    if (n == 0) return hipSuccess;
    T *sums = static_cast<T *>(temp);
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3(tiles), dim3(kScanThreads), 0, s, in, n, sums);
    hipLaunchKernelGGL(k_scan_sums<T>, dim3(1), dim3(kScanThreads), 0, s, sums, tiles);
    hipLaunchKernelGGL(k_scan_down<T>, dim3(tiles), dim3(kScanThreads), 0, s, in, out, n, sums);
    return hipGetLastError();
}

// ---- radix sort -------------------------------------------------------------
constexpr int kRsBits = 4, kRsDigits = 1 << kRsBits;
constexpr int kRsThreads = 256, kRsItems = 16, kRsTile = kRsThreads * kRsItems;

// Per thread: its items' digit counts in its own LDS column (cnt[d][t]).
__device__ __forceinline__ void rs_count(const unsigned long long *__restrict__ keys, uint32_t n, uint32_t shift,
                                         uint16_t (*cnt)[kRsThreads]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int d = 0; d < kRsDigits; ++d) cnt[d][t] = 0;
    const size_t b = (size_t)blockIdx.x * kRsTile + (size_t)t * kRsItems;
#pragma unroll
    for (int k = 0; k < kRsItems; ++k)
        if (b + k < n) {
            const uint32_t d = (uint32_t)(keys[b + k] >> shift) & (kRsDigits - 1);
            cnt[d][t] += 1;
        }
}

// ghist[d * nblocks + blk] = workgroup blk's items of digit d.
__global__ void __launch_bounds__(kRsThreads) k_rs_hist(const unsigned long long *__restrict__ keys, uint32_t n,
                                                        uint32_t shift, uint32_t *__restrict__ ghist) {
    __shared__ uint16_t cnt[kRsDigits][kRsThreads];
    __shared__ uint32_t lds[kScanThreads / 64];
    rs_count(keys, n, shift, cnt);
    __syncthreads();
    for (int d = 0; d < kRsDigits; ++d) {
        uint32_t tot;
        (void)block_excl<uint32_t>(cnt[d][threadIdx.x], lds, &tot);
        if (threadIdx.x == 0) ghist[(size_t)d * gridDim.x + blockIdx.x] = tot;
    }
}

// Stable scatter: item k of thread t of workgroup blk, digit d, goes to
// gofs[d * nblocks + blk] + (thread t's offset among the workgroup's digit-d
// items) + (its rank among thread t's own digit-d items).
__global__ void __launch_bounds__(kRsThreads) k_rs_scatter(const unsigned long long *__restrict__ kin,
                                                           const uint32_t *__restrict__ vin, uint32_t n,
                                                           uint32_t shift, const uint32_t *__restrict__ gofs,
                                                           unsigned long long *__restrict__ kout,
                                                           uint32_t *__restrict__ vout) {
    __shared__ uint16_t cnt[kRsDigits][kRsThreads];
    __shared__ uint32_t base[kRsDigits][kRsThreads];
    __shared__ uint32_t lds[kScanThreads / 64];
    rs_count(kin, n, shift, cnt);
    __syncthreads();
    for (int d = 0; d < kRsDigits; ++d) {
        uint32_t tot;
        const uint32_t ex = block_excl<uint32_t>(cnt[d][threadIdx.x], lds, &tot);
        base[d][threadIdx.x] = gofs[(size_t)d * gridDim.x + blockIdx.x] + ex;
    }
    __syncthreads();
    const int t = threadIdx.x;
    const size_t b = (size_t)blockIdx.x * kRsTile + (size_t)t * kRsItems;
#pragma unroll
    for (int k = 0; k < kRsItems; ++k)
        if (b + k < n) {
            const unsigned long long key = kin[b + k];
            const uint32_t d = (uint32_t)(key >> shift) & (kRsDigits - 1);
            const uint32_t p = base[d][t]++;
            kout[p] = key;
            vout[p] = vin[b + k];
        }
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
    const uint32_t nblk = (n + kRsTile - 1) / kRsTile;
    const uint32_t passes = (end_bit + kRsBits - 1) / kRsBits;
    const size_t hist_n = (size_t)kRsDigits * (nblk ? nblk : 1);
    size_t scan_bytes = 0;
    (void)scan_excl<uint32_t>(nullptr, nullptr, (uint32_t)hist_n, nullptr, &scan_bytes, s);
    auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t need = up((size_t)n * 8) + up((size_t)n * 4) + 2 * up(hist_n * 4) + up(scan_bytes);
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
    uint32_t *ghist = reinterpret_cast<uint32_t *>(p);
    p += up(hist_n * 4);
    uint32_t *gofs = reinterpret_cast<uint32_t *>(p);
    p += up(hist_n * 4);
    void *stemp = p;
    const unsigned long long *ki = static_cast<const unsigned long long *>(keys_in);
    unsigned long long *ko = static_cast<unsigned long long *>(keys_out);
    if (passes == 0) {  // (no key bits: the identity order)
        hipError_t e = hipMemcpyAsync(ko, ki, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(vals_out, vals_in, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
        return e;
    }
    const unsigned long long *sk = ki;
    const uint32_t *sv = vals_in;
    for (uint32_t q = 0; q < passes; ++q) {
        // the last pass lands in keys_out / vals_out
        const bool to_out = ((passes - 1 - q) & 1u) == 0;
        unsigned long long *dk = to_out ? ko : tk;
        uint32_t *dv = to_out ? vals_out : tv;
        const uint32_t shift = q * kRsBits;
        hipLaunchKernelGGL(k_rs_hist, dim3(nblk), dim3(kRsThreads), 0, s, sk, n, shift, ghist);
        hipError_t e = scan_excl<uint32_t>(ghist, gofs, (uint32_t)hist_n, stemp, &scan_bytes, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_rs_scatter, dim3(nblk), dim3(kRsThreads), 0, s, sk, sv, n, shift, gofs, dk, dv);
        sk = dk;
        sv = dv;
    }
    return hipGetLastError();
}

}  // extern "C"
