// sort_bench.cpp — checks and times libprk_hip.so's span-path scan and radix
// sort (csrc/prk_sort.hip) against std::stable_sort / a host prefix sum.
// usage: sort_bench [n] [end_bit] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

extern "C" {
hipError_t prk_obj_sort(void *keys_in, uint32_t *vals_in, void *keys_out, uint32_t *vals_out, uint32_t n,
                        uint32_t end_bit, void *temp, size_t *temp_bytes, hipStream_t s);
hipError_t prk_scan_u32(const uint32_t *in, uint32_t *out, uint32_t n, void *temp, size_t *temp_bytes,
                        hipStream_t s);
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorName(e_)); \
            return 2;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atol(argv[1]) : 6624;
    const uint32_t bits = argc > 2 ? (uint32_t)std::atol(argv[2]) : 26;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 20;
    std::mt19937_64 rng(7);
    std::vector<unsigned long long> k(n);
    std::vector<uint32_t> v(n);
    const unsigned long long mask = bits >= 64 ? ~0ull : ((1ull << bits) - 1ull);
    for (uint32_t i = 0; i < n; ++i) {
        k[i] = rng() & mask & ~0xFull;  // (low bits equal: ties exercise the stability)
        v[i] = i;
    }
    unsigned long long *dk, *dk2;
    uint32_t *dv, *dv2;
    CK(hipMalloc(&dk, n * 8ull + 8));
    CK(hipMalloc(&dk2, n * 8ull + 8));
    CK(hipMalloc(&dv, n * 4ull + 4));
    CK(hipMalloc(&dv2, n * 4ull + 4));
    CK(hipMemcpy(dk, k.data(), n * 8ull, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, v.data(), n * 4ull, hipMemcpyHostToDevice));
    size_t tb = 0;
    CK(prk_obj_sort(dk, dv, dk2, dv2, n, bits, nullptr, &tb, nullptr));
    void *tmp;
    CK(hipMalloc(&tmp, tb + 256));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(prk_obj_sort(dk, dv, dk2, dv2, n, bits, tmp, &tb, nullptr));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, nullptr));
    for (int r = 0; r < reps; ++r) CK(prk_obj_sort(dk, dv, dk2, dv2, n, bits, tmp, &tb, nullptr));
    CK(hipEventRecord(b, nullptr));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> gk(n);
    std::vector<uint32_t> gv(n);
    CK(hipMemcpy(gk.data(), dk2, n * 8ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gv.data(), dv2, n * 4ull, hipMemcpyDeviceToHost));
    std::vector<uint32_t> ord(n);
    std::iota(ord.begin(), ord.end(), 0u);
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return k[x] < k[y]; });
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; ++i) bad += (gv[i] != ord[i] || gk[i] != k[ord[i]]) ? 1u : 0u;
    // scan
    std::vector<uint32_t> c(n);
    for (uint32_t i = 0; i < n; ++i) c[i] = (uint32_t)(rng() & 7);
    CK(hipMemcpy(dv, c.data(), n * 4ull, hipMemcpyHostToDevice));
    size_t sb = 0;
    CK(prk_scan_u32(dv, dv2, n, nullptr, &sb, nullptr));
    CK(prk_scan_u32(dv, dv2, n, tmp, &sb, nullptr));
    CK(hipMemcpy(gv.data(), dv2, n * 4ull, hipMemcpyDeviceToHost));
    uint32_t sbad = 0, run = 0;
    for (uint32_t i = 0; i < n; ++i) {
        sbad += gv[i] != run ? 1u : 0u;
        run += c[i];
    }
    std::printf("sort_bench n=%u bits=%u: %.1f us/sort, sort mismatches %u, scan mismatches %u\n", n, bits,
                1000.0f * ms / reps, bad, sbad);
    return bad || sbad ? 1 : 0;
}
