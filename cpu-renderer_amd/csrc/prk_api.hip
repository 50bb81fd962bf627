// prk_api.cpp — host side of libprk_hip.so: the C-ABI declared in include/prk.h.
//
// Owns device resources (geometry, textures, scratch for binning) and turns the
// reference's draw calls into one GPU frame per prk_flush:
//   FillEdgeTable + DrawModelOptimized / DrawModel (projekt.cpp:3882, 3615, 162)
//   -> prk_draw records {geometry range, P, semantics, Phong, Bitmap}
//   Platform.CompleteAllWork -> prk_flush runs bin + raster kernels.
// There is no CPU fallback: every entry point that computes pixels needs the
// HIP device and fails with PRK_ERR_DEVICE without one.
#include <hip/hip_runtime.h>
#include <link.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/prk.h"
#include "../../include/prk_edge_count.h"
#include "prk_device.h"

extern "C" {
hipError_t prk_launch_tri_draw(const prk::DrawRec *, uint32_t, uint32_t *, uint32_t, hipStream_t);
hipError_t prk_bin_count(const prk::FrameParams *, uint32_t *, void *, uint32_t *, uint32_t *, uint8_t *, hipStream_t);
hipError_t prk_band_records(const prk::FrameParams *, const uint32_t *, const uint32_t *, hipStream_t);
#ifndef PRK_REC_AFTER_CS
#define PRK_REC_AFTER_CS 1  // a band's k_band_rec queued after the counting sort's launches
#endif
#ifndef PRK_BINNED_EARLY
#define PRK_BINNED_EARLY 0  // 1: binned_ev before the entry count's copy to the host (serial band binning
                            // 0.084 -> 0.075 ms, but C3b N = 8 pipelined 0.186 -> 0.21-0.22 ms: the copy,
                            // which the host waits for, then queues behind k_vis)
#endif
uint32_t prk_cs_chunks(uint32_t);
uint32_t prk_cs_nchunks(uint32_t, uint32_t);
uint32_t prk_cs_band_runs_per_chunk(const prk::FrameParams *);
uint32_t prk_bin_runs(uint32_t);
uint32_t prk_bin_run_len(void);
uint32_t prk_cs_max_tiles(void);
uint32_t prk_cs_max_pairs(void);
int prk_cs_ready(uint32_t);
hipError_t prk_bin_cs(const prk::FrameParams *, const void *, const uint32_t *, uint32_t *, uint32_t *, uint32_t *,
                      uint32_t *, uint32_t *, uint32_t, uint32_t *, uint32_t *, void *, uint32_t *, uint8_t *, uint32_t,
                      uint8_t *, const uint32_t *, const uint32_t *, uint32_t, hipStream_t);
hipError_t prk_launch_raster(const prk::FrameParams *, int, const uint32_t *, const void *, const uint32_t *,
                             const uint32_t *, const void *, uint8_t *, uint8_t *, uint32_t *, void *, size_t,
                             uint32_t *, uint32_t *, uint32_t *, void *, uint32_t *, hipEvent_t, hipEvent_t,
                             hipStream_t, hipStream_t);
hipError_t prk_walk_select_bytes(uint32_t, size_t *);
hipError_t prk_selftest_div_launch(uint32_t n, uint64_t seed, unsigned long long *bad, hipStream_t s);
hipError_t prk_obj_tables(const void *, uint32_t, uint32_t, uint32_t, void *, uint32_t *, uint32_t *, hipStream_t);
hipError_t prk_objtri_count(const prk::FrameParams *, const void *, const uint32_t *, const uint32_t *, uint32_t,
                            uint32_t, uint32_t *, unsigned long long *, hipStream_t);
hipError_t prk_objtri_emit(const prk::FrameParams *, const void *, const uint32_t *, const uint32_t *, uint32_t,
                           uint32_t, const uint32_t *, uint32_t, uint32_t, int32_t, void *, void *, uint32_t *, int,
                           hipStream_t);
hipError_t prk_obj_sort_local(const void *, const uint32_t *, uint32_t, const uint32_t *, const void *, const void *,
                              void *, void *, uint32_t *, hipStream_t);
hipError_t prk_obj_sort(void *, uint32_t *, void *, uint32_t *, uint32_t, uint32_t, void *, size_t *, hipStream_t);
hipError_t prk_obj_gather(const void *, const uint32_t *, const uint32_t *, const void *, const uint32_t *, uint32_t,
                          void *, uint32_t, void *, hipStream_t);
hipError_t prk_obj_bound(const prk::FrameParams *, const void *, uint32_t, const unsigned long long *, const void *,
                         unsigned long long *, hipStream_t);
uint32_t prk_obj_walk_lcap(void);
hipError_t prk_obj_walk(const prk::FrameParams *, const void *, uint32_t, const uint32_t *, const uint32_t *, void *,
                        const unsigned long long *, void *, void *, void *, uint32_t *, const void *, uint32_t *, int,
                        const void *, const uint32_t *, uint32_t, hipStream_t);
hipError_t prk_obj_seg(const prk::FrameParams *, const void *, uint32_t, const uint32_t *, const uint32_t *,
                       const void *, const unsigned long long *, uint32_t *, const uint32_t *, void *, void *, hipStream_t);
uint32_t prk_obj_link_cap(void);
hipError_t prk_obj_maxact(const prk::FrameParams *, const void *, const uint32_t *, uint32_t, const uint32_t *,
                          const uint32_t *, const void *, int32_t *, uint32_t, hipStream_t);
size_t prk_maxact_huge_scratch(void);
hipError_t prk_obj_maxact_huge(const prk::FrameParams *, const void *, const uint32_t *, uint32_t, uint32_t, uint32_t,
                               const uint32_t *, const uint32_t *, const void *, int32_t *, void *, hipStream_t);
uint32_t prk_obj_walk_threads(uint32_t);
hipError_t prk_obj_walk_group(const prk::FrameParams *, int32_t, uint32_t, const void *, const uint32_t *,
                              const unsigned long long *, const uint32_t *, uint32_t, int32_t *, const uint32_t *,
                              const uint32_t *, void *, const unsigned long long *, void *, void *, void *, void *,
                              uint32_t *, uint32_t *, const uint32_t *, hipStream_t);
uint32_t prk_big_max_entries(void);
uint64_t prk_big_slice_ints(uint32_t, uint32_t, uint32_t);
uint32_t prk_big_lds_cap(void);
hipError_t prk_big_walk(const prk::FrameParams *, int32_t, int, const void *, const uint32_t *, const unsigned long long *,
                        const uint32_t *, const uint32_t *, uint32_t, uint32_t, int32_t *, const uint32_t *,
                        const uint32_t *, const void *, const unsigned long long *, void *, void *, uint32_t *,
                        uint32_t *, const uint32_t *, hipStream_t);
hipError_t prk_pr_walk_begin(const prk::FrameParams *, const prk::PrWalkArgs *, hipStream_t);
hipError_t prk_pr_walk_group(const prk::FrameParams *, const prk::PrWalkArgs *, int32_t, uint32_t, const uint32_t *,
                             uint32_t, uint32_t, hipStream_t);
hipError_t prk_pr_walk_end(const prk::PrWalkArgs *, hipStream_t);
uint32_t prk_pr_chunk_rows(void);
int32_t prk_pr_max_row_entries(void);
int32_t prk_pr_max_rows(void);
hipError_t prk_span_finish(const prk::FrameParams *, const void *, uint32_t, void *, void *, void *, hipStream_t);
hipError_t prk_scan_u32(const uint32_t *, uint32_t *, uint32_t, void *, size_t *, hipStream_t);
hipError_t prk_scan_u64(const unsigned long long *, unsigned long long *, uint32_t, void *, size_t *, hipStream_t);
hipError_t prk_span_count(const prk::FrameParams *, const void *, uint32_t, uint32_t *, hipStream_t);
hipError_t prk_span_bin(const prk::FrameParams *, const void *, uint32_t, const uint32_t *, uint32_t *, uint32_t *,
                        hipStream_t);
hipError_t prk_launch_spans(const prk::FrameParams *, const uint32_t *, const uint32_t *, const void *,
                            const void *, const void *, uint32_t, const uint32_t *, uint32_t *, uint32_t *,
                            hipStream_t);
}

// prk_spans.hip's object descriptor, and the runs of objects the device
// expands into them (prk_spans.hip ObjRun).
struct ObjDesc {
    uint32_t draw, g0, tris, tri0, kind, src, nsrc, k1off;
};
struct ObjRun {
    uint32_t kind, draw, obj0, count, per, tri_count, first_global, tri0, k0base, src_off, src_n, k1off;
};
constexpr uint32_t kObjWaveTris = 48;        // objects of this many triangles or more
constexpr uint64_t kPrMaxEntries = 1ull << 23;  // the chunked walk's list entries per pass (~3 GB of scratch)
constexpr int kWaveListArrays = 9;           // prk_spans.hip WaveList: int32 arrays of cap + 2 entries

// AVX frames shade through span records (k_walk + k_pix); must match
// PRK_SPAN_RECORDS of prk_kernels.hip.
#define PRK_SPAN_RECORDS_HOST 1
// Per-frame scratch sets in flight: a frame whose target band has at most
// kSmallBandPx pixels (64 Mpx) cycles PRK_FRAME_SETS sets, larger ones 2 (the set
// count nsets; consecutive frames take consecutive sets): with three, frame k+1's binning need not wait for
// frame k-1's raster (round 2, band of 512 x 4096 px, one rank of 8: 0.284 ->
// 0.247 ms; 1024 rows: 0.405 -> 0.378; the whole 4096^2 frame then 1-3 %
// slower, with the host waiting for every frame's count).
#ifndef PRK_FRAME_SETS
#define PRK_FRAME_SETS 3
#endif
// Round 3 (lazy bin count): three sets for every target up to 64 Mpx (C5
// included) — the whole C3b frame 1.049-1.053 -> 1.041-1.044 ms (interleaved
// A/B, three rounds); round 2 measured three sets 1-3 % slower there when the
// host waited for every frame's count.
#ifndef PRK_SMALL_BAND_LOG2
#define PRK_SMALL_BAND_LOG2 26
#endif
constexpr size_t kSmallBandPx = (size_t)1 << PRK_SMALL_BAND_LOG2;

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct Geometry {
    const float *V = nullptr, *C = nullptr, *N = nullptr, *UV = nullptr;
    uint32_t vertex_count = 0;
    uint32_t cap[4] = {0, 0, 0, 0};  // owned V / C / N / UV buffers hold this many vertices
    bool owned = false;
};

struct Texture {
    uint8_t *mem = nullptr;
    int32_t w = 0, h = 0, pitch = 0;
    int32_t filter = 0;  // PRK_FILTER_*
};

int status_of(hipError_t e) {
    if (e == hipSuccess) return PRK_OK;
    static const bool trace = std::getenv("PRK_TRACE_HIP") != nullptr;  // diagnostics: name the HIP error
    if (trace) std::fprintf(stderr, "prk: HIP error %d (%s)\n", (int)e, hipGetErrorName(e));
    if (e == hipErrorOutOfMemory) return PRK_ERR_NOMEM;
    return PRK_ERR_DEVICE;
}

}  // namespace

struct prk_context {
    int device = 0;
    hipStream_t own_stream = nullptr;
    // prk_geometry_write: copies on copy_stream after read_ev (the end of the
    // last flush); the next flush's streams wait for in_ev
    hipStream_t copy_stream = nullptr;
    hipEvent_t in_ev = nullptr, read_ev = nullptr;
    bool in_wait = false, read_rec = false;
    // target
    void *color = nullptr;
    int32_t pitch = 0;
    float *zbuf = nullptr;
    int32_t W = 0, H = 0, row0 = 0, row1 = 0;
    bool owns_target = false;
    // camera + lights: transform / lights set the draws up (FillEdgeTable's
    // ProjectVertex and Gouraud lighting), shade_* shade their spans (Phong and
    // UnprojectVertex, read when DrawModel* runs); prk_set_camera sets both
    prk_transform transform{};
    prk_light_data lights{};
    prk_transform shade_transform{};
    prk_light_data shade_lights{};
    bool have_camera = false;
    bool clear_pending = false;  // prk_target_clear_on_flush
    uint32_t clear_color = 0;
    float clear_z = 0.0f;
    // resources
    std::vector<Geometry> geoms;
    std::vector<Texture> texs;
    std::vector<prk::DrawRec> draws;
    uint32_t pending_tris = 0;
    std::vector<prk_edge> pend_edges;  // prk_draw_edges input of the pending frame
    std::vector<prk_span> pend_spans;  // prk_draw_spans input of the pending frame
    // Per-frame scratch, nsets of them in use (2, or PRK_FRAME_SETS for small
    // bands): frame k bins (and, on span-record frames, runs k_vis) into the
    // set after frame k-1's on bin_stream while frame k-1 shades on the
    // flush's stream.
    struct BinSet {
        DevBuf d_draws, d_texs, d_tri_draw, d_ranges, d_tri_n, d_tri_off, d_pair_tri, d_keys_a, d_vals_a, d_keys_b,
            d_bins, d_offs, d_temp, d_won, d_list, d_nwin, d_wtag, d_recs, d_trwon, d_wlist, d_seltemp, d_trec,
            d_ghist, d_tile_tot, d_chunk, d_info, d_runlist, d_run_n;
        uint32_t *h_info = nullptr;       // pinned: [entry count, overflow] of the set's last binning
        hipEvent_t counted_ev = nullptr;  // h_info of this set's binning has landed
        hipEvent_t listed_ev = nullptr;   // a band frame's run lists are written (k_band_rec may start)
        // bytes last uploaded into d_draws / d_texs and the buffer they went
        // to: an unchanged table (every frame of a static scene) is not sent again
        std::vector<uint8_t> h_draws, h_texs;
        const void *h_draws_at = nullptr, *h_texs_at = nullptr;
        hipEvent_t free_ev = nullptr;    // the raster that read this set is done
        hipEvent_t binned_ev = nullptr;  // this set's binning is done
        bool used = false;
    };
    static constexpr int kSets = PRK_FRAME_SETS;
    BinSet bset[kSets];
    hipStream_t bin_stream = nullptr;
    hipStream_t vis_stream = nullptr;  // k_vis of span-record frames
    DevBuf d_winners, d_anomaly, d_prof;
    // z early: the last flush was a span-record pass, whose k_vis writes the
    // final z (k_pix only the colour): a download takes z from the event after
    // k_vis (ev[z_slot][3]) while the frame shades.  d_negz counts the -0.0
    // z k_pix wrote over k_vis's +0.0 since the last download.
    DevBuf d_negz;
    bool early_z = false;  // prk_set_early_z
    bool z_early = false;
    int z_slot = -1;
    hipEvent_t s_mark = nullptr;  // flush-stream point the bin stream waits for (prior target contents)
    uint32_t *h_total = nullptr;  // pinned
    uint32_t pair_hint = 0;       // entry count of the last frame (counting-sort capacity)
    int32_t tile_w = 256, tile_h = 8;  // measured best for C3b
    // Automatic tile (until prk_set_tile): 256x8, or narrower tiles for frames
    // with few bin entries per tile (under one wave's 64-entry chunk per
    // tile: 32x8, C2; under 8: 64x8, C1 — the binning's per-tile passes then
    // cost more than the extra parallelism gains), decided from a frame's
    // count at 256x8 and kept while the triangle count and the band stay
    // within 2x of that frame's (measured, profiles/r02b/small_config_tiles.log).
    bool tile_auto = true;
    int32_t auto_small = 0;  // 0: 256x8; else the small tile width (64: under 8 entries per tile, 32: under 64)
    // Wide tiles: an all-AVX frame whose triangles make >= 4.5 bin entries
    // each at 256x8 (large triangles: C5's radius-32 soup makes 5.6) draws
    // faster at 512x8 (C5 3.24 -> 2.97 ms, its band of 8 0.474 -> 0.426 ms;
    // C3b, 3.2 entries a triangle, is fastest at 256x8: 1.021 vs 1.029 ms;
    // scalar C3a is slower at 512x8), decided and kept like auto_small.
    int32_t auto_wide = 0;
    uint32_t auto_T = 0;
    int32_t auto_px = 0;
    // all-AVX frames: per-triangle setup records; the AVX k_vis / k_walk read
    // them (prk_kernels.hip PRK_SETUP_REC), so they are not optional
    bool setup_rec = true;
    bool debug = false;
    bool winners_valid = false;
    prk_stats stats{};
    // Timing ring: 6 events per flush.
    static constexpr int kRing = 32;
    // bin start, bin end (bin_stream); raster end, k_vis end, k_walk end,
    // raster start (flush stream)
    hipEvent_t ev[kRing][6] = {};
    bool pending[kRing] = {};
    bool split_span[kRing] = {};  // the slot's flush ran k_walk + k_pix
    uint32_t frame = 0;
    int last_slot = -1;
    int last_set = -1;  // scratch set of the last per-triangle pass
    // The last per-triangle pass, whose bin entry count the host has not read
    // yet (flush_tris with `defer`): prk_flush returns once the frame is
    // queued, and the count is read at the next call that needs it
    // (resolve_count) — by then the binning has long finished, so the host
    // no longer waits for every frame's binning before queueing the next
    // frame.  A pass whose entries overflowed the scratch is re-run there,
    // before anything else is queued or read, with the state it was queued
    // with (target, camera, tile, clear).
    struct PendingCount {
        bool active = false;
        int set = 0;
        hipStream_t s = nullptr;
        std::vector<prk::DrawRec> draws;
        uint32_t T = 0, win_base = 0, ntiles = 0;
        bool fuse = false, debug = false;
        void *color = nullptr;
        int32_t pitch = 0;
        float *zbuf = nullptr;
        int32_t W = 0, H = 0, row0 = 0, row1 = 0, tile_w = 0, tile_h = 0;
        prk_transform transform{}, shade_transform{};
        prk_light_data lights{}, shade_lights{};
        uint32_t clear_color = 0;
        float clear_z = 0.0f;
    } pcount;
    // Span path (whole-object AETs) scratch, reused frame to frame.
    struct SpanScratch {
        DevBuf d_stage, d_edges, d_ord, d_temp, d_recs, d_pos, d_span_tri, d_scnt, d_soff, d_keys_a, d_vals_a,
            d_keys_b, d_vals_b, d_offs, d_nwin, d_wtag, d_srecs, d_work, d_ekeys, d_ekeys2, d_evals, d_ecnt, d_escan,
            d_rcnt, d_rscan, d_bound, d_oslot, d_pool, d_err, d_raw, d_most, d_cls, d_prrow, d_prcnt, d_preoff,
            d_prfge, d_prccur, d_prkey, d_prest, d_prsst, d_preend, d_preendm, d_prmatch, d_prsidx, d_prsm, d_prstat,
            d_segcnt, d_segoff, d_segs, d_wy, d_mhuge, d_objtab, d_k0tab;
        // the pass's host tables, packed into pinned memory for one upload
        // (stage_ev: that upload, before the staging is rewritten)
        char *h_stage = nullptr;
        size_t stage_cap = 0;
        hipEvent_t stage_ev = nullptr;
        bool stage_busy = false;
        // host tables of the pass, kept until their asynchronous uploads ran
        std::vector<ObjRun> h_runs;
        std::vector<uint32_t> h_big_gl, h_big_cap, h_k1src;
        std::vector<unsigned long long> h_big_off;
        std::vector<prk::DrawRec> h_draws;
        std::vector<prk::TexRec> h_texs;
        uint32_t *h_rb = nullptr;  // pinned readback words
        char *h_cls = nullptr;     // pinned: the large objects' most active entries, then their walk groups
        size_t cls_cap = 0;
    } spans;
};

static int resolve_count(prk_context *c);
// Calls that read or replace the target, or change what a re-run of the
// pending pass would read, first resolve its count (PendingCount).
#define RESOLVE_COUNT(c)                             \
    do {                                             \
        const int _rc = resolve_count(c);            \
        if (_rc != PRK_OK) return _rc;               \
    } while (0)

#define PRK_TRY(expr)                              \
    do {                                           \
        hipError_t _e = (expr);                    \
        if (_e != hipSuccess) return status_of(_e); \
    } while (0)

// ---- one ROCm runtime per process (prk.h prk_create) ------
namespace {
struct MapScan {
    std::vector<std::string> hip, smi;  // distinct mapped files of each library
};
int scan_object(struct dl_phdr_info *info, size_t, void *data) {
    MapScan &m = *static_cast<MapScan *>(data);
    const char *path = info->dlpi_name;
    if (!path || !*path) return 0;
    const char *base = std::strrchr(path, '/');
    base = base ? base + 1 : path;
    std::vector<std::string> *v = nullptr;
    if (std::strncmp(base, "libamdhip64", 11) == 0) v = &m.hip;
    else if (std::strncmp(base, "librocm_smi64", 13) == 0) v = &m.smi;
    if (!v) return 0;
    char real[4096];
    const std::string key = realpath(path, real) ? std::string(real) : std::string(path);
    if (std::find(v->begin(), v->end(), key) == v->end()) v->push_back(key);
    return 0;
}
// Runs before the destructors of every library loaded earlier (exit handlers
// run last-registered first): ends the process with its own exit status
// before the duplicated librocm_smi64 destructors free one map twice.
void exit_guard(int status, void *) {
    std::fflush(nullptr);
    _exit(status);
}
std::atomic<bool> g_guarded{false};
}  // namespace

extern "C" {

int prk_runtime_check(void) {
    MapScan m;
    dl_iterate_phdr(scan_object, &m);
    if (m.hip.size() <= 1 && m.smi.size() <= 1) return PRK_OK;
    if (!g_guarded.exchange(true)) {
        std::fprintf(stderr,
                     "prk: %zu copies of libamdhip64 and %zu of librocm_smi64 are mapped in this process (e.g. "
                     "/opt/rocm's, loaded with libprk_hip.so, and torch's own): load torch (or the framework that "
                     "ships its own ROCm) BEFORE libprk_hip.so (INTEGRATION.md, 'One ROCm stack per process'); "
                     "the process will end at exit before their destructors run\n",
                     m.hip.size(), m.smi.size());
        // The guard ends the process before every exit handler registered
        // earlier (profiler flushes, LSan, earlier libraries' static
        // destructors): without it the duplicated librocm_smi64 destructors
        // abort the process there anyway (SIGABRT, the same handlers lost).
        // PRK_EXIT_GUARD=0 leaves the exit path alone (the host takes the abort).
        const char *g = std::getenv("PRK_EXIT_GUARD");
        if (!(g && g[0] == '0')) on_exit(exit_guard, nullptr);
    }
    return PRK_ERR_RUNTIME_MIX;
}

const char *prk_version(void) { return "prk 0.1 (gfx950)"; }

int prk_device_count(int *out) {
    if (!out) return PRK_ERR_ARG;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return PRK_OK;
}

// Self-test of the shared-divisor quotients against the compiler's division
// (prk.h).  Runs on `device`, synchronously.
int prk_selftest_div(int32_t device, uint32_t n, uint64_t seed, uint64_t *mismatches) {
    if (!mismatches || device < 0) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(device));
    unsigned long long *d = nullptr;
    PRK_TRY(hipMalloc(&d, sizeof(unsigned long long)));
    hipError_t e = hipMemset(d, 0, sizeof(unsigned long long));
    if (e == hipSuccess) e = prk_selftest_div_launch(n, seed, d, nullptr);
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return status_of(e);
    *mismatches = h;
    return PRK_OK;
}

int prk_create(int device, prk_context **out) {
    if (!out) return PRK_ERR_ARG;
    *out = nullptr;
    {
        const int rc = prk_runtime_check();
        if (rc != PRK_OK) return rc;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return PRK_ERR_DEVICE;
    if (device < 0 || device >= n) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(device));
    prk_context *c = new (std::nothrow) prk_context();
    if (!c) return PRK_ERR_NOMEM;
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->bin_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->vis_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->s_mark, hipEventDisableTiming);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->in_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->read_ev, hipEventDisableTiming);
    for (int i = 0; i < prk_context::kSets && e == hipSuccess; ++i) {
        e = hipEventCreateWithFlags(&c->bset[i].free_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->bset[i].binned_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->bset[i].counted_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->bset[i].listed_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipHostMalloc((void **)&c->bset[i].h_info, 2 * sizeof(uint32_t), hipHostMallocDefault);
    }
    for (int i = 0; i < prk_context::kRing && e == hipSuccess; ++i)
        for (int k = 0; k < 6 && e == hipSuccess; ++k) e = hipEventCreate(&c->ev[i][k]);
    if (e == hipSuccess) e = hipHostMalloc((void **)&c->h_total, sizeof(uint32_t), hipHostMallocDefault);
    if (e != hipSuccess) {
        prk_destroy(c);
        return status_of(e);
    }
    *out = c;
    return PRK_OK;
}

int prk_destroy(prk_context *c) {
    if (!c) return PRK_ERR_ARG;
    (void)prk_runtime_check();  // (a runtime loaded since prk_create: guard the exit)
    // Destroy never queues GPU work: a frame whose bin count was never read
    // (PendingCount) is dropped, not re-run — its target may already belong
    // to someone else (a torch tensor freed at interpreter exit, a peer
    // context), and a re-run there is exactly what a caller tearing down does
    // not expect.  Only waits and frees follow.
    c->pcount.active = false;
    c->pcount.draws.clear();
    (void)hipSetDevice(c->device);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    (void)hipDeviceSynchronize();
    for (auto &g : c->geoms)
        if (g.owned) {
            (void)hipFree((void *)g.V);
            (void)hipFree((void *)g.C);
            (void)hipFree((void *)g.N);
            (void)hipFree((void *)g.UV);
        }
    for (auto &t : c->texs) (void)hipFree(t.mem);
    if (c->owns_target) {
        (void)hipFree(c->color);
        (void)hipFree(c->zbuf);
    }
    for (auto &B : c->bset) {
        DevBuf *bb[] = {&B.d_draws, &B.d_texs, &B.d_tri_draw, &B.d_ranges, &B.d_tri_n, &B.d_tri_off, &B.d_pair_tri,
                        &B.d_keys_a, &B.d_vals_a, &B.d_keys_b, &B.d_bins, &B.d_offs, &B.d_temp, &B.d_won,
                        &B.d_list, &B.d_nwin, &B.d_wtag, &B.d_recs, &B.d_trwon, &B.d_wlist, &B.d_seltemp,
                        &B.d_trec, &B.d_ghist, &B.d_tile_tot, &B.d_chunk, &B.d_info, &B.d_runlist, &B.d_run_n};
        for (DevBuf *b : bb) b->release();
        if (B.free_ev) (void)hipEventDestroy(B.free_ev);
        if (B.binned_ev) (void)hipEventDestroy(B.binned_ev);
        if (B.counted_ev) (void)hipEventDestroy(B.counted_ev);
        if (B.listed_ev) (void)hipEventDestroy(B.listed_ev);
        if (B.h_info) (void)hipHostFree(B.h_info);
    }
    DevBuf *bufs[] = {&c->d_winners, &c->d_anomaly, &c->d_prof, &c->d_negz};
    for (DevBuf *b : bufs) b->release();
    {
        auto &S = c->spans;
        DevBuf *sb[] = {&S.d_stage, &S.d_edges, &S.d_ord, &S.d_temp, &S.d_recs, &S.d_pos, &S.d_span_tri, &S.d_scnt,
                        &S.d_soff, &S.d_keys_a, &S.d_vals_a, &S.d_keys_b, &S.d_vals_b, &S.d_offs, &S.d_nwin,
                        &S.d_wtag, &S.d_srecs, &S.d_work, &S.d_ekeys, &S.d_ekeys2, &S.d_evals, &S.d_ecnt,
                        &S.d_escan, &S.d_rcnt, &S.d_rscan, &S.d_bound, &S.d_oslot, &S.d_pool, &S.d_err,
                        &S.d_raw, &S.d_most, &S.d_cls, &S.d_prrow, &S.d_prcnt, &S.d_preoff, &S.d_prfge,
                        &S.d_prccur, &S.d_prkey, &S.d_prest, &S.d_prsst, &S.d_preend, &S.d_preendm,
                        &S.d_prmatch, &S.d_prsidx, &S.d_prsm, &S.d_prstat, &S.d_segcnt, &S.d_segoff,
                        &S.d_segs, &S.d_wy, &S.d_mhuge, &S.d_objtab, &S.d_k0tab};
        for (DevBuf *b : sb) b->release();
        if (S.h_rb) (void)hipHostFree(S.h_rb);
        if (S.stage_ev) {
            if (S.stage_busy) (void)hipEventSynchronize(S.stage_ev);
            (void)hipEventDestroy(S.stage_ev);
        }
        if (S.h_stage) (void)hipHostFree(S.h_stage);
        if (S.h_cls) (void)hipHostFree(S.h_cls);
    }
    if (c->s_mark) (void)hipEventDestroy(c->s_mark);
    if (c->in_ev) (void)hipEventDestroy(c->in_ev);
    if (c->read_ev) (void)hipEventDestroy(c->read_ev);
    if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
    if (c->h_total) (void)hipHostFree(c->h_total);
    for (auto &slot : c->ev)
        for (auto &e : slot)
            if (e) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->bin_stream) (void)hipStreamDestroy(c->bin_stream);
    if (c->vis_stream) (void)hipStreamDestroy(c->vis_stream);
    delete c;
    return PRK_OK;
}

static void drop_target(prk_context *c) {
    c->z_early = false;
    if (c->owns_target) {
        (void)hipFree(c->color);
        (void)hipFree(c->zbuf);
    }
    c->color = nullptr;
    c->zbuf = nullptr;
    c->owns_target = false;
    c->W = c->H = c->row0 = c->row1 = 0;
}

int prk_target_bind(prk_context *c, void *color, int32_t pitch_bytes, float *zbuf, int32_t width,
                    int32_t height, int32_t row0, int32_t row1) {
    if (!c || !color || !zbuf || width <= 0 || height <= 0 || row0 < 0 || row1 > height || row0 >= row1 ||
        pitch_bytes < width * 4 || (pitch_bytes & 3))
        return PRK_ERR_ARG;
    // the pending frame's count first, whoever owns its target: an overflowed
    // frame is re-run into the target it was queued with before a caller
    // hands that memory to anything else (a gather, the next frame)
    RESOLVE_COUNT(c);
    drop_target(c);
    c->color = color;
    c->pitch = pitch_bytes;
    c->zbuf = zbuf;
    c->W = width;
    c->H = height;
    c->row0 = row0;
    c->row1 = row1;
    c->winners_valid = false;
    return PRK_OK;
}

int prk_target_alloc(prk_context *c, int32_t width, int32_t height, int32_t row0, int32_t row1,
                     void **color_out, float **zbuf_out) {
    if (!c || width <= 0 || height <= 0 || row0 < 0 || row1 > height || row0 >= row1) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    PRK_TRY(hipSetDevice(c->device));
    drop_target(c);
    size_t px = (size_t)width * (row1 - row0);
    void *col = nullptr;
    float *z = nullptr;
    hipError_t e = hipMalloc(&col, px * 4);
    if (e == hipSuccess) e = hipMalloc((void **)&z, px * 4);
    if (e != hipSuccess) {
        (void)hipFree(col);
        (void)hipFree(z);
        return status_of(e);
    }
    c->color = col;
    c->zbuf = z;
    c->pitch = width * 4;
    c->W = width;
    c->H = height;
    c->row0 = row0;
    c->row1 = row1;
    c->owns_target = true;
    c->winners_valid = false;
    if (color_out) *color_out = col;
    if (zbuf_out) *zbuf_out = z;
    return PRK_OK;
}

__global__ void k_fill_target(uint32_t *color, int32_t pitch, float *z, int32_t W, int32_t rows,
                              uint32_t cval, float zval) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t n = (size_t)W * rows;
    if (i >= n) return;
    size_t r = i / W, x = i % W;
    reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(color) + r * pitch)[x] = cval;
    z[i] = zval;
}

int prk_target_clear(prk_context *c, uint32_t color, float z) {
    if (!c) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    c->z_early = false;  // (z written outside a frame)
    if (!c->color) return PRK_ERR_NO_TARGET;
    PRK_TRY(hipSetDevice(c->device));
    // after a prk_target_upload_async still in flight (it would land on top)
    if (c->in_wait) PRK_TRY(hipStreamWaitEvent(c->own_stream, c->in_ev, 0));
    size_t n = (size_t)c->W * (c->row1 - c->row0);
    hipLaunchKernelGGL(k_fill_target, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->own_stream,
                       (uint32_t *)c->color, c->pitch, c->zbuf, c->W, c->row1 - c->row0, color, z);
    PRK_TRY(hipGetLastError());
    return PRK_OK;
}

int prk_target_clear_on_flush(prk_context *c, uint32_t color, float z) {
    if (!c) return PRK_ERR_ARG;
    if (!c->color) return PRK_ERR_NO_TARGET;
    c->clear_pending = true;
    c->clear_color = color;
    c->clear_z = z;
    return PRK_OK;
}

int prk_target_download(prk_context *c, uint32_t *color_host, int32_t host_pitch, float *z_host) {
    if (!c) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    if (!c->color) return PRK_ERR_NO_TARGET;
    PRK_TRY(hipSetDevice(c->device));
    int rows = c->row1 - c->row0;
    const size_t zbytes = (size_t)c->W * rows * 4;
    // A span-record frame's z is final after its k_vis: it goes down while
    // the frame shades (the copy engine holds the link while k_walk / k_pix
    // run), the colour after the frame.
    const bool early = z_host && c->z_early && c->z_slot >= 0 && c->d_negz.p;
    if (early) {
        PRK_TRY(hipStreamWaitEvent(c->copy_stream, c->ev[c->z_slot][3], 0));
        PRK_TRY(hipMemcpyAsync(z_host, c->zbuf, zbytes, hipMemcpyDeviceToHost, c->copy_stream));
    }
    PRK_TRY(hipStreamSynchronize(c->own_stream));
    PRK_TRY(hipDeviceSynchronize());
    if (color_host)
        PRK_TRY(hipMemcpy2D(color_host, host_pitch, c->color, c->pitch, (size_t)c->W * 4, rows,
                            hipMemcpyDeviceToHost));
    if (early) {  // a -0.0 z written by k_pix after k_vis's +0.0: take z again
        uint32_t negz = 0;
        PRK_TRY(hipMemcpy(&negz, c->d_negz.p, 4, hipMemcpyDeviceToHost));
        if (negz) {
            PRK_TRY(hipMemcpy(z_host, c->zbuf, zbytes, hipMemcpyDeviceToHost));
            PRK_TRY(hipMemset(c->d_negz.p, 0, 4));
        }
    } else if (z_host) {
        PRK_TRY(hipMemcpy(z_host, c->zbuf, zbytes, hipMemcpyDeviceToHost));
    }
    return PRK_OK;
}

int prk_target_upload(prk_context *c, const uint32_t *color_host, int32_t host_pitch, const float *z_host) {
    if (!c) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    c->z_early = false;  // (z written outside a frame)
    if (!c->color) return PRK_ERR_NO_TARGET;
    PRK_TRY(hipSetDevice(c->device));
    PRK_TRY(hipStreamSynchronize(c->own_stream));
    if (c->in_wait) PRK_TRY(hipEventSynchronize(c->in_ev));  // an earlier asynchronous upload lands first
    int rows = c->row1 - c->row0;
    if (color_host)
        PRK_TRY(hipMemcpy2D(c->color, c->pitch, color_host, host_pitch, (size_t)c->W * 4, rows,
                            hipMemcpyHostToDevice));
    if (z_host) PRK_TRY(hipMemcpy(c->zbuf, z_host, (size_t)c->W * rows * 4, hipMemcpyHostToDevice));
    return PRK_OK;
}

int prk_target_upload_async(prk_context *c, const uint32_t *color_host, int32_t host_pitch, const float *z_host) {
    if (!c) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    c->z_early = false;  // (z written outside a frame)
    if (!c->color) return PRK_ERR_NO_TARGET;
    PRK_TRY(hipSetDevice(c->device));
    // after the frames already flushed (they read and write the target) and
    // whatever the context's stream holds (a clear, an earlier upload)
    if (c->read_rec) PRK_TRY(hipStreamWaitEvent(c->copy_stream, c->read_ev, 0));
    PRK_TRY(hipEventRecord(c->s_mark, c->own_stream));
    PRK_TRY(hipStreamWaitEvent(c->copy_stream, c->s_mark, 0));
    const int rows = c->row1 - c->row0;
    if (color_host)
        PRK_TRY(hipMemcpy2DAsync(c->color, c->pitch, color_host, host_pitch, (size_t)c->W * 4, rows,
                                 hipMemcpyHostToDevice, c->copy_stream));
    if (z_host)
        PRK_TRY(hipMemcpyAsync(c->zbuf, z_host, (size_t)c->W * rows * 4, hipMemcpyHostToDevice, c->copy_stream));
    PRK_TRY(hipEventRecord(c->in_ev, c->copy_stream));
    c->in_wait = true;
    return PRK_OK;
}

int prk_set_camera(prk_context *c, const prk_transform *t, const prk_light_data *l) {
    if (!c || !t || !l || l->LightCount > PRK_MAX_LIGHTS) return PRK_ERR_ARG;
    c->transform = *t;
    c->lights = *l;
    c->shade_transform = *t;
    c->shade_lights = *l;
    c->have_camera = true;
    return PRK_OK;
}

int prk_set_shade_camera(prk_context *c, const prk_transform *t, const prk_light_data *l) {
    if (!c || !t || !l || l->LightCount > PRK_MAX_LIGHTS) return PRK_ERR_ARG;
    if (!c->have_camera) return PRK_ERR_ARG;  // the setup camera first (prk_set_camera)
    c->shade_transform = *t;
    c->shade_lights = *l;
    return PRK_OK;
}

static bool bitmap_ok(const prk_bitmap *b) {
    return b && b->Memory && b->Width > 0 && b->Height > 0 && b->Pitch >= 4 * b->Width && !(b->Pitch & 3);
}

// Copy the caller's Height rows (Pitch bytes each) into a texture holding
// Height + 1 rows, the last one the zeroed guard row that the u == 1 / v == 1
// over-read lands on: the caller's loaded_bitmap is read
// exactly as the reference reads it (Memory, Width, Height, Pitch,
// projekt.cpp:1506, 1881-1935) and never past its last row.
static hipError_t texture_fill(const Texture &t, const prk_bitmap *b) {
    hipError_t e = hipMemcpy(t.mem, b->Memory, (size_t)b->Pitch * b->Height, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(t.mem + (size_t)b->Pitch * b->Height, 0, (size_t)b->Pitch);
    return e;
}

int prk_texture_create(prk_context *c, const prk_bitmap *b, int32_t *handle_out) {
    if (!c || !bitmap_ok(b) || !handle_out) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    Texture t;
    t.w = b->Width;
    t.h = b->Height;
    t.pitch = b->Pitch;
    PRK_TRY(hipMalloc((void **)&t.mem, (size_t)b->Pitch * (b->Height + 1)));
    hipError_t e = texture_fill(t, b);
    if (e != hipSuccess) {
        (void)hipFree(t.mem);
        return status_of(e);
    }
    *handle_out = (int32_t)c->texs.size();
    c->texs.push_back(t);
    return PRK_OK;
}

int prk_texture_update(prk_context *c, int32_t handle, const prk_bitmap *b) {
    if (!c || handle < 0 || (size_t)handle >= c->texs.size() || !bitmap_ok(b)) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    PRK_TRY(hipSetDevice(c->device));
    Texture &t = c->texs[handle];
    PRK_TRY(hipDeviceSynchronize());  // frames in flight may still sample it
    if (t.w != b->Width || t.h != b->Height || t.pitch != b->Pitch) {
        uint8_t *m = nullptr;
        PRK_TRY(hipMalloc((void **)&m, (size_t)b->Pitch * (b->Height + 1)));
        (void)hipFree(t.mem);
        t.mem = m;
        t.w = b->Width;
        t.h = b->Height;
        t.pitch = b->Pitch;
    }
    PRK_TRY(texture_fill(t, b));
    return PRK_OK;
}

// Allocations of 2 MB and more: heap memory on transparent huge pages,
// page-locked with hipHostRegister, instead of hipHostMalloc's 4-KB pinned
// pages -- the drop-in's staging arena takes ~150 MB of per-call vertex
// snapshots a frame, which the 2-MB pages make cheaper for the CPU (TLB).
// PRK_HOST_ALLOC_THP=0: hipHostMalloc for every size.
static std::mutex g_thp_mu;
static std::map<void *, size_t> g_thp;  // (any context may free)
static bool host_alloc_thp() {
    static const bool on = [] {
        const char *e = std::getenv("PRK_HOST_ALLOC_THP");
        return !(e && e[0] == '0');
    }();
    return on;
}

int prk_host_alloc(prk_context *c, size_t bytes, void **out) {
    if (!c || !out) return PRK_ERR_ARG;
    *out = nullptr;
    PRK_TRY(hipSetDevice(c->device));
    constexpr size_t kHuge = (size_t)2 << 20;
    if (bytes >= kHuge && host_alloc_thp()) {
        const size_t sz = (bytes + kHuge - 1) & ~(kHuge - 1);
        void *p = std::aligned_alloc(kHuge, sz);
        if (!p) return PRK_ERR_NOMEM;
        (void)madvise(p, sz, MADV_HUGEPAGE);  // (best effort)
        memset(p, 0, sz);                      // (faulted in on huge pages before the pinning)
        const hipError_t e = hipHostRegister(p, sz, hipHostRegisterPortable);
        if (e != hipSuccess) {
            std::free(p);
            return status_of(e);
        }
        std::lock_guard<std::mutex> g(g_thp_mu);
        g_thp[p] = sz;
        *out = p;
        return PRK_OK;
    }
    PRK_TRY(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return PRK_OK;
}

int prk_host_free(prk_context *c, void *p) {
    if (!c) return PRK_ERR_ARG;
    if (!p) return PRK_OK;
    {
        std::lock_guard<std::mutex> g(g_thp_mu);
        auto it = g_thp.find(p);
        if (it != g_thp.end()) {
            g_thp.erase(it);
            const hipError_t e = hipHostUnregister(p);
            std::free(p);
            return e == hipSuccess ? PRK_OK : status_of(e);
        }
    }
    PRK_TRY(hipHostFree(p));
    return PRK_OK;
}

int prk_host_register(prk_context *c, void *p, size_t bytes) {
    if (!c || !p || !bytes) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    PRK_TRY(hipHostRegister(p, bytes, hipHostRegisterDefault));
    return PRK_OK;
}

int prk_host_unregister(prk_context *c, void *p) {
    if (!c || !p) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    PRK_TRY(hipHostUnregister(p));
    return PRK_OK;
}

int prk_texture_set_filter(prk_context *c, int32_t handle, int32_t filter) {
    if (!c || handle < 0 || (size_t)handle >= c->texs.size()) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    if (filter != PRK_FILTER_NEAREST && filter != PRK_FILTER_BILINEAR) return PRK_ERR_ARG;
    c->texs[handle].filter = filter;
    return PRK_OK;
}

static int upload_array(const float *src, size_t n, const float **dst) {
    *dst = nullptr;
    if (!src) return PRK_OK;
    float *d = nullptr;
    PRK_TRY(hipMalloc((void **)&d, n * sizeof(float)));
    hipError_t e = hipMemcpy(d, src, n * sizeof(float), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(d);
        return status_of(e);
    }
    *dst = d;
    return PRK_OK;
}

int prk_geometry_create(prk_context *c, const float *v, const float *col, const float *n, const float *uv,
                        uint32_t vertex_count, int32_t *handle_out) {
    if (!c || !v || !handle_out || vertex_count % 3) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    Geometry g;
    g.vertex_count = vertex_count;
    for (int k = 0; k < 4; ++k) g.cap[k] = vertex_count;
    g.owned = true;
    int rc = upload_array(v, (size_t)vertex_count * 3, &g.V);
    if (rc == PRK_OK) rc = upload_array(col, (size_t)vertex_count * 4, &g.C);
    if (rc == PRK_OK) rc = upload_array(n, (size_t)vertex_count * 3, &g.N);
    if (rc == PRK_OK) rc = upload_array(uv, (size_t)vertex_count * 2, &g.UV);
    if (rc != PRK_OK) {
        (void)hipFree((void *)g.V);
        (void)hipFree((void *)g.C);
        (void)hipFree((void *)g.N);
        (void)hipFree((void *)g.UV);
        return rc;
    }
    *handle_out = (int32_t)c->geoms.size();
    c->geoms.push_back(g);
    return PRK_OK;
}

// Replace a library-owned geometry's contents (the reference re-reads
// VertexData at every FillEdgeTable, projekt.cpp:3898-3925).  Buffers are kept
// when large enough; frames in flight finish first.  Draws recorded before
// the update read the new contents.
int prk_geometry_update(prk_context *c, int32_t handle, const float *v, const float *col, const float *n,
                        const float *uv, uint32_t vertex_count) {
    if (!c || handle < 0 || (size_t)handle >= c->geoms.size() || !v || vertex_count % 3) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    Geometry &g = c->geoms[handle];
    if (!g.owned) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    PRK_TRY(hipDeviceSynchronize());
    const float *src[4] = {v, col, n, uv};
    const float **dst[4] = {&g.V, &g.C, &g.N, &g.UV};
    const size_t comp[4] = {3, 4, 3, 2};
    for (int k = 0; k < 4; ++k) {  // an array passed as null keeps its previous contents
        const size_t bytes = (size_t)vertex_count * comp[k] * sizeof(float);
        if (!src[k]) {
            // ... and grows with the vertex count: its first cap[k] vertices
            // kept, the new ones zero, so no draw reads past its allocation.
            if (*dst[k] && vertex_count > g.cap[k]) {
                const size_t old = (size_t)g.cap[k] * comp[k] * sizeof(float);
                float *d = nullptr;
                PRK_TRY(hipMalloc((void **)&d, bytes));
                hipError_t e = hipMemcpy(d, *dst[k], old, hipMemcpyDeviceToDevice);
                if (e == hipSuccess) e = hipMemset((uint8_t *)d + old, 0, bytes - old);
                if (e != hipSuccess) {
                    (void)hipFree(d);
                    return status_of(e);
                }
                (void)hipFree((void *)*dst[k]);
                *dst[k] = d;
                g.cap[k] = vertex_count;
            }
            continue;
        }
        if (!*dst[k] || vertex_count > g.cap[k]) {
            float *d = nullptr;
            PRK_TRY(hipMalloc((void **)&d, bytes ? bytes : 4));
            (void)hipFree((void *)*dst[k]);
            *dst[k] = d;
            g.cap[k] = vertex_count;
        }
        PRK_TRY(hipMemcpy((void *)*dst[k], src[k], bytes, hipMemcpyHostToDevice));
    }
    g.vertex_count = vertex_count;
    // recorded draws carry the geometry's device pointers: refresh them
    for (auto &d : c->draws)
        if (d.src_kind == 0 && d.geom == handle) {
            d.V = g.V; d.C = g.C; d.N = g.N; d.UV = g.UV;
        }
    return PRK_OK;
}

int prk_geometry_write(prk_context *c, int32_t handle, uint32_t first_vertex, uint32_t vertex_count,
                       const float *v, const float *col, const float *n, const float *uv) {
    if (!c || handle < 0 || (size_t)handle >= c->geoms.size() || first_vertex % 3 || vertex_count % 3)
        return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    const uint64_t end64 = (uint64_t)first_vertex + vertex_count;
    if (end64 > 0xFFFFFFF0ull) return PRK_ERR_ARG;
    const uint32_t end = (uint32_t)end64;
    Geometry &g = c->geoms[handle];
    if (!g.owned) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    const float *src[4] = {v, col, n, uv};
    const float **dst[4] = {&g.V, &g.C, &g.N, &g.UV};
    const size_t comp[4] = {3, 4, 3, 2};
    // Buffers that must grow (an array that exists, or is given now): by
    // half again at least, so a frame streamed in chunks reallocates rarely.
    bool grow = false;
    for (int k = 0; k < 4; ++k) grow |= (src[k] || *dst[k]) && end > g.cap[k];
    if (grow) {
        PRK_TRY(hipDeviceSynchronize());  // frames in flight and earlier writes read / fill the old buffers
        for (int k = 0; k < 4; ++k) {
            if (!(src[k] || *dst[k]) || end <= g.cap[k]) continue;
            const uint64_t want = std::max<uint64_t>(end, (uint64_t)g.cap[k] + g.cap[k] / 2);
            const uint32_t cap = (uint32_t)std::min<uint64_t>(want, 0xFFFFFFF0ull);
            const size_t bytes = (size_t)cap * comp[k] * sizeof(float);
            const size_t old = *dst[k] ? (size_t)g.cap[k] * comp[k] * sizeof(float) : 0;
            float *d = nullptr;
            PRK_TRY(hipMalloc((void **)&d, bytes));
            hipError_t e = old ? hipMemcpy(d, *dst[k], old, hipMemcpyDeviceToDevice) : hipSuccess;
            if (e == hipSuccess) e = hipMemset((uint8_t *)d + old, 0, bytes - old);
            if (e != hipSuccess) {
                (void)hipFree(d);
                return status_of(e);
            }
            (void)hipFree((void *)*dst[k]);
            *dst[k] = d;
            g.cap[k] = cap;
        }
        for (auto &d : c->draws)
            if (d.src_kind == 0 && d.geom == handle) {
                d.V = g.V; d.C = g.C; d.N = g.N; d.UV = g.UV;
            }
        c->read_rec = false;  // the device is idle
    }
    if (c->read_rec) PRK_TRY(hipStreamWaitEvent(c->copy_stream, c->read_ev, 0));
    bool any = false;
    for (int k = 0; k < 4; ++k) {
        if (!src[k] || !vertex_count) continue;
        const size_t off = (size_t)first_vertex * comp[k];
        PRK_TRY(hipMemcpyAsync((void *)(*dst[k] + off), src[k], (size_t)vertex_count * comp[k] * sizeof(float),
                               hipMemcpyHostToDevice, c->copy_stream));
        any = true;
    }
    if (any) {
        PRK_TRY(hipEventRecord(c->in_ev, c->copy_stream));
        c->in_wait = true;
    }
    g.vertex_count = end;
    return PRK_OK;
}

int prk_geometry_wrap_device(prk_context *c, const float *v, const float *col, const float *n,
                             const float *uv, uint32_t vertex_count, int32_t *handle_out) {
    if (!c || !v || !handle_out || vertex_count % 3) return PRK_ERR_ARG;
    Geometry g;
    g.V = v;
    g.C = col;
    g.N = n;
    g.UV = uv;
    g.vertex_count = vertex_count;
    g.owned = false;
    *handle_out = (int32_t)c->geoms.size();
    c->geoms.push_back(g);
    return PRK_OK;
}

int prk_draw(prk_context *c, int32_t geometry, uint32_t first_tri, uint32_t tri_count, const float P[3],
             int32_t semantics, int32_t phong, int32_t texture) {
    return prk_draw_objects(c, geometry, first_tri, tri_count, 1, P, semantics, phong, texture);
}

int prk_draw_objects(prk_context *c, int32_t geometry, uint32_t first_tri, uint32_t tri_count,
                     uint32_t tris_per_object, const float P[3], int32_t semantics, int32_t phong, int32_t texture) {
    return prk_draw_objects_setup(c, geometry, first_tri, tri_count, tris_per_object, P, semantics, phong, texture,
                                  -1);
}

int prk_draw_objects_setup(prk_context *c, int32_t geometry, uint32_t first_tri, uint32_t tri_count,
                           uint32_t tris_per_object, const float P[3], int32_t semantics, int32_t phong,
                           int32_t texture, int32_t setup) {
    if (!c || geometry < 0 || geometry >= (int32_t)c->geoms.size() || tris_per_object == 0) return PRK_ERR_ARG;
    const Geometry &g = c->geoms[geometry];
    if ((uint64_t)first_tri + tri_count > g.vertex_count / 3) return PRK_ERR_ARG;
    if (texture >= (int32_t)c->texs.size()) return PRK_ERR_ARG;
    if (setup > (PRK_SETUP_PHONG | PRK_SETUP_BITMAP)) return PRK_ERR_ARG;
    const bool tex = texture >= 0;
    // FillEdgeTable's PhongShading and Object->Bitmap (prk.h prk_setup)
    const bool fe_phong = setup < 0 ? phong != 0 : (setup & PRK_SETUP_PHONG) != 0;
    const bool fe_bitmap = setup < 0 ? tex : (setup & PRK_SETUP_BITMAP) != 0;
    int mode;
    uint32_t flags = 0;
    if (semantics == PRK_SEM_AVX || semantics == PRK_SEM_AVX_ST) {
        // FillLineOptimized dereferences Bitmap at entry (projekt.cpp:1506) and
        // its non-Phong branch stores garbage (2285-2316): undefined -> rejected.
        // The single-thread overload (2350-3358) shares both (2494, 3262-3290).
        if (!tex || !phong) return PRK_ERR_UNSUPPORTED;
        mode = prk::MODE_AVX;
        if (semantics == PRK_SEM_AVX_ST) flags = prk::DRAW_ST;
    } else if (semantics == PRK_SEM_SCALAR) {
        mode = phong ? (tex ? prk::MODE_SC_PHONG_TEX : prk::MODE_SC_PHONG)
                     : (tex ? prk::MODE_SC_GOURAUD_TEX : prk::MODE_SC_GOURAUD);
    } else {
        return PRK_ERR_ARG;
    }
    // Edge fields FillEdgeTable never wrote: MinNormal without PhongShading
    // (4012-4064), the U/V/(1/z) gradients without Object->Bitmap (4078-4089).
    if ((phong && !fe_phong) || (tex && !fe_bitmap)) return PRK_ERR_UNSUPPORTED;
    if (mode == prk::MODE_SC_GOURAUD) {
        if (fe_phong) flags |= prk::DRAW_RAWCOL;        // raw colours, unlit (4014-4015)
        else if (fe_bitmap) flags |= prk::DRAW_WHITELIT;  // lighting from white (4034-4054)
    }
    if ((phong || !tex) && !g.N) return PRK_ERR_ARG;  // (the Gouraud setup kernels load them in every case)
    if (tex && !g.UV) return PRK_ERR_ARG;
    if ((mode == prk::MODE_SC_GOURAUD || mode == prk::MODE_SC_PHONG) && !g.C) return PRK_ERR_ARG;
    if (tri_count == 0) return PRK_OK;
    if ((uint64_t)c->pending_tris + tri_count >= 0xFFFFFFF0ull) return PRK_ERR_ARG;
    // A draw that continues the previous one (same geometry, the next
    // triangles, same object offset, semantics, texture and object size, the
    // previous one ending on an object boundary) extends it: per-object AETs
    // in submission order are unchanged, and a caller submitting one object
    // per call (the reference's render_entry_3d_object pattern) yields a few
    // draws per frame instead of one per triangle.
    if (!c->draws.empty()) {
        prk::DrawRec &b = c->draws.back();
        const float p0 = P ? P[0] : 0.0f, p1 = P ? P[1] : 0.0f, p2 = P ? P[2] : 0.0f;
        if (b.src_kind == 0 && b.geom == geometry && b.geom_tri0 + b.tri_count == first_tri && b.mode == mode &&
            b.flags == flags && b.tex == texture && b.obj_tris == tris_per_object &&
            b.tri_count % tris_per_object == 0 && b.P[0] == p0 && b.P[1] == p1 && b.P[2] == p2 &&
            std::signbit(b.P[0]) == std::signbit(p0) && std::signbit(b.P[1]) == std::signbit(p1) &&
            std::signbit(b.P[2]) == std::signbit(p2)) {
            b.tri_count += tri_count;
            c->pending_tris += tri_count;
            return PRK_OK;
        }
    }
    prk::DrawRec d{};
    d.V = g.V;
    d.C = g.C;
    d.N = g.N;
    d.UV = g.UV;
    d.geom = geometry;
    d.geom_tri0 = first_tri;
    d.first_global = c->pending_tris;
    d.tri_count = tri_count;
    d.mode = mode;
    d.tex = texture;
    d.P[0] = P ? P[0] : 0.0f;
    d.P[1] = P ? P[1] : 0.0f;
    d.P[2] = P ? P[2] : 0.0f;
    d.flags = flags;
    d.obj_tris = tris_per_object;
    c->draws.push_back(d);
    c->pending_tris += tri_count;
    return PRK_OK;
}

// A draw of caller edges or spans (span path): semantics / texture checks as
// prk_draw; it takes `ids` triangle ids of the frame's numbering.
static int draw_src(prk_context *c, uint32_t kind, uint32_t off, uint32_t n, uint32_t ids, int32_t semantics,
                    int32_t phong, int32_t texture) {
    if (texture >= (int32_t)c->texs.size()) return PRK_ERR_ARG;
    int mode = prk::MODE_AVX;
    if (semantics == PRK_SEM_SCALAR) {
        // DrawModel on a caller's edge list (projekt.cpp:162-601); work
        // records (kind 2) are FillLineOptimized spans only
        if (kind != 1) return PRK_ERR_UNSUPPORTED;
        const bool tex = texture >= 0;
        mode = phong ? (tex ? prk::MODE_SC_PHONG_TEX : prk::MODE_SC_PHONG)
                     : (tex ? prk::MODE_SC_GOURAUD_TEX : prk::MODE_SC_GOURAUD);
    } else if (semantics != PRK_SEM_AVX && semantics != PRK_SEM_AVX_ST) {
        return PRK_ERR_ARG;
    } else if (texture < 0 || !phong) {
        return PRK_ERR_UNSUPPORTED;  // projekt.cpp:1506, 2285-2316
    }
    if ((uint64_t)c->pending_tris + ids >= 0xFFFFFFF0ull) return PRK_ERR_ARG;
    prk::DrawRec d{};
    d.first_global = c->pending_tris;
    d.tri_count = ids;
    d.mode = mode;
    d.tex = texture;
    d.flags = semantics == PRK_SEM_AVX_ST ? prk::DRAW_ST : 0u;
    d.obj_tris = 1;
    d.src_kind = kind;
    d.src_off = off;
    d.src_n = n;
    c->draws.push_back(d);
    c->pending_tris += ids;
    return PRK_OK;
}

int prk_draw_edges(prk_context *c, const prk_edge *edges, uint32_t edge_count, int32_t semantics, int32_t phong,
                   int32_t texture) {
    if (!c || (!edges && edge_count)) return PRK_ERR_ARG;
    if (edge_count == 0) return PRK_OK;  // 0 edges: nothing to draw (P1)
    const uint32_t off = (uint32_t)c->pend_edges.size();
    const int rc = draw_src(c, 1, off, edge_count, 1, semantics, phong, texture);
    if (rc == PRK_OK) c->pend_edges.insert(c->pend_edges.end(), edges, edges + edge_count);
    return rc;
}

int prk_draw_spans(prk_context *c, const prk_span *spans, uint32_t count, int32_t semantics, int32_t phong,
                   int32_t texture) {
    if (!c || (!spans && count)) return PRK_ERR_ARG;
    if (count == 0) return PRK_OK;
    const uint32_t off = (uint32_t)c->pend_spans.size();
    const int rc = draw_src(c, 2, off, count, count, semantics, phong, texture);
    if (rc == PRK_OK) c->pend_spans.insert(c->pend_spans.end(), spans, spans + count);
    return rc;
}

int prk_reset_draws(prk_context *c) {
    if (!c) return PRK_ERR_ARG;
    c->draws.clear();
    c->pending_tris = 0;
    c->pend_edges.clear();
    c->pend_spans.clear();
    return PRK_OK;
}

int prk_set_tile(prk_context *c, int32_t tw, int32_t th) {
    // tile_w: a power of two >= 8 (pixel index <-> (x, y) by shifts)
    if (!c || tw < 8 || th <= 0 || (tw & (tw - 1)) || tw * th > 8192 || tw * th < 64) return PRK_ERR_ARG;
    c->tile_w = tw;
    c->tile_h = th;
    c->tile_auto = false;
    return PRK_OK;
}

int prk_set_early_z(prk_context *c, int on) {
    if (!c) return PRK_ERR_ARG;
    c->early_z = on != 0;
    return PRK_OK;
}

int prk_set_debug(prk_context *c, int32_t enable) {
    if (!c) return PRK_ERR_ARG;
    c->debug = enable != 0;
    return PRK_OK;
}

// Accumulate the kernel times of a timed flush slot (waits for its last event).
static void harvest(prk_context *c, int slot) {
    if (!c->pending[slot]) return;
    c->pending[slot] = false;
    if (hipEventSynchronize(c->ev[slot][2]) != hipSuccess) return;
    float a = 0, b = 0, v = 0, sp = 0;
    if (hipEventElapsedTime(&a, c->ev[slot][0], c->ev[slot][1]) != hipSuccess) a = 0;
    if (hipEventElapsedTime(&b, c->ev[slot][5], c->ev[slot][2]) != hipSuccess) b = 0;
    if (hipEventElapsedTime(&v, c->ev[slot][5], c->ev[slot][3]) != hipSuccess) v = 0;
    if (!c->split_span[slot] || hipEventElapsedTime(&sp, c->ev[slot][3], c->ev[slot][4]) != hipSuccess) sp = 0;
    c->stats.sum_ms_bin += a;
    c->stats.sum_ms_raster += b;
    c->stats.sum_ms_vis += v;
    c->stats.sum_ms_span += sp;
    c->stats.frames_timed += 1;
    if (slot == c->last_slot) {
        c->stats.ms_bin = a;
        c->stats.ms_raster = b;
    }
}

int prk_timing_reset(prk_context *c) {
    if (!c) return PRK_ERR_ARG;
    for (int i = 0; i < prk_context::kRing; ++i) c->pending[i] = false;
    c->stats.frames_timed = 0;
    c->stats.sum_ms_bin = c->stats.sum_ms_raster = c->stats.sum_ms_vis = c->stats.sum_ms_span = 0.0;
    if (c->d_prof.p) PRK_TRY(hipMemset(c->d_prof.p, 0, 16 * sizeof(uint64_t)));
    return PRK_OK;
}

int prk_debug_counters(prk_context *c, uint64_t *out, int32_t n) {
    if (!c || !out || n < 0 || n > 16) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    PRK_TRY(hipSetDevice(c->device));
    PRK_TRY(hipDeviceSynchronize());
    for (int i = 0; i < n; ++i) out[i] = 0;
    if (c->d_prof.p && n) PRK_TRY(hipMemcpy(out, c->d_prof.p, (size_t)n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PRK_OK;
}

// The frame parameters every pass of a flush shares (camera, lights, target, tiling).
static void frame_params(const prk_context *c, prk::FrameParams &fp) {
    fp = prk::FrameParams{};
    fp.D = c->transform.DistanceAboveTarget;
    fp.F = c->transform.FocalLength;
    fp.M2P = c->transform.MetersToPixels;
    fp.Cx = c->transform.ScreenCenter[0];
    fp.Cy = c->transform.ScreenCenter[1];
    fp.InvM2P = 1.0f / fp.M2P;
    {
        int e = 0;
        const float m = std::frexp(fp.F, &e);  // F = m * 2^e, |m| in [0.5, 1)
        fp.f_pow2 = (std::isfinite(fp.F) && (m == 0.5f || m == -0.5f) && e - 1 >= -125 && e - 1 <= 126) ? 1 : 0;
        fp.InvF = fp.f_pow2 ? 1.0f / fp.F : 0.0f;
    }
    fp.light_count = c->lights.LightCount;
    for (int k = 0; k < 4; ++k) fp.amb[k] = c->lights.AmbientIntensity[k];
    for (uint32_t l = 0; l < PRK_MAX_LIGHTS; ++l) {
        for (int k = 0; k < 3; ++k) fp.lp[l][k] = c->lights.Lights[l].P[k];
        for (int k = 0; k < 4; ++k) fp.li[l][k] = c->lights.Lights[l].Intensity[k];
    }
    // the span shading's camera and lights (prk_set_shade_camera)
    {
        const prk_transform &t = c->shade_transform;
        const prk_light_data &L = c->shade_lights;
        prk::ShadeCam &sh = fp.sh;
        sh.D = t.DistanceAboveTarget;
        sh.F = t.FocalLength;
        sh.Cx = t.ScreenCenter[0];
        sh.Cy = t.ScreenCenter[1];
        sh.InvM2P = 1.0f / t.MetersToPixels;
        int e = 0;
        const float m = std::frexp(sh.F, &e);  // F = m * 2^e, |m| in [0.5, 1)
        sh.f_pow2 = (std::isfinite(sh.F) && (m == 0.5f || m == -0.5f) && e - 1 >= -125 && e - 1 <= 126) ? 1 : 0;
        sh.InvF = sh.f_pow2 ? 1.0f / sh.F : 0.0f;
        sh.light_count = L.LightCount;
        for (int k = 0; k < 4; ++k) sh.amb[k] = L.AmbientIntensity[k];
        for (uint32_t l = 0; l < PRK_MAX_LIGHTS; ++l) {
            for (int k = 0; k < 3; ++k) sh.lp[l][k] = L.Lights[l].P[k];
            for (int k = 0; k < 4; ++k) sh.li[l][k] = L.Lights[l].Intensity[k];
        }
    }
    fp.W = c->W;
    fp.H = c->H;
    fp.row0 = c->row0;
    fp.row1 = c->row1;
    fp.pitch = c->pitch;
    fp.color = (uint32_t *)c->color;
    fp.zbuf = c->zbuf;
    // The context's tile, made taller (then wider) while the frame would have
    // more tiles than the counting-sort binning holds (kCsMaxTiles): results
    // never depend on the tile, and every tile keeps <= 8192 pixels.
    int32_t tw = c->tile_w, th = c->tile_h;
    auto ntl = [&](int32_t w, int32_t h) {
        return (uint64_t)((c->W + w - 1) / w) * (uint64_t)((c->row1 - c->row0 + h - 1) / h);
    };
    while (ntl(tw, th) > prk_cs_max_tiles() && tw * th * 2 <= 8192) {
        if (th < tw / 8) th *= 2;
        else tw *= 2;
    }
    fp.tile_w = tw;
    fp.tile_h = th;
    fp.tile_w_log2 = 0;
    while ((1 << fp.tile_w_log2) < tw) ++fp.tile_w_log2;
    fp.tiles_x = (c->W + tw - 1) / tw;
    fp.tiles_y = (c->row1 - c->row0 + th - 1) / th;
    fp.prof = (unsigned long long *)c->d_prof.p;
    fp.negz = (uint32_t *)c->d_negz.p;
    fp.z_in_vis = c->early_z && c->d_negz.p ? 1 : 0;
    fp.winners = c->debug ? (int32_t *)c->d_winners.p : nullptr;
    fp.clear_color = c->clear_color;
    fp.clear_z = c->clear_z;
}

// A pending clear that the pass cannot fuse into its kernels: fill first.
static int fill_pending_clear(prk_context *c, hipStream_t s) {
    c->z_early = false;
    if (!c->clear_pending) return PRK_OK;
    c->clear_pending = false;
    const size_t n = (size_t)c->W * (c->row1 - c->row0);
    if (n) {
        hipLaunchKernelGGL(k_fill_target, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (uint32_t *)c->color,
                           c->pitch, c->zbuf, c->W, c->row1 - c->row0, c->clear_color, c->clear_z);
        PRK_TRY(hipGetLastError());
    }
    return PRK_OK;
}

// One pass of per-triangle AETs (draws of one triangle per object): bin +
// raster into the target.  `draws` number their triangles from 0; winner ids
// are win_base + that index.
static int flush_tris(prk_context *c, hipStream_t s, const std::vector<prk::DrawRec> &draws, uint32_t T,
                      uint32_t win_base, bool defer = false) {
    int modeset = -2;
    for (const auto &d : draws) {
        if (modeset == -2) modeset = d.mode;
        else if (modeset != d.mode) modeset = -1;
    }
    if (modeset != prk::MODE_AVX && modeset != prk::MODE_SC_GOURAUD && modeset != prk::MODE_SC_PHONG)
        modeset = -1;
    prk::FrameParams fp;
    frame_params(c, fp);
    fp.tri_count = T;
    fp.ndraws = (uint32_t)draws.size();
    fp.win_base = win_base;
    const uint32_t ntiles = (uint32_t)(fp.tiles_x * fp.tiles_y);

    c->stats.triangles = T;
    c->stats.tiles = ntiles;
    c->stats.bin_entries = 0;
    const int slot = (int)(c->frame % prk_context::kRing);
    harvest(c, slot);  // a flush kRing frames old: long finished
    // A pending fused clear: the span-record kernels (AVX frames) fold it in;
    // every other frame fills the target first, on this stream.
    const bool fuse = c->clear_pending && T > 0 && modeset == prk::MODE_AVX && PRK_SPAN_RECORDS_HOST;
    if (!fuse) {
        const int rc = fill_pending_clear(c, s);
        if (rc != PRK_OK) return rc;
    }
    c->clear_pending = false;
    fp.clear_fused = fuse ? 1 : 0;
    if (T == 0) return PRK_OK;
    // Binning runs on bin_stream into one of the scratch sets, so it overlaps
    // the previous frame's raster on the flush stream; the raster waits for
    // it.  Consecutive frames take consecutive sets (nsets of them), and a
    // set's reuse waits for its own last reader.
    const int nsets = (size_t)c->W * (size_t)(c->row1 - c->row0) <= kSmallBandPx ? prk_context::kSets
                                                                                : std::min(prk_context::kSets, 2);
    const int si = (c->last_set + 1) % nsets;
    c->last_set = si;
    prk_context::BinSet &B = c->bset[si];
    // Any error below leaves the set's table mirrors unknown: forget them.
    struct MirrorGuard {
        prk_context::BinSet &b;
        bool ok = false;
        ~MirrorGuard() {
            if (!ok) b.h_draws_at = b.h_texs_at = nullptr;
        }
    } guard{B};
    hipStream_t bs = c->bin_stream;
    if (B.used) PRK_TRY(hipStreamWaitEvent(bs, B.free_ev, 0));  // the raster of frame k-nsets read this set
    // A set buffer that must grow is freed by the host: wait for its reader.
    auto bset_ensure = [&](DevBuf &d, size_t n) -> hipError_t {
        if (d.cap < n && B.used) {
            hipError_t e = hipEventSynchronize(B.free_ev);
            if (e != hipSuccess) return e;
        }
        return d.ensure(n);
    };
    // Device-side draw + texture tables.
    std::vector<prk::TexRec> texs(c->texs.size());
    for (size_t i = 0; i < texs.size(); ++i) {
        texs[i].mem = c->texs[i].mem;
        texs[i].w = c->texs[i].w;
        texs[i].h = c->texs[i].h;
        texs[i].pitch = c->texs[i].pitch;
        texs[i].filter = c->texs[i].filter;
    }
    // Upload a table into this set unless the set already holds the same
    // bytes (the set's previous reader, frame k-nsets's raster, is waited for above).
    auto upload_table = [&](DevBuf &d, std::vector<uint8_t> &mirror, const void *&at, const void *src,
                            size_t bytes) -> hipError_t {
        hipError_t e = bset_ensure(d, bytes);
        if (e != hipSuccess) return e;
        if (at == d.p && mirror.size() == bytes && std::memcmp(mirror.data(), src, bytes) == 0) return hipSuccess;
        at = nullptr;  // unknown until the copy is queued
        mirror.assign((const uint8_t *)src, (const uint8_t *)src + bytes);
        // from the mirror: it outlives this call (the set's next use waits for
        // this frame's raster, which follows the copy on the bin stream)
        e = hipMemcpyAsync(d.p, mirror.data(), bytes, hipMemcpyHostToDevice, bs);
        if (e == hipSuccess) at = d.p;
        return e;
    };
    PRK_TRY(upload_table(B.d_draws, B.h_draws, B.h_draws_at, draws.data(), draws.size() * sizeof(prk::DrawRec)));
    if (!texs.empty())
        PRK_TRY(upload_table(B.d_texs, B.h_texs, B.h_texs_at, texs.data(), texs.size() * sizeof(prk::TexRec)));
    fp.draws = (const prk::DrawRec *)B.d_draws.p;
    fp.texs = (const prk::TexRec *)B.d_texs.p;
    fp.draw0 = draws[0];
    fp.tex0 = prk::TexRec{};
    if (fp.draw0.tex >= 0 && (size_t)fp.draw0.tex < texs.size()) fp.tex0 = texs[fp.draw0.tex];
    fp.tri_draw = nullptr;
    if (fp.ndraws > 1) {
        PRK_TRY(bset_ensure(B.d_tri_draw, (size_t)T * 4));
        PRK_TRY(prk_launch_tri_draw(fp.draws, fp.ndraws, (uint32_t *)B.d_tri_draw.p, T, bs));
        fp.tri_draw = (const uint32_t *)B.d_tri_draw.p;
    }
    PRK_TRY(bset_ensure(B.d_ranges, (size_t)T * 16));
    PRK_TRY(bset_ensure(B.d_tri_n, (size_t)(T + 1) * 4));
    PRK_TRY(bset_ensure(B.d_tri_off, (size_t)(T + 1) * 4));
    PRK_TRY(bset_ensure(B.d_offs, (size_t)(ntiles + 1) * 4));
    fp.trec = nullptr;
    if (modeset == prk::MODE_AVX && c->setup_rec) {
        PRK_TRY(bset_ensure(B.d_trec, (size_t)T * sizeof(prk::TriRec)));
        fp.trec = (prk::TriRec *)B.d_trec.p;
    }
    const bool span_rec = modeset == prk::MODE_AVX;
    // won flags: per (pair, row in tile) for span-record (AVX) frames, per
    // pair otherwise; the binning clears them (and trwon) for every pair.
    const uint32_t won_stride = span_rec ? (uint32_t)fp.tile_h : 1u;
    size_t sel_bytes = 0;
    if (span_rec) PRK_TRY(prk_walk_select_bytes(T, &sel_bytes));
    // Every per-pair array of the set, for `np` pairs.
    auto ensure_pairs = [&](size_t np) -> hipError_t {
        const size_t ne = std::max<size_t>(np, 1);
        hipError_t e = hipSuccess;
        if (e == hipSuccess) e = bset_ensure(B.d_pair_tri, ne * 4);
        if (e == hipSuccess) e = bset_ensure(B.d_bins, ne * 8);  // (triangle, pair) per bin slot
        if (e == hipSuccess) e = bset_ensure(B.d_list, ne * 4);
        if (e == hipSuccess) e = bset_ensure(B.d_won, ne * won_stride);
        // span records: 64 B per (pair, row in tile); only won ones are written
        if (e == hipSuccess && span_rec) e = bset_ensure(B.d_recs, ne * won_stride * 64);
        return e;
    };
    PRK_TRY(bset_ensure(B.d_nwin, (size_t)ntiles * 4));
    PRK_TRY(bset_ensure(B.d_wtag, (size_t)ntiles * fp.tile_w * fp.tile_h * 4));
    if (span_rec) {
        PRK_TRY(bset_ensure(B.d_trwon, T));
        PRK_TRY(bset_ensure(B.d_wlist, ((size_t)T + 1) * 4));  // won triangles + their count
        PRK_TRY(bset_ensure(B.d_seltemp, std::max<size_t>(sel_bytes, 16)));
    }
    uint8_t *won, *trwon;
    // (frame_params keeps every frame within the counting sort's tile count)
    if (ntiles > prk_cs_max_tiles()) return PRK_ERR_LIMIT;
    if (!prk_cs_ready(ntiles)) return PRK_ERR_DEVICE;
    {
        // Counting-sort binning (prk_bin.hip k_cs_*): all sizes stay on the
        // device.  The per-pair arrays hold `cap` pairs (the last frame's
        // count plus room; a first frame guesses 2.5 per triangle, C3b has
        // 3.2); a frame with more entries leaves its bins empty and is re-run
        // below, once the count is known.
        // a row band's sort walks only its triangles (listed per run by k_bin_band)
        const uint32_t per = prk_cs_band_runs_per_chunk(&fp);
        if (per) {
            PRK_TRY(bset_ensure(B.d_runlist, (size_t)prk_bin_runs(T) * prk_bin_run_len() * 4));
            PRK_TRY(bset_ensure(B.d_run_n, (size_t)prk_bin_runs(T) * 4));
        }
        const uint32_t nch = prk_cs_nchunks(T, per);
        const uint64_t want64 = c->pair_hint ? (uint64_t)c->pair_hint + c->pair_hint / 8 + 4096
                                             : std::max<uint64_t>(5ull * T / 2, 1u << 16);
        const uint32_t want = (uint32_t)std::min<uint64_t>(want64, prk_cs_max_pairs());
        // pairs the set's per-pair arrays hold now (they never shrink)
        auto pairs_held = [&]() -> size_t {
            size_t m = std::min(B.d_pair_tri.cap / 4, B.d_bins.cap / 8);
            m = std::min(m, B.d_list.cap / 4);
            m = std::min(m, B.d_won.cap / won_stride);
            if (span_rec) m = std::min(m, B.d_recs.cap / ((size_t)won_stride * 64));
            return m;
        };
        if (pairs_held() > 4ull * want && pairs_held() > (1u << 20)) {
            // far more room than the frames need (a big frame earlier): give
            // it back once the set's last reader is done
            if (B.used) PRK_TRY(hipEventSynchronize(B.free_ev));
            DevBuf *pb[] = {&B.d_pair_tri, &B.d_bins, &B.d_list, &B.d_won, &B.d_recs};
            for (DevBuf *b : pb) b->release();
        }
        if (pairs_held() < want) PRK_TRY(ensure_pairs(want));
        const uint32_t cap = (uint32_t)std::min<size_t>(pairs_held(), prk_cs_max_pairs());
        PRK_TRY(bset_ensure(B.d_ghist, std::max<size_t>((size_t)nch * ntiles * 4, 4)));
        PRK_TRY(bset_ensure(B.d_tile_tot, (size_t)ntiles * 4));
        PRK_TRY(bset_ensure(B.d_chunk, std::max<size_t>((size_t)nch * 8, 8)));
        PRK_TRY(bset_ensure(B.d_info, 8));
        won = (uint8_t *)B.d_won.p;
        trwon = span_rec ? (uint8_t *)B.d_trwon.p : nullptr;
        PRK_TRY(hipEventRecord(c->ev[slot][0], bs));
        uint32_t *runlist = per ? (uint32_t *)B.d_runlist.p : nullptr, *run_n = per ? (uint32_t *)B.d_run_n.p : nullptr;
        PRK_TRY(prk_bin_count(&fp, (uint32_t *)B.d_tri_n.p, B.d_ranges.p, runlist, run_n, trwon, bs));
        // a row band's setup records (k_band_rec) run on the vis stream beside
        // the counting sort, once k_bin_band has listed the runs; queued after
        // the sort's launches, so a host that is only just ahead of the GPU
        // (a frame after a wait) does not hold the sort back
        const bool band_rec = runlist && fp.trec;
        if (band_rec) PRK_TRY(hipEventRecord(B.listed_ev, bs));
        if (band_rec && !PRK_REC_AFTER_CS) {
            PRK_TRY(hipStreamWaitEvent(c->vis_stream, B.listed_ev, 0));
            PRK_TRY(prk_band_records(&fp, runlist, run_n, c->vis_stream));
        }
        uint32_t *chunk = (uint32_t *)B.d_chunk.p;
        PRK_TRY(prk_bin_cs(&fp, B.d_ranges.p, (const uint32_t *)B.d_tri_n.p, (uint32_t *)B.d_ghist.p,
                           (uint32_t *)B.d_tile_tot.p, chunk, chunk + nch, (uint32_t *)B.d_offs.p, cap,
                           (uint32_t *)B.d_info.p, (uint32_t *)B.d_tri_off.p, B.d_bins.p, (uint32_t *)B.d_pair_tri.p,
                           won, won_stride, trwon, runlist, run_n, per, bs));
        // the bins are ready: the raster may start (after the entry count's
        // copy to the host, PRK_BINNED_EARLY)
        if (PRK_BINNED_EARLY) {
            PRK_TRY(hipEventRecord(c->ev[slot][1], bs));
            PRK_TRY(hipEventRecord(B.binned_ev, bs));
        }
        PRK_TRY(hipMemcpyAsync(B.h_info, B.d_info.p, 8, hipMemcpyDeviceToHost, bs));
        PRK_TRY(hipEventRecord(B.counted_ev, bs));
        if (!PRK_BINNED_EARLY) {
            PRK_TRY(hipEventRecord(c->ev[slot][1], bs));
            PRK_TRY(hipEventRecord(B.binned_ev, bs));
        }
        if (band_rec && PRK_REC_AFTER_CS) {  // (this frame's k_vis follows the records on the vis stream)
            PRK_TRY(hipStreamWaitEvent(c->vis_stream, B.listed_ev, 0));
            PRK_TRY(prk_band_records(&fp, runlist, run_n, c->vis_stream));
        }
    }

    // Raster.  Span-record frames run k_vis on vis_stream once their binning
    // is done (so it overlaps the previous frame's k_walk / k_pix on the
    // flush stream, while the next frame bins on bin_stream) and shade on the
    // flush stream after it; k_vis waits for the flush stream only when it
    // reads the target's prior z (no fused clear), writes the debug winner
    // map, or writes z itself (early z: the flush stream may still hold an
    // earlier frame's z writers -- k_shade, k_pix, k_span_shade, a -0.0
    // fix-up -- that must land before this frame's z).
    // Other frames run on the flush stream.
    if (!c->d_anomaly.p) {
        PRK_TRY(c->d_anomaly.ensure(8));  // [anomalies, slow replays]
        PRK_TRY(hipMemsetAsync(c->d_anomaly.p, 0, 8, s));
        PRK_TRY(hipStreamSynchronize(s));
    }
    hipStream_t sv = s;
    if (span_rec) {
        sv = c->vis_stream;
        PRK_TRY(hipStreamWaitEvent(sv, B.binned_ev, 0));
        if (!fuse || c->debug || fp.z_in_vis) {  // prior z / winner map / early z: after the flush stream's work so far
            PRK_TRY(hipEventRecord(c->s_mark, s));
            PRK_TRY(hipStreamWaitEvent(sv, c->s_mark, 0));
        }
    } else {
        PRK_TRY(hipStreamWaitEvent(s, B.binned_ev, 0));
    }
    PRK_TRY(hipEventRecord(c->ev[slot][5], sv));
    PRK_TRY(prk_launch_raster(&fp, modeset, (const uint32_t *)B.d_offs.p, B.d_bins.p,
                              (const uint32_t *)B.d_pair_tri.p, (const uint32_t *)B.d_tri_off.p, B.d_ranges.p,
                              (uint8_t *)B.d_won.p, (uint8_t *)B.d_trwon.p, (uint32_t *)B.d_wlist.p,
                              B.d_seltemp.p, sel_bytes, (uint32_t *)B.d_list.p,
                              (uint32_t *)B.d_nwin.p, (uint32_t *)B.d_wtag.p, B.d_recs.p,
                              (uint32_t *)c->d_anomaly.p, c->ev[slot][3], span_rec ? c->ev[slot][4] : nullptr, sv,
                              s));
    PRK_TRY(hipEventRecord(c->ev[slot][2], s));
    PRK_TRY(hipEventRecord(B.free_ev, s));
    // a span-record pass's z is final after k_vis (ev[slot][3], on the vis stream)
    c->z_early = span_rec && sv != s && fp.z_in_vis;
    c->z_slot = slot;
    B.used = true;
    c->pending[slot] = true;
    c->split_span[slot] = modeset == prk::MODE_AVX;
    c->last_slot = slot;
    c->frame++;
    guard.ok = true;
    {
        // The whole frame is queued; now the entry count (the binning's first
        // few kernels) decides whether it fitted — read here, or, for the
        // frame's last pass once a previous frame has sized the scratch, by
        // the next call that needs it (resolve_count).
        prk_context::PendingCount &P = c->pcount;
        P.set = si;
        P.s = s;
        P.draws = draws;
        P.T = T;
        P.win_base = win_base;
        P.ntiles = ntiles;
        P.fuse = fuse;
        P.debug = c->debug;
        P.color = c->color; P.pitch = c->pitch; P.zbuf = c->zbuf;
        P.W = c->W; P.H = c->H; P.row0 = c->row0; P.row1 = c->row1;
        P.tile_w = c->tile_w; P.tile_h = c->tile_h;
        P.transform = c->transform; P.lights = c->lights;
        P.shade_transform = c->shade_transform; P.shade_lights = c->shade_lights;
        P.clear_color = c->clear_color; P.clear_z = c->clear_z;
        P.active = true;
        if (!(defer && c->pair_hint)) return resolve_count(c);
    }
    return PRK_OK;
}

// The entry count of the pending pass (PendingCount): stats, the next
// frame's capacity and tile; an over-capacity pass drew nothing (empty bins;
// with a fused clear its k_pix wrote the clear values, which the re-run
// writes again) and is re-run with room for every entry, with the state it
// was queued with.
static int resolve_count(prk_context *c) {
    prk_context::PendingCount &P = c->pcount;
    if (!P.active) return PRK_OK;
    P.active = false;
    PRK_TRY(hipSetDevice(c->device));
    prk_context::BinSet &B = c->bset[P.set];
    PRK_TRY(hipEventSynchronize(B.counted_ev));
    const uint32_t total = B.h_info[0];
    c->stats.bin_entries = total;
    c->pair_hint = total;
    if (c->tile_auto && !c->auto_small && P.tile_w == 256 && total < 64u * P.ntiles &&
        8u * P.ntiles <= prk_cs_max_tiles()) {  // (32x8 tiles stay within the counting sort)
        c->auto_small = total < 8u * P.ntiles ? 64 : 32;  // (from the next frame on)
        c->auto_T = P.T;
        c->auto_px = P.W * (P.row1 - P.row0);
    }
    // (a row band's entries against its share of the triangles, T * rows / H)
    if (c->tile_auto && !c->auto_small && !c->auto_wide && P.tile_w == 256 && P.tile_h == 8 && P.T && P.H > 0 &&
        2ull * total * (uint64_t)P.H >= 9ull * P.T * (uint64_t)std::max(1, P.row1 - P.row0) &&
        std::all_of(P.draws.begin(), P.draws.end(), [](const prk::DrawRec &d) { return d.mode == prk::MODE_AVX; })) {
        c->auto_wide = 512;  // (from the next frame on)
        c->auto_T = P.T;
        c->auto_px = P.W * (P.row1 - P.row0);
    }
    if (!B.h_info[1]) return PRK_OK;
    if (total > prk_cs_max_pairs()) return PRK_ERR_LIMIT;  // 29-bit pair index in the bins
    // re-run with the pass's own state, then give the caller's back
    struct Saved {
        void *color; int32_t pitch; float *zbuf; int32_t W, H, row0, row1, tile_w, tile_h;
        prk_transform transform, shade_transform; prk_light_data lights, shade_lights;
        uint32_t clear_color; float clear_z; bool clear_pending, debug;
    } sv{c->color, c->pitch, c->zbuf, c->W, c->H, c->row0, c->row1, c->tile_w, c->tile_h,
         c->transform, c->shade_transform, c->lights, c->shade_lights, c->clear_color, c->clear_z,
         c->clear_pending, c->debug};
    c->color = P.color; c->pitch = P.pitch; c->zbuf = P.zbuf;
    c->W = P.W; c->H = P.H; c->row0 = P.row0; c->row1 = P.row1;
    c->tile_w = P.tile_w; c->tile_h = P.tile_h;
    c->transform = P.transform; c->lights = P.lights;
    c->shade_transform = P.shade_transform; c->shade_lights = P.shade_lights;
    c->clear_color = P.clear_color; c->clear_z = P.clear_z;
    c->clear_pending = P.fuse;
    c->debug = P.debug;
    const std::vector<prk::DrawRec> draws = std::move(P.draws);
    const int rc = flush_tris(c, P.s, draws, P.T, P.win_base);
    c->read_rec = hipEventRecord(c->read_ev, P.s) == hipSuccess;  // (geometry writes wait for the re-run)
    c->z_early = false;  // (a re-run: the download takes z after everything)
    c->color = sv.color; c->pitch = sv.pitch; c->zbuf = sv.zbuf;
    c->W = sv.W; c->H = sv.H; c->row0 = sv.row0; c->row1 = sv.row1;
    c->tile_w = sv.tile_w; c->tile_h = sv.tile_h;
    c->transform = sv.transform; c->lights = sv.lights;
    c->shade_transform = sv.shade_transform; c->shade_lights = sv.shade_lights;
    c->clear_color = sv.clear_color; c->clear_z = sv.clear_z;
    c->clear_pending = sv.clear_pending;
    c->debug = sv.debug;
    return rc;
}

// One pass of whole-object AETs (prk_spans.hip): FillEdgeTable per triangle,
// MergeSort per object (one radix sort), one walk of every object's AET into
// span records (each object writing into its own slots, as many as its edges'
// active rows allow), bin the spans to tiles, then visibility + shading.
// Stream-ordered on s; the host waits at the two sizes it reads back (the
// span slots, the bin entry count).
static int flush_spans(prk_context *c, hipStream_t s, const std::vector<prk::DrawRec> &draws, uint32_t T,
                       uint32_t win_base) {
    c->z_early = false;  // (k_pix / k_span_shade write a span pass's z)
    prk::FrameParams fp;
    frame_params(c, fp);
    fp.tri_count = T;
    fp.ndraws = (uint32_t)draws.size();
    fp.win_base = win_base;
    const uint32_t ntiles = (uint32_t)(fp.tiles_x * fp.tiles_y);
    const bool fuse = c->clear_pending && T > 0;
    c->clear_pending = false;
    fp.clear_fused = fuse ? 1 : 0;
    if (T == 0) return PRK_OK;
    prk_context::SpanScratch &S = c->spans;
    if (!S.h_rb) PRK_TRY(hipHostMalloc((void **)&S.h_rb, 8 * sizeof(uint32_t), hipHostMallocDefault));
    const uint32_t lcap = prk_obj_walk_lcap();  // LDS list capacity of the wave walk (edges)
    // Objects in submission order (ObjDesc kinds: prk_spans.hip): kind 0
    // objects' triangles numbered 0..ntri-1 in order (FillEdgeTable runs per
    // triangle), caller edge lists' edges after the triangles' edges.  Objects
    // of kObjWaveTris triangles or more are walked by one wave each, their
    // list in LDS when their most active edges fit the launch's LDS capacity
    // (min(lcap, the largest such object's edges)), else in their pool slice.
    // (the objects themselves are expanded on the device from runs: a draw
    // of kind 0 is a run of ceil(tris / obj_tris) objects, kind 2 one of its
    // spans; only the large objects are listed here)
    S.h_runs.clear();
    S.h_big_gl.clear();
    S.h_big_off.clear();
    S.h_big_cap.clear();
    S.h_k1src.clear();
    uint64_t ntri = 0, nk1 = 0, pool = 0, maxn = 1, small_tris = 0, nobj64 = 0, nk064 = 0;
    bool thread_links = false;  // a thread-walked triangle object small enough for LDS list links
    std::vector<uint32_t> bigm[prk::MODE_COUNT], bige[prk::MODE_COUNT];  // wave-walked objects by mode, their edges
    for (uint32_t di = 0; di < draws.size(); ++di) {
        const prk::DrawRec &d = draws[di];
        if (d.src_kind == 1) {
            S.h_runs.push_back(ObjRun{1u, di, (uint32_t)nobj64, 1u, 0u, 0u, d.first_global, 0u, 0u, d.src_off, d.src_n,
                                      (uint32_t)nk1});
            for (uint32_t e = 0; e < d.src_n; ++e) S.h_k1src.push_back(d.src_off + e);
            nk1 += d.src_n;
            nobj64 += 1;
        } else if (d.src_kind == 2) {
            if (!d.src_n) continue;
            S.h_runs.push_back(ObjRun{2u, di, (uint32_t)nobj64, d.src_n, 0u, 0u, d.first_global, 0u, 0u, d.src_off, 0u, 0u});
            nobj64 += d.src_n;
        } else {
            const uint32_t per = std::max<uint32_t>(1u, d.obj_tris);
            const uint32_t cnt = (uint32_t)(((uint64_t)d.tri_count + per - 1) / per);
            if (!cnt) continue;
            S.h_runs.push_back(ObjRun{0u, di, (uint32_t)nobj64, cnt, per, d.tri_count, d.first_global, (uint32_t)ntri,
                                      (uint32_t)nk064, 0u, 0u, 0u});
            maxn = std::max<uint64_t>(maxn, 3ull * std::min(per, d.tri_count));  // the most its FillEdgeTable writes
            if (per >= kObjWaveTris) {
                for (uint32_t j = 0; j < cnt; ++j) {
                    const uint32_t n = std::min(per, d.tri_count - j * per);
                    if (n >= kObjWaveTris) {
                        bigm[d.mode].push_back((uint32_t)(nobj64 + j));
                        bige[d.mode].push_back(3u * n);
                    } else {
                        small_tris += n;
                        thread_links = thread_links || 3ull * n <= prk_obj_link_cap();
                    }
                }
            } else {
                const uint32_t rem = d.tri_count % per;
                small_tris += d.tri_count;
                thread_links = thread_links || (d.tri_count >= per && 3ull * per <= prk_obj_link_cap()) ||
                               (rem && 3ull * rem <= prk_obj_link_cap());
            }
            nobj64 += cnt;
            nk064 += cnt;
            ntri += d.tri_count;
        }
        if (nobj64 >= 0x7FFFFFFFull) return PRK_ERR_LIMIT;
    }
    std::vector<uint32_t> big_edges;  // (h_big_gl order)
    for (int mo = 0; mo < prk::MODE_COUNT; ++mo)  // the large objects, by mode (their walk groups: after the readback)
        for (size_t i = 0; i < bigm[mo].size(); ++i) {
            S.h_big_gl.push_back(bigm[mo][i]);
            big_edges.push_back(bige[mo][i]);
        }
    // edge slots (3 per triangle + the caller edges) are indexed by 31 bits
    if (3 * ntri + nk1 >= 0x7FFFFFFFull) return PRK_ERR_LIMIT;
    const uint32_t nobj = (uint32_t)nobj64, nk0 = (uint32_t)nk064;
    const uint32_t nt = (uint32_t)ntri, nbig_all = (uint32_t)S.h_big_gl.size();
    // MergeSort key: (object, min(YMin, H), recursion path) in one radix sort
    auto bitlen = [](uint64_t v) { uint32_t b = 0; while (v) { ++b; v >>= 1; } return b; };
    const uint32_t pbits = bitlen(maxn) + 1, ybits = std::max(1u, bitlen((uint64_t)c->H));
    const uint32_t obits = std::max(1u, bitlen(nk0 > 0 ? nk0 - 1 : 0));
    if (obits + ybits + pbits > 64) return PRK_ERR_LIMIT;
    S.h_texs.resize(c->texs.size());
    for (size_t i = 0; i < S.h_texs.size(); ++i)
        S.h_texs[i] = prk::TexRec{c->texs[i].mem, c->texs[i].w, c->texs[i].h, c->texs[i].pitch, c->texs[i].filter};
    S.h_draws = draws;
    // (the scratch below is reused frame to frame: stream order on s covers it)
    // The pass's host tables go up in one copy from pinned staging (a pageable
    // hipMemcpyAsync per table held the host for each).
    enum { T_DRAWS, T_TEXS, T_OBJS, T_K0OBJ, T_K0TRI0, T_BIG, T_BIG_OFF, T_BIG_CAP, T_K1SRC, T_EDGES, T_SPANS, T_N };  // (T_OBJS: the runs)
    struct Part {
        const void *src;
        size_t bytes, off;
    } parts[T_N] = {{S.h_draws.data(), S.h_draws.size() * sizeof(prk::DrawRec), 0},
                    {S.h_texs.data(), S.h_texs.size() * sizeof(prk::TexRec), 0},
                    {S.h_runs.data(), S.h_runs.size() * sizeof(ObjRun), 0},
                    {nullptr, 0, 0},
                    {nullptr, 0, 0},
                    {S.h_big_gl.data(), S.h_big_gl.size() * 4, 0},
                    {nullptr, 0, 0},
                    {nullptr, 0, 0},
                    {S.h_k1src.data(), S.h_k1src.size() * 4, 0},
                    {c->pend_edges.data(), c->pend_edges.size() * sizeof(prk_edge), 0},
                    {c->pend_spans.data(), c->pend_spans.size() * sizeof(prk_span), 0}};
    size_t stage_bytes = 0;
    for (Part &pt : parts) {
        pt.off = stage_bytes;
        stage_bytes = (stage_bytes + pt.bytes + 255) & ~(size_t)255;
    }
    stage_bytes = std::max<size_t>(stage_bytes, 256);
    if (!S.stage_ev) PRK_TRY(hipEventCreateWithFlags(&S.stage_ev, hipEventDisableTiming));
    if (S.stage_busy) {  // the previous pass's upload still reads the staging
        PRK_TRY(hipEventSynchronize(S.stage_ev));
        S.stage_busy = false;
    }
    if (stage_bytes > S.stage_cap) {
        if (S.h_stage) (void)hipHostFree(S.h_stage);
        S.h_stage = nullptr;
        S.stage_cap = 0;
        const size_t want = stage_bytes + stage_bytes / 4;
        PRK_TRY(hipHostMalloc((void **)&S.h_stage, want, hipHostMallocDefault));
        S.stage_cap = want;
    }
    for (const Part &pt : parts)
        if (pt.bytes && pt.src) std::memcpy(S.h_stage + pt.off, pt.src, pt.bytes);
    PRK_TRY(S.d_stage.ensure(stage_bytes));
    PRK_TRY(hipMemcpyAsync(S.d_stage.p, S.h_stage, stage_bytes, hipMemcpyHostToDevice, s));
    PRK_TRY(hipEventRecord(S.stage_ev, s));
    S.stage_busy = true;
    auto dev = [&](int t) -> void * { return static_cast<char *>(S.d_stage.p) + parts[t].off; };
    fp.draws = (const prk::DrawRec *)dev(T_DRAWS);
    fp.texs = (const prk::TexRec *)dev(T_TEXS);
    fp.draw0 = draws[0];
    fp.tex0 = prk::TexRec{};
    if (fp.draw0.tex >= 0 && (size_t)fp.draw0.tex < S.h_texs.size()) fp.tex0 = S.h_texs[fp.draw0.tex];
    void *d_edges_in = dev(T_EDGES), *d_spans_in = dev(T_SPANS);
    // the objects (ObjDesc), the kind-0 objects' indices and first triangles
    PRK_TRY(S.d_objtab.ensure((size_t)std::max<uint32_t>(nobj, 1) * sizeof(ObjDesc)));
    PRK_TRY(S.d_k0tab.ensure((size_t)std::max<uint32_t>(nk0, 1) * 8));
    void *d_objs = S.d_objtab.p;
    uint32_t *k0tab = (uint32_t *)S.d_k0tab.p;
    const uint32_t *d_k0obj = k0tab, *d_k0tri0 = k0tab + nk0;
    PRK_TRY(prk_obj_tables(dev(T_OBJS), (uint32_t)S.h_runs.size(), nobj, kObjWaveTris, d_objs, k0tab, k0tab + nk0, s));
    const uint32_t *d_big = (const uint32_t *)dev(T_BIG);
    const uint32_t *d_k1src = (const uint32_t *)dev(T_K1SRC);
    uint32_t modes = 0;  // the pass's span kinds: bit per Mode
    for (const auto &d : draws) modes |= 1u << d.mode;
    const bool scalar = (modes & ~(1u << prk::MODE_AVX)) != 0;
    // FillEdgeTable per triangle: counts, scans, edges + MergeSort keys.
    const size_t es = std::max<size_t>(3 * (size_t)nt, 1);
    PRK_TRY(S.d_ecnt.ensure(((size_t)nt + 1) * 4));
    PRK_TRY(S.d_escan.ensure(((size_t)nt + 1) * 4));
    PRK_TRY(S.d_rcnt.ensure(((size_t)nt + 1) * 8));
    PRK_TRY(S.d_rscan.ensure(((size_t)nt + 1) * 8));
    PRK_TRY(S.d_edges.ensure(es * 112));  // prk_spans.hip ObjEdge
    PRK_TRY(S.d_ekeys.ensure(es * 8));
    PRK_TRY(S.d_ekeys2.ensure(es * 8));
    PRK_TRY(S.d_evals.ensure(es * 4));
    PRK_TRY(S.d_ord.ensure(es * 4));
    PRK_TRY(S.d_err.ensure(16));
    PRK_TRY(hipMemsetAsync(S.d_err.p, 0, 16, s));  // (error bits, then the chunked walk's tally)
    uint32_t *escan = (uint32_t *)S.d_escan.p, *ord = (uint32_t *)S.d_ord.p;
    unsigned long long *rscan = (unsigned long long *)S.d_rscan.p;
    const uint32_t *total0p = escan + nt;
    size_t tb = 0;
    auto temp = [&](size_t b) -> hipError_t { return S.d_temp.ensure(std::max<size_t>(b, 16)); };
    if (nt) {
        PRK_TRY(prk_objtri_count(&fp, d_objs, d_k0obj, d_k0tri0, nk0,
                                 nt, (uint32_t *)S.d_ecnt.p, (unsigned long long *)S.d_rcnt.p, s));
    } else {
        PRK_TRY(hipMemsetAsync(S.d_ecnt.p, 0, 4, s));
        PRK_TRY(hipMemsetAsync(S.d_rcnt.p, 0, 8, s));
    }
    PRK_TRY(prk_scan_u32((const uint32_t *)S.d_ecnt.p, escan, nt + 1, nullptr, &tb, s));
    PRK_TRY(temp(tb));
    PRK_TRY(prk_scan_u32((const uint32_t *)S.d_ecnt.p, escan, nt + 1, S.d_temp.p, &tb, s));
    PRK_TRY(prk_scan_u64((const unsigned long long *)S.d_rcnt.p, rscan, nt + 1, nullptr, &tb, s));
    PRK_TRY(temp(tb));
    PRK_TRY(prk_scan_u64((const unsigned long long *)S.d_rcnt.p, rscan, nt + 1, S.d_temp.p, &tb, s));
    // MergeSort of every object: per object when none has more than 64
    // edges (k_obj_sort_local, with the gather), else one radix sort of the
    // padded keys (prk_spans.hip); PRK_OBJ_LOCAL_SORT=0 forces the radix sort
    bool local_sort = nt && maxn <= 64;
    {
        const char *env = std::getenv("PRK_OBJ_LOCAL_SORT");
        if (env && env[0] == '0') local_sort = false;
    }
    PRK_TRY(prk_objtri_emit(&fp, d_objs, d_k0obj, d_k0tri0, nk0, nt, escan, pbits, ybits, c->H, S.d_edges.p,
                            S.d_ekeys.p, (uint32_t *)S.d_evals.p, local_sort ? 0 : 1, s));
    if (nt && !local_sort) {
        const uint32_t end_bit = obits + ybits + pbits;
        PRK_TRY(prk_obj_sort(S.d_ekeys.p, (uint32_t *)S.d_evals.p, S.d_ekeys2.p, ord, 3 * nt, end_bit, nullptr, &tb,
                             s));
        PRK_TRY(temp(tb));
        PRK_TRY(prk_obj_sort(S.d_ekeys.p, (uint32_t *)S.d_evals.p, S.d_ekeys2.p, ord, 3 * nt, end_bit, S.d_temp.p,
                             &tb, s));
    }
    // Span slots: each object's bound, exclusive-scanned into its first slot.
    PRK_TRY(S.d_bound.ensure(((size_t)nobj + 1) * 8));
    PRK_TRY(S.d_oslot.ensure(((size_t)nobj + 1) * 8));
    unsigned long long *oslot = (unsigned long long *)S.d_oslot.p;
    PRK_TRY(prk_obj_bound(&fp, d_objs, nobj, rscan, d_edges_in, (unsigned long long *)S.d_bound.p, s));
    PRK_TRY(prk_scan_u64((const unsigned long long *)S.d_bound.p, oslot, nobj + 1, nullptr, &tb, s));
    PRK_TRY(temp(tb));
    PRK_TRY(prk_scan_u64((const unsigned long long *)S.d_bound.p, oslot, nobj + 1, S.d_temp.p, &tb, s));
    // The walk's working copy, and each large object's most active edges
    // (read back with the slot total: they size its walk's workgroup).
    const uint32_t nwork = 3 * nt + (uint32_t)nk1;
    PRK_TRY(S.d_work.ensure(std::max<size_t>(nwork, 1) * 112));
    // The small triangle objects' segments (prk_spans.hip k_obj_seg, below):
    // a thread per stretch of rows with a non-empty list (PRK_OBJ_SEGMENTS=0:
    // a thread per object).
    const uint64_t max_segs = 3 * small_tris;
    bool segmented = false;
    {
        const char *env = std::getenv("PRK_OBJ_SEGMENTS");
        segmented = max_segs && max_segs < 0x7FFFFFFFull && !(env && env[0] == '0');
    }
    if (segmented) PRK_TRY(S.d_wy.ensure((size_t)std::max<uint64_t>(3 * nt, 1) * 8));
    if (local_sort)
        PRK_TRY(prk_obj_sort_local(d_objs, d_k0obj, nk0, escan, S.d_ekeys.p, S.d_edges.p, S.d_work.p,
                                   segmented ? S.d_wy.p : nullptr, (uint32_t *)S.d_err.p, s));
    if (!local_sort || nk1)
        PRK_TRY(prk_obj_gather(S.d_edges.p, local_sort ? nullptr : ord, total0p, d_edges_in, d_k1src, (uint32_t)nk1,
                               S.d_work.p, nwork, segmented ? S.d_wy.p : nullptr, s));
    // per large object: most, rows, entries (12, k_obj_maxact) | big (4) |
    // off (8) | cap (4) | the chunked walk's table (32, prk_spans.hip PrObj)
    // and groups (4)
    // | the huge walk's (rows, ents) (8)
    const size_t cls_bytes = (size_t)nbig_all * 72 + 64;
    if (cls_bytes > S.cls_cap) {
        if (S.h_cls) (void)hipHostFree(S.h_cls);
        S.h_cls = nullptr;
        S.cls_cap = 0;
        PRK_TRY(hipHostMalloc((void **)&S.h_cls, cls_bytes + cls_bytes / 4, hipHostMallocDefault));
        S.cls_cap = cls_bytes + cls_bytes / 4;
    }
    int32_t *h_most = reinterpret_cast<int32_t *>(S.h_cls);
    if (nbig_all) {
        PRK_TRY(S.d_most.ensure((size_t)nbig_all * 12));
        // (objects of kMaxactHugeEdges edges or more: many workgroups each;
        // PRK_OBJ_HUGE_EDGES=n (tests): n instead)
        const char *henv = std::getenv("PRK_OBJ_HUGE_EDGES");
        const uint32_t kMaxactHugeEdges = henv ? (uint32_t)std::max(1l, std::atol(henv)) : (1u << 18);
        PRK_TRY(prk_obj_maxact(&fp, d_objs, d_big, nbig_all, escan, total0p, S.d_work.p, (int32_t *)S.d_most.p,
                               kMaxactHugeEdges, s));
        for (uint32_t b = 0; b < nbig_all; ++b)
            if (big_edges[b] >= kMaxactHugeEdges) {
                PRK_TRY(S.d_mhuge.ensure(prk_maxact_huge_scratch()));
                PRK_TRY(prk_obj_maxact_huge(&fp, d_objs, d_big, b, nbig_all, big_edges[b], escan, total0p,
                                            S.d_work.p, (int32_t *)S.d_most.p, S.d_mhuge.p, s));
            }
        PRK_TRY(hipMemcpyAsync(h_most, S.d_most.p, (size_t)nbig_all * 12, hipMemcpyDeviceToHost, s));
    }
    PRK_TRY(hipMemcpyAsync(S.h_rb, oslot + nobj, 8, hipMemcpyDeviceToHost, s));
    PRK_TRY(hipStreamSynchronize(s));
    uint64_t nslot64;
    std::memcpy(&nslot64, S.h_rb, 8);
    if (nslot64 >= prk::kMaxPairs) return PRK_ERR_LIMIT;  // 31-bit span tags
    const uint32_t nslot = (uint32_t)nslot64;
    const size_t ns = std::max<uint32_t>(nslot, 1);
    PRK_TRY(S.d_recs.ensure(ns * 64));
    PRK_TRY(S.d_pos.ensure(ns * 16));
    PRK_TRY(S.d_span_tri.ensure(ns * 4));
    if (scalar) PRK_TRY(S.d_srecs.ensure(ns * 96));  // DrawModel span records (prk_spans.hip ScSpanRecG)
    if (nbig_all) PRK_TRY(S.d_raw.ensure(ns * 96));   // the slot walks' pairs (prk_spans.hip PairRaw)
    // slots no span takes stay row -1: binned nowhere.  Without large objects
    // every slot belongs to the thread or segment walks (walk_object,
    // k_obj_seg), which mark their unused ones themselves (C3b as 16-triangle
    // objects: ~21 M slots, a 0.34-GB memset); the large objects' walks rely
    // on this one.  PRK_POS_MEMSET=1 forces it.
    {
        const char *env = std::getenv("PRK_POS_MEMSET");
        if (nbig_all || (env && env[0] == '1')) PRK_TRY(hipMemsetAsync(S.d_pos.p, 0xFF, ns * 16, s));
    }
    // Walk groups: per mode, the large objects by the workgroup their list
    // needs (slot_threads(lcap) >= most + 2, lcap <= the device's), the rest
    // (more than lcap, or rows past k_obj_maxact's histogram) one wave each
    // with the list in a pool slice.
    struct Group {
        int32_t mode;
        uint32_t lcap, start, count;
        bool big;             // the huge-object walk (k_obj_walk_big / k_obj_walk_lds)
        uint32_t max_rows;    // (big: its objects' most rows)
        bool lds;             // (big: the list in LDS, k_obj_walk_lds)
    };
    std::vector<Group> groups;
    uint32_t *cls_big = reinterpret_cast<uint32_t *>(S.h_cls + (size_t)nbig_all * 12);
    unsigned long long *cls_off = reinterpret_cast<unsigned long long *>(S.h_cls + ((((size_t)nbig_all * 16) + 7) & ~(size_t)7));
    uint32_t *cls_cap = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(cls_off) + (size_t)nbig_all * 8);
    uint32_t *cls_pr = cls_cap + nbig_all;  // PrObj[npr] (8 words each)
    uint32_t *cls_grp = cls_pr + 8 * (size_t)nbig_all;  // its objects grouped by (mode, LDS capacity)
    uint32_t *cls_meta = cls_grp + nbig_all;           // (rows, ents) per object, walk-group order
    // Objects whose lists outgrow the workgroup walk's LDS slots take the
    // huge-object walk (a workgroup of 1024: k_obj_walk_lds with the whole
    // list in LDS when it fits prk_big_lds_cap() entries, else k_obj_walk_big
    // with it in device memory) when their sizes are known (k_obj_maxact) and
    // fit, else one wave each (k_obj_walk_wave).  PRK_OBJ_BIG=0: always the
    // wave; PRK_OBJ_LDSWALK=0: never the LDS form; PRK_OBJ_BIG_MIN=n (tests):
    // objects of more than n active edges skip the LDS slot classes.
    {
        const char *benv = std::getenv("PRK_OBJ_BIG"), *menv = std::getenv("PRK_OBJ_BIG_MIN"),
                   *lenv = std::getenv("PRK_OBJ_LDSWALK");
        const bool big_on = !(benv && benv[0] == '0'), lds_on = !(lenv && lenv[0] == '0');
        const int64_t big_min = menv ? std::atoll(menv) : INT64_MAX;
        const int32_t *h_rows = h_most + nbig_all, *h_ents = h_most + 2 * (size_t)nbig_all;
        static const uint32_t kCaps[] = {62, 126, 254, 510, 1022};
        uint32_t k = 0, b = 0;
        for (int mo = 0; mo < prk::MODE_COUNT; ++mo) {
            const uint32_t b0 = b;
            for (int ci = 0; ci <= 7; ++ci) {  // ci 5 / 6: the huge-object walk in LDS / device memory, 7: one wave each
                const uint32_t capc = ci < 5 ? kCaps[ci] : 0u;
                if (ci < 5 && capc > lcap) continue;
                const uint32_t start = k;
                uint32_t gmax = 0;  // (the huge walk: its objects' most rows)
                for (uint32_t i = 0; i < bigm[mo].size(); ++i) {
                    const uint32_t bi = b0 + i;
                    const int32_t most = h_most[bi];
                    uint32_t want = 0;  // the class this object takes
                    for (int cj = 0; cj < 5; ++cj)
                        if (kCaps[cj] <= lcap && most >= 0 && (uint32_t)most <= kCaps[cj] && most <= big_min) {
                            want = kCaps[cj];
                            break;
                        }
                    if (want != capc) continue;
                    const int32_t rows = h_rows[bi], ents = h_ents[bi];
                    const bool huge = ci == 5 || ci == 6;
                    if (ci >= 5) {
                        const bool hb = big_on && most > 0 && (uint32_t)most <= prk_big_max_entries() && rows > 0 &&
                                        rows < INT32_MAX && ents >= 0 && ents < INT32_MAX &&
                                        bigm[mo].size() <= 65535;
                        const bool hl = hb && lds_on && (uint32_t)most <= prk_big_lds_cap() && rows < 16000;
                        if ((hb ? (hl ? 5 : 6) : 7) != ci) continue;
                    }
                    const uint32_t cap = huge ? (uint32_t)most : bige[mo][i];
                    if (huge) pool = (pool + 3) & ~3ull;  // (16-B aligned slices)
                    cls_big[k] = bigm[mo][i];
                    cls_off[k] = capc ? 0ull : pool;
                    cls_cap[k] = capc ? 0u : cap;
                    cls_meta[2 * k] = huge ? (uint32_t)rows : 0u;
                    cls_meta[2 * k + 1] = huge ? (uint32_t)ents : 0u;
                    if (!capc)
                        pool += huge ? prk_big_slice_ints(cap, (uint32_t)rows, (uint32_t)ents)
                                     : (uint64_t)kWaveListArrays * (cap + 2);
                    if (huge) gmax = std::max(gmax, (uint32_t)rows);
                    ++k;
                }
                if (k > start) groups.push_back(Group{mo, capc, start, k - start, ci == 5 || ci == 6, gmax, ci == 5});
            }
            b += (uint32_t)bigm[mo].size();
        }
    }
    // The chunked walk (prk_spans.hip k_pr_*): the large objects walked with
    // their lists in LDS whose rows fit its histogram (PRK_OBJ_ROWS=0: none;
    // every object then takes the workgroup walk alone).  Objects by
    // (mode, LDS capacity class), as the walk groups.
    struct PrGroup {
        int32_t mode;
        uint32_t cap, start, count, max_chunks;
    };
    std::vector<PrGroup> prgroups;
    uint32_t npr = 0, pr_rows = 0, pr_chunks = 0, pr_max_edges = 0;
    uint64_t pr_ents = 0;
    {
        const char *env = std::getenv("PRK_OBJ_ROWS");
        const bool on = !(env && env[0] == '0');
        const uint32_t K = prk_pr_chunk_rows();
        const int32_t *h_rows = h_most + nbig_all;
        static const uint32_t kCapsPr[] = {62, 126, 254, 510, 1022};
        uint32_t b = 0;
        for (int mo = 0; on && mo < prk::MODE_COUNT; ++mo) {
            const uint32_t b0 = b;
            for (int ci = 0; ci < 5; ++ci) {
                const uint32_t capc = kCapsPr[ci];
                if (capc > lcap) continue;
                PrGroup g{mo, capc, npr, 0, 0};
                for (uint32_t i = 0; i < bigm[mo].size(); ++i) {
                    const uint32_t bi = b0 + i;
                    const int32_t most = h_most[bi], rows = h_rows[bi];
                    if (most <= 0 || most > prk_pr_max_row_entries() || rows <= 0 || rows > prk_pr_max_rows())
                        continue;
                    uint32_t want = 0;  // its capacity class (the walk groups' rule)
                    for (int cj = 0; cj < 5; ++cj)
                        if (kCapsPr[cj] <= lcap && (uint32_t)most <= kCapsPr[cj]) {
                            want = kCapsPr[cj];
                            break;
                        }
                    if (want != capc) continue;
                    const uint32_t nch = ((uint32_t)rows + K - 1) / K;
                    const uint64_t ents = (uint64_t)most * nch;
                    if (pr_ents + ents > kPrMaxEntries || npr >= 65535 || (uint64_t)pr_rows + rows + 1 > 0x7FFFFFFFull)
                        continue;
                    uint32_t *q = cls_pr + 8 * (size_t)npr;
                    q[0] = S.h_big_gl[bi];
                    q[1] = pr_rows;
                    q[2] = (uint32_t)rows;
                    q[3] = pr_chunks;
                    q[4] = (uint32_t)most;
                    q[5] = (uint32_t)pr_ents;
                    q[6] = q[7] = 0;
                    cls_grp[npr] = npr;
                    pr_rows += (uint32_t)rows + 1;
                    pr_chunks += nch;
                    pr_ents += ents;
                    pr_max_edges = std::max(pr_max_edges, big_edges[bi]);
                    g.max_chunks = std::max(g.max_chunks, nch);
                    ++g.count;
                    ++npr;
                }
                if (g.count) prgroups.push_back(g);
            }
            b += (uint32_t)bigm[mo].size();
        }
    }
    const uint32_t *d_cbig = nullptr, *d_ccap = nullptr, *d_cmeta = nullptr;
    const unsigned long long *d_coff = nullptr;
    const void *d_cpr = nullptr;
    const uint32_t *d_cgrp = nullptr;
    if (nbig_all) {
        const size_t lo = (size_t)nbig_all * 12, hi = reinterpret_cast<char *>(cls_meta + 2 * (size_t)nbig_all) - S.h_cls;
        PRK_TRY(S.d_cls.ensure(hi));
        PRK_TRY(hipMemcpyAsync(static_cast<char *>(S.d_cls.p) + lo, S.h_cls + lo, hi - lo, hipMemcpyHostToDevice, s));
        d_cbig = reinterpret_cast<const uint32_t *>(static_cast<char *>(S.d_cls.p) + lo);
        d_coff = reinterpret_cast<const unsigned long long *>(static_cast<char *>(S.d_cls.p) +
                                                              (reinterpret_cast<char *>(cls_off) - S.h_cls));
        d_ccap = reinterpret_cast<const uint32_t *>(static_cast<char *>(S.d_cls.p) +
                                                    (reinterpret_cast<char *>(cls_cap) - S.h_cls));
        d_cpr = static_cast<char *>(S.d_cls.p) + (reinterpret_cast<char *>(cls_pr) - S.h_cls);
        d_cgrp = reinterpret_cast<const uint32_t *>(static_cast<char *>(S.d_cls.p) +
                                                    (reinterpret_cast<char *>(cls_grp) - S.h_cls));
        d_cmeta = reinterpret_cast<const uint32_t *>(static_cast<char *>(S.d_cls.p) +
                                                     (reinterpret_cast<char *>(cls_meta) - S.h_cls));
        if (pool) PRK_TRY(S.d_pool.ensure(pool * 4));
    }
    const uint32_t *d_prstat = nullptr;
    if (npr) {
        // The chunked walk is an optimisation: when its scratch (up to
        // kPrMaxEntries * ~356 B) cannot be had, every object takes the
        // workgroup walk instead (d_prstat stays null) -- never PRK_ERR_NOMEM.
        hipError_t ae = S.d_prstat.ensure((size_t)nobj * 4);
        if (ae == hipSuccess) ae = S.d_prrow.ensure((size_t)npr * 8);
        if (ae == hipSuccess) ae = S.d_prcnt.ensure((size_t)pr_rows * 4);
        if (ae == hipSuccess) ae = S.d_preoff.ensure((size_t)pr_rows * 4);
        if (ae == hipSuccess) ae = S.d_prfge.ensure((size_t)pr_rows * 4);
        if (ae == hipSuccess) ae = S.d_prccur.ensure((size_t)pr_chunks * 4);
        if (ae == hipSuccess) ae = S.d_preendm.ensure((size_t)pr_chunks * 4);
        if (ae == hipSuccess) ae = S.d_prmatch.ensure((size_t)pr_chunks * 4);
        if (ae == hipSuccess) ae = S.d_prsm.ensure((size_t)pr_chunks * 4);
        if (ae == hipSuccess) ae = S.d_prsidx.ensure(pr_ents * 4);
        if (ae == hipSuccess) ae = S.d_prkey.ensure(pr_ents * 16);
        if (ae == hipSuccess) ae = S.d_prest.ensure(pr_ents * 112);  // prk_spans.hip ObjEdge
        if (ae == hipSuccess) ae = S.d_prsst.ensure(pr_ents * 112);
        if (ae == hipSuccess) ae = S.d_preend.ensure(pr_ents * 112);
        if (ae == hipErrorOutOfMemory) {
            (void)hipGetLastError();
            DevBuf *big[] = {&S.d_prsidx, &S.d_prkey, &S.d_prest, &S.d_prsst, &S.d_preend};
            for (DevBuf *b : big) b->release();
            npr = 0;
        } else {
            PRK_TRY(ae);
        }
    }
    if (npr) {
        PRK_TRY(hipMemsetAsync(S.d_prstat.p, 0, (size_t)nobj * 4, s));
        prk::PrWalkArgs pa{};
        pa.objs = d_objs;
        pa.pro = d_cpr;
        pa.npr = npr;
        pa.nchunks = pr_chunks;
        pa.max_edges = pr_max_edges;
        pa.escan = escan;
        pa.total0p = total0p;
        pa.work = S.d_work.p;
        pa.prrow = S.d_prrow.p;
        pa.cnt = (uint32_t *)S.d_prcnt.p;
        pa.eoff = (uint32_t *)S.d_preoff.p;
        pa.fge = (uint32_t *)S.d_prfge.p;
        pa.ccur = (uint32_t *)S.d_prccur.p;
        pa.key = S.d_prkey.p;
        pa.est = S.d_prest.p;
        pa.sst = S.d_prsst.p;
        pa.eend = S.d_preend.p;
        pa.eend_m = (uint32_t *)S.d_preendm.p;
        pa.match = (uint32_t *)S.d_prmatch.p;
        pa.sidx = (uint32_t *)S.d_prsidx.p;
        pa.s_m = (uint32_t *)S.d_prsm.p;
        pa.prstat = (uint32_t *)S.d_prstat.p;
        pa.soff = oslot;
        pa.raw = S.d_raw.p;
        pa.pos = S.d_pos.p;
        pa.span_tri = (uint32_t *)S.d_span_tri.p;
        pa.err = (uint32_t *)S.d_err.p;
        const char *warm = std::getenv("PRK_OBJ_CHUNK_WARMUP");  // 0: no warm-up (tests: every fix-up path)
        pa.warmup = !(warm && warm[0] == '0');
        PRK_TRY(prk_pr_walk_begin(&fp, &pa, s));
        for (const PrGroup &g : prgroups)
            PRK_TRY(prk_pr_walk_group(&fp, &pa, g.mode, g.cap, d_cgrp + g.start, g.count, g.max_chunks, s));
        PRK_TRY(prk_pr_walk_end(&pa, s));
        d_prstat = (const uint32_t *)S.d_prstat.p;
    }
    const void *d_segs = nullptr;  // (the segments)
    const uint32_t *d_nseg = nullptr;
    {
        if (segmented) {
            PRK_TRY(S.d_segcnt.ensure(((size_t)nobj + 1) * 4));
            PRK_TRY(S.d_segoff.ensure(((size_t)nobj + 1) * 4));
            PRK_TRY(S.d_segs.ensure((size_t)max_segs * 24));  // prk_spans.hip ObjSeg
            uint32_t *segcnt = (uint32_t *)S.d_segcnt.p, *segoff = (uint32_t *)S.d_segoff.p;
            PRK_TRY(prk_obj_seg(&fp, d_objs, nobj, escan, total0p, S.d_wy.p, oslot, segcnt, segoff, nullptr, nullptr,
                                s));
            PRK_TRY(prk_scan_u32(segcnt, segoff, nobj + 1, nullptr, &tb, s));
            PRK_TRY(temp(tb));
            PRK_TRY(prk_scan_u32(segcnt, segoff, nobj + 1, S.d_temp.p, &tb, s));
            PRK_TRY(prk_obj_seg(&fp, d_objs, nobj, escan, total0p, S.d_wy.p, oslot, segcnt, segoff, S.d_segs.p,
                                S.d_pos.p, s));
            d_segs = S.d_segs.p;
            d_nseg = segoff + nobj;
        }
    }
    PRK_TRY(prk_obj_walk(&fp, d_objs, nobj, escan, total0p, S.d_work.p, oslot, S.d_recs.p,
                         scalar ? S.d_srecs.p : nullptr, S.d_pos.p, (uint32_t *)S.d_span_tri.p, d_spans_in,
                         (uint32_t *)S.d_err.p, thread_links ? 1 : 0, d_segs, d_nseg, (uint32_t)max_segs, s));
    for (const Group &g : groups) {
        if (g.big)
            PRK_TRY(prk_big_walk(&fp, g.mode, g.lds ? 1 : 0, d_objs, d_cbig + g.start, d_coff + g.start, d_ccap + g.start,
                                 d_cmeta + 2 * (size_t)g.start, g.count, g.max_rows, (int32_t *)S.d_pool.p, escan,
                                 total0p, S.d_work.p, oslot, S.d_raw.p, S.d_pos.p, (uint32_t *)S.d_span_tri.p,
                                 (uint32_t *)S.d_err.p, d_prstat, s));
        else
            PRK_TRY(prk_obj_walk_group(&fp, g.mode, g.lcap, d_objs, d_cbig + g.start, d_coff + g.start,
                                       d_ccap + g.start, g.count, (int32_t *)S.d_pool.p, escan, total0p, S.d_work.p,
                                       oslot, S.d_recs.p, scalar ? S.d_srecs.p : nullptr, S.d_raw.p, S.d_pos.p,
                                       (uint32_t *)S.d_span_tri.p, (uint32_t *)S.d_err.p, d_prstat, s));
    }
    if (nbig_all)  // the slot walks' pairs into span records
        PRK_TRY(prk_span_finish(&fp, S.d_raw.p, nslot, S.d_recs.p, scalar ? S.d_srecs.p : nullptr, S.d_pos.p, s));
    // span -> tile bin entries: the tiles' counts and their scan (the
    // total comes back with the walk's status), then every span placed
    PRK_TRY(S.d_scnt.ensure(((size_t)ntiles + 1) * 4));
    PRK_TRY(S.d_offs.ensure(((size_t)ntiles + 1) * 4));
    uint32_t *tcnt = (uint32_t *)S.d_scnt.p, *toff = (uint32_t *)S.d_offs.p;
    PRK_TRY(prk_span_count(&fp, S.d_pos.p, nslot, tcnt, s));
    PRK_TRY(prk_scan_u32(tcnt, toff, ntiles + 1, nullptr, &tb, s));
    PRK_TRY(temp(tb));
    PRK_TRY(prk_scan_u32(tcnt, toff, ntiles + 1, S.d_temp.p, &tb, s));
    PRK_TRY(hipMemcpyAsync(S.h_rb + 2, toff + ntiles, 4, hipMemcpyDeviceToHost, s));
    PRK_TRY(hipMemcpyAsync(S.h_rb + 3, S.d_err.p, 16, hipMemcpyDeviceToHost, s));
    PRK_TRY(hipStreamSynchronize(s));
    const uint32_t total = S.h_rb[2];
    if (S.h_rb[3]) return PRK_ERR_DEVICE;  // a walk outside its LDS list or span slots (never)
    if (std::getenv("PRK_PR_DEBUG"))
        std::fprintf(stderr, "prk: large objects %u, chunked: taken %u done %u failed %u; chunks %u, walked again %u\n",
                     nbig_all, npr, S.h_rb[4], S.h_rb[5], pr_chunks, S.h_rb[6]);
    c->stats.objects_chunked += S.h_rb[4];
    c->stats.objects_walked += nbig_all - S.h_rb[4];
    c->stats.object_chunks += pr_chunks;
    c->stats.object_chunks_rewalked += S.h_rb[6];
    c->stats.triangles = T;
    c->stats.tiles = ntiles;
    c->stats.bin_entries = total;
    PRK_TRY(S.d_vals_b.ensure((size_t)std::max<uint32_t>(total, 1) * 4));
    PRK_TRY(prk_span_bin(&fp, S.d_pos.p, nslot, toff, tcnt, (uint32_t *)S.d_vals_b.p, s));
    PRK_TRY(S.d_nwin.ensure((size_t)ntiles * 4));
    PRK_TRY(S.d_wtag.ensure((size_t)ntiles * fp.tile_w * fp.tile_h * 4));
    PRK_TRY(prk_launch_spans(&fp, (const uint32_t *)S.d_offs.p, (const uint32_t *)S.d_vals_b.p, S.d_pos.p,
                             S.d_recs.p, scalar ? S.d_srecs.p : nullptr, modes, (const uint32_t *)S.d_span_tri.p,
                             (uint32_t *)S.d_nwin.p, (uint32_t *)S.d_wtag.p, s));
    return PRK_OK;
}

int prk_flush(prk_context *c, void *stream) {
    if (!c) return PRK_ERR_ARG;
    if (!c->color) return PRK_ERR_NO_TARGET;
    if (!c->have_camera) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    {
        const int rc = resolve_count(c);  // the previous frame's count first: it may change the tile
        if (rc != PRK_OK) return rc;
    }
    if (c->tile_auto) {  // the frame's tile (see prk_context::tile_auto)
        const int64_t px = (int64_t)c->W * (c->row1 - c->row0);
        if ((c->auto_small || c->auto_wide) &&
            ((uint64_t)c->pending_tris > 2ull * c->auto_T || 2ull * c->pending_tris < c->auto_T ||
             px > 2 * (int64_t)c->auto_px || 2 * px < (int64_t)c->auto_px))
            c->auto_small = c->auto_wide = 0;  // re-decide from this frame's count
        c->tile_w = c->auto_small ? c->auto_small : (c->auto_wide ? c->auto_wide : 256);
        c->tile_h = 8;
    }
    hipStream_t s = stream ? (hipStream_t)stream : c->own_stream;
    if (c->in_wait) {  // prk_geometry_write copies still in flight: every stream of the frame waits for them
        PRK_TRY(hipStreamWaitEvent(s, c->in_ev, 0));
        PRK_TRY(hipStreamWaitEvent(c->bin_stream, c->in_ev, 0));
        PRK_TRY(hipStreamWaitEvent(c->vis_stream, c->in_ev, 0));
        c->in_wait = false;
    }
    bool any_avx = false;
    for (const auto &d : c->draws) any_avx |= d.mode == prk::MODE_AVX;
    if (any_avx && (c->W % 8)) return PRK_ERR_UNSUPPORTED;  // aligned 8-wide z load, projekt.cpp:2218
    prk::FrameParams probe;
    frame_params(c, probe);
    if (probe.tiles_x > 65535 || probe.tiles_y > 65535) return PRK_ERR_UNSUPPORTED;
    if (!c->d_prof.p) {
        PRK_TRY(c->d_prof.ensure(16 * sizeof(uint64_t)));
        PRK_TRY(hipMemsetAsync(c->d_prof.p, 0, 16 * sizeof(uint64_t), s));
    }
    if (!c->d_negz.p) {
        PRK_TRY(c->d_negz.ensure(4));
        PRK_TRY(hipMemsetAsync(c->d_negz.p, 0, 4, s));
    }
    c->z_early = false;  // (the passes below say whether the frame's last one allows it)
    if (c->debug) {
        PRK_TRY(c->d_winners.ensure((size_t)c->W * (c->row1 - c->row0) * 4));
        PRK_TRY(hipMemsetAsync(c->d_winners.p, 0xFF, (size_t)c->W * (c->row1 - c->row0) * 4, s));
        c->winners_valid = true;
    }
    // Passes: maximal runs of draws of one kind (per-triangle AETs, or
    // whole-object AETs); each pass z-tests against the target as the
    // previous one left it, which is the reference's sequential order.
    std::vector<prk::DrawRec> dr = std::move(c->draws);
    c->draws.clear();
    c->pending_tris = 0;
    struct Clear {  // the frame's edge / span input goes with its draws
        prk_context *c;
        ~Clear() { c->pend_edges.clear(); c->pend_spans.clear(); }
    } clear_src{c};
    if (dr.empty()) return c->clear_pending ? fill_pending_clear(c, s) : PRK_OK;
    auto span_path = [](const prk::DrawRec &d) { return d.obj_tris > 1 || d.src_kind != 0; };
    size_t i = 0;
    int rc = PRK_OK;
    while (i < dr.size() && rc == PRK_OK) {
        const bool obj = span_path(dr[i]);
        size_t j = i;
        std::vector<prk::DrawRec> seg;
        uint32_t T = 0;
        const uint32_t base = dr[i].first_global;
        while (j < dr.size() && span_path(dr[j]) == obj) {
            prk::DrawRec d = dr[j];
            d.first_global -= base;
            T += d.tri_count;
            seg.push_back(d);
            ++j;
        }
        // (only the frame's last pass defers its count: a later pass z-tests
        // against this one's output, so an overflow must be re-run first)
        rc = obj ? flush_spans(c, s, seg, T, base) : flush_tris(c, s, seg, T, base, j == dr.size());
        i = j;
    }
    // the frame's last reader of the geometry (the flush stream ends every pass)
    c->read_rec = hipEventRecord(c->read_ev, s) == hipSuccess;
    return rc;
}


int prk_get_target(prk_context *c, void **color, int32_t *pitch_bytes, float **zbuf, int32_t *width,
                   int32_t *height, int32_t *row0, int32_t *row1) {
    if (!c) return PRK_ERR_ARG;
    if (!c->color) return PRK_ERR_NO_TARGET;
    if (color) *color = c->color;
    if (pitch_bytes) *pitch_bytes = c->pitch;
    if (zbuf) *zbuf = c->zbuf;
    if (width) *width = c->W;
    if (height) *height = c->H;
    if (row0) *row0 = c->row0;
    if (row1) *row1 = c->row1;
    return PRK_OK;
}

int prk_get_device(prk_context *c, int32_t *device, void **stream) {
    if (!c) return PRK_ERR_ARG;
    if (device) *device = c->device;
    if (stream) *stream = (void *)c->own_stream;
    return PRK_OK;
}

// prk_dist.hip: gathers read the band's finished frame (library-internal).
// The pending count is resolved first (an overflowed frame is re-run on its
// own flush stream), then `stream` (the gather's, any stream of the
// context's device) waits for the end of the context's last frame.
__attribute__((visibility("hidden"))) int prk_resolve_pending(prk_context *c, void *stream) {
    if (!c) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    if (stream && c->read_rec) {
        PRK_TRY(hipSetDevice(c->device));
        PRK_TRY(hipStreamWaitEvent((hipStream_t)stream, c->read_ev, 0));
    }
    return PRK_OK;
}

int prk_resolve(prk_context *c, void *stream) { return prk_resolve_pending(c, stream); }

int prk_synchronize(prk_context *c) {
    if (!c) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    PRK_TRY(hipSetDevice(c->device));
    PRK_TRY(hipStreamSynchronize(c->own_stream));
    PRK_TRY(hipDeviceSynchronize());
    return PRK_OK;
}

int prk_get_stats(prk_context *c, prk_stats *out) {
    if (!c || !out) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    (void)hipSetDevice(c->device);
    for (int i = 1; i <= prk_context::kRing; ++i)  // oldest first
        harvest(c, (int)((c->frame + i) % prk_context::kRing));
    if (c->d_anomaly.p) {
        PRK_TRY(hipDeviceSynchronize());
        static_assert(offsetof(prk_stats, slow_replays) == offsetof(prk_stats, anomalies) + 4, "counter pair");
        PRK_TRY(hipMemcpy(&c->stats.anomalies, c->d_anomaly.p, 8, hipMemcpyDeviceToHost));
    }
    *out = c->stats;
    return PRK_OK;
}

int prk_download_winners(prk_context *c, int32_t *w) {
    if (!c || !w) return PRK_ERR_ARG;
    RESOLVE_COUNT(c);
    if (!c->winners_valid || !c->d_winners.p) return PRK_ERR_ARG;
    PRK_TRY(hipSetDevice(c->device));
    PRK_TRY(hipDeviceSynchronize());
    PRK_TRY(hipMemcpy(w, c->d_winners.p, (size_t)c->W * (c->row1 - c->row0) * 4, hipMemcpyDeviceToHost));
    return PRK_OK;
}

// FillEdgeTable's return value (projekt.cpp:3882-4121), computed on the host
// at the call so the drop-in can return it there: the number of edge_info
// records the reference writes for one object, i.e. over its triangles that
// pass the back-face test (3926-3943) the edges with MaxY > 0 (3968) and
// MinY != MaxY (4066).  The same float operations as the device setup
// (ProjectVertex 74-93, Normalize(a) = (1/sqrt(a.a))*a); the library is built
// with -ffp-contract=off, so host and device round alike.  The setup itself
// (edges, gradients, lighting, MergeSort) runs on the GPU at the flush.
// Per triangle: include/prk_edge_count.h (the drop-in header inlines it).
int prk_fill_edge_count(const float *V, uint32_t vertex_count, const float P[3], const prk_transform *T,
                        uint32_t *count_out) {
    if (!count_out || !T || (!V && vertex_count >= 3)) return PRK_ERR_ARG;
    const float p0 = P ? P[0] : 0.0f, p1 = P ? P[1] : 0.0f, p2 = P ? P[2] : 0.0f;
    uint32_t n = 0;
    for (uint32_t t = 0; t < vertex_count / 3; ++t) n += prk_tri_edge_count(V + 9 * (size_t)t, p0, p1, p2, T);
    *count_out = n;
    return PRK_OK;
}

// ConstructSphere (projekt.cpp:4123-4289): the reference's only test mesh.
// 24 inclination x 48 azimuth steps, r = 0.5, 6624 vertices.
int prk_construct_sphere(float *V, float *Col, float *N, float *UV, uint32_t *count_out) {
    if (!V || !Col || !N || !UV || !count_out) return PRK_ERR_ARG;
    const float Pi32 = 3.14159265359f;
    const float Radius = 0.5f;
    const uint32_t StepCount = 24;
    const float Up[4] = {1, 0, 0, 1}, Down[4] = {0, 1, 0, 1};
    float Inc[4];
    for (int k = 0; k < 4; ++k) Inc[k] = (Down[k] - Up[k]) / (float)StepCount;
    const float IncI = Pi32 / StepCount;
    const float IncA = (2.0f * Pi32) / (StepCount * 2);
    float Cur[4] = {Up[0], Up[1], Up[2], Up[3]};
    uint32_t n = 0;
    auto emit = [&](float x, float y, float z, float u, float v, const float *c4, const float *blue, bool inc) {
        V[3 * n] = Radius * x; V[3 * n + 1] = Radius * y; V[3 * n + 2] = Radius * z;
        N[3 * n] = x; N[3 * n + 1] = y; N[3 * n + 2] = z;
        UV[2 * n] = u; UV[2 * n + 1] = v;
        for (int k = 0; k < 4; ++k) Col[4 * n + k] = inc ? (c4[k] + Inc[k]) + blue[k] : c4[k] + blue[k];
        ++n;
    };
    for (uint32_t ii = 0; ii < StepCount; ++ii) {
        for (uint32_t ai = 0; ai < StepCount * 2; ++ai) {
            float I0 = (float)ii * IncI, I1 = (float)(ii + 1) * IncI;
            float A0 = (float)ai * IncA, A1 = (float)(ai + 1) * IncA;
            float Blue[4] = {0, 0, (1.0f + cosf(A0)) / 2.0f, 0};
            float NBlue[4] = {0, 0, (1.0f + cosf(A1)) / 2.0f, 0};
            if (ii == 0) {
                float S[3] = {sinf(I1) * cosf(A0), cosf(I1), sinf(I1) * sinf(A0)};
                float Tt[3] = {sinf(I1) * cosf(A1), cosf(I1), sinf(I1) * sinf(A1)};
                emit(0, 1, 0, 0.5f, 0.5f, Cur, Blue, false);
                emit(S[0], S[1], S[2], S[0], S[2], Cur, Blue, true);
                emit(Tt[0], Tt[1], Tt[2], Tt[0], Tt[2], Cur, NBlue, true);
            } else if (ii == StepCount - 1) {
                float F[3] = {sinf(I0) * cosf(A0), cosf(I0), sinf(I0) * sinf(A0)};
                float Tt[3] = {sinf(I0) * cosf(A1), cosf(I0), sinf(I0) * sinf(A1)};
                emit(F[0], F[1], F[2], 0.5f, 0.5f, Cur, Blue, false);
                emit(0, -1, 0, 0.0f, 0.0f, Cur, Blue, true);
                emit(Tt[0], Tt[1], Tt[2], Tt[0], Tt[2], Cur, NBlue, true);
            } else {
                float F[3] = {sinf(I0) * cosf(A0), cosf(I0), sinf(I0) * sinf(A0)};
                float S[3] = {sinf(I1) * cosf(A0), cosf(I1), sinf(I1) * sinf(A0)};
                float Tt[3] = {sinf(I1) * cosf(A1), cosf(I1), sinf(I1) * sinf(A1)};
                float Fo[3] = {sinf(I0) * cosf(A1), cosf(I0), sinf(I0) * sinf(A1)};
                auto uvx = [](float a) { return (a + 1.0f) / 2.0f; };
                emit(F[0], F[1], F[2], uvx(F[0]), uvx(F[1]), Cur, Blue, false);
                emit(S[0], S[1], S[2], uvx(S[0]), uvx(S[1]), Cur, Blue, true);
                emit(Tt[0], Tt[1], Tt[2], uvx(Tt[0]), uvx(Tt[1]), Cur, NBlue, true);
                emit(F[0], F[1], F[2], uvx(F[0]), uvx(F[1]), Cur, Blue, false);
                emit(Tt[0], Tt[1], Tt[2], uvx(Tt[0]), uvx(Tt[1]), Cur, NBlue, true);
                emit(Fo[0], Fo[1], Fo[2], uvx(Fo[0]), uvx(Fo[1]), Cur, NBlue, false);
            }
        }
        for (int k = 0; k < 4; ++k) Cur[k] = Cur[k] + Inc[k];
    }
    *count_out = n;
    return PRK_OK;
}

}  // extern "C"
