// prk_host_stub.cpp — a stand-in libprk_hip for timing the drop-in header's
// host side (include/projekt.h) on a machine without a GPU.
//
// Every entry point projekt.h and examples/dropin_bench.cpp call returns
// PRK_OK at once; host memory entry points use the C heap; the edge count is
// the real one (include/prk_edge_count.h).  Built with
//   make -C tools/hoststub        ->  tools/hoststub/dropin_bench_stub
// and run as `dropin_bench_stub [frames] [triangles]`: its host_calls_ms and
// fill_edge_table_only_ms are the header's per-call cost on this CPU (the
// GPU columns read 0).  Profiling aid only: never shipped, never loaded by
// the product or its tests.
#include <cstdlib>
#include <cstring>

#include "prk.h"
#include "prk_edge_count.h"

struct prk_context {
    int dummy;
};
static prk_context g_ctx;

extern "C" {
int prk_create(int, prk_context **out) {
    *out = &g_ctx;
    return PRK_OK;
}
int prk_destroy(prk_context *) { return PRK_OK; }
int prk_band_rows(int32_t height, int32_t rank, int32_t nranks, int32_t *row0, int32_t *row1) {
    *row0 = (int32_t)((int64_t)height * rank / nranks);
    *row1 = (int32_t)((int64_t)height * (rank + 1) / nranks);
    return PRK_OK;
}
int prk_draw_edges(prk_context *, const prk_edge *, uint32_t, int32_t, int32_t, int32_t) { return PRK_OK; }
int prk_draw_objects_setup(prk_context *, int32_t, uint32_t, uint32_t, uint32_t, const float *, int32_t, int32_t,
                           int32_t, int32_t) {
    return PRK_OK;
}
int prk_draw_spans(prk_context *, const prk_span *, uint32_t, int32_t, int32_t, int32_t) { return PRK_OK; }
int prk_fill_edge_count(const float *V, uint32_t vertex_count, const float P[3], const prk_transform *T,
                        uint32_t *count_out) {
    uint32_t n = 0;
    for (uint32_t t = 0; t < vertex_count / 3; ++t) n += prk_tri_edge_count(V + 9 * (size_t)t, P[0], P[1], P[2], T);
    *count_out = n;
    return PRK_OK;
}
int prk_flush(prk_context *, void *) { return PRK_OK; }
int prk_advance_edge_records(void *, uint32_t, size_t, size_t, int32_t) { return PRK_OK; }
int prk_fill_edge_records(const float *, const float *, const float *, const float *, uint32_t, const float *,
                          const prk_transform *, const prk_light_data *, int32_t, void *, size_t, size_t, void *,
                          uint32_t *count_out) {
    *count_out = 0;
    return PRK_OK;
}
int prk_geometry_create(prk_context *, const float *, const float *, const float *, const float *, uint32_t,
                        int32_t *h) {
    *h = 0;
    return PRK_OK;
}
int prk_geometry_write(prk_context *, int32_t, uint32_t, uint32_t, const float *, const float *, const float *,
                       const float *) {
    return PRK_OK;
}
int prk_get_stats(prk_context *, prk_stats *out) {
    std::memset(out, 0, sizeof *out);
    return PRK_OK;
}
int prk_host_alloc(prk_context *, size_t bytes, void **out) {
    *out = std::aligned_alloc(4096, (bytes + 4095) & ~(size_t)4095);
    if (*out) std::memset(*out, 0, bytes);  // (pinned memory comes committed)
    return *out ? PRK_OK : PRK_ERR_NOMEM;
}
int prk_host_free(prk_context *, void *p) {
    std::free(p);
    return PRK_OK;
}
int prk_host_register(prk_context *, void *, size_t) { return PRK_OK; }
int prk_host_unregister(prk_context *, void *) { return PRK_OK; }
int prk_reset_draws(prk_context *) { return PRK_OK; }
int prk_set_camera(prk_context *, const prk_transform *, const prk_light_data *) { return PRK_OK; }
int prk_set_early_z(prk_context *, int) { return PRK_OK; }
int prk_set_shade_camera(prk_context *, const prk_transform *, const prk_light_data *) { return PRK_OK; }
int prk_synchronize(prk_context *) { return PRK_OK; }
int prk_target_alloc(prk_context *, int32_t, int32_t, int32_t, int32_t, void **, float **) { return PRK_OK; }
int prk_target_clear_on_flush(prk_context *, uint32_t, float) { return PRK_OK; }
int prk_target_download(prk_context *, uint32_t *, int32_t, float *) { return PRK_OK; }
int prk_target_upload(prk_context *, const uint32_t *, int32_t, const float *) { return PRK_OK; }
int prk_target_upload_async(prk_context *, const uint32_t *, int32_t, const float *) { return PRK_OK; }
int prk_texture_create(prk_context *, const prk_bitmap *, int32_t *h) {
    *h = 0;
    return PRK_OK;
}
int prk_texture_update(prk_context *, int32_t, const prk_bitmap *) { return PRK_OK; }
int prk_timing_reset(prk_context *) { return PRK_OK; }
int prk_construct_sphere(float *, float *, float *, float *, uint32_t *n) {
    *n = 0;
    return PRK_OK;
}
}
