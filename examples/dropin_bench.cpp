// dropin_bench.cpp — the headline workload (C3b: 4096 x 4096, 1M random
// triangles with offsets of +-16 px, Phong + 256^2 texture, one light) driven
// the way a reference caller drives it: every triangle its own
// render_entry_3d_object through FillEdgeTable + DrawModelOptimized(RenderQueue,
// ...) of include/projekt.h, then PRK_CompleteAllWork, frame after frame.
//
// Per frame it reports the host time of the 1M FillEdgeTable + DrawModel
// calls (vertex snapshot into the pinned arena), the time of
// PRK_CompleteAllWork (geometry upload over PCIe, the GPU frame, colour + z
// download into the caller's buffers), and the GPU kernels' own time.  Two
// modes: "upload" (the generic drop-in: the caller's framebuffer and z-buffer
// go up as the frame's prior contents) and "clear" (PRK_ClearNextFrame: the
// caller clears, the clear is fused into the GPU frame instead of uploaded).
// The scene is generated here with std::mt19937 (same distribution as
// prk.scenes.random_soup, not the same numbers).
//
// usage: dropin_bench [frames] [triangles] [width]
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "projekt.h"

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); }

int main(int argc, char **argv) {
    const int frames = argc > 1 ? std::atoi(argv[1]) : 5;
    const u32 T = argc > 2 ? (u32)std::atoi(argv[2]) : 1000000u;
    const s32 W = argc > 3 ? std::atoi(argv[3]) : 4096, H = W;
    if (PRK_Init(0) != PRK_OK) {
        std::fprintf(stderr, "dropin_bench: no HIP device (status %d)\n", PRK_LastStatus());
        return 2;
    }
    // camera of prk.scenes: D = 4, F = 1, M2P = W/2, C = (W/2, H/2)
    const float D = 4.0f, M2P = W / 2.0f, cx = W / 2.0f, cy = H / 2.0f, R = 16.0f;
    std::mt19937 rng(2024);
    std::uniform_real_distribution<float> U01(0.0f, 1.0f);
    std::vector<v3> V(3 * (size_t)T), N(3 * (size_t)T);
    std::vector<v4> C(3 * (size_t)T);
    std::vector<v2> UV(3 * (size_t)T);
    for (u32 t = 0; t < T; ++t) {
        const float ccx = -R + (W + 2 * R) * U01(rng), ccy = -R + (H + 2 * R) * U01(rng);
        float sx[3], sy[3];
        for (int k = 0; k < 3; ++k) {
            sx[k] = ccx + (2 * U01(rng) - 1) * R;
            sy[k] = ccy + (2 * U01(rng) - 1) * R;
        }
        if ((sx[1] - sx[0]) * (sy[2] - sy[0]) - (sy[1] - sy[0]) * (sx[2] - sx[0]) > 0) {  // front-facing winding
            std::swap(sx[1], sx[2]);
            std::swap(sy[1], sy[2]);
        }
        const float z0 = 2 * U01(rng) - 1;
        for (int k = 0; k < 3; ++k) {
            const float z = z0 + (2 * U01(rng) - 1) * 0.15f;
            const size_t i = 3 * (size_t)t + k;
            V[i] = {{(sx[k] - cx) * (D - z) / M2P, (sy[k] - cy) * (D - z) / M2P, z}};
            float nx = 2 * U01(rng) - 1, ny = 2 * U01(rng) - 1, nz = 2 * U01(rng) - 1;
            const float l = std::sqrt(nx * nx + ny * ny + nz * nz) + 1e-6f;
            N[i] = {{nx / l, ny / l, nz / l}};
            C[i] = {{U01(rng), U01(rng), U01(rng), 1.0f}};
            UV[i] = {{U01(rng), U01(rng)}};
        }
    }
    std::vector<u32> texels(256 * 256);
    for (auto &x : texels) x = (u32)rng();
    loaded_bitmap Texture = {texels.data(), 256, 256, 256 * 4};
    std::vector<u32> pixels((size_t)W * H);
    std::vector<r32> zbuf((size_t)W * H);
    loaded_bitmap Buffer = {pixels.data(), W, H, W * 4};
    game_render_commands Commands = {};
    Commands.ZBuffer = zbuf.data();
    Commands.Width = (u32)W;
    Commands.Transform.DistanceAboveTarget = D;
    Commands.Transform.FocalLength = 1.0f;
    Commands.Transform.MetersToPixels = M2P;
    Commands.Transform.ScreenCenter.x = cx;
    Commands.Transform.ScreenCenter.y = cy;
    Commands.LightData.LightCount = 1;
    Commands.LightData.Lights[0].P = {{1.0f, 1.0f, 3.0f}};
    Commands.LightData.Lights[0].Intensity = {{0.8f, 0.8f, 0.8f, 1.0f}};
    Commands.LightData.AmbientIntensity = {{0.2f, 0.2f, 0.2f, 1.0f}};
    std::vector<edge_info> EdgeMemory(3);

    std::printf("{\"workload\": \"C3b through include/projekt.h: %u per-triangle objects, %dx%d\", \"modes\": {", T, W, H);
    for (int m = 0; m < 2; ++m) {
        const bool clear = m == 1;
        double calls = 0, complete = 0, total = 0, gpu = 0, issue = 0, flush = 0, down = 0;
        int timed = 0;
        for (int f = 0; f < frames + 1; ++f) {
            // the caller's own clear of its buffers (both modes: the reference caller does it)
            const auto t0 = clk::now();
            std::fill(pixels.begin(), pixels.end(), 0xFF000000u);
            std::fill(zbuf.begin(), zbuf.end(), -FLT_MAX);
            if (clear) PRK_ClearNextFrame(0xFF000000u, -FLT_MAX);
            prk_timing_reset(prk_dropin::S().Ctx);
            const auto t1 = clk::now();
            for (u32 t = 0; t < T; ++t) {
                render_entry_3d_object Object = {};
                Object.VertexCount = 3;
                Object.PhongShading = 1;
                Object.VertexData = &V[3 * (size_t)t];
                Object.ColorData = &C[3 * (size_t)t];
                Object.NormalData = &N[3 * (size_t)t];
                Object.UVData = &UV[3 * (size_t)t];
                Object.EdgeMemory = EdgeMemory.data();
                Object.Bitmap = &Texture;
                const u32 n = FillEdgeTable(&Object, &Commands, 1);
                DrawModelOptimized(nullptr, &Buffer, EdgeMemory.data(), n, &Commands, &Texture, 1);
            }
            const double tc = ms_since(t1);
            const auto t2 = clk::now();
            if (PRK_CompleteAllWork(&Buffer, &Commands) != PRK_OK) {
                std::fprintf(stderr, "dropin_bench: CompleteAllWork failed (status %d)\n", PRK_LastStatus());
                return 2;
            }
            const double tw = ms_since(t2), tt = ms_since(t0);
            prk_stats st;
            prk_get_stats(prk_dropin::S().Ctx, &st);
            if (f > 0) {  // frame 0 warms up (allocations, page locking)
                calls += tc;
                complete += tw;
                total += tt;
                gpu += st.frames_timed ? (st.sum_ms_raster + st.sum_ms_bin) / st.frames_timed : 0.0;
                issue += prk_dropin::S().LastIssueMs;
                flush += prk_dropin::S().LastFlushMs;
                down += prk_dropin::S().LastDownloadMs;
                ++timed;
            }
        }
        std::printf("%s\"%s\": {\"frame_ms\": %.3f, \"host_calls_ms\": %.3f, \"complete_all_work_ms\": %.3f, "
                    "\"complete_split_ms\": {\"record_draws_and_tail\": %.3f, \"queue_frame\": %.3f, "
                    "\"wait_and_download\": %.3f}, \"gpu_bin_plus_raster_ms\": %.3f, \"mpixels_s\": %.1f}",
                    m ? ", " : "", clear ? "clear" : "upload", total / timed, calls / timed, complete / timed,
                    issue / timed, flush / timed, down / timed, gpu / timed,
                    (double)W * H / (total / timed * 1e-3) / 1e6);
    }
    // The host calls split by entry point: every object's FillEdgeTable into
    // an EdgeMemory of its own, then every DrawModelOptimized, timed apart
    // (the frame is then run and downloaded as above, untimed).
    double fill_pass = 0, draw_pass = 0;
    {
        std::vector<edge_info> EM(T);
        std::vector<u32> ne(T);
        for (int f = 0; f < frames + 1; ++f) {
            PRK_ClearNextFrame(0xFF000000u, -FLT_MAX);
            auto t1 = clk::now();
            for (u32 t = 0; t < T; ++t) {
                render_entry_3d_object Object = {};
                Object.VertexCount = 3;
                Object.PhongShading = 1;
                Object.VertexData = &V[3 * (size_t)t];
                Object.ColorData = &C[3 * (size_t)t];
                Object.NormalData = &N[3 * (size_t)t];
                Object.UVData = &UV[3 * (size_t)t];
                Object.EdgeMemory = &EM[t];
                Object.Bitmap = &Texture;
                ne[t] = FillEdgeTable(&Object, &Commands, 1);
            }
            if (f > 0) fill_pass += ms_since(t1);
            t1 = clk::now();
            for (u32 t = 0; t < T; ++t) DrawModelOptimized(nullptr, &Buffer, &EM[t], ne[t], &Commands, &Texture, 1);
            if (f > 0) draw_pass += ms_since(t1);
            if (PRK_CompleteAllWork(&Buffer, &Commands) != PRK_OK) {
                std::fprintf(stderr, "dropin_bench: CompleteAllWork failed (status %d)\n", PRK_LastStatus());
                return 2;
            }
        }
    }
    // The host calls split: frames of FillEdgeTable calls alone.
    double fill = 0;
    for (int f = 0; f < frames + 1; ++f) {
        const auto t1 = clk::now();
        for (u32 t = 0; t < T; ++t) {
            render_entry_3d_object Object = {};
            Object.VertexCount = 3;
            Object.PhongShading = 1;
            Object.VertexData = &V[3 * (size_t)t];
            Object.ColorData = &C[3 * (size_t)t];
            Object.NormalData = &N[3 * (size_t)t];
            Object.UVData = &UV[3 * (size_t)t];
            Object.EdgeMemory = EdgeMemory.data();
            Object.Bitmap = &Texture;
            (void)FillEdgeTable(&Object, &Commands, 1);
        }
        if (f > 0) fill += ms_since(t1);
        // nothing was drawn (no frame is open): drop the frame's objects
        prk_synchronize(prk_dropin::S().Ctx);
        prk_dropin::end_frame(prk_dropin::S());
    }
    // ... and its parts: the visible-edge count (the call's return value) and
    // the vertex snapshot into pinned memory, each alone.
    double count = 0, count_inline = 0, copy = 0, copy_heap = 0, copy_nt = 0;
    {
        const prk_dropin::camera cam = prk_dropin::camera_of(&Commands);
        const float P[3] = {0.0f, 0.0f, 0.0f};
        float *a[4] = {nullptr, nullptr, nullptr, nullptr};
        const size_t comp[4] = {3, 4, 3, 2};
        for (int k = 0; k < 4; ++k) prk_host_alloc(prk_dropin::S().Ctx, 3 * (size_t)T * comp[k] * 4, (void **)&a[k]);
        float *h[4] = {nullptr, nullptr, nullptr, nullptr};
        for (int k = 0; k < 4; ++k) {
            const size_t bytes = ((3 * (size_t)T * comp[k] * 4) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
            h[k] = (float *)std::aligned_alloc(2u << 20, bytes);
            if (h[k]) memset(h[k], 0, bytes);
        }
        uint64_t sink = 0;
        for (int f = 0; f < frames + 1; ++f) {
            auto t1 = clk::now();
            for (u32 t = 0; t < T; ++t) {
                u32 e = 0;
                prk_fill_edge_count((const float *)&V[3 * (size_t)t], 3, P, &cam.T, &e);
                sink += e;
            }
            if (f > 0) count += ms_since(t1);
#if PRK_EC_SSE
            t1 = clk::now();
            for (u32 t = 0; t < T; ++t) {
                const float *v = (const float *)&V[3 * (size_t)t];
                sink += prk_tri_edge_count_sse(_mm_loadu_ps(v), _mm_loadu_ps(v + 4), _mm_load_ss(v + 8), P[0], P[1],
                                               P[2], &cam.T);
            }
            if (f > 0) count_inline += ms_since(t1);
#endif
            t1 = clk::now();
            if (a[0] && a[1] && a[2] && a[3])
                for (u32 t = 0; t < T; ++t) {
                    memcpy(a[0] + 9 * (size_t)t, &V[3 * (size_t)t], 36);
                    memcpy(a[1] + 12 * (size_t)t, &C[3 * (size_t)t], 48);
                    memcpy(a[2] + 9 * (size_t)t, &N[3 * (size_t)t], 36);
                    memcpy(a[3] + 6 * (size_t)t, &UV[3 * (size_t)t], 24);
                }
            if (f > 0) copy += ms_since(t1);
            // the same copy into pageable heap memory (transparent huge pages)
            t1 = clk::now();
            if (h[0] && h[1] && h[2] && h[3])
                for (u32 t = 0; t < T; ++t) {
                    memcpy(h[0] + 9 * (size_t)t, &V[3 * (size_t)t], 36);
                    memcpy(h[1] + 12 * (size_t)t, &C[3 * (size_t)t], 48);
                    memcpy(h[2] + 9 * (size_t)t, &N[3 * (size_t)t], 36);
                    memcpy(h[3] + 6 * (size_t)t, &UV[3 * (size_t)t], 24);
                }
            if (f > 0) copy_heap += ms_since(t1);
#if PRK_EC_SSE
            // ... and into pinned memory with streaming stores, four triangles
            // (whole 16-byte blocks of every array) at a time
            t1 = clk::now();
            if (a[0] && a[1] && a[2] && a[3]) {
                const float *src[4] = {(const float *)V.data(), (const float *)C.data(), (const float *)N.data(),
                                       (const float *)UV.data()};
                for (u32 t = 0; t + 4 <= T; t += 4)
                    for (int k = 0; k < 4; ++k) {
                        const size_t w = 3 * comp[k];  // floats per triangle
                        const float *sp = src[k] + w * t;
                        float *dp = a[k] + w * t;
                        for (size_t q = 0; q < w; ++q) _mm_stream_ps(dp + 4 * q, _mm_loadu_ps(sp + 4 * q));
                    }
                _mm_sfence();
            }
            if (f > 0) copy_nt += ms_since(t1);
#endif
        }
        for (int k = 0; k < 4; ++k) prk_host_free(prk_dropin::S().Ctx, a[k]);
        for (int k = 0; k < 4; ++k) std::free(h[k]);
        if (sink == 1) std::printf(" ");
    }
    std::printf("}, \"fill_edge_table_pass_ms\": %.3f, \"draw_model_pass_ms\": %.3f, \"fill_edge_table_only_ms\": %.3f, "
                "\"edge_count_only_ms\": %.3f, \"edge_count_inline_ms\": %.3f, \"snapshot_copy_only_ms\": %.3f, "
                "\"snapshot_copy_heap_ms\": %.3f, \"snapshot_copy_stream_ms\": %.3f, \"frames\": %d}\n",
                fill_pass / frames, draw_pass / frames, fill / frames, count / frames, count_inline / frames,
                copy / frames, copy_heap / frames, copy_nt / frames, frames);
    PRK_Shutdown();
    return 0;
}
