// dropin_demo.cpp — a reference-style caller of the drop-in projekt.h.
//
// It does what the absent game layer of MacSpain/cpu-renderer does: fills a
// game_render_commands, builds the ConstructSphere mesh, submits it through
// the reference's own entry points, completes the work and writes the
// framebuffer and z-buffer as raw files.  Modes (argv[3]):
//   queue    every triangle its own render_entry_3d_object, FillEdgeTable +
//            DrawModelOptimized(RenderQueue, ...)           (projekt.cpp:3615)
//   lines    the same through DrawModelOptimizedLines             (3362)
//   st       the same through DrawModelOptimized(Buffer, ...)     (2350)
//   scalar   the same through DrawModel, untextured Gouraud       (162); the
//            objects carry the Bitmap, so FillEdgeTable(..., 0) lights them
//            from white (4034-4054)
//   vertexlit  the same with no Bitmap on the objects: lit vertex colours
//   interp   FillEdgeTable(..., 1) + DrawModel(..., Bitmap = 0, Phong = 0):
//            the raw vertex colours interpolated unlit (4012-4019)
//   object   the whole sphere as ONE object (one active edge table)
//   scalar_object / scalar_object_phong   the whole sphere as ONE object
//            through DrawModel (untextured Gouraud / Phong)
//   interp_object  the whole sphere as ONE object, FillEdgeTable(..., 1) +
//            DrawModel(..., 0, 0)
//   camera   per-triangle objects; halfway through, the caller moves the
//            camera (ScreenCenter) and changes the light between FillEdgeTable
//            calls: each object draws as its FillEdgeTable call saw them
//   split_st / split_queue   per-triangle objects; every FillEdgeTable runs
//            under camera and lights A, then the caller switches Commands to B
//            and draws through the single-thread overload / the queue overload,
//            then back to A: set up under A (3885-4063), shaded under B
//            (3030-3034 / 2042-2046)
//   split_object  the sphere as ONE object, FillEdgeTable(..., 1) under A,
//            DrawModel(..., Bitmap = 0, Phong = 1) under B (452-458)
//   mutate   two frames; between them the vertices, normals and texture are
//            rewritten in place (same pointers): frame 2 is written
//   edges F  DrawModelOptimized on a ready edge_info list read from file F
//            (prk_edge words), i.e. edges the caller built itself
//   work F   the work-queue callbacks: DoLineRenderWork on the first half of
//            the spans of file F (prk_span words), DoBufferLineRenderWork on
//            the rest (one record per row), then DoModelRenderWork on the
//            sphere as one object
//   records F  record mode (PRK_SetEdgeRecords): the sphere as ONE object,
//            FillEdgeTable(..., 1) writes edge_info records into EdgeMemory
//            (dumped to F.fill), DrawModelOptimized(RenderQueue, ...) draws them
//            and leaves them advanced (dumped to F.adv); dumps are 27 words +
//            the Next index (-1: NULL) per edge
//   records_scalar F  the same with FillEdgeTable(..., 0) (Gouraud, white lit:
//            the objects carry the Bitmap) and DrawModel(..., 0, 0)
//   records_queue  record mode, per-triangle objects through
//            DrawModelOptimized(RenderQueue, ...)
// The texture is a loaded_bitmap of exactly Height rows whose last byte is
// followed by an inaccessible page: a read past it faults.
//
// usage: [PRK_DEMO_BANDS=n] dropin_demo <out_color.u32> <out_z.f32> [mode [file]]
// exit: 0 ok, 1 usage, 2 no GPU / library error
#include <sys/mman.h>
#include <unistd.h>

#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "projekt.h"

// EdgeMemory[0, n) as 27 words + the Next index per edge.
static bool dump_edges(const std::string &path, const edge_info *E, u32 n) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    for (u32 i = 0; i < n; ++i) {
        std::fwrite(&E[i], 4, 27, f);
        const int32_t nx = E[i].Next ? (int32_t)(E[i].Next - E) : -1;
        std::fwrite(&nx, 4, 1, f);
    }
    std::fclose(f);
    return true;
}

static std::vector<uint32_t> read_words(const char *path) {
    std::vector<uint32_t> w;
    FILE *f = std::fopen(path, "rb");
    if (!f) return w;
    uint32_t x;
    while (std::fread(&x, 4, 1, f) == 1) w.push_back(x);
    std::fclose(f);
    return w;
}

// Texels ending exactly at a PROT_NONE page (prk_texture_create must read
// Height rows of Pitch bytes and nothing past them).
static u32 *guarded_texels(size_t bytes) {
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    const size_t span = (bytes + page - 1) / page * page;
    uint8_t *base = (uint8_t *)mmap(nullptr, span + page, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (base == MAP_FAILED) return nullptr;
    if (mprotect(base + span, page, PROT_NONE) != 0) return nullptr;
    return (u32 *)(base + span - bytes);
}

static void fill_texture(u32 *t, int salt) {
    for (int y = 0; y < 64; ++y)
        for (int x = 0; x < 64; ++x)
            t[y * 64 + x] = (((x ^ y) & 8) ? 0xFFE0C080u : 0xFF4060A0u) ^ (u32)(salt * 0x00102030);
}

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s out_color.u32 out_z.f32 [mode [file]]\n", argv[0]);
        return 1;
    }
    const std::string mode = argc > 3 ? argv[3] : "queue";
    // PRK_DEMO_BANDS=n: the frame split into n row bands, one context each,
    // on the visible GPUs round robin (several bands may share one GPU).
    const char *nb = std::getenv("PRK_DEMO_BANDS");
    const int bands = nb ? std::atoi(nb) : 1;
    int ndev = 0;
    prk_device_count(&ndev);
    std::vector<int> devs(bands > 0 ? bands : 1);
    for (size_t r = 0; r < devs.size(); ++r) devs[r] = ndev > 0 ? (int)r % ndev : 0;
    if (PRK_InitDevices(devs.data(), (int)devs.size()) != PRK_OK) {
        std::fprintf(stderr, "dropin_demo: no HIP device (status %d)\n", PRK_LastStatus());
        return 2;
    }
    const s32 W = 256, H = 256;
    std::vector<u32> pixels(W * H, 0xFF000000u);
    std::vector<r32> zbuf(W * H, -FLT_MAX);
    loaded_bitmap Buffer = {pixels.data(), W, H, W * 4};

    u32 *texels = guarded_texels(64 * 64 * 4);
    if (!texels) return 1;
    fill_texture(texels, 0);
    loaded_bitmap Texture = {texels, 64, 64, 64 * 4};

    game_render_commands Commands = {};
    Commands.ZBuffer = zbuf.data();
    Commands.Width = W;
    Commands.Transform.DistanceAboveTarget = 4.0f;
    Commands.Transform.FocalLength = 1.0f;
    Commands.Transform.MetersToPixels = W / 2.0f;
    Commands.Transform.ScreenCenter.x = W / 2.0f;
    Commands.Transform.ScreenCenter.y = H / 2.0f;
    Commands.LightData.LightCount = 1;
    Commands.LightData.Lights[0].P = {{1.0f, 1.0f, 3.0f}};
    Commands.LightData.Lights[0].Intensity = {{0.8f, 0.8f, 0.8f, 1.0f}};
    Commands.LightData.AmbientIntensity = {{0.2f, 0.2f, 0.2f, 1.0f}};

    std::vector<v3> V(6624), N(6624);
    std::vector<v4> C(6624);
    std::vector<v2> UV(6624);
    const u32 VertexCount = ConstructSphere(V.data(), C.data(), N.data(), UV.data());
    std::vector<edge_info> EdgeMemory(3 * (VertexCount / 3));

    auto fail = [](const char *what) {
        std::fprintf(stderr, "dropin_demo: %s failed (status %d)\n", what, PRK_LastStatus());
        return 2;
    };
    // Camera and lights B of the split modes (A is the above).
    auto to_b = [&]() {
        Commands.Transform.DistanceAboveTarget = 4.5f;
        Commands.Transform.ScreenCenter.x = W / 2.0f + 24.0f;
        Commands.LightData.Lights[0].P = {{-1.0f, 2.0f, 2.5f}};
        Commands.LightData.Lights[0].Intensity = {{0.3f, 0.9f, 0.5f, 1.0f}};
        Commands.LightData.AmbientIntensity = {{0.1f, 0.15f, 0.3f, 1.0f}};
    };
    auto to_a = [&]() {
        Commands.Transform.DistanceAboveTarget = 4.0f;
        Commands.Transform.ScreenCenter.x = W / 2.0f;
        Commands.LightData.Lights[0].P = {{1.0f, 1.0f, 3.0f}};
        Commands.LightData.Lights[0].Intensity = {{0.8f, 0.8f, 0.8f, 1.0f}};
        Commands.LightData.AmbientIntensity = {{0.2f, 0.2f, 0.2f, 1.0f}};
    };
    // One frame of per-triangle objects through the chosen entry point.
    unsigned long long edges_total = 0;  // sum of FillEdgeTable's return values
    auto per_triangle = [&](const std::string &m) {
        for (u32 t = 0; t < VertexCount / 3; ++t) {
            if (m == "camera" && t == VertexCount / 6) {  // the caller changes camera and light mid-frame
                Commands.Transform.ScreenCenter.x = W / 2.0f + 24.0f;
                Commands.LightData.Lights[0].Intensity = {{0.3f, 0.9f, 0.5f, 1.0f}};
            }
            render_entry_3d_object Object = {};
            Object.P = {{0.0f, 0.0f, 2.0f}};
            Object.VertexCount = 3;
            Object.PhongShading = 1;
            Object.VertexData = &V[3 * t];
            Object.ColorData = &C[3 * t];
            Object.NormalData = &N[3 * t];
            Object.UVData = &UV[3 * t];
            Object.EdgeMemory = EdgeMemory.data();
            Object.Bitmap = m == "vertexlit" ? nullptr : &Texture;
            const bool scalar = m == "scalar" || m == "vertexlit" || m == "interp";
            const u32 EdgeCount = FillEdgeTable(&Object, &Commands, !scalar || m == "interp");
            edges_total += EdgeCount;
            if (m == "split_st" || m == "split_queue") {  // the draw under B, the next setup under A
                to_b();
                if (m == "split_st") DrawModelOptimized(&Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
                else DrawModelOptimized(nullptr, &Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
                to_a();
            } else if (scalar) DrawModel(&Buffer, EdgeMemory.data(), EdgeCount, &Commands, 0, 0);
            else if (m == "lines") DrawModelOptimizedLines(nullptr, &Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
            else if (m == "st") DrawModelOptimized(&Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
            else DrawModelOptimized(nullptr, &Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
            if (PRK_LastStatus() != PRK_OK) return false;
        }
        return true;
    };
    render_entry_3d_object Sphere = {};
    Sphere.P = {{0.0f, 0.0f, 2.0f}};
    Sphere.VertexCount = VertexCount;
    Sphere.PhongShading = 1;
    Sphere.VertexData = V.data();
    Sphere.ColorData = C.data();
    Sphere.NormalData = N.data();
    Sphere.UVData = UV.data();
    Sphere.EdgeMemory = EdgeMemory.data();
    Sphere.Bitmap = &Texture;

    if (mode == "queue" || mode == "lines" || mode == "st" || mode == "scalar" || mode == "camera" ||
        mode == "vertexlit" || mode == "interp" || mode == "split_st" || mode == "split_queue") {
        if (!per_triangle(mode)) return fail("draw");
    } else if (mode == "records_queue") {
        PRK_SetEdgeRecords(1);
        if (!per_triangle("queue")) return fail("draw");
    } else if ((mode == "records" || mode == "records_scalar") && argc > 4) {
        PRK_SetEdgeRecords(1);
        std::vector<edge_info> SortMemory(EdgeMemory.size());
        Commands.SortMemory = SortMemory.data();  // MergeSort's scratch (4117)
        const bool scalar = mode == "records_scalar";
        const u32 EdgeCount = FillEdgeTable(&Sphere, &Commands, scalar ? 0 : 1);
        edges_total += EdgeCount;
        if (PRK_LastStatus() != PRK_OK || !dump_edges(std::string(argv[4]) + ".fill", EdgeMemory.data(), EdgeCount))
            return fail("FillEdgeTable");
        if (scalar) DrawModel(&Buffer, EdgeMemory.data(), EdgeCount, &Commands, 0, 0);
        else DrawModelOptimized(nullptr, &Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
        if (PRK_LastStatus() != PRK_OK || !dump_edges(std::string(argv[4]) + ".adv", EdgeMemory.data(), EdgeCount))
            return fail("draw");
        Commands.SortMemory = nullptr;
    } else if (mode == "split_object") {
        const u32 EdgeCount = FillEdgeTable(&Sphere, &Commands, 1);
        edges_total += EdgeCount;
        to_b();
        DrawModel(&Buffer, EdgeMemory.data(), EdgeCount, &Commands, 0, 1);
        if (PRK_LastStatus() != PRK_OK) return fail("draw");
    } else if (mode == "scalar_object" || mode == "scalar_object_phong" || mode == "interp_object") {
        const b32 Phong = mode == "scalar_object_phong";
        const u32 EdgeCount = FillEdgeTable(&Sphere, &Commands, Phong || mode == "interp_object");
        edges_total += EdgeCount;
        DrawModel(&Buffer, EdgeMemory.data(), EdgeCount, &Commands, 0, Phong);
        if (PRK_LastStatus() != PRK_OK) return fail("draw");
    } else if (mode == "object") {
        const u32 EdgeCount = FillEdgeTable(&Sphere, &Commands, 1);
        DrawModelOptimized(nullptr, &Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
        if (PRK_LastStatus() != PRK_OK) return fail("draw");
    } else if (mode == "mutate") {
        if (!per_triangle("queue")) return fail("draw");
        if (PRK_CompleteAllWork(&Buffer, &Commands) != PRK_OK) return fail("CompleteAllWork 1");
        // the same buffers, new contents: the next frame must see them
        for (u32 i = 0; i < VertexCount; ++i) {
            V[i].x = V[i].x * 0.75f + 0.125f;
            V[i].y = V[i].y * 1.25f - 0.0625f;
            N[i].z = -N[i].z;
        }
        fill_texture(texels, 1);
        std::fill(pixels.begin(), pixels.end(), 0xFF000000u);
        std::fill(zbuf.begin(), zbuf.end(), -FLT_MAX);
        if (!per_triangle("queue")) return fail("draw");
    } else if (mode == "edges" && argc > 4) {
        std::vector<uint32_t> w = read_words(argv[4]);
        const u32 n = (u32)(w.size() / 27);
        std::vector<edge_info> E(n);
        for (u32 i = 0; i < n; ++i) {  // prk_edge words -> edge_info
            const uint32_t *r = &w[27 * i];
            edge_info &e = E[i];
            std::memcpy(&e.YMax, r + 0, 4); std::memcpy(&e.XMin, r + 1, 4); std::memcpy(&e.ZMin, r + 2, 4);
            std::memcpy(&e.OneOverZMin, r + 3, 4); std::memcpy(&e.Gradient, r + 4, 4);
            std::memcpy(&e.ZGradient, r + 5, 4); std::memcpy(&e.OneOverZGradient, r + 6, 4);
            std::memcpy(&e.YMin, r + 7, 4); std::memcpy(&e.UMin, r + 8, 4); std::memcpy(&e.VMin, r + 9, 4);
            std::memcpy(&e.UGradient, r + 10, 4); std::memcpy(&e.VGradient, r + 11, 4);
            std::memcpy(&e.Left, r + 12, 4); std::memcpy(e.MinColor.E, r + 13, 16);
            std::memcpy(e.ColorGradient.E, r + 17, 16); std::memcpy(e.MinNormal.E, r + 21, 12);
            std::memcpy(e.NormalGradient.E, r + 24, 12);
            e.Next = nullptr;
        }
        DrawModelOptimized(nullptr, &Buffer, E.data(), n, &Commands, &Texture, 1);
        if (PRK_LastStatus() != PRK_OK) return fail("draw");
    } else if (mode == "work" && argc > 4) {
        std::vector<uint32_t> w = read_words(argv[4]);
        const u32 n = (u32)(w.size() / 25);
        auto end_of = [&](u32 k, int side, edge_info &e) {
            std::memset(&e, 0, sizeof e);
            const uint32_t *r = &w[25 * k + 12 * side];
            std::memcpy(&e.XMin, r + 0, 4); std::memcpy(&e.ZMin, r + 1, 4); std::memcpy(&e.OneOverZMin, r + 2, 4);
            std::memcpy(&e.UMin, r + 3, 4); std::memcpy(&e.VMin, r + 4, 4);
            std::memcpy(e.MinColor.E, r + 5, 16); std::memcpy(e.MinNormal.E, r + 9, 12);
        };
        const u32 half = n / 2;
        for (u32 k = 0; k < half; ++k) {  // one span per record (3756-3809)
            line_render_work Work = {};
            Work.Commands = &Commands;
            Work.OutputTarget = &Buffer;
            Work.Bitmap = &Texture;
            end_of(k, 0, Work.CurrentEdgeInList);
            end_of(k, 1, Work.NextEdgeInList);
            Work.RowIndex = (s32)w[25 * k + 24];
            Work.PhongShading = 1;
            DoLineRenderWork(nullptr, &Work);
            if (PRK_LastStatus() != PRK_OK) return fail("DoLineRenderWork");
        }
        // buffer_line_render_work: consecutive spans of one row share a record
        for (u32 k = half; k < n;) {
            u32 e = k;
            while (e < n && w[25 * e + 24] == w[25 * k + 24]) ++e;
            std::vector<uint8_t> mem(sizeof(buffer_line_render_work) + (e - k) * sizeof(thread_edge_info));
            buffer_line_render_work *Work = (buffer_line_render_work *)mem.data();
            Work->Commands = &Commands;
            Work->OutputTarget = &Buffer;
            Work->Bitmap = &Texture;
            Work->RowIndex = (s32)w[25 * k + 24];
            Work->PhongShading = 1;
            Work->EdgeCount = e - k;
            thread_edge_info *T = &Work->Edges;
            for (u32 j = k; j < e; ++j) {
                edge_info L, R;
                end_of(j, 0, L);
                end_of(j, 1, R);
                thread_edge_info &t = T[j - k];
                t.LeftXMin = L.XMin; t.RightXMin = R.XMin; t.LeftZMin = L.ZMin; t.RightZMin = R.ZMin;
                t.LeftOneOverZMin = L.OneOverZMin; t.RightOneOverZMin = R.OneOverZMin;
                t.LeftUMin = L.UMin; t.RightUMin = R.UMin; t.LeftVMin = L.VMin; t.RightVMin = R.VMin;
                t.LeftMinColor = L.MinColor; t.RightMinColor = R.MinColor;
                t.LeftMinNormal = L.MinNormal; t.RightMinNormal = R.MinNormal;
            }
            DoBufferLineRenderWork(nullptr, Work);
            if (PRK_LastStatus() != PRK_OK) return fail("DoBufferLineRenderWork");
            k = e;
        }
        model_render_work M = {};  // the whole sphere, single-thread overload (3873-3878)
        M.Commands = &Commands;
        M.OutputTarget = &Buffer;
        M.Bitmap = &Texture;
        M.EdgeMemory = EdgeMemory.data();
        M.EdgeCount = FillEdgeTable(&Sphere, &Commands, 1);
        M.PhongShading = 1;
        DoModelRenderWork(nullptr, &M);
        if (PRK_LastStatus() != PRK_OK) return fail("DoModelRenderWork");
    } else {
        std::fprintf(stderr, "dropin_demo: unknown mode %s\n", mode.c_str());
        return 1;
    }
    if (PRK_CompleteAllWork(&Buffer, &Commands) != PRK_OK) return fail("CompleteAllWork");
    FILE *f = std::fopen(argv[1], "wb");
    FILE *g = std::fopen(argv[2], "wb");
    if (!f || !g) return 1;
    std::fwrite(pixels.data(), 4, pixels.size(), f);
    std::fwrite(zbuf.data(), 4, zbuf.size(), g);
    std::fclose(f);
    std::fclose(g);
    PRK_Shutdown();
    std::printf("dropin_demo: %u triangles, mode %s, edges=%llu\n", VertexCount / 3, mode.c_str(), edges_total);
    return 0;
}
