// dropin_demo.cpp — a reference-style caller of the drop-in projekt.h.
//
// It does what the absent game layer of MacSpain/cpu-renderer does: fills a
// game_render_commands, builds the ConstructSphere mesh, submits every
// triangle as its own render_entry_3d_object through FillEdgeTable +
// DrawModelOptimized (or DrawModel), completes the work and writes the
// framebuffer and z-buffer as raw files.
//
// usage: dropin_demo <out_color.u32> <out_z.f32> [scalar]
// exit: 0 ok, 2 no GPU / library error
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "projekt.h"

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s out_color.u32 out_z.f32 [scalar]\n", argv[0]);
        return 1;
    }
    const bool scalar = argc > 3;
    if (PRK_Init(0) != PRK_OK) {
        std::fprintf(stderr, "dropin_demo: no HIP device (status %d)\n", PRK_LastStatus());
        return 2;
    }
    const s32 W = 256, H = 256;
    std::vector<u32> pixels(W * H, 0xFF000000u);
    std::vector<r32> zbuf(W * H, -FLT_MAX);
    loaded_bitmap Buffer = {pixels.data(), W, H, W * 4};

    // 64x64 checker texture with its zeroed guard row (prk.h).
    std::vector<u32> texels(64 * 65, 0u);
    for (int y = 0; y < 64; ++y)
        for (int x = 0; x < 64; ++x) texels[y * 64 + x] = ((x ^ y) & 8) ? 0xFFE0C080u : 0xFF4060A0u;
    loaded_bitmap Texture = {texels.data(), 64, 64, 64 * 4};

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
    std::vector<edge_info> EdgeMemory(3);

    for (u32 t = 0; t < VertexCount / 3; ++t) {
        render_entry_3d_object Object = {};
        Object.P = {{0.0f, 0.0f, 2.0f}};
        Object.VertexCount = 3;
        Object.PhongShading = 1;
        Object.VertexData = &V[3 * t];
        Object.ColorData = &C[3 * t];
        Object.NormalData = &N[3 * t];
        Object.UVData = &UV[3 * t];
        Object.EdgeMemory = EdgeMemory.data();
        Object.Bitmap = &Texture;
        const u32 EdgeCount = FillEdgeTable(&Object, &Commands, 1);
        if (scalar)
            DrawModel(&Buffer, EdgeMemory.data(), EdgeCount, &Commands, 0, 0);
        else
            DrawModelOptimized(nullptr, &Buffer, EdgeMemory.data(), EdgeCount, &Commands, &Texture, 1);
        if (PRK_LastStatus() != PRK_OK) {
            std::fprintf(stderr, "dropin_demo: draw failed (status %d)\n", PRK_LastStatus());
            return 2;
        }
    }
    if (PRK_CompleteAllWork(&Buffer, &Commands) != PRK_OK) {
        std::fprintf(stderr, "dropin_demo: CompleteAllWork failed (status %d)\n", PRK_LastStatus());
        return 2;
    }
    FILE *f = std::fopen(argv[1], "wb");
    FILE *g = std::fopen(argv[2], "wb");
    if (!f || !g) return 1;
    std::fwrite(pixels.data(), 4, pixels.size(), f);
    std::fwrite(zbuf.data(), 4, zbuf.size(), g);
    std::fclose(f);
    std::fclose(g);
    PRK_Shutdown();
    std::printf("dropin_demo: %u triangles, %s semantics\n", VertexCount / 3, scalar ? "DrawModel" : "FillLineOptimized");
    return 0;
}
