// projekt.h — drop-in replacement for the reference's draw path
// (MacSpain/cpu-renderer projekt.h + the hot-path entry points of projekt.cpp),
// implemented header-only over the C-ABI of libprk_hip.so (prk.h).
//
// A caller of the reference keeps its code:
//
//     u32 EdgeCount = FillEdgeTable(Object, Commands, Phong);          // projekt.cpp:3882
//     DrawModelOptimized(RenderQueue, Buffer, (edge_info *)Object->EdgeMemory,
//                        EdgeCount, Commands, Bitmap, Phong);          // projekt.cpp:3615
//     ... or DrawModel(Buffer, Edges, EdgeCount, Commands, Bitmap, Phong);   // 162
//     Platform.CompleteAllWork(RenderQueue)  ->  PRK_CompleteAllWork(Buffer, Commands)
//
// and links libprk_hip.so.  Differences from the reference, all deliberate:
//  * FillEdgeTable does not build a CPU edge list: it registers the object
//    (geometry is uploaded to HBM once per VertexData pointer) and leaves a
//    token in Object->EdgeMemory that DrawModel* reads back.  It returns the
//    reference's upper bound 3*T (a non-zero EdgeCount).
//  * Every triangle is its own active edge table ("per-triangle
//    submission").  For objects of one triangle this is exactly
//    the reference; for multi-triangle objects the reference pairs edges of
//    different triangles into one AET, which DESIGN.md §2 lists as not yet
//    emulated.
//  * Work runs on the GPU at PRK_CompleteAllWork (the reference's
//    CompleteAllWork point), which downloads colour and z into Buffer->Memory
//    and Commands->ZBuffer.  The prior contents of both are uploaded at the
//    first draw of a frame, so draws still z-test against them.
//  * Inputs the reference crashes on are rejected or pinned, see
//    prk.h.
//
// The caller-owned types of the reference live in its absent platform and
// math headers.  If the caller has them, define PRK_CALLER_TYPES before
// including this file; otherwise minimal definitions with the fields the
// reference uses are provided here.
#ifndef PRK_PROJEKT_H
#define PRK_PROJEKT_H

#include <stdint.h>
#include <string.h>

#include <map>
#include <utility>

#include "prk.h"

#ifndef PRK_CALLER_TYPES
typedef float r32;
typedef int32_t s32;
typedef uint32_t u32;
typedef int32_t b32;
typedef uint8_t u8;
union v2 { struct { r32 x, y; }; struct { r32 u, v; }; r32 E[2]; };
union v3 { struct { r32 x, y, z; }; r32 E[3]; };
union v4 { struct { r32 r, g, b, a; }; struct { r32 x, y, z, w; }; r32 E[4]; };

struct loaded_bitmap {       // fields as used at projekt.cpp:1506, 1837-1847, 1881-1935
    void *Memory;
    s32 Width;
    s32 Height;
    s32 Pitch;
};
struct projective_transform { // projekt.cpp:77-90, 122-141
    r32 DistanceAboveTarget;
    r32 FocalLength;
    r32 MetersToPixels;
    v2 ScreenCenter;
};
struct light_info { v3 P; v4 Intensity; };
struct light_data {
    light_info Lights[PRK_MAX_LIGHTS];
    u32 LightCount;
    v4 AmbientIntensity;
};
struct game_render_commands { // fields as used at projekt.cpp:170-171, 452-458, 1509-1511, 2211, 3756
    r32 *ZBuffer;
    u8 *ZMask;
    u32 Width;
    void *ThreadMemory;
    u32 ThreadMemorySize;
    u32 ThreadMemorySizeUsed;
    void *SortMemory;
    light_data LightData;
    projective_transform Transform;
};
struct platform_work_queue;
#endif  // PRK_CALLER_TYPES

// The reference's own structs (projekt.h:2-37), field for field.
struct render_entry_3d_object {
    v3 P;
    u32 VertexCount;
    b32 Optimized;
    b32 PhongShading;
    void *VertexData;   // v3[VertexCount]
    void *ColorData;    // v4[VertexCount]
    void *NormalData;   // v3[VertexCount]
    void *UVData;       // v2[VertexCount]
    void *EdgeMemory;   // >= 3*T edge_info (reference contract); receives a token here
    loaded_bitmap *Bitmap;
};

struct edge_info {
    s32 YMax;
    r32 XMin, ZMin, OneOverZMin, Gradient, ZGradient, OneOverZGradient;
    s32 YMin;
    r32 UMin, VMin, UGradient, VGradient;
    b32 Left;
    v4 MinColor, ColorGradient;
    v3 MinNormal, NormalGradient;
    edge_info *Next;
};

namespace prk_dropin {

// Token FillEdgeTable leaves in Object->EdgeMemory for DrawModel*.
struct object_token {
    uint32_t Magic;
    int32_t Geometry;
    uint32_t TriCount;
    int32_t Phong;
    float P[3];
    int32_t Texture;
};
static_assert(sizeof(object_token) <= sizeof(edge_info), "token must fit one edge_info");
static const uint32_t kMagic = 0x4B525031u;  // "PRK1"

struct state {
    prk_context *Ctx = nullptr;
    int LastStatus = PRK_OK;
    std::map<const void *, std::pair<int32_t, uint32_t>> Geometry;  // VertexData -> (handle, vertices)
    std::map<const void *, int32_t> Textures;                       // Bitmap->Memory -> handle
    loaded_bitmap *Target = nullptr;
    game_render_commands *Commands = nullptr;
    bool FrameOpen = false;
};
inline state &S() {
    static state s;
    return s;
}

inline int32_t texture_for(loaded_bitmap *Bitmap) {
    if (!Bitmap || !Bitmap->Memory) return -1;
    state &st = S();
    auto it = st.Textures.find(Bitmap->Memory);
    if (it != st.Textures.end()) return it->second;
    prk_bitmap b = {Bitmap->Memory, Bitmap->Width, Bitmap->Height, Bitmap->Pitch};
    int32_t h = -1;
    st.LastStatus = prk_texture_create(st.Ctx, &b, &h);  // needs the zeroed guard row (prk.h)
    if (st.LastStatus == PRK_OK) st.Textures[Bitmap->Memory] = h;
    return h;
}

inline void set_camera(game_render_commands *Commands) {
    prk_transform t;
    t.DistanceAboveTarget = Commands->Transform.DistanceAboveTarget;
    t.FocalLength = Commands->Transform.FocalLength;
    t.MetersToPixels = Commands->Transform.MetersToPixels;
    t.ScreenCenter[0] = Commands->Transform.ScreenCenter.x;
    t.ScreenCenter[1] = Commands->Transform.ScreenCenter.y;
    prk_light_data l;
    memset(&l, 0, sizeof l);
    l.LightCount = Commands->LightData.LightCount;
    for (int c = 0; c < 4; ++c) l.AmbientIntensity[c] = Commands->LightData.AmbientIntensity.E[c];
    for (u32 i = 0; i < l.LightCount && i < PRK_MAX_LIGHTS; ++i) {
        for (int c = 0; c < 3; ++c) l.Lights[i].P[c] = Commands->LightData.Lights[i].P.E[c];
        for (int c = 0; c < 4; ++c) l.Lights[i].Intensity[c] = Commands->LightData.Lights[i].Intensity.E[c];
    }
    S().LastStatus = prk_set_camera(S().Ctx, &t, &l);
}

// First draw of a frame: bind a device target of the Buffer's size and upload
// the caller's current colour and z (draws z-test against them).
inline bool open_frame(loaded_bitmap *Buffer, game_render_commands *Commands) {
    state &st = S();
    if (st.FrameOpen && st.Target == Buffer && st.Commands == Commands) return true;
    st.LastStatus = prk_target_alloc(st.Ctx, Buffer->Width, Buffer->Height, 0, Buffer->Height, nullptr, nullptr);
    if (st.LastStatus != PRK_OK) return false;
    st.LastStatus = prk_target_upload(st.Ctx, (const uint32_t *)Buffer->Memory, Buffer->Pitch, Commands->ZBuffer);
    if (st.LastStatus != PRK_OK) return false;
    st.Target = Buffer;
    st.Commands = Commands;
    st.FrameOpen = true;
    return true;
}

inline void draw(loaded_bitmap *Buffer, edge_info *Edges, u32 EdgeCount, game_render_commands *Commands,
                 loaded_bitmap *Bitmap, b32 PhongShading, int32_t semantics) {
    state &st = S();
    if (!st.Ctx || !Edges || EdgeCount == 0) return;  // 0 edges: nothing to draw (P1)
    object_token tok;
    memcpy(&tok, Edges, sizeof tok);
    if (tok.Magic != kMagic) { st.LastStatus = PRK_ERR_ARG; return; }
    if (!open_frame(Buffer, Commands)) return;
    set_camera(Commands);
    int32_t tex = Bitmap ? texture_for(Bitmap) : -1;
    st.LastStatus = prk_draw(st.Ctx, tok.Geometry, 0, tok.TriCount, tok.P, semantics, PhongShading ? 1 : 0, tex);
}

}  // namespace prk_dropin

// ---- platform hooks --------------------------------------------------------
inline int PRK_Init(int device) {
    prk_dropin::state &st = prk_dropin::S();
    if (st.Ctx) return PRK_OK;
    st.LastStatus = prk_create(device, &st.Ctx);
    return st.LastStatus;
}
inline int PRK_LastStatus() { return prk_dropin::S().LastStatus; }
inline void PRK_Shutdown() {
    prk_dropin::state &st = prk_dropin::S();
    if (st.Ctx) prk_destroy(st.Ctx);
    st = prk_dropin::state();
}
// Platform.CompleteAllWork equivalent: run the frame, copy colour and z back.
inline int PRK_CompleteAllWork(loaded_bitmap *Buffer, game_render_commands *Commands) {
    prk_dropin::state &st = prk_dropin::S();
    if (!st.Ctx || !st.FrameOpen) return PRK_OK;
    int rc = prk_flush(st.Ctx, nullptr);
    if (rc == PRK_OK)
        rc = prk_target_download(st.Ctx, (uint32_t *)Buffer->Memory, Buffer->Pitch, Commands->ZBuffer);
    st.FrameOpen = false;
    st.LastStatus = rc;
    return rc;
}

// ---- the reference's entry points ------------------------------------------
// projekt.cpp:3882-4121
inline u32 FillEdgeTable(render_entry_3d_object *Object, game_render_commands *Commands, b32 PhongShading = 0) {
    (void)Commands;
    prk_dropin::state &st = prk_dropin::S();
    if (!st.Ctx || !Object || !Object->EdgeMemory || Object->VertexCount < 3) return 0;
    const u32 T = Object->VertexCount / 3;
    auto it = st.Geometry.find(Object->VertexData);
    int32_t g = -1;
    if (it != st.Geometry.end() && it->second.second == Object->VertexCount) {
        g = it->second.first;
    } else {
        st.LastStatus = prk_geometry_create(st.Ctx, (const float *)Object->VertexData,
                                            (const float *)Object->ColorData, (const float *)Object->NormalData,
                                            (const float *)Object->UVData, T * 3, &g);
        if (st.LastStatus != PRK_OK) return 0;
        st.Geometry[Object->VertexData] = std::make_pair(g, Object->VertexCount);
    }
    prk_dropin::object_token tok;
    tok.Magic = prk_dropin::kMagic;
    tok.Geometry = g;
    tok.TriCount = T;
    tok.Phong = PhongShading ? 1 : 0;
    tok.P[0] = Object->P.x;
    tok.P[1] = Object->P.y;
    tok.P[2] = Object->P.z;
    tok.Texture = -1;
    memcpy(Object->EdgeMemory, &tok, sizeof tok);
    return 3 * T;
}

// projekt.cpp:3615-3871 (+ FillLineOptimized 1492-2320)
inline void DrawModelOptimized(platform_work_queue *RenderQueue, loaded_bitmap *Buffer, edge_info *Edges,
                               u32 EdgeCount, game_render_commands *Commands, loaded_bitmap *Bitmap = 0,
                               b32 PhongShading = 0) {
    (void)RenderQueue;
    prk_dropin::draw(Buffer, Edges, EdgeCount, Commands, Bitmap, PhongShading, PRK_SEM_AVX);
}

// projekt.cpp:162-601
inline void DrawModel(loaded_bitmap *Buffer, edge_info *Edges, u32 EdgeCount, game_render_commands *Commands,
                      loaded_bitmap *Bitmap = 0, b32 PhongShading = 0) {
    prk_dropin::draw(Buffer, Edges, EdgeCount, Commands, Bitmap, PhongShading, PRK_SEM_SCALAR);
}

// The reference's test mesh (projekt.cpp:4123-4289).
inline u32 ConstructSphere(v3 *Vertices, v4 *Colors, v3 *Normals, v2 *UVs) {
    uint32_t n = 0;
    prk_construct_sphere((float *)Vertices, (float *)Colors, (float *)Normals, (float *)UVs, &n);
    return n;
}

#endif  // PRK_PROJEKT_H
