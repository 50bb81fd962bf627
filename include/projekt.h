// projekt.h — drop-in replacement for the reference's draw path
// (MacSpain/cpu-renderer projekt.h + the hot-path entry points of projekt.cpp),
// implemented header-only over the C-ABI of libprk_hip.so (prk.h).
//
// A caller of the reference keeps its code:
//
//     u32 EdgeCount = FillEdgeTable(Object, Commands, Phong);                  // projekt.cpp:3882
//     DrawModelOptimized(RenderQueue, Buffer, (edge_info *)Object->EdgeMemory,
//                        EdgeCount, Commands, Bitmap, Phong);                  // 3615
//     ... or DrawModelOptimizedLines(RenderQueue, Buffer, Edges, ...)         // 3362
//     ... or DrawModelOptimized(Buffer, Edges, EdgeCount, Commands, ...)      // 2350 (single thread)
//     ... or DrawModel(Buffer, Edges, EdgeCount, Commands, Bitmap, Phong)     // 162
//     ... work records run through DoLineRenderWork / DoBufferLineRenderWork /
//         DoModelRenderWork (2336, 2343, 3873)
//     Platform.CompleteAllWork(RenderQueue)  ->  PRK_CompleteAllWork(Buffer, Commands)
//
// and links libprk_hip.so.  What each entry point does here:
//  * FillEdgeTable copies the object's VertexData / ColorData / NormalData /
//    UVData as they are at the call (the reference reads them there,
//    3898-3925) into the frame's pinned staging arena (sent on to the GPU in
//    chunks of 64K triangles while the caller keeps submitting), snapshots
//    Commands->Transform and LightData as they are at the call (3885,
//    3907-3909, 4022-4061) and its own inputs PhongShading and
//    Object->Bitmap != 0 (raw colours + normals vs per-vertex lighting,
//    4012-4063; white-based lighting and UV gradients, 4034-4054, 4078-4089:
//    the edges are built from them whatever DrawModel* later draws them
//    with), and leaves a token in Object->EdgeMemory (the object's arena
//    range, P, camera and setup: 36 bytes) that DrawModel* read back; the
//    setup itself (projection, cull, edges, lighting, MergeSort) runs on the
//    GPU at PRK_CompleteAllWork.  It returns the reference's value, the
//    visible edge count (4119; 0 for an object that draws nothing, e.g. a
//    back-facing triangle), computed on the host (include/prk_edge_count.h,
//    inline for one-triangle objects, else prk_fill_edge_count).  EdgeMemory
//    holds the token, not edge_info records.
//  * DrawModelOptimized(RenderQueue, ...) and DrawModelOptimizedLines draw
//    the object with FillLineOptimized semantics (FillLinesOptimized has the
//    same block math); DrawModelOptimized(Buffer, ...) with the
//    single-thread overload's quirks (PRK_SEM_AVX_ST); DrawModel with the
//    scalar semantics.  An object of several triangles is ONE active edge
//    table, as in the reference (prk_draw_objects), for every semantics.
//  * DrawModel* given edges that are NOT a FillEdgeTable token (a caller's
//    own edge_info list, e.g. built by the reference's FillEdgeTable) draw
//    that list as is (prk_draw_edges).  The work-queue callbacks draw the
//    spans of their work records (prk_draw_spans) or, for DoModelRenderWork,
//    the object (single-thread overload).
//  * PRK_CompleteAllWork (the absent platform's CompleteAllWork) sends the
//    geometry's last chunk, runs every recorded draw in order on the GPU and copies
//    colour and z back into Buffer->Memory and Commands->ZBuffer.  The device
//    target is allocated once per size; the caller's framebuffer and z-buffer
//    are page-locked once, so the prior contents go up (draws z-test against
//    them) and the result comes down as DMA.  PRK_ClearNextFrame(color, z)
//    replaces that upload by a clear fused into the frame's kernels.
//  * Textures (loaded_bitmap) are read at their first use in each frame.
//  * Cameras and lights: an object is set up (projection, Gouraud lighting)
//    with Commands->Transform / LightData as they were at its FillEdgeTable
//    call and shaded (Phong, unprojection) with them as they are at its
//    DrawModel* call, as the reference reads them (3885-4063; 452-458,
//    2042-2046, 3030-3034); edge lists and work records use them as they are
//    at their DrawModel* / callback call.  A frame whose draws saw several
//    cameras runs as consecutive flushes, one per change, in order.
//  * Record mode (PRK_SetEdgeRecords(1), or PRK_DROPIN_EDGES=1 in the
//    environment at PRK_Init*): FillEdgeTable writes the reference's sorted
//    edge_info records into Object->EdgeMemory (3894-4117, MergeSort with
//    Commands->SortMemory) instead of the token, and DrawModel* draws them as
//    the caller's edge list.  For a caller that reads its edges back, copies
//    them or draws them twice; the object's setup then runs on the host at the
//    call (prk_fill_edge_records) and the per-object batching of the token
//    path is gone.
//  * DrawModel* on an edge_info list (a caller's own, or record mode's) leaves
//    the list as the reference's walk does: every edge stepped once per row it
//    was paired on, the Next pointers as the walk left them (3654-3869,
//    prk_advance_edge_records).  The GPU draws the copy taken at the call.
//  * Inputs the reference crashes on are rejected or pinned, see
//    prk.h; PRK_LastStatus() reports the last library status.
//
// The caller-owned types of the reference live in its absent platform and
// math headers.  If the caller has them, define PRK_CALLER_TYPES before
// including this file; otherwise minimal definitions with the fields the
// reference uses are provided here.
#ifndef PRK_PROJEKT_H
#define PRK_PROJEKT_H

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <cstddef>
#include <map>
#include <set>
#include <vector>

#include "prk.h"
#include "prk_edge_count.h"

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

#ifndef PLATFORM_WORK_QUEUE_CALLBACK
#define PLATFORM_WORK_QUEUE_CALLBACK(name) void name(platform_work_queue *Queue, void *Data)
#endif

// The reference's own structs (projekt.h:2-98), field for field.
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

struct thread_edge_info {
    r32 LeftXMin, RightXMin;
    r32 LeftZMin, RightZMin;
    r32 LeftOneOverZMin, RightOneOverZMin;
    r32 LeftUMin, RightUMin;
    r32 LeftVMin, RightVMin;
    v4 LeftMinColor, RightMinColor;
    v3 LeftMinNormal, RightMinNormal;
};

struct line_render_work {
    game_render_commands *Commands;
    loaded_bitmap *OutputTarget;
    loaded_bitmap *Bitmap;
    edge_info CurrentEdgeInList;
    edge_info NextEdgeInList;
    s32 RowIndex;
    b32 PhongShading;
};

struct buffer_line_render_work {
    game_render_commands *Commands;
    loaded_bitmap *OutputTarget;
    loaded_bitmap *Bitmap;
    s32 RowIndex;
    b32 PhongShading;
    u32 EdgeCount;
    u32 Pad;
    thread_edge_info Edges;  // the first of EdgeCount (3604-3607)
};

struct model_render_work {
    game_render_commands *Commands;
    loaded_bitmap *OutputTarget;
    loaded_bitmap *Bitmap;
    edge_info *EdgeMemory;
    u32 EdgeCount;
    b32 PhongShading;
};

namespace prk_dropin {

// What FillEdgeTable leaves in Object->EdgeMemory for DrawModel*: the
// object itself (its triangles in the frame's arena, P, camera and setup), so
// the draw reads back the record its FillEdgeTable just wrote, and the frame
// keeps no per-object table.
struct object_token {
    uint32_t Magic;
    uint32_t Frame;           // frame serial the object was filled in
    uint32_t FirstTri, Tris;  // its triangles in the arena; Tris == 0: no edge (nothing to draw)
    float P[3];
    uint32_t Camera;          // Commands->Transform / LightData as they were at FillEdgeTable
    int32_t Setup;            // FillEdgeTable's PhongShading and Object->Bitmap != 0 (PRK_SETUP_*)
};
static_assert(sizeof(object_token) <= sizeof(edge_info), "token must fit one edge_info");
static const uint32_t kMagic = 0x4B525033u;  // "PRK3"

// Commands->Transform and LightData as one draw saw them.
struct camera {
    prk_transform T;
    prk_light_data L;
};

enum { DRAW_OBJECT = 0, DRAW_EDGES = 1, DRAW_SPANS = 2 };
struct pending_draw {
    int Kind;
    uint32_t First, Count;  // DRAW_OBJECT: first triangle, objects; else range of Edges / Spans
    int32_t Semantics, Phong, Texture;
    // indices into the frame's cameras: the one FillEdgeTable saw (setup:
    // projection, Gouraud lighting, 3885-4063) and the one the DrawModel* call
    // sees (span shading: Phong + unprojection, 452-458, 2042-2046, 3030-3034)
    uint32_t SetupCamera, Camera;
    // DRAW_OBJECT: Count objects drawn alike, consecutive in the arena, of
    // ObjTris triangles each, one offset P and setup, RunTris triangles in
    // all: one library call (the per-triangle objects of a reference caller
    // make one run per frame)
    uint32_t RunTris, ObjTris;
    float P[3];
    int32_t Setup;
};

struct state {
    prk_context *Ctx = nullptr;         // band 0's context (and the one of a 1-GPU drop-in)
    std::vector<prk_context *> Ctxs;    // one per GPU: context r renders rows prk_band_rows(H, r, N)
    int LastStatus = PRK_OK;
    // frame geometry: pinned staging arena (vertices), uploaded at CompleteAllWork
    float *AV = nullptr, *AC = nullptr, *AN = nullptr, *AUV = nullptr;
    uint32_t ArenaCap = 0, ArenaUsed = 0;  // vertices
    // vertices [0, Uploaded) of the frame are on their way to every device
    // (prk_geometry_write), sent in chunks while the caller submits objects
    uint32_t Uploaded = 0;
    int PushStatus = PRK_OK;               // the frame's first failed chunk write
    // host time of the last PRK_CompleteAllWork: recording the draws (and the
    // geometry tail), queueing the frames, waiting + downloading (ms)
    double LastIssueMs = 0, LastFlushMs = 0, LastDownloadMs = 0;
    int32_t Geom = -1;
    std::vector<pending_draw> Draws;
    std::vector<camera> Cameras;               // the frame's distinct camera / light snapshots, in order
    // Commands->Transform and the used part of LightData at the last camera
    // lookup, as raw bytes, and the camera they gave: an unchanged Commands
    // (every call of a usual frame) costs a compare of ~70 bytes
    projective_transform RawT;
    light_data RawL;
    uint32_t RawCamId = 0xFFFFFFFFu;
    std::vector<prk_edge> Edges;
    std::vector<prk_span> Spans;
    std::map<const void *, int32_t> Textures;  // Bitmap->Memory -> handle
    std::set<int32_t> TexFresh;                // handles re-read this frame
    std::map<void *, size_t> Registered;       // page-locked caller buffers
    loaded_bitmap *Target = nullptr;
    game_render_commands *Commands = nullptr;
    int32_t TW = 0, TH = 0;                    // device target size
    bool FrameOpen = false;
    uint32_t Frame = 1;
    bool ClearNext = false;
    uint32_t ClearColor = 0;
    float ClearZ = 0.0f;
    loaded_bitmap *LastBitmap = nullptr;        // texture of the previous draw this frame
    void *LastBitmapMemory = nullptr;
    int32_t LastTexture = -1;
    bool EdgeRecords = false;                   // record mode (PRK_SetEdgeRecords)
};
inline state g_state;  // (a namespace-scope inline variable: no guard check per call)
inline state &S() { return g_state; }

inline bool ok(int rc) {
    S().LastStatus = rc;
    return rc == PRK_OK;
}

inline void free_arena(state &st) {
    prk_host_free(st.Ctx, st.AV);
    prk_host_free(st.Ctx, st.AC);
    prk_host_free(st.Ctx, st.AN);
    prk_host_free(st.Ctx, st.AUV);
    st.AV = st.AC = st.AN = st.AUV = nullptr;
    st.ArenaCap = 0;
}

// Room for `more` vertices in the pinned arena (grows by doubling).
inline bool arena_reserve(state &st, uint32_t more) {
    const uint64_t need = (uint64_t)st.ArenaUsed + more;
    if (need <= st.ArenaCap) return true;
    if (need > 0xFFFFFFF0ull) return ok(PRK_ERR_ARG);
    uint64_t cap = st.ArenaCap ? st.ArenaCap : 3u * 4096u;
    while (cap < need) cap *= 2;
    if (cap > 0xFFFFFFF0ull) cap = need;
    void *p[4] = {nullptr, nullptr, nullptr, nullptr};
    const size_t comp[4] = {3, 4, 3, 2};
    for (int k = 0; k < 4; ++k)
        if (!ok(prk_host_alloc(st.Ctx, (size_t)cap * comp[k] * sizeof(float), &p[k]))) {
            for (int j = 0; j < k; ++j) prk_host_free(st.Ctx, p[j]);
            return false;
        }
    float *old[4] = {st.AV, st.AC, st.AN, st.AUV};
    for (int k = 0; k < 4; ++k)
        if (old[k]) memcpy(p[k], old[k], (size_t)st.ArenaUsed * comp[k] * sizeof(float));
    if (st.Uploaded)  // chunk copies may still read the old arena
        for (prk_context *c : st.Ctxs) prk_synchronize(c);
    free_arena(st);
    st.AV = (float *)p[0];
    st.AC = (float *)p[1];
    st.AN = (float *)p[2];
    st.AUV = (float *)p[3];
    st.ArenaCap = (uint32_t)cap;
    return true;
}

// f(ctx) on every band's context in rank order; the first failing status.
template <class F>
inline int each(F &&f) {
    for (prk_context *c : S().Ctxs) {
        const int rc = f(c);
        if (rc != PRK_OK) return rc;
    }
    return PRK_OK;
}

// Arena vertices [Uploaded, ArenaUsed) to every device: positions, normals
// and uvs, asynchronously on each context's copy stream, so PCIe runs while
// the caller is still submitting objects and PRK_CompleteAllWork waits for
// the tail only.  Colours reach the output only through DrawModel (scalar)
// (the FillLineOptimized paths replace them by the texel, 2029-2032): they
// go at issue(), for frames with scalar draws.  The first push ever creates
// the geometry (synchronously, colours included).
// Chunk size in triangles: PRK_DROPIN_CHUNK_TRIS (0: everything at
// PRK_CompleteAllWork, the round-2 behaviour), default 65536.
inline uint32_t chunk_vertices() {
    static const uint32_t v = [] {
        const char *e = std::getenv("PRK_DROPIN_CHUNK_TRIS");
        const long t = e ? std::atol(e) : 65536L;
        return t > 0 && t < (1L << 28) ? 3u * (uint32_t)t : 0xFFFFFFFFu;
    }();
    return v;
}
inline int push_vertices(state &st) {
    if (st.ArenaUsed == st.Uploaded) return PRK_OK;
    const uint32_t a = st.Uploaded, n = st.ArenaUsed - a;
    int rc;
    if (st.Geom < 0) {
        int32_t g = -1;
        rc = each([&](prk_context *c) {
            int32_t gc = -1;
            const int r = prk_geometry_create(c, st.AV, st.AC, st.AN, st.AUV, st.ArenaUsed, &gc);
            if (r == PRK_OK && g >= 0 && gc != g) return (int)PRK_ERR_ARG;
            g = gc;
            return r;
        });
        if (rc == PRK_OK) st.Geom = g;
    } else {
        rc = each([&](prk_context *c) {
            return prk_geometry_write(c, st.Geom, a, n, st.AV + 3 * (size_t)a, nullptr, st.AN + 3 * (size_t)a,
                                      st.AUV + 2 * (size_t)a);
        });
    }
    if (rc == PRK_OK) st.Uploaded = st.ArenaUsed;
    else if (st.PushStatus == PRK_OK) st.PushStatus = rc;
    return rc;
}

// f(ctx, first colour byte, first z float) of every band's rows of the
// caller's buffers.
template <class F>
inline int each_band(loaded_bitmap *Buffer, game_render_commands *Commands, F &&f) {
    const int n = (int)S().Ctxs.size();
    for (int r = 0; r < n; ++r) {
        int32_t a = 0, b = 0;
        int rc = prk_band_rows(Buffer->Height, r, n, &a, &b);
        if (rc == PRK_OK)
            rc = f(S().Ctxs[r], (uint8_t *)Buffer->Memory + (size_t)a * Buffer->Pitch,
                   Commands->ZBuffer ? Commands->ZBuffer + (size_t)a * Buffer->Width : nullptr);
        if (rc != PRK_OK) return rc;
    }
    return PRK_OK;
}

// The bitmap as it is now: created on first use, re-read once per frame.
inline int32_t texture_for(loaded_bitmap *Bitmap) {
    if (!Bitmap || !Bitmap->Memory) return -1;
    state &st = S();
    prk_bitmap b = {Bitmap->Memory, Bitmap->Width, Bitmap->Height, Bitmap->Pitch};
    auto it = st.Textures.find(Bitmap->Memory);
    if (it != st.Textures.end()) {
        if (!st.TexFresh.count(it->second)) {
            if (!ok(each([&](prk_context *c) { return prk_texture_update(c, it->second, &b); }))) return -1;
            st.TexFresh.insert(it->second);
        }
        return it->second;
    }
    int32_t h = -1;
    // every context creates its textures in the same order: same handles
    if (!ok(each([&](prk_context *c) {
            int32_t hc = -1;
            const int rc = prk_texture_create(c, &b, &hc);
            if (rc == PRK_OK && h >= 0 && hc != h) return (int)PRK_ERR_ARG;
            h = hc;
            return rc;
        })))
        return -1;
    st.Textures[Bitmap->Memory] = h;
    st.TexFresh.insert(h);
    return h;
}

// Commands->Transform and LightData as they are now (FillEdgeTable reads them
// at its call, projekt.cpp:3885, 3907-3909, 4022-4061; the span kernels read
// them when the draw runs).
inline camera camera_of(const game_render_commands *Commands) {
    camera k;
    memset(&k, 0, sizeof k);
    k.T.DistanceAboveTarget = Commands->Transform.DistanceAboveTarget;
    k.T.FocalLength = Commands->Transform.FocalLength;
    k.T.MetersToPixels = Commands->Transform.MetersToPixels;
    k.T.ScreenCenter[0] = Commands->Transform.ScreenCenter.x;
    k.T.ScreenCenter[1] = Commands->Transform.ScreenCenter.y;
    k.L.LightCount = Commands->LightData.LightCount;
    for (int c = 0; c < 4; ++c) k.L.AmbientIntensity[c] = Commands->LightData.AmbientIntensity.E[c];
    for (u32 i = 0; i < k.L.LightCount && i < PRK_MAX_LIGHTS; ++i) {
        for (int c = 0; c < 3; ++c) k.L.Lights[i].P[c] = Commands->LightData.Lights[i].P.E[c];
        for (int c = 0; c < 4; ++c) k.L.Lights[i].Intensity[c] = Commands->LightData.Lights[i].Intensity.E[c];
    }
    return k;
}

// The frame's camera index of a snapshot: the last one when unchanged (the
// usual frame has one), else a new entry.
inline bool same_bits(float a, float b) {
    uint32_t x, y;
    memcpy(&x, &a, 4);
    memcpy(&y, &b, 4);
    return x == y;
}
// k == camera_of(Commands), bit for bit, without building the snapshot (the
// drop-in asks once per FillEdgeTable call).
inline bool camera_is(const camera &k, const game_render_commands *C) {
    const auto &T = C->Transform;
    if (!same_bits(k.T.DistanceAboveTarget, T.DistanceAboveTarget) || !same_bits(k.T.FocalLength, T.FocalLength) ||
        !same_bits(k.T.MetersToPixels, T.MetersToPixels) || !same_bits(k.T.ScreenCenter[0], T.ScreenCenter.x) ||
        !same_bits(k.T.ScreenCenter[1], T.ScreenCenter.y) || k.L.LightCount != C->LightData.LightCount)
        return false;
    for (int c = 0; c < 4; ++c)
        if (!same_bits(k.L.AmbientIntensity[c], C->LightData.AmbientIntensity.E[c])) return false;
    for (u32 i = 0; i < k.L.LightCount && i < PRK_MAX_LIGHTS; ++i) {
        for (int c = 0; c < 3; ++c)
            if (!same_bits(k.L.Lights[i].P[c], C->LightData.Lights[i].P.E[c])) return false;
        for (int c = 0; c < 4; ++c)
            if (!same_bits(k.L.Lights[i].Intensity[c], C->LightData.Lights[i].Intensity.E[c])) return false;
    }
    return true;
}
// The bytes a camera lookup compares: the transform, the light count and
// ambient term, and the lights in use.
// (fixed-size compares, inlined: this runs twice per drawn object)
inline bool raw_camera_same(const state &st, const game_render_commands *C) {
    const light_data &a = C->LightData, &b = st.RawL;
    if (__builtin_memcmp(&C->Transform, &st.RawT, sizeof(projective_transform)) != 0 || a.LightCount != b.LightCount ||
        a.LightCount > PRK_MAX_LIGHTS ||
        __builtin_memcmp(&a.AmbientIntensity, &b.AmbientIntensity, sizeof a.AmbientIntensity) != 0)
        return false;
    for (u32 i = 0; i < a.LightCount; ++i)
        if (__builtin_memcmp(&a.Lights[i], &b.Lights[i], sizeof(a.Lights[0])) != 0) return false;
    return true;
}
// (the lookup when the raw bytes changed: out of line, so the per-call fast
// path below stays a few compares)
__attribute__((noinline)) inline uint32_t camera_id_slow(state &st, const game_render_commands *C) {
    // a camera seen lately (a caller switching between two, e.g. one for
    // FillEdgeTable and one for DrawModel*), else a new entry
    uint32_t id = (uint32_t)st.Cameras.size();
    for (uint32_t k = 0; k < 4 && k < st.Cameras.size(); ++k)
        if (camera_is(st.Cameras[st.Cameras.size() - 1 - k], C)) {
            id = (uint32_t)st.Cameras.size() - 1 - k;
            break;
        }
    if (id == st.Cameras.size()) st.Cameras.push_back(camera_of(C));
    memcpy(&st.RawT, &C->Transform, sizeof(projective_transform));
    memcpy(&st.RawL, &C->LightData, sizeof(light_data));
    st.RawCamId = id;
    return id;
}
// (RawCamId is reset with the frame's cameras, end_frame)
inline uint32_t camera_id(state &st, const game_render_commands *C) {
    if (st.RawCamId != 0xFFFFFFFFu && raw_camera_same(st, C)) return st.RawCamId;
    return camera_id_slow(st, C);
}

inline int set_camera(const camera &setup, const camera &shade, bool split) {
    return each([&](prk_context *c) {
        const int rc = prk_set_camera(c, &setup.T, &setup.L);
        return rc == PRK_OK && split ? prk_set_shade_camera(c, &shade.T, &shade.L) : rc;
    });
}

inline void register_host(state &st, void *p, size_t bytes) {
    auto it = st.Registered.find(p);
    if (it != st.Registered.end()) {
        if (it->second >= bytes) return;
        prk_host_unregister(st.Ctx, p);
        st.Registered.erase(it);
    }
    // best effort: unregistered memory still works, through staging copies
    if (prk_host_register(st.Ctx, p, bytes) == PRK_OK) st.Registered[p] = bytes;
}

// First draw of a frame: the device target (reallocated only when the size
// changes) takes the caller's current colour and z, so draws z-test against
// them; PRK_ClearNextFrame replaces that upload by a fused clear.
inline bool open_frame(loaded_bitmap *Buffer, game_render_commands *Commands) {
    state &st = S();
    if (st.FrameOpen) {
        if (st.Target == Buffer && st.Commands == Commands) return true;
        return ok(PRK_ERR_ARG);  // one target per frame: CompleteAllWork first
    }
    if (!Buffer || !Commands || !Buffer->Memory || Buffer->Width <= 0 || Buffer->Height <= 0 ||
        (Commands->Width != (u32)Buffer->Width))  // z rows are Commands->Width floats (170, 1511)
        return ok(PRK_ERR_ARG);
    if (Buffer->Width != st.TW || Buffer->Height != st.TH) {
        const int n = (int)st.Ctxs.size();
        for (int r = 0; r < n; ++r) {
            int32_t a = 0, b = 0;
            if (!ok(prk_band_rows(Buffer->Height, r, n, &a, &b))) return false;
            if (!ok(prk_target_alloc(st.Ctxs[r], Buffer->Width, Buffer->Height, a, b, nullptr, nullptr)))
                return false;
        }
        st.TW = Buffer->Width;
        st.TH = Buffer->Height;
    }
    register_host(st, Buffer->Memory, (size_t)Buffer->Pitch * Buffer->Height);
    if (Commands->ZBuffer) register_host(st, Commands->ZBuffer, (size_t)Buffer->Width * Buffer->Height * 4);
    if (st.ClearNext) {
        if (!ok(each([&](prk_context *c) { return prk_target_clear_on_flush(c, st.ClearColor, st.ClearZ); })))
            return false;
        st.ClearNext = false;
    } else {
        // the prior contents go up on the copy stream while the caller keeps
        // submitting (page-locked buffers; else a synchronous upload)
        const bool pinned = st.Registered.count(Buffer->Memory) &&
                            (!Commands->ZBuffer || st.Registered.count(Commands->ZBuffer));
        if (!ok(each_band(Buffer, Commands, [&](prk_context *c, uint8_t *col, float *z) {
                return pinned ? prk_target_upload_async(c, (const uint32_t *)col, Buffer->Pitch, z)
                              : prk_target_upload(c, (const uint32_t *)col, Buffer->Pitch, z);
            })))
            return false;
    }
    st.Target = Buffer;
    st.Commands = Commands;
    st.FrameOpen = true;
    return true;
}

inline void edge_in(prk_edge &o, const edge_info &e) {
    o.YMax = e.YMax; o.XMin = e.XMin; o.ZMin = e.ZMin; o.OneOverZMin = e.OneOverZMin; o.Gradient = e.Gradient;
    o.ZGradient = e.ZGradient; o.OneOverZGradient = e.OneOverZGradient; o.YMin = e.YMin; o.UMin = e.UMin;
    o.VMin = e.VMin; o.UGradient = e.UGradient; o.VGradient = e.VGradient; o.Left = e.Left;
    for (int c = 0; c < 4; ++c) { o.MinColor[c] = e.MinColor.E[c]; o.ColorGradient[c] = e.ColorGradient.E[c]; }
    for (int c = 0; c < 3; ++c) { o.MinNormal[c] = e.MinNormal.E[c]; o.NormalGradient[c] = e.NormalGradient.E[c]; }
}

inline void span_end(prk_span_end &o, const edge_info &e) {  // line_render_work's edges by value
    o.XMin = e.XMin; o.ZMin = e.ZMin; o.OneOverZMin = e.OneOverZMin; o.UMin = e.UMin; o.VMin = e.VMin;
    for (int c = 0; c < 4; ++c) o.MinColor[c] = e.MinColor.E[c];
    for (int c = 0; c < 3; ++c) o.MinNormal[c] = e.MinNormal.E[c];
}

inline void draw(loaded_bitmap *Buffer, edge_info *Edges, u32 EdgeCount, game_render_commands *Commands,
                 loaded_bitmap *Bitmap, b32 PhongShading, int32_t semantics) {
    state &st = S();
    if (!st.Ctx || !Edges || EdgeCount == 0) return;  // 0 edges: nothing to draw (P1)
    if (!(st.FrameOpen && st.Target == Buffer && st.Commands == Commands) && !open_frame(Buffer, Commands)) return;
    int32_t tex = -1;
    if (Bitmap) {  // the same bitmap as the previous draw: its handle, already fresh this frame
        if (Bitmap == st.LastBitmap && Bitmap->Memory == st.LastBitmapMemory) tex = st.LastTexture;
        else {
            tex = texture_for(Bitmap);
            st.LastBitmap = Bitmap;
            st.LastBitmapMemory = Bitmap->Memory;
            st.LastTexture = tex;
        }
    }
    object_token o;
    memcpy(&o, Edges, sizeof o);
    const int32_t phong = PhongShading ? 1 : 0;
    // a token of this frame whose triangles are in the arena (a stale or
    // foreign one is drawn as an edge list, which is what it then is)
    if (o.Magic == kMagic && o.Frame == st.Frame && o.Camera < st.Cameras.size() &&
        (uint64_t)o.FirstTri + o.Tris <= st.ArenaUsed / 3) {
        if (o.Tris == 0) return;  // FillEdgeTable wrote no edge: nothing to draw
        const uint32_t cam = camera_id(st, Commands);  // as this call sees it (shading)
        if (!st.Draws.empty()) {  // the next object of the previous draw's run
            pending_draw &b = st.Draws.back();
            if (b.Kind == DRAW_OBJECT && o.FirstTri == b.First + b.RunTris && o.Tris == b.ObjTris &&
                b.Camera == cam && b.SetupCamera == o.Camera && b.Semantics == semantics && b.Phong == phong &&
                b.Texture == tex && b.Setup == o.Setup && __builtin_memcmp(o.P, b.P, sizeof o.P) == 0) {
                ++b.Count;
                b.RunTris += o.Tris;
                st.LastStatus = PRK_OK;
                return;
            }
        }
        pending_draw d{};
        d.Kind = DRAW_OBJECT;
        d.Semantics = semantics;
        d.Phong = phong;
        d.Texture = tex;
        d.First = o.FirstTri;
        d.Count = 1;
        d.RunTris = d.ObjTris = o.Tris;
        memcpy(d.P, o.P, sizeof d.P);
        d.Setup = o.Setup;
        d.SetupCamera = o.Camera;  // as FillEdgeTable saw it
        d.Camera = cam;
        st.Draws.push_back(d);
    } else {  // a caller's own edge_info list, drawn as given
        pending_draw d{};
        d.Semantics = semantics;
        d.Phong = phong;
        d.Texture = tex;
        d.Camera = d.SetupCamera = camera_id(st, Commands);
        d.Kind = DRAW_EDGES;
        d.First = (uint32_t)st.Edges.size();
        d.Count = EdgeCount;
        st.Edges.resize(st.Edges.size() + EdgeCount);
        for (u32 i = 0; i < EdgeCount; ++i) edge_in(st.Edges[d.First + i], Edges[i]);
        st.Draws.push_back(d);
        // what the reference's walk leaves in the caller's list (3654-3869):
        // the GPU draws the copy above
        if (!ok(prk_advance_edge_records(Edges, EdgeCount, sizeof(edge_info), offsetof(edge_info, Next),
                                         Buffer->Height)))
            return;
    }
    st.LastStatus = PRK_OK;
}

inline void draw_spans(loaded_bitmap *Buffer, game_render_commands *Commands, loaded_bitmap *Bitmap,
                       b32 PhongShading, const prk_span *spans, uint32_t n) {
    state &st = S();
    if (!st.Ctx || n == 0) return;
    if (!open_frame(Buffer, Commands)) return;
    pending_draw d{};
    d.Kind = DRAW_SPANS;
    d.First = (uint32_t)st.Spans.size();
    d.Count = n;
    d.Semantics = PRK_SEM_AVX;
    d.Phong = PhongShading ? 1 : 0;
    d.Texture = Bitmap ? texture_for(Bitmap) : -1;
    d.Camera = d.SetupCamera = camera_id(st, Commands);
    st.Spans.insert(st.Spans.end(), spans, spans + n);
    st.Draws.push_back(d);
}

// Records the frame's draws with the library, in order.  Draws that saw
// different cameras or lights (Commands changed between calls) run as
// consecutive flushes, one per (setup camera, shading camera) run, each set up
// with the camera its FillEdgeTable saw and shaded with the one its DrawModel*
// call saw (prk_set_shade_camera); a later flush z-tests against what the
// earlier ones left, which is the reference's sequential order.  The last
// flush is left to the caller (PRK_CompleteAllWork).
inline int issue(state &st) {
    int rc = PRK_OK;
    if (st.LastStatus != PRK_OK) return st.LastStatus;
    if (st.PushStatus != PRK_OK) return st.PushStatus;
    if (st.ArenaUsed) {
        const bool created = st.Geom < 0;
        rc = push_vertices(st);  // the tail (most of the frame went during the host calls)
        if (rc != PRK_OK) return rc;
        bool colors = false;
        for (const pending_draw &d : st.Draws) colors |= d.Kind == DRAW_OBJECT && d.Semantics == PRK_SEM_SCALAR;
        if (colors && !created)
            rc = each([&](prk_context *c) {
                return prk_geometry_write(c, st.Geom, 0, st.ArenaUsed, nullptr, st.AC, nullptr, nullptr);
            });
        if (rc != PRK_OK) return rc;
    }
    // every band records every draw (each bins all triangles against its rows)
    if (st.Cameras.empty()) st.Cameras.push_back(camera_of(st.Commands));
    size_t i = 0;
    while (i < st.Draws.size() || i == 0) {
        const uint32_t cam = st.Draws.empty() ? 0u : st.Draws[i].Camera;
        const uint32_t scam = st.Draws.empty() ? 0u : st.Draws[i].SetupCamera;
        size_t j = i;
        while (j < st.Draws.size() && st.Draws[j].Camera == cam && st.Draws[j].SetupCamera == scam) ++j;
        if (i > 0) {  // camera / lights changed: the draws so far run first
            rc = each([](prk_context *k) { return prk_flush(k, nullptr); });
            if (rc != PRK_OK) return rc;
        }
        rc = set_camera(st.Cameras[scam], st.Cameras[cam], scam != cam);
        if (rc != PRK_OK) return rc;
        rc = each([&](prk_context *c) {
            int r = PRK_OK;
            for (size_t k = i; k < j && r == PRK_OK; ++k) {
                const pending_draw &d = st.Draws[k];
                if (d.Kind == DRAW_OBJECT) {
                    r = prk_draw_objects_setup(c, st.Geom, d.First, d.RunTris, d.ObjTris, d.P, d.Semantics,
                                               d.Phong, d.Texture, d.Setup);
                } else if (d.Kind == DRAW_EDGES) {
                    r = prk_draw_edges(c, st.Edges.data() + d.First, d.Count, d.Semantics, d.Phong, d.Texture);
                } else {
                    r = prk_draw_spans(c, st.Spans.data() + d.First, d.Count, d.Semantics, d.Phong, d.Texture);
                }
            }
            return r;
        });
        if (rc != PRK_OK || j == i) return rc;
        i = j;
    }
    return rc;
}

inline void end_frame(state &st) {
    st.LastBitmap = nullptr;
    st.LastBitmapMemory = nullptr;
    st.LastTexture = -1;
    st.ArenaUsed = 0;
    st.Uploaded = 0;
    st.PushStatus = PRK_OK;
    st.Draws.clear();
    st.Cameras.clear();
    st.RawCamId = 0xFFFFFFFFu;
    st.Edges.clear();
    st.Spans.clear();
    st.TexFresh.clear();
    st.FrameOpen = false;
    st.Target = nullptr;
    st.Commands = nullptr;
    ++st.Frame;
}

}  // namespace prk_dropin

// ---- platform hooks --------------------------------------------------------
// Extension: the frame split into n row bands, band r rendered by GPU
// devices[r] (a device may appear more than once); every band's colour and z
// come back into the caller's buffers over that GPU's own link.
inline int PRK_InitDevices(const int *devices, int n) {
    prk_dropin::state &st = prk_dropin::S();
    if (st.Ctx) return PRK_OK;
    if (!devices || n <= 0) return st.LastStatus = PRK_ERR_ARG;
    for (int r = 0; r < n; ++r) {
        prk_context *c = nullptr;
        st.LastStatus = prk_create(devices[r], &c);
        if (st.LastStatus != PRK_OK) {
            for (prk_context *k : st.Ctxs) prk_destroy(k);
            st.Ctxs.clear();
            return st.LastStatus;
        }
        (void)prk_set_early_z(c, 1);  // every frame is downloaded (PRK_CompleteAllWork): z goes down while it shades
        st.Ctxs.push_back(c);
    }
    st.Ctx = st.Ctxs[0];
    const char *rec = std::getenv("PRK_DROPIN_EDGES");
    st.EdgeRecords = rec && rec[0] == '1';
    return st.LastStatus;
}
inline int PRK_Init(int device) { return PRK_InitDevices(&device, 1); }
inline int PRK_LastStatus() { return prk_dropin::S().LastStatus; }
inline void PRK_Shutdown() {
    prk_dropin::state &st = prk_dropin::S();
    if (st.Ctx) {
        for (prk_context *c : st.Ctxs) prk_synchronize(c);
        for (auto &r : st.Registered) prk_host_unregister(st.Ctx, r.first);
        prk_dropin::free_arena(st);
        for (prk_context *c : st.Ctxs) prk_destroy(c);
    }
    st = prk_dropin::state();
}
// Extension: record mode on (1) or off (0): FillEdgeTable writes real
// edge_info records into Object->EdgeMemory (see the top of this file).
inline void PRK_SetEdgeRecords(int on) { prk_dropin::S().EdgeRecords = on != 0; }
// Extension: the next frame starts from (color, z) instead of the caller's
// buffers (no upload; the clear is fused into the frame's kernels).
inline void PRK_ClearNextFrame(uint32_t color, float z) {
    prk_dropin::state &st = prk_dropin::S();
    st.ClearNext = true;
    st.ClearColor = color;
    st.ClearZ = z;
}
// Platform.CompleteAllWork equivalent: run the frame, copy colour and z back.
inline int PRK_CompleteAllWork(loaded_bitmap *Buffer, game_render_commands *Commands) {
    prk_dropin::state &st = prk_dropin::S();
    if (!st.Ctx || !st.FrameOpen) return PRK_OK;
    using clk = std::chrono::steady_clock;
    const auto ms = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t0 = clk::now();
    int rc = prk_dropin::issue(st);
    const auto t1 = clk::now();
    // all bands' frames are queued before the first download waits
    if (rc == PRK_OK) rc = prk_dropin::each([](prk_context *c) { return prk_flush(c, nullptr); });
    else  // nothing drawn; the arena's chunk copies finish before the next frame reuses it
        prk_dropin::each([](prk_context *c) { return prk_reset_draws(c) | prk_synchronize(c); });
    const auto t2 = clk::now();
    if (rc == PRK_OK)
        rc = prk_dropin::each_band(Buffer, Commands, [&](prk_context *c, uint8_t *col, float *z) {
            return prk_target_download(c, (uint32_t *)col, Buffer->Pitch, z);
        });
    st.LastIssueMs = ms(t0, t1);
    st.LastFlushMs = ms(t1, t2);
    st.LastDownloadMs = ms(t2, clk::now());
    prk_dropin::end_frame(st);
    st.LastStatus = rc;
    return rc;
}

// ---- the reference's entry points ------------------------------------------
// projekt.cpp:3882-4121
inline u32 FillEdgeTable(render_entry_3d_object *Object, game_render_commands *Commands, b32 PhongShading = 0) {
    prk_dropin::state &st = prk_dropin::S();
    if (!st.Ctx || !Object || !Commands || !Object->EdgeMemory || !Object->VertexData || Object->VertexCount < 3)
        return 0;
    const u32 T = Object->VertexCount / 3, nv = 3 * T;
    if (st.EdgeRecords) {  // the reference's records, in the caller's EdgeMemory (3894-4117)
        const prk_dropin::camera &k = st.Cameras[prk_dropin::camera_id(st, Commands)];
        const float P[3] = {Object->P.x, Object->P.y, Object->P.z};
        u32 n = 0;
        const int32_t setup = (PhongShading ? PRK_SETUP_PHONG : 0) | (Object->Bitmap ? PRK_SETUP_BITMAP : 0);
        if (!prk_dropin::ok(prk_fill_edge_records((const float *)Object->VertexData, (const float *)Object->ColorData,
                                                  (const float *)Object->NormalData, (const float *)Object->UVData,
                                                  nv, P, &k.T, &k.L, setup, Object->EdgeMemory, sizeof(edge_info),
                                                  offsetof(edge_info, Next), Commands->SortMemory, &n)))
            return 0;
        return n;
    }
    prk_dropin::object_token o;
    o.Magic = prk_dropin::kMagic;
    o.Frame = st.Frame;
    o.P[0] = Object->P.x;
    o.P[1] = Object->P.y;
    o.P[2] = Object->P.z;
    // what this call's own inputs make of the edges (raw colours + normals vs
    // Gouraud lighting, 4012-4063; white base and UV gradients with a Bitmap,
    // 4034-4054, 4078-4089), whatever DrawModel* later draws them with
    o.Setup = (PhongShading ? PRK_SETUP_PHONG : 0) | (Object->Bitmap ? PRK_SETUP_BITMAP : 0);
    // the camera and lights of this call (3885, 3907-3909, 4022-4061)
    o.Camera = prk_dropin::camera_id(st, Commands);
    const prk_dropin::camera &cam = st.Cameras[o.Camera];
    // the reference's return value: the visible edge count (4119), 0 when no
    // edge is visible (e.g. a back-facing triangle)
    u32 edges = 0;
#if PRK_EC_SSE && !defined(PRK_DROPIN_LIB_COUNT)
    // one triangle (the per-triangle objects of a reference caller): counted
    // inline from the registers the snapshot then stores
    const bool one = nv == 3;
    __m128 q0 = _mm_setzero_ps(), q1 = q0, q2 = q0;
    if (one) {
        const float *v = (const float *)Object->VertexData;
        q0 = _mm_loadu_ps(v);
        q1 = _mm_loadu_ps(v + 4);
        q2 = _mm_load_ss(v + 8);
        edges = prk_tri_edge_count_sse(q0, q1, q2, o.P[0], o.P[1], o.P[2], &cam.T);
        st.LastStatus = PRK_OK;
    } else
#endif
        if (!prk_dropin::ok(prk_fill_edge_count((const float *)Object->VertexData, nv, o.P, &cam.T, &edges)))
        return 0;
    o.FirstTri = 0;
    o.Tris = 0;
    if (edges) {  // an object with no visible edge draws nothing: nothing to upload
        if (!prk_dropin::arena_reserve(st, nv)) return 0;
        const uint32_t v0 = st.ArenaUsed;
        if (nv == 3 && Object->ColorData && Object->NormalData && Object->UVData) {  // one triangle: fixed-size copies
#if PRK_EC_SSE && !defined(PRK_DROPIN_LIB_COUNT)
            float *av = st.AV + 3 * (size_t)v0;  // (the registers the count read)
            _mm_storeu_ps(av, q0);
            _mm_storeu_ps(av + 4, q1);
            _mm_store_ss(av + 8, q2);
#else
            memcpy(st.AV + 3 * (size_t)v0, Object->VertexData, 36);
#endif
            memcpy(st.AC + 4 * (size_t)v0, Object->ColorData, 48);
            memcpy(st.AN + 3 * (size_t)v0, Object->NormalData, 36);
            memcpy(st.AUV + 2 * (size_t)v0, Object->UVData, 24);
        } else {
            memcpy(st.AV + 3 * (size_t)v0, Object->VertexData, (size_t)nv * 12);
            if (Object->ColorData) memcpy(st.AC + 4 * (size_t)v0, Object->ColorData, (size_t)nv * 16);
            else memset(st.AC + 4 * (size_t)v0, 0, (size_t)nv * 16);
            if (Object->NormalData) memcpy(st.AN + 3 * (size_t)v0, Object->NormalData, (size_t)nv * 12);
            else memset(st.AN + 3 * (size_t)v0, 0, (size_t)nv * 12);
            if (Object->UVData) memcpy(st.AUV + 2 * (size_t)v0, Object->UVData, (size_t)nv * 8);
            else memset(st.AUV + 2 * (size_t)v0, 0, (size_t)nv * 8);
        }
        st.ArenaUsed += nv;
        o.FirstTri = v0 / 3;
        o.Tris = T;
        if (st.ArenaUsed - st.Uploaded >= prk_dropin::chunk_vertices() && st.PushStatus == PRK_OK)
            prk_dropin::push_vertices(st);  // a failure is reported by PRK_CompleteAllWork
    }
    memcpy(Object->EdgeMemory, &o, sizeof o);
    return edges;
}

// projekt.cpp:3615-3871 (+ FillLineOptimized 1492-2320)
inline void DrawModelOptimized(platform_work_queue *RenderQueue, loaded_bitmap *Buffer, edge_info *Edges,
                               u32 EdgeCount, game_render_commands *Commands, loaded_bitmap *Bitmap = 0,
                               b32 PhongShading = 0) {
    (void)RenderQueue;
    prk_dropin::draw(Buffer, Edges, EdgeCount, Commands, Bitmap, PhongShading, PRK_SEM_AVX);
}

// projekt.cpp:3362-3613 (+ FillLinesOptimized 629-1490: FillLineOptimized's block math)
inline void DrawModelOptimizedLines(platform_work_queue *RenderQueue, loaded_bitmap *Buffer, edge_info *Edges,
                                    u32 EdgeCount, game_render_commands *Commands, loaded_bitmap *Bitmap = 0,
                                    b32 PhongShading = 0) {
    (void)RenderQueue;
    prk_dropin::draw(Buffer, Edges, EdgeCount, Commands, Bitmap, PhongShading, PRK_SEM_AVX);
}

// projekt.cpp:2350-3358, the single-thread overload
inline void DrawModelOptimized(loaded_bitmap *Buffer, edge_info *Edges, u32 EdgeCount, game_render_commands *Commands,
                               loaded_bitmap *Bitmap = 0, b32 PhongShading = 0) {
    prk_dropin::draw(Buffer, Edges, EdgeCount, Commands, Bitmap, PhongShading, PRK_SEM_AVX_ST);
}

// projekt.cpp:162-601
inline void DrawModel(loaded_bitmap *Buffer, edge_info *Edges, u32 EdgeCount, game_render_commands *Commands,
                      loaded_bitmap *Bitmap = 0, b32 PhongShading = 0) {
    prk_dropin::draw(Buffer, Edges, EdgeCount, Commands, Bitmap, PhongShading, PRK_SEM_SCALAR);
}

// projekt.cpp:2336-2341: one span of a line_render_work
inline PLATFORM_WORK_QUEUE_CALLBACK(DoLineRenderWork) {
    (void)Queue;
    line_render_work *Work = (line_render_work *)Data;
    prk_span sp;
    prk_dropin::span_end(sp.Left, Work->CurrentEdgeInList);
    prk_dropin::span_end(sp.Right, Work->NextEdgeInList);
    sp.Row = Work->RowIndex;
    prk_dropin::draw_spans(Work->OutputTarget, Work->Commands, Work->Bitmap, Work->PhongShading, &sp, 1);
}

// projekt.cpp:2343-2348: the spans of one row (FillLinesOptimized 629-1490)
inline PLATFORM_WORK_QUEUE_CALLBACK(DoBufferLineRenderWork) {
    (void)Queue;
    buffer_line_render_work *Work = (buffer_line_render_work *)Data;
    const thread_edge_info *E = &Work->Edges;
    std::vector<prk_span> sp(Work->EdgeCount);
    for (u32 k = 0; k < Work->EdgeCount; ++k) {  // 648-670
        prk_span &s = sp[k];
        s.Left.XMin = E[k].LeftXMin; s.Right.XMin = E[k].RightXMin;
        s.Left.ZMin = E[k].LeftZMin; s.Right.ZMin = E[k].RightZMin;
        s.Left.OneOverZMin = E[k].LeftOneOverZMin; s.Right.OneOverZMin = E[k].RightOneOverZMin;
        s.Left.UMin = E[k].LeftUMin; s.Right.UMin = E[k].RightUMin;
        s.Left.VMin = E[k].LeftVMin; s.Right.VMin = E[k].RightVMin;
        for (int c = 0; c < 4; ++c) { s.Left.MinColor[c] = E[k].LeftMinColor.E[c]; s.Right.MinColor[c] = E[k].RightMinColor.E[c]; }
        for (int c = 0; c < 3; ++c) { s.Left.MinNormal[c] = E[k].LeftMinNormal.E[c]; s.Right.MinNormal[c] = E[k].RightMinNormal.E[c]; }
        s.Row = Work->RowIndex;
    }
    prk_dropin::draw_spans(Work->OutputTarget, Work->Commands, Work->Bitmap, Work->PhongShading, sp.data(),
                           (uint32_t)sp.size());
}

// projekt.cpp:3873-3878: a whole object through the single-thread overload
inline PLATFORM_WORK_QUEUE_CALLBACK(DoModelRenderWork) {
    (void)Queue;
    model_render_work *Work = (model_render_work *)Data;
    DrawModelOptimized(Work->OutputTarget, Work->EdgeMemory, Work->EdgeCount, Work->Commands, Work->Bitmap,
                       Work->PhongShading);
}

// The reference's test mesh (projekt.cpp:4123-4289).
inline u32 ConstructSphere(v3 *Vertices, v4 *Colors, v3 *Normals, v2 *UVs) {
    uint32_t n = 0;
    prk_construct_sphere((float *)Vertices, (float *)Colors, (float *)Normals, (float *)UVs, &n);
    return n;
}

#endif  // PRK_PROJEKT_H
