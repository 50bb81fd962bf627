/*
 * prk.h — C-ABI of the MI355X-native rasterizer (libprk_hip.so).
 *
 * This is the drop-in boundary for the reference's ONE hot path:
 *
 *     FillEdgeTable            projekt.cpp:3882-4121   (triangle setup)
 *     DrawModelOptimized(Queue) projekt.cpp:3615-3871  (AET walk, per-span tasks)
 *       -> FillLineOptimized   projekt.cpp:1492-2320   (8-px AVX span kernel)
 *     DrawModel                projekt.cpp:162-601     (scalar span kernel)
 *     Platform.CompleteAllWork (absent platform layer, inferred from
 *                               projekt.cpp:3609,3809)
 *
 * The reference exports nothing (every function is `internal`), so the
 * boundary is the set of C++ signatures above plus the caller-owned types
 * they take.  `include/projekt.h` re-declares those C++ signatures and
 * forwards them to the plain-C entry points below.  Signatures here use only
 * plain pointers, sizes and POD structs; no torch or HIP types.
 *
 * Every prk_* function returns an int status (PRK_OK == 0, negative on
 * error) — the reference has no error convention at all (Assert only,
 * projekt.cpp:2327), and crashes on several ordinary inputs;
 * here those inputs are rejected with a status code instead.
 *
 * Semantics: prk_draw submits every triangle as its own AET
 * (one render_entry_3d_object per triangle, "per-triangle submission", SURVEY
 * §0.6); prk_draw_objects submits objects of several triangles, each one AET
 * as FillEdgeTable + DrawModel* build it.  Draws run in submission order and
 * share one z-buffer.
 */
#ifndef PRK_H
#define PRK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRK_MAX_LIGHTS 8

enum prk_status {
    PRK_OK = 0,
    PRK_ERR_ARG = -1,          /* bad pointer / size / handle            */
    PRK_ERR_UNSUPPORTED = -2,  /* combination the reference leaves undefined */
    PRK_ERR_DEVICE = -3,       /* HIP runtime error                      */
    PRK_ERR_NOMEM = -4,        /* device allocation failed               */
    PRK_ERR_NO_TARGET = -5,    /* flush without a render target          */
    PRK_ERR_LIMIT = -6,        /* beyond this build's index capacity (more than
                                  2^31 edges, span slots or bin entries in one
                                  pass): a limit of the build, not of the input */
    PRK_ERR_RUNTIME_MIX = -7   /* two copies of the ROCm runtime are mapped in
                                  this process (e.g. /opt/rocm's, pulled in by
                                  this library, and torch's own, loaded after
                                  it): see prk_create */
};

/* Which of the reference's span kernels a draw reproduces. */
enum prk_semantics {
    PRK_SEM_SCALAR = 0,  /* DrawModel            projekt.cpp:162-601   */
    PRK_SEM_AVX = 1,     /* FillLineOptimized    projekt.cpp:1492-2320, driven by
                            DrawModelOptimized(RenderQueue,...) 3615-3871, or by
                            DrawModelOptimizedLines 3362-3613 (FillLinesOptimized
                            629-1490 has the same block math) */
    PRK_SEM_AVX_ST = 2   /* the single-thread overload DrawModelOptimized(Buffer,...)
                            2350-3358: FillLineOptimized's math with two quirks:
                            a left-clipped span keeps XOffset = -0.0f (2508) and the
                            z-test is z >= zbuf (predicate 29, 3205): among equal z
                            the latest fragment wins */
};

/* Texture sampling of a texture handle (prk_texture_set_filter).  The
 * reference samples the nearest texel only (projekt.cpp:1881-2032);
 * PRK_FILTER_BILINEAR is an EXTENSION of this build for the AVX semantics
 * (BASELINE config 4) with its own definition: weights from
 * texel centres at +0.5, clamp to the edge, fp32.  DrawModel (scalar)
 * draws always sample nearest. */
enum prk_filter {
    PRK_FILTER_NEAREST = 0,
    PRK_FILTER_BILINEAR = 1
};

/* projective_transform (absent header; fields as used at projekt.cpp:77-90,
 * 122-141, 152-155). */
typedef struct prk_transform {
    float DistanceAboveTarget;
    float FocalLength;
    float MetersToPixels;
    float ScreenCenter[2];
} prk_transform;

/* light_info / light_data (absent header; projekt.cpp:452-484, 2046-2128,
 * 3885, 4025-4061). */
typedef struct prk_light_info {
    float P[3];
    float Intensity[4]; /* r g b a */
} prk_light_info;

typedef struct prk_light_data {
    uint32_t LightCount;
    float AmbientIntensity[4]; /* r g b a */
    prk_light_info Lights[PRK_MAX_LIGHTS];
} prk_light_data;

/* loaded_bitmap (absent header): 0xAARRGGBB texels, Pitch in bytes.  For a
 * texture, Memory holds Height rows; the library appends the zeroed "guard"
 * row the reference's u==1 / v==1 over-read lands on (SURVEY App. A.2.3,
 * prk_texture_create below). */
typedef struct prk_bitmap {
    void *Memory;
    int32_t Width;
    int32_t Height;
    int32_t Pitch;
} prk_bitmap;

/* Frame statistics.  Kernel times come from HIP events recorded on the
 * launch stream around the binning and raster kernels of every flush; they
 * are harvested without stalling the stream and accumulated until
 * prk_timing_reset. */
typedef struct prk_stats {
    uint64_t triangles;      /* triangles of the last flush            */
    uint64_t bin_entries;    /* (triangle, tile) pairs of the last flush */
    uint32_t tiles;          /* tiles in the render target band        */
    uint32_t frames_timed;   /* flushes accumulated in sum_ms_*        */
    float ms_bin;            /* last flush: project/cull/bin kernels   */
    float ms_raster;         /* last flush: k_vis + shading kernels    */
    double sum_ms_bin;       /* accumulated since prk_timing_reset     */
    double sum_ms_raster;
    uint32_t anomalies;      /* triangles whose AET left the proven
                                per-triangle shape (always 0) */
    uint32_t slow_replays;   /* bin entries whose rows above their tile were
                                replayed row by row (irregular edge list or
                                an X tie); cumulative like
                                anomalies */
    double sum_ms_vis;       /* accumulated: the k_vis (visibility) part
                                of sum_ms_raster */
    double sum_ms_span;      /* accumulated: the k_walk part (AVX frames:
                                raster = k_vis + k_walk + k_pix) */
    uint32_t objects_chunked; /* large objects (48+ triangles) whose AET walk
                                 ran as chunks of rows walked at once, each
                                 from its first row's sorted list, checked and
                                 walked again where that was not the true
                                 list; cumulative */
    uint32_t objects_walked;  /* large objects walked row after row from the
                                 first (an odd row, a NaN key, lists past the
                                 LDS); cumulative */
    uint32_t object_chunks;   /* the chunked walk's chunks; cumulative */
    uint32_t object_chunks_rewalked; /* ... walked a second time (their start
                                 was not the true list); cumulative */
} prk_stats;

typedef struct prk_context prk_context;

/* Library / device lifetime.
 * prk_create checks that the process maps ONE copy of libamdhip64 and of
 * librocm_smi64.  A host that loads this library (and so /opt/rocm's
 * runtime, plus its RCCL once prk_comm_* runs) before a framework that ships
 * its own copies under other names (torch) ends up with two; their
 * librocm_smi64 copies then free one interposed static map twice at exit
 * (glibc "double free", SIGABRT).  prk_create returns
 * PRK_ERR_RUNTIME_MIX then, names the fix on stderr (load the framework
 * before libprk_hip.so), and guards the exit: an on_exit handler registered
 * after both copies' destructors flushes stdio and ends the process with its
 * own exit status before those destructors run.  The guard skips every
 * exit handler registered before it (atexit/on_exit work, earlier libraries'
 * static destructors) -- work the double-free abort would skip as well;
 * PRK_EXIT_GUARD=0 in the environment leaves the exit path untouched.
 * prk_destroy and prk_comm_init run the same check (and install the same
 * guard). */
int prk_create(int device, prk_context **out);
/* prk_destroy queues no GPU work: it waits for the context's streams and frees
 * what the context owns.  A frame whose bin count is still unresolved (prk_flush
 * returned, nothing has read the count since) is DROPPED, not re-run: if its
 * entries overflowed the scratch, a caller-owned target (prk_target_bind) is
 * left with the frame's cleared or partial contents.  A caller that reads its
 * own target after destroying the context calls prk_synchronize (or
 * prk_resolve) first. */
int prk_destroy(prk_context *ctx);
/* The check alone: PRK_OK, or PRK_ERR_RUNTIME_MIX (guard installed). */
int prk_runtime_check(void);
int prk_device_count(int *out);
const char *prk_version(void);

/* Render target: device memory owned by the caller (e.g. a torch tensor) or
 * by the library (prk_target_alloc).  The target covers frame rows
 * [row0, row1) of a frame `height` rows tall; `color` and `zbuf` point at
 * frame row row0.  z-buffer row stride is `width` floats (Commands->Width,
 * projekt.cpp:170,1511); colour row stride is `pitch_bytes`.
 * A target for the AVX semantics needs width % 8 == 0 (the reference's
 * aligned 8-wide z load, projekt.cpp:2218). */
int prk_target_bind(prk_context *ctx, void *color, int32_t pitch_bytes, float *zbuf,
                    int32_t width, int32_t height, int32_t row0, int32_t row1);
int prk_target_alloc(prk_context *ctx, int32_t width, int32_t height, int32_t row0,
                     int32_t row1, void **color_out, float **zbuf_out);
/* Fill the bound target: colour with `color`, z with `z` (reference callers
 * clear z to -FLT_MAX). */
int prk_target_clear(prk_context *ctx, uint32_t color, float z);
/* The same fill, fused into the next prk_flush: the frame's kernels take
 * (color, z) as the target's prior contents and write every pixel of the
 * target (the winners shaded, the rest the fill values), so no separate
 * fill pass runs.  Frames that do not shade through span records (scalar or
 * mixed semantics) and empty flushes fill first, on the flush's stream. */
int prk_target_clear_on_flush(prk_context *ctx, uint32_t color, float z);
/* Copy the bound target to/from host memory (rows [row0,row1)). */
int prk_target_download(prk_context *ctx, uint32_t *color_host, int32_t host_pitch_bytes,
                        float *z_host);
/* Early z (off by default; the drop-in header turns it on): in frames shaded
 * through span records (all-AVX semantics, per triangle) the visibility
 * kernel writes the final z and the shading only the colour, so
 * prk_target_download copies z while the frame still shades (C3b through
 * projekt.h: 0.45 ms less per frame over PCIe).  It costs a frame that is not
 * downloaded ~0.4 % (the z stores move to the frame's busiest kernel).  The
 * result is the same bit for bit (a -0.0 z, which the visibility key holds
 * as +0.0, is written by the shading and makes the download take z again). */
int prk_set_early_z(prk_context *ctx, int on);
int prk_target_upload(prk_context *ctx, const uint32_t *color_host, int32_t host_pitch_bytes,
                      const float *z_host);
/* prk_target_upload on the context's copy stream: returns at once; the next
 * prk_flush's kernels wait for it.  The host buffers must be page-locked
 * (prk_host_register) and stay unchanged until prk_target_download or
 * prk_synchronize returns (the drop-in sends the caller's framebuffer this
 * way at a frame's first draw, so the copy overlaps the caller's calls). */
int prk_target_upload_async(prk_context *ctx, const uint32_t *color_host, int32_t host_pitch, const float *z_host);

/* Pinned host memory for staging (prk_host_alloc / prk_host_free), and
 * page-locking of caller memory (a framebuffer, a z-buffer) so uploads and
 * downloads run as DMA at full PCIe rate.  Allocations of 2 MB and more are
 * heap memory on transparent huge pages, page-locked for every device
 * (cheaper for the CPU to fill than 4-KB pinned pages;
 * PRK_HOST_ALLOC_THP=0 turns this off).  Free with prk_host_free only. */
int prk_host_alloc(prk_context *ctx, size_t bytes, void **out);
int prk_host_free(prk_context *ctx, void *p);
int prk_host_register(prk_context *ctx, void *p, size_t bytes);
int prk_host_unregister(prk_context *ctx, void *p);

/* Camera and lights (game_render_commands::Transform / LightData) of the
 * draws executed by the next prk_flush, for both what FillEdgeTable reads
 * (ProjectVertex 3906-3910, Gouraud vertex lighting 4020-4063) and what the
 * span kernels read (Phong + UnprojectVertex: DrawModel 452-458,
 * FillLineOptimized 2042-2046, the single-thread overload 3030-3034). */
int prk_set_camera(prk_context *ctx, const prk_transform *transform,
                   const prk_light_data *lights);
/* After prk_set_camera: the span shading (Phong lighting and unprojection)
 * of the next flush uses (transform, lights) instead, the setup keeps
 * prk_set_camera's.  The reference's FillEdgeTable and DrawModel* each read
 * Commands when they run, so a caller that changes Commands between an
 * object's FillEdgeTable and its DrawModel* call gets the setup of the first
 * and the shading of the second; the drop-in passes them this way.  (For the
 * queue overload the spans run on workers that read Commands as they go,
 * 2042-2046; the drop-in uses Commands as they are at the DrawModel* call.)
 * PRK_ERR_ARG before any prk_set_camera. */
int prk_set_shade_camera(prk_context *ctx, const prk_transform *transform,
                         const prk_light_data *lights);

/* Textures.  `bitmap->Memory` is host memory of Height rows of Pitch bytes
 * (loaded_bitmap as the reference reads it, projekt.cpp:1506, 1881-1935); the
 * library appends the zeroed guard row the u == 1 / v == 1 over-read lands
 * on and never reads past the caller's last row.
 * Returns a handle >= 0.  prk_texture_update re-reads a bitmap into a handle
 * (the drop-in refreshes every texture once per frame). */
int prk_texture_create(prk_context *ctx, const prk_bitmap *bitmap, int32_t *handle_out);
int prk_texture_update(prk_context *ctx, int32_t handle, const prk_bitmap *bitmap);
int prk_texture_set_filter(prk_context *ctx, int32_t handle, int32_t filter);  /* PRK_FILTER_* */

/* Geometry: non-indexed SoA vertex arrays exactly as render_entry_3d_object
 * (projekt.h:2-15): positions v3, colours v4, normals v3, uvs v2, three
 * vertices per triangle.  Copied to HBM once; a draw references a range. */
int prk_geometry_create(prk_context *ctx, const float *vertices, const float *colors,
                        const float *normals, const float *uvs, uint32_t vertex_count,
                        int32_t *handle_out);
/* New contents for a library-owned geometry (grows its buffers if needed);
 * an array passed as NULL keeps its previous contents (vertices past them
 * read as zero); draws already recorded read the new contents.  Waits for
 * frames in flight; synchronous. */
int prk_geometry_update(prk_context *ctx, int32_t handle, const float *vertices, const float *colors,
                        const float *normals, const float *uvs, uint32_t vertex_count);
/* Asynchronous partial update: vertices [first_vertex, first_vertex +
 * vertex_count) of the arrays given (NULL: that array unchanged there) are
 * copied on the context's copy stream, after the frames already flushed have
 * read the geometry and before the next prk_flush's kernels read it.  The
 * geometry's vertex count becomes first_vertex + vertex_count; buffers grow
 * (kept contents, zeros past them) when needed, which waits for the device.
 * The host arrays must be page-locked (prk_host_alloc / prk_host_register)
 * and stay unchanged until prk_synchronize or prk_target_download returns.
 * The drop-in streams FillEdgeTable's vertices this way while the caller is
 * still submitting objects.  first_vertex and vertex_count are multiples of 3. */
int prk_geometry_write(prk_context *ctx, int32_t handle, uint32_t first_vertex, uint32_t vertex_count,
                       const float *vertices, const float *colors, const float *normals, const float *uvs);
/* Same as prk_geometry_create, but from device pointers the caller keeps
 * alive (no copy). */
int prk_geometry_wrap_device(prk_context *ctx, const float *vertices, const float *colors,
                             const float *normals, const float *uvs, uint32_t vertex_count,
                             int32_t *handle_out);

/* Record one draw: triangles [first_tri, first_tri+tri_count) of a geometry,
 * object offset P (render_entry_3d_object::P), semantics PRK_SEM_*,
 * PhongShading flag, texture handle (-1 = no Bitmap).
 * PRK_SEM_AVX requires a texture and PhongShading != 0: the reference
 * dereferences Bitmap unconditionally (projekt.cpp:1506) and its non-Phong
 * branch writes garbage (projekt.cpp:2285-2316). */
int prk_draw(prk_context *ctx, int32_t geometry, uint32_t first_tri, uint32_t tri_count,
             const float P[3], int32_t semantics, int32_t phong, int32_t texture);
/* The same draw as consecutive render_entry_3d_objects of `tris_per_object`
 * triangles each (the last one may be smaller): every object is ONE active
 * edge table, as FillEdgeTable + DrawModelOptimized(RenderQueue,...) build it
 * (projekt.cpp:3894-4117, 3654-3869), so spans pair edges of different
 * triangles of the object.  tris_per_object == 1 is prk_draw.  Objects of
 * more than one triangle are supported for every semantics (DrawModel's
 * AET, 162-601, has the same list logic), of any size: the active edge list
 * has no length limit (a wave walks it in LDS, or in device memory once it
 * outgrows LDS).  The edges are set up as FillEdgeTable(Object, Commands,
 * phong) does for an object whose Bitmap is set iff texture >= 0. */
int prk_draw_objects(prk_context *ctx, int32_t geometry, uint32_t first_tri, uint32_t tri_count,
                     uint32_t tris_per_object, const float P[3], int32_t semantics, int32_t phong,
                     int32_t texture);

/* FillEdgeTable's own inputs, which shape the edge records independently of
 * the later DrawModel* call (projekt.cpp:3882-4121):
 *   PRK_SETUP_PHONG   its PhongShading argument != 0: raw vertex colours and
 *                     normals (4012-4019); 0: per-vertex Gouraud lighting
 *                     (4020-4063) and no normals;
 *   PRK_SETUP_BITMAP  Object->Bitmap != 0: the lighting starts from white
 *                     (4034-4054) and the U/V/(1/z) gradients are set
 *                     (4078-4089); 0: no gradients.
 * prk_draw_objects_setup draws with explicit setup flags (setup < 0: derived
 * from the draw, as prk_draw_objects).  Combinations the reference leaves
 * undefined are PRK_ERR_UNSUPPORTED: a Phong draw (any semantics) of edges
 * set up without PRK_SETUP_PHONG (MinNormal never written, 4012-4064), and a
 * textured draw of edges set up without PRK_SETUP_BITMAP (UGradient,
 * VGradient, OneOverZGradient never written, 4078-4089).  So
 * FillEdgeTable(..., 1) + DrawModel(..., Bitmap = 0, Phong = 0) interpolates
 * the raw colours unlit, and an object with a Bitmap drawn by
 * DrawModel(..., Bitmap = 0, Phong = 0) after FillEdgeTable(..., 0) gets the
 * white-based lighting. */
enum prk_setup {
    PRK_SETUP_PHONG = 1,
    PRK_SETUP_BITMAP = 2
};
int prk_draw_objects_setup(prk_context *ctx, int32_t geometry, uint32_t first_tri, uint32_t tri_count,
                           uint32_t tris_per_object, const float P[3], int32_t semantics, int32_t phong,
                           int32_t texture, int32_t setup);

/* edge_info (projekt.h:17-37) without its list pointer: what the reference's
 * FillEdgeTable leaves in EdgeMemory and DrawModel* walk.  prk_draw_edges
 * draws one object from such a list, already sorted by YMin as FillEdgeTable
 * leaves it, exactly as DrawModelOptimized(RenderQueue,...) (3615-3871), the
 * single-thread overload (2350-3358) or DrawModel (162-601, PRK_SEM_SCALAR)
 * walks it.  The winner id of its pixels is the draw's position in the
 * frame's triangle numbering (it counts as one). */
typedef struct prk_edge {
    int32_t YMax;
    float XMin, ZMin, OneOverZMin, Gradient, ZGradient, OneOverZGradient;
    int32_t YMin;
    float UMin, VMin, UGradient, VGradient;
    int32_t Left;
    float MinColor[4], ColorGradient[4], MinNormal[3], NormalGradient[3];
} prk_edge;
int prk_draw_edges(prk_context *ctx, const prk_edge *edges, uint32_t edge_count, int32_t semantics, int32_t phong,
                   int32_t texture);

/* One span end as line_render_work carries it by value (projekt.h:65-74) or
 * thread_edge_info holds it (39-63): what FillLineOptimized /
 * FillLinesOptimized read of an edge (1543-1835; 648-670). */
typedef struct prk_span_end {
    float XMin, ZMin, OneOverZMin, UMin, VMin;
    float MinColor[4];
    float MinNormal[3];
} prk_span_end;
typedef struct prk_span {
    prk_span_end Left, Right;
    int32_t Row;
} prk_span;
/* Draw caller-built spans (the work records DoLineRenderWork /
 * DoBufferLineRenderWork run, 2336-2348), in order, each with
 * FillLineOptimized's span body.  Each span counts as one triangle id. */
int prk_draw_spans(prk_context *ctx, const prk_span *spans, uint32_t count, int32_t semantics, int32_t phong,
                   int32_t texture);

/* Execute every recorded draw, in submission order, into the bound target
 * (the reference's Platform.CompleteAllWork).  `stream` is a hipStream_t or
 * NULL for the library's own stream.  Asynchronous w.r.t. the host: it
 * returns once the frame is queued, without waiting for its binning.  The
 * frame's bin entry count (scratch sizing, prk_stats.bin_entries) is read by
 * the next call that needs it: the next prk_flush, prk_synchronize,
 * prk_resolve, prk_target_download / upload / clear, prk_get_stats, a texture
 * or geometry update, a gather, prk_target_alloc, or prk_target_bind (any
 * target: rebinding waits on the host for the previous frame's count, so a
 * caller rotating its own buffers pays that wait at the bind).  A frame whose entries overflowed the scratch is
 * re-run there, into the target and with the camera, tile and clear it was
 * queued with, before anything else is queued — so a caller that reads the
 * target through its own device pointers (not prk_target_download) after a
 * flush calls prk_synchronize first.  (The first frame of a context is
 * counted at once.) */
int prk_flush(prk_context *ctx, void *stream);
/* Drop recorded draws without executing them. */
int prk_reset_draws(prk_context *ctx);
int prk_synchronize(prk_context *ctx);
/* Resolve the last flush's pending bin count (re-running an overflowed frame,
 * as above) and make `stream` (a hipStream_t of the context's device, or NULL
 * for none) wait for the end of the context's last frame, without blocking
 * the host on the frame's raster.  For callers that read the target through
 * their own device pointers on their own stream (a torch RCCL strip gather):
 * the asynchronous counterpart of prk_synchronize. */
int prk_resolve(prk_context *ctx, void *stream);
int prk_get_stats(prk_context *ctx, prk_stats *out); /* waits for timed flushes */
int prk_timing_reset(prk_context *ctx);

/* Debug/test: per-pixel winning triangle index of the last flush (-1 = none),
 * rows [row0,row1).  Requires prk_set_debug(ctx, 1) before the flush. */
int prk_set_debug(prk_context *ctx, int32_t enable);
int prk_download_winners(prk_context *ctx, int32_t *winners_host);
/* Debug: the raster kernels' phase cycle counters (written only by builds
 * with -DPRK_PROF; zeroed by prk_timing_reset), n <= 16. */
int prk_debug_counters(prk_context *ctx, uint64_t *out, int32_t n);

/* Test: the raster kernels divide several values by one divisor through a
 * shared reciprocal; this checks n hashed (x, d) draws and
 * normalisations on `device` against the compiler's own division, bit for
 * bit.  *mismatches = quotient mismatches | normalisation mismatches << 32. */
int prk_selftest_div(int32_t device, uint32_t n, uint64_t seed, uint64_t *mismatches);

/* The bound target (any pointer may be NULL) and the context's device and
 * own stream (a hipStream_t; prk_flush(ctx, NULL) runs on it). */
int prk_get_target(prk_context *ctx, void **color, int32_t *pitch_bytes, float **zbuf, int32_t *width,
                   int32_t *height, int32_t *row0, int32_t *row1);
int prk_get_device(prk_context *ctx, int32_t *device, void **stream);

/* ---- Multi-GPU: row bands and the frame gather ------------
 * The reference has no distribution; this is the build's.  Rank r of N binds
 * (or allocates) a target for frame rows prk_band_rows(H, r, N) and records
 * the same draws as every other rank: each rank bins all triangles against
 * its band, so every pixel has one owner and submission order holds.  The
 * only exchange is the gather of the band strips into one frame on rank 0
 * (colour, and z when with_z).  A caller that wants the frame in host memory
 * needs no gather: each rank downloads its band into its rows.
 *
 * One process per GPU: RCCL over xGMI.  Rank 0 makes a unique id
 * (PRK_COMM_ID_BYTES bytes), the caller hands it to every rank (its own
 * channel: MPI, a socket, torch.distributed ...), and every rank creates its
 * communicator with prk_comm_init.  librccl is loaded on first use;
 * PRK_ERR_UNSUPPORTED when it is absent (prk_comm_available() == 0). */
#define PRK_COMM_ID_BYTES 128
typedef struct prk_comm prk_comm;
int prk_band_rows(int32_t height, int32_t rank, int32_t nranks, int32_t *row0, int32_t *row1);
int prk_comm_available(void);
int prk_comm_unique_id(void *id);
int prk_comm_init(prk_context *ctx, const void *id, int32_t nranks, int32_t rank, prk_comm **out);
/* One process driving N GPUs: one communicator per context (ncclCommInitAll). */
int prk_comm_init_all(prk_context *const *ctxs, int32_t n, prk_comm **comms_out);
int prk_comm_destroy(prk_comm *comm);
/* Every rank's band into rank 0's device frame (W x H; colour rows of
 * frame_pitch == 4*W bytes, z rows of W floats).  Rank 0 passes the frame,
 * other ranks pass NULL (their bands must be packed: pitch 4*W).  Enqueued on
 * `stream` (NULL: the context's own stream) after the work already there;
 * rank 0's own band is copied unless its target is the frame's slice. */
int prk_gather_frame(prk_context *ctx, prk_comm *comm, int32_t with_z, void *frame_color, int32_t frame_pitch,
                     float *frame_z, void *stream);
/* The same for N contexts of one process, as one RCCL group (ctxs[r] and
 * comms[r] are rank r; each rank's ops go on its context's own stream). */
int prk_gather_frame_all(prk_context *const *ctxs, prk_comm *const *comms, int32_t n, int32_t with_z,
                         void *frame_color, int32_t frame_pitch, float *frame_z);
/* One process driving N GPUs without RCCL: each band's device copies its
 * strip into ctxs[0]'s frame over xGMI (peer access), after the work on its
 * own stream; ctxs[0]'s own stream waits for every copy (prk_synchronize on
 * ctxs[0] waits for the whole frame).  Contexts may share a device. */
int prk_gather_frame_local(prk_context *const *ctxs, int32_t n, int32_t with_z, void *frame_color,
                           int32_t frame_pitch, float *frame_z);

/* Tunables (testing / benchmarking). tile_w must be a power of two >= 8,
 * 64 <= tile_w * tile_h <= 8192.  Without a call the context picks its tile
 * itself: 256x8, or 32x8 / 64x8 once a frame shows fewer than 64 / 8 bin
 * entries per 256x8 tile, or 512x8 once an all-AVX frame shows 4.5 or more
 * entries a triangle (large triangles; a band: per its share of the
 * triangles), kept while the triangle count and the band stay within 2x.
 * Results never depend on the tile. */
int prk_set_tile(prk_context *ctx, int32_t tile_w, int32_t tile_h);

/* Host utility: FillEdgeTable's return value (projekt.cpp:3882-4121, 4119)
 * for one object of vertex_count vertices (positions v3, three per
 * triangle) at offset P (may be NULL: 0) under transform T: the number of
 * edges of its front-facing triangles (3926-3943) with MaxY > 0 (3968) and
 * MinY != MaxY (4066), 0 for an object that draws nothing.  The drop-in's
 * FillEdgeTable returns it at the call; the setup runs on the GPU. */
int prk_fill_edge_count(const float *vertices, uint32_t vertex_count, const float P[3],
                        const prk_transform *transform, uint32_t *count_out);

/* Host utilities: edge_info records in the caller's own memory (the drop-in's
 * opt-in record mode, projekt.h PRK_SetEdgeRecords).  The frame never comes
 * from these: the GPU sets objects up from their vertices (prk_draw_objects)
 * and draws edge lists from their copies (prk_draw_edges).  They reproduce
 * what the reference leaves in the caller's memory, in place: `edges` is an
 * array of elements of `stride` bytes whose first 108 bytes are edge_info's
 * 27 fields in prk_edge order and whose list pointer (edge_info.Next) sits at
 * byte `next_offset` (x86-64 edge_info: stride 120, next_offset 112).  A field
 * the reference does not write keeps the caller's bytes.
 *
 * prk_fill_edge_records: FillEdgeTable (projekt.cpp:3894-4117) of one object
 * of vertex_count vertices at offset P under T / L, with its own PhongShading
 * and Bitmap != 0 as PRK_SETUP_* bits in `setup`: the visible edges written
 * at edges[0 ..), Next = NULL, then MergeSort (2-72) with sort_memory
 * (Commands->SortMemory, >= count elements; NULL: a library buffer) as its
 * scratch.  *count_out = FillEdgeTable's return value (4119). */
int prk_fill_edge_records(const float *vertices, const float *colors, const float *normals, const float *uvs,
                          uint32_t vertex_count, const float P[3], const prk_transform *transform,
                          const prk_light_data *lights, int32_t setup, void *edges, size_t stride,
                          size_t next_offset, void *sort_memory, uint32_t *count_out);
/* prk_advance_edge_records: what DrawModel* (every overload: the same list
 * walk and edge step, 3654-3869, 3811-3829) leaves in the list it drew over a
 * frame of `height` rows: every edge stepped once per row it was paired on,
 * the list pointers as the walk left them (real addresses into `edges`).
 * The reference's crashes are pinned as the draw pins them (prk.h above): a
 * first-pair swap moves the list head (P3), an emptied list skips the row. */
int prk_advance_edge_records(void *edges, uint32_t count, size_t stride, size_t next_offset, int32_t height);

/* Host utility: the reference's test mesh, ConstructSphere
 * (projekt.cpp:4123-4289).  Arrays must hold 6624 vertices; returns the
 * vertex count through *count_out. */
int prk_construct_sphere(float *vertices, float *colors, float *normals, float *uvs,
                         uint32_t *count_out);

#ifdef __cplusplus
}
#endif

#endif /* PRK_H */
