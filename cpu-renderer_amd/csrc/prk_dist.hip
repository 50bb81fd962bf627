// prk_dist.hip — multi-GPU row bands and the frame gather.
//
// A frame is split into N row bands, rank r rendering rows
// [r*H/N, (r+1)*H/N) with its own context (every rank records the same draws
// and bins all triangles against its band, so each pixel has one owner and
// submission order is kept).  The only exchange on the path is the gather of
// the band strips into one frame on rank 0:
//   * one process per GPU: RCCL point-to-point over xGMI (ncclSend / ncclRecv
//     inside one group, every strip received straight into its slice of rank
//     0's frame; one message per peer, each on its own link);
//   * one process driving N GPUs: the same gather through RCCL communicators
//     of ncclCommInitAll, or as peer copies (each band's device writes its
//     strip into rank 0's frame over xGMI, rank 0's stream waits for them).
// librccl is loaded on first use (dlopen), so the library itself has no RCCL
// dependency; a process that already holds librccl.so.1 (torch) shares it.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>  // types only; the functions come from dlopen

#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/prk.h"

static_assert(PRK_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

extern "C" int prk_resolve_pending(prk_context *c, void *stream);  // prk_api.hip (library-internal)
namespace {

struct Rccl {
    bool ok = false;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
};

template <class F>
bool sym(void *h, const char *name, F &f) {
    f = reinterpret_cast<F>(dlsym(h, name));
    return f != nullptr;
}

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
        if (!h) return;
        r.ok = sym(h, "ncclGetUniqueId", r.GetUniqueId) && sym(h, "ncclCommInitRank", r.CommInitRank) &&
               sym(h, "ncclCommInitAll", r.CommInitAll) && sym(h, "ncclCommDestroy", r.CommDestroy) &&
               sym(h, "ncclSend", r.Send) && sym(h, "ncclRecv", r.Recv) && sym(h, "ncclGroupStart", r.GroupStart) &&
               sym(h, "ncclGroupEnd", r.GroupEnd);
    });
    return r;
}

int nstat(ncclResult_t e) { return e == ncclSuccess ? PRK_OK : PRK_ERR_DEVICE; }
int hstat(hipError_t e) {
    if (e == hipSuccess) return PRK_OK;
    return e == hipErrorOutOfMemory ? PRK_ERR_NOMEM : PRK_ERR_DEVICE;
}

void band(int32_t H, int32_t r, int32_t n, int32_t &a, int32_t &b) {
    a = (int32_t)((int64_t)H * r / n);
    b = (int32_t)((int64_t)H * (r + 1) / n);
}

// One rank's bound band, checked against prk_band_rows.
struct Band {
    void *color;
    float *z;
    int32_t pitch, W, H, row0, row1, device;
    hipStream_t stream;
};

// `stream`: the stream the band's strip is read on (NULL: the context's own);
// it is made to wait for the end of the band's last frame — whatever stream
// that frame (or its deferred re-run, queued here first) ran on.
int band_of(prk_context *ctx, int32_t rank, int32_t nranks, Band &B, void *stream = nullptr) {
    void *s = nullptr;
    int rc = prk_get_device(ctx, &B.device, &s);
    if (rc != PRK_OK) return rc;
    B.stream = stream ? (hipStream_t)stream : (hipStream_t)s;
    rc = prk_resolve_pending(ctx, (void *)B.stream);
    if (rc != PRK_OK) return rc;
    rc = prk_get_target(ctx, &B.color, &B.pitch, &B.z, &B.W, &B.H, &B.row0, &B.row1);
    if (rc != PRK_OK) return rc;
    int32_t a, b;
    band(B.H, rank, nranks, a, b);
    if (B.row0 != a || B.row1 != b) return PRK_ERR_ARG;  // the target is not this rank's band
    return PRK_OK;
}

// Rank 0's own strip into its frame slice (nothing when it IS the slice).
hipError_t own_copy(const Band &B, int32_t with_z, void *frame_color, int32_t frame_pitch, float *frame_z,
                    hipStream_t s) {
    uint8_t *dc = (uint8_t *)frame_color + (size_t)B.row0 * frame_pitch;
    const int32_t rows = B.row1 - B.row0;
    hipError_t e = hipSuccess;
    if (dc != B.color)
        e = hipMemcpy2DAsync(dc, frame_pitch, B.color, B.pitch, (size_t)B.W * 4, rows, hipMemcpyDeviceToDevice, s);
    float *dz = frame_z + (size_t)B.row0 * B.W;
    if (e == hipSuccess && with_z && dz != B.z)
        e = hipMemcpyAsync(dz, B.z, (size_t)B.W * rows * 4, hipMemcpyDeviceToDevice, s);
    return e;
}

// The point-to-point operations of one rank (inside the caller's group).
int gather_ops(const Rccl &R, prk_comm *comm, const Band &B, int32_t with_z, void *frame_color,
               int32_t frame_pitch, float *frame_z, hipStream_t s);

}  // namespace

struct prk_comm {
    ncclComm_t comm = nullptr;
    int32_t rank = 0, nranks = 1, device = 0;
};

namespace {
int gather_ops(const Rccl &R, prk_comm *comm, const Band &B, int32_t with_z, void *frame_color,
               int32_t frame_pitch, float *frame_z, hipStream_t s) {
    const size_t W = (size_t)B.W;
    if (comm->rank == 0) {
        for (int32_t r = 1; r < comm->nranks; ++r) {
            int32_t a, b;
            band(B.H, r, comm->nranks, a, b);
            const size_t n = W * (size_t)(b - a);
            if (!n) continue;
            int rc = nstat(R.Recv((uint8_t *)frame_color + (size_t)a * frame_pitch, n, ncclUint32, r, comm->comm, s));
            if (rc == PRK_OK && with_z) rc = nstat(R.Recv(frame_z + (size_t)a * W, n, ncclFloat32, r, comm->comm, s));
            if (rc != PRK_OK) return rc;
        }
        return PRK_OK;
    }
    const size_t n = W * (size_t)(B.row1 - B.row0);
    if (!n) return PRK_OK;
    int rc = nstat(R.Send(B.color, n, ncclUint32, 0, comm->comm, s));
    if (rc == PRK_OK && with_z) rc = nstat(R.Send(B.z, n, ncclFloat32, 0, comm->comm, s));
    return rc;
}

// Frame checks on rank 0 (strips are received as packed rows).
bool frame_ok(const Band &B, void *frame_color, int32_t frame_pitch, int32_t with_z, float *frame_z) {
    return frame_color && frame_pitch == B.W * 4 && (!with_z || frame_z);
}
}  // namespace

extern "C" {

int prk_band_rows(int32_t height, int32_t rank, int32_t nranks, int32_t *row0, int32_t *row1) {
    if (height <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || !row0 || !row1) return PRK_ERR_ARG;
    band(height, rank, nranks, *row0, *row1);
    return PRK_OK;
}

int prk_comm_available(void) { return rccl().ok ? 1 : 0; }

int prk_comm_unique_id(void *id) {
    if (!id) return PRK_ERR_ARG;
    const Rccl &R = rccl();
    if (!R.ok) return PRK_ERR_UNSUPPORTED;
    return nstat(R.GetUniqueId(reinterpret_cast<ncclUniqueId *>(id)));
}

int prk_comm_init(prk_context *ctx, const void *id, int32_t nranks, int32_t rank, prk_comm **out) {
    {  // librccl (and its librocm_smi64) beside another framework's copies
        const int rc = prk_runtime_check();
        if (rc != PRK_OK) return rc;
    }
    if (!ctx || !id || !out || nranks <= 0 || rank < 0 || rank >= nranks) return PRK_ERR_ARG;
    *out = nullptr;
    const Rccl &R = rccl();
    if (!R.ok) return PRK_ERR_UNSUPPORTED;
    int32_t dev = 0;
    int rc = prk_get_device(ctx, &dev, nullptr);
    if (rc != PRK_OK) return rc;
    rc = hstat(hipSetDevice(dev));
    if (rc != PRK_OK) return rc;
    prk_comm *c = new (std::nothrow) prk_comm();
    if (!c) return PRK_ERR_NOMEM;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    rc = nstat(R.CommInitRank(&c->comm, nranks, uid, rank));
    if (rc != PRK_OK) {
        delete c;
        return rc;
    }
    c->rank = rank;
    c->nranks = nranks;
    c->device = dev;
    *out = c;
    return PRK_OK;
}

int prk_comm_init_all(prk_context *const *ctxs, int32_t n, prk_comm **out) {
    if (!ctxs || !out || n <= 0) return PRK_ERR_ARG;
    const Rccl &R = rccl();
    if (!R.ok) return PRK_ERR_UNSUPPORTED;
    std::vector<int> devs((size_t)n);
    for (int32_t r = 0; r < n; ++r) {
        out[r] = nullptr;
        int32_t d = 0;
        int rc = ctxs[r] ? prk_get_device(ctxs[r], &d, nullptr) : PRK_ERR_ARG;
        if (rc != PRK_OK) return rc;
        devs[(size_t)r] = d;
    }
    std::vector<ncclComm_t> comms((size_t)n, nullptr);
    int rc = nstat(R.CommInitAll(comms.data(), n, devs.data()));
    if (rc != PRK_OK) return rc;
    for (int32_t r = 0; r < n; ++r) {
        prk_comm *c = new (std::nothrow) prk_comm();
        if (!c) {
            for (int32_t k = 0; k < n; ++k) {
                if (k < r) delete out[k];
                out[k] = nullptr;
                (void)R.CommDestroy(comms[(size_t)k]);
            }
            return PRK_ERR_NOMEM;
        }
        c->comm = comms[(size_t)r];
        c->rank = r;
        c->nranks = n;
        c->device = devs[(size_t)r];
        out[r] = c;
    }
    return PRK_OK;
}

int prk_comm_destroy(prk_comm *comm) {
    if (!comm) return PRK_ERR_ARG;
    const Rccl &R = rccl();
    int rc = PRK_OK;
    if (R.ok && comm->comm) rc = nstat(R.CommDestroy(comm->comm));
    delete comm;
    return rc;
}

int prk_gather_frame(prk_context *ctx, prk_comm *comm, int32_t with_z, void *frame_color, int32_t frame_pitch,
                     float *frame_z, void *stream) {
    if (!ctx || !comm) return PRK_ERR_ARG;
    const Rccl &R = rccl();
    if (!R.ok) return PRK_ERR_UNSUPPORTED;
    Band B;
    int rc = band_of(ctx, comm->rank, comm->nranks, B, stream);
    if (rc != PRK_OK) return rc;
    if (comm->rank == 0 && !frame_ok(B, frame_color, frame_pitch, with_z, frame_z)) return PRK_ERR_ARG;
    if (comm->rank != 0 && B.pitch != B.W * 4) return PRK_ERR_UNSUPPORTED;  // strips go out as packed rows
    hipStream_t s = B.stream;
    rc = hstat(hipSetDevice(B.device));
    if (rc != PRK_OK) return rc;
    if (comm->rank == 0) {
        rc = hstat(own_copy(B, with_z, frame_color, frame_pitch, frame_z, s));
        if (rc != PRK_OK) return rc;
    }
    rc = nstat(R.GroupStart());
    if (rc != PRK_OK) return rc;
    rc = gather_ops(R, comm, B, with_z, frame_color, frame_pitch, frame_z, s);
    const int rc2 = nstat(R.GroupEnd());
    return rc != PRK_OK ? rc : rc2;
}

int prk_gather_frame_all(prk_context *const *ctxs, prk_comm *const *comms, int32_t n, int32_t with_z,
                         void *frame_color, int32_t frame_pitch, float *frame_z) {
    if (!ctxs || !comms || n <= 0) return PRK_ERR_ARG;
    const Rccl &R = rccl();
    if (!R.ok) return PRK_ERR_UNSUPPORTED;
    std::vector<Band> bands((size_t)n);
    for (int32_t r = 0; r < n; ++r) {
        if (!ctxs[r] || !comms[r] || comms[r]->rank != r || comms[r]->nranks != n) return PRK_ERR_ARG;
        int rc = band_of(ctxs[r], r, n, bands[(size_t)r]);
        if (rc != PRK_OK) return rc;
        if (r > 0 && bands[(size_t)r].pitch != bands[(size_t)r].W * 4) return PRK_ERR_UNSUPPORTED;
    }
    if (!frame_ok(bands[0], frame_color, frame_pitch, with_z, frame_z)) return PRK_ERR_ARG;
    int rc = hstat(hipSetDevice(bands[0].device));
    if (rc == PRK_OK) rc = hstat(own_copy(bands[0], with_z, frame_color, frame_pitch, frame_z, bands[0].stream));
    if (rc != PRK_OK) return rc;
    rc = nstat(R.GroupStart());
    if (rc != PRK_OK) return rc;
    for (int32_t r = 0; r < n && rc == PRK_OK; ++r)
        rc = gather_ops(R, comms[r], bands[(size_t)r], with_z, frame_color, frame_pitch, frame_z,
                        bands[(size_t)r].stream);
    const int rc2 = nstat(R.GroupEnd());
    return rc != PRK_OK ? rc : rc2;
}

int prk_gather_frame_local(prk_context *const *ctxs, int32_t n, int32_t with_z, void *frame_color,
                           int32_t frame_pitch, float *frame_z) {
    if (!ctxs || n <= 0) return PRK_ERR_ARG;
    std::vector<Band> bands((size_t)n);
    for (int32_t r = 0; r < n; ++r) {
        if (!ctxs[r]) return PRK_ERR_ARG;
        int rc = band_of(ctxs[r], r, n, bands[(size_t)r]);
        if (rc != PRK_OK) return rc;
    }
    const Band &B0 = bands[0];
    if (!frame_color || frame_pitch < B0.W * 4 || (with_z && !frame_z)) return PRK_ERR_ARG;
    for (int32_t r = 0; r < n; ++r) {
        const Band &B = bands[(size_t)r];
        if (B.W != B0.W || B.H != B0.H) return PRK_ERR_ARG;
        int rc = hstat(hipSetDevice(B.device));
        if (rc != PRK_OK) return rc;
        if (B.device != B0.device) {
            hipError_t e = hipDeviceEnablePeerAccess(B0.device, 0);
            if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            else if (e != hipSuccess) return PRK_ERR_UNSUPPORTED;  // no xGMI / PCIe peer path
        }
        // The strip's device writes it into rank 0's frame (after its flush,
        // on the stream the flush ran on); rank 0's stream waits for it.
        rc = hstat(own_copy(B, with_z, frame_color, frame_pitch, frame_z, B.stream));
        if (rc != PRK_OK) return rc;
        if (r > 0) {
            hipEvent_t ev = nullptr;
            hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventRecord(ev, B.stream);
            if (e == hipSuccess) e = hipSetDevice(B0.device);
            if (e == hipSuccess) e = hipStreamWaitEvent(B0.stream, ev, 0);
            if (ev) (void)hipEventDestroy(ev);
            if (e != hipSuccess) return hstat(e);
        }
    }
    return PRK_OK;
}

}  // extern "C"
