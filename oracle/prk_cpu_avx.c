/*
 * prk_cpu_avx.c — the AVX2 CPU baseline of bench.py.
 *
 *   TEST INFRASTRUCTURE ONLY, like prk_oracle.c: only tests/ and bench.py's
 *   cpu_baseline leg load liborcpu.so.  The product never links or calls it.
 *
 *   It is prk_oracle.c (setup, MergeSort, AET: compiled in below, unchanged)
 *   with FillLineOptimized (projekt.cpp:1492-2320) restated 8 lanes wide in
 *   AVX2 the way the reference computes it, op for op in the order of the
 *   scalar restatement or_fill_line_optimized (no FMA: built without -mfma
 *   and with -ffp-contract=off; _mm256_div_ps / _mm256_sqrt_ps are IEEE).
 *   tests/test_cpu_baseline.py requires its frames to equal the scalar
 *   oracle's bit for bit.
 *
 *   Two schedules, both timed by bench.py (SURVEY §8(d) "CPU path timing"):
 *   * banded (cpu_avx_draw_banded): 32-row bands, thread t owns bands
 *     b % threads == t, every thread walks the triangles meeting its bands in
 *     submission order; no locks; deterministic.
 *   * queue (cpu_avx_draw_queue), the reference's own schedule: one producer
 *     runs FillEdgeTable + the AET of DrawModelOptimized(RenderQueue,...)
 *     (projekt.cpp:3615-3871) and posts one work record per span (both edges
 *     by value + row, 3759-3809) to a lock-free queue; workers run the span
 *     and take the per-8-pixel ZMask byte spinlock around the z-test/store
 *     (2211-2237).  The producer drains the queue with the workers once it is
 *     done (Platform.CompleteAllWork).  Strict `z > zbuf` makes the result
 *     independent of the order spans run in, except for exactly equal z
 *     (the earlier fragment wins sequentially, whichever runs first here).
 *   * rows (cpu_avx_draw_rows): DrawModelOptimizedLines (3362-3613) +
 *     FillLinesOptimized (629-1490): the same producer AET, but every row of
 *     an object becomes ONE task carrying the row's span end points
 *     (thread_edge_info: left/right X, z, 1/z, U, V, normal; projekt.h:39-63,
 *     3518-3544) and a worker fills the row's spans in order under the same
 *     ZMask spinlock.  FillLinesOptimized's block math is FillLineOptimized's
 *     (SURVEY §2 #12), so the frame is identical; only the task grain differs.
 */
#include <immintrin.h>
#include <stdatomic.h>
#include <stdint.h>

struct or_ctx;
struct or_edge;
static void cpu_fill_line_avx2(struct or_ctx *X_, const struct or_edge *L, const struct or_edge *R, int32_t Row);
#define OR_AVX_SPAN cpu_fill_line_avx2
#include "prk_oracle.c"

/* Per-worker hooks of the queue schedule: the ZMask spinlock array. */
typedef struct cpu_lockset {
    atomic_uchar *ZMask; /* one byte per 8 pixels of the frame (projekt.cpp:2211) */
    int32_t Width;
} cpu_lockset;
static _Thread_local const cpu_lockset *tl_locks = NULL;

static inline __m256 v8(float a) { return _mm256_set1_ps(a); }

/* NormalizeVector_8x (projekt.cpp:603-620): x / sqrt((x*x + y*y) + z*z). */
static inline void v_normalize_div(__m256 *x, __m256 *y, __m256 *z)
{
    __m256 len = _mm256_sqrt_ps(_mm256_add_ps(_mm256_add_ps(_mm256_mul_ps(*x, *x), _mm256_mul_ps(*y, *y)),
                                              _mm256_mul_ps(*z, *z)));
    *x = _mm256_div_ps(*x, len);
    *y = _mm256_div_ps(*y, len);
    *z = _mm256_div_ps(*z, len);
}

/* min(1, max(0, a)) with MINPS/MAXPS operand order (or_minps(1, or_maxps(0, a))). */
static inline __m256 v_sat_lo(__m256 a) { return _mm256_min_ps(v8(1.0f), _mm256_max_ps(v8(0.0f), a)); }
/* or_maxps(or_minps(a, 1), 0): the final clamp (2129-2133). */
static inline __m256 v_sat_hi(__m256 a) { return _mm256_max_ps(_mm256_min_ps(a, v8(1.0f)), v8(0.0f)); }

static inline __m256 v_chan(__m256i t, int sh)
{
    __m256i b = _mm256_and_si256(_mm256_srli_epi32(t, sh), _mm256_set1_epi32(0xFF));
    return _mm256_div_ps(_mm256_cvtepi32_ps(b), v8(255.0f));
}

/* FillLineOptimized, 8 lanes (projekt.cpp:1492-2283); span setup is the
 * scalar restatement's (or_fill_line_optimized), the block loop is AVX2. */
static void cpu_fill_line_avx2(or_ctx *X_, const or_edge *L, const or_edge *R, int32_t Row)
{
    if (!or_owns(X_, Row)) return;
    const prk_bitmap *Bm = X_->Bitmap;
    const prk_transform *T = X_->T;
    const int32_t W = X_->Width;
    float XOffset = 0.0f;
    if (Row < 0) return;

    float LeftX = L->XMin; /* 1545-1565 */
    if (LeftX < 0) { XOffset = -L->XMin; LeftX = 0; }
    else if (LeftX >= W) LeftX = (float)W - 1;
    float RightX = R->XMin;
    if (RightX < 0) RightX = 0;
    else if (RightX >= W) RightX = (float)W - 1;
    if (LeftX != LeftX || RightX != RightX) return;

    int32_t CLP = or_round_s32(L->XMin), CRP = or_round_s32(R->XMin); /* 1568-1570 */
    int32_t XDiff = (int32_t)((uint32_t)CRP - (uint32_t)CLP);
    LeftX = (float)or_round_s32(LeftX);
    RightX = (float)or_round_s32(RightX);
    int32_t MinX = (int32_t)LeftX, MaxX = (int32_t)RightX;

    __m256i lane = _mm256_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7);
    __m256i Start = _mm256_set1_epi32(-1), End = _mm256_set1_epi32(-1);
    if (MinX & 7) { /* 1594-1609 */
        Start = _mm256_cmpgt_epi32(lane, _mm256_set1_epi32((MinX & 7) - 1));
        LeftX = (float)(MinX & ~7);
        XOffset -= (float)(MinX & 7) * 1.0f;
    }
    if (MaxX & 7) { /* 1611-1624 */
        End = _mm256_cmpgt_epi32(_mm256_set1_epi32(MaxX & 7), lane);
        RightX = (float)((MaxX & ~7) + 8);
    }
    if ((LeftX + 8) >= RightX) Start = _mm256_and_si256(Start, End); /* 1627-1664 */

    if (MaxX > MinX) X_->SpanPixels += (uint64_t)(MaxX - MinX);
    X_->Spans++;

    float fXD = (float)XDiff; /* 1666-1835 */
    float IncW = 0, IncU = 0, IncV = 0, IncN[3] = {0, 0, 0}, IncZ = 0;
    if (XDiff != 0) {
        IncW = (R->OneOverZMin - L->OneOverZMin) / fXD;
        IncU = (R->UMin - L->UMin) / fXD;
        IncV = (R->VMin - L->VMin) / fXD;
        for (int c = 0; c < 3; ++c) IncN[c] = (R->MinNormal[c] - L->MinNormal[c]) / fXD;
        IncZ = (R->ZMin - L->ZMin) / fXD;
    }
    const __m256 o = _mm256_add_ps(v8(XOffset), _mm256_setr_ps(0, 1, 2, 3, 4, 5, 6, 7));
    __m256 Wl = _mm256_add_ps(v8(L->OneOverZMin), _mm256_mul_ps(o, v8(IncW)));
    __m256 Ul = _mm256_add_ps(v8(L->UMin), _mm256_mul_ps(o, v8(IncU)));
    __m256 Vl = _mm256_add_ps(v8(L->VMin), _mm256_mul_ps(o, v8(IncV)));
    __m256 Nx = _mm256_add_ps(v8(L->MinNormal[0]), _mm256_mul_ps(o, v8(IncN[0])));
    __m256 Ny = _mm256_add_ps(v8(L->MinNormal[1]), _mm256_mul_ps(o, v8(IncN[1])));
    __m256 Nz = _mm256_add_ps(v8(L->MinNormal[2]), _mm256_mul_ps(o, v8(IncN[2])));
    v_normalize_div(&Nx, &Ny, &Nz); /* 1754 */
    __m256 Zl = _mm256_add_ps(v8(L->ZMin), _mm256_mul_ps(o, v8(IncZ)));
    const __m256 IncW8 = v8(IncW * 8.0f), IncU8 = v8(IncU * 8.0f), IncV8 = v8(IncV * 8.0f);
    const __m256 IncNx8 = v8(IncN[0] * 8.0f), IncNy8 = v8(IncN[1] * 8.0f), IncNz8 = v8(IncN[2] * 8.0f);
    const __m256 IncZ8 = v8(8.0f * IncZ);

    const __m256 Tw = v8((float)Bm->Width), Th = v8((float)Bm->Height);
    const float InvM2P = 1.0f / T->MetersToPixels;
    const __m256i Pitch = _mm256_set1_epi32(Bm->Pitch);
    const __m256i Limit = _mm256_set1_epi32((int32_t)((int64_t)Bm->Pitch * (Bm->Height + 1) - 4));
    const __m256 Amb0 = v8(X_->Lights->AmbientIntensity[0]), Amb1 = v8(X_->Lights->AmbientIntensity[1]);
    const __m256 Amb2 = v8(X_->Lights->AmbientIntensity[2]), Amb3 = v8(X_->Lights->AmbientIntensity[3]);
    const __m256 DF = v8(T->DistanceAboveTarget), F = v8(T->FocalLength);
    const float AY = ((float)Row + 0.0f - T->ScreenCenter[1]) * InvM2P;
    __m256i Clip = Start;

    uint32_t *rowp = (uint32_t *)((uint8_t *)X_->Color + (size_t)Row * X_->Pitch);
    float *zrow = X_->Z + (size_t)Row * W;
    const int32_t X0 = (int32_t)LeftX, X1 = (int32_t)RightX;
    for (int32_t X = X0; X < X1; X += 8) { /* 1858 */
        __m256 IW = _mm256_div_ps(v8(1.0f), Wl);
        __m256 FU = _mm256_mul_ps(IW, Ul), FV = _mm256_mul_ps(IW, Vl);
        __m256 M = _mm256_and_ps(_mm256_and_ps(_mm256_cmp_ps(FU, v8(0.0f), _CMP_GE_OQ),
                                               _mm256_cmp_ps(FU, v8(1.0f), _CMP_LE_OQ)),
                                 _mm256_and_ps(_mm256_cmp_ps(FV, v8(0.0f), _CMP_GE_OQ),
                                               _mm256_cmp_ps(FV, v8(1.0f), _CMP_LE_OQ)));
        __m256i Mask = _mm256_and_si256(_mm256_castps_si256(M), Clip);
        int mbits = _mm256_movemask_ps(_mm256_castsi256_ps(Mask));
        if (mbits) {
            __m256 CA, CR, CG, CB;
            if (X_->Filter == PRK_FILTER_BILINEAR) { /* extension: per lane, the restatement's sampler */
                float fu[8], fv[8], a[8], r[8], g[8], b[8];
                _mm256_storeu_ps(fu, FU);
                _mm256_storeu_ps(fv, FV);
                for (int i = 0; i < 8; ++i) {
                    a[i] = r[i] = g[i] = b[i] = 0.0f;
                    if (mbits >> i & 1) or_bilinear(Bm, fu[i], fv[i], &a[i], &r[i], &g[i], &b[i]);
                }
                CA = _mm256_loadu_ps(a); CR = _mm256_loadu_ps(r);
                CG = _mm256_loadu_ps(g); CB = _mm256_loadu_ps(b);
            } else { /* 1881-2032: trunc(Tw*u)*4 + mul16(trunc(Th*v), Pitch), P2 clamp */
                __m256i FX = _mm256_slli_epi32(_mm256_cvttps_epi32(_mm256_mul_ps(Tw, FU)), 2);
                __m256i TY = _mm256_cvttps_epi32(_mm256_mul_ps(Th, FV));
                __m256i FY = _mm256_or_si256(_mm256_mullo_epi16(TY, Pitch),
                                             _mm256_slli_epi32(_mm256_mulhi_epi16(TY, Pitch), 16));
                __m256i Off = _mm256_add_epi32(FX, FY);
                __m256i Bad = _mm256_or_si256(_mm256_cmpgt_epi32(_mm256_setzero_si256(), Off),
                                              _mm256_cmpgt_epi32(Off, Limit));
                Off = _mm256_andnot_si256(Bad, Off);
                __m256i Tx = _mm256_mask_i32gather_epi32(_mm256_setzero_si256(), (const int *)Bm->Memory, Off,
                                                         Mask, 1);
                CA = v_chan(Tx, 24); CR = v_chan(Tx, 16); CG = v_chan(Tx, 8); CB = v_chan(Tx, 0);
            }
            /* Phong (2040-2128) with UnprojectVertex_8x (102-145). */
            __m256 d = _mm256_sub_ps(DF, Zl);
            __m256 Xf = _mm256_add_ps(v8((float)X), _mm256_setr_ps(0, 1, 2, 3, 4, 5, 6, 7));
            __m256 AX = _mm256_mul_ps(_mm256_sub_ps(Xf, v8(T->ScreenCenter[0])), v8(InvM2P));
            __m256 dF = _mm256_div_ps(d, F);
            __m256 PX = _mm256_mul_ps(dF, AX), PY = _mm256_mul_ps(dF, v8(AY)), PZ = Zl;
            __m256 Fr = v8(0), Fg = v8(0), Fb = v8(0), Fa = v8(0);
            for (uint32_t li = 0; li < X_->Lights->LightCount; ++li) {
                const prk_light_info *Lt = &X_->Lights->Lights[li];
                if (li == 0) {
                    Fr = _mm256_mul_ps(CR, Amb0); Fg = _mm256_mul_ps(CG, Amb1);
                    Fb = _mm256_mul_ps(CB, Amb2); Fa = _mm256_mul_ps(CA, Amb3);
                }
                __m256 Lx = _mm256_sub_ps(v8(Lt->P[0]), PX), Ly = _mm256_sub_ps(v8(Lt->P[1]), PY);
                __m256 Lz = _mm256_sub_ps(v8(Lt->P[2]), PZ);
                v_normalize_div(&Lx, &Ly, &Lz);
                __m256 Cos = v_sat_lo(_mm256_add_ps(_mm256_add_ps(_mm256_mul_ps(Nx, Lx), _mm256_mul_ps(Ny, Ly)),
                                                    _mm256_mul_ps(Nz, Lz)));
                __m256 Vx = _mm256_sub_ps(v8(0), PX), Vy = _mm256_sub_ps(v8(0), PY), Vz = _mm256_sub_ps(v8(0), PZ);
                v_normalize_div(&Vx, &Vy, &Vz);
                __m256 Hx = _mm256_add_ps(Lx, Vx), Hy = _mm256_add_ps(Ly, Vy), Hz = _mm256_add_ps(Lz, Vz);
                v_normalize_div(&Hx, &Hy, &Hz);
                __m256 Ph = v_sat_lo(_mm256_add_ps(_mm256_add_ps(_mm256_mul_ps(Nx, Hx), _mm256_mul_ps(Ny, Hy)),
                                                   _mm256_mul_ps(Nz, Hz)));
                for (int f = 0; f < 4; ++f) Ph = _mm256_mul_ps(Ph, Ph);
#define PRK_ACC(Fc, Cc, k)                                                                             \
    Fc = _mm256_add_ps(Fc, _mm256_add_ps(_mm256_mul_ps(Cos, _mm256_mul_ps(Cc, v8(Lt->Intensity[k]))), \
                                         _mm256_mul_ps(Ph, v8(1.0f * Lt->Intensity[k]))))
                PRK_ACC(Fr, CR, 0); PRK_ACC(Fg, CG, 1); PRK_ACC(Fb, CB, 2); PRK_ACC(Fa, CA, 3);
#undef PRK_ACC
            }
            Fr = v_sat_hi(Fr); Fg = v_sat_hi(Fg); Fb = v_sat_hi(Fb); Fa = v_sat_hi(Fa);
            __m256i Packed = _mm256_or_si256(
                _mm256_or_si256(_mm256_slli_epi32(_mm256_cvtps_epi32(_mm256_mul_ps(Fr, v8(255.0f))), 16),
                                _mm256_slli_epi32(_mm256_cvtps_epi32(_mm256_mul_ps(Fg, v8(255.0f))), 8)),
                _mm256_or_si256(_mm256_cvtps_epi32(_mm256_mul_ps(Fb, v8(255.0f))),
                                _mm256_slli_epi32(_mm256_cvtps_epi32(_mm256_mul_ps(Fa, v8(255.0f))), 24)));
            /* z-test GT_OQ and masked store (2202-2239), under the ZMask lock
             * in the queue schedule. */
            atomic_uchar *lk = NULL;
            if (tl_locks) {
                lk = tl_locks->ZMask + ((size_t)Row * (size_t)tl_locks->Width + (size_t)X) / 8;
                unsigned char exp = 0;
                while (!atomic_compare_exchange_weak_explicit(lk, &exp, 1, memory_order_acquire,
                                                              memory_order_relaxed)) {
                    exp = 0;
                    _mm_pause();
                }
            }
            __m256 zb = _mm256_loadu_ps(zrow + X);
            __m256i Wm = _mm256_and_si256(_mm256_castps_si256(_mm256_cmp_ps(Zl, zb, _CMP_GT_OQ)), Mask);
            int wbits = _mm256_movemask_ps(_mm256_castsi256_ps(Wm));
            if (wbits) {
                _mm256_storeu_ps(zrow + X, _mm256_blendv_ps(zb, Zl, _mm256_castsi256_ps(Wm)));
                __m256i cold = _mm256_loadu_si256((const __m256i *)(rowp + X));
                _mm256_storeu_si256((__m256i *)(rowp + X), _mm256_blendv_epi8(cold, Packed, Wm));
                if (X_->Winners)
                    for (int i = 0; i < 8; ++i)
                        if (wbits >> i & 1) X_->Winners[(size_t)Row * W + X + i] = X_->TriIndex;
                X_->Writes += (uint64_t)__builtin_popcount((unsigned)wbits);
            }
            if (lk) atomic_store_explicit(lk, 0, memory_order_release);
        }
        /* Next clip mask (2241-2256), then the block step (2262-2282). */
        Clip = ((X + 16) < RightX) ? _mm256_set1_epi32(-1) : End;
        __m256 a = _mm256_add_ps(Nx, IncNx8), b = _mm256_add_ps(Ny, IncNy8), c = _mm256_add_ps(Nz, IncNz8);
        v_normalize_div(&a, &b, &c);
        Nx = a; Ny = b; Nz = c;
        Zl = _mm256_add_ps(Zl, IncZ8);
        Wl = _mm256_add_ps(Wl, IncW8);
        Ul = _mm256_add_ps(Ul, IncU8);
        Vl = _mm256_add_ps(Vl, IncV8);
    }
}

/* ---------------------------------------------------------------------- */
/* Banded schedule: prk_oracle.c's oracle_draw_mt with the AVX2 span.      */
/* ---------------------------------------------------------------------- */
int cpu_avx_draw_banded(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                        const prk_light_data *Lights, int32_t threads, uint64_t *stats)
{
    return oracle_draw_mt(D, Tg, T, Lights, threads, stats);
}

int cpu_avx_draw(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                 const prk_light_data *Lights, uint64_t *stats)
{
    return oracle_draw(D, Tg, T, Lights, stats);
}

/* ---------------------------------------------------------------------- */
/* Queue schedule (the reference's): producer AET -> span records -> workers */
/* ---------------------------------------------------------------------- */
typedef struct cpu_work { /* line_render_work: both edges by value + row (3759-3809) */
    or_edge L, R;
    int32_t Row, TriIndex;
    int32_t NPairs;          /* rows schedule: pairs of the row's task (0: one span in L/R) */
    int32_t First;           /* rows schedule: first pair in the pair ring */
} cpu_work;

/* rows schedule: span end points of one pair (thread_edge_info, projekt.h:39-63) */
typedef struct cpu_pair {
    float LX, RX, LZ, RZ, LW, RW, LU, RU, LV, RV, LN[3], RN[3];
} cpu_pair;
#define CPU_PBITS 20
#define CPU_PSIZE (1u << CPU_PBITS)

#define CPU_QBITS 16
#define CPU_QSIZE (1u << CPU_QBITS)
typedef struct cpu_queue { /* single producer, many consumers, bounded ring */
    cpu_work *Slots;
    cpu_pair *Pairs;                /* rows schedule: pair ring (CPU_PSIZE) */
    atomic_uint_fast64_t *Seq;      /* per slot: the ticket it is ready for */
    _Alignas(64) atomic_uint_fast64_t Head; /* next ticket to post */
    _Alignas(64) atomic_uint_fast64_t Tail; /* next ticket to take */
    _Alignas(64) atomic_int Done;
    _Alignas(64) atomic_int Running;  /* rows schedule: tasks taken and not yet finished */
} cpu_queue;

typedef struct cpu_qctx {
    cpu_queue *Q;
    or_ctx Base;            /* target, transform, lights, bitmap */
    const cpu_lockset *Locks;
    uint64_t stats[3];
} cpu_qctx;

static _Thread_local cpu_queue *tl_post_q = NULL;
static _Thread_local or_ctx *tl_exec = NULL; /* the producer's span-running context */

/* Take one posted span and run it; 0 when none is ready. */
static int cpu_take_one(cpu_queue *Q, or_ctx *X_)
{
    for (;;) {
        uint64_t t = atomic_load_explicit(&Q->Tail, memory_order_relaxed);
        size_t i = t & (CPU_QSIZE - 1);
        uint64_t s = atomic_load_explicit(&Q->Seq[i], memory_order_acquire);
        if (s == t + 1) {
            if (!atomic_compare_exchange_weak_explicit(&Q->Tail, &t, t + 1, memory_order_relaxed,
                                                       memory_order_relaxed))
                continue;
            cpu_work w = Q->Slots[i];
            if (w.NPairs == 0) {
                atomic_store_explicit(&Q->Seq[i], t + CPU_QSIZE, memory_order_release);
                X_->TriIndex = w.TriIndex;
                cpu_fill_line_avx2(X_, &w.L, &w.R, w.Row);
                return 1;
            }
            /* FillLinesOptimized (629-1490): the row's pairs in order, each
             * rebuilt as an edge pair from its end points (648-670).  The pair
             * slots stay owned by this task until Running drops. */
            atomic_fetch_add_explicit(&Q->Running, 1, memory_order_acq_rel);
            atomic_store_explicit(&Q->Seq[i], t + CPU_QSIZE, memory_order_release);
            X_->TriIndex = w.TriIndex;
            for (int32_t k = 0; k < w.NPairs; ++k) {
                const cpu_pair *p = &Q->Pairs[(uint32_t)(w.First + k) & (CPU_PSIZE - 1)];
                or_edge L, R;
                memset(&L, 0, sizeof L);
                memset(&R, 0, sizeof R);
                L.XMin = p->LX; R.XMin = p->RX; L.ZMin = p->LZ; R.ZMin = p->RZ;
                L.OneOverZMin = p->LW; R.OneOverZMin = p->RW; L.UMin = p->LU; R.UMin = p->RU;
                L.VMin = p->LV; R.VMin = p->RV;
                for (int c = 0; c < 3; ++c) { L.MinNormal[c] = p->LN[c]; R.MinNormal[c] = p->RN[c]; }
                cpu_fill_line_avx2(X_, &L, &R, w.Row);
            }
            atomic_fetch_sub_explicit(&Q->Running, 1, memory_order_acq_rel);
            return 1;
        }
        if (s < t + 1) return 0; /* empty */
        /* s > t + 1: another consumer took ticket t meanwhile; reload */
    }
}

/* Claim the next ring slot (the producer runs queued tasks itself while the
 * ring is full, so one thread, or slow workers, cannot deadlock it). */
static cpu_work *cpu_claim(cpu_queue *Q, uint64_t *ticket)
{
    uint64_t t = atomic_load_explicit(&Q->Head, memory_order_relaxed);
    size_t i = t & (CPU_QSIZE - 1);
    while (atomic_load_explicit(&Q->Seq[i], memory_order_acquire) != t)
        if (!cpu_take_one(Q, tl_exec)) _mm_pause();
    *ticket = t;
    return &Q->Slots[i];
}

static void cpu_publish(cpu_queue *Q, uint64_t t)
{
    atomic_store_explicit(&Q->Seq[t & (CPU_QSIZE - 1)], t + 1, memory_order_release);
    atomic_store_explicit(&Q->Head, t + 1, memory_order_release);
}

static void cpu_post_span(or_ctx *X_, const or_edge *L, const or_edge *R, int32_t Row)
{
    uint64_t t;
    cpu_work *w = cpu_claim(tl_post_q, &t);
    w->L = *L;
    w->R = *R;
    w->Row = Row;
    w->TriIndex = X_->TriIndex;
    w->NPairs = 0;
    cpu_publish(tl_post_q, t);
}

/* rows schedule producer: the AET walk hands over its spans one at a time, in
 * row order; the spans of one row are gathered and posted as one task
 * (3518-3609) when the row changes or the object ends. */
typedef struct cpu_rowbuf {
    int32_t Row, Tri, N, First;
    uint32_t Next;       /* pair ring write position */
    uint64_t TaskBase;   /* first ring ticket of the pending pair run */
} cpu_rowbuf;
static _Thread_local cpu_rowbuf tl_row;

static void cpu_row_flush(void)
{
    if (tl_row.N == 0) return;
    uint64_t t;
    cpu_work *w = cpu_claim(tl_post_q, &t);
    w->Row = tl_row.Row;
    w->TriIndex = tl_row.Tri;
    w->NPairs = tl_row.N;
    w->First = tl_row.First;
    cpu_publish(tl_post_q, t);
    tl_row.N = 0;
}

static void cpu_post_row_pair(or_ctx *X_, const or_edge *L, const or_edge *R, int32_t Row)
{
    cpu_queue *Q = tl_post_q;
    if (tl_row.N && (Row != tl_row.Row || tl_row.N >= 1000)) cpu_row_flush(); /* ThreadEdges[1000] */
    /* The pair ring wraps only when no task holds pair slots: the producer
     * helps drain the queue, then waits for the tasks still running. */
    if (tl_row.Next + 1000u > CPU_PSIZE && tl_row.N == 0) {
        while (atomic_load_explicit(&Q->Tail, memory_order_acquire) !=
               atomic_load_explicit(&Q->Head, memory_order_acquire))
            if (!cpu_take_one(Q, tl_exec)) _mm_pause();
        while (atomic_load_explicit(&Q->Running, memory_order_acquire) != 0) _mm_pause();
        tl_row.Next = 0;
    }
    if (tl_row.N == 0) { tl_row.Row = Row; tl_row.Tri = X_->TriIndex; tl_row.First = (int32_t)tl_row.Next; }
    cpu_pair *p = &Q->Pairs[tl_row.Next & (CPU_PSIZE - 1)];
    tl_row.Next++;
    p->LX = L->XMin; p->RX = R->XMin; p->LZ = L->ZMin; p->RZ = R->ZMin;
    p->LW = L->OneOverZMin; p->RW = R->OneOverZMin; p->LU = L->UMin; p->RU = R->UMin;
    p->LV = L->VMin; p->RV = R->VMin;
    for (int c = 0; c < 3; ++c) { p->LN[c] = L->MinNormal[c]; p->RN[c] = R->MinNormal[c]; }
    tl_row.N++;
}

/* Take and run spans until the producer is done and the queue is empty. */
static void cpu_drain(cpu_qctx *C, or_ctx *X_, int wait_done)
{
    cpu_queue *Q = C->Q;
    for (;;) {
        if (cpu_take_one(Q, X_)) continue;
        if (!wait_done || atomic_load_explicit(&Q->Done, memory_order_acquire)) {
            /* Done is stored after the last post: empty now means empty for good */
            uint64_t t = atomic_load_explicit(&Q->Tail, memory_order_acquire);
            if (atomic_load_explicit(&Q->Head, memory_order_acquire) == t) return;
        }
        _mm_pause();
    }
}

static void *cpu_worker(void *p)
{
    cpu_qctx *C = (cpu_qctx *)p;
    or_ctx X_ = C->Base;
    tl_locks = C->Locks;
    cpu_drain(C, &X_, 1);
    tl_locks = NULL;
    C->stats[0] = X_.Spans; C->stats[1] = X_.SpanPixels; C->stats[2] = X_.Writes;
    return NULL;
}

static int cpu_avx_draw_tasks(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                              const prk_light_data *Lights, int32_t threads, uint64_t *stats, int rows)
{
    if (!D || !Tg || !T || !Lights) return PRK_ERR_ARG;
    if (D->Semantics != PRK_SEM_AVX || !D->Bitmap || !D->Phong || (Tg->Width % 8)) return PRK_ERR_UNSUPPORTED;
    if (Lights->LightCount > PRK_MAX_LIGHTS) return PRK_ERR_ARG;
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    const int nworkers = threads - 1; /* the producer is the last thread */
    cpu_queue Q;
    memset(&Q, 0, sizeof Q);
    Q.Slots = (cpu_work *)malloc(sizeof(cpu_work) * CPU_QSIZE);
    Q.Seq = (atomic_uint_fast64_t *)malloc(sizeof(atomic_uint_fast64_t) * CPU_QSIZE);
    Q.Pairs = rows ? (cpu_pair *)malloc(sizeof(cpu_pair) * CPU_PSIZE) : NULL;
    size_t nlock = ((size_t)Tg->Width * Tg->Height + 7) / 8;
    atomic_uchar *zm = (atomic_uchar *)calloc(nlock, 1);
    uint32_t per = D->TrisPerObject ? D->TrisPerObject : 1;
    or_edge *Edges = (or_edge *)malloc(sizeof(or_edge) * 3 * per);
    or_edge *Sort = (or_edge *)malloc(sizeof(or_edge) * 3 * per);
    if (!Q.Slots || !Q.Seq || !zm || !Edges || !Sort || (rows && !Q.Pairs)) {
        free(Q.Slots); free(Q.Seq); free(Q.Pairs); free(zm); free(Edges); free(Sort);
        return PRK_ERR_NOMEM;
    }
    for (size_t i = 0; i < CPU_QSIZE; ++i) atomic_init(&Q.Seq[i], i);
    cpu_lockset locks = {zm, Tg->Width};

    or_ctx base;
    memset(&base, 0, sizeof base);
    base.T = T; base.Lights = Lights; base.Bitmap = D->Bitmap;
    base.Color = Tg->Color; base.Pitch = Tg->Pitch; base.Z = Tg->Z;
    base.Width = Tg->Width; base.Height = Tg->Height; base.Winners = Tg->Winners;
    base.RowLo = 0; base.RowHi = Tg->Height; base.Phong = D->Phong; base.Filter = D->Filter;
    base.BandH = 1; base.BandMod = 1; base.BandRem = 0;

    cpu_qctx *ctx = (cpu_qctx *)calloc((size_t)threads, sizeof(cpu_qctx));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    int *started = (int *)calloc((size_t)threads, sizeof(int));
    if (!ctx || !th || !started) {
        free(ctx); free(th); free(started);
        free(Q.Slots); free(Q.Seq); free(Q.Pairs); free(zm); free(Edges); free(Sort);
        return PRK_ERR_NOMEM;
    }
    for (int k = 0; k < threads; ++k) {
        memset(&ctx[k], 0, sizeof ctx[k]);
        ctx[k].Q = &Q; ctx[k].Base = base; ctx[k].Locks = &locks;
    }
    for (int k = 0; k < nworkers; ++k) started[k] = pthread_create(&th[k], NULL, cpu_worker, &ctx[k]) == 0;

    /* Producer: FillEdgeTable + the AET, posting spans (3615-3871). */
    or_ctx P = base;
    cpu_qctx *me = &ctx[threads - 1];
    or_ctx X_ = base;
    tl_post_q = &Q;
    tl_exec = &X_;
    tl_locks = &locks;
    memset(&tl_row, 0, sizeof tl_row);
    for (uint32_t t0 = 0; t0 < D->TriCount; t0 += per) {
        uint32_t n = D->TriCount - t0 < per ? D->TriCount - t0 : per;
        uint32_t ec = or_fill_edge_table(D->Vertices, D->Colors, D->Normals, D->UVs, t0, n, D->P, 1, D->Phong,
                                         or_setup_t(D, T), or_setup_l(D, Lights), Edges, Sort);
        P.TriIndex = D->TriIndexBase + (int32_t)t0;
        or_aet_walk(&P, Edges, ec, rows ? cpu_post_row_pair : cpu_post_span);
        if (rows) cpu_row_flush(); /* the object's last row (3609) */
    }
    tl_post_q = NULL;
    atomic_store_explicit(&Q.Done, 1, memory_order_release);
    /* CompleteAllWork: the producer drains with the workers. */
    cpu_drain(me, &X_, 1);
    tl_exec = NULL;
    tl_locks = NULL;
    me->stats[0] = X_.Spans; me->stats[1] = X_.SpanPixels; me->stats[2] = X_.Writes;
    for (int k = 0; k < nworkers; ++k) {
        if (started[k]) pthread_join(th[k], NULL);
        else cpu_worker(&ctx[k]);
    }
    if (stats)
        for (int k = 0; k < threads; ++k)
            for (int j = 0; j < 3; ++j) stats[j] += ctx[k].stats[j];
    free(Q.Slots); free(Q.Seq); free(Q.Pairs); free(zm); free(Edges); free(Sort);
    free(ctx); free(th); free(started);
    return PRK_OK;
}

int cpu_avx_draw_queue(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                       const prk_light_data *Lights, int32_t threads, uint64_t *stats)
{
    return cpu_avx_draw_tasks(D, Tg, T, Lights, threads, stats, 0);
}

int cpu_avx_draw_rows(const or_draw_desc *D, const or_target *Tg, const prk_transform *T,
                      const prk_light_data *Lights, int32_t threads, uint64_t *stats)
{
    return cpu_avx_draw_tasks(D, Tg, T, Lights, threads, stats, 1);
}

int cpu_avx_supported(void) { return __builtin_cpu_supports("avx2") ? 1 : 0; }
