/*
 * niti_oracle.c -- CPU restatement of the reference NITI int8 training path.
 *
 * TEST INFRASTRUCTURE ONLY (see niti_oracle.h): the checker for tests/, smoke()
 * and bench.py's cpu_baseline leg.  Parity unpinned: no reference fixtures exist
 * and running the reference was denied; anchored by SURVEY.md Appendix A and by
 * agreement of the naive and reference-structured restatements below.
 *
 * Every function cites the reference file:line it restates; paths are relative
 * to execution-engine/ of the reference.
 */
#include "niti_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define UP_DIV(x, y) (((x) + (y)-1) / (y))
#define ALIMIN(a, b) ((a) < (b) ? (a) : (b))
#define ALIMAX(a, b) ((a) > (b) ? (a) : (b))

/* int32 arithmetic with the wrap-around x86-64 executes (the reference's signed
 * overflow in these spots is UB in C; imul/add wrap on the machine it targets). */
static inline int32_t wrap_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t wrap_sub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static inline int32_t wrap_mul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

/* ---------------------------------------------------------------------------- */
/* scalar helpers: source/backend/cpu/compute/CommonOptFunction.cpp:1548-1627   */
/* ---------------------------------------------------------------------------- */

int32_t niti_ref_int8_clip(int32_t a) { /* :1548-1555 */
    if (a > 127) return 127;
    if (a < -127) return -127;
    return a;
}

int32_t niti_ref_sign(int32_t a) { /* :1556-1563 */
    return a > 0 ? 1 : (a < 0 ? -1 : 0);
}

/* (1 << s) for a run-time int s as x86-64 `shl` executes it: the count is taken
 * mod 32 and the result is an int32 bit pattern (1<<31 == INT32_MIN). */
int32_t niti_ref_pow2(int32_t s) { return (int32_t)(1u << ((uint32_t)s & 31u)); }

/* :1565-1576.  max|a| then ceil(log2(max)); in integers: m<=1 -> 0, else the bit
 * length of m-1.  abs(INT32_MIN) is INT32_MIN on x86 (never > the running max). */
int32_t niti_ref_range_estimate(const int32_t* a, int64_t n) {
    int32_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        int32_t v = a[i];
        if (v == INT32_MIN) continue;
        v = v < 0 ? -v : v;
        if (m < v) m = v;
    }
    if (m <= 1) return 0;
    uint32_t t = (uint32_t)(m - 1);
    int bits = 0;
    while (t) {
        ++bits;
        t >>= 1;
    }
    return bits;
}

int32_t niti_ref_range_estimate_libm(const int32_t* a, int64_t n) {
    int32_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        int32_t v = a[i];
        if (v == INT32_MIN) continue;
        v = v < 0 ? -v : v;
        if (m < v) m = v;
    }
    if (m == 0) return 0;
    return (int32_t)ceil(log2((double)m));
}

/* One element of NITI_MNNPstoShiftInt32, :1595-1627 (PSTO defined at :1593). */
int32_t niti_ref_psto1(int32_t a, int32_t shift) {
    const int32_t p = niti_ref_pow2(shift);
    const int32_t q = a / p; /* C division truncates toward zero */
    int32_t prob = wrap_sub(a, wrap_mul(q, p));
    prob = prob < 0 ? -prob : prob;
    const int32_t hp = niti_ref_pow2(shift / 2);
    const int32_t qp = prob / hp;
    int32_t pr = wrap_sub(prob, wrap_mul(qp, hp));
    if (shift % 2 == 1) pr = wrap_mul(pr, 2);
    const int32_t round1 = qp > pr;
    return niti_ref_int8_clip(wrap_add(q, round1 * niti_ref_sign(a)));
}

void niti_ref_psto_shift(const int32_t* in, int32_t shift, int32_t* out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) out[i] = niti_ref_psto1(in[i], shift);
}

/* ---------------------------------------------------------------------------- */
/* requantisation rules                                                          */
/* ---------------------------------------------------------------------------- */

/* NITI_Conv_Int8.cpp:260-307 (and NITI_DeConv_Int8.cpp:294-329, which drops the exponent). */
int32_t niti_ref_requant_fwd(const int32_t* acc, int64_t n, int8_t* out) {
    const int32_t bw = niti_ref_range_estimate(acc, n);
    const int32_t shift = bw - 7;
    if (shift > 1) {
        for (int64_t i = 0; i < n; ++i) out[i] = (int8_t)niti_ref_psto1(acc[i], shift);
        return shift;
    } else if (shift == 1) {
        for (int64_t i = 0; i < n; ++i) out[i] = (int8_t)niti_ref_psto1(acc[i], 2);
        return 2;
    }
    for (int64_t i = 0; i < n; ++i) out[i] = (int8_t)acc[i]; /* raw cast: 128 wraps to -128 */
    return 0;
}

/* NITI_GradientConv_Int8.cpp:272-296 */
int32_t niti_ref_requant_wgrad(const int32_t* acc, int64_t n, int8_t* out) {
    const int32_t bw = niti_ref_range_estimate(acc, n);
    if (bw == 0) {
        memset(out, 0, (size_t)n);
        return 0;
    }
    for (int64_t i = 0; i < n; ++i) out[i] = (int8_t)niti_ref_psto1(acc[i], bw - 2);
    return bw;
}

/* NITI_Matmul_Int8.cpp:214-228 */
int32_t niti_ref_requant_matmul(const int32_t* acc, int64_t n, int8_t* out) {
    const int32_t bw = niti_ref_range_estimate(acc, n);
    if (bw == 0) {
        memset(out, 0, (size_t)n);
        return 0;
    }
    for (int64_t i = 0; i < n; ++i) out[i] = (int8_t)niti_ref_psto1(acc[i], bw - 3);
    return bw;
}

/* ---------------------------------------------------------------------------- */
/* geometry: source/shape/ShapeNITI_Conv_Int8.cpp:41-76 (Caffe pads)             */
/* ---------------------------------------------------------------------------- */

int niti_ref_geom_finalize(niti_ref_geom* g) {
    if (g->stride_h <= 0 || g->stride_w <= 0 || g->dilate_h <= 0 || g->dilate_w <= 0) return -1;
    const int keh = g->dilate_h * (g->kh - 1) + 1;
    const int kew = g->dilate_w * (g->kw - 1) + 1;
    g->oh = (g->h + g->pad_t + g->pad_b - keh) / g->stride_h + 1;
    g->ow = (g->w + g->pad_l + g->pad_r - kew) / g->stride_w + 1;
    return (g->oh > 0 && g->ow > 0) ? 0 : -1;
}

static inline void stat_add(niti_ref_stats* st, int64_t s, int64_t a) {
    if (!st) return;
    if (a >= (1 << 24)) st->guard++;
    if (s > INT32_MAX || s < INT32_MIN) st->overflow++;
}

/* ---------------------------------------------------------------------------- */
/* naive exact-integer restatement                                              */
/* ---------------------------------------------------------------------------- */

/* The naive loops run over contiguous ranges of their outermost index on niti_ref_set_threads()
 * pthreads (default 1); each output is still one exact int64 sum, so the thread count changes
 * nothing but the wall time.  Stats are per-range and summed. */
static int g_naive_threads = 1;
void niti_ref_set_threads(int threads) { g_naive_threads = threads < 1 ? 1 : threads > 256 ? 256 : threads; }

typedef void (*range_fn)(const void* ctx, int64_t b0, int64_t b1, niti_ref_stats* st);
typedef struct {
    range_fn f;
    const void* ctx;
    int64_t b0, b1;
    niti_ref_stats st;
} range_job;
static void* range_worker(void* p) {
    range_job* J = (range_job*)p;
    J->f(J->ctx, J->b0, J->b1, &J->st);
    return NULL;
}
static void par_range(int64_t n, range_fn f, const void* ctx, niti_ref_stats* st) {
    int t = g_naive_threads;
    if (t > n) t = n > 0 ? (int)n : 1;
    range_job jobs[256];
    pthread_t tids[256];
    for (int i = 0; i < t; ++i) {
        jobs[i].f = f;
        jobs[i].ctx = ctx;
        jobs[i].b0 = n * i / t;
        jobs[i].b1 = n * (i + 1) / t;
        jobs[i].st.guard = jobs[i].st.overflow = 0;
    }
    if (t == 1) {
        range_worker(&jobs[0]);
    } else {
        for (int i = 0; i < t; ++i) pthread_create(&tids[i], NULL, range_worker, &jobs[i]);
        for (int i = 0; i < t; ++i) pthread_join(tids[i], NULL);
    }
    if (st)
        for (int i = 0; i < t; ++i) {
            st->guard += jobs[i].st.guard;
            st->overflow += jobs[i].st.overflow;
        }
}

typedef struct {
    const niti_ref_geom* g;
    const int8_t *a, *b;
    int32_t* acc;
} conv_ctx;

static void fwd_range(const void* c, int64_t b0, int64_t b1, niti_ref_stats* st) {
    const conv_ctx* C = (const conv_ctx*)c;
    const niti_ref_geom* g = C->g;
    const int8_t *x = C->a, *w = C->b;
    for (int64_t r = b0; r < b1; ++r) { /* r = n * c_out + co */
        const int n = (int)(r / g->c_out), co = (int)(r % g->c_out);
        for (int oy = 0; oy < g->oh; ++oy)
            for (int ox = 0; ox < g->ow; ++ox) {
                int64_t s = 0, a = 0;
                for (int ci = 0; ci < g->c_in; ++ci)
                    for (int ky = 0; ky < g->kh; ++ky) {
                        const int iy = oy * g->stride_h - g->pad_t + ky * g->dilate_h;
                        if (iy < 0 || iy >= g->h) continue;
                        for (int kx = 0; kx < g->kw; ++kx) {
                            const int ix = ox * g->stride_w - g->pad_l + kx * g->dilate_w;
                            if (ix < 0 || ix >= g->w) continue;
                            const int32_t p = (int32_t)x[(((int64_t)n * g->c_in + ci) * g->h + iy) * g->w + ix] *
                                              (int32_t)w[(((int64_t)co * g->c_in + ci) * g->kh + ky) * g->kw + kx];
                            s += p;
                            a += p < 0 ? -p : p;
                        }
                    }
                stat_add(st, s, a);
                C->acc[(((int64_t)n * g->c_out + co) * g->oh + oy) * g->ow + ox] = (int32_t)(uint32_t)s;
            }
    }
}

void niti_ref_conv_fwd_acc(const niti_ref_geom* g, const int8_t* x, const int8_t* w, int32_t* acc,
                           niti_ref_stats* st) {
    const conv_ctx c = {g, x, w, acc};
    par_range((int64_t)g->n * g->c_out, fwd_range, &c, st);
}

static void wgrad_range(const void* c, int64_t b0, int64_t b1, niti_ref_stats* st) {
    const conv_ctx* C = (const conv_ctx*)c;
    const niti_ref_geom* g = C->g;
    const int8_t *x = C->a, *dy = C->b;
    for (int64_t r = b0; r < b1; ++r) { /* r = co * c_in + ci */
        const int co = (int)(r / g->c_in), ci = (int)(r % g->c_in);
        for (int ky = 0; ky < g->kh; ++ky)
            for (int kx = 0; kx < g->kw; ++kx) {
                int64_t s = 0, a = 0;
                for (int n = 0; n < g->n; ++n)
                    for (int oy = 0; oy < g->oh; ++oy) {
                        const int iy = oy * g->stride_h - g->pad_t + ky * g->dilate_h;
                        if (iy < 0 || iy >= g->h) continue;
                        for (int ox = 0; ox < g->ow; ++ox) {
                            const int ix = ox * g->stride_w - g->pad_l + kx * g->dilate_w;
                            if (ix < 0 || ix >= g->w) continue;
                            const int32_t p = (int32_t)x[(((int64_t)n * g->c_in + ci) * g->h + iy) * g->w + ix] *
                                              (int32_t)dy[(((int64_t)n * g->c_out + co) * g->oh + oy) * g->ow + ox];
                            s += p;
                            a += p < 0 ? -p : p;
                        }
                    }
                stat_add(st, s, a);
                C->acc[(((int64_t)co * g->c_in + ci) * g->kh + ky) * g->kw + kx] = (int32_t)(uint32_t)s;
            }
    }
}

void niti_ref_conv_wgrad_acc(const niti_ref_geom* g, const int8_t* x, const int8_t* dy, int32_t* acc,
                             niti_ref_stats* st) {
    const conv_ctx c = {g, x, dy, acc};
    par_range((int64_t)g->c_out * g->c_in, wgrad_range, &c, st);
}

static void dgrad_range(const void* c, int64_t b0, int64_t b1, niti_ref_stats* st) {
    const conv_ctx* C = (const conv_ctx*)c;
    const niti_ref_geom* g = C->g;
    const int8_t *dy = C->a, *w = C->b;
    for (int64_t r = b0; r < b1; ++r) { /* r = n * c_in + ci */
        const int n = (int)(r / g->c_in), ci = (int)(r % g->c_in);
        for (int iy = 0; iy < g->h; ++iy)
            for (int ix = 0; ix < g->w; ++ix) {
                int64_t s = 0, a = 0;
                for (int co = 0; co < g->c_out; ++co)
                    for (int ky = 0; ky < g->kh; ++ky) {
                        const int ty = iy + g->pad_t - ky * g->dilate_h;
                        if (ty < 0 || ty % g->stride_h) continue;
                        const int oy = ty / g->stride_h;
                        if (oy >= g->oh) continue;
                        for (int kx = 0; kx < g->kw; ++kx) {
                            const int tx = ix + g->pad_l - kx * g->dilate_w;
                            if (tx < 0 || tx % g->stride_w) continue;
                            const int ox = tx / g->stride_w;
                            if (ox >= g->ow) continue;
                            const int32_t p = (int32_t)dy[(((int64_t)n * g->c_out + co) * g->oh + oy) * g->ow + ox] *
                                              (int32_t)w[(((int64_t)co * g->c_in + ci) * g->kh + ky) * g->kw + kx];
                            s += p;
                            a += p < 0 ? -p : p;
                        }
                    }
                stat_add(st, s, a);
                C->acc[(((int64_t)n * g->c_in + ci) * g->h + iy) * g->w + ix] = (int32_t)(uint32_t)s;
            }
    }
}

void niti_ref_conv_dgrad_acc(const niti_ref_geom* g, const int8_t* dy, const int8_t* w, int32_t* acc,
                             niti_ref_stats* st) {
    const conv_ctx c = {g, dy, w, acc};
    par_range((int64_t)g->n * g->c_in, dgrad_range, &c, st);
}

void niti_ref_matmul_acc(int m, int o, int k, const int8_t* B, const int8_t* A, int32_t* acc,
                         niti_ref_stats* st) {
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < o; ++j) {
            int64_t s = 0, a = 0;
            for (int t = 0; t < k; ++t) {
                const int32_t p = (int32_t)B[(int64_t)i * k + t] * (int32_t)A[(int64_t)j * k + t];
                s += p;
                a += p < 0 ? -p : p;
            }
            stat_add(st, s, a);
            acc[(int64_t)i * o + j] = (int32_t)(uint32_t)s;
        }
}

/* ---------------------------------------------------------------------------- */
/* MNN C4 layout: source/backend/cpu/CPUTensorConvert.cpp:98-178                 */
/* [ceil(C/4)][N][H][W][4], zero in the padded channels                         */
/* ---------------------------------------------------------------------------- */

void niti_ref_nchw_to_c4(const int8_t* src, int n, int c, int h, int w, int8_t* dst) {
    const int64_t hw = (int64_t)h * w, cq = UP_DIV(c, 4);
    memset(dst, 0, (size_t)(cq * 4 * n * hw));
    for (int b = 0; b < n; ++b)
        for (int ch = 0; ch < c; ++ch)
            for (int64_t p = 0; p < hw; ++p)
                dst[(((ch / 4) * (int64_t)n + b) * hw + p) * 4 + ch % 4] = src[((int64_t)b * c + ch) * hw + p];
}

void niti_ref_c4_to_nchw(const int8_t* src, int n, int c, int h, int w, int8_t* dst) {
    const int64_t hw = (int64_t)h * w;
    for (int b = 0; b < n; ++b)
        for (int ch = 0; ch < c; ++ch)
            for (int64_t p = 0; p < hw; ++p)
                dst[((int64_t)b * c + ch) * hw + p] = src[(((ch / 4) * (int64_t)n + b) * hw + p) * 4 + ch % 4];
}

void niti_ref_c4_to_nchw_i32(const int32_t* src, int n, int c, int h, int w, int32_t* dst) {
    const int64_t hw = (int64_t)h * w;
    for (int b = 0; b < n; ++b)
        for (int ch = 0; ch < c; ++ch)
            for (int64_t p = 0; p < hw; ++p)
                dst[((int64_t)b * c + ch) * hw + p] = src[(((ch / 4) * (int64_t)n + b) * hw + p) * 4 + ch % 4];
}

/* ---------------------------------------------------------------------------- */
/* reference-structured conv core: NITI_Conv_Int8.cpp:19-64, 162-249,           */
/* compute/Int8FunctionsOpt.cpp:201-232 (GEMM unit), :296-392 (im2col)          */
/* ---------------------------------------------------------------------------- */

enum { UNIT = 4, SRC_UNIT = 16, DST_XUNIT = 4 };

typedef struct {
    const niti_ref_geom* g;
    const int8_t* x;
    const int8_t* wr;
    int32_t* acc;
    int kcu, ic_div4, acc_mode;
    int b0, b1;
} core_job;

/* _im2colCommon (:342-392); _im2colCommonZ1 (:296-340) and _fastIm2Col (:270-294)
 * produce the same bytes for the shapes they accept. */
static void im2col_tile(const core_job* J, const int8_t* src, int x_start, int real, int8_t* col) {
    const niti_ref_geom* g = J->g;
    memset(col, 0, (size_t)J->kcu * DST_XUNIT * SRC_UNIT);
    const int64_t src_z_step = (int64_t)g->h * g->w * UNIT * g->n;
    const int64_t src_y_step = (int64_t)g->w * UNIT;
    for (int i = 0; i < real; ++i) {
        const int xi = x_start + i;
        const int ox = xi % g->ow, oy = xi / g->ow;
        const int sx = ox * g->stride_w - g->pad_l;
        const int sy = oy * g->stride_h - g->pad_t;
        const int sfy = ALIMAX(0, UP_DIV(-sy, g->dilate_h));
        const int efy = ALIMIN(g->kh, UP_DIV(g->h - sy, g->dilate_h));
        const int sfx = ALIMAX(0, UP_DIV(-sx, g->dilate_w));
        const int efx = ALIMIN(g->kw, UP_DIV(g->w - sx, g->dilate_w));
        for (int fy = sfy; fy < efy; ++fy)
            for (int fx = sfx; fx < efx; ++fx) {
                const int8_t* in_k = src + (int64_t)(sy + fy * g->dilate_h) * src_y_step +
                                     (int64_t)(sx + fx * g->dilate_w) * UNIT;
                const int idx0 = (fy * g->kw + fx) * J->ic_div4;
                for (int sz = 0; sz < J->ic_div4; ++sz) {
                    const int y = idx0 + sz;
                    memcpy(col + (int64_t)(y / UNIT) * (DST_XUNIT * SRC_UNIT) + i * SRC_UNIT + (y % UNIT) * 4,
                           in_k + sz * src_z_step, 4);
                }
            }
    }
}

/* NITI_MNNGemmInt8AddBiasScale_16x4_Unit, x86/portable form (:201-232). */
static void gemm_unit(const core_job* J, int32_t* dst, const int8_t* col, int64_t dst_step, int oc_div4,
                      int real) {
    for (int dz = 0; dz < oc_div4; ++dz) {
        const int8_t* w_dz = J->wr + (int64_t)dz * J->kcu * (UNIT * SRC_UNIT);
        int32_t* dst_z = dst + dz * dst_step;
        for (int w = 0; w < real; ++w) {
            const int8_t* src_x = col + w * SRC_UNIT;
            int32_t* dst_x = dst_z + w * UNIT;
            for (int j = 0; j < UNIT; ++j) {
                if (J->acc_mode == NITI_REF_ACC_F32_SEQ) {
                    float t = 0.0f;
                    for (int sz = 0; sz < J->kcu; ++sz) {
                        const int8_t* wj = w_dz + (UNIT * SRC_UNIT) * sz + j * SRC_UNIT;
                        const int8_t* sz_ = src_x + sz * DST_XUNIT * SRC_UNIT;
                        for (int i = 0; i < SRC_UNIT; ++i) t += (float)sz_[i] * (float)wj[i];
                    }
                    dst_x[j] = (int32_t)t;
                } else {
                    int64_t t = 0;
                    for (int sz = 0; sz < J->kcu; ++sz) {
                        const int8_t* wj = w_dz + (UNIT * SRC_UNIT) * sz + j * SRC_UNIT;
                        const int8_t* sz_ = src_x + sz * DST_XUNIT * SRC_UNIT;
                        for (int i = 0; i < SRC_UNIT; ++i) t += (int32_t)sz_[i] * (int32_t)wj[i];
                    }
                    dst_x[j] = (int32_t)(uint32_t)t;
                }
            }
        }
    }
}

static void* core_worker(void* arg) {
    const core_job* J = (const core_job*)arg;
    const niti_ref_geom* g = J->g;
    const int ohw = g->oh * g->ow;
    const int tiles = UP_DIV(ohw, DST_XUNIT);
    const int64_t dst_z_step = (int64_t)ohw * UNIT * g->n;
    const int oc_div4 = UP_DIV(g->c_out, UNIT);
    int8_t* col = (int8_t*)malloc((size_t)J->kcu * DST_XUNIT * SRC_UNIT);
    for (int b = J->b0; b < J->b1; ++b) {
        const int8_t* src = J->x + (int64_t)b * UNIT * g->h * g->w;
        int32_t* dst = J->acc + (int64_t)b * UNIT * ohw;
        for (int t = 0; t < tiles; ++t) {
            const int xs = t * DST_XUNIT;
            const int real = ALIMIN(ohw - xs, DST_XUNIT);
            im2col_tile(J, src, xs, real, col);
            gemm_unit(J, dst + (int64_t)xs * UNIT, col, dst_z_step, oc_div4, real);
        }
    }
    free(col);
    return NULL;
}

void niti_ref_mnn_conv_core(const niti_ref_geom* g, const int8_t* x_c4, const int8_t* w_oihw,
                            int32_t* acc_c4, int acc_mode, int threads) {
    const int ic_div4 = UP_DIV(g->c_in, UNIT);
    const int kcount = g->kh * g->kw;
    const int kcu = UP_DIV(ic_div4 * kcount, SRC_UNIT / UNIT);
    const int oc_div4 = UP_DIV(g->c_out, UNIT);
    /* reorderWeight, NITI_Conv_Int8.cpp:19-64: [oc/4][kcu][4 oc][16] */
    const int64_t stride0 = (int64_t)kcu * UNIT * SRC_UNIT, stride1 = UNIT * SRC_UNIT;
    int8_t* wr = (int8_t*)calloc((size_t)(oc_div4 * stride0), 1);
    for (int k = 0; k < kcount; ++k)
        for (int y = 0; y < g->c_in; ++y) {
            const int yi = y / UNIT + k * ic_div4;
            int8_t* dst_y = wr + (yi / (SRC_UNIT / UNIT)) * stride1 + (yi % (SRC_UNIT / UNIT)) * UNIT + y % UNIT;
            for (int x = 0; x < g->c_out; ++x)
                dst_y[(x / UNIT) * stride0 + (x % UNIT) * SRC_UNIT] = w_oihw[(int64_t)x * kcount * g->c_in + y * kcount + k];
        }
    memset(acc_c4, 0, (size_t)oc_div4 * UNIT * g->n * g->oh * g->ow * sizeof(int32_t));
    if (threads < 1) threads = 1;
    if (threads > g->n) threads = g->n > 0 ? g->n : 1;
    core_job jobs[256];
    pthread_t tids[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; ++t) {
        core_job* J = &jobs[t];
        J->g = g;
        J->x = x_c4;
        J->wr = wr;
        J->acc = acc_c4;
        J->kcu = kcu;
        J->ic_div4 = ic_div4;
        J->acc_mode = acc_mode;
        /* NITI_Conv_Int8.cpp:224-229: contiguous batch ranges, remainder to the last thread */
        J->b0 = t * (g->n / threads);
        J->b1 = (t == threads - 1) ? g->n : J->b0 + g->n / threads;
    }
    if (threads == 1) {
        core_worker(&jobs[0]);
    } else {
        for (int t = 0; t < threads; ++t) pthread_create(&tids[t], NULL, core_worker, &jobs[t]);
        for (int t = 0; t < threads; ++t) pthread_join(tids[t], NULL);
    }
    free(wr);
}

int32_t niti_ref_mnn_conv_fwd(const niti_ref_geom* g, const int8_t* x_c4, const int8_t* w_oihw,
                              int32_t exp_in, int32_t wscale, int8_t* y_c4, int acc_mode, int threads) {
    const int64_t osize = (int64_t)UP_DIV(g->c_out, UNIT) * UNIT * g->n * g->oh * g->ow;
    int32_t* acc = (int32_t*)malloc((size_t)osize * sizeof(int32_t));
    niti_ref_mnn_conv_core(g, x_c4, w_oihw, acc, acc_mode, threads);
    const int32_t inc = niti_ref_requant_fwd(acc, osize, y_c4);
    free(acc);
    return (int32_t)(int8_t)(exp_in + wscale + inc); /* :255-258, :307 -- stored as int8 */
}

static void transpose01(const int8_t* src, int d0, int d1, int64_t inner, int8_t* dst) {
    for (int a = 0; a < d0; ++a)
        for (int b = 0; b < d1; ++b)
            memcpy(dst + ((int64_t)b * d0 + a) * inner, src + ((int64_t)a * d1 + b) * inner, (size_t)inner);
}

/* NITI_CPULeftPoolGrad_Int8.cpp:18-52: dy[oy][ox] -> out[oy*s][ox*s] inside an osz x osz plane */
static void left_pool_grad(const int8_t* dy, int planes, int ih, int iw, int s, int osz, int8_t* out) {
    memset(out, 0, (size_t)planes * osz * osz);
    for (int p = 0; p < planes; ++p)
        for (int y = 0; y < osz; y += s)
            for (int x = 0; x < osz; x += s) {
                const int sy = y / s, sx = x / s;
                if (sy < ih && sx < iw) out[((int64_t)p * osz + y) * osz + x] = dy[((int64_t)p * ih + sy) * iw + sx];
            }
}

int32_t niti_ref_mnn_conv_wgrad(const niti_ref_geom* g, const int8_t* x, const int8_t* dy, int8_t* dw,
                                int32_t* acc_oihw, int acc_mode, int threads) {
    /* graph: grad/NITI_Conv_Int8_Grad.cpp:124-191 */
    const int s = g->stride_h;
    int kdim_h = g->oh, kdim_w = g->ow;
    const int8_t* dyk = dy;
    int8_t* dil = NULL;
    if (s == 2) { /* :143-166: LeftPoolGrad into the stride-1 output size */
        const int ow1 = g->w + g->pad_l * 2 - g->kw + 1;
        dil = (int8_t*)malloc((size_t)g->n * g->c_out * ow1 * ow1);
        left_pool_grad(dy, g->n * g->c_out, g->oh, g->ow, 2, ow1, dil);
        dyk = dil;
        kdim_h = kdim_w = ow1;
    }
    /* inputs: C4(x^T) [ceil(N/4)][C_in][H][W][4], kernel dy^T as OIHW [C_out][N][kh][kw] */
    const int64_t hw = (int64_t)g->h * g->w;
    int8_t* xt = (int8_t*)malloc((size_t)(g->n * g->c_in * hw));
    transpose01(x, g->n, g->c_in, hw, xt);
    int8_t* xt_c4 = (int8_t*)malloc((size_t)(UP_DIV(g->n, 4) * 4 * g->c_in * hw));
    niti_ref_nchw_to_c4(xt, g->c_in, g->n, g->h, g->w, xt_c4);
    const int64_t khw = (int64_t)kdim_h * kdim_w;
    int8_t* dyt = (int8_t*)malloc((size_t)(g->n * g->c_out * khw));
    transpose01(dyk, g->n, g->c_out, khw, dyt);

    niti_ref_geom g2;
    memset(&g2, 0, sizeof(g2));
    g2.n = g->c_in;
    g2.c_in = g->n;
    g2.h = g->h;
    g2.w = g->w;
    g2.c_out = g->c_out;
    g2.kh = kdim_h;
    g2.kw = kdim_w;
    g2.stride_h = g2.stride_w = 1;
    g2.pad_t = g->pad_t;
    g2.pad_l = g->pad_l;
    g2.pad_b = g->pad_t; /* the grad op keeps padX/padY: symmetric */
    g2.pad_r = g->pad_l;
    g2.dilate_h = g2.dilate_w = 1;
    niti_ref_geom_finalize(&g2); /* == (KH, KW) */

    const int64_t osize = (int64_t)UP_DIV(g2.c_out, 4) * 4 * g2.n * g2.oh * g2.ow;
    int32_t* acc = (int32_t*)malloc((size_t)osize * sizeof(int32_t));
    niti_ref_mnn_conv_core(&g2, xt_c4, dyt, acc, acc_mode, threads);
    int8_t* q = (int8_t*)malloc((size_t)osize);
    const int32_t bw = niti_ref_requant_wgrad(acc, osize, q);
    /* C4 [ceil(C_out/4)][C_in][KH][KW][4] -> NCHW [C_in][C_out][KH][KW] -> transpose -> OIHW */
    const int64_t k2 = (int64_t)g2.oh * g2.ow;
    int8_t* q_nchw = (int8_t*)malloc((size_t)(g->c_in * g->c_out * k2));
    niti_ref_c4_to_nchw(q, g2.n, g2.c_out, g2.oh, g2.ow, q_nchw);
    transpose01(q_nchw, g->c_in, g->c_out, k2, dw);
    if (acc_oihw) {
        int32_t* a_nchw = (int32_t*)malloc((size_t)(g->c_in * g->c_out * k2) * sizeof(int32_t));
        niti_ref_c4_to_nchw_i32(acc, g2.n, g2.c_out, g2.oh, g2.ow, a_nchw);
        for (int ci = 0; ci < g->c_in; ++ci)
            for (int co = 0; co < g->c_out; ++co)
                memcpy(acc_oihw + ((int64_t)co * g->c_in + ci) * k2, a_nchw + ((int64_t)ci * g->c_out + co) * k2,
                       (size_t)k2 * sizeof(int32_t));
        free(a_nchw);
    }
    free(q_nchw);
    free(q);
    free(acc);
    free(dyt);
    free(xt_c4);
    free(xt);
    free(dil);
    return bw;
}

/* NITI_Pad_Int8.cpp:26-67: symmetric zero pad e on H and W of an NCHW tensor */
static void pad_nchw(const int8_t* src, int planes, int h, int w, int e, int8_t* dst) {
    const int oh = h + 2 * e, ow = w + 2 * e;
    memset(dst, 0, (size_t)planes * oh * ow);
    for (int p = 0; p < planes; ++p)
        for (int y = 0; y < h; ++y)
            memcpy(dst + ((int64_t)p * oh + y + e) * ow + e, src + ((int64_t)p * h + y) * w, (size_t)w);
}

int32_t niti_ref_mnn_conv_dgrad(const niti_ref_geom* g, const int8_t* dy, const int8_t* w, int8_t* dx,
                                int32_t* acc_nchw, int acc_mode, int threads) {
    /* graph: grad/NITI_Conv_Int8_Grad.cpp:29-122 */
    const int p = g->pad_l;
    int dh = g->oh, dw_ = g->ow;
    const int8_t* d0 = dy;
    int8_t* dil = NULL;
    if (g->stride_h == 2) { /* :86-106 */
        const int ow1 = g->w + p * 2 - g->kw + 1;
        dil = (int8_t*)malloc((size_t)g->n * g->c_out * ow1 * ow1);
        left_pool_grad(dy, g->n * g->c_out, g->oh, g->ow, 2, ow1, dil);
        d0 = dil;
        dh = dw_ = ow1;
    }
    const int e = (g->w - (dw_ + p * 2 - g->kw + 1)) / 2; /* extraPad :94 / :113 */
    int8_t* padded = NULL;
    const int8_t* d1 = d0;
    if (e != 0) {
        padded = (int8_t*)malloc((size_t)g->n * g->c_out * (dh + 2 * e) * (dw_ + 2 * e));
        pad_nchw(d0, g->n * g->c_out, dh, dw_, e, padded);
        d1 = padded;
        dh += 2 * e;
        dw_ += 2 * e;
    }
    int8_t* d_c4 = (int8_t*)malloc((size_t)UP_DIV(g->c_out, 4) * 4 * g->n * dh * dw_);
    niti_ref_nchw_to_c4(d1, g->n, g->c_out, dh, dw_, d_c4);
    /* w^T (transpose {1,0,2,3}) then rotate180 per plane (NITI_DeConv_Int8.cpp:179-219) */
    const int64_t kk = (int64_t)g->kh * g->kw;
    int8_t* wt = (int8_t*)malloc((size_t)(g->c_out * g->c_in * kk));
    transpose01(w, g->c_out, g->c_in, kk, wt);
    int8_t* w180 = (int8_t*)malloc((size_t)(g->c_out * g->c_in * kk));
    for (int64_t pl = 0; pl < (int64_t)g->c_out * g->c_in; ++pl) {
        const int rows = g->kw, cols = g->kh; /* rotate180(src, dst, wwidth, wheight) */
        for (int i = 0; i < rows; ++i)
            for (int j = 0; j < cols; ++j)
                w180[pl * kk + (int64_t)(rows - i - 1) * cols + (cols - j - 1)] = wt[pl * kk + (int64_t)i * cols + j];
    }
    niti_ref_geom g3;
    memset(&g3, 0, sizeof(g3));
    g3.n = g->n;
    g3.c_in = g->c_out;
    g3.h = dh;
    g3.w = dw_;
    g3.c_out = g->c_in;
    g3.kh = g->kh;
    g3.kw = g->kw;
    g3.stride_h = g3.stride_w = 1;
    g3.pad_t = g3.pad_b = g->pad_t;
    g3.pad_l = g3.pad_r = p;
    g3.dilate_h = g3.dilate_w = 1;
    niti_ref_geom_finalize(&g3); /* == (H, W) */
    const int64_t osize = (int64_t)UP_DIV(g3.c_out, 4) * 4 * g3.n * g3.oh * g3.ow;
    int32_t* acc = (int32_t*)malloc((size_t)osize * sizeof(int32_t));
    niti_ref_mnn_conv_core(&g3, d_c4, w180, acc, acc_mode, threads);
    int8_t* q = (int8_t*)malloc((size_t)osize);
    const int32_t inc = niti_ref_requant_fwd(acc, osize, q);
    niti_ref_c4_to_nchw(q, g3.n, g3.c_out, g3.oh, g3.ow, dx);
    if (acc_nchw) niti_ref_c4_to_nchw_i32(acc, g3.n, g3.c_out, g3.oh, g3.ow, acc_nchw);
    free(q);
    free(acc);
    free(w180);
    free(wt);
    free(d_c4);
    free(padded);
    free(dil);
    return inc;
}

/* ---------------------------------------------------------------------------- */
/* the rest of the NITI step                                                     */
/* ---------------------------------------------------------------------------- */

void niti_ref_relu(const int8_t* x, int64_t n, int8_t* y) { /* NITI_CPURelu_Int8.cpp:41-50 */
    for (int64_t i = 0; i < n; ++i) y[i] = x[i] >= 0 ? x[i] : 0;
}

void niti_ref_relu_grad(const int8_t* x, const int8_t* dy, int64_t n, int8_t* out) {
    for (int64_t i = 0; i < n; ++i) out[i] = x[i] > 0 ? dy[i] : 0; /* NITI_CPUReluGrad_Int8.cpp:42-51 */
}

/* poolingMaxNHWCInt8, NITI_Maxpool_Int8.cpp:24-72 (kernel clipped to the input, :97-98) */
void niti_ref_maxpool(const int8_t* x, int n, int c, int h, int w, int k, int s, int p, int8_t* y,
                      int oh, int ow) {
    const int kh = ALIMIN(k, h), kw = ALIMIN(k, w);
    for (int b = 0; b < n; ++b)
        for (int ch = 0; ch < c; ++ch) {
            const int8_t* src = x + ((int64_t)b * c + ch) * h * w;
            int8_t* dst = y + ((int64_t)b * c + ch) * oh * ow;
            for (int oy = 0; oy < oh; ++oy)
                for (int ox = 0; ox < ow; ++ox) {
                    const int sx0 = ox * s - p, sy0 = oy * s - p;
                    const int kxs = ALIMAX(0, -sx0), kxe = ALIMIN(kw, w - sx0);
                    const int kys = ALIMAX(0, -sy0), kye = ALIMIN(kh, h - sy0);
                    int8_t r = INT8_MIN;
                    for (int yy = kys; yy < kye; ++yy)
                        for (int xx = kxs; xx < kxe; ++xx) {
                            const int8_t v = src[(sy0 + yy) * w + sx0 + xx];
                            if (v > r) r = v;
                        }
                    dst[oy * ow + ox] = r;
                }
        }
}

/* NITI_CPUMaxPoolGrad_Int8::onExecute, NITI_CPUPoolGrad_Int8.cpp:21-77 */
void niti_ref_maxpool_grad(const int8_t* x, const int8_t* y, const int8_t* dy, int n, int c, int h,
                           int w, int k, int s, int p, int oh, int ow, int8_t* dx) {
    memset(dx, 0, (size_t)n * c * h * w);
    for (int b = 0; b < n; ++b)
        for (int ch = 0; ch < c; ++ch) {
            const int64_t pi = ((int64_t)b * c + ch) * h * w, po = ((int64_t)b * c + ch) * oh * ow;
            for (int oy = 0; oy < oh; ++oy)
                for (int ox = 0; ox < ow; ++ox) {
                    const int8_t mx = y[po + oy * ow + ox], d = dy[po + oy * ow + ox];
                    int done = 0;
                    for (int ky = 0; ky < k && !done; ++ky) {
                        const int sy = oy * s + ky - p;
                        if (sy < 0 || sy >= h) continue;
                        for (int kx = 0; kx < k; ++kx) {
                            const int sx = ox * s + kx - p;
                            if (sx < 0 || sx >= w) continue;
                            if (x[pi + sy * w + sx] >= mx) {
                                dx[pi + sy * w + sx] = (int8_t)(dx[pi + sy * w + sx] + d);
                                done = 1;
                                break;
                            }
                        }
                    }
                }
        }
}

/* (1 << t) with an int left operand, as x86-64 executes it, widened to int64 */
static inline int64_t ipow2_64(int64_t t) { return (int64_t)niti_ref_pow2((int32_t)(t & 31)); }

/* NITI_CPULossGrad_Int8::onExecute, NITI_CPULossGrad_Int8.cpp:81-200 */
void niti_ref_loss_grad(const int8_t* logits, int batch, int classes, int32_t ascale,
                        const int32_t* onehot, int target_classes, int8_t* out) {
    const int64_t n = (int64_t)batch * classes;
    int64_t* sv = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* o = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int64_t* g = (int64_t*)malloc((size_t)n * sizeof(int64_t));
    int32_t* gf = (int32_t*)malloc((size_t)n * sizeof(int32_t));
    const int8_t as = (int8_t)ascale;
    if (as > -7) {
        for (int64_t i = 0; i < n; ++i) {
            int64_t t = (int64_t)logits[i] * 47274;
            t = t / (1 << 15);
            sv[i] = (as >= 0) ? t * ipow2_64(as) : t / ipow2_64(-as);
        }
        for (int i = 0; i < batch; ++i) {
            int64_t mx = sv[(int64_t)i * classes];
            for (int j = 1; j < classes; ++j)
                if (mx < sv[(int64_t)i * classes + j]) mx = sv[(int64_t)i * classes + j];
            mx -= 10;
            for (int j = 0; j < classes; ++j) {
                int64_t t = sv[(int64_t)i * classes + j] - mx;
                t = t > 0 ? t : 0;
                o[(int64_t)i * classes + j] = ipow2_64(t) - 1;
            }
        }
    } else {
        const int64_t base = ipow2_64(1 - 2 * (int64_t)as);
        const int64_t shiftbase = ipow2_64(1 - (int64_t)as);
        for (int64_t i = 0; i < n; ++i) {
            const int64_t t = logits[i];
            o[i] = base + t * shiftbase + t * t;
        }
    }
    for (int i = 0; i < batch; ++i) {
        int64_t sum = 0;
        for (int j = 0; j < classes; ++j) sum += o[(int64_t)i * classes + j];
        for (int j = 0; j < classes; ++j) g[(int64_t)i * classes + j] = (o[(int64_t)i * classes + j] * (1 << 11)) / sum;
    }
    for (int i = 0; i < batch; ++i) {
        int tmax = 0; /* target_max is uninitialised in the reference when no 1 is present */
        for (int j = 0; j < target_classes; ++j)
            if (onehot[(int64_t)i * target_classes + j] == 1) {
                tmax = j;
                break;
            }
        int64_t sum = 0;
        for (int j = 0; j < classes; ++j) sum += g[(int64_t)i * classes + j];
        for (int j = 0; j < classes; ++j) gf[(int64_t)i * classes + j] = (int32_t)g[(int64_t)i * classes + j];
        gf[(int64_t)i * classes + tmax] = (int32_t)(g[(int64_t)i * classes + tmax] - sum);
    }
    for (int64_t i = 0; i < n; ++i) out[i] = (int8_t)niti_ref_psto1(gf[i], 4); /* :198, ToInt8 form :1629-1654 */
    free(gf);
    free(g);
    free(o);
    free(sv);
}

void niti_ref_sgd_update(int8_t* w, const int8_t* g, int64_t n) {
    for (int64_t i = 0; i < n; ++i) w[i] = (int8_t)niti_ref_int8_clip((int32_t)w[i] - (int32_t)g[i]);
}

/* MnistUtils.cpp:83-93 in float, in the operation order the expression graph states it, with the
 * two full reductions (_ReduceMean, _ReduceSum: one axis of n values, OpCommonUtils.cpp:332-333,
 * summed by CPUReduction.cpp:86-95 `summer += src[a]`) accumulated in `lanes` interleaved partial
 * sums (value i into partial i % lanes, partials then added in order).  lanes = 1 is the C source's
 * sequential loop; the engine is compiled with -ffast-math (CMakeLists.txt:429-430), which lets the
 * compiler reassociate that loop into vector lanes (4-wide NEON / SSE, x2-x4 interleaved), so
 * lanes = 4 / 8 / 16 are orders the reference binary may equally execute.  The variance divisor is
 * the reference's literal `batchSize * 28 * 28` (:86): var_n = images * 784 whatever the image size.
 * _Log on a float is taken as the correctly rounded float natural log, (float)log((double)r). */
static float sum_lanes(const float* x, int64_t n, int lanes, float mean, int sq) {
    float part[64];
    if (lanes < 1) lanes = 1;
    if (lanes > 64) lanes = 64;
    for (int l = 0; l < lanes; ++l) part[l] = 0.f;
    for (int64_t i = 0; i < n; ++i) {
        const float v = sq ? (x[i] - mean) * (x[i] - mean) : x[i];
        part[i % lanes] += v;
    }
    float s = part[0];
    for (int l = 1; l < lanes; ++l) s += part[l];
    return s;
}

int32_t niti_ref_quantize_input_lanes(const float* x, int64_t n, int64_t var_n, int lanes, int8_t* out) {
    const float sum = sum_lanes(x, n, lanes, 0.f, 0);
    const float mean = sum / (float)n;
    const float ss = sum_lanes(x, n, lanes, mean, 1);
    const float sd = sqrtf(ss / (float)var_n);
    float range = 0.f;
    for (int64_t i = 0; i < n; ++i) {
        const float y = fabsf((x[i] - mean) / sd);
        if (y > range) range = y;
    }
    const float bw = ceilf((float)log((double)range));
    for (int64_t i = 0; i < n; ++i) out[i] = (int8_t)roundf((x[i] - mean) / sd / range * 127.0f);
    return (int32_t)(int8_t)(bw - 7.0f);
}

int32_t niti_ref_quantize_input(const float* x, int64_t n, int64_t var_n, int8_t* out) {
    return niti_ref_quantize_input_lanes(x, n, var_n, 1, out);
}

/* MnistUtils.cpp:83-93 stated over exact integer statistics of the uint8 pixels (the
 * reference leaves its float summation order to MNN's reductions; this is the order-free
 * contract the device implements, mandheling-dsp-training_amd/csrc/niti_quant.hip):
 *   S1 = sum p, S2 = sum p^2, xmin, xmax over `count` pixels (stats[] = {S1, S2, xmax, 255-xmin})
 *   mean = float(S1) / float(count); ss = S2 - 2 mean S1 + count mean^2 (double, this order);
 *   sd = sqrtf(float(ss / var_count)), var_count = the reference's literal divisor
 *   `batchSize * 28 * 28` (MnistUtils.cpp:86: global images x 784 for any image size; equal to
 *   count for MNIST); range = max(|xmax - mean|, |xmin - mean|) / sd (float);
 *   x = (int8) roundf(((p - mean) / sd) / range * 127);
 *   ascale = int8(ceilf(logf(range)) - 7) in float as the graph computes it (_Ceil(_Log(range)),
 *   :89-91), logf taken as the correctly rounded float log, (float)log((double)range).
 * std == 0 (a constant batch, 0/0 in the reference): x = 0, ascale = -7.
 * This file is compiled without FMA contraction (x86-64 baseline, -ffp-contract=off). */
void niti_ref_image_stats(const uint8_t* img, int64_t n, uint64_t stats[4]) {
    uint64_t s1 = 0, s2 = 0;
    uint32_t mx = 0, mn = 255;
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t p = img[i];
        s1 += p;
        s2 += (uint64_t)p * p;
        if (p > mx) mx = p;
        if (p < mn) mn = p;
    }
    stats[0] = s1;
    stats[1] = s2;
    stats[2] = mx;
    stats[3] = 255u - mn;
}

int32_t niti_ref_image_quantize(const uint8_t* img, int64_t n, const uint64_t stats[4], int64_t count,
                                int64_t var_count, int8_t* out) {
    const double s1 = (double)stats[0], s2 = (double)stats[1];
    const float xmax = (float)stats[2], xmin = (float)(255u - stats[3]);
    const float mean = (float)stats[0] / (float)count;
    const double m = (double)mean;
    const double a = 2.0 * m;
    const double b = a * s1;
    const double c = (double)count * m;
    const double d = c * m;
    const double ss = (s2 - b) + d;
    const float var = (float)(ss / (double)var_count);
    const float sd = sqrtf(var > 0.f ? var : 0.f);
    if (!(sd > 0.f)) {
        memset(out, 0, (size_t)n);
        return -7;
    }
    const float hi = fabsf(xmax - mean) / sd, lo = fabsf(xmin - mean) / sd;
    const float range = hi > lo ? hi : lo;
    for (int64_t i = 0; i < n; ++i) {
        const float y = ((float)img[i] - mean) / sd;
        out[i] = (int8_t)(int)roundf(y / range * 127.0f);
    }
    return (int32_t)(int8_t)(int)(ceilf((float)log((double)range)) - 7.0f);
}

/* ---------------------------------------------------------------------------- */
/* CPU baseline: one layer's fwd + wgrad (+ dgrad) in the reference's structure  */
/* ---------------------------------------------------------------------------- */
int niti_ref_layer_step(const niti_ref_geom* g, const int8_t* x_nchw, const int8_t* w_oihw,
                        const int8_t* dy_nchw, int8_t* y_c4, int8_t* dw, int8_t* dx, int threads,
                        int with_dgrad) {
    int8_t* x_c4 = (int8_t*)malloc((size_t)UP_DIV(g->c_in, 4) * 4 * g->n * g->h * g->w);
    niti_ref_nchw_to_c4(x_nchw, g->n, g->c_in, g->h, g->w, x_c4);
    niti_ref_mnn_conv_fwd(g, x_c4, w_oihw, -7, -7, y_c4, NITI_REF_ACC_F32_SEQ, threads);
    niti_ref_mnn_conv_wgrad(g, x_nchw, dy_nchw, dw, NULL, NITI_REF_ACC_F32_SEQ, threads);
    if (with_dgrad) niti_ref_mnn_conv_dgrad(g, dy_nchw, w_oihw, dx, NULL, NITI_REF_ACC_F32_SEQ, threads);
    free(x_c4);
    return 0;
}

/* ---------------------------------------------------------------------------- */
/* Sampled accumulation statistics (tools/guard_sample.py): for chosen outputs of a   */
/* forward (kind 0), weight-gradient (1) or stride-1 input-gradient (2) conv, the      */
/* exact integer sum, sum|p| (the 2^24 guard) and the sum accumulated product by      */
/* product in float32 in the order the reference's 16x4 unit walks K                  */
/* (Int8FunctionsOpt.cpp:211-226; K = ((tap) * ceil(C/4) + c/4) * 4 + c % 4, i.e. tap- */
/* major then channel ascending, NITI_Conv_Int8.cpp:19-64 / the grad graph's convs),   */
/* cast to int32 as the reference does.  NCHW activations, OIHW weights.               */
/* ---------------------------------------------------------------------------- */
void niti_ref_sample_stats(const niti_ref_geom* g, int kind, const int8_t* a, const int8_t* b, const int64_t* idx,
                           int64_t ns, int64_t* exact, uint64_t* sabs, int32_t* f32) {
    const int N = g->n, CI = g->c_in, H = g->h, W = g->w, CO = g->c_out, KH = g->kh, KW = g->kw;
    const int OH = g->oh, OW = g->ow, SH = g->stride_h, SW = g->stride_w, PT = g->pad_t, PL = g->pad_l;
    for (int64_t s = 0; s < ns; ++s) {
        int64_t e = 0;
        uint64_t sa = 0;
        float f = 0.f;
        int64_t q = idx[s];
        if (kind == 0) { /* y[n][co][oy][ox], a = x, b = w */
            const int ox = (int)(q % OW); q /= OW;
            const int oy = (int)(q % OH); q /= OH;
            const int co = (int)(q % CO);
            const int n = (int)(q / CO);
            for (int ky = 0; ky < KH; ++ky)
                for (int kx = 0; kx < KW; ++kx) {
                    const int iy = oy * SH - PT + ky * g->dilate_h, ix = ox * SW - PL + kx * g->dilate_w;
                    if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
                    for (int c = 0; c < CI; ++c) {
                        const int32_t p = (int32_t)a[(((int64_t)n * CI + c) * H + iy) * W + ix] *
                                          (int32_t)b[(((int64_t)co * CI + c) * KH + ky) * KW + kx];
                        e += p;
                        sa += (uint64_t)(p < 0 ? -p : p);
                        f += (float)p;
                    }
                }
        } else if (kind == 1) { /* dw[co][ci][ky][kx], a = x, b = dy; K = (oy, ox) then n */
            const int kx = (int)(q % KW); q /= KW;
            const int ky = (int)(q % KH); q /= KH;
            const int ci = (int)(q % CI);
            const int co = (int)(q / CI);
            for (int oy = 0; oy < OH; ++oy)
                for (int ox = 0; ox < OW; ++ox) {
                    const int iy = oy * SH - PT + ky * g->dilate_h, ix = ox * SW - PL + kx * g->dilate_w;
                    if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
                    for (int n = 0; n < N; ++n) {
                        const int32_t p = (int32_t)a[(((int64_t)n * CI + ci) * H + iy) * W + ix] *
                                          (int32_t)b[(((int64_t)n * CO + co) * OH + oy) * OW + ox];
                        e += p;
                        sa += (uint64_t)(p < 0 ? -p : p);
                        f += (float)p;
                    }
                }
        } else { /* stride 1: dx[n][ci][y][x], a = dy, b = w; rotated taps ky' kx', then co */
            const int x = (int)(q % W); q /= W;
            const int y = (int)(q % H); q /= H;
            const int ci = (int)(q % CI);
            const int n = (int)(q / CI);
            for (int kyr = 0; kyr < KH; ++kyr)
                for (int kxr = 0; kxr < KW; ++kxr) {
                    const int ky = KH - 1 - kyr, kx = KW - 1 - kxr;
                    const int oy = y + PT - ky, ox = x + PL - kx;
                    if (oy < 0 || oy >= OH || ox < 0 || ox >= OW) continue;
                    for (int co = 0; co < CO; ++co) {
                        const int32_t p = (int32_t)a[(((int64_t)n * CO + co) * OH + oy) * OW + ox] *
                                          (int32_t)b[(((int64_t)co * CI + ci) * KH + ky) * KW + kx];
                        e += p;
                        sa += (uint64_t)(p < 0 ? -p : p);
                        f += (float)p;
                    }
                }
        }
        exact[s] = e;
        sabs[s] = sa;
        f32[s] = (int32_t)f;
    }
}
