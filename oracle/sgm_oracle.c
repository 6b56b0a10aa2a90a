/*
 * sgm_oracle.c -- CPU restatement of hilbertw/stereo_matching's CPU SGM path.
 *
 * TEST INFRASTRUCTURE ONLY (see sgm_oracle.h): the parity checker for tests/,
 * __graft_entry__.smoke() and the timed CPU baseline of bench.py.  Never
 * linked into, loaded by, or called from the product library.
 *
 * PARITY STATUS: "parity unpinned" -- the reference is unbuildable here
 * (needs OpenCV + ROS headers, inc/global.h:11-20) and ships no golden
 * vectors; see sgm_oracle.h and DESIGN.md section "Oracle".
 *
 * Three schedules of the same arithmetic, bit-identical outputs:
 *  - orc_process: per-stage functions with 10 volumes (cost, S, L1..L8), the
 *    parity checker at sizes up to HD256.  It parallelises loops the
 *    reference runs sequentially (both cost filters, the aggregation), since
 *    their rows/columns are independent; it is NOT the reference's placement.
 *  - orc_process_lean: 3 volumes, streamed path states (4K256 parity).
 *  - orc_process_refplace: the reference's OpenMP placement (parallel only at
 *    its `omp parallel for` sites; filters and aggregation + WTA sequential),
 *    the timed CPU baseline of bench.py.
 * Every parallel loop writes disjoint outputs, so results do not depend on
 * the thread count.
 */
#include "sgm_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* OpenCV's MIN/MAX macros as used by the reference (src/SGM.cpp:96-108). */
#define ORC_MIN(a, b) ((a) > (b) ? (b) : (a))
#define ORC_MAX(a, b) ((a) < (b) ? (b) : (a))

typedef long long i64;

int orc_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

/* ------------------------------------------------------------------ blur */

static int reflect101(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        else i = 2 * n - 2 - i;
    }
    return i;
}

/* cv::GaussianBlur(src, dst, Size(3,3), 2, 1) -- src/Solver.cpp:124-125.
 * Pinned formula (OpenCV 3.x createSeparableLinearFilter 8U fixed-point
 * branch): row kernel round(256*g(sigma=2)) = {82,93,82}, column kernel
 * round(256*g(sigma=1)) = {70,116,70}, int32 intermediate, output
 * sat_u8((acc + (1<<15)) >> 16), BORDER_REFLECT_101. */
void orc_blur(const uint8_t *src, uint8_t *dst, int H, int W)
{
    static const int kx[3] = {82, 93, 82};
    static const int ky[3] = {70, 116, 70};
    int *rows = (int *)malloc(sizeof(int) * (size_t)H * (size_t)W);
    for (int i = 0; i < H; ++i) {
        const uint8_t *p = src + (i64)i * W;
        for (int j = 0; j < W; ++j) {
            int a = p[reflect101(j - 1, W)], b = p[j], c = p[reflect101(j + 1, W)];
            rows[(i64)i * W + j] = kx[0] * a + kx[1] * b + kx[2] * c;
        }
    }
    for (int i = 0; i < H; ++i) {
        const int *r0 = rows + (i64)reflect101(i - 1, H) * W;
        const int *r1 = rows + (i64)i * W;
        const int *r2 = rows + (i64)reflect101(i + 1, H) * W;
        for (int j = 0; j < W; ++j) {
            int acc = ky[0] * r0[j] + ky[1] * r1[j] + ky[2] * r2[j];
            int v = (acc + (1 << 15)) >> 16;
            dst[(i64)i * W + j] = (uint8_t)(v > 255 ? 255 : v);
        }
    }
    free(rows);
}

/* ---------------------------------------------------------------- census */

/* CT_pts, src/cost.cpp:99-129: window (WIN_H/scale) x (WIN_W/scale)
 * (inc/Solver.h:10-11, Solver.cpp:127-128), MSB-first, centre skipped,
 * coordinates clamped to the image edge, strict '>' against the centre. */
void orc_census(const uint8_t *img, uint64_t *ct, int H, int W, int scale)
{
    const int win_h = 7 / scale, win_w = 9 / scale;
#pragma omp parallel for
    for (int v = 0; v < H; ++v) {
        for (int u = 0; u < W; ++u) {
            uint64_t value = 0;
            const uint8_t ctr = img[(i64)v * W + u];
            for (int i = -win_h / 2; i <= win_h / 2; ++i) {
                int y = ORC_MAX(v + i, 0);
                y = ORC_MIN(y, H - 1);
                for (int j = -win_w / 2; j <= win_w / 2; ++j) {
                    if (i == 0 && j == 0) continue;
                    int x = ORC_MAX(u + j, 0);
                    x = ORC_MIN(x, W - 1);
                    value = (value << 1) | (uint64_t)(img[(i64)y * W + x] > ctr);
                }
            }
            ct[(i64)v * W + u] = value;
        }
    }
}

/* hamming_cost, src/cost.cpp:132-144 (bit loop == popcount). */
static inline int hamming(uint64_t a, uint64_t b)
{
    return __builtin_popcountll(a ^ b);
}

/* ------------------------------------------------------------------- DSI */

void orc_dsi(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
             float *cost, int H, int W, int D, int scale, int view)
{
#pragma omp parallel for
    for (int i = 0; i < H; ++i) {
        for (int j = 0; j < W; ++j) {
            i64 bias = ((i64)i * W + j) * D;
            if (sky && sky[(i64)i * W + j] == 255) {
                /* Solver.cpp:165-178 / 219-232 */
                for (int d = 0; d < D; ++d) cost[bias + d] = d == 0 ? 0.0f : 999999.0f;
            } else if (view == 0) {
                /* Solver.cpp:182-190: d_bk = max(j - d/scale, 0) */
                for (int d = 0; d < D; ++d) {
                    int d_bk = ORC_MAX(j - d / scale, 0);
                    cost[bias + d] = (float)hamming(ctl[(i64)i * W + j], ctr[(i64)i * W + d_bk]);
                }
            } else {
                /* Solver.cpp:236-244: d_bk = min(j + d/scale, W-1) */
                for (int d = 0; d < D; ++d) {
                    int d_bk = ORC_MIN(j + d / scale, W - 1);
                    cost[bias + d] = (float)hamming(ctl[(i64)i * W + d_bk], ctr[(i64)i * W + j]);
                }
            }
        }
    }
}

/* -------------------------------------------------------- in-place IIRs */

/* cost_horizontal_filter, src/Solver.cpp:296-330, literally (sequential in
 * the reference; rows are independent so the restatement may parallelise). */
static void hfilter_impl(float *cost, int H, int W, int D, int win, int par)
{
    const i64 index_step = (i64)(win / 2 + 1) * D;
#pragma omp parallel for if (par)
    for (int i = 0; i < H; ++i) {
        for (int d = 0; d < D; ++d) {
            float sum = 0;
            i64 index = (i64)i * W * D + d;
            for (int j = 0; j < win; ++j) {
                sum += cost[index];
                index += D;
            }
            for (int j = win / 2; j < W - win / 2; ++j) {
                cost[index - index_step] = sum / win;
                if (j == W - win / 2 - 1) break;
                sum += cost[index];
                sum -= cost[index - (i64)win * D];
                index += D;
            }
        }
    }
}

/* cost_vertical_filter, src/Solver.cpp:333-368, literally. */
static void vfilter_impl(float *cost, int H, int W, int D, int win, int par)
{
    const i64 step = (i64)W * D;
    const i64 index_step = (i64)(win / 2 + 1) * step;
#pragma omp parallel for if (par)
    for (int j = 0; j < W; ++j) {
        for (int d = 0; d < D; ++d) {
            float sum = 0;
            i64 index = (i64)j * D + d;
            for (int i = 0; i < win; ++i) {
                sum += cost[index];
                index += step;
            }
            for (int i = win / 2; i < H - win / 2; ++i) {
                cost[index - index_step] = sum / win;
                if (i == H - win / 2 - 1) break;
                sum += cost[index];
                sum -= cost[index - (i64)win * step];
                index += step;
            }
        }
    }
}

void orc_hfilter(float *cost, int H, int W, int D, int win) { hfilter_impl(cost, H, W, D, win, 1); }
void orc_vfilter(float *cost, int H, int W, int D, int win) { vfilter_impl(cost, H, W, D, win, 1); }

/* ---------------------------------------------------------- path DPs */

/* One pixel of one path, src/SGM.cpp:93-117 (identical body in all eight
 * directions): prev == NULL means the path starts here.  The d loop is split
 * into its two clamped ends and a clamp-free interior, and the minimum is
 * taken over 8 interleaved partial minima, so that the compiler vectorises
 * both; the values are unchanged (every L is >= 0 and finite, and a minimum
 * of such values does not depend on the order it is taken in). */
static inline float dp_one(const float *prev, int d, int dm, int dp, float P1, float base,
                           float cd, float min_prev)
{
    float v = ORC_MIN(prev[d], prev[dm] + P1);
    v = ORC_MIN(v, prev[dp] + P1);
    v = ORC_MIN(v, base);
    return v + (cd - min_prev);
}

static inline void dp_pixel(const float *c, float *l, const float *prev, float min_prev,
                            int D, float P1, float P2, float *min_out)
{
    if (!prev) {
        for (int d = 0; d < D; ++d) l[d] = c[d];
    } else if (D < 3) {
        for (int d = 0; d < D; ++d)
            l[d] = dp_one(prev, d, ORC_MAX(d - 1, 0), ORC_MIN(d + 1, D - 1), P1, min_prev + P2,
                          c[d], min_prev);
    } else {
        const float base = min_prev + P2;
        l[0] = dp_one(prev, 0, 0, 1, P1, base, c[0], min_prev);
        for (int d = 1; d < D - 1; ++d) {
            float v = ORC_MIN(prev[d], prev[d - 1] + P1);
            v = ORC_MIN(v, prev[d + 1] + P1);
            v = ORC_MIN(v, base);
            l[d] = v + (c[d] - min_prev);
        }
        l[D - 1] = dp_one(prev, D - 1, D - 2, D - 1, P1, base, c[D - 1], min_prev);
    }
    float m8[8] = {FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX, FLT_MAX};
    int d = 0;
    for (; d + 8 <= D; d += 8)
        for (int k = 0; k < 8; ++k) m8[k] = l[d + k] < m8[k] ? l[d + k] : m8[k];
    float m = FLT_MAX;
    for (; d < D; ++d) m = l[d] < m ? l[d] : m;
    for (int k = 0; k < 8; ++k) m = m8[k] < m ? m8[k] : m;
    *min_out = m;
}

void orc_path(const float *cost, float *L, float *minL, int H, int W, int D,
              int dir, int P1i, int P2i)
{
    const float P1 = (float)P1i, P2 = (float)P2i;
#define PIX(i, j) (((i64)(i) * W + (j)))
#define STEP(i, j, pi, pj, start)                                                      \
    do {                                                                               \
        i64 q = PIX(i, j);                                                             \
        if (start) dp_pixel(cost + q * D, L + q * D, NULL, 0.f, D, P1, P2, minL + q);  \
        else {                                                                         \
            i64 p = PIX(pi, pj);                                                       \
            dp_pixel(cost + q * D, L + q * D, L + p * D, minL[p], D, P1, P2, minL + q);\
        }                                                                              \
    } while (0)

    switch (dir) {
    case ORC_L1: /* src/SGM.cpp:82-119, omp over rows */
#pragma omp parallel for
        for (int i = 0; i < H; ++i)
            for (int j = 0; j < W; ++j) STEP(i, j, i, j - 1, j == 0);
        break;
    case ORC_L2: /* src/SGM.cpp:122-159 */
#pragma omp parallel for
        for (int i = 0; i < H; ++i)
            for (int j = W - 1; j >= 0; --j) STEP(i, j, i, j + 1, j == W - 1);
        break;
    case ORC_L3: /* src/SGM.cpp:162-199, omp over columns */
#pragma omp parallel for
        for (int j = 0; j < W; ++j)
            for (int i = 0; i < H; ++i) STEP(i, j, i - 1, j, i == 0);
        break;
    case ORC_L4: /* src/SGM.cpp:202-239 */
#pragma omp parallel for
        for (int j = 0; j < W; ++j)
            for (int i = H - 1; i >= 0; --i) STEP(i, j, i + 1, j, i == H - 1);
        break;
    case ORC_L5: /* src/SGM.cpp:247-305: rows in order, omp over columns */
        for (int i = 0; i < H; ++i) {
#pragma omp parallel for
            for (int j = 0; j < W; ++j) STEP(i, j, i - 1, j - 1, i == 0 || j == 0);
        }
        break;
    case ORC_L6:
        for (int i = 0; i < H; ++i) {
#pragma omp parallel for
            for (int j = 0; j < W; ++j) STEP(i, j, i - 1, j + 1, i == 0 || j == W - 1);
        }
        break;
    case ORC_L7: /* src/SGM.cpp:311-369 */
        for (int i = H - 1; i >= 0; --i) {
#pragma omp parallel for
            for (int j = 0; j < W; ++j) STEP(i, j, i + 1, j - 1, i == H - 1 || j == 0);
        }
        break;
    case ORC_L8:
        for (int i = H - 1; i >= 0; --i) {
#pragma omp parallel for
            for (int j = 0; j < W; ++j) STEP(i, j, i + 1, j + 1, i == H - 1 || j == W - 1);
        }
        break;
    default:
        break;
    }
#undef STEP
#undef PIX
}

/* ------------------------------------------------ aggregation + WTA */

void orc_aggregate(const float *const *L, float *S, int H, int W, int D)
{
    const i64 n = (i64)H * W * D;
#pragma omp parallel for
    for (i64 k = 0; k < n; ++k) {
        /* src/SGM.cpp:386-390 */
        float s = L[0][k] + L[1][k] + L[2][k] + L[3][k];
        s += (L[4][k] + L[5][k] + L[6][k] + L[7][k]);
        S[k] = s;
    }
}

/* src/SGM.cpp:373-418 (sequential in the reference; min_d and sec_min_d
 * persist across pixels exactly as there). */
void orc_wta(const float *S, int32_t *disp, int H, int W, int D, float uniq)
{
    const int invalid = D + 1;
    float min_cost = FLT_MAX, sec_min_cost = FLT_MAX;
    int min_d = invalid, sec_min_d = invalid;
    for (int i = 0; i < H; ++i) {
        for (int j = 0; j < W; ++j) {
            min_cost = FLT_MAX;
            const float *s = S + ((i64)i * W + j) * D;
            for (int d = 0; d < D; ++d) {
                if (s[d] < min_cost) {
                    min_cost = s[d];
                    min_d = d;
                }
            }
            sec_min_cost = FLT_MAX;
            for (int d = 0; d < D; ++d) {
                if (s[d] < sec_min_cost && s[d] != min_cost) {
                    sec_min_cost = s[d];
                    sec_min_d = d;
                }
            }
            if (min_cost / sec_min_cost > uniq && abs(min_d - sec_min_d) > 1)
                disp[(i64)i * W + j] = invalid;
            else
                disp[(i64)i * W + j] = min_d;
        }
    }
}

/* compute_subpixel, src/Solver.cpp:569-597. */
void orc_subpixel(const int32_t *disp, const float *S, float *out, int H, int W, int D)
{
#pragma omp parallel for
    for (int i = 0; i < H; ++i) {
        for (int j = 0; j < W; ++j) {
            int d = disp[(i64)i * W + j];
            float r;
            if (d > D - 1) {
                r = (float)(D + 1);
            } else if (!d || d == D - 1) {
                r = (float)d;
            } else {
                i64 index = ((i64)i * W + j) * D + d;
                float cost_d = S[index];
                float cost_d_sub = S[index - 1];
                float cost_d_plus = S[index + 1];
                float x = d + (cost_d_sub - cost_d_plus) / (2 * (cost_d_sub + cost_d_plus - 2 * cost_d));
                float lim = (D - 1) * 1.f;
                r = (lim < x) ? lim : x; /* std::min(x, lim) */
            }
            out[(i64)i * W + j] = r;
        }
    }
}

/* src/SGM.cpp:803-818.
 * The column read FR(i, (int)(j - dl/s)) is clamped to [0, W-1], as the GPU's
 * lr_kernel does.  For every map compute_subpixel can produce the clamp never
 * acts: dl is NaN (j >= NaN is false), D+1, an integer d, min(+inf, D-1) or a
 * parabola vertex in [d-1/2, d+1/2] (DESIGN.md "LR check domain"), so
 * 0 <= (int)(j - dl/s) <= j.  It only matters for arbitrary maps handed to the
 * stage entry points, where the reference's cv::Mat::at reads a neighbouring
 * row (or outside the buffer, undefined); the clamp is this build's choice. */
void orc_lr_check(float *FL, const float *FR, int H, int W, int D, int scale, float lr_dis)
{
    const float invalid = (float)(D + 1);
#pragma omp parallel for
    for (int i = 0; i < H; ++i) {
        for (int j = 0; j < W; ++j) {
            float *dl = FL + (i64)i * W + j;
            if (j >= *dl) {
                const float x = j - *dl / scale;   /* clamped before the int
                                                      conversion: defined for any dl */
                const int jr = x < 0 ? 0 : (x > (float)(W - 1) ? W - 1 : (int)x);
                float dr = FR[(i64)i * W + jr];
                if (fabsf(*dl - dr) > lr_dis) *dl = invalid;
            }
        }
    }
}

/* ---------------------------------------------------------- post filter */

static int cmp_int(const void *a, const void *b)
{
    int x = *(const int *)a, y = *(const int *)b;
    return (x > y) - (x < y);
}

static int uf_find(int *parent, int i)
{
    while (parent[i] != i) {
        parent[i] = parent[parent[i]];
        i = parent[i];
    }
    return i;
}

/* post_filter, src/Solver.cpp:600-649.  Median fill: sequential, row-major,
 * in place, values truncated to int (std::vector<int>, :605,619).
 * Speckle: speckle_filter_new (:514-566).  Its result is fully determined by
 * the 4-connected components of the relation |a-b| < SPECKLE_DIS and their
 * sizes (the union-find at :525-546 is exact when run by one thread), so any
 * exact component labelling reproduces it; this one uses path halving. */
void orc_post_filter(float *F, int H, int W, int D, int scale)
{
    const int MH = 5, MW = 5;
    int v[25];
    for (int i = MH / 2; i < H - MH / 2; ++i) {
        for (int j = MW / 2; j < W - MW / 2; ++j) {
            if (F[(i64)i * W + j] <= D - 1) continue;
            int valid_cnt = 0;
            for (int m = i - MH / 2; m <= i + MH / 2; ++m)
                for (int n = j - MW / 2; n <= j + MW / 2; ++n) {
                    float x = F[(i64)m * W + n];
                    if (x <= D - 1) v[valid_cnt++] = (int)x;
                }
            if (valid_cnt > MW * MH / 2) {
                qsort(v, (size_t)valid_cnt, sizeof(int), cmp_int);
                F[(i64)i * W + j] = (float)v[valid_cnt / 2];
            }
        }
    }

    const int max_size = 1000 / scale, max_dis = 2;
    const float value = (float)(D + 1);
    const i64 n = (i64)H * W;
    int *parent = (int *)malloc(sizeof(int) * (size_t)n);
    int *area = (int *)calloc((size_t)n, sizeof(int));
    for (i64 k = 0; k < n; ++k) parent[k] = (int)k;
    for (int i = 0; i < H; ++i) {
        for (int j = 0; j < W; ++j) {
            i64 k = (i64)i * W + j;
            if (j + 1 < W && fabsf(F[k] - F[k + 1]) < max_dis) {
                int a = uf_find(parent, (int)k), b = uf_find(parent, (int)(k + 1));
                if (a != b) parent[a] = b;
            }
            if (i + 1 < H && fabsf(F[k] - F[k + W]) < max_dis) {
                int a = uf_find(parent, (int)k), b = uf_find(parent, (int)(k + W));
                if (a != b) parent[a] = b;
            }
        }
    }
    for (i64 k = 0; k < n; ++k) area[uf_find(parent, (int)k)]++;
    for (i64 k = 0; k < n; ++k)
        if (area[uf_find(parent, (int)k)] <= max_size) F[k] = value;
    free(parent);
    free(area);
}

/* ---------------------------------------------------------- LK refine */

/* LKSubPixelImpl::LKRefine + LKRefineCore (LKRefine/LKSubPixelImpl.cpp:13-235,
 * constants LKSubPixelImpl.h:31-48: win_size 7, iter_num 10, GradValid
 * g > 2, DispValid 0 < d < max_disp).  L, R: working-grid images (the caller
 * decimates, :29-44); disp: working-grid float map, refined in place.
 *
 * The reference's linear algebra is Eigen (third-party, not in this image);
 * its 1x1 products are restated as plain fp32 sums in index order k = 0..48,
 * evaluated the way its expression groups them:
 *   Hessian = (J^T * W) * J        -> sum_k (Ix_k * w_k) * Ix_k         (:176)
 *   doff    = ((H^-1 * J^T) * W) * r -> sum_k ((hinv * Ix_k) * w_k) * r_k (:185)
 *   w       = w / ||w||            -> w_k / sqrtf(sum_k w_k * w_k)       (:172)
 * Eigen's vectorised reductions may sum in another order; that order is not
 * pinned (no reference output exists), the GPU matches this one bit-for-bit.
 * Slots with zero weight leave win_Ix / win_Ires uninitialised in the
 * reference (:117-160); they are 0 here. */
void orc_lk_refine(const uint8_t *L, const uint8_t *R, float *disp, int H, int W, int D)
{
    const int hw = 3, win = 7, iters = 10;
    const i64 n = (i64)H * W;
    float *Ix = (float *)calloc((size_t)n, sizeof(float));
    float *dt = (float *)malloc(sizeof(float) * (size_t)n);
    float *nd = (float *)malloc(sizeof(float) * (size_t)n);
    memcpy(dt, disp, sizeof(float) * (size_t)n);
    memcpy(nd, disp, sizeof(float) * (size_t)n);
    /* gradients + integer truncation of the interior (:70-82) */
    for (int i = hw; i < H - hw; ++i)
        for (int j = hw; j < W - hw; ++j) {
            const i64 k = (i64)i * W + j;
            Ix[k] = (float)((int)L[k + 1] - (int)L[k - 1]) * 0.5f;
            nd[k] = (float)(int)disp[k];
            dt[k] = (float)(int)disp[k];
        }
    /* per-pixel Gauss-Newton on the disparity offset (:86-233); pixels are
     * independent (each reads dt/Ix/L/R, writes only its own nd) */
#pragma omp parallel for schedule(dynamic, 4)
    for (int i = hw; i < H - hw; ++i) {
        for (int j = hw; j < W - hw; ++j) {
            const i64 c = (i64)i * W + j;
            if (!(Ix[c] > 2)) continue;
            const float d0 = dt[c];
            if (!(d0 > 0 && d0 < D)) continue;
            float last_disp = d0, last_doff = 0.f, last_diff = FLT_MAX;
            for (int it = 0; it < iters; ++it) {
                float w[49], jx[49], res[49];
                int cnt = 0, valid = 0;
                for (int v = -hw; v <= hw; ++v)
                    for (int u = -hw; u <= hw; ++u, ++cnt) {
                        const int m = i + v, nn = j + u;
                        const i64 k = (i64)m * W + nn;
                        w[cnt] = 0.f;
                        jx[cnt] = 0.f;
                        res[cnt] = 0.f;
                        if (!(Ix[k] > 2)) continue;
                        const float dm = dt[k];
                        if (!(dm > 0 && dm < D)) continue;
                        if (fabsf(d0 - dm) > 2) continue;
                        const float dw = dm + last_doff;
                        if ((float)nn - dw < 0 || (float)nn - dw > (float)(W - 1)) continue;
                        /* exp of an int: -(v^2+u^2)/(2*3*3) is 0 or -1 (:154) */
                        w[cnt] = (float)exp((double)(-(v * v + u * u) / (2 * hw * hw)));
                        res[cnt] = (float)((int)R[(i64)m * W + (int)((float)nn - dw)] - (int)L[k]);
                        jx[cnt] = Ix[k];
                        ++valid;
                    }
                if (valid < win * win * 0.1) break;                    /* :165 */
                float s2 = 0.f;
                for (int k = 0; k < 49; ++k) s2 += w[k] * w[k];
                const float nrm = sqrtf(s2);
                for (int k = 0; k < 49; ++k) w[k] = w[k] / nrm;
                float hs = 0.f;
                for (int k = 0; k < 49; ++k) hs += (jx[k] * w[k]) * jx[k];
                if (isnan(hs) || (double)hs < 1e-3) break;               /* :178 */
                const float hinv = 1.0f / hs;
                float doff = 0.f;
                for (int k = 0; k < 49; ++k) doff += ((hinv * jx[k]) * w[k]) * res[k];
                if (isnan(doff)) break;                                /* :188 */
                if (fabsf(doff - last_doff) > last_diff) break;        /* :201 */
                if (!(d0 + doff > 0 && d0 + doff < D)) break;          /* :207 */
                last_disp = d0 + doff;
                last_diff = fabsf(doff - last_doff);
                last_doff = doff;
                if ((double)last_diff < 1e-6) break;                   /* :222 */
            }
            nd[c] = last_disp;
        }
    }
    memcpy(disp, nd, sizeof(float) * (size_t)n);
    free(Ix);
    free(dt);
    free(nd);
}

/* ---------------------------------------------------------- sky detector */

static int sky_cmp_sobel2(const uint8_t *G, int H, int W, int r, int c)
{
    /* cv::Sobel(gray, CV_64F, 1, 0) and (0, 1), ksize 3, BORDER_REFLECT_101:
     * squared magnitude as an exact integer (imageSkyDetector.cpp:215-232) */
    const int rm = r > 0 ? r - 1 : (H > 1 ? 1 : 0), rp = r < H - 1 ? r + 1 : (H > 1 ? H - 2 : 0);
    const int cm = c > 0 ? c - 1 : (W > 1 ? 1 : 0), cp = c < W - 1 ? c + 1 : (W > 1 ? W - 2 : 0);
#define PX(a, b) ((int)G[(i64)(a) * W + (b)])
    const int dx = (PX(rm, cp) + 2 * PX(r, cp) + PX(rp, cp)) - (PX(rm, cm) + 2 * PX(r, cm) + PX(rp, cm));
    const int dy = (PX(rp, cm) + 2 * PX(rp, c) + PX(rp, cp)) - (PX(rm, cm) + 2 * PX(rm, c) + PX(rm, cp));
#undef PX
    return dx * dx + dy * dy;
}

/* SkyAreaDetector::detect (sky_detector/imageSkyDetector.cpp:166-208) on a
 * single-channel image, the path node.cpp:82-86 uses: extract_sky (:76-88) =
 * extract_border_optimal (:240-281) + check_sky_border_by_gray_value
 * (:90-164) + make_sky_mask (:796-829, type 1).  refine_border / kmeans
 * (:356-557) are not on that path.
 *
 * Pinned numerics (OpenCV is not in this image):
 *  - scale > 1: cv::resize INTER_LINEAR to (w/s, h/s) as the 8U fixed-point
 *    2x2 average (sum + 2) >> 2 (s = 2, the only legal scale);
 *  - grad = sqrt(dx^2 + dy^2) > t  <=>  dx^2 + dy^2 > t^2 (integers, t <= 362);
 *  - the image is gray replicated to BGR (:175), so each 3x3 channel
 *    covariance is v * ones(3,3): determinant 0, largest eigenvalue 3v, with
 *    v = (n*S2 - S1^2) / n^2 from exact integer moments;
 *  - calculate_sky_energy (:564-705) = 1 / ((2*det_s + det_g) + (2*eig_s + eig_g)).
 * The grad_y probe at :309-314 reads (row +- 1, col +- 1) with the row-major
 * flat index (col -1 / W wrap into the neighbouring row), as cv::Mat::at
 * does; it is never reached for row <= 5.
 * mask: rows x cols, 255 = sky, 0 = not (the sky_label of :180-194). */
void orc_sky_detect(const uint8_t *img, int h, int w, int pitch, int scale, uint8_t *mask)
{
    const int H = h / scale, W = w / scale;
    const i64 n = (i64)H * W;
    uint8_t *G = (uint8_t *)malloc((size_t)n);
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
            if (scale == 1) {
                G[(i64)i * W + j] = img[(i64)i * pitch + j];
            } else {
                const uint8_t *a = img + (i64)(2 * i) * pitch + 2 * j, *b = a + pitch;
                G[(i64)i * W + j] = (uint8_t)(((int)a[0] + a[1] + b[0] + b[1] + 2) >> 2);
            }
        }
    /* extract_border_optimal: n = floor((600-5)/5)+1 = 120 thresholds,
     * step = floor(595/120) - 1 = 3, t_k = 5 + 3(k-1) (:248-263) */
    const double tmax = 600, tmin = 5, tstep = 5;
    const int nt = (int)floor((tmax - tmin) / tstep) + 1;
    const double step = floor((tmax - tmin) / nt) - 1;
    int *b = (int *)malloc(sizeof(int) * (size_t)W);
    int *best = (int *)malloc(sizeof(int) * (size_t)W);
    for (int c = 0; c < W; ++c) best[c] = H - 1;
    /* totals of the non-zero pixels (calculate_sky_energy skips (0,0,0)) */
    long long N = 0, S1 = 0, S2 = 0;
    for (i64 k = 0; k < n; ++k)
        if (G[k]) { ++N; S1 += G[k]; S2 += (long long)G[k] * G[k]; }
    double jn_max = 0.0;
    const int half = H / 2;
    for (int k = 1; k < nt + 1; ++k) {
        const double t = tmin + step * (k - 1);
        const long long t2 = (long long)t * (long long)t;
        long long ns = 0, s1 = 0, s2 = 0;
        for (int c = 0; c < W; ++c) {
            /* extract_border (:288-343) */
            int row_index = -1, bc = -1;
            for (int row = 0; row < H; ++row) {
                row_index = row;
                if (sky_cmp_sobel2(G, H, W, row, c) > t2) {
                    if (row <= 5) { bc = -1; break; }   /* overwritten at :340-342 */
                    const i64 up = (i64)(row - 1) * W + c, dn = (i64)(row + 1) * W + c;
                    const int gy = (2 * G[dn] + G[dn + 1] + G[dn - 1]) - (2 * G[up] + G[up + 1] + G[up - 1]);
                    bc = gy > 0 ? -1 : row;
                    break;
                }
                if (row_index >= half) { bc = -1; break; }
            }
            if (row_index >= half) bc = -1;
            if (row_index <= 5) bc = -1;
            b[c] = bc;
            for (int row = 0; row < bc; ++row) {   /* sky: row < border (:639) */
                const int g = G[(i64)row * W + c];
                if (g) { ++ns; s1 += g; s2 += (long long)g * g; }
            }
        }
        double jn;
        const long long ng = N - ns, g1 = S1 - s1, g2 = S2 - s2;
        if (ng == 0 || ns == 0) {
            jn = DBL_MIN;                             /* :650-652 */
        } else {
            const double vs = (double)(ns * s2 - s1 * s1) / ((double)ns * (double)ns);
            const double vg = (double)(ng * g2 - g1 * g1) / ((double)ng * (double)ng);
            const int para = 2;
            const double sky_det = 0.0, ground_det = 0.0;
            jn = 1 / ((para * sky_det + ground_det) + (para * (3 * vs) + (3 * vg)));
        }
        if (jn > jn_max) {                           /* :273-276 */
            jn_max = jn;
            memcpy(best, b, sizeof(int) * (size_t)W);
        }
    }
    /* check_sky_border_by_gray_value (:90-164) */
    for (int i = 0; i < W; ++i) {
        const int border = best[i];
        for (int j = 0; j < border; ++j)
            if (G[(i64)j * W + i] < 128) { best[i] = -1; break; }
        if (border != -1 && (i > 1 && best[i - 1] == -1) && (i < W - 1 && best[i + 1] == -1))
            best[i] = -1;
    }
    {
        const double f_thres_sky_width = 30;
        int p = -1, q = -1;
        for (int i = 0; i < W; ++i) {
            if (best[i] != -1) {
                p = i;
                if (i == W - 1) q = W;
                for (int j = i + 1; j < W; ++j) {
                    if (best[j] == -1 || j == W - 1) {
                        q = j;
                        if (j == W - 1) q = W;
                        break;
                    }
                }
                if (q > p && q - p < f_thres_sky_width)
                    for (int j = p; j < q; ++j) best[j] = -1;
                i = q;
            }
        }
    }
    /* make_sky_mask type 1 (:804-812): row <= border */
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) mask[(i64)r * W + c] = r <= best[c] ? 255 : 0;
    free(G);
    free(b);
    free(best);
}

/* ------------------------------------------------------------------ BM */

/* BM::process (src/BM.cpp:9-97): decimation with the rows NOT strided
 * (:24-25 read img.ptr(i), column j*scale; SGM.cpp:47-48 reads ptr(i*scale)),
 * build_cost_table + build_dsi_from_table (view 0, sky mask, :39-41), the two
 * cost filters (:45-46), then a WTA straight on the filtered cost with the
 * uniqueness test |min_d - sec_min_d| > 2 (:53-85).  disp is int32 (the
 * reference's uchar, widened), invalid = D+1.  The reference's get_disp()
 * after BM::process returns post_filter() of a filtered_disp BM never writes
 * (:88, Solver.cpp:20); see DESIGN.md for what this build returns instead. */
int orc_bm_process(const uint8_t *left, const uint8_t *right, const uint8_t *sky,
                   int h, int w, int scale, int D, float uniq, int blur, int32_t *disp)
{
    if (h <= 0 || w <= 0 || (scale != 1 && scale != 2) || D <= 0) return -1;
    const int H = h / scale, W = w / scale;
    const i64 npx = (i64)H * W;
    if (W < 5 || H < 3) return -1;
    uint8_t *l = (uint8_t *)malloc((size_t)npx), *r = (uint8_t *)malloc((size_t)npx);
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
            l[(i64)i * W + j] = left[(i64)i * w + (i64)j * scale];
            r[(i64)i * W + j] = right[(i64)i * w + (i64)j * scale];
        }
    uint8_t *lb = l, *rb = r;
    if (blur) {
        lb = (uint8_t *)malloc((size_t)npx);
        rb = (uint8_t *)malloc((size_t)npx);
        orc_blur(l, lb, H, W);
        orc_blur(r, rb, H, W);
    }
    uint64_t *ctl = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)npx);
    uint64_t *ctr = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)npx);
    orc_census(lb, ctl, H, W, scale);
    orc_census(rb, ctr, H, W, scale);
    float *cost = (float *)malloc(sizeof(float) * (size_t)(npx * D));
    orc_dsi(ctl, ctr, sky, cost, H, W, D, scale, 0);
    orc_hfilter(cost, H, W, D, 5 / scale);
    orc_vfilter(cost, H, W, D, 3 / scale);
    const int invalid = D + 1;
    int sec_min_d = invalid;   /* declared once outside the pixel loops (:54) */
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
            const float *c = cost + ((i64)i * W + j) * D;
            float min_cost = FLT_MAX, sec_min_cost = FLT_MAX;
            int min_d = invalid;
            for (int d = 0; d < D; ++d)
                if (c[d] < min_cost) { min_cost = c[d]; min_d = d; }
            for (int d = 0; d < D; ++d)
                if (c[d] < sec_min_cost && c[d] != min_cost) { sec_min_cost = c[d]; sec_min_d = d; }
            disp[(i64)i * W + j] =
                (min_cost / sec_min_cost > uniq && abs(min_d - sec_min_d) > 2) ? invalid : min_d;
        }
    free(cost); free(ctl); free(ctr);
    if (blur) { free(lb); free(rb); }
    free(l); free(r);
    return 0;
}

/* ------------------------------------------------------ lean schedule */

/* The same per-view result as orc_path x 8 + orc_aggregate + orc_wta +
 * orc_subpixel, holding 3 volumes (C, S, T) instead of 10: every path
 * streams its chain state (one D-vector per chain; the diagonal passes keep
 * the previous row's W states) and adds into an accumulator in the
 * reference's association order (src/SGM.cpp:386-390):
 *     S = L1; S += L2; S += L3; S += L4          -> ((L1+L2)+L3)+L4
 *     T = L5 + L6 (one top-down pass, as SGM.cpp:247-305 computes L5, L6)
 *     S += (T + L7) + L8 (one bottom-up pass, as SGM.cpp:311-369)
 * IEEE addition is commutative, so S + L2 == L1 + L2 bit for bit.  At 4K256
 * that is 3 x 8.5 GB instead of 10 x 8.5 GB (tests/test_oracle.py proves it
 * identical to orc_process on the golden and fuzz shapes). */
static void lean_rows(const float *C, float *S, int H, int W, int D, float P1, float P2)
{
#pragma omp parallel
    {
        float *a = (float *)malloc(sizeof(float) * (size_t)D);
        float *b = (float *)malloc(sizeof(float) * (size_t)D);
#pragma omp for schedule(dynamic, 1)
        for (int i = 0; i < H; ++i) {
            float *prev = a, *cur = b, mp = 0.f, m;
            for (int j = 0; j < W; ++j) {                    /* L1, SGM.cpp:82-119 */
                const i64 q = ((i64)i * W + j) * D;
                dp_pixel(C + q, cur, j == 0 ? NULL : prev, mp, D, P1, P2, &m);
                memcpy(S + q, cur, sizeof(float) * (size_t)D);
                float *t = prev; prev = cur; cur = t; mp = m;
            }
            for (int j = W - 1; j >= 0; --j) {               /* L2, SGM.cpp:122-159 */
                const i64 q = ((i64)i * W + j) * D;
                dp_pixel(C + q, cur, j == W - 1 ? NULL : prev, mp, D, P1, P2, &m);
                for (int d = 0; d < D; ++d) S[q + d] = S[q + d] + cur[d];
                float *t = prev; prev = cur; cur = t; mp = m;
            }
        }
        free(a);
        free(b);
    }
}

static void lean_cols(const float *C, float *S, int H, int W, int D, float P1, float P2)
{
#pragma omp parallel
    {
        float *a = (float *)malloc(sizeof(float) * (size_t)D);
        float *b = (float *)malloc(sizeof(float) * (size_t)D);
#pragma omp for schedule(dynamic, 4)
        for (int j = 0; j < W; ++j) {
            float *prev = a, *cur = b, mp = 0.f, m;
            for (int i = 0; i < H; ++i) {                    /* L3, SGM.cpp:162-199 */
                const i64 q = ((i64)i * W + j) * D;
                dp_pixel(C + q, cur, i == 0 ? NULL : prev, mp, D, P1, P2, &m);
                for (int d = 0; d < D; ++d) S[q + d] = S[q + d] + cur[d];
                float *t = prev; prev = cur; cur = t; mp = m;
            }
            for (int i = H - 1; i >= 0; --i) {               /* L4, SGM.cpp:202-239 */
                const i64 q = ((i64)i * W + j) * D;
                dp_pixel(C + q, cur, i == H - 1 ? NULL : prev, mp, D, P1, P2, &m);
                for (int d = 0; d < D; ++d) S[q + d] = S[q + d] + cur[d];
                float *t = prev; prev = cur; cur = t; mp = m;
            }
        }
        free(a);
        free(b);
    }
}

/* Both diagonal pairs.  down = 1: L5 (i-1, j-1) and L6 (i-1, j+1), T = L5+L6.
 * down = 0: L7 (i+1, j-1) and L8 (i+1, j+1), S += (T + L7) + L8. */
static void lean_diag(const float *C, float *S, float *T, int H, int W, int D, float P1,
                      float P2, int down)
{
    const i64 row = (i64)W * D;
    float *pa = (float *)malloc(sizeof(float) * (size_t)row), *ca = (float *)malloc(sizeof(float) * (size_t)row);
    float *pb = (float *)malloc(sizeof(float) * (size_t)row), *cb = (float *)malloc(sizeof(float) * (size_t)row);
    float *ma = (float *)malloc(sizeof(float) * (size_t)W), *na = (float *)malloc(sizeof(float) * (size_t)W);
    float *mb = (float *)malloc(sizeof(float) * (size_t)W), *nb = (float *)malloc(sizeof(float) * (size_t)W);
    for (int k = 0; k < H; ++k) {
        const int i = down ? k : H - 1 - k;
        const int first = k == 0;
#pragma omp parallel for schedule(static)
        for (int j = 0; j < W; ++j) {
            const i64 q = ((i64)i * W + j) * D;
            float *la = ca + (i64)j * D, *lb = cb + (i64)j * D;
            /* path a comes from column j-1 (L5 / L7), path b from j+1 (L6 / L8) */
            if (first || j == 0) dp_pixel(C + q, la, NULL, 0.f, D, P1, P2, na + j);
            else dp_pixel(C + q, la, pa + (i64)(j - 1) * D, ma[j - 1], D, P1, P2, na + j);
            if (first || j == W - 1) dp_pixel(C + q, lb, NULL, 0.f, D, P1, P2, nb + j);
            else dp_pixel(C + q, lb, pb + (i64)(j + 1) * D, mb[j + 1], D, P1, P2, nb + j);
            if (down) {
                for (int d = 0; d < D; ++d) T[q + d] = la[d] + lb[d];
            } else {
                for (int d = 0; d < D; ++d) S[q + d] = S[q + d] + ((T[q + d] + la[d]) + lb[d]);
            }
        }
        float *t;
        t = pa; pa = ca; ca = t;
        t = pb; pb = cb; cb = t;
        t = ma; ma = na; na = t;
        t = mb; mb = nb; nb = t;
    }
    free(pa); free(ca); free(pb); free(cb); free(ma); free(na); free(mb); free(nb);
}

/* orc_wta's result computed per pixel in parallel: the reference's sec_min_d
 * persists from the previous pixel in raster order when every cost equals the
 * minimum (SGM.cpp:374-375, 398-407), so pixels without a second minimum take
 * it from the last earlier pixel that had one, in a sequential pass. */
static void wta_par(const float *S, int32_t *disp, int H, int W, int D, float uniq)
{
    const int invalid = D + 1;
    const i64 n = (i64)H * W;
    int32_t *mind = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int32_t *secd = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    float *ratio = (float *)malloc(sizeof(float) * (size_t)n);
#pragma omp parallel for schedule(static)
    for (i64 p = 0; p < n; ++p) {
        const float *s = S + p * D;
        float mc = FLT_MAX, sc = FLT_MAX;
        int md = invalid, sd = -1;
        for (int d = 0; d < D; ++d)
            if (s[d] < mc) { mc = s[d]; md = d; }
        for (int d = 0; d < D; ++d)
            if (s[d] < sc && s[d] != mc) { sc = s[d]; sd = d; }
        mind[p] = md;
        secd[p] = sd;
        ratio[p] = mc / sc;
    }
    int last = invalid;
    for (i64 p = 0; p < n; ++p) {
        if (secd[p] >= 0) last = secd[p];
        disp[p] = (ratio[p] > uniq && abs(mind[p] - last) > 1) ? invalid : mind[p];
    }
    free(mind);
    free(secd);
    free(ratio);
}

/* ------------------------------------- the reference's OpenMP placement */

/* L5/L6 and L7/L8 as the reference computes them: one row loop per pair,
 * rows in order, omp over the columns of a row (SGM.cpp:247-305, 311-369). */
static void refplace_diag_pair(const float *C, float *La, float *Lb, float *ma, float *mb,
                               int H, int W, int D, float P1, float P2, int down)
{
    for (int k = 0; k < H; ++k) {
        const int i = down ? k : H - 1 - k;
        const int pi = down ? i - 1 : i + 1;
        const int edge = k == 0;
#pragma omp parallel for
        for (int j = 0; j < W; ++j) {
            const i64 q = (i64)i * W + j;
            if (edge || j == 0) dp_pixel(C + q * D, La + q * D, NULL, 0.f, D, P1, P2, ma + q);
            else {
                const i64 p = (i64)pi * W + j - 1;
                dp_pixel(C + q * D, La + q * D, La + p * D, ma[p], D, P1, P2, ma + q);
            }
            if (edge || j == W - 1) dp_pixel(C + q * D, Lb + q * D, NULL, 0.f, D, P1, P2, mb + q);
            else {
                const i64 p = (i64)pi * W + j + 1;
                dp_pixel(C + q * D, Lb + q * D, Lb + p * D, mb[p], D, P1, P2, mb + q);
            }
        }
    }
}

/* Aggregation + WTA + uniqueness fused and sequential, as SGM.cpp:372-418
 * (the sum is written over cost there; here into S). */
static void refplace_agg_wta(float *const *L, float *S, int32_t *disp, int H, int W, int D,
                             float uniq)
{
    const int invalid = D + 1;
    float min_cost = FLT_MAX, sec_min_cost = FLT_MAX;
    int min_d = invalid, sec_min_d = invalid;
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
            min_cost = FLT_MAX;
            const i64 b = ((i64)i * W + j) * D;
            for (int d = 0; d < D; ++d) {
                const i64 k = b + d;
                S[k] = L[0][k] + L[1][k] + L[2][k] + L[3][k];
                S[k] += (L[4][k] + L[5][k] + L[6][k] + L[7][k]);
                if (S[k] < min_cost) { min_cost = S[k]; min_d = d; }
            }
            sec_min_cost = FLT_MAX;
            for (int d = 0; d < D; ++d)
                if (S[b + d] < sec_min_cost && S[b + d] != min_cost) {
                    sec_min_cost = S[b + d];
                    sec_min_d = d;
                }
            disp[(i64)i * W + j] =
                (min_cost / sec_min_cost > uniq && abs(min_d - sec_min_d) > 1) ? invalid : min_d;
        }
}

/* --------------------------------------------------------- whole process */

enum { MODE_PARITY = 0, MODE_LEAN = 1, MODE_REFPLACE = 2 };

static int process_mode(const uint8_t *left, const uint8_t *right,
                        const uint8_t *sky_l, const uint8_t *sky_r,
                        int h, int w, int scale, int D, int P1i, int P2i,
                        float uniq, float lr_dis, int blur, int views, orc_result *res, int mode)
{
    if (h <= 0 || w <= 0 || (scale != 1 && scale != 2) || D <= 0) return -1;
    const int H = h / scale, W = w / scale;
    const i64 npx = (i64)H * W, nvol = npx * D;
    if (W < 5 || H < 3) return -1;
    const float P1 = (float)P1i, P2 = (float)P2i;

    uint8_t *l = (uint8_t *)malloc((size_t)npx), *r = (uint8_t *)malloc((size_t)npx);
    /* decimation, src/SGM.cpp:40-61 */
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
            l[(i64)i * W + j] = left[(i64)i * scale * w + (i64)j * scale];
            r[(i64)i * W + j] = right[(i64)i * scale * w + (i64)j * scale];
        }
    /* build_cost_table, src/Solver.cpp:120-140 */
    uint8_t *lb = l, *rb = r;
    if (blur) {
        lb = (uint8_t *)malloc((size_t)npx);
        rb = (uint8_t *)malloc((size_t)npx);
        orc_blur(l, lb, H, W);
        orc_blur(r, rb, H, W);
    }
    uint64_t *ctl = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)npx);
    uint64_t *ctr = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)npx);
    orc_census(lb, ctl, H, W, scale);
    orc_census(rb, ctr, H, W, scale);

    float *cost = (float *)malloc(sizeof(float) * (size_t)nvol);
    float *S = (float *)malloc(sizeof(float) * (size_t)nvol);
    float *T = NULL;
    float *Ls[8] = {0}, *mins[8] = {0};
    if (mode == MODE_LEAN) {
        T = (float *)malloc(sizeof(float) * (size_t)nvol);
    } else {
        for (int k = 0; k < 8; ++k) {
            Ls[k] = (float *)malloc(sizeof(float) * (size_t)nvol);
            mins[k] = (float *)malloc(sizeof(float) * (size_t)npx);
        }
    }
    int32_t *disp = (int32_t *)malloc(sizeof(int32_t) * (size_t)npx);
    int32_t *disp_b = (int32_t *)malloc(sizeof(int32_t) * (size_t)npx);
    float *sub = (float *)malloc(sizeof(float) * (size_t)npx);
    float *sub_b = (float *)malloc(sizeof(float) * (size_t)npx);

    for (int view = 0; view < (views >= 2 ? 2 : 1); ++view) {
        int32_t *dv = view == 0 ? disp : disp_b;
        orc_dsi(ctl, ctr, view == 0 ? sky_l : sky_r, cost, H, W, D, scale, view);
        /* the reference runs both filters sequentially (Solver.cpp:296-368) */
        hfilter_impl(cost, H, W, D, 5 / scale, mode != MODE_REFPLACE);
        vfilter_impl(cost, H, W, D, 3 / scale, mode != MODE_REFPLACE);
        if (mode == MODE_LEAN) {
            lean_rows(cost, S, H, W, D, P1, P2);
            lean_cols(cost, S, H, W, D, P1, P2);
            lean_diag(cost, S, T, H, W, D, P1, P2, 1);
            lean_diag(cost, S, T, H, W, D, P1, P2, 0);
            wta_par(S, dv, H, W, D, uniq);
        } else if (mode == MODE_REFPLACE) {
            for (int k = 0; k < 4; ++k) orc_path(cost, Ls[k], mins[k], H, W, D, k, P1i, P2i);
            refplace_diag_pair(cost, Ls[4], Ls[5], mins[4], mins[5], H, W, D, P1, P2, 1);
            refplace_diag_pair(cost, Ls[6], Ls[7], mins[6], mins[7], H, W, D, P1, P2, 0);
            refplace_agg_wta(Ls, S, dv, H, W, D, uniq);
        } else {
            for (int k = 0; k < 8; ++k) orc_path(cost, Ls[k], mins[k], H, W, D, k, P1i, P2i);
            orc_aggregate((const float *const *)Ls, S, H, W, D);
            orc_wta(S, dv, H, W, D, uniq);
        }
        orc_subpixel(dv, S, view == 0 ? sub : sub_b, H, W, D);
    }

    if (res) {
        if (res->disp) memcpy(res->disp, disp, sizeof(int32_t) * (size_t)npx);
        if (res->sub) memcpy(res->sub, sub, sizeof(float) * (size_t)npx);
        if (views >= 2) {
            if (res->disp_beta) memcpy(res->disp_beta, disp_b, sizeof(int32_t) * (size_t)npx);
            if (res->sub_beta) memcpy(res->sub_beta, sub_b, sizeof(float) * (size_t)npx);
            float *lr = (float *)malloc(sizeof(float) * (size_t)npx);
            memcpy(lr, sub, sizeof(float) * (size_t)npx);
            orc_lr_check(lr, sub_b, H, W, D, scale, lr_dis);
            if (res->lr) memcpy(res->lr, lr, sizeof(float) * (size_t)npx);
            if (res->final_disp) {
                orc_post_filter(lr, H, W, D, scale);
                memcpy(res->final_disp, lr, sizeof(float) * (size_t)npx);
            }
            free(lr);
        }
    }

    for (int k = 0; k < 8; ++k) {
        free(Ls[k]);
        free(mins[k]);
    }
    free(T);
    free(cost); free(S); free(disp); free(disp_b); free(sub); free(sub_b);
    free(ctl); free(ctr);
    if (blur) { free(lb); free(rb); }
    free(l); free(r);
    return 0;
}

int orc_process(const uint8_t *left, const uint8_t *right,
                const uint8_t *sky_l, const uint8_t *sky_r,
                int h, int w, int scale, int D, int P1, int P2,
                float uniq, float lr_dis, int blur, int views, orc_result *res)
{
    return process_mode(left, right, sky_l, sky_r, h, w, scale, D, P1, P2, uniq, lr_dis, blur,
                        views, res, MODE_PARITY);
}

int orc_process_lean(const uint8_t *left, const uint8_t *right,
                     const uint8_t *sky_l, const uint8_t *sky_r,
                     int h, int w, int scale, int D, int P1, int P2,
                     float uniq, float lr_dis, int blur, int views, orc_result *res)
{
    return process_mode(left, right, sky_l, sky_r, h, w, scale, D, P1, P2, uniq, lr_dis, blur,
                        views, res, MODE_LEAN);
}

int orc_process_refplace(const uint8_t *left, const uint8_t *right,
                         const uint8_t *sky_l, const uint8_t *sky_r,
                         int h, int w, int scale, int D, int P1, int P2,
                         float uniq, float lr_dis, int blur, int views, orc_result *res)
{
    return process_mode(left, right, sky_l, sky_r, h, w, scale, D, P1, P2, uniq, lr_dis, blur,
                        views, res, MODE_REFPLACE);
}
