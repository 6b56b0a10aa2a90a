/*
 * lk_orders.c -- how far LKRefine's result moves under other fp32 evaluation
 * orders of its Eigen sums (north_star: LK sub-pixel
 * values within 1e-4 of the reference).
 *
 * ANALYSIS TOOL (test infrastructure, like oracle/): restates
 * oracle/sgm_oracle.c:orc_lk_refine (LKRefine/LKSubPixelImpl.cpp:56-240) with
 * the three 49-term reductions of one Gauss-Newton iteration made pluggable:
 *   s2   = win_weight.squaredNorm()            (:172, norm() = sqrt(s2))
 *   H    = (J^T * Weight) * J                  (:176, inner product)
 *   doff = ((H^-1 * J^T) * Weight) * win_Ires  (:185, inner product)
 * Weight is a DENSE 49x49 MatrixXf (:175, win_weight.asDiagonal() converted),
 * so J^T * Weight is a GEMV whose every output sums 48 explicit zero terms and
 * one product; ORDER_GEMV evaluates it that way (all 49 terms, index order)
 * to show the zeros change nothing for finite J.
 * Orders:
 *   0 ORDER_INDEX  k = 0..48 sequentially (the oracle's and the GPU's order)
 *   1 ORDER_SSE    Eigen's LinearVectorizedTraversal redux with Packet4f (the
 *                  reference's flags, -O3 without -march = SSE2): accumulators
 *                  r0 = P0+P2+..+P10, r1 = P1+P3+..+P11 (packets of 4), r0+r1,
 *                  predux (l0+l2)+(l1+l3), then + element 48
 *   2 ORDER_AVX    the same with Packet8f (an -mavx build): r0 = P0+P2+P4,
 *                  r1 = P1+P3+P5, r0+r1, 8->4 lanes (lo+hi), then the 4-lane
 *                  predux, then + element 48
 *   3 ORDER_PAIR   pairwise (recursive halving)
 *   4 ORDER_GEMV   J^T*Weight and (H^-1 J^T)*Weight as full 49-term GEMVs
 *                  with explicit zeros (index order), dot products as SSE
 * Per pixel it records the refined value, the iterations run and the exit
 * reason, so a caller can count break tests that flip between orders.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef long long i64;
enum { ORDER_INDEX = 0, ORDER_SSE = 1, ORDER_AVX = 2, ORDER_PAIR = 3, ORDER_GEMV = 4 };

static float sum_index(const float *x, int n)
{
    float s = 0.f;
    for (int k = 0; k < n; ++k) s += x[k];
    return s;
}

static float predux4(const float *l) { return (l[0] + l[2]) + (l[1] + l[3]); }

static float sum_packets(const float *x, int n, int P)
{
    /* Eigen/src/Core/Redux.h, LinearVectorizedTraversal, NoUnrolling, aligned start 0 */
    const int aligned2 = (n / (2 * P)) * (2 * P), aligned = (n / P) * P;
    if (aligned == 0) return sum_index(x, n);
    float r0[8], r1[8];
    for (int l = 0; l < P; ++l) r0[l] = x[l];
    if (aligned > P) {
        for (int l = 0; l < P; ++l) r1[l] = x[P + l];
        for (int i = 2 * P; i < aligned2; i += 2 * P)
            for (int l = 0; l < P; ++l) {
                r0[l] = r0[l] + x[i + l];
                r1[l] = r1[l] + x[i + P + l];
            }
        for (int l = 0; l < P; ++l) r0[l] = r0[l] + r1[l];
        if (aligned > aligned2)
            for (int l = 0; l < P; ++l) r0[l] = r0[l] + x[aligned2 + l];
    }
    float res;
    if (P == 8) {
        float h[4];
        for (int l = 0; l < 4; ++l) h[l] = r0[l] + r0[l + 4];
        res = predux4(h);
    } else {
        res = predux4(r0);
    }
    for (int i = aligned; i < n; ++i) res = res + x[i];
    return res;
}

static float sum_pair(const float *x, int n)
{
    if (n == 1) return x[0];
    const int h = n / 2;
    return sum_pair(x, h) + sum_pair(x + h, n - h);
}

static float reduce(const float *x, int n, int order)
{
    switch (order) {
    case ORDER_SSE:
    case ORDER_GEMV: return sum_packets(x, n, 4);
    case ORDER_AVX: return sum_packets(x, n, 8);
    case ORDER_PAIR: return sum_pair(x, n);
    default: return sum_index(x, n);
    }
}

/* GEMV of a row vector a (1x49) with the dense diagonal matrix diag(w):
 * out[k] = sum_m a[m] * W[m][k], every term evaluated, index order. */
static void gemv_diag(const float *a, const float *w, float *out)
{
    for (int k = 0; k < 49; ++k) {
        float s = 0.f;
        for (int m = 0; m < 49; ++m) s += a[m] * (m == k ? w[k] : 0.f);
        out[k] = s;
    }
}

/* exit reasons */
enum { EXIT_NONE = 0, EXIT_ITERS, EXIT_VALID, EXIT_HESS, EXIT_NAN, EXIT_DIVERGE, EXIT_RANGE, EXIT_CONV };

void lk_refine_order(const uint8_t *L, const uint8_t *R, float *disp, int H, int W, int D,
                     int order, int32_t *iters_out, int32_t *exit_out)
{
    const int hw = 3, win = 7, iters = 10;
    const i64 n = (i64)H * W;
    float *Ix = (float *)calloc((size_t)n, sizeof(float));
    float *dt = (float *)malloc(sizeof(float) * (size_t)n);
    float *nd = (float *)malloc(sizeof(float) * (size_t)n);
    memcpy(dt, disp, sizeof(float) * (size_t)n);
    memcpy(nd, disp, sizeof(float) * (size_t)n);
    for (i64 k = 0; k < n; ++k) { iters_out[k] = 0; exit_out[k] = EXIT_NONE; }
    for (int i = hw; i < H - hw; ++i)
        for (int j = hw; j < W - hw; ++j) {
            const i64 k = (i64)i * W + j;
            Ix[k] = (float)((int)L[k + 1] - (int)L[k - 1]) * 0.5f;
            nd[k] = (float)(int)disp[k];
            dt[k] = (float)(int)disp[k];
        }
#pragma omp parallel for schedule(dynamic, 4)
    for (int i = hw; i < H - hw; ++i) {
        for (int j = hw; j < W - hw; ++j) {
            const i64 c = (i64)i * W + j;
            if (!(Ix[c] > 2)) continue;
            const float d0 = dt[c];
            if (!(d0 > 0 && d0 < D)) continue;
            float last_disp = d0, last_doff = 0.f, last_diff = FLT_MAX;
            int it = 0, why = EXIT_ITERS;
            for (; it < iters; ++it) {
                float w[49], jx[49], res[49], t[49], u[49];
                int cnt = 0, valid = 0;
                for (int v = -hw; v <= hw; ++v)
                    for (int uu = -hw; uu <= hw; ++uu, ++cnt) {
                        const int m = i + v, nn = j + uu;
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
                        w[cnt] = (float)exp((double)(-(v * v + uu * uu) / (2 * hw * hw)));
                        res[cnt] = (float)((int)R[(i64)m * W + (int)((float)nn - dw)] - (int)L[k]);
                        jx[cnt] = Ix[k];
                        ++valid;
                    }
                if (valid < win * win * 0.1) { why = EXIT_VALID; break; }
                for (int k = 0; k < 49; ++k) t[k] = w[k] * w[k];
                const float nrm = sqrtf(reduce(t, 49, order));
                for (int k = 0; k < 49; ++k) w[k] = w[k] / nrm;
                if (order == ORDER_GEMV) gemv_diag(jx, w, u);              /* J^T * Weight */
                else for (int k = 0; k < 49; ++k) u[k] = jx[k] * w[k];
                for (int k = 0; k < 49; ++k) t[k] = u[k] * jx[k];
                const float hs = reduce(t, 49, order);
                if (isnan(hs) || (double)hs < 1e-3) { why = EXIT_HESS; break; }
                const float hinv = 1.0f / hs;
                for (int k = 0; k < 49; ++k) t[k] = hinv * jx[k];            /* H^-1 * J^T */
                if (order == ORDER_GEMV) gemv_diag(t, w, u);                /* ... * Weight */
                else for (int k = 0; k < 49; ++k) u[k] = t[k] * w[k];
                for (int k = 0; k < 49; ++k) t[k] = u[k] * res[k];
                const float doff = reduce(t, 49, order);
                if (isnan(doff)) { why = EXIT_NAN; break; }
                if (fabsf(doff - last_doff) > last_diff) { why = EXIT_DIVERGE; break; }
                if (!(d0 + doff > 0 && d0 + doff < D)) { why = EXIT_RANGE; break; }
                last_disp = d0 + doff;
                last_diff = fabsf(doff - last_doff);
                last_doff = doff;
                if ((double)last_diff < 1e-6) { why = EXIT_CONV; ++it; break; }
            }
            nd[c] = last_disp;
            iters_out[c] = it;
            exit_out[c] = why;
        }
    }
    memcpy(disp, nd, sizeof(float) * (size_t)n);
    free(Ix);
    free(dt);
    free(nd);
}
