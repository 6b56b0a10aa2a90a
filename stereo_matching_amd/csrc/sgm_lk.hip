// sgm_lk.hip -- LKRefine (LKRefine/LKSubPixelImpl.cpp:13-235) on the GPU:
// per-pixel Gauss-Newton refinement of the disparity offset over a 7x7
// window, bit-exact against oracle/sgm_oracle.c:orc_lk_refine (whose fp32
// evaluation order of the reference's Eigen expressions it follows).
//
// One thread per pixel, 64x4 pixels per workgroup.  The window inputs that do
// not move between iterations -- the truncated disparities, the gradients
// Ix = (L(j+1) - L(j-1)) * 0.5 and the left pixels -- are staged in LDS for
// the tile plus a 3-pixel apron; the right-image samples R(m, n - d) move
// with the offset and are gathered from global memory, all 49 in flight at
// once, into registers.  The slot tests that do not depend on the offset
// are made once per pixel; an iteration then makes up to three passes over
// the window: (A) the image-edge test, sum w^2 and the right samples, (B) the
// Hessian, only when the set of valid slots changed (it is a function of that
// set), (C) the offset.  Zero-weight slots are skipped: adding +0 (or -0)
// never changes an fp32 sum, so the sums equal the reference's 49-term ones.
#include "sgm_device.h"

namespace sgm {
namespace {

constexpr int kLkTW = 64, kLkTH = 4;      // pixels per workgroup
constexpr int kLkHW = 3;                  // half window (win_size 7, LKSubPixelImpl.h:45)
constexpr int kLkAW = kLkTW + 2 * kLkHW;  // apron tile width  (70)
constexpr int kLkAH = kLkTH + 2 * kLkHW;  // apron tile height (10)
constexpr int kLkThreads = kLkTW * kLkTH;

__global__ __launch_bounds__(kLkThreads) void lk_refine_kernel(
    const uint8_t *__restrict__ left, const uint8_t *__restrict__ right, int pitch, int s,
    const float *__restrict__ din, float *__restrict__ dout, int out_pitch, int H, int W, int D) {
    __shared__ float dtT[kLkAH][kLkAW];   // truncated disparity (interior), else as given
    __shared__ float ixT[kLkAH][kLkAW];   // gradient, 0 outside the interior
    __shared__ int lT[kLkAH][kLkAW];      // left pixel

    const int t = tid_x();
    const int i0 = bid_y() * kLkTH, j0 = bid_x() * kLkTW;
    const float fD = (float)D;
    // apron: rows i0-3 .. i0+6, cols j0-3 .. j0+66 (+1 column each side for Ix)
    for (int q = t; q < kLkAH * kLkAW; q += kLkThreads) {
        const int r = q / kLkAW, c = q % kLkAW;
        const int m = i0 - kLkHW + r, n = j0 - kLkHW + c;
        float d = 0.f, ix = 0.f;
        int lv = 0;
        if (m >= 0 && m < H && n >= 0 && n < W) {
            const uint8_t *lrow = left + (size_t)m * s * pitch;
            lv = lrow[(size_t)n * s];
            d = din[(size_t)m * W + n];
            if (m >= kLkHW && m < H - kLkHW && n >= kLkHW && n < W - kLkHW) {  // :70-82
                ix = (float)((int)lrow[(size_t)(n + 1) * s] - (int)lrow[(size_t)(n - 1) * s]) * 0.5f;
                d = (float)(int)d;
            }
        }
        dtT[r][c] = d;
        ixT[r][c] = ix;
        lT[r][c] = lv;
    }
    __syncthreads();

    const int tr = t / kLkTW, tc = t % kLkTW;
    const int i = i0 + tr, j = j0 + tc;
    if (i >= H || j >= W) return;
    const int ar = tr + kLkHW, ac = tc + kLkHW;  // this pixel in the apron
    const float d0 = dtT[ar][ac];
    float result = d0;  // interior: truncated (:80); border: untouched
    const bool interior = i >= kLkHW && i < H - kLkHW && j >= kLkHW && j < W - kLkHW;
    if (interior && ixT[ar][ac] > 2.f && d0 > 0.f && d0 < fD) {  // :90-101
        const float wc = 0.36787945f;            // (float)exp(-1): corner slots (:154)
        const float wc2 = wc * wc;
        float last_disp = d0, last_doff = 0.f, last_diff = FLT_MAX;
        // the slot tests that do not move with the offset (:131-140):
        // gradient, disparity range, |d0 - dm| <= 2
        unsigned long long fixed = 0;
#pragma unroll
        for (int k = 0; k < 49; ++k) {
            const int v = k / 7 - kLkHW, u = k % 7 - kLkHW;
            const float ix = ixT[ar + v][ac + u];
            const float dm = dtT[ar + v][ac + u];
            if (ix > 2.f && dm > 0.f && dm < fD && !(fabsf(d0 - dm) > 2.f)) fixed |= 1ull << k;
        }
        // the Hessian depends only on the set of valid slots; only the
        // image-edge test moves with the offset, so after the first iteration
        // it is usually reused (bit-identical: the same sum over the same set)
        unsigned long long hs_valid = ~0ull;     // no set of 49 slots is all ones
        float hs = 0.f;
        for (int it = 0; it < 10; ++it) {        // iter_num (LKSubPixelImpl.h:46)
            // (A) the window (:114-163): valid slots and sum w^2, then the
            // right samples, all 49 loads issued before any is used
            unsigned long long valid = 0;
            int nvalid = 0;
            float s2 = 0.f;
            int rx[49];
#pragma unroll
            for (int k = 0; k < 49; ++k) {
                const int v = k / 7 - kLkHW, u = k % 7 - kLkHW;
                const float dm = dtT[ar + v][ac + u];
                const int n = j + u;
                const float x = (float)n - (dm + last_doff);
                const bool ok = ((fixed >> k) & 1) && !(x < 0.f || x > (float)(W - 1));
                rx[k] = ok ? (int)x : j;  // a safe column for the skipped slots
                if (ok) {
                    valid |= 1ull << k;
                    ++nvalid;
                    s2 += (v * v + u * u >= 18) ? wc2 : 1.f;
                }
            }
            int rv[49];
#pragma unroll
            for (int k = 0; k < 49; ++k) {
                const int v = k / 7 - kLkHW;
                rv[k] = right[(size_t)(i + v) * s * pitch + (size_t)rx[k] * s];
            }
            if (nvalid < 5) break;               // valid_cnt < 4.9 (:165)
            const float nrm = sqrtf(s2);         // win_weight.norm() (:172)
            const float wn1 = 1.f / nrm, wnc = wc / nrm;
            // (B) Hessian = (J^T W) J (:176)
            if (valid != hs_valid) {
                hs_valid = valid;
                hs = 0.f;
#pragma unroll
                for (int k = 0; k < 49; ++k) {
                    if (!((valid >> k) & 1)) continue;
                    const int v = k / 7 - kLkHW, u = k % 7 - kLkHW;
                    const float ix = ixT[ar + v][ac + u];
                    hs += (ix * ((v * v + u * u >= 18) ? wnc : wn1)) * ix;
                }
            }
            if ((double)hs < 1e-3) break;        // :178 (Hessian(0,0) < 1e-3, a double)
            // (C) doff = ((H^-1 J^T) W) Ires (:185)
            const float hinv = 1.f / hs;
            float doff = 0.f;
#pragma unroll
            for (int k = 0; k < 49; ++k) {
                if (!((valid >> k) & 1)) continue;
                const int v = k / 7 - kLkHW, u = k % 7 - kLkHW;
                const float ix = ixT[ar + v][ac + u];
                const float res = (float)(rv[k] - lT[ar + v][ac + u]);  // Ires (:156)
                doff += ((hinv * ix) * ((v * v + u * u >= 18) ? wnc : wn1)) * res;
            }
            if (fabsf(doff - last_doff) > last_diff) break;   // :201
            const float dn = d0 + doff;
            if (!(dn > 0.f && dn < fD)) break;               // :207
            last_disp = dn;
            last_diff = fabsf(doff - last_doff);
            last_doff = doff;
            if ((double)last_diff < 1e-6) break;              // :222
        }
        result = last_disp;
    }
    dout[(size_t)i * out_pitch + j] = result;
}

}  // namespace

hipError_t launch_lk_refine(const uint8_t *left, const uint8_t *right, int pitch, const float *din,
                            float *dout, int out_pitch, Geom g, hipStream_t st) {
    const dim3 grid((g.W + kLkTW - 1) / kLkTW, (g.H + kLkTH - 1) / kLkTH);
    hipLaunchKernelGGL(lk_refine_kernel, grid, dim3(kLkThreads), 0, st, left, right, pitch,
                       g.scale, din, dout, out_pitch, g.H, g.W, g.D);
    return hipGetLastError();
}

}  // namespace sgm
