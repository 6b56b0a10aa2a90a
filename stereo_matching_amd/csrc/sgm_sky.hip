// sgm_sky.hip -- SkyAreaDetector::detect (sky_detector/imageSkyDetector.cpp:
// 166-208, the path node.cpp:82-86 feeds into SGM::process) on the GPU,
// bit-exact against oracle/sgm_oracle.c:orc_sky_detect, whose numerics
// reproduce the reference's own mask for example/000017_14.
//
// The detector picks, among 120 gradient thresholds t_k = 5 + 3(k-1), the
// per-column sky border (first row of the top half whose Sobel magnitude
// exceeds t_k) that maximises an energy of the sky and ground intensity
// variances; then drops columns with a dark sky pixel, isolated columns and
// runs narrower than 30.  Four launches, no host round trip:
//   1. gray:    working-grid image (2x2 average at scale 2) + moments of all
//               non-zero pixels;
//   2. columns: one thread per column scans the top half once: a row whose
//               |grad|^2 exceeds the next thresholds' t^2 is their border
//               (or -1), recorded with the sky moments above it; the first
//               dark (< 128) row; then per-threshold sums over the wave;
//   3. select:  one workgroup: energies, the first maximum, the gray-value
//               and isolated-column checks (parallel: a dropped isolated
//               column can never enable its right neighbour's drop), and the
//               narrow-run removal with ballot words;
//   4. mask:    255 where row <= border.
#include "sgm_device.h"

namespace sgm {
namespace {

constexpr int kSkyT = 120;            // thresholds: floor((600-5)/5)+1 (:248-249)
constexpr int kSkyMaxW = 8192;        // widest working grid the select kernel holds in LDS
constexpr size_t kSkyTotBytes = 4096; // scratch header: 3 x (kSkyT + 1) u64 totals
__device__ __forceinline__ long long sky_t2(int k) {  // t_k^2, t_k = 5 + 3k (:259-263)
    const long long t = 5 + 3 * k;
    return t * t;
}

__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// 1. working-grid gray image + totals of the non-zero pixels (tot[kSkyT][*])
__global__ __launch_bounds__(256) void sky_gray_kernel(const uint8_t *__restrict__ img, int pitch,
                                                      int s, uint8_t *__restrict__ G, int H, int W,
                                                      unsigned long long *tot) {
    const int j = bid_x() * 64 + (tid_x() & 63), i = bid_y() * 4 + (tid_x() >> 6);
    long long n = 0, s1 = 0, s2 = 0;
    if (i < H && j < W) {
        int g;
        if (s == 1) {
            g = img[(size_t)i * pitch + j];
        } else {  // cv::resize INTER_LINEAR to half size as the 8U fixed-point 2x2 mean
            const uint8_t *a = img + (size_t)(2 * i) * pitch + 2 * j, *b = a + pitch;
            g = ((int)a[0] + a[1] + b[0] + b[1] + 2) >> 2;
        }
        G[(size_t)i * W + j] = (uint8_t)g;
        if (g) { n = 1; s1 = g; s2 = (long long)g * g; }
    }
    n = wave_sum64(n);
    s1 = wave_sum64(s1);
    s2 = wave_sum64(s2);
    if ((tid_x() & 63) == 0 && n) {
        atomicAdd(tot + 3 * kSkyT + 0, (unsigned long long)n);
        atomicAdd(tot + 3 * kSkyT + 1, (unsigned long long)s1);
        atomicAdd(tot + 3 * kSkyT + 2, (unsigned long long)s2);
    }
}

__device__ __forceinline__ int reflect101(int x, int n) {  // BORDER_REFLECT_101
    if (n == 1) return 0;
    x = x < 0 ? -x : x;
    x = x >= n ? 2 * n - 2 - x : x;
    return x < 0 ? 0 : (x >= n ? n - 1 : x);
}

// 2. per column: the border of every threshold (extract_border, :288-343) with
// the sky moments above it (calculate_sky_energy, :633-646), the first dark
// row (check_sky_border_by_gray_value, :101-109); per-threshold wave sums.
// Rows are read 8 at a time ahead of use (3 pixels each: c-1, c, c+1).
__global__ __launch_bounds__(64) void sky_columns_kernel(const uint8_t *__restrict__ G, int H,
                                                        int W, int *__restrict__ B,
                                                        int *__restrict__ M,
                                                        int *__restrict__ dark,
                                                        unsigned long long *tot) {
    const int c = bid_x() * 64 + tid_x();
    const int half = H / 2, last = half < H - 1 ? half : H - 1;
    const size_t kW = (size_t)kSkyT * W;
    if (c < W) {
        const int cm = reflect101(c - 1, W), cp = reflect101(c + 1, W);
        auto row3 = [&](int r) {  // (G[r][c-1], G[r][c], G[r][c+1]) packed
            const uint8_t *q = G + (size_t)reflect101(r, H) * W;
            return (int)q[cm] | ((int)q[c] << 8) | ((int)q[cp] << 16);
        };
        int kk = 0, n = 0, s1 = 0, s2 = 0, fd = H;
        int pv = row3(-1), cu = row3(0);
        for (int r0 = 0; r0 <= last; r0 += 8) {
            int nx[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) nx[q] = row3(r0 + q + 1);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int r = r0 + q;
                if (r > last) break;
                const int nv = nx[q];
                // |Sobel|^2, ksize 3 (:215-232)
                const int dx = (((pv >> 16) & 255) + 2 * ((cu >> 16) & 255) + ((nv >> 16) & 255)) -
                               ((pv & 255) + 2 * (cu & 255) + (nv & 255));
                const int dy = ((nv & 255) + 2 * ((nv >> 8) & 255) + ((nv >> 16) & 255)) -
                               ((pv & 255) + 2 * ((pv >> 8) & 255) + ((pv >> 16) & 255));
                const long long a = dx * dx + dy * dy;
                while (kk < kSkyT && a > sky_t2(kk)) {
                    int b = -1;
                    if (r < half && r > 5) {
                        // grad_y (:309-314): row-major flat neighbours, as cv::Mat::at
                        const size_t up = (size_t)(r - 1) * W + c, dn = (size_t)(r + 1) * W + c;
                        const int gy = (2 * (int)G[dn] + G[dn + 1] + G[dn - 1]) -
                                       (2 * (int)G[up] + G[up + 1] + G[up - 1]);
                        b = gy > 0 ? -1 : r;
                    }
                    B[(size_t)kk * W + c] = b;
                    M[(size_t)kk * W + c] = b < 0 ? 0 : n;
                    M[kW + (size_t)kk * W + c] = b < 0 ? 0 : s1;
                    M[2 * kW + (size_t)kk * W + c] = b < 0 ? 0 : s2;
                    ++kk;
                }
                const int g = (cu >> 8) & 255;
                if (g < 128 && fd == H) fd = r;
                if (g) { ++n; s1 += g; s2 += g * g; }
                pv = cu;
                cu = nv;
            }
        }
        for (; kk < kSkyT; ++kk) {
            B[(size_t)kk * W + c] = -1;
            M[(size_t)kk * W + c] = 0;
            M[kW + (size_t)kk * W + c] = 0;
            M[2 * kW + (size_t)kk * W + c] = 0;
        }
        dark[c] = fd;
    }
    for (int k = 0; k < kSkyT; ++k) {
        long long n = 0, s1 = 0, s2 = 0;
        if (c < W) {
            n = M[(size_t)k * W + c];
            s1 = M[kW + (size_t)k * W + c];
            s2 = (unsigned)M[2 * kW + (size_t)k * W + c];
        }
        n = wave_sum64(n);
        s1 = wave_sum64(s1);
        s2 = wave_sum64(s2);
        if (tid_x() == 0 && n) {
            atomicAdd(tot + 3 * k + 0, (unsigned long long)n);
            atomicAdd(tot + 3 * k + 1, (unsigned long long)s1);
            atomicAdd(tot + 3 * k + 2, (unsigned long long)s2);
        }
    }
}

// 3. energies, the chosen border, the column checks (one workgroup)
__global__ __launch_bounds__(1024) void sky_select_kernel(const int *__restrict__ B,
                                                         const int *__restrict__ dark,
                                                         const unsigned long long *tot, int H,
                                                         int W, int *__restrict__ border) {
    __shared__ double jn[kSkyT];
    __shared__ int kbest;
    __shared__ int bo[kSkyMaxW], bg[kSkyMaxW], bx[kSkyMaxW];
    __shared__ unsigned long long vw[kSkyMaxW / 64];
    const int t = tid_x();
    if (t < kSkyT) {  // calculate_sky_energy (:564-705) with a gray (rank-1) covariance
        const long long N = (long long)tot[3 * kSkyT], S1 = (long long)tot[3 * kSkyT + 1],
                        S2 = (long long)tot[3 * kSkyT + 2];
        const long long ns = (long long)tot[3 * t], s1 = (long long)tot[3 * t + 1],
                        s2 = (long long)tot[3 * t + 2];
        const long long ng = N - ns, g1 = S1 - s1, g2 = S2 - s2;
        double e;
        if (ng == 0 || ns == 0) {
            e = DBL_MIN;
        } else {
            const double vs = (double)(ns * s2 - s1 * s1) / ((double)ns * (double)ns);
            const double vg = (double)(ng * g2 - g1 * g1) / ((double)ng * (double)ng);
            const double sky_det = 0.0, ground_det = 0.0;
            e = 1 / ((2 * sky_det + ground_det) + (2 * (3 * vs) + (3 * vg)));
        }
        jn[t] = e;
    }
    __syncthreads();
    if (t == 0) {  // jn > jn_max keeps the first maximum (:273-276)
        double m = 0.0;
        int kb = -1;
        for (int k = 0; k < kSkyT; ++k)
            if (jn[k] > m) { m = jn[k]; kb = k; }
        kbest = kb;
    }
    __syncthreads();
    const int kb = kbest;
    for (int c = t; c < W; c += 1024) {
        const int b = kb < 0 ? H - 1 : B[(size_t)kb * W + c];
        bo[c] = b;
        bg[c] = b > dark[c] ? -1 : b;  // a row j < border with gray < 128 (:101-109)
    }
    __syncthreads();
    // isolated columns (:111-116): x[c-1] = bg[c-1] whenever the rule can
    // fire at c (it needs bo[c] != -1, which keeps the rule off at c-1)
    for (int c = t; c < W; c += 1024) {
        int x = bg[c];
        if (bo[c] != -1 && c > 1 && bg[c - 1] == -1 && c < W - 1 && bo[c + 1] == -1) x = -1;
        bx[c] = x;
    }
    __syncthreads();
    for (int c0 = 0; c0 < W; c0 += 1024) {
        const int c = c0 + t;
        const unsigned long long m = __ballot(c < W && bx[c] != -1);
        if ((t & 63) == 0 && c < W) vw[c >> 6] = m;
    }
    __syncthreads();
    // runs of kept columns (:119-163): [p, q) with q = end + 1, except that a
    // run whose next column is the last one counts it (q = W); q - p < 30 drops
    const int nw = (W + 63) >> 6;
    for (int c = t; c < W; c += 1024) {
        int x = bx[c];
        if (x != -1) {
            int w = c >> 6;
            // start: the highest clear bit below c
            unsigned long long z = ~vw[w] & ((1ull << (c & 63)) - 1);
            while (!z && w > 0) z = ~vw[--w];
            const int p = z ? (w << 6) + 63 - __builtin_clzll(z) + 1 : 0;
            // end: the lowest clear bit above c (bits past W are clear)
            w = c >> 6;
            unsigned long long y = (c & 63) == 63 ? 0 : (~vw[w] & ~((2ull << (c & 63)) - 1));
            while (!y && w + 1 < nw) y = ~vw[++w];
            int e = y ? (w << 6) + __builtin_ctzll(y) - 1 : W - 1;
            if (e > W - 1) e = W - 1;
            const int q = (e + 1 == W - 1) ? W : e + 1;
            if (q - p < 30) x = -1;  // f_thres_sky_width (imageSkyDetector.h:33)
        }
        border[c] = x;
    }
}

// 4. make_sky_mask type 1 (:804-812)
__global__ __launch_bounds__(256) void sky_mask_kernel(const int *__restrict__ border, int H, int W,
                                                      uint8_t *__restrict__ mask, int pitch) {
    const int j = bid_x() * 64 + (tid_x() & 63), i = bid_y() * 4 + (tid_x() >> 6);
    if (i < H && j < W) mask[(size_t)i * pitch + j] = i <= border[j] ? 255 : 0;
}

}  // namespace

size_t sky_scratch_bytes(Geom g) {
    const size_t W = (size_t)g.W, npx = (size_t)g.H * g.W;
    return kSkyTotBytes                          // totals
           + 4 * kSkyT * W                       // borders per threshold
           + 3 * 4 * kSkyT * W                   // sky moments per threshold
           + 2 * 4 * W                           // dark rows, final border
           + npx;                                // gray image
}

hipError_t launch_sky_detect(const uint8_t *img, int pitch, uint8_t *mask, int mask_pitch,
                             void *scratch, Geom g, hipStream_t st) {
    if (g.W > kSkyMaxW) return hipErrorInvalidValue;
    const size_t W = (size_t)g.W;
    char *p = (char *)scratch;
    unsigned long long *tot = (unsigned long long *)p;
    p += kSkyTotBytes;
    int *B = (int *)p;             p += 4 * kSkyT * W;
    int *M = (int *)p;             p += 3 * 4 * kSkyT * W;
    int *dark = (int *)p;          p += 4 * W;
    int *border = (int *)p;        p += 4 * W;
    uint8_t *G = (uint8_t *)p;
    hipError_t e = hipMemsetAsync(tot, 0, 8 * 3 * (kSkyT + 1), st);
    if (e != hipSuccess) return e;
    const dim3 grid2((g.W + 63) / 64, (g.H + 3) / 4);
    hipLaunchKernelGGL(sky_gray_kernel, grid2, dim3(256), 0, st, img, pitch, g.scale, G, g.H, g.W,
                       tot);
    hipLaunchKernelGGL(sky_columns_kernel, dim3((g.W + 63) / 64), dim3(64), 0, st, G, g.H, g.W, B,
                       M, dark, tot);
    hipLaunchKernelGGL(sky_select_kernel, dim3(1), dim3(1024), 0, st, B, dark, tot, g.H, g.W,
                       border);
    hipLaunchKernelGGL(sky_mask_kernel, grid2, dim3(256), 0, st, border, g.H, g.W, mask,
                       mask_pitch);
    return hipGetLastError();
}

}  // namespace sgm
