// sgm_sky.hip -- SkyAreaDetector::detect (sky_detector/imageSkyDetector.cpp:
// 166-208, the path node.cpp:82-86 feeds into SGM::process) on the GPU,
// bit-exact against oracle/sgm_oracle.c:orc_sky_detect, whose numerics
// reproduce the reference's own mask for example/000017_14.
//
// The detector picks, among 120 gradient thresholds t_k = 5 + 3(k-1), the
// per-column sky border (first row of the top half whose Sobel magnitude
// exceeds t_k) that maximises an energy of the sky and ground intensity
// variances; then drops columns with a dark sky pixel, isolated columns and
// runs narrower than 30.  Five launches, no host round trip:
//   1. gray:    working-grid image (2x2 average at scale 2) + moments of all
//               non-zero pixels;
//   2. columns: one thread per column scans the top half once: a row whose
//               |grad|^2 exceeds the next thresholds' t^2 is their border
//               (or -1), recorded with the sky moments above it; the first
//               dark (< 128) row; then one workgroup per threshold sums the
//               columns' sky moments;
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

// One detection's buffers; launches take both views and pick theirs by the
// workgroup's z index (node.cpp:83-86 detects on both images).
struct SkyView {
    const uint8_t *img;
    uint8_t *mask;
    unsigned long long *tot;
    int *B, *M, *dark, *border;
    uint8_t *G;
    long long *partial;
};
struct SkyViews {
    SkyView v[2];
};
__device__ __forceinline__ int bid_z() { return (int)__builtin_amdgcn_workgroup_id_z(); }

__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// 1. working-grid gray image + moments of the non-zero pixels: 64 x 16
// pixels per workgroup, one partial triple per workgroup (summed in 2b).
__global__ __launch_bounds__(256) void sky_gray_kernel(SkyViews sv, int pitch, int s, int H, int W) {
    const SkyView &V = sv.v[bid_z()];
    const uint8_t *__restrict__ img = V.img;
    uint8_t *__restrict__ G = V.G;
    long long *partial = V.partial;
    __shared__ long long part[3][4];
    const int lane = tid_x() & 63, wave = tid_x() >> 6;
    const int j = bid_x() * 64 + lane;
    int n = 0, s1 = 0, s2 = 0;  // <= 4 pixels per thread
    for (int r = 0; r < 4; ++r) {
        const int i = bid_y() * 16 + wave * 4 + r;
        if (i >= H || j >= W) continue;
        int g;
        if (s == 1) {
            g = img[(size_t)i * pitch + j];
        } else {  // cv::resize INTER_LINEAR to half size as the 8U fixed-point 2x2 mean
            const uint8_t *a = img + (size_t)(2 * i) * pitch + 2 * j, *b = a + pitch;
            g = ((int)a[0] + a[1] + b[0] + b[1] + 2) >> 2;
        }
        G[(size_t)i * W + j] = (uint8_t)g;
        if (g) { ++n; s1 += g; s2 += g * g; }
    }
    const long long wn = wave_sum64(n), w1 = wave_sum64(s1), w2 = wave_sum64(s2);
    if (lane == 0) { part[0][wave] = wn; part[1][wave] = w1; part[2][wave] = w2; }
    __syncthreads();
    if (tid_x() < 3)
        partial[3 * (bid_y() * (int)gridDim.x + bid_x()) + tid_x()] =
            part[tid_x()][0] + part[tid_x()][1] + part[tid_x()][2] + part[tid_x()][3];
}

__device__ __forceinline__ int reflect101(int x, int n) {  // BORDER_REFLECT_101
    if (n == 1) return 0;
    x = x < 0 ? -x : x;
    x = x >= n ? 2 * n - 2 - x : x;
    return x < 0 ? 0 : (x >= n ? n - 1 : x);
}

// 2. per column: the border of every threshold (extract_border, :288-343) with
// the sky moments above it (calculate_sky_energy, :633-646), the first dark
// row (check_sky_border_by_gray_value, :101-109).  A workgroup owns 64
// columns: its four waves first stage the top-half strip (rows 0..half+1,
// columns c0-1..c0+64 at reflected coordinates, plus columns W-1 and 0 for the
// row-wrapping grad_y probe of the edge columns) in LDS, then wave 0 scans it,
// one lane per column.
constexpr int kSkyStripW = 68;  // 66 window columns, then G[r][W-1], G[r][0]
constexpr size_t kSkyStripMax = 160 * 1024 - 1024;
__global__ __launch_bounds__(256) void sky_columns_kernel(SkyViews sv, int H, int W) {
    const SkyView &V = sv.v[bid_z()];
    const uint8_t *__restrict__ G = V.G;
    int *__restrict__ B = V.B;
    int *__restrict__ M = V.M;
    int *__restrict__ dark = V.dark;
    extern __shared__ uint8_t strip[];  // [rows 0..last+1][kSkyStripW]
    const int c0 = bid_x() * 64, t = tid_x();
    const int half = H / 2, last = half < H - 1 ? half : H - 1;
    const int nrows = last + 2 < H ? last + 2 : H;  // rows 0..last+1 that exist
    // 8 loads in flight per thread before their LDS stores
    const int total = nrows * kSkyStripW;
    for (int q0 = 0; q0 < total; q0 += 8 * 256) {
        uint8_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * 256 + t;
            const int r = q / kSkyStripW, x = q - r * kSkyStripW;
            const int col = x < 66 ? reflect101(c0 - 1 + x, W) : (x == 66 ? W - 1 : 0);
            v[u] = q < total ? G[(size_t)r * W + col] : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * 256 + t;
            if (q < total) strip[q] = v[u];
        }
    }
    __syncthreads();
    if (t >= 64) return;
    const int c = c0 + t;
    if (c >= W) return;
    const size_t kW = (size_t)kSkyT * W;
    auto row3 = [&](int r) {  // (G[r][c-1], G[r][c], G[r][c+1]) packed, reflected
        const uint8_t *q = strip + reflect101(r, H) * kSkyStripW + t;
        return (int)q[0] | ((int)q[1] << 8) | ((int)q[2] << 16);
    };
    // |Sobel|^2 of row r from rows r-1, r, r+1 (ksize 3, :215-232)
    auto sob2 = [](int pv, int cu, int nv) {
        const int dx = (((pv >> 16) & 255) + 2 * ((cu >> 16) & 255) + ((nv >> 16) & 255)) -
                       ((pv & 255) + 2 * (cu & 255) + (nv & 255));
        const int dy = ((nv & 255) + 2 * ((nv >> 8) & 255) + ((nv >> 16) & 255)) -
                       ((pv & 255) + 2 * ((pv >> 8) & 255) + ((pv >> 16) & 255));
        return (long long)(dx * dx + dy * dy);
    };
    // Thresholds in increasing order: the first row whose |grad|^2 > t_k^2
    // never moves up as k grows, so one pointer walks the column once; the
    // moments of the rows above it are the sky moments of that border.
    int r = 0, n = 0, s1 = 0, s2 = 0, fd = H;
    int pv = row3(-1), cu = row3(0), nv = row3(1);
    long long a = sob2(pv, cu, nv);
    for (int k = 0; k < kSkyT; ++k) {
        const long long t2 = sky_t2(k);
        while (r <= last && !(a > t2)) {
            const int g = (cu >> 8) & 255;
            if (g < 128 && fd == H) fd = r;
            if (g) { ++n; s1 += g; s2 += g * g; }
            ++r;
            pv = cu;
            cu = nv;
            nv = row3(r + 1);
            a = sob2(pv, cu, nv);
        }
        int b = -1;
        if (r <= last && r < half && r > 5) {
            // grad_y (:309-314) reads (r +- 1, c +- 1) by row-major flat index
            // (cv::Mat::at): the register window for inner columns; at the edge
            // columns the index wraps into the neighbouring row
            const uint8_t *sr = strip + t + 1;  // (row 0, column c)
            auto S = [&](int rr, int dc) { return (int)sr[rr * kSkyStripW + dc]; };
            int gy;
            if (c > 0 && c < W - 1) {
                gy = (2 * ((nv >> 8) & 255) + ((nv >> 16) & 255) + (nv & 255)) -
                     (2 * ((pv >> 8) & 255) + ((pv >> 16) & 255) + (pv & 255));
            } else if (c == 0) {  // (r+1, -1) = (r, W-1); (r-1, -1) = (r-2, W-1)
                gy = (2 * S(r + 1, 0) + S(r + 1, 1) + (int)strip[r * kSkyStripW + 66]) -
                     (2 * S(r - 1, 0) + S(r - 1, 1) + (int)strip[(r - 2) * kSkyStripW + 66]);
            } else {              // (r+1, W) = (r+2, 0); (r-1, W) = (r, 0)
                gy = (2 * S(r + 1, 0) + (int)strip[(r + 2) * kSkyStripW + 67] + S(r + 1, -1)) -
                     (2 * S(r - 1, 0) + (int)strip[r * kSkyStripW + 67] + S(r - 1, -1));
            }
            b = gy > 0 ? -1 : r;
        }
        B[(size_t)k * W + c] = b;
        M[(size_t)k * W + c] = b < 0 ? 0 : n;
        M[kW + (size_t)k * W + c] = b < 0 ? 0 : s1;
        M[2 * kW + (size_t)k * W + c] = b < 0 ? 0 : s2;
    }
    for (; r <= last && fd == H; ++r)  // the first dark row of the top half
        if ((int)strip[r * kSkyStripW + t + 1] < 128) fd = r;
    dark[c] = fd;
}

// 2b. per threshold k < kSkyT: the sums of the columns' sky moments; block
// kSkyT: the image totals from the gray kernel's partials
__global__ __launch_bounds__(256) void sky_reduce_kernel(SkyViews sv, int W, int npart) {
    const SkyView &V = sv.v[bid_z()];
    const int *__restrict__ M = V.M;
    const long long *__restrict__ partial = V.partial;
    unsigned long long *tot = V.tot;
    __shared__ long long part[3][4];
    const int k = bid_x(), lane = tid_x() & 63, wave = tid_x() >> 6;
    const size_t kW = (size_t)kSkyT * W;
    long long n = 0, s1 = 0, s2 = 0;
    if (k < kSkyT) {
        const int *m0 = M + (size_t)k * W, *m1 = m0 + kW, *m2 = m1 + kW;
        for (int c = tid_x(); c < W; c += 256) {
            n += m0[c];
            s1 += m1[c];
            s2 += (unsigned)m2[c];
        }
    } else {
        for (int b = tid_x(); b < npart; b += 256) {
            n += partial[3 * b];
            s1 += partial[3 * b + 1];
            s2 += partial[3 * b + 2];
        }
    }
    n = wave_sum64(n);
    s1 = wave_sum64(s1);
    s2 = wave_sum64(s2);
    if (lane == 0) { part[0][wave] = n; part[1][wave] = s1; part[2][wave] = s2; }
    __syncthreads();
    if (tid_x() < 3)
        tot[3 * k + tid_x()] = (unsigned long long)(part[tid_x()][0] + part[tid_x()][1] +
                                                    part[tid_x()][2] + part[tid_x()][3]);
}

// 3. energies, the chosen border, the column checks (one workgroup)
__global__ __launch_bounds__(1024) void sky_select_kernel(SkyViews sv, int H, int W) {
    const SkyView &V = sv.v[bid_z()];
    const int *__restrict__ B = V.B;
    const int *__restrict__ dark = V.dark;
    const unsigned long long *tot = V.tot;
    int *__restrict__ border = V.border;
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
__global__ __launch_bounds__(256) void sky_mask_kernel(SkyViews sv, int H, int W, int pitch) {
    const SkyView &V = sv.v[bid_z()];
    const int *__restrict__ border = V.border;
    uint8_t *__restrict__ mask = V.mask;
    const int j = bid_x() * 64 + (tid_x() & 63), i = bid_y() * 4 + (tid_x() >> 6);
    if (i < H && j < W) mask[(size_t)i * pitch + j] = i <= border[j] ? 255 : 0;
}

}  // namespace

size_t sky_scratch_bytes(Geom g) {
    const size_t W = (size_t)g.W, npx = (size_t)g.H * g.W;
    const size_t bytes = kSkyTotBytes            // totals
                         + 4 * kSkyT * W         // borders per threshold
                         + 3 * 4 * kSkyT * W     // sky moments per threshold
                         + 2 * 4 * W             // dark rows, final border
                         + npx                   // gray image
                         + 64 + 24 * (size_t)((g.W + 63) / 64) * ((g.H + 15) / 16);  // partials
    return (bytes + 255) & ~(size_t)255;  // the second view's scratch starts here: keep it aligned
}

hipError_t launch_sky_detect(const uint8_t *const *img, int pitch, uint8_t *const *mask,
                             int mask_pitch, void *scratch, int nviews, Geom g, hipStream_t st) {
    if (g.W > kSkyMaxW || nviews < 1 || nviews > 2) return hipErrorInvalidValue;
    const size_t W = (size_t)g.W;
    SkyViews sv{};
    for (int v = 0; v < nviews; ++v) {
        char *p = (char *)scratch + v * sky_scratch_bytes(g);
        SkyView &V = sv.v[v];
        V.img = img[v];
        V.mask = mask[v];
        V.tot = (unsigned long long *)p;  p += kSkyTotBytes;
        V.B = (int *)p;                   p += 4 * kSkyT * W;
        V.M = (int *)p;                   p += 3 * 4 * kSkyT * W;
        V.dark = (int *)p;                p += 4 * W;
        V.border = (int *)p;              p += 4 * W;
        V.G = (uint8_t *)p;               p += (size_t)g.H * W;
        V.partial = (long long *)(((uintptr_t)p + 63) & ~(uintptr_t)63);
    }
    const dim3 gridg((g.W + 63) / 64, (g.H + 15) / 16, nviews);
    hipLaunchKernelGGL(sky_gray_kernel, gridg, dim3(256), 0, st, sv, pitch, g.scale, g.H, g.W);
    const int half = g.H / 2, last = half < g.H - 1 ? half : g.H - 1;
    const size_t strip = (size_t)(last + 2) * kSkyStripW;
    if (strip > kSkyStripMax) return hipErrorInvalidValue;  // H > ~4700 rows
    hipError_t e = hipFuncSetAttribute((const void *)sky_columns_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)strip);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sky_columns_kernel, dim3((g.W + 63) / 64, 1, nviews), dim3(256), strip, st,
                       sv, g.H, g.W);
    hipLaunchKernelGGL(sky_reduce_kernel, dim3(kSkyT + 1, 1, nviews), dim3(256), 0, st, sv, g.W,
                       (int)(gridg.x * gridg.y));
    hipLaunchKernelGGL(sky_select_kernel, dim3(1, 1, nviews), dim3(1024), 0, st, sv, g.H, g.W);
    hipLaunchKernelGGL(sky_mask_kernel, dim3((g.W + 63) / 64, (g.H + 3) / 4, nviews), dim3(256), 0,
                       st, sv, g.H, g.W, mask_pitch);
    return hipGetLastError();
}

}  // namespace sgm
