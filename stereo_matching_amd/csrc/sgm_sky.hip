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
//   2. columns: per (row, column) the number of thresholds whose t^2 its
//               |grad|^2 exceeds; then one thread per column walks the top
//               half once: a row whose count exceeds every earlier row's is
//               the border (or -1) of the new thresholds, recorded with the
//               sky moments above it; the first dark (< 128) row; then one
//               workgroup per threshold sums the columns' sky moments;
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
// row (check_sky_border_by_gray_value, :101-109).  A workgroup owns 16
// columns.  Its four waves stage the top-half strip (rows 0..half+1, columns
// c0-1..c0+16 at reflected coordinates, plus columns W-1 and 0 for the
// row-wrapping grad_y probe of the edge columns) in LDS.  Then, per column
// and group of 16 rows, they compute every row's count of the thresholds its
// |grad|^2 exceeds, and the group's largest count and sky moments.  The
// border of threshold k is the first row whose count exceeds k, so one lane
// per column walks its groups: a group whose largest count resolves no new
// threshold only adds its moments; in the others, a row whose count exceeds
// every earlier row's is the border of the new thresholds, whose results
// (border or -1, the moments of the rows above it) go to an LDS table.  All
// threads then write the table out, one coalesced row of columns per
// threshold.
constexpr int kSkyCols = 16;             // columns per workgroup
constexpr int kSkyStripW = kSkyCols + 4; // 18 window columns, then G[r][W-1], G[r][0]
constexpr int kSkyGrp = 16;              // rows per group
constexpr size_t kSkyStripMax = 160 * 1024 - 1024;
// #{k < kSkyT : t_k^2 < a}, thresholds t_k = 5 + 3k (:259-263)
__device__ __forceinline__ int sky_count(int a) {
    if (a <= 25) return 0;                          // t_0 = 5
    const int x = a - 1;                            // t^2 < a  <=>  t <= isqrt(a - 1)
    int q = (int)sqrtf((float)x);
    while (q * q > x) --q;
    while ((q + 1) * (q + 1) <= x) ++q;
    const int n = (q - 5) / 3 + 1;                  // t_k = 5 + 3k <= q
    return n < kSkyT ? n : kSkyT;
}
#ifdef SGM_STAMPS
__device__ unsigned long long sky_stamps[4];  // staging, counts, walk + table cycles; blocks
#endif
// LDS layout: strip [last+2][kSkyStripW] u8 | (16 B aligned) counts
// [kSkyCols][ngrp] x 16 u8 | group stats [kSkyCols][ngrp] int4 (largest count,
// n, s1, s2) | results [kSkyT][kSkyCols] int4 | first dark row, resolved
// thresholds per column
struct SkyLds {
    size_t counts, stats, table, dark, done, bytes;
    __host__ __device__ SkyLds(int last) {
        const size_t ngrp = (size_t)(last + kSkyGrp) / kSkyGrp;
        counts = ((size_t)(last + 2) * kSkyStripW + 15) & ~(size_t)15;
        stats = counts + 16 * kSkyCols * ngrp;
        table = stats + 16 * kSkyCols * ngrp;
        dark = table + (size_t)16 * kSkyT * kSkyCols;
        done = dark + 4 * kSkyCols;
        bytes = done + 4 * kSkyCols;
    }
};
__global__ __launch_bounds__(256) void sky_columns_kernel(SkyViews sv, int H, int W) {
    const SkyView &V = sv.v[bid_z()];
    const uint8_t *__restrict__ G = V.G;
    int *__restrict__ B = V.B;
    int *__restrict__ M = V.M;
    int *__restrict__ dark = V.dark;
    extern __shared__ uint8_t strip[];
    const int c0 = bid_x() * kSkyCols, t = tid_x();
#ifdef SGM_STAMPS
    const long long ts0 = __builtin_amdgcn_s_memtime();
#endif
    const int half = H / 2, last = half < H - 1 ? half : H - 1;
    const int nrows = last + 2 < H ? last + 2 : H;  // rows 0..last+1 that exist
    const int ngrp = (last + kSkyGrp) / kSkyGrp;
    const SkyLds lay(last);
    uint4 *counts = reinterpret_cast<uint4 *>(strip + lay.counts);
    int4 *stats = reinterpret_cast<int4 *>(strip + lay.stats);
    int4 *table = reinterpret_cast<int4 *>(strip + lay.table);
    int *darkL = reinterpret_cast<int *>(strip + lay.dark);
    int *kdone = reinterpret_cast<int *>(strip + lay.done);
    if (t < kSkyCols) darkL[t] = H;
    // 8 loads in flight per thread before their LDS stores
    const int total = nrows * kSkyStripW;
    for (int q0 = 0; q0 < total; q0 += 8 * 256) {
        uint8_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * 256 + t;
            const int r = q / kSkyStripW, x = q - r * kSkyStripW;
            const int col = x < kSkyCols + 2 ? reflect101(c0 - 1 + x, W) : (x == kSkyCols + 2 ? W - 1 : 0);
            v[u] = q < total ? G[(size_t)r * W + col] : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int q = q0 + u * 256 + t;
            if (q < total) strip[q] = v[u];
        }
    }
    __syncthreads();
#ifdef SGM_STAMPS
    const long long ts1 = __builtin_amdgcn_s_memtime();
#endif
    // per (column, group of 16 rows): |Sobel|^2 (ksize 3, :215-232) of each
    // row from rows r-1, r, r+1 at reflected coordinates, as the count of
    // thresholds it exceeds; the group's largest count and moments; the
    // column's first dark row
    for (int q = t; q < ngrp * kSkyCols; q += 256) {
        const int x = q % kSkyCols, grp = q / kSkyCols;
        unsigned w[4] = {0, 0, 0, 0};
        int mx = 0, n = 0, s1 = 0, s2 = 0, fd = H;
#pragma unroll
        for (int i = 0; i < kSkyGrp; ++i) {
            const int r = grp * kSkyGrp + i;
            if (r <= last) {
                const uint8_t *p = strip + reflect101(r - 1, H) * kSkyStripW + x;
                const uint8_t *m = strip + r * kSkyStripW + x;
                const uint8_t *nx = strip + reflect101(r + 1, H) * kSkyStripW + x;
                const int dx = ((int)p[2] + 2 * m[2] + nx[2]) - ((int)p[0] + 2 * m[0] + nx[0]);
                const int dy = ((int)nx[0] + 2 * nx[1] + nx[2]) - ((int)p[0] + 2 * p[1] + p[2]);
                const int k = sky_count(dx * dx + dy * dy);
                w[i >> 2] |= (unsigned)k << (8 * (i & 3));
                mx = k > mx ? k : mx;
                const int g = m[1];
                if (g) { ++n; s1 += g; s2 += g * g; }
                if (g < 128 && fd == H) fd = r;
            }
        }
        counts[x * ngrp + grp] = make_uint4(w[0], w[1], w[2], w[3]);
        stats[x * ngrp + grp] = make_int4(mx, n, s1, s2);
        if (fd < H) atomicMin(&darkL[x], fd);
    }
    __syncthreads();
#ifdef SGM_STAMPS
    const long long ts2 = __builtin_amdgcn_s_memtime();
#endif
    const int c = c0 + t;
    if (t < kSkyCols && c < W) {
        const uint8_t *sr = strip + t + 1;  // (row 0, column c)
        auto S = [&](int rr, int dc) { return (int)sr[rr * kSkyStripW + dc]; };
        int kcur = 0, n = 0, s1 = 0, s2 = 0;
        for (int grp = 0; grp < ngrp; ++grp) {
            const int4 st = stats[t * ngrp + grp];
            if (st.x <= kcur) {  // no row of the group resolves a new threshold
                n += st.y;
                s1 += st.z;
                s2 += st.w;
                continue;
            }
            const uint4 kq = counts[t * ngrp + grp];
            const unsigned kw[4] = {kq.x, kq.y, kq.z, kq.w};
            int gv[kSkyGrp];
#pragma unroll
            for (int i = 0; i < kSkyGrp; ++i) {
                const int r = grp * kSkyGrp + i;
                gv[i] = r <= last ? S(r, 0) : 0;
            }
#pragma unroll
            for (int i = 0; i < kSkyGrp; ++i) {
                const int r = grp * kSkyGrp + i;
                const int kr = (kw[i >> 2] >> (8 * (i & 3))) & 255;  // 0 past the last row
                if (kr > kcur) {  // the border of thresholds kcur..kr-1
                    int b = -1;
                    if (r < half && r > 5) {
                        // grad_y (:309-314) reads (r +- 1, c +- 1) by row-major flat
                        // index (cv::Mat::at): at the edge columns the index wraps
                        // into the neighbouring row
                        int gy;
                        if (c > 0 && c < W - 1) {
                            gy = (2 * S(r + 1, 0) + S(r + 1, 1) + S(r + 1, -1)) -
                                 (2 * S(r - 1, 0) + S(r - 1, 1) + S(r - 1, -1));
                        } else if (c == 0) {  // (r+1, -1) = (r, W-1); (r-1, -1) = (r-2, W-1)
                            gy = (2 * S(r + 1, 0) + S(r + 1, 1) + S(r, kSkyCols + 1 - t)) -
                                 (2 * S(r - 1, 0) + S(r - 1, 1) + S(r - 2, kSkyCols + 1 - t));
                        } else {              // (r+1, W) = (r+2, 0); (r-1, W) = (r, 0)
                            gy = (2 * S(r + 1, 0) + S(r + 2, kSkyCols + 2 - t) + S(r + 1, -1)) -
                                 (2 * S(r - 1, 0) + S(r, kSkyCols + 2 - t) + S(r - 1, -1));
                        }
                        b = gy > 0 ? -1 : r;
                    }
                    const int4 e = b < 0 ? make_int4(-1, 0, 0, 0) : make_int4(b, n, s1, s2);
                    for (; kcur < kr; ++kcur) table[kcur * kSkyCols + t] = e;
                }
                const int g = gv[i];
                if (g) { ++n; s1 += g; s2 += g * g; }
            }
        }
        kdone[t] = kcur;  // thresholds kcur.. have no border in the top half
        dark[c] = darkL[t];
    }
    __syncthreads();
    const size_t kW = (size_t)kSkyT * W;
    for (int q = t; q < kSkyT * kSkyCols; q += 256) {
        const int k = q / kSkyCols, x = q - k * kSkyCols, cc = c0 + x;
        if (cc >= W) continue;
        const int4 e = k < kdone[x] ? table[q] : make_int4(-1, 0, 0, 0);
        const size_t o = (size_t)k * W + cc;
        B[o] = e.x;
        M[o] = e.y;
        M[kW + o] = e.z;
        M[2 * kW + o] = e.w;
    }
#ifdef SGM_STAMPS
    const long long ts3 = __builtin_amdgcn_s_memtime();
    if (t == 0) {
        atomicAdd(&sky_stamps[0], (unsigned long long)(ts1 - ts0));
        atomicAdd(&sky_stamps[1], (unsigned long long)(ts2 - ts1));
        atomicAdd(&sky_stamps[2], (unsigned long long)(ts3 - ts2));
        atomicAdd(&sky_stamps[3], 1ull);
    }
#endif
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
    const size_t strip = SkyLds(last).bytes;
    if (strip > kSkyStripMax) return hipErrorInvalidValue;  // H > ~4700 rows
    // the kernel's dynamic-LDS ceiling is one value for the whole process:
    // always the same maximum, so handles of other frame sizes running on
    // other host threads can never lower it under this launch
    hipError_t e = hipFuncSetAttribute((const void *)sky_columns_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSkyStripMax);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sky_columns_kernel, dim3((g.W + kSkyCols - 1) / kSkyCols, 1, nviews),
                       dim3(256), strip, st,
                       sv, g.H, g.W);
    hipLaunchKernelGGL(sky_reduce_kernel, dim3(kSkyT + 1, 1, nviews), dim3(256), 0, st, sv, g.W,
                       (int)(gridg.x * gridg.y));
    hipLaunchKernelGGL(sky_select_kernel, dim3(1, 1, nviews), dim3(1024), 0, st, sv, g.H, g.W);
    hipLaunchKernelGGL(sky_mask_kernel, dim3((g.W + 63) / 64, (g.H + 3) / 4, nviews), dim3(256), 0,
                       st, sv, g.H, g.W, mask_pitch);
    return hipGetLastError();
}

}  // namespace sgm

#ifdef SGM_STAMPS
extern "C" int sgm_debug_stamps_sky(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sgm::sky_stamps), sizeof(sgm::sky_stamps)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[4] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sgm::sky_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
