// sgm_kernels.hip -- CDNA4 (gfx950) kernels of the semi-global matcher.
//
// Stage map (reference -> kernel), full design in DESIGN.md:
//   cv::GaussianBlur + CT_pts     Solver.cpp:120-140, cost.cpp:99-129  -> census_kernel
//   build_dsi_from_table[_beta]   Solver.cpp:143-248
//     + cost_horizontal_filter    Solver.cpp:296-330                   -> cost_h_kernel
//   cost_vertical_filter          Solver.cpp:333-368                   -> cost_v_kernel
//   L1..L8 path DP                SGM.cpp:81-369                       -> sweep_kernel<DIR,..>
//   aggregation + WTA + unique    SGM.cpp:372-418
//     + compute_subpixel          Solver.cpp:569-597                   -> sweep_kernel<..,FINAL>
//   LR check                      SGM.cpp:803-818                      -> lr_kernel
//
// Bit-exactness rules (DESIGN.md "Numerics"): built with -ffp-contract=off,
// no fast-math, correctly rounded f32 division; every float expression keeps
// the reference's association order.
#include "sgm_internal.h"

#include <float.h>
#include <limits.h>

namespace sgm {

#define SGM_INF __builtin_inff()

// ---------------------------------------------------------------- helpers

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// DPP move with an explicit fill value for lanes whose source is invalid or
// masked off (bound_ctrl = 0 keeps `old`).
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ float dppf(float old, float src) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src),
                                                      CTRL, ROW_MASK, BANK_MASK, false));
}
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ int dppi(int old, int src) {
    return __builtin_amdgcn_update_dpp(old, src, CTRL, ROW_MASK, BANK_MASK, false);
}

// DPP controls (GFX9 encoding, valid on gfx950).
constexpr int DPP_QP_1032 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int DPP_QP_2301 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141;
constexpr int DPP_MIRROR = 0x140;
constexpr int DPP_BCAST15 = 0x142;
constexpr int DPP_BCAST31 = 0x143;
constexpr int DPP_WAVE_SHL1 = 0x130;  // lane i reads lane i+1
constexpr int DPP_WAVE_SHR1 = 0x138;  // lane i reads lane i-1

// Plain DPP move (no fill value, bound_ctrl set): only for patterns whose
// consumed lanes all have a valid source, so the compiler folds the move into
// the consuming VALU op (v_min_f32_dpp).
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ int movdpp(int src) {
    return __builtin_amdgcn_mov_dpp(src, CTRL, ROW_MASK, BANK_MASK, true);
}
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
__device__ __forceinline__ float movdppf(float src) {
    return __int_as_float(movdpp<CTRL, ROW_MASK, BANK_MASK>(__float_as_int(src)));
}

// Minimum over the 64 lanes, left in EVERY lane (a VGPR, no readlane on the
// DP chain): the quad, half-row and row mirrors give each lane its row (16
// lane) minimum; v_permlane16_swap pairs rows 0<->1 and 2<->3, and
// v_permlane32_swap the two wave halves (gfx950).
__device__ __forceinline__ float wave_min(float x) {
    x = fminf(x, movdppf<DPP_QP_1032>(x));
    x = fminf(x, movdppf<DPP_QP_2301>(x));
    x = fminf(x, movdppf<DPP_HALF_MIRROR>(x));
    x = fminf(x, movdppf<DPP_MIRROR>(x));
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x),
                                                    false, false);
    x = fminf(__uint_as_float(p[0]), __uint_as_float(p[1]));
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x),
                                                    false, false);
    return fminf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}

// Same, returned as a wave-uniform scalar.
__device__ __forceinline__ float wave_min_u(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_min(x))));
}

__device__ __forceinline__ int wave_min_i(int x) {
    x = min(x, movdpp<DPP_QP_1032>(x));
    x = min(x, movdpp<DPP_QP_2301>(x));
    x = min(x, movdpp<DPP_HALF_MIRROR>(x));
    x = min(x, movdpp<DPP_MIRROR>(x));
    x = min(x, movdpp<DPP_BCAST15, 0xA>(x));
    x = min(x, movdpp<DPP_BCAST31, 0xC>(x));
    return __builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ float readlane_f(float x, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane));
}

// ---------------------------------------------------------------- census

// Pinned cv::GaussianBlur(Size(3,3), 2, 1) on CV_8U (Solver.cpp:124-125):
// OpenCV 3.x fixed-point separable filter, kernels {82,93,82} x {70,116,70},
// BORDER_REFLECT_101, (acc + 2^15) >> 16, saturated.  Same formula as
// oracle/sgm_oracle.c:orc_blur (parity unpinned at this boundary).
__device__ __forceinline__ int reflect101(int i, int n) {
    if (n == 1) return 0;
    i = i < 0 ? -i : i;
    return i >= n ? 2 * n - 2 - i : i;
}

__device__ __forceinline__ int blur_at(const uint8_t *src, int pitch, int step, int H, int W,
                                       int y, int x) {
    const int xm = reflect101(x - 1, W) * step, x0 = x * step, xp = reflect101(x + 1, W) * step;
    const int ys[3] = {reflect101(y - 1, H), y, reflect101(y + 1, H)};
    const int ky[3] = {70, 116, 70};
    int acc = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const uint8_t *row = src + (size_t)ys[r] * step * pitch;
        acc += ky[r] * (82 * row[xm] + 93 * row[x0] + 82 * row[xp]);
    }
    const int v = (acc + (1 << 15)) >> 16;
    return v > 255 ? 255 : v;
}

constexpr int CT_TW = 64, CT_TH = 8;

// CT_pts (cost.cpp:99-129) for one image; window (7/s) x (9/s), MSB first,
// centre skipped, coordinates clamped to the (working-grid) edge.  The
// (blurred) window is staged in LDS at clamped coordinates.
template <int HH, int HWW>
__global__ __launch_bounds__(256) void census_kernel(const uint8_t *__restrict__ src, int pitch,
                                                     int step, int H, int W, int blur,
                                                     uint64_t *__restrict__ ct) {
    constexpr int TR = CT_TH + 2 * HH, TC = CT_TW + 2 * HWW;
    __shared__ uint8_t tile[TR][TC];
    const int x0 = blockIdx.x * CT_TW, y0 = blockIdx.y * CT_TH;
    for (int idx = threadIdx.x; idx < TR * TC; idx += 256) {
        const int ty = idx / TC, tx = idx - ty * TC;
        const int y = clampi(y0 + ty - HH, 0, H - 1), x = clampi(x0 + tx - HWW, 0, W - 1);
        tile[ty][tx] = blur ? (uint8_t)blur_at(src, pitch, step, H, W, y, x)
                            : src[(size_t)y * step * pitch + (size_t)x * step];
    }
    __syncthreads();
    const int tx = threadIdx.x & 63;
    for (int r = threadIdx.x >> 6; r < CT_TH; r += 4) {
        const int y = y0 + r, x = x0 + tx;
        if (y >= H || x >= W) continue;
        const uint8_t c = tile[r + HH][tx + HWW];
        uint64_t v = 0;
#pragma unroll
        for (int di = -HH; di <= HH; ++di)
#pragma unroll
            for (int dj = -HWW; dj <= HWW; ++dj) {
                if (di == 0 && dj == 0) continue;
                v = (v << 1) | (uint64_t)(tile[r + HH + di][tx + HWW + dj] > c);
            }
        ct[(size_t)y * W + x] = v;
    }
}

hipError_t launch_census(const uint8_t *src, int pitch, Geom g, int blur, uint64_t *ct,
                         hipStream_t st) {
    dim3 grid((g.W + CT_TW - 1) / CT_TW, (g.H + CT_TH - 1) / CT_TH);
    if (g.scale == 1)
        census_kernel<3, 4><<<grid, 256, 0, st>>>(src, pitch, 1, g.H, g.W, blur, ct);
    else
        census_kernel<1, 2><<<grid, 256, 0, st>>>(src, pitch, 2, g.H, g.W, blur, ct);
    return hipGetLastError();
}

// ------------------------------------------------ DSI + horizontal IIR

// One thread per (row, d) chain, R rows per block (R*D threads).  The census
// rows of both images (and the sky row) are staged in LDS once per block; the
// raw Hamming DSI (Solver.cpp:143-248, sky override :165-178) is produced on
// the fly and fed straight into the in-place horizontal IIR of
// Solver.cpp:296-330, restated with a register history: with h = WIN/2 and
// LAG = WIN-h-1 the reference writes position LAG+t at step t, adds raw[WIN+t]
// and subtracts the value at position t, which is the step-(t-LAG) output once
// t >= LAG and raw before.
constexpr int COSTH_MAX_LDS = 64 * 1024;

template <int VIEW, int WIN, bool SKY, bool FILTER>
__global__ __launch_bounds__(256) void cost_h_kernel(const uint64_t *__restrict__ ctl,
                                                     const uint64_t *__restrict__ ctr,
                                                     const uint8_t *__restrict__ sky,
                                                     int sky_pitch, int H, int W, int D, int scale,
                                                     int R, float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint64_t *sl = reinterpret_cast<uint64_t *>(smem);
    uint64_t *sr = sl + (size_t)R * W;
    uint8_t *ss = reinterpret_cast<uint8_t *>(sr + (size_t)R * W);
    const int row0 = blockIdx.x * R;
    for (int idx = threadIdx.x; idx < R * W; idx += blockDim.x) {
        const int r = idx / W, j = idx - r * W, i = row0 + r;
        if (i < H) {
            sl[idx] = ctl[(size_t)i * W + j];
            sr[idx] = ctr[(size_t)i * W + j];
            if (SKY) ss[idx] = sky[(size_t)i * sky_pitch + j];
        }
    }
    __syncthreads();
    const int r = threadIdx.x / D, d = threadIdx.x - r * D;
    const int i = row0 + r;
    if (i >= H) return;
    const uint64_t *cl = sl + (size_t)r * W;
    const uint64_t *cr = sr + (size_t)r * W;
    const uint8_t *sk = ss + (size_t)r * W;
    const int ds = d / scale;
    float *o = out + (size_t)i * W * D + d;

    auto raw = [&](int j) -> float {
        uint64_t a, b;
        if (VIEW == 0) {
            a = cl[j];
            b = cr[max(j - ds, 0)];
        } else {
            a = cl[min(j + ds, W - 1)];
            b = cr[j];
        }
        const float c = (float)__popcll(a ^ b);
        if (SKY && sk[j] == 255) return d == 0 ? 0.0f : 999999.0f;
        return c;
    };

    if (!FILTER) {
        for (int j = 0; j < W; ++j) o[(size_t)j * D] = raw(j);
        return;
    }
    constexpr int HALF = WIN / 2, LAG = WIN - HALF - 1;
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < WIN; ++k) sum += raw(k);
#pragma unroll
    for (int p = 0; p < LAG; ++p) o[(size_t)p * D] = raw(p);
    const int T = W - 2 * HALF;
    float o1 = 0.0f, o2 = 0.0f;
    const float r0 = raw(0), r1 = raw(1);
#pragma unroll 8
    for (int t = 0; t < T; ++t) {
        const float v = sum / (float)WIN;
        o[(size_t)(LAG + t) * D] = v;
        if (t == T - 1) break;
        sum += raw(WIN + t);
        float a;
        if (LAG == 0) a = v;
        else if (LAG == 1) a = t >= 1 ? o1 : r0;
        else a = t >= 2 ? o2 : (t == 0 ? r0 : r1);
        sum -= a;
        o2 = o1;
        o1 = v;
    }
    for (int p = LAG + T; p < W; ++p) o[(size_t)p * D] = raw(p);
}

// Fallback for rows too wide to stage in LDS (W*16 B > 64 KiB): census words
// read straight from global memory.
template <int VIEW, int WIN, bool SKY, bool FILTER>
__global__ __launch_bounds__(256) void cost_h_global_kernel(const uint64_t *__restrict__ ctl,
                                                            const uint64_t *__restrict__ ctr,
                                                            const uint8_t *__restrict__ sky,
                                                            int sky_pitch, int H, int W, int D,
                                                            int scale, float *__restrict__ out) {
    const int rows_per_block = 256 / D;
    const int r = threadIdx.x / D, d = threadIdx.x - r * D;
    const int i = blockIdx.x * rows_per_block + r;
    if (i >= H) return;
    const uint64_t *cl = ctl + (size_t)i * W;
    const uint64_t *cr = ctr + (size_t)i * W;
    const uint8_t *sk = SKY ? sky + (size_t)i * sky_pitch : nullptr;
    const int ds = d / scale;
    float *o = out + (size_t)i * W * D + d;
    auto raw = [&](int j) -> float {
        if (SKY && sk[j] == 255) return d == 0 ? 0.0f : 999999.0f;
        const uint64_t a = VIEW == 0 ? cl[j] : cl[min(j + ds, W - 1)];
        const uint64_t b = VIEW == 0 ? cr[max(j - ds, 0)] : cr[j];
        return (float)__popcll(a ^ b);
    };
    if (!FILTER) {
        for (int j = 0; j < W; ++j) o[(size_t)j * D] = raw(j);
        return;
    }
    constexpr int HALF = WIN / 2, LAG = WIN - HALF - 1;
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < WIN; ++k) sum += raw(k);
#pragma unroll
    for (int p = 0; p < LAG; ++p) o[(size_t)p * D] = raw(p);
    const int T = W - 2 * HALF;
    float o1 = 0.0f, o2 = 0.0f;
    for (int t = 0; t < T; ++t) {
        const float v = sum / (float)WIN;
        o[(size_t)(LAG + t) * D] = v;
        if (t == T - 1) break;
        sum += raw(WIN + t);
        float a;
        if (LAG == 0) a = v;
        else if (LAG == 1) a = t >= 1 ? o1 : raw(t);
        else a = t >= 2 ? o2 : raw(t);
        sum -= a;
        o2 = o1;
        o1 = v;
    }
    for (int p = LAG + T; p < W; ++p) o[(size_t)p * D] = raw(p);
}

template <int VIEW, int WIN, bool SKY, bool FILTER>
static void launch_cost_h_t(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
                            int sky_pitch, Geom g, float *out, hipStream_t st) {
    const size_t row_bytes = (size_t)g.W * (16 + (SKY ? 1 : 0));
    int R = (int)(COSTH_MAX_LDS / row_bytes);
    if (R > 256 / g.D) R = 256 / g.D;
    if (R >= 1) {
        const size_t smem = (size_t)R * row_bytes;
        cost_h_kernel<VIEW, WIN, SKY, FILTER><<<dim3((g.H + R - 1) / R), R * g.D, smem, st>>>(
            ctl, ctr, sky, sky_pitch, g.H, g.W, g.D, g.scale, R, out);
    } else {
        const int rpb = 256 / g.D;
        cost_h_global_kernel<VIEW, WIN, SKY, FILTER><<<dim3((g.H + rpb - 1) / rpb), 256, 0, st>>>(
            ctl, ctr, sky, sky_pitch, g.H, g.W, g.D, g.scale, out);
    }
}

template <int VIEW, int WIN>
static void launch_cost_h_w(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
                            int sky_pitch, int filter, Geom g, float *out, hipStream_t st) {
    if (sky) {
        if (filter) launch_cost_h_t<VIEW, WIN, true, true>(ctl, ctr, sky, sky_pitch, g, out, st);
        else launch_cost_h_t<VIEW, WIN, true, false>(ctl, ctr, sky, sky_pitch, g, out, st);
    } else {
        if (filter) launch_cost_h_t<VIEW, WIN, false, true>(ctl, ctr, sky, sky_pitch, g, out, st);
        else launch_cost_h_t<VIEW, WIN, false, false>(ctl, ctr, sky, sky_pitch, g, out, st);
    }
}

hipError_t launch_cost_h(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
                         int sky_pitch, int view, int filter, Geom g, float *out,
                         hipStream_t st) {
    if (view == 0) {
        if (g.scale == 1) launch_cost_h_w<0, 5>(ctl, ctr, sky, sky_pitch, filter, g, out, st);
        else launch_cost_h_w<0, 2>(ctl, ctr, sky, sky_pitch, filter, g, out, st);
    } else {
        if (g.scale == 1) launch_cost_h_w<1, 5>(ctl, ctr, sky, sky_pitch, filter, g, out, st);
        else launch_cost_h_w<1, 2>(ctl, ctr, sky, sky_pitch, filter, g, out, st);
    }
    return hipGetLastError();
}

// ------------------------------------------------------ vertical IIR

// One thread per (col, d) chain walking the rows (Solver.cpp:333-368), out of
// place: in = horizontally filtered volume, out = final cost volume.  The raw
// rows the recurrence adds (raw[WIN+t]) stream through a register ring
// VPF steps ahead of the arithmetic.
constexpr int VPF = 16;

template <int WIN>
__global__ __launch_bounds__(256) void cost_v_kernel(const float *__restrict__ in,
                                                     float *__restrict__ out, int H, int W,
                                                     int D) {
    const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t stride = (size_t)W * D;
    if (idx >= stride) return;
    const float *a = in + idx;
    float *o = out + idx;
    constexpr int HALF = WIN / 2, LAG = WIN - HALF - 1;
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < WIN; ++k) sum += a[k * stride];
    const float r0 = a[0], r1 = LAG >= 2 ? a[stride] : 0.0f;
#pragma unroll
    for (int p = 0; p < LAG; ++p) o[p * stride] = a[p * stride];
    const int T = H - 2 * HALF;
    float ring[VPF];
#pragma unroll
    for (int u = 0; u < VPF; ++u) ring[u] = a[(size_t)min(WIN + u, H - 1) * stride];
    float o1 = 0.0f, o2 = 0.0f;
    auto step = [&](int t, int u, bool refill) {
        const float v = sum / (float)WIN;
        o[(size_t)(LAG + t) * stride] = v;
        const float rw = ring[u];
        if (refill) ring[u] = a[(size_t)min(WIN + t + VPF, H - 1) * stride];
        float s;
        if (LAG == 0) s = v;
        else if (LAG == 1) s = t >= 1 ? o1 : r0;
        else s = t >= 2 ? o2 : (t == 0 ? r0 : r1);
        sum = (sum + rw) - s;
        o2 = o1;
        o1 = v;
    };
    // steps 0 .. T-2 update the running sum; step T-1 only writes
    int t0 = 0;
    for (; t0 + VPF <= T - 1; t0 += VPF) {
#pragma unroll
        for (int u = 0; u < VPF; ++u) step(t0 + u, u, true);
    }
#pragma unroll
    for (int u = 0; u < VPF; ++u)
        if (t0 + u < T - 1) step(t0 + u, u, false);
    o[(size_t)(LAG + T - 1) * stride] = sum / (float)WIN;
    for (int p = LAG + T; p < H; ++p) o[(size_t)p * stride] = a[(size_t)p * stride];
}

__global__ __launch_bounds__(256) void copy_kernel(const float *__restrict__ in,
                                                   float *__restrict__ out, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i];
}

hipError_t launch_cost_v(const float *in, float *out, int filter, Geom g, hipStream_t st) {
    const size_t chains = (size_t)g.W * g.D;
    const dim3 grid((unsigned)((chains + 255) / 256));
    if (!filter) {
        const size_t n = chains * g.H;
        copy_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, st>>>(in, out, n);
    } else if (g.scale == 1) {
        cost_v_kernel<3><<<grid, 256, 0, st>>>(in, out, g.H, g.W, g.D);
    } else {
        cost_v_kernel<1><<<grid, 256, 0, st>>>(in, out, g.H, g.W, g.D);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------- sweeps

// Position of one path along its scanline.  Horizontal paths are rows;
// vertical and diagonal paths are indexed by a column g and visit row k at
// column g (vertical) or (g +/- k) mod W (diagonal): when the column wraps the
// chain meets the image edge, which is exactly where the reference restarts
// a diagonal path (SGM.cpp:266,282,330,346), so W chains of H steps cover
// every pixel once per direction.  `off` is the element offset (i*W + j)*D of
// the pixel's disparity vector; everything here is wave-uniform (SALU).
template <int DIR>
struct Cursor {
    int i, j, k;
    long long off;
    __device__ __forceinline__ void init(int path, int H, int W, int D) {
        k = 0;
        if (DIR == 0) { i = path; j = 0; }
        else if (DIR == 1) { i = path; j = W - 1; }
        else if (DIR == 2 || DIR == 4 || DIR == 5) { i = 0; j = path; }
        else { i = H - 1; j = path; }
        off = ((long long)i * W + j) * D;
    }
    __device__ __forceinline__ bool start(int W) const {
        if (k == 0) return true;
        if (DIR == 4 || DIR == 6) return j == 0;
        if (DIR == 5 || DIR == 7) return j == W - 1;
        return false;
    }
    __device__ __forceinline__ void advance(int W, long long D, long long WD) {
        ++k;
        switch (DIR) {
        case 0: ++j; off += D; break;
        case 1: --j; off -= D; break;
        case 2: ++i; off += WD; break;
        case 3: --i; off -= WD; break;
        case 4:
        case 6: {
            const long long di = DIR == 4 ? WD : -WD;
            if (j == W - 1) { j = 0; off += di - (long long)(W - 1) * D; }
            else { ++j; off += di + D; }
            i += DIR == 4 ? 1 : -1;
            break;
        }
        default: {
            const long long di = DIR == 5 ? WD : -WD;
            if (j == 0) { j = W - 1; off += di + (long long)(W - 1) * D; }
            else { --j; off += di - D; }
            i += DIR == 5 ? 1 : -1;
            break;
        }
        }
    }
};

template <int V>
__device__ __forceinline__ void load_v(float (&dst)[V], const float *p, bool active) {
    if (V == 4) {
        float4 t = active ? *reinterpret_cast<const float4 *>(p) : make_float4(SGM_INF, SGM_INF, SGM_INF, SGM_INF);
        dst[0] = t.x; dst[1] = t.y; dst[2] = t.z; dst[3] = t.w;
    } else if (V == 2) {
        float2 t = active ? *reinterpret_cast<const float2 *>(p) : make_float2(SGM_INF, SGM_INF);
        dst[0] = t.x; dst[1] = t.y;
    } else {
        dst[0] = active ? *p : SGM_INF;
    }
}

template <int V>
__device__ __forceinline__ void store_v(float *p, const float (&v)[V], bool active) {
    if (!active) return;
    if (V == 4) *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
    else if (V == 2) *reinterpret_cast<float2 *>(p) = make_float2(v[0], v[1]);
    else *p = v[0];
}

// One DP step of SGM.cpp:93-117 for the V disparities a lane holds
// (d = lane*V + v).  The reference's
//   MIN(MIN(MIN(Lp[d], Lp[d-1]+P1), Lp[d+1]+P1), minLp+P2) + (C - minLp)
// is evaluated as min3(Lp[d], min(Lp[d-1],Lp[d+1]) + P1, minLp+P2) + (C - minLp):
// rounding is monotone so min(a,b)+P1 == min(a+P1,b+P1) bit-for-bit, and a
// missing neighbour at d = 0 / D-1 (the reference clamps to d itself) is
// +inf, which gives the same minimum because fl(x + P1) >= x.
template <int V>
__device__ __forceinline__ void dp_step(const float (&prev)[V], float pmin, const float (&c)[V],
                                        float (&L)[V], float p1, float p2) {
    const float left = dppf<DPP_WAVE_SHR1>(SGM_INF, prev[V - 1]);
    const float right = dppf<DPP_WAVE_SHL1>(SGM_INF, prev[0]);
    const float pmin_p2 = pmin + p2;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const float dm = v == 0 ? left : prev[v - 1];
        const float dp = v == V - 1 ? right : prev[v + 1];
        const float t = fminf(dm, dp) + p1;
        const float m = fminf(fminf(prev[v], t), pmin_p2);
        L[v] = m + (c[v] - pmin);
    }
}

template <int V>
__device__ __forceinline__ float pick(const float (&x)[V], int v) {
    float r = x[0];
#pragma unroll
    for (int k = 1; k < V; ++k) r = v == k ? x[k] : r;
    return r;
}

// Aggregated WTA + uniqueness (SGM.cpp:376-418) and compute_subpixel
// (Solver.cpp:577-593) for one pixel whose total cost vector is spread over
// the wave (d = lane*V + v); everything after the two wave minima is scalar:
// the first index holding a value is the lowest set bit of a ballot.
// Lanes without data hold +inf (never equal to a finite minimum).
template <int V>
__device__ __forceinline__ int first_index(const float (&tot)[V], float x) {
    int best = INT_MAX;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const unsigned long long m = __ballot(tot[v] == x);
        const int cand = m ? (int)__builtin_ctzll(m) * V + v : INT_MAX;
        best = cand < best ? cand : best;
    }
    return best;
}

template <int V>
__device__ __forceinline__ void wta_subpixel(const float (&tot)[V], int D, float uniq,
                                             int &disp_out, float &sub_out) {
    float lm = tot[0];
#pragma unroll
    for (int v = 1; v < V; ++v) lm = fminf(lm, tot[v]);
    const float m = wave_min_u(lm);
    float ls = SGM_INF;
#pragma unroll
    for (int v = 0; v < V; ++v) ls = fminf(ls, tot[v] != m ? tot[v] : SGM_INF);
    const float sec = wave_min_u(ls);
    const int min_d = first_index<V>(tot, m);
    int d = min_d;
    if (sec != SGM_INF) {  // a second distinct value exists (else sec = FLT_MAX: ratio ~ 0)
        const int sec_d = first_index<V>(tot, sec);
        if (m / sec > uniq && abs(min_d - sec_d) > 1) d = D + 1;
    }
    float f;
    if (d > D - 1) {
        f = (float)(D + 1);
    } else if (d == 0 || d == D - 1) {
        f = (float)d;
    } else {
        const float a = readlane_f(pick(tot, (d - 1) % V), (d - 1) / V);
        const float b = readlane_f(pick(tot, (d + 1) % V), (d + 1) / V);
        const float c = readlane_f(pick(tot, d % V), d / V);
        const float x = d + (a - b) / (2 * (a + b - 2 * c));
        const float lim = (D - 1) * 1.f;
        f = (lim < x) ? lim : x;  // std::min(x, lim)
    }
    disp_out = d;
    sub_out = f;
}

// One wavefront per path; lane l holds disparities l*V .. l*V+V-1 (FULL: all
// 64 lanes hold data, i.e. D >= 64; D = 32 uses lanes 0..31 and +inf above).
// Loads run PF steps ahead of the DP through a register ring.  In FINAL mode
// the WTA of pixel k runs one step behind (after the DP of pixel k+1), so the
// scheduler can interleave the two dependency chains.
template <int DIR, int V, int MODE, bool FULL, int PF>
__global__ __launch_bounds__(64) void sweep_kernel(SweepArgs a, Geom g) {
    const int lane = threadIdx.x;
    const int path = blockIdx.x;
    const int H = g.H, W = g.W;
    const long long D = g.D, WD = (long long)g.W * g.D;
    const int n = DIR < 2 ? W : H;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;
    constexpr bool NEED_ACC = MODE == SWEEP_ACC || MODE == SWEEP_FINAL;
    constexpr bool NEED_S = MODE == SWEEP_FINAL;

    Cursor<DIR> cc, pc;
    cc.init(path, H, W, g.D);
    pc.init(path, H, W, g.D);

    float cb[PF][V], ab[PF][V], sb[PF][V];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        load_v<V>(cb[u], a.cost + pc.off + e0, active);
        if (NEED_ACC) load_v<V>(ab[u], a.acc_in + pc.off + e0, active);
        if (NEED_S) load_v<V>(sb[u], a.s_in + pc.off + e0, active);
        if (pc.k < n - 1) pc.advance(W, D, WD);
    }

    float prev[V];
#pragma unroll
    for (int v = 0; v < V; ++v) prev[v] = SGM_INF;
    float pmin = 0.0f;
    // FINAL: the previous pixel's total vector and position (WTA deferred)
    float ptot[V];
#pragma unroll
    for (int v = 0; v < V; ++v) ptot[v] = SGM_INF;
    long long ppx = -1;

    auto finish_prev = [&]() {
        if (ppx >= 0) {
            int dsp;
            float f;
            wta_subpixel<V>(ptot, g.D, a.uniq, dsp, f);
            if (lane == 0) {
                a.disp[ppx] = (uint16_t)dsp;
                a.sub[ppx] = f;
            }
        }
    };

    // One DP step on ring slot u; branch-free so the waitcnt pass can keep
    // exact counts (each slot's loads are waited for PF steps later).
    auto step = [&](int u, bool refill) {
        float c[V], ai[V], si[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            c[v] = cb[u][v];
            ai[v] = ab[u][v];
            si[v] = sb[u][v];
        }
        float L[V];
        dp_step<V>(prev, pmin, c, L, a.p1, a.p2);
        const bool st = cc.start(W);
#pragma unroll
        for (int v = 0; v < V; ++v) L[v] = st ? c[v] : L[v];
        float lm = L[0];
#pragma unroll
        for (int v = 1; v < V; ++v) lm = fminf(lm, L[v]);
        const float nmin = wave_min(lm);

        if (MODE == SWEEP_STORE_L) {
            store_v<V>(a.acc_out + cc.off + e0, L, active);
            if (lane == 0) a.min_out[cc.off / D] = nmin;
        } else if (MODE == SWEEP_INIT) {
            store_v<V>(a.acc_out + cc.off + e0, L, active);
        } else if (MODE == SWEEP_ACC) {
            float o[V];
#pragma unroll
            for (int v = 0; v < V; ++v) o[v] = ai[v] + L[v];
            store_v<V>(a.acc_out + cc.off + e0, o, active);
        } else {
            finish_prev();
            // cost = ((L1+L2)+L3)+L4 ; cost += ((L5+L6)+L7)+L8  (SGM.cpp:386-390)
#pragma unroll
            for (int v = 0; v < V; ++v) ptot[v] = si[v] + (ai[v] + L[v]);
            ppx = (long long)cc.i * W + cc.j;
        }
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = L[v];
        pmin = nmin;
        cc.advance(W, D, WD);
        if (refill) {
            // refill this ring slot only after its old contents are dead, so
            // the new load lands in the same registers (no copy, no wait)
            load_v<V>(cb[u], a.cost + pc.off + e0, active);
            if (NEED_ACC) load_v<V>(ab[u], a.acc_in + pc.off + e0, active);
            if (NEED_S) load_v<V>(sb[u], a.s_in + pc.off + e0, active);
            if (pc.k < n - 1) pc.advance(W, D, WD);
        }
    };

    int k0 = 0;
    for (; k0 + PF <= n; k0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) step(u, true);
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (k0 + u < n) step(u, false);
    if (MODE == SWEEP_FINAL) finish_prev();
}

// LDS-only workgroup barrier: waits for this wave's LDS traffic, not for its
// global loads (the prefetch ring stays in flight across the barrier).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Partial WTA state over a set of disparities: the minimum m and the first
// index i holding it, and the smallest value s != m with its first index si
// (SGM.cpp:383-408: min_cost/min_d, sec_min_cost/sec_min_d).
struct Wta {
    float m, s;
    int i, si;
};

// Combine two disjoint partial states (ties go to the lower index, so the
// merge is symmetric and any lane pairing may be used).
__device__ __forceinline__ Wta wta_merge(const Wta &A, const Wta &B) {
    Wta r;
    float c1, c2;
    int j1, j2;
    if (A.m < B.m) {
        r.m = A.m; r.i = A.i; c1 = A.s; j1 = A.si; c2 = B.m; j2 = B.i;
    } else if (B.m < A.m) {
        r.m = B.m; r.i = B.i; c1 = B.s; j1 = B.si; c2 = A.m; j2 = A.i;
    } else {
        r.m = A.m; r.i = min(A.i, B.i); c1 = A.s; j1 = A.si; c2 = B.s; j2 = B.si;
    }
    r.s = fminf(c1, c2);
    r.si = c1 < c2 ? j1 : (c2 < c1 ? j2 : min(j1, j2));
    return r;
}

template <int CTRL>
__device__ __forceinline__ Wta wta_dpp(const Wta &x) {
    Wta y;
    y.m = movdppf<CTRL>(x.m);
    y.s = movdppf<CTRL>(x.s);
    y.i = movdpp<CTRL>(x.i);
    y.si = movdpp<CTRL>(x.si);
    return wta_merge(x, y);
}

// LDS image of one chunk: PF pixels x D total costs, rows padded by 16 bytes
// so the consumer's per-pixel reads spread over all banks.
template <int V>
constexpr int tbuf_stride() { return 64 * V + 4; }

// The last sweep of a view, fused with the aggregation and the WTA.  Two
// waves per path: wave 0 runs the DP of direction DIR and forms
// total = S + (T + L) (SGM.cpp:386-390) for PF pixels at a time into a
// double-buffered LDS ring; wave 1 runs WTA + uniqueness + sub-pixel
// (SGM.cpp:376-418, Solver.cpp:577-593) for the previous chunk, all PF pixels
// at once: 64/PF lanes per pixel, each scanning D*PF/64 costs, merged with
// DPP.  The DP chain and the WTA then run on two SIMDs in parallel.
template <int DIR, int V, bool FULL, int PF>
__global__ __launch_bounds__(128) void sweep_final_kernel(SweepArgs a, Geom g) {
    constexpr int TS = tbuf_stride<V>();
    __shared__ __attribute__((aligned(16))) float tbuf[2][PF][TS];
    __shared__ long long pbuf[2][PF];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int path = blockIdx.x;
    const int H = g.H, W = g.W;
    const long long D = g.D, WD = (long long)g.W * g.D;
    const int n = DIR < 2 ? W : H;
    const int nchunks = (n + PF - 1) / PF;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;

    if (wave == 0) {
        Cursor<DIR> cc, pc;
        cc.init(path, H, W, g.D);
        pc.init(path, H, W, g.D);
        float cb[PF][V], ab[PF][V], sb[PF][V];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            load_v<V>(cb[u], a.cost + pc.off + e0, active);
            load_v<V>(ab[u], a.acc_in + pc.off + e0, active);
            load_v<V>(sb[u], a.s_in + pc.off + e0, active);
            if (pc.k < n - 1) pc.advance(W, D, WD);
        }
        float prev[V];
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = SGM_INF;
        float pmin = 0.0f;

        auto step = [&](int buf, int u, bool refill) {
            float L[V];
            dp_step<V>(prev, pmin, cb[u], L, a.p1, a.p2);
            const bool st = cc.start(W);
#pragma unroll
            for (int v = 0; v < V; ++v) L[v] = st ? cb[u][v] : L[v];
            float lm = L[0];
#pragma unroll
            for (int v = 1; v < V; ++v) lm = fminf(lm, L[v]);
            const float nmin = wave_min(lm);
            float tot[V];
#pragma unroll
            for (int v = 0; v < V; ++v) tot[v] = sb[u][v] + (ab[u][v] + L[v]);
            float *dst = &tbuf[buf][u][e0];
            if (V == 4) *reinterpret_cast<float4 *>(dst) = make_float4(tot[0], tot[1], tot[2], tot[3]);
            else if (V == 2) *reinterpret_cast<float2 *>(dst) = make_float2(tot[0], tot[1]);
            else dst[0] = tot[0];
            if (lane == 0) pbuf[buf][u] = (long long)cc.i * W + cc.j;
#pragma unroll
            for (int v = 0; v < V; ++v) prev[v] = L[v];
            pmin = nmin;
            cc.advance(W, D, WD);
            if (refill) {
                load_v<V>(cb[u], a.cost + pc.off + e0, active);
                load_v<V>(ab[u], a.acc_in + pc.off + e0, active);
                load_v<V>(sb[u], a.s_in + pc.off + e0, active);
                if (pc.k < n - 1) pc.advance(W, D, WD);
            }
        };
        int c = 0;
        for (; (c + 1) * PF <= n; ++c) {
#pragma unroll
            for (int u = 0; u < PF; ++u) step(c & 1, u, true);
            lds_barrier();
        }
        if (c < nchunks) {
#pragma unroll
            for (int u = 0; u < PF; ++u)
                if (c * PF + u < n) step(c & 1, u, false);
            lds_barrier();
        }
        lds_barrier();
    } else {
        constexpr int LPP = 64 / PF;        // lanes per pixel
        const int Dn = g.D;
        const int Q = Dn / LPP;             // disparities per lane (>= 8)
        const int px = lane / LPP, q = lane - px * LPP;
        const int d0 = q * Q;
        lds_barrier();
        for (int c = 0; c < nchunks; ++c) {
            const int cnt = min(PF, n - c * PF);
            const float *row = &tbuf[c & 1][px < cnt ? px : 0][0];
            // in-lane scan of d0 .. d0+Q-1 in ascending order (SGM.cpp:383-408)
            Wta w;
            w.m = SGM_INF; w.s = SGM_INF; w.i = INT_MAX; w.si = INT_MAX;
            for (int k = 0; k < Q; k += 4) {
                const float4 x4 = *reinterpret_cast<const float4 *>(row + d0 + k);
                const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = xs[e];
                    const int d = d0 + k + e;
                    if (x < w.m) {
                        w.s = w.m; w.si = w.i; w.m = x; w.i = d;
                    } else if (x != w.m && x < w.s) {
                        w.s = x; w.si = d;
                    }
                }
            }
            w = wta_dpp<DPP_QP_1032>(w);
            w = wta_dpp<DPP_QP_2301>(w);
            if (LPP == 8) w = wta_dpp<DPP_HALF_MIRROR>(w);
            int d = w.i;
            if (w.s != SGM_INF && w.m / w.s > a.uniq && abs(w.i - w.si) > 1) d = Dn + 1;
            float f;
            if (d > Dn - 1) {
                f = (float)(Dn + 1);
            } else if (d == 0 || d == Dn - 1) {
                f = (float)d;
            } else {
                const float av = row[d - 1], bv = row[d + 1], cv = row[d];
                const float x = d + (av - bv) / (2 * (av + bv - 2 * cv));
                const float lim = (Dn - 1) * 1.f;
                f = (lim < x) ? lim : x;  // std::min(x, lim)
            }
            if (q == 0 && px < cnt) {
                const long long pix = pbuf[c & 1][px];
                a.disp[pix] = (uint16_t)d;
                a.sub[pix] = f;
            }
            lds_barrier();
        }
    }
}

// Steps of loads kept in flight: horizontal paths (few, long, latency-bound)
// need a deeper ring than the W column/diagonal paths.
template <int DIR>
constexpr int sweep_pf() { return DIR < 2 ? 32 : 16; }

template <int DIR, int MODE>
static void launch_sweep_v(const SweepArgs &a, Geom g, hipStream_t st) {
    const dim3 grid(DIR < 2 ? g.H : g.W);
    constexpr int PF = sweep_pf<DIR>();
    if (MODE == SWEEP_FINAL) {
        if (g.D == 32)
            sweep_final_kernel<DIR, 1, false, 16><<<grid, 128, 0, st>>>(a, g);
        else if (g.D == 64)
            sweep_final_kernel<DIR, 1, true, 16><<<grid, 128, 0, st>>>(a, g);
        else if (g.D == 128)
            sweep_final_kernel<DIR, 2, true, 16><<<grid, 128, 0, st>>>(a, g);
        else
            sweep_final_kernel<DIR, 4, true, 8><<<grid, 128, 0, st>>>(a, g);
        return;
    }
    if (g.D == 32)
        sweep_kernel<DIR, 1, MODE, false, PF><<<grid, 64, 0, st>>>(a, g);
    else if (g.D == 64)
        sweep_kernel<DIR, 1, MODE, true, PF><<<grid, 64, 0, st>>>(a, g);
    else if (g.D == 128)
        sweep_kernel<DIR, 2, MODE, true, PF><<<grid, 64, 0, st>>>(a, g);
    else
        sweep_kernel<DIR, 4, MODE, true, PF / 2><<<grid, 64, 0, st>>>(a, g);
}

template <int MODE>
static void launch_sweep_m(int dir, const SweepArgs &a, Geom g, hipStream_t st) {
    switch (dir) {
    case 0: launch_sweep_v<0, MODE>(a, g, st); break;
    case 1: launch_sweep_v<1, MODE>(a, g, st); break;
    case 2: launch_sweep_v<2, MODE>(a, g, st); break;
    case 3: launch_sweep_v<3, MODE>(a, g, st); break;
    case 4: launch_sweep_v<4, MODE>(a, g, st); break;
    case 5: launch_sweep_v<5, MODE>(a, g, st); break;
    case 6: launch_sweep_v<6, MODE>(a, g, st); break;
    default: launch_sweep_v<7, MODE>(a, g, st); break;
    }
}

hipError_t launch_sweep(int dir, int mode, const SweepArgs &a, Geom g, hipStream_t st) {
    switch (mode) {
    case SWEEP_STORE_L: launch_sweep_m<SWEEP_STORE_L>(dir, a, g, st); break;
    case SWEEP_INIT: launch_sweep_m<SWEEP_INIT>(dir, a, g, st); break;
    case SWEEP_ACC: launch_sweep_m<SWEEP_ACC>(dir, a, g, st); break;
    default: launch_sweep_m<SWEEP_FINAL>(dir, a, g, st); break;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------- LR check

// SGM.cpp:803-818: dr = FR[i][(int)(j - dl/s)] when j >= dl; invalid if
// |dl - dr| > LR_CHECK_DIS.
__global__ __launch_bounds__(256) void lr_kernel(const float *__restrict__ fl,
                                                 const float *__restrict__ fr,
                                                 float *__restrict__ out, int out_pitch, int H,
                                                 int W, int D, int scale, float lr) {
    const int j = blockIdx.x * 256 + threadIdx.x, i = blockIdx.y;
    if (j >= W) return;
    float dl = fl[(size_t)i * W + j];
    if (j >= dl) {
        const int jr = clampi((int)(j - dl / scale), 0, W - 1);
        const float dr = fr[(size_t)i * W + jr];
        if (fabsf(dl - dr) > lr) dl = (float)(D + 1);
    }
    out[(size_t)i * out_pitch + j] = dl;
}

hipError_t launch_lr(const float *fl, const float *fr, float *out, int out_pitch, float lr,
                     Geom g, hipStream_t st) {
    lr_kernel<<<dim3((g.W + 255) / 256, g.H), 256, 0, st>>>(fl, fr, out, out_pitch, g.H, g.W, g.D,
                                                           g.scale, lr);
    return hipGetLastError();
}

}  // namespace sgm
