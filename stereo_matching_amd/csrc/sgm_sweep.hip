// sgm_sweep.hip -- single-direction path sweeps (the production L8 pass and
// the per-direction parity stages), LR check.
// CDNA4 (gfx950) kernels of the semi-global matcher.
//
// Stage map (reference -> kernel), full design in DESIGN.md:
//   cv::GaussianBlur + CT_pts     Solver.cpp:120-140, cost.cpp:99-129  -> census_kernel
//   build_dsi_from_table[_beta]   Solver.cpp:143-248
//     + cost_horizontal_filter    Solver.cpp:296-330                   -> cost_h_kernel
//   cost_vertical_filter          Solver.cpp:333-368                   -> vfwd_kernel
//   L1..L8 path DP                SGM.cpp:81-369                       -> sweep_kernel<DIR,..>
//                                                     (pairs: sgm_pair.hip)
//   aggregation + WTA + unique    SGM.cpp:372-418
//     + compute_subpixel          Solver.cpp:569-597                   -> pair_final_kernel
//   LR check                      SGM.cpp:803-818                      -> lr_kernel
//
// Bit-exactness rules (DESIGN.md "Numerics"): built with -ffp-contract=off,
// no fast-math, correctly rounded f32 division; every float expression keeps
// the reference's association order.
#include <cstdlib>

#include "sgm_bodies.h"

namespace sgm {

template <int DIR, int V, int MODE, bool FULL, int PF, bool BAND = false>
__global__ __launch_bounds__(64) void sweep_kernel(SweepArgs a, Geom g) {
    sweep_body<DIR, V, MODE, FULL, PF, BAND>(a, g, bid_x());
}

// The same sweep over both views' volumes (workgroup y = view): the L8 pass
// of frames whose two cost volumes fit the Infinity Cache together (K64).
template <int DIR, int V, int MODE, bool FULL, int PF>
__global__ __launch_bounds__(64) void sweep2_kernel(SweepArgs a0, SweepArgs a1, Geom g) {
    sweep_body<DIR, V, MODE, FULL, PF>(__builtin_amdgcn_workgroup_id_y() != 0 ? a1 : a0, g, bid_x());
}

hipError_t launch_sweep2_l8(const SweepArgs &a0, const SweepArgs &a1, Geom g, hipStream_t st) {
    const dim3 grid(g.W, 2);
    constexpr int PF = 16;
    if (g.D == 32) sweep2_kernel<7, 1, SWEEP_ACC, false, PF><<<grid, 64, 0, st>>>(a0, a1, g);
    else if (g.D == 64) sweep2_kernel<7, 1, SWEEP_ACC, true, PF><<<grid, 64, 0, st>>>(a0, a1, g);
    else if (g.D == 128) sweep2_kernel<7, 2, SWEEP_ACC, true, PF><<<grid, 64, 0, st>>>(a0, a1, g);
    else sweep2_kernel<7, 4, SWEEP_ACC, true, PF / 2><<<grid, 64, 0, st>>>(a0, a1, g);
    return hipGetLastError();
}

// Diagonal INIT/ACC sweeps (the L8 pass): memory wave + DP wave
// (sweep_split_body), blocks of 4 steps.
template <int DIR, int V, int MODE, bool FULL>
__global__ __launch_bounds__(128) void sweep_split_kernel(SweepArgs a, Geom g) {
    __shared__ __attribute__((aligned(16))) SweepSplitLds<V, 4> lds;
    sweep_split_body<DIR, V, MODE, FULL, 4>(a, g, bid_x(), lds);
}

// The split sweep pays where the pass streams from HBM (a cost volume larger
// than the 256 MB Infinity Cache: HD256 L8 1224 -> 1118 us); on a volume the
// cache holds it is slower (K128 L8 114 -> 122 us).  SGM_SWEEP_SPLIT=0/1
// forces it off/on (tests use it to cover both bodies at every size).
static bool use_split_sweep(const Geom &g) {
    const char *e = std::getenv("SGM_SWEEP_SPLIT");
    if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
    return (size_t)g.H * g.W * g.D * sizeof(float) > (size_t(256) << 20);
}

// Steps of loads kept in flight: horizontal paths (few, long, latency-bound)
// need a deeper ring than the W column/diagonal paths.
template <int DIR>
constexpr int sweep_pf() { return DIR < 2 ? 32 : 16; }

template <int DIR, int MODE>
static void launch_sweep_v(const SweepArgs &a, Geom g, hipStream_t st) {
    const dim3 grid(DIR < 2 ? g.H : g.W);
    if constexpr (DIR >= 4 && MODE != SWEEP_STORE_L) {
        if (a.band.ke == 0 && use_split_sweep(g)) {  // (bands: the one-wave body, below)
            if (g.D == 32)
                sweep_split_kernel<DIR, 1, MODE, false><<<grid, 128, 0, st>>>(a, g);
            else if (g.D == 64)
                sweep_split_kernel<DIR, 1, MODE, true><<<grid, 128, 0, st>>>(a, g);
            else if (g.D == 128)
                sweep_split_kernel<DIR, 2, MODE, true><<<grid, 128, 0, st>>>(a, g);
            else
                sweep_split_kernel<DIR, 4, MODE, true><<<grid, 128, 0, st>>>(a, g);
            return;
        }
    }
    constexpr int PF = sweep_pf<DIR>();
    if constexpr (DIR >= 4 && MODE != SWEEP_STORE_L) {
        if (a.band.ke > 0) {  // one band (L7/L8: backward bands; L5/L6: forward bands)
            if (g.D == 32)
                sweep_kernel<DIR, 1, MODE, false, PF, true><<<grid, 64, 0, st>>>(a, g);
            else if (g.D == 64)
                sweep_kernel<DIR, 1, MODE, true, PF, true><<<grid, 64, 0, st>>>(a, g);
            else if (g.D == 128)
                sweep_kernel<DIR, 2, MODE, true, PF, true><<<grid, 64, 0, st>>>(a, g);
            else
                sweep_kernel<DIR, 4, MODE, true, PF / 2, true><<<grid, 64, 0, st>>>(a, g);
            return;
        }
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
    default: return hipErrorInvalidValue;  // the final pass is pair_final_kernel
    }
    return hipGetLastError();
}

// ------------------------------------------------------------- LR check

// SGM.cpp:803-818: dr = FR[i][(int)(j - dl/s)] when j >= dl; invalid if
// |dl - dr| > LR_CHECK_DIS.  Pitches in floats; out may alias fl.  The column
// is clamped to the row before the int conversion (as oracle/sgm_oracle.c's
// orc_lr_check): a no-op for every map compute_subpixel produces (dl >= 0 or
// NaN, so 0 <= j - dl/s <= j; DESIGN.md "LR check domain"); for arbitrary maps
// passed to sgm_lr_check_device the reference would read another row.
__global__ __launch_bounds__(256) void lr_kernel(const float *fl, int fl_pitch,
                                                 const float *__restrict__ fr, int fr_pitch,
                                                 float *out, int out_pitch, int H, int W, int D,
                                                 int scale, float lr) {
    const int j = bid_x() * 256 + tid_x(), i = bid_y();
    if (j >= W) return;
    float dl = fl[(size_t)i * fl_pitch + j];
    // j >= NaN is false (IEEE); tested on the bits: the library builds with
    // -fno-honor-nans, under which the compiler may assume dl is not NaN
    const bool nan = (__float_as_uint(dl) & 0x7fffffffu) > 0x7f800000u;
    if (!nan && j >= dl) {
        const float x = j - dl / scale;
        const int jr = x < 0.f ? 0 : (x > (float)(W - 1) ? W - 1 : (int)x);
        const float dr = fr[(size_t)i * fr_pitch + jr];
        if (fabsf(dl - dr) > lr) dl = (float)(D + 1);
    }
    out[(size_t)i * out_pitch + j] = dl;
}

hipError_t launch_lr(const float *fl, int fl_pitch, const float *fr, int fr_pitch, float *out,
                     int out_pitch, float lr, Geom g, hipStream_t st) {
    lr_kernel<<<dim3((g.W + 255) / 256, g.H), 256, 0, st>>>(fl, fl_pitch, fr, fr_pitch, out,
                                                           out_pitch, g.H, g.W, g.D, g.scale, lr);
    return hipGetLastError();
}

// The LR check of a two-view frame on the final passes' COLUMN-major maps
// (x[col * H + row]: whole cache lines per column chunk for the final pass's
// one-column workgroups) with a row-major output.  A workgroup takes 64
// columns x 32 rows: its fl tile is staged through LDS with 128-byte column
// reads (a transpose), then each wave checks rows of 64 consecutive pixels
// exactly as lr_kernel does, gathering fr(i, jr) straight from the column-
// major map: a row's 64 reads touch ~64 columns, the same lines for all 32
// rows of the tile, so after the first row they hit the L1/L2.
constexpr int LRT_J = 64, LRT_I = 32;

__global__ __launch_bounds__(256) void lr_cm_kernel(const float *__restrict__ fl,
                                                    const float *__restrict__ fr,
                                                    float *__restrict__ out, int out_pitch, int H,
                                                    int W, int D, int scale, float lr) {
    __shared__ float fls[LRT_J][LRT_I + 1];
    const int j0 = bid_x() * LRT_J, i0 = bid_y() * LRT_I;
    const int t = tid_x();
#pragma unroll
    for (int k = 0; k < LRT_J * LRT_I / 256; ++k) {
        const int idx = t + k * 256, c = idx / LRT_I, ii = idx - c * LRT_I, j = j0 + c, i = i0 + ii;
        fls[c][ii] = (j < W && i < H) ? fl[(size_t)j * H + i] : 0.f;
    }
    __syncthreads();
    const int jj = t & (LRT_J - 1), j = j0 + jj;
    if (j >= W) return;
#pragma unroll
    for (int k = 0; k < LRT_I / 4; ++k) {
        const int ii = (t >> 6) + 4 * k, i = i0 + ii;
        if (i >= H) break;
        float dl = fls[jj][ii];
        const bool nan = (__float_as_uint(dl) & 0x7fffffffu) > 0x7f800000u;
        if (!nan && j >= dl) {
            const float x = j - dl / scale;
            const int jr = x < 0.f ? 0 : (x > (float)(W - 1) ? W - 1 : (int)x);
            const float dr = fr[(size_t)jr * H + i];
            if (fabsf(dl - dr) > lr) dl = (float)(D + 1);
        }
        out[(size_t)i * out_pitch + j] = dl;
    }
}

hipError_t launch_lr_cm(const float *fl_cm, const float *fr_cm, float *out, int out_pitch, float lr,
                        Geom g, hipStream_t st) {
    lr_cm_kernel<<<dim3((g.W + LRT_J - 1) / LRT_J, (g.H + LRT_I - 1) / LRT_I), 256, 0, st>>>(
        fl_cm, fr_cm, out, out_pitch, g.H, g.W, g.D, g.scale, lr);
    return hipGetLastError();
}

}  // namespace sgm

#ifdef SGM_STAMPS
extern "C" int sgm_debug_stamps_sweep(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sgm::sgm_stamps), sizeof(sgm::sgm_stamps)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[16][3] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sgm::sgm_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
