// sgm_cost.hip -- census, DSI + horizontal IIR (the vertical IIR runs fused
// with the L3 forward pass in sgm_pair.hip).
// CDNA4 (gfx950) kernels of the semi-global matcher.
//
// Stage map (reference -> kernel), full design in DESIGN.md:
//   cv::GaussianBlur + CT_pts     Solver.cpp:120-140, cost.cpp:99-129  -> census_kernel
//   build_dsi_from_table[_beta]   Solver.cpp:143-248
//     + cost_horizontal_filter    Solver.cpp:296-330                   -> cost_h_kernel,
//                                                                         cost_h2_kernel (both views)
//   cost_vertical_filter          Solver.cpp:333-368                   -> vfwd_kernel (sgm_pair.hip)
//   L1..L8 path DP                SGM.cpp:81-369                       -> stage_a/stage_b kernels,
//                                                                         sweep_kernel (sgm_sweep.hip)
//   aggregation + WTA + unique    SGM.cpp:372-418
//     + compute_subpixel          Solver.cpp:569-597                   -> pair_final_kernel
//   LR check                      SGM.cpp:803-818                      -> lr_kernel
//
// Bit-exactness rules (DESIGN.md "Numerics"): built with -ffp-contract=off,
// no fast-math, correctly rounded f32 division; every float expression keeps
// the reference's association order.
#include "sgm_device.h"

namespace sgm {

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

// Census inputs: rpitch = bytes between working-grid rows (step * pitch for
// SGM.cpp:47-48's decimation, pitch for BM.cpp:24-25's); step = pixels
// between columns.
constexpr int CT_TW = 64, CT_TH = 16, CT_RPT = CT_TH / 4;  // 4 waves x CT_RPT rows

// CT_pts (cost.cpp:99-129) for one image; window (2HH+1) x (2HWW+1) = 7x9 (3x5
// at scale 2), MSB first, centre skipped, coordinates clamped to the
// (working-grid) edge.  A workgroup owns a 64 x 16 pixel tile:
//   1. the raw pixels the blur of the tile + census apron needs are loaded
//      once (rows/columns lo-1 .. hi+1 at BORDER_REFLECT_101 coordinates);
//   2. the blurred window is built in LDS at clamped coordinates from them;
//   3. each lane walks CT_RPT consecutive rows of its column: every window
//      row is read once and feeds the census words of all the rows whose
//      window holds it (bits appended in row-major order, as the reference).
// Both images in one launch: workgroup z selects (src0, ct0) or (src1, ct1).
template <int HH, int HWW>
__global__ __launch_bounds__(256) void census_kernel(const uint8_t *__restrict__ src0,
                                                     const uint8_t *__restrict__ src1, int rpitch,
                                                     int step, int H, int W, int blur,
                                                     uint64_t *__restrict__ ct0,
                                                     uint64_t *__restrict__ ct1) {
    const bool second = __builtin_amdgcn_workgroup_id_z() != 0;
    const uint8_t *__restrict__ src = second ? src1 : src0;
    uint64_t *__restrict__ ct = second ? ct1 : ct0;
    constexpr int TR = CT_TH + 2 * HH, TC = CT_TW + 2 * HWW;
    constexpr int RR = TR + 2, RC = TC + 2;       // raw staging bound
    constexpr int RAW_IT = (RR * RC + 255) / 256;
    __shared__ uint8_t tile[TR][TC];
    __shared__ uint8_t raw[RR][RC];
    const int x0 = bid_x() * CT_TW, y0 = bid_y() * CT_TH;
    const int t = tid_x();
    if (blur) {
        // real rows/columns the clamped window touches, and the raw pixels
        // (one further, reflected) their 3x3 blur reads
        const int ylo = y0 - HH > 0 ? y0 - HH : 0, xlo = x0 - HWW > 0 ? x0 - HWW : 0;
        uint8_t v[RAW_IT];
#pragma unroll
        for (int u = 0; u < RAW_IT; ++u) {
            const int idx = u * 256 + t;
            const int ry = idx / RC, rx = idx - ry * RC;
            const int y = reflect101(clampi(ylo - 1 + ry, -1, H), H);
            const int x = reflect101(clampi(xlo - 1 + rx, -1, W), W);
            v[u] = idx < RR * RC ? src[(size_t)y * rpitch + (size_t)x * step] : 0;
        }
#pragma unroll
        for (int u = 0; u < RAW_IT; ++u) {
            const int idx = u * 256 + t;
            if (idx < RR * RC) (&raw[0][0])[idx] = v[u];
        }
        __syncthreads();
        for (int idx = t; idx < TR * TC; idx += 256) {
            const int ty = idx / TC, tx = idx - ty * TC;
            const int ry = clampi(y0 + ty - HH, 0, H - 1) - ylo;
            const int rx = clampi(x0 + tx - HWW, 0, W - 1) - xlo;
            constexpr int ky[3] = {70, 116, 70};
            int acc = 0;
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const uint8_t *row = &raw[ry + r][rx];
                acc += ky[r] * (82 * row[0] + 93 * row[1] + 82 * row[2]);
            }
            const int b = (acc + (1 << 15)) >> 16;  // the pinned blur (top of file)
            tile[ty][tx] = (uint8_t)(b > 255 ? 255 : b);
        }
    } else {
        for (int idx = t; idx < TR * TC; idx += 256) {
            const int ty = idx / TC, tx = idx - ty * TC;
            const int y = clampi(y0 + ty - HH, 0, H - 1), x = clampi(x0 + tx - HWW, 0, W - 1);
            tile[ty][tx] = src[(size_t)y * rpitch + (size_t)x * step];
        }
    }
    __syncthreads();
    const int tx = t & 63, r0 = wave_id() * CT_RPT;
    constexpr int NB = (2 * HH + 1) * (2 * HWW + 1) - 1;  // census bits (62 at 7x9)
    static_assert(NB <= 64, "census word");
    constexpr int NHI = NB > 32 ? NB - 32 : 0;            // bits in the high word
    int c[CT_RPT];
#pragma unroll
    for (int p = 0; p < CT_RPT; ++p) c[p] = tile[r0 + p + HH][tx + HWW];
    unsigned hi[CT_RPT], lo[CT_RPT];
#pragma unroll
    for (int p = 0; p < CT_RPT; ++p) hi[p] = lo[p] = 0;
    // window row rr (tile row r0 + rr) is row di = rr - HH - p of pixel p
#pragma unroll
    for (int rr = 0; rr < CT_RPT + 2 * HH; ++rr) {
        int b[2 * HWW + 1];
#pragma unroll
        for (int dj = 0; dj <= 2 * HWW; ++dj) b[dj] = tile[r0 + rr][tx + dj];
#pragma unroll
        for (int p = 0; p < CT_RPT; ++p) {
            const int di = rr - p;  // 0 .. 2HH within the window
            if (di < 0 || di > 2 * HH) continue;
#pragma unroll
            for (int dj = 0; dj <= 2 * HWW; ++dj) {
                if (di == HH && dj == HWW) continue;
                // bit position k (0 = first, MSB) of the reference's order
                const int k = di * (2 * HWW + 1) + dj - (di * (2 * HWW + 1) + dj > HH * (2 * HWW + 1) + HWW ? 1 : 0);
                // (c - b) has its sign bit set iff b > c (bytes, no overflow):
                // w << 1 | x >> 31 is one funnel shift (v_alignbit_b32)
                const unsigned x = (unsigned)(c[p] - b[dj]);
                if (k < NHI) hi[p] = (hi[p] << 1) | (x >> 31);
                else lo[p] = (lo[p] << 1) | (x >> 31);
            }
        }
    }
    const int x = x0 + tx;
#pragma unroll
    for (int p = 0; p < CT_RPT; ++p) {
        const int y = y0 + r0 + p;
        if (y < H && x < W) ct[(size_t)y * W + x] = ((uint64_t)hi[p] << 32) | lo[p];
    }
}

hipError_t launch_census(const uint8_t *src, int pitch, Geom g, int blur, uint64_t *ct,
                         hipStream_t st, bool bm_rows, const uint8_t *src2, uint64_t *ct2) {
    dim3 grid((g.W + CT_TW - 1) / CT_TW, (g.H + CT_TH - 1) / CT_TH, src2 ? 2 : 1);
    const int rpitch = bm_rows ? pitch : pitch * g.scale;
    if (g.scale == 1)
        census_kernel<3, 4><<<grid, 256, 0, st>>>(src, src2, rpitch, 1, g.H, g.W, blur, ct, ct2);
    else
        census_kernel<1, 2><<<grid, 256, 0, st>>>(src, src2, rpitch, 2, g.H, g.W, blur, ct, ct2);
    return hipGetLastError();
}

// ------------------------------------------------ DSI + horizontal IIR

// One thread per (row, d) chain, R rows per block (R*D threads).  The census
// rows of both images (and the sky row) are staged in LDS once per block,
// padded on both sides with copies of the edge words so the clamped lookups
// of Solver.cpp:143-248 become plain offsets; the raw Hamming DSI (sky
// override :165-178) is produced on the fly and fed straight into the
// in-place horizontal IIR of Solver.cpp:296-330, restated with a register
// history: with h = WIN/2 and LAG = WIN-h-1 the reference writes position
// LAG+t at step t, adds raw[WIN+t] and subtracts the value at position t,
// which is the step-(t-LAG) output once t >= LAG and raw before.
//
// The IIR is one serial chain per (row, d) and a frame has only H*D of them
// (750 waves at KITTI D=128), so a wave's step latency is the kernel time:
// the main loop runs blocks of COSTH_U steps with no branches, their raw
// costs fetched one block ahead.
constexpr int COSTH_MAX_LDS = 64 * 1024;

// The horizontally filtered volume is read once, by vfwd: non-temporal stores
// keep it from evicting the final cost C from the Infinity Cache (default-
// policy stores: cost_h 58 -> 50 us but vfwd and stage A slower, r02 and
// profiles/r03_experiments/inplace_c.txt).
__device__ __forceinline__ void costh_store(float v, float *p) { __builtin_nontemporal_store(v, p); }
constexpr int COSTH_U = 8;

__host__ __device__ constexpr int costh_pad(int D, int scale) { return D / scale + 2 * COSTH_U; }

// UNI (D >= 64, one row per wave): the census word every lane of a row needs
// at step j -- cl[j] for the left view, cr[j] for the right -- is a uniform
// scalar load from global memory; only the per-lane shifted row is staged in
// LDS, which halves the staging and keeps 4K rows (3840 px) inside 64 KiB.
// DC: D as a compile-time constant (0: runtime D), so the stores of an
// unrolled block take immediate offsets instead of a 64-bit address add each
// CK > 0 (the strip schedule's checkpoint pass, sgm_vstrip.hip): no volume
// is written; at every output position p = CK * s (2 <= p <= W-3) the state
// before the step that produces p -- the running sum and the values at
// positions p-2, p-1 it will subtract -- goes to out[((i * ck_ns + s) * 3 +
// k) * D + d], k = 0 .. 2.
template <int VIEW, int WIN, bool SKY, bool FILTER, bool UNI, int DC = 0, int CK = 0>
__device__ __forceinline__ void cost_h_body(const uint64_t *__restrict__ ctl,
                                            const uint64_t *__restrict__ ctr,
                                            const uint8_t *__restrict__ sky, int sky_pitch, int H,
                                            int W, int D, int scale, int R,
                                            float *__restrict__ out, int blk, unsigned char *smem,
                                            int ck_ns = 0) {
    static_assert(CK == 0 || (WIN == 5 && FILTER), "checkpoints of the 5-wide filter");
    const int P = costh_pad(D, scale), RS = W + 2 * P;
    constexpr int NS = UNI ? 1 : 2;  // staged census rows per image row
    uint64_t *sl = reinterpret_cast<uint64_t *>(smem);
    uint64_t *sr = sl + (UNI ? 0 : (size_t)R * RS);
    uint8_t *ss = reinterpret_cast<uint8_t *>(sl + (size_t)NS * R * RS);
    const int row0 = blk * R;
    for (int idx = tid_x(); idx < R * RS; idx += R * D) {
        const int r = idx / RS, jp = idx - r * RS, i = row0 + r;
        const int j = clampi(jp - P, 0, W - 1);
        if (i < H) {
            if (!UNI || VIEW == 1) sl[idx] = ctl[(size_t)i * W + j];
            if (!UNI || VIEW == 0) sr[idx] = ctr[(size_t)i * W + j];
            if (SKY) ss[idx] = sky[(size_t)i * sky_pitch + j];
        }
    }
    __syncthreads();
    const int r = UNI ? uniform(tid_x() / D) : tid_x() / D, d = tid_x() - r * D;
    const int i = row0 + r;
    if (i >= H) return;
    const int ds = d / scale;
    // raw(j) reads cl[j (+ds)] and cr[j (-ds)] through the padded rows
    const uint64_t *cl = sl + (size_t)r * RS + P + (VIEW == 1 ? ds : 0);
    const uint64_t *cr = sr + (size_t)r * RS + P - (VIEW == 0 ? ds : 0);
    const uint64_t *cu = (VIEW == 0 ? ctl : ctr) + (size_t)i * W;  // UNI: the uniform row
    const uint8_t *sk = ss + (size_t)r * RS + P;
    float *o = out + (CK ? (size_t)i * ck_ns * 3 * D : (size_t)i * W * D) + d;
    const size_t DS = DC ? (size_t)DC : (size_t)D;  // store stride

    auto word_l = [&](int j) { return UNI && VIEW == 0 ? cu[j < W - 1 ? j : W - 1] : cl[j]; };
    auto word_r = [&](int j) { return UNI && VIEW == 1 ? cu[j < W - 1 ? j : W - 1] : cr[j]; };

    auto raw = [&](int j) -> float {
        const float c = hamming(word_l(j), word_r(j));
        if (SKY) {
            const float sv = d == 0 ? 0.0f : 999999.0f;
            return sk[j] == 255 ? sv : c;
        }
        return c;
    };

    if (!FILTER) {
        for (int j = 0; j < W; ++j) costh_store(raw(j), o + (size_t)j * DS);
        return;
    }
    constexpr int HALF = WIN / 2, LAG = WIN - HALF - 1, U = COSTH_U;
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < WIN; ++k) sum += raw(k);
    if constexpr (CK == 0) {
#pragma unroll
        for (int p = 0; p < LAG; ++p) costh_store(raw(p), o + (size_t)p * DS);
    }
    const int T = W - 2 * HALF;
    // hist[0] is what step t subtracts: raw[t] for t < LAG, output t-LAG after
    float hist[LAG > 0 ? LAG : 1];
#pragma unroll
    for (int p = 0; p < LAG; ++p) hist[p] = raw(p);
    auto ck_store = [&](int p) {
        if constexpr (CK > 0) {
            if (p % CK == 0) {
                float *q = o + (size_t)(p / CK) * 3 * DS;
                q[0] = sum;
                q[DS] = hist[0];
                q[2 * DS] = hist[LAG - 1];
            }
        }
    };
    auto step = [&](int t, float rw) {
        ck_store(LAG + t);
        const float v = div_win<WIN>(sum);
        if constexpr (CK == 0) costh_store(v, o + (size_t)(LAG + t) * DS);
        sum += rw;
        float a;
        if constexpr (LAG == 0) {
            a = v;
        } else {
            a = hist[0];
#pragma unroll
            for (int p = 0; p + 1 < LAG; ++p) hist[p] = hist[p + 1];
            hist[LAG - 1] = v;
        }
        sum -= a;
    };
    // steps t < T-1 also add raw[WIN+t]; the last step only writes.  The
    // next block's census words (and sky bytes) are loaded before the current
    // block's steps run and only turned into costs after them, so the LDS
    // round trips overlap the serial chain.
    int t = 0;
    float cur[U];
    if (T - 1 >= U) {
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = raw(WIN + u);
    }
    for (; t + 2 * U <= T - 1; t += U) {
        uint64_t nl[U], nr[U];
        uint8_t nk[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = WIN + t + U + u;
            nl[u] = word_l(j);
            nr[u] = word_r(j);
            if (SKY) nk[u] = sk[j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) step(t + u, cur[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float c = hamming(nl[u], nr[u]);
            if (SKY) cur[u] = nk[u] == 255 ? (d == 0 ? 0.0f : 999999.0f) : c;
            else cur[u] = c;
        }
    }
    if (t + U <= T - 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) step(t + u, cur[u]);
        t += U;
    }
    for (; t < T - 1; ++t) step(t, raw(WIN + t));
    if constexpr (CK > 0) {
        if (T >= 1) ck_store(LAG + T - 1);
        return;
    }
    if (T >= 1) costh_store(div_win<WIN>(sum), o + (size_t)(LAG + T - 1) * DS);
    for (int p = LAG + T; p < W; ++p) costh_store(raw(p), o + (size_t)p * DS);
}

template <int VIEW, int WIN, bool SKY, bool FILTER, bool UNI, int DC>
__global__ __launch_bounds__(256) void cost_h_kernel(const uint64_t *__restrict__ ctl,
                                                     const uint64_t *__restrict__ ctr,
                                                     const uint8_t *__restrict__ sky,
                                                     int sky_pitch, int H, int W, int D, int scale,
                                                     int R, float *__restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cost_h_body<VIEW, WIN, SKY, FILTER, UNI, DC>(ctl, ctr, sky, sky_pitch, H, W, D, scale, R, out,
                                             bid_x(), smem);
}

// Both views in one launch (workgroup z = view): the DSI of
// build_dsi_from_table into out0 and of build_dsi_from_table_beta into out1,
// each with its own sky mask.  A view's H*D chains fill less than the chip at
// KITTI sizes, so the two views' chains run side by side.
template <int WIN, bool SKY, bool FILTER, bool UNI, int DC>
__global__ __launch_bounds__(256) void cost_h2_kernel(const uint64_t *__restrict__ ctl,
                                                      const uint64_t *__restrict__ ctr,
                                                      const uint8_t *__restrict__ sky0,
                                                      const uint8_t *__restrict__ sky1,
                                                      int sky_pitch, int H, int W, int D, int scale,
                                                      int R, float *__restrict__ out0,
                                                      float *__restrict__ out1) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if (__builtin_amdgcn_workgroup_id_z() == 0)
        cost_h_body<0, WIN, SKY, FILTER, UNI, DC>(ctl, ctr, sky0, sky_pitch, H, W, D, scale, R, out0,
                                              bid_x(), smem);
    else
        cost_h_body<1, WIN, SKY, FILTER, UNI, DC>(ctl, ctr, sky1, sky_pitch, H, W, D, scale, R, out1,
                                              bid_x(), smem);
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
    const int r = tid_x() / D, d = tid_x() - r * D;
    const int i = bid_x() * rows_per_block + r;
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
        return hamming(a, b);
    };
    if (!FILTER) {
        for (int j = 0; j < W; ++j) costh_store(raw(j), o + (size_t)j * D);
        return;
    }
    constexpr int HALF = WIN / 2, LAG = WIN - HALF - 1;
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < WIN; ++k) sum += raw(k);
#pragma unroll
    for (int p = 0; p < LAG; ++p) costh_store(raw(p), o + (size_t)p * D);
    const int T = W - 2 * HALF;
    float o1 = 0.0f, o2 = 0.0f;
    for (int t = 0; t < T; ++t) {
        const float v = div_win<WIN>(sum);
        costh_store(v, o + (size_t)(LAG + t) * D);
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
    for (int p = LAG + T; p < W; ++p) costh_store(raw(p), o + (size_t)p * D);
}

// rows per block and LDS bytes of the staged cost_h_kernel (R = 0: the
// global-memory fallback)
static void costh_shape(Geom g, bool sky, bool &uni, int &R, size_t &smem) {
    const size_t rs = (size_t)(g.W + 2 * costh_pad(g.D, g.scale));
    uni = g.D >= 64 && rs * (16 + (sky ? 1 : 0)) > (size_t)COSTH_MAX_LDS;
    const size_t row_bytes = rs * ((uni ? 8 : 16) + (sky ? 1 : 0));
    R = (int)(COSTH_MAX_LDS / row_bytes);
    if (R > 256 / g.D) R = 256 / g.D;
    smem = (size_t)(R > 0 ? R : 0) * row_bytes;
}

template <int VIEW, int WIN, bool SKY, bool FILTER>
static void launch_cost_h_t(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
                            int sky_pitch, Geom g, float *out, hipStream_t st) {
    // stage both census rows when they fit (faster: LDS reads for both
    // operands); rows too wide for that (4K) stage one and load the uniform
    // operand as scalars
    bool uni;
    int R;
    size_t smem;
    costh_shape(g, SKY, uni, R, smem);
    if (R >= 1) {
        if (uni)
            cost_h_kernel<VIEW, WIN, SKY, FILTER, true, 0><<<dim3((g.H + R - 1) / R), R * g.D, smem, st>>>(
                ctl, ctr, sky, sky_pitch, g.H, g.W, g.D, g.scale, R, out);
        else if (g.D == 128)
            cost_h_kernel<VIEW, WIN, SKY, FILTER, false, 128><<<dim3((g.H + R - 1) / R), R * g.D, smem, st>>>(
                ctl, ctr, sky, sky_pitch, g.H, g.W, g.D, g.scale, R, out);
        else
            cost_h_kernel<VIEW, WIN, SKY, FILTER, false, 0><<<dim3((g.H + R - 1) / R), R * g.D, smem, st>>>(
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

template <int WIN, bool SKY, bool FILTER>
static hipError_t launch_cost_h2_t(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky0,
                                   const uint8_t *sky1, int sky_pitch, Geom g, float *out0,
                                   float *out1, hipStream_t st) {
    bool uni;
    int R;
    size_t smem;
    costh_shape(g, SKY, uni, R, smem);
    if (R < 1) return hipErrorInvalidValue;  // the caller launches the views one by one
    const dim3 grid((g.H + R - 1) / R, 1, 2);
    if (uni)
        cost_h2_kernel<WIN, SKY, FILTER, true, 0><<<grid, R * g.D, smem, st>>>(
            ctl, ctr, sky0, sky1, sky_pitch, g.H, g.W, g.D, g.scale, R, out0, out1);
    else if (g.D == 128)
        cost_h2_kernel<WIN, SKY, FILTER, false, 128><<<grid, R * g.D, smem, st>>>(
            ctl, ctr, sky0, sky1, sky_pitch, g.H, g.W, g.D, g.scale, R, out0, out1);
    else
        cost_h2_kernel<WIN, SKY, FILTER, false, 0><<<grid, R * g.D, smem, st>>>(
            ctl, ctr, sky0, sky1, sky_pitch, g.H, g.W, g.D, g.scale, R, out0, out1);
    return hipGetLastError();
}

bool cost_h2_supported(Geom g, bool sky) {
    bool uni;
    int R;
    size_t smem;
    costh_shape(g, sky, uni, R, smem);
    return R >= 1;
}

hipError_t launch_cost_h2(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky0,
                          const uint8_t *sky1, int sky_pitch, Geom g, float *out0, float *out1,
                          hipStream_t st) {
    if ((sky0 == nullptr) != (sky1 == nullptr)) return hipErrorInvalidValue;
    if (sky0) {
        if (g.scale == 1) return launch_cost_h2_t<5, true, true>(ctl, ctr, sky0, sky1, sky_pitch, g, out0, out1, st);
        return launch_cost_h2_t<2, true, true>(ctl, ctr, sky0, sky1, sky_pitch, g, out0, out1, st);
    }
    if (g.scale == 1) return launch_cost_h2_t<5, false, true>(ctl, ctr, sky0, sky1, sky_pitch, g, out0, out1, st);
    return launch_cost_h2_t<2, false, true>(ctl, ctr, sky0, sky1, sky_pitch, g, out0, out1, st);
}

// The checkpoint pass's chain (sgm_vstrip.hip): cost_h_body's horizontal IIR
// (WIN = 5, no sky mask), storing only the state at every strip edge.  Its
// bytes are negligible, so the chains' latency is its time: the steps run in
// blocks of one strip (U = kVStripNC) that start at an edge, so the
// checkpoint is the block's first action (no branch), and the next block's
// census words are loaded one block ahead -- the uniform row (UNI) by vector
// loads from an opaque per-lane address: SMEM returns out of order, so its
// waits are lgkmcnt(0), which hipcc placed right before each block.
template <int VIEW, bool UNI>
__device__ __forceinline__ void cost_ck_body(const uint64_t *__restrict__ ctl,
                                             const uint64_t *__restrict__ ctr, int H, int W, int D,
                                             int R, float *__restrict__ out, int blk,
                                             unsigned char *smem, int ns) {
    constexpr int U = kVStripNC;
    const int P = costh_pad(D, 1), RS = W + 2 * P;
    constexpr int NS = UNI ? 1 : 2;
    uint64_t *sl = reinterpret_cast<uint64_t *>(smem);
    uint64_t *sr = sl + (UNI ? 0 : (size_t)R * RS);
    const int row0 = blk * R;
    for (int idx = tid_x(); idx < R * RS; idx += R * D) {
        const int r = idx / RS, jp = idx - r * RS, i = row0 + r;
        const int j = clampi(jp - P, 0, W - 1);
        if (i < H) {
            if (!UNI || VIEW == 1) sl[idx] = ctl[(size_t)i * W + j];
            if (!UNI || VIEW == 0) sr[idx] = ctr[(size_t)i * W + j];
        }
    }
    (void)NS;
    __syncthreads();
    const int r = UNI ? uniform(tid_x() / D) : tid_x() / D, d = tid_x() - r * D;
    const int i = row0 + r;
    if (i >= H) return;
    const uint64_t *cl = sl + (size_t)r * RS + P + (VIEW == 1 ? d : 0);
    const uint64_t *cr = sr + (size_t)r * RS + P - (VIEW == 0 ? d : 0);
    const uint64_t *cu = (VIEW == 0 ? ctl : ctr) + (size_t)i * W;
#ifdef COSTCK_VLOAD
    if constexpr (UNI) {
        int z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        cu += z;
    }
#endif
    float *o = out + (size_t)i * ns * 3 * D + d;
    // the shifted operand (LDS) and the other one (UNI: global) of position
    // j <= W-1 (positions past the row are clamped; their costs feed nothing)
    auto wu = [&](int j) { return UNI ? cu[j] : (VIEW == 0 ? cl[j] : cr[j]); };
    auto ws = [&](int j) { return VIEW == 0 ? cr[j] : cl[j]; };
    auto raw = [&](int j) {
        j = min(j, W - 1);
        return VIEW == 0 ? hamming(wu(j), ws(j)) : hamming(ws(j), wu(j));
    };
    float sum = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) sum += raw(k);
    float h0 = raw(0), h1 = raw(1);
    const int T = W - 4;  // steps: output position t+2; steps t < T-1 update
    auto step = [&](float rw) {
        const float v = div_win<5>(sum);
        sum += rw;
        sum -= h0;
        h0 = h1;
        h1 = v;
    };
    auto ck_store = [&](int s) {
        float *q = o + (size_t)s * 3 * D;
        q[0] = sum;
        q[D] = h0;
        q[2 * D] = h1;
    };
    // a step with its conditions (the prologue and the tail): the checkpoint
    // of the strip starting at position t+2, then the update
    auto gstep = [&](int t) {
        if ((t + 2) % U == 0) ck_store((t + 2) / U);
        if (t < T - 1) step(raw(t + 5));
    };
    int t = 0;
    for (; t < U - 2 && t < T; ++t) gstep(t);
    // full blocks b (steps U*b-2 .. U*b+U-3, all updating): U*(b+1) - 2 < T
    int b = 1;
    if (U * (b + 1) - 2 < T) {
        float cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = raw(U * b + 3 + u);
        for (; U * (b + 1) - 2 < T; ++b) {
            uint64_t nu[U], nw[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = min(U * (b + 1) + 3 + u, W - 1);
                nu[u] = wu(j);
                nw[u] = ws(j);
            }
            // (scheduling fences: else hipcc pulls each word's hamming up next
            // to its load and waits for it inside the chain)
            __builtin_amdgcn_sched_barrier(0);
            ck_store(b);
#pragma unroll
            for (int u = 0; u < U; ++u) step(cur[u]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = VIEW == 0 ? hamming(nu[u], nw[u]) : hamming(nw[u], nu[u]);
        }
        t = U * b - 2;
    }
    for (; t < T; ++t) gstep(t);
}

// The strip schedule's checkpoint pass (sgm_vstrip.hip): each view slot's
// horizontal IIR state at every strip edge, both slots in one launch
// (workgroup z = slot; dsi0/dsi1: the slot's DSI, 0 left view, 1 right).
template <bool SKY, bool UNI, int DC>
__global__ __launch_bounds__(256) void cost_ck_kernel(const uint64_t *__restrict__ ctl,
                                                      const uint64_t *__restrict__ ctr,
                                                      const uint8_t *__restrict__ sky0,
                                                      const uint8_t *__restrict__ sky1, int sky_pitch,
                                                      int H, int W, int D, int R, float *__restrict__ out0,
                                                      float *__restrict__ out1, int dsi0, int dsi1, int ns) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const bool z = __builtin_amdgcn_workgroup_id_z() != 0;
    if constexpr (!SKY) {
        if ((z ? dsi1 : dsi0) == 0) cost_ck_body<0, UNI>(ctl, ctr, H, W, D, R, z ? out1 : out0, bid_x(), smem, ns);
        else cost_ck_body<1, UNI>(ctl, ctr, H, W, D, R, z ? out1 : out0, bid_x(), smem, ns);
    } else if ((z ? dsi1 : dsi0) == 0) {
        cost_h_body<0, 5, SKY, true, UNI, DC, kVStripNC>(ctl, ctr, z ? sky1 : sky0, sky_pitch, H, W, D, 1, R,
                                                         z ? out1 : out0, bid_x(), smem, ns);
    } else {
        cost_h_body<1, 5, SKY, true, UNI, DC, kVStripNC>(ctl, ctr, z ? sky1 : sky0, sky_pitch, H, W, D, 1, R,
                                                         z ? out1 : out0, bid_x(), smem, ns);
    }
}

template <bool SKY>
static hipError_t launch_cost_ck_t(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky0,
                                   const uint8_t *sky1, int sky_pitch, int dsi0, int dsi1, int nviews,
                                   Geom g, float *ck0, float *ck1, hipStream_t st) {
    bool uni;
    int R;
    size_t smem;
    costh_shape(g, SKY, uni, R, smem);
    if (R < 1 || g.scale != 1) return hipErrorInvalidValue;  // (vstrip_supported)
    const dim3 grid((g.H + R - 1) / R, 1, nviews);
    const int ns = (int)vstrip_strips(g);
    // (census operands straight from global memory instead of the staged
    // rows measured slower: HD256 610 vs 317 us, 4K256 2.33 vs 1.82 ms; one
    // row per block, for more waves per CU, changed nothing:
    // profiles/r06_experiments/r06q_vstrip.txt)
#define CK_ARGS ctl, ctr, sky0, sky1, sky_pitch, g.H, g.W, g.D, R, ck0, ck1, dsi0, dsi1, ns
    if (uni) cost_ck_kernel<SKY, true, 0><<<grid, R * g.D, smem, st>>>(CK_ARGS);
    else if (g.D == 128) cost_ck_kernel<SKY, false, 128><<<grid, R * g.D, smem, st>>>(CK_ARGS);
    else cost_ck_kernel<SKY, false, 0><<<grid, R * g.D, smem, st>>>(CK_ARGS);
#undef CK_ARGS
    return hipGetLastError();
}

hipError_t launch_cost_ck(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky0,
                          const uint8_t *sky1, int sky_pitch, int dsi0, int dsi1, int nviews, Geom g,
                          float *ck0, float *ck1, hipStream_t st) {
    if (nviews == 2 && (sky0 == nullptr) != (sky1 == nullptr)) return hipErrorInvalidValue;
    if (sky0) return launch_cost_ck_t<true>(ctl, ctr, sky0, sky1, sky_pitch, dsi0, dsi1, nviews, g, ck0, ck1, st);
    return launch_cost_ck_t<false>(ctl, ctr, sky0, sky1, sky_pitch, dsi0, dsi1, nviews, g, ck0, ck1, st);
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

// ------------------------------------------------------ vertical pass

// The vertical IIR (Solver.cpp:333-368) runs fused with the L3 forward pass in
// sgm_pair.hip (vfwd_kernel); without the filter the volume is copied.
__global__ __launch_bounds__(256) void copy_kernel(const float *__restrict__ in,
                                                   float *__restrict__ out, size_t n) {
    const size_t i = (size_t)bid_x() * 256 + tid_x();
    if (i < n) out[i] = in[i];
}

hipError_t launch_copy(const float *in, float *out, Geom g, hipStream_t st) {
    const size_t n = (size_t)g.W * g.D * g.H;
    copy_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, st>>>(in, out, n);
    return hipGetLastError();
}


}  // namespace sgm
