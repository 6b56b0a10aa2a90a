// sgm_pair.hip -- forward/backward path pairs with checkpoint recompute.
//
// Two opposite directions on the same scanlines (L1/L2 rows, L3/L4 columns,
// L6/L7 wrapped anti-diagonals) are computed by one forward kernel that only
// stores its path state every K steps, and one backward kernel that, per
// K-step segment, recomputes the forward costs from the checkpoint into
// registers (reading each cost once for both directions) and combines
//   S12 = L1 + L2, T = (T5 + L6) + L7, total = ((S12 + L3) + L4) + T
// on the fly -- the reference's association order (SGM.cpp:386-390) -- so no
// single-direction volume is ever written (DESIGN.md "Pairs").
//
// Segments are counted from the END of a chain of n steps: segment 0 covers
// positions [0, r0) with r0 = n - (nseg-1)*K, segment s >= 1 covers
// [r0 + (s-1)K, r0 + sK).  Checkpoint m (0 <= m < nseg-1) is the forward state
// after position r0-1 + mK and seeds segment m+1.  The backward pass therefore
// meets full segments first and the partial one last.
#include "sgm_bodies.h"

namespace sgm {


static inline int chain_len(int family, Geom g) { return family == PAIR_H ? g.W : g.H; }
static inline int num_chains(int family, Geom g) { return family == PAIR_H ? g.H : g.W; }

size_t pair_ckpt_floats(int family, Geom g) {
    const int V = vals_per_lane(g.D);
    const int K = family == PAIR_V ? seg_k_v(V) : seg_k_hd(V);
    const int n = chain_len(family, g);
    const size_t nseg = (size_t)((n + K - 1) / K);
    return (size_t)num_chains(family, g) * nseg * g.D;
}

// ------------------------------------------------------------ kernels

// vfwd_body (sgm_bodies.h): the vertical IIR fused with the L3 forward pass,
// one wave per column.
template <int V, bool FULL, int WIN, int PF, bool BAND = false, bool L3OUT = false>
__global__ __launch_bounds__(64) void vfwd_kernel(const float *__restrict__ in,
                                                  float *__restrict__ out, PairArgs a, Geom g) {
    vfwd_body<V, FULL, WIN, PF, BAND, L3OUT>(in, out, a, g, bid_x(), tid_x());
}

// Both views' vertical passes in one launch, workgroup y = view: W chains per
// view leave about one wave per SIMD at KITTI and two at HD, one launch of 2W
// twice that.  L3OUT: writing C and the whole L3 volume (the slanted
// schedule), else C and the L3 checkpoints (the joint whole-volume one).
template <int V, bool FULL, int WIN, int PF, bool L3OUT>
__global__ __launch_bounds__(64) void vfwd2_kernel(const float *__restrict__ in0, float *__restrict__ out0,
                                                   PairArgs a0, const float *__restrict__ in1,
                                                   float *__restrict__ out1, PairArgs a1, Geom g) {
    const bool vb = __builtin_amdgcn_workgroup_id_y() != 0;
    vfwd_body<V, FULL, WIN, PF, false, L3OUT>(vb ? in1 : in0, vb ? out1 : out0, vb ? a1 : a0, g, bid_x(),
                                              tid_x());
}

template <int FD, int V, bool FULL, int PF>
__global__ __launch_bounds__(64) void pair_fwd_kernel(PairArgs a, Geom g) {
    pair_fwd_body<FD, V, FULL, PF>(a, g, bid_x());
}

template <int FAM, int V, bool FULL, int MODE>
__global__ __launch_bounds__(64) void pair_bwd_kernel(PairArgs a, Geom g) {
    pair_bwd_body<FAM, V, FULL, MODE>(a, g, bid_x(), nullptr, nullptr);
}

// The final pass of a view: PAIR_V backward (L4, recomputing L3) summed with
// S12 and T, then WTA.  Three waves (pair_split_body): wave 0 recomputes L3
// segments from their checkpoints, wave 1 runs L4 and sums the totals into an
// LDS ring, wave 2 runs the batched WTA on the chunk before.
// D >= 64 run two WTA waves per column (each takes half of a chunk's pixels).
template <int V, bool FULL>
constexpr int final_nwta() { return FULL ? 2 : 1; }

// BAND: one band of the banded backward phase (a.band).  NTC: C by
// non-temporal loads (a.nt_cost: two-view frames, whose views' cost volumes
// alternate in the Infinity Cache; profiles/r06_experiments/r06aa_final_nt.txt)
template <int V, bool FULL, bool BAND = false, bool NTC = false>
__global__ __launch_bounds__(256) void pair_final_kernel(PairArgs a, Geom g) {
    constexpr int K = pair_kv<V>();
    __shared__ __attribute__((aligned(16))) SplitFinalLds<K, V> lds;
#ifdef SGM_NO_XCD_COLUMNS
    const int path = bid_x();
#else
    // row-major output maps (one-view frames): a line's columns on one XCD
    const int path = a.sub_cm ? bid_x() : xcd_column(bid_x(), g.W);
#endif
    pair_split_body<PAIR_V, V, FULL, PAIR_FINAL, K, 3, 2, final_nwta<V, FULL>(), BAND, NTC>(
        a, g, path, wave_id(), lds.s, &lds);
}

// Both views' final passes in one launch (workgroup z = view).  Above the
// Infinity Cache nothing is gained by finishing a view before the other one
// starts, and one launch of 2W columns packs the workgroups into fewer rounds
// (HD256: 2 x 1920 columns at 1280 resident workgroups take 3 rounds instead
// of 2 + 2).
template <int V, bool FULL>
__global__ __launch_bounds__(256) void pair_final2_kernel(PairArgs a0, PairArgs a1, Geom g) {
    constexpr int K = pair_kv<V>();
    __shared__ __attribute__((aligned(16))) SplitFinalLds<K, V> lds;
    const PairArgs a = __builtin_amdgcn_workgroup_id_z() != 0 ? a1 : a0;
    pair_split_body<PAIR_V, V, FULL, PAIR_FINAL, K, 3, 2, final_nwta<V, FULL>()>(
        a, g, bid_x(), wave_id(), lds.s, &lds);
}

// Multi-role stage kernels of the frame schedule: block ranges run different
// (independent) roles, so a latency-bound horizontal role (H chains, few and
// long) overlaps the bandwidth-bound diagonal roles inside one launch.  The
// H blocks come first so they start at once.
//   stage A: L1 forward (ckpt)  |  L5 -> T5         |  L6 forward (ckpt)
//   stage B: L2 backward -> S12 |  L7 backward: T = (T5 + L6) + L7
// ROLES 1 (the forward bands, volumes above the Infinity Cache): the
// diagonal roles only, steps [kb, ke) of each chain (l5.band, d6.band); the
// H pair then runs as its own launch (hpair_kernel) after the last forward
// band -- its whole-row chains would set every band launch's length.
template <int V, bool FULL, int ROLES = 0>
__global__ __launch_bounds__(64) void stage_a_kernel(PairArgs h1, SweepArgs l5, PairArgs d6,
                                                     Geom g) {
    constexpr int PFH = V >= 4 ? 16 : 32, PFD = V >= 4 ? 8 : 16;
    int b = bid_x();
    if constexpr (ROLES == 1) {
        if (b < g.W) sweep_body<4, V, SWEEP_INIT, FULL, PFD, true>(l5, g, b);
        else pair_fwd_body<5, V, FULL, PFD, true>(d6, g, b - g.W);
        return;
    }
    if (b < g.H) {
        // the H chains (few, long) are the launch's critical path
        __builtin_amdgcn_s_setprio(3);
        pair_fwd_body<0, V, FULL, PFH>(h1, g, b);
        return;
    }
    b -= g.H;
    if (b < g.W) {
        sweep_body<4, V, SWEEP_INIT, FULL, PFD>(l5, g, b);
        return;
    }
    pair_fwd_body<5, V, FULL, PFD>(d6, g, b - g.W);
}

// The forward bands' H pair (L1 forward, then L2 backward recomputing L1 from
// the checkpoints it has just written -> S12) of one or two views in one
// launch (workgroup y = view).  With the diagonal roles in the band launches
// this launch holds only H (per view) single-wave chains, about one per SIMD
// at HD256, so it waits on memory latency; both views' rows side by side
// double the loads in flight.
template <int V, bool FULL>
__global__ __launch_bounds__(64) void hpair_kernel(PairArgs h1a, PairArgs h2a, PairArgs h1b,
                                                   PairArgs h2b, Geom g) {
#ifdef SGM_HPF
    constexpr int PFH = V >= 4 ? SGM_HPF : 2 * SGM_HPF;
#else
    constexpr int PFH = V >= 4 ? 16 : 32;
#endif
    const bool vb = __builtin_amdgcn_workgroup_id_y() != 0;
    const PairArgs h1 = vb ? h1b : h1a;
    const PairArgs h2 = vb ? h2b : h2a;
    // C is read by non-temporal loads (NTC): the H pair runs only above the
    // Infinity Cache, where its two reads of C pass through once each (the
    // top-down pass beside it -2.6%, HD256 frame -1.0%, 4K256 -0.6% paired,
    // profiles/r06_experiments/r06x_hpair_nt.txt)
    pair_fwd_body<0, V, FULL, PFH, false, true>(h1, g, bid_x());
    __threadfence();  // this wave's checkpoint stores, before it reads them back
    pair_bwd_body<PAIR_H, V, FULL, PAIR_INIT2, false, true>(h2, g, bid_x(), nullptr, nullptr);
}

// Stage B blocks are two waves: an H block splits its row's L2 pass into a
// recompute wave and a backward wave (pair_split_body); a D2 block runs two
// anti-diagonal L7 chains, one per wave.
// HROWS = false: a banded stage B (d7.band: the diagonal pair's steps
// [kb, ke)) without H rows -- the banded schedule's H pair ran them
// (hpair_kernel).
template <int V, bool FULL, bool HROWS>
__global__ __launch_bounds__(128) void stage_b_kernel(PairArgs h2, PairArgs d7, Geom g) {
    constexpr int K = pair_k<V>();
    __shared__ __attribute__((aligned(16))) SplitLds<K, V> lds;
    const int b = bid_x(), wave = wave_id();
    const int nh = HROWS ? g.H : 0;
    if (HROWS && b < nh) {
        pair_split_body<PAIR_H, V, FULL, PAIR_INIT2, K, 3>(h2, g, b, wave, lds, nullptr);
        return;
    }
    const int path = 2 * (b - nh) + wave;
    if (path < g.W) pair_bwd_body<PAIR_D2, V, FULL, PAIR_ACC, !HROWS>(d7, g, path, nullptr, nullptr);
}

// Both views' stage A / stage B in one launch (workgroup y = view): frames
// whose two cost volumes fit the 256 MB Infinity Cache together (K64), where
// one view's launches leave most SIMDs with a single chain.
template <int V, bool FULL>
__global__ __launch_bounds__(64) void stage_a2_kernel(PairArgs h1a, SweepArgs l5a, PairArgs d6a,
                                                      PairArgs h1b, SweepArgs l5b, PairArgs d6b,
                                                      Geom g) {
    constexpr int PFH = V >= 4 ? 16 : 32, PFD = V >= 4 ? 8 : 16;
    const bool vb = __builtin_amdgcn_workgroup_id_y() != 0;
    int b = bid_x();
    if (b < g.H) {
        __builtin_amdgcn_s_setprio(3);
        pair_fwd_body<0, V, FULL, PFH>(vb ? h1b : h1a, g, b);
        return;
    }
    b -= g.H;
    if (b < g.W) {
        sweep_body<4, V, SWEEP_INIT, FULL, PFD>(vb ? l5b : l5a, g, b);
        return;
    }
    pair_fwd_body<5, V, FULL, PFD>(vb ? d6b : d6a, g, b - g.W);
}

template <int V, bool FULL>
__global__ __launch_bounds__(128) void stage_b2_kernel(PairArgs h2a, PairArgs d7a, PairArgs h2b,
                                                       PairArgs d7b, Geom g) {
    constexpr int K = pair_k<V>();
    __shared__ __attribute__((aligned(16))) SplitLds<K, V> lds;
    const bool vb = __builtin_amdgcn_workgroup_id_y() != 0;
    const int b = bid_x(), wave = wave_id();
    if (b < g.H) {
        pair_split_body<PAIR_H, V, FULL, PAIR_INIT2, K, 3>(vb ? h2b : h2a, g, b, wave, lds, nullptr);
        return;
    }
    const int path = 2 * (b - g.H) + wave;
    if (path < g.W) pair_bwd_body<PAIR_D2, V, FULL, PAIR_ACC>(vb ? d7b : d7a, g, path, nullptr, nullptr);
}

hipError_t launch_stage_a2(const PairArgs *h1, const SweepArgs *l5, const PairArgs *d6, Geom g,
                           hipStream_t st) {
    const dim3 grid(g.H + 2 * g.W, 2);
    if (g.D == 32) stage_a2_kernel<1, false><<<grid, 64, 0, st>>>(h1[0], l5[0], d6[0], h1[1], l5[1], d6[1], g);
    else if (g.D == 64) stage_a2_kernel<1, true><<<grid, 64, 0, st>>>(h1[0], l5[0], d6[0], h1[1], l5[1], d6[1], g);
    else if (g.D == 128) stage_a2_kernel<2, true><<<grid, 64, 0, st>>>(h1[0], l5[0], d6[0], h1[1], l5[1], d6[1], g);
    else stage_a2_kernel<4, true><<<grid, 64, 0, st>>>(h1[0], l5[0], d6[0], h1[1], l5[1], d6[1], g);
    return hipGetLastError();
}

hipError_t launch_stage_b2(const PairArgs *h2, const PairArgs *d7, Geom g, hipStream_t st) {
    const dim3 grid(g.H + (g.W + 1) / 2, 2);
    if (g.D == 32) stage_b2_kernel<1, false><<<grid, 128, 0, st>>>(h2[0], d7[0], h2[1], d7[1], g);
    else if (g.D == 64) stage_b2_kernel<1, true><<<grid, 128, 0, st>>>(h2[0], d7[0], h2[1], d7[1], g);
    else if (g.D == 128) stage_b2_kernel<2, true><<<grid, 128, 0, st>>>(h2[0], d7[0], h2[1], d7[1], g);
    else stage_b2_kernel<4, true><<<grid, 128, 0, st>>>(h2[0], d7[0], h2[1], d7[1], g);
    return hipGetLastError();
}

template <int ROLES = 0>
static void launch_stage_a_t(const PairArgs &h1, const SweepArgs &l5, const PairArgs &d6, Geom g,
                             hipStream_t st, int nblk) {
    const dim3 grid(nblk);
    if (g.D == 32) stage_a_kernel<1, false, ROLES><<<grid, 64, 0, st>>>(h1, l5, d6, g);
    else if (g.D == 64) stage_a_kernel<1, true, ROLES><<<grid, 64, 0, st>>>(h1, l5, d6, g);
    else if (g.D == 128) stage_a_kernel<2, true, ROLES><<<grid, 64, 0, st>>>(h1, l5, d6, g);
    else stage_a_kernel<4, true, ROLES><<<grid, 64, 0, st>>>(h1, l5, d6, g);
}

hipError_t launch_stage_a(const PairArgs &h1, const SweepArgs &l5, const PairArgs &d6, Geom g,
                          hipStream_t st) {
    launch_stage_a_t(h1, l5, d6, g, st, g.H + 2 * g.W);
    return hipGetLastError();
}

hipError_t launch_stage_a_hpair(const PairArgs *h1, const PairArgs *h2, int nviews, Geom g,
                                hipStream_t st) {
    const dim3 grid(g.H, nviews);
    const PairArgs &b1 = h1[nviews - 1], &b2 = h2[nviews - 1];
    if (g.D == 32) hpair_kernel<1, false><<<grid, 64, 0, st>>>(h1[0], h2[0], b1, b2, g);
    else if (g.D == 64) hpair_kernel<1, true><<<grid, 64, 0, st>>>(h1[0], h2[0], b1, b2, g);
    else if (g.D == 128) hpair_kernel<2, true><<<grid, 64, 0, st>>>(h1[0], h2[0], b1, b2, g);
    else hpair_kernel<4, true><<<grid, 64, 0, st>>>(h1[0], h2[0], b1, b2, g);
    return hipGetLastError();
}

hipError_t launch_stage_a_band(const SweepArgs &l5, const PairArgs &d6, Geom g, hipStream_t st) {
    launch_stage_a_t<1>(d6, l5, d6, g, st, 2 * g.W);
    return hipGetLastError();
}

template <bool HROWS>
static void launch_stage_b_t(const PairArgs &h2, const PairArgs &d7, Geom g, hipStream_t st) {
    const dim3 grid((HROWS ? g.H : 0) + (g.W + 1) / 2);
    if (g.D == 32) stage_b_kernel<1, false, HROWS><<<grid, 128, 0, st>>>(h2, d7, g);
    else if (g.D == 64) stage_b_kernel<1, true, HROWS><<<grid, 128, 0, st>>>(h2, d7, g);
    else if (g.D == 128) stage_b_kernel<2, true, HROWS><<<grid, 128, 0, st>>>(h2, d7, g);
    else stage_b_kernel<4, true, HROWS><<<grid, 128, 0, st>>>(h2, d7, g);
}

hipError_t launch_stage_b(const PairArgs &h2, const PairArgs &d7, Geom g, hipStream_t st) {
    if (d7.band.ke > 0) launch_stage_b_t<false>(h2, d7, g, st);
    else launch_stage_b_t<true>(h2, d7, g, st);
    return hipGetLastError();
}

// -------------------------------------------------------------- launch

template <int FD>
static void launch_fwd_t(const PairArgs &a, Geom g, hipStream_t st) {
    const dim3 grid(FD == 0 ? g.H : g.W);
    constexpr int PF = FD == 0 ? 32 : 16;
    if (g.D == 32) pair_fwd_kernel<FD, 1, false, PF><<<grid, 64, 0, st>>>(a, g);
    else if (g.D == 64) pair_fwd_kernel<FD, 1, true, PF><<<grid, 64, 0, st>>>(a, g);
    else if (g.D == 128) pair_fwd_kernel<FD, 2, true, PF><<<grid, 64, 0, st>>>(a, g);
    else pair_fwd_kernel<FD, 4, true, PF / 2><<<grid, 64, 0, st>>>(a, g);
}

hipError_t launch_pair_fwd(int family, const PairArgs &a, Geom g, hipStream_t st) {
    // (the production schedule runs PAIR_V's forward pass fused into the
    // vertical cost filter, launch_vfwd; this one starts from a final volume)
    if (family == PAIR_H) launch_fwd_t<0>(a, g, st);
    else if (family == PAIR_V) launch_fwd_t<2>(a, g, st);
    else launch_fwd_t<5>(a, g, st);
    return hipGetLastError();
}

template <int WIN, bool BAND, bool L3OUT = false>
static void launch_vfwd_t(const float *in, float *out, const PairArgs &a, Geom g, hipStream_t st) {
    const dim3 grid(g.W);
    if (g.D == 32) vfwd_kernel<1, false, WIN, 16, BAND, L3OUT><<<grid, 64, 0, st>>>(in, out, a, g);
    else if (g.D == 64) vfwd_kernel<1, true, WIN, 16, BAND, L3OUT><<<grid, 64, 0, st>>>(in, out, a, g);
    else if (g.D == 128) vfwd_kernel<2, true, WIN, 16, BAND, L3OUT><<<grid, 64, 0, st>>>(in, out, a, g);
    else vfwd_kernel<4, true, WIN, 8, BAND, L3OUT><<<grid, 64, 0, st>>>(in, out, a, g);
}

hipError_t launch_vfwd(const float *in, float *out, const PairArgs &a, Geom g, hipStream_t st) {
    const bool band = a.band.ke > 0;
    if (g.scale == 1) band ? launch_vfwd_t<3, true>(in, out, a, g, st) : launch_vfwd_t<3, false>(in, out, a, g, st);
    else band ? launch_vfwd_t<1, true>(in, out, a, g, st) : launch_vfwd_t<1, false>(in, out, a, g, st);
    return hipGetLastError();
}

hipError_t launch_vfwd_l3(const float *in, float *out, float *l3, const PairArgs &a, Geom g,
                          hipStream_t st) {
    PairArgs b = a;
    b.out = l3;
    if (g.scale == 1) launch_vfwd_t<3, false, true>(in, out, b, g, st);
    else launch_vfwd_t<1, false, true>(in, out, b, g, st);
    return hipGetLastError();
}

template <int WIN, bool L3OUT>
static void launch_vfwd2_t(const float *const *in, float *const *out, const PairArgs *b, Geom g,
                           hipStream_t st) {
    const dim3 grid(g.W, 2);
#define VFWD2_ARGS in[0], out[0], b[0], in[1], out[1], b[1], g
    if (g.D == 32) vfwd2_kernel<1, false, WIN, 16, L3OUT><<<grid, 64, 0, st>>>(VFWD2_ARGS);
    else if (g.D == 64) vfwd2_kernel<1, true, WIN, 16, L3OUT><<<grid, 64, 0, st>>>(VFWD2_ARGS);
    else if (g.D == 128) vfwd2_kernel<2, true, WIN, 16, L3OUT><<<grid, 64, 0, st>>>(VFWD2_ARGS);
#ifndef VFWD2_PF4
#define VFWD2_PF4 8
#endif
    else vfwd2_kernel<4, true, WIN, L3OUT ? VFWD2_PF4 : 8, L3OUT><<<grid, 64, 0, st>>>(VFWD2_ARGS);
#undef VFWD2_ARGS
}

hipError_t launch_vfwd2_l3(const float *const *in, float *const *out, float *const *l3, const PairArgs *a,
                           Geom g, hipStream_t st) {
    PairArgs b[2] = {a[0], a[1]};
    b[0].out = l3[0];
    b[1].out = l3[1];
    if (g.scale == 1) launch_vfwd2_t<3, true>(in, out, b, g, st);
    else launch_vfwd2_t<1, true>(in, out, b, g, st);
    return hipGetLastError();
}

hipError_t launch_vfwd2(const float *const *in, float *const *out, const PairArgs *a, Geom g, hipStream_t st) {
    if (g.scale == 1) launch_vfwd2_t<3, false>(in, out, a, g, st);
    else launch_vfwd2_t<1, false>(in, out, a, g, st);
    return hipGetLastError();
}

template <int FAM, int MODE>
static void launch_bwd_t(const PairArgs &a, Geom g, hipStream_t st) {
    const dim3 grid(FAM == PAIR_H ? g.H : g.W);
    if (g.D == 32) pair_bwd_kernel<FAM, 1, false, MODE><<<grid, 64, 0, st>>>(a, g);
    else if (g.D == 64) pair_bwd_kernel<FAM, 1, true, MODE><<<grid, 64, 0, st>>>(a, g);
    else if (g.D == 128) pair_bwd_kernel<FAM, 2, true, MODE><<<grid, 64, 0, st>>>(a, g);
    else pair_bwd_kernel<FAM, 4, true, MODE><<<grid, 64, 0, st>>>(a, g);
}

template <bool BAND, bool NTC = false>
static void launch_final_b(const PairArgs &a, Geom g, hipStream_t st) {
    const dim3 grid(g.W);
    if (g.D == 32) pair_final_kernel<1, false, BAND, NTC><<<grid, 64 * (2 + final_nwta<1, false>()), 0, st>>>(a, g);
    else if (g.D == 64) pair_final_kernel<1, true, BAND, NTC><<<grid, 64 * (2 + final_nwta<1, true>()), 0, st>>>(a, g);
    else if (g.D == 128) pair_final_kernel<2, true, BAND, NTC><<<grid, 64 * (2 + final_nwta<2, true>()), 0, st>>>(a, g);
    else pair_final_kernel<4, true, BAND, NTC><<<grid, 64 * (2 + final_nwta<4, true>()), 0, st>>>(a, g);
}

static void launch_final_t(const PairArgs &a, Geom g, hipStream_t st) {
    if (a.band.ke > 0) launch_final_b<true>(a, g, st);
    else if (a.nt_cost) launch_final_b<false, true>(a, g, st);
    else launch_final_b<false>(a, g, st);
}

hipError_t launch_final2(const PairArgs &a0, const PairArgs &a1, Geom g, hipStream_t st) {
    const dim3 grid(g.W, 1, 2);
    if (g.D == 32) pair_final2_kernel<1, false><<<grid, 64 * (2 + final_nwta<1, false>()), 0, st>>>(a0, a1, g);
    else if (g.D == 64) pair_final2_kernel<1, true><<<grid, 64 * (2 + final_nwta<1, true>()), 0, st>>>(a0, a1, g);
    else if (g.D == 128) pair_final2_kernel<2, true><<<grid, 64 * (2 + final_nwta<2, true>()), 0, st>>>(a0, a1, g);
    else pair_final2_kernel<4, true><<<grid, 64 * (2 + final_nwta<4, true>()), 0, st>>>(a0, a1, g);
    return hipGetLastError();
}

hipError_t launch_pair_bwd(int family, int mode, const PairArgs &a, Geom g, hipStream_t st) {
    // the production schedule uses H/INIT2, D2/ACC and V/FINAL
    if (family == PAIR_H && mode == PAIR_INIT2) launch_bwd_t<PAIR_H, PAIR_INIT2>(a, g, st);
    else if (family == PAIR_D2 && mode == PAIR_ACC) launch_bwd_t<PAIR_D2, PAIR_ACC>(a, g, st);
    else if (family == PAIR_V && mode == PAIR_FINAL) launch_final_t(a, g, st);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace sgm

#ifdef SGM_STAMPS
extern "C" int sgm_debug_stamps_pair(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sgm::sgm_stamps), sizeof(sgm::sgm_stamps)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[16][3] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sgm::sgm_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
