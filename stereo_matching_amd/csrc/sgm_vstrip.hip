// sgm_vstrip.hip -- the strip pass of the slanted schedule: the horizontal
// IIR (Solver.cpp:296-330), the vertical IIR (Solver.cpp:333-368) and the
// L3 forward pass (SGM.cpp:161-199) in ONE pass, writing the final cost C and
// the L3 volume and nothing else (DESIGN.md 5f "Strips").
//
// The two filters are serial chains along perpendicular axes, so a single
// pass needs, at every row, the horizontal chain's state at the first column
// it owns.  A checkpoint pass (cost_h_body<..., CK = kVStripNC>, sgm_cost.hip)
// runs the horizontal chains alone and keeps only that state -- the running
// sum and the two values it will subtract -- at every strip edge: 3 floats
// per (row, strip, d), 0.5 B per element written and read again here,
// instead of the horizontally filtered volume's 4 B written by cost_h and
// read by vfwd.  Per element the pair moves 9 B where cost_h + vfwd_l3 moved
// 16.
//
// One workgroup per strip of kVStripNC columns of one view walks all rows
// top-down, one row per iteration (one LDS barrier each):
//   * NH "horizontal" waves (lane = one disparity) turn row `it`'s census
//     words (staged in LDS the iteration before) into raw costs and run the
//     horizontal IIR across the strip from the row's checkpoint, writing the
//     row's filtered costs Ch into an LDS ring of 4 rows;
//   * NV "vertical" waves (CPW columns each, lane l holding disparities
//     l*V .. l*V+V-1 as in vfwd_body) produce output row it-3 from the ring
//     -- the vertical IIR reads Ch two rows ahead -- and run the L3 DP on it.
// Every chain keeps the reference's order of operations (cost_h_body and
// vfwd_body restate them; this pass computes the same values), so C and L3
// are bit-identical to cost_h + vfwd_l3 (tests/test_gpu_vstrip.py).
#include "sgm_bodies.h"

namespace sgm {

// A row's staged census (double-buffered): the shifted image's words, the
// other image's (one per column), the sky flags (one word per column, from
// the sky-word array launch_sky_words writes), one dummy word for the idle
// lanes (every thread stores one word: no branches).
template <int V, int NC>
struct VStripStage {
    static constexpr int NSH = NC + 3 + 64 * V, UN = NSH, SK = UN + NC + 3, N = SK + NC + 3 + 1;
};
template <int V, int NC>
struct VStripLds {
    float ch[4][NC][64 * V];       // Ch of row r in ring slot r & 3
    float raw[2][NC + 3][64 * V];  // raw costs of a row (the strip's columns + 3)
    uint64_t st[2][VStripStage<V, NC>::N];
};

size_t vstrip_strips(Geom g) { return (size_t)((g.W + kVStripNC - 1) / kVStripNC); }
size_t vstrip_ck_floats(Geom g) { return (size_t)g.H * vstrip_strips(g) * 3 * g.D; }

// Iteration it (one LDS barrier each):
//   vertical waves: raw costs of row it+1 (from its staged census words) into
//     raw[(it+1) & 1], then output row it-3 (C and L3) from the Ch ring;
//   horizontal waves: the horizontal IIR of row it across the strip, from
//     raw[it & 1] and the row's checkpoint, into the Ch ring;
//   every thread: row it+2's census word to stage buffer it & 1, and the
//     register ring slot it held takes row it+2+PD.
// The raw costs are computed by the vertical waves (lane l: disparities
// l*V .. l*V+V-1 of one column, its V shifted words one 32-byte LDS read):
// the horizontal waves' part, a serial chain across the strip per disparity,
// would otherwise set the iteration's time.
template <int V, bool FULL, int NH, int NV, int CPW, int PD>
__global__ __launch_bounds__(64 * (NH + NV)) void vstrip_kernel(VStripArgs a, Geom g) {
    constexpr int NC = NV * CPW, NR = NC + 3;
    static_assert(NC == kVStripNC, "strip width");
    static_assert(CPW == 2, "two columns per vertical wave (wave_min_n<2>)");
    static_assert(PD >= 2, "the prologue stages two rows");
    __shared__ __attribute__((aligned(16))) VStripLds<V, NC> L;
    const int wave = wave_id(), lane = tid_x() & 63;
    const int H = g.H, W = g.W, D = g.D;
    const int NS = (W + NC - 1) / NC;
    const int slot = __builtin_amdgcn_workgroup_id_y();
    // neighbouring strips (which stage overlapping census words) on one XCD
    const int s = xcd_column(bid_x(), NS);
    const int j0 = s * NC;
    const int dsi = slot ? a.dsi1 : a.dsi0;

    // ---- census staging, one word per thread and row: the shifted image's
    // words for columns j0 - D + 1 .. j0 + NC + 2 (left-view DSI: the right
    // image at j - d, clamped at 0) or j0 .. j0 + NC + D + 1 (right-view DSI:
    // the left image at j + d, clamped at W-1) and the other image's for
    // columns j0 .. j0 + NC + 2 (clamped at W-1), and their sky flags.  Loads
    // run PD rows ahead of their LDS store through a register ring; every
    // thread loads one 8-byte word from a valid address, no branches (a branch
    // around a load makes the waitcnt pass drain the ring).  The sky mask comes
    // as words too (launch_sky_words): a byte load's zero-extension, which
    // hipcc scheduled right after its issue, waited for every load in flight.
    const int nsh = NC + 2 + D;
    const int sbase = dsi == 0 ? j0 - D + 1 : j0;
    const uint64_t *shimg = dsi == 0 ? a.ctr : a.ctl, *unimg = dsi == 0 ? a.ctl : a.ctr;
    using SG = VStripStage<V, NC>;
    const int x = tid_x();
    const uint64_t *skw = slot ? a.skw1 : a.skw0;
    const int kind = x < nsh ? 0 : (x < nsh + NR ? 1 : (x < nsh + 2 * NR ? 2 : 3));
    const int xi = kind == 0 ? x : (kind == 1 ? x - nsh : (kind == 2 ? x - nsh - NR : 0));
    const int scol = kind == 0 ? min(max(sbase + xi, 0), W - 1) : min(j0 + xi, W - 1);
    const int sidx = kind == 0 ? xi : (kind == 1 ? SG::UN + xi : (kind == 2 ? SG::SK + xi : SG::N - 1));
    const bool nosky = kind == 2 && skw == nullptr;  // (its lanes load a census word, store 0)
    const uint64_t *wsrc = (kind == 0 ? shimg : (kind == 2 && skw ? skw : unimg)) + scol;
    uint64_t rw_[PD];
    auto stage_load = [&](int u, int r) { rw_[u] = wsrc[(size_t)uniform(min(r, H - 1)) * W]; };
    auto stage_store = [&](int b, int u) { L.st[b][sidx] = nosky ? 0ull : rw_[u]; };
    // rows 0 and 1 to stage buffers 0 and 1; the ring then holds rows 2 .. PD+1
#pragma unroll
    for (int u = 0; u < PD; ++u) stage_load(u, u);
    stage_store(0, 0);
    stage_load(0, PD);
    stage_store(1, 1);
    stage_load(1, PD + 1);
    const int NIT = H + 3;  // iteration it: Ch row it, output row it - 3

    if (wave < NH) {
        // ------------------------------------------------ horizontal waves
        const int d = wave * 64 + lane;
        const int dd = d < D ? d : D - 1;  // (lanes past D read valid words)
        const float *ck = (slot ? a.ck1 : a.ck0) + (size_t)s * 3 * D + dd;
        const size_t ck_row = (size_t)NS * 3 * D;
        // the rows' checkpoints (strips past the first; strip 0 starts the
        // chain from raw costs), PD rows ahead
        float ks_[PD], k0_[PD], k1_[PD];
        auto ck_load = [&](int u, int r) {
            const float *q = ck + (size_t)uniform(min(r, H - 1)) * ck_row;
            ks_[u] = q[0];
            k0_[u] = q[D];
            k1_[u] = q[2 * D];
        };
#pragma unroll
        for (int u = 0; u < PD; ++u) ck_load(u, u);
        // a strip whose columns all lie in 2 .. W-4 (filtered, each followed
        // by an update): no selects
        const bool interior = s > 0 && j0 + NC - 1 < W - 3;
        auto iter = [&](int it, int u) {
            stage_store(it & 1, (u + 2) % PD);
            stage_load((u + 2) % PD, it + 2 + PD);
            if (it < H) {
                const float *rr = &L.raw[it & 1][0][d];
                float rw[NR];
#pragma unroll
                for (int xx = 0; xx < NR; ++xx) rw[xx] = rr[xx * 64 * V];
                float sum, h0, h1;
                if (s == 0) {
                    // cost_h_body's start: sum of raw[0 .. 4], positions 0, 1 raw
                    sum = 0.0f;
#pragma unroll
                    for (int k = 0; k < 5; ++k) sum += rw[k];
                    h0 = rw[0];
                    h1 = rw[1];
                } else {
                    sum = ks_[u];
                    h0 = k0_[u];
                    h1 = k1_[u];
                }
                float *row = &L.ch[it & 3][0][d];
                // cost_h_body's steps with LAG = 2: output p = div(sum) for
                // 2 <= p <= W-3 (raw outside), then for p < W-3 sum += raw[p+3],
                // sum -= the value at p-2
                if (interior) {
#pragma unroll
                    for (int xx = 0; xx < NC; ++xx) {
                        const float c = div_win<5>(sum);
                        sum += rw[xx + 3];
                        sum -= h0;
                        h0 = h1;
                        h1 = c;
                        row[xx * 64 * V] = c;
                    }
                } else {
                    // (uniform conditions as selects; columns past W compute
                    // values nobody reads)
#pragma unroll
                    for (int xx = 0; xx < NC; ++xx) {
                        const int p = j0 + xx;
                        const bool filt = p >= 2 && p <= W - 3, upd = p >= 2 && p < W - 3;
                        const float q = div_win<5>(sum);
                        const float c = filt ? q : rw[xx];
                        float ns = sum + rw[xx + 3];
                        ns -= h0;
                        sum = upd ? ns : sum;
                        h0 = filt ? h1 : h0;
                        h1 = filt ? c : h1;
                        row[xx * 64 * V] = c;
                    }
                }
            }
            ck_load(u, it + PD);
            lds_barrier();
        };
        lds_barrier();  // (the prologue's raw costs of row 0)
        lds_barrier();
        int it0 = 0;
        for (; it0 + PD <= NIT; it0 += PD) {
#pragma unroll
            for (int u = 0; u < PD; ++u) iter(it0 + u, u);
        }
#pragma unroll
        for (int u = 0; u < PD; ++u)
            if (it0 + u < NIT) iter(it0 + u, u);
        return;
    }

    // ---------------------------------------------------- vertical waves
    const int w = wave - NH;
    const int e0 = lane * V;
    const bool act = FULL || e0 < D;
    const float p2v = to_vgpr(a.p2);
    float *cout = slot ? a.c1 : a.c0;
    float *lout = slot ? a.l31 : a.l30;
    // raw costs of staged row (buffer b) at strip columns w, w + NV, w + 2NV
    // (< NR): lane l's disparities e0 .. e0+V-1 read V consecutive shifted
    // words (descending for the left-view DSI: word index xx + D-1-d)
    const int e0c = act ? e0 : 0;
    const int sh0 = dsi == 0 ? D - V - e0c : e0c;  // word of d = e0+V-1 (left) / e0 (right)
    auto raws = [&](int b) {
#pragma unroll
        for (int k = 0; k < (NR + NV - 1) / NV; ++k) {
            const int xx = w + k * NV;
            if (xx < NR) {
                const uint64_t *sw = &L.st[b][xx + sh0];
                const uint64_t un = L.st[b][SG::UN + xx];
                const bool sk = L.st[b][SG::SK + xx] != 0;
                float r[V];
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    // the sky override of Solver.cpp:165-178
                    const float c = hamming(un, sw[dsi == 0 ? V - 1 - v : v]);
                    r[v] = sk ? (e0 + v == 0 ? 0.0f : 999999.0f) : c;
                }
                store_lds_v<V>(&L.raw[b][xx][e0], r);
            }
        }
    };
    float sum[CPW][V], o1[CPW][V], prev[CPW][V], pmin[CPW];
    // the outputs of the iteration's row, stored after the branch (an
    // iteration without a row stores to the dummy area: a store inside a
    // branch makes the waitcnt pass wait for it before the ring's next use)
    float c[CPW][V], Lv[CPW][V];
#pragma unroll
    for (int q = 0; q < CPW; ++q)
#pragma unroll
        for (int v = 0; v < V; ++v) c[q][v] = Lv[q][v] = 0.0f;
    // Ch of (row r, strip column xx); lanes past D hold +inf, as vfwd's loads
    auto rd = [&](int r, int xx, float (&t)[V]) {
        load_lds_v<V>(t, &L.ch[r & 3][xx][e0]);
#pragma unroll
        for (int v = 0; v < V; ++v) t[v] = act ? t[v] : SGM_INF;
    };
    auto iter = [&](int it, int u) {
        // (the staging first: its wait then covers none of this iteration's stores)
        stage_store(it & 1, (u + 2) % PD);
        stage_load((u + 2) % PD, it + 2 + PD);
        if (it + 1 < H) raws((it + 1) & 1);
        const int i = it - 3;  // output row
        if (i >= 0) {
            float mn[CPW];
#pragma unroll
            for (int q = 0; q < CPW; ++q) {
                const int xx = w * CPW + q;
                if (i == 0) {
                    // vfwd_body's start: sum = 0 + Ch0 + Ch1 + Ch2, row 0 raw
                    float r0[V], r1[V], r2[V];
                    rd(0, xx, r0);
                    rd(1, xx, r1);
                    rd(2, xx, r2);
#pragma unroll
                    for (int v = 0; v < V; ++v) {
                        sum[q][v] = 0.0f;
                        sum[q][v] += r0[v];
                        sum[q][v] += r1[v];
                        sum[q][v] += r2[v];
                        prev[q][v] = 0.0f;
                        c[q][v] = r0[v];
                        o1[q][v] = r0[v];
                    }
                    pmin[q] = 0.0f;
                } else if (i == H - 1) {
                    rd(H - 1, xx, c[q]);
                } else {
#pragma unroll
                    for (int v = 0; v < V; ++v) c[q][v] = div_win<3>(sum[q][v]);
                    if (i < H - 2) {
                        float rr[V];
                        rd(i + 2, xx, rr);
#pragma unroll
                        for (int v = 0; v < V; ++v) sum[q][v] = (sum[q][v] + rr[v]) - o1[q][v];
                    }
#pragma unroll
                    for (int v = 0; v < V; ++v) o1[q][v] = c[q][v];
                }
                // L3 forward step (L = 0, minL = 0 before row 0 gives L = C)
                dp_step<V>(prev[q], pmin[q], c[q], Lv[q], a.p1, p2v);
                mn[q] = lane_min(Lv[q]);
            }
            wave_min_n<CPW>(mn);
#pragma unroll
            for (int q = 0; q < CPW; ++q) {
#pragma unroll
                for (int v = 0; v < V; ++v) prev[q][v] = Lv[q][v];
                pmin[q] = mn[q];
            }
        }
#pragma unroll
        for (int q = 0; q < CPW; ++q) {
            const int col = j0 + w * CPW + q;
            const bool st = act && i >= 0 && col < W;
            const size_t o = ((size_t)(i > 0 ? i : 0) * W + col) * D + e0;
            store_v_nt<V>(st ? cout + o : a.dummy + e0, c[q], true);
            store_v_nt<V>(st ? lout + o : a.dummy + e0, Lv[q], true);
        }
        lds_barrier();
    };
    lds_barrier();
    raws(0);  // row 0's raw costs before the first iteration
    lds_barrier();
    int it0 = 0;
    for (; it0 + PD <= NIT; it0 += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) iter(it0 + u, u);
    }
#pragma unroll
    for (int u = 0; u < PD; ++u)
        if (it0 + u < NIT) iter(it0 + u, u);
}

bool vstrip_supported(Geom g, bool sky) { return g.scale == 1 && cost_h2_supported(g, sky); }

// The sky mask as one word per pixel (0 or 1) for the strip pass's staging.
__global__ __launch_bounds__(256) void sky_words_kernel(const uint8_t *__restrict__ sky, int pitch, int H,
                                                         int W, uint64_t *__restrict__ out) {
    const size_t n = (size_t)H * W;
    for (size_t k = (size_t)bid_x() * 256 + tid_x(); k < n; k += (size_t)gridDim.x * 256) {
        const size_t i = k / W, j = k - i * W;
        out[k] = sky[i * pitch + j] == 255 ? 1ull : 0ull;
    }
}

size_t vstrip_sky_words_offset(Geom g) { return (vstrip_ck_floats(g) + 1) & ~(size_t)1; }

hipError_t launch_sky_words(const uint8_t *sky, int pitch, Geom g, uint64_t *out, hipStream_t st) {
    const size_t n = (size_t)g.H * g.W;
    const unsigned blocks = (unsigned)min((n + 255) / 256, (size_t)4096);
    sky_words_kernel<<<blocks, 256, 0, st>>>(sky, pitch, g.H, g.W, out);
    return hipGetLastError();
}

hipError_t launch_vstrip(const VStripArgs &a, int nviews, Geom g, hipStream_t st) {
    const dim3 grid((unsigned)vstrip_strips(g), nviews);
    constexpr int NV = kVStripNC / 2;
#ifndef VSTRIP_PD
#define VSTRIP_PD 4
#endif
    constexpr int PD = VSTRIP_PD;  // rows of census / checkpoint loads in flight
    if (g.D == 32) vstrip_kernel<1, false, 1, NV, 2, PD><<<grid, 64 * (1 + NV), 0, st>>>(a, g);
    else if (g.D == 64) vstrip_kernel<1, true, 1, NV, 2, PD><<<grid, 64 * (1 + NV), 0, st>>>(a, g);
    else if (g.D == 128) vstrip_kernel<2, true, 2, NV, 2, PD><<<grid, 64 * (2 + NV), 0, st>>>(a, g);
    else if (g.D == 256) vstrip_kernel<4, true, 4, NV, 2, PD><<<grid, 64 * (4 + NV), 0, st>>>(a, g);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace sgm
