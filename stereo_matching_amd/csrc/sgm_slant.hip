// sgm_slant.hip -- the slanted-tile aggregation passes (DESIGN.md "Slanted
// tiles"): several scanline directions in ONE pass over the cost volume.
//
// The reference runs each of its eight directions as its own loop nest
// (SGM.cpp:81-369); the pair kernels (sgm_pair.hip) fuse two opposite
// directions per chain, but every chain family still needs its own passes
// over C.  A pass that walks rows can carry the vertical and both diagonal
// families at once only if the workgroups that own neighbouring columns hand
// their diagonal states to each other every row.  Here the columns are cut
// into tiles that lean along one diagonal: tile t owns the skewed columns
// u = j - s in [u_lo, u_lo + NW) at every step s (row i = H-1-s for the
// bottom-up pass), wave k of the tile following the pixel (H-1-s, u_lo+k+s).
// The leaning direction's chains (L7 for the bottom-up pass) then stay inside
// one wave, and the other two families (L4 straight up, L8 up-left) move to
// LOWER wave numbers: L4 from wave k+1, L8 from wave k+2 of the previous
// step.  Waves exchange them through LDS; the last one or two waves of a tile
// take them from the next tile (t+1), whose first waves publish them as
// 8-byte {value, tag} granules (no flag, no fence: the data is the flag,
// cdna_hip_programming.md Guideline 16, R2).  All dependencies point from
// tile t+1 to tile t, so tiles claimed in the order t = T-1, T-2, ... never
// wait on a tile no workgroup holds: no deadlock for any grid size, and a
// tile may run any number of steps behind its right neighbour.
//
// The bottom-up pass (slant_up_kernel) computes, per pixel,
//   L4 (SGM.cpp:201-239), L7, L8 (:311-369),
//   total = ((S12 + L3) + L4) + ((T56 + L7) + L8)   (SGM.cpp:386-390)
// and the WTA + uniqueness + sub-pixel (SGM.cpp:372-418, Solver.cpp:569-597),
// reading C, S12 = L1+L2, L3 and T56 = L5+L6 once each (16 B per element
// instead of the 36.75 of stage B's diagonal pair + L8 + the final pass).
#include "sgm_bodies.h"

namespace sgm {

// Per-step LDS exchange of one tile: the L4 and L8 states (and their minima)
// of every wave for the previous step (parity (s-1)&1) and this one (s&1);
// slots NW and NW+1 hold the next tile's wave 0 / wave 1 states, put there
// by the courier wave.
template <int V, int NW>
struct SlantUpLds {
    float st[2][NW + 2][2][64 * V];
    float pm[2][NW + 2][2];
    int ticket;
    unsigned epoch;
};

// granule index of (view, tile, step, slot 0..2, disparity): slot 0 = wave 0's
// L4, slot 1 = wave 0's L8, slot 2 = wave 1's L8
__device__ __forceinline__ size_t gran_index(int T, int H, int D, int view, int t, int s, int slot) {
    return ((((size_t)view * T + t) * H + s) * 3 + slot) * D;
}

template <int V>
__device__ __forceinline__ void store_granules(unsigned long long *g, const float (&x)[V], unsigned tag) {
#pragma unroll
    for (int v = 0; v < V; ++v)
        __hip_atomic_store(g + v, ((unsigned long long)tag << 32) | __float_as_uint(x[v]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float uni_f(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

#ifdef SGM_SLANT_STAMPS
// [0] tile-steps (compute wave 0)  [1] courier phases that re-polled
// [2] courier re-polls  [3] courier cycles in re-polls  [4] compute wave 0
// cycles between barriers  [5] compute wave 0 cycles in barriers
// [6] courier cycles between barriers  [7] cycles inside tiles (wave 0)
// [8] workgroups  [9] tiles
static __device__ unsigned long long slant_stamps[16];
#define SLANT_STAMP(i, v) atomicAdd(&slant_stamps[i], (unsigned long long)(v))
#endif

// polls before a courier gives up (a hang guard: ~seconds; SlantCtl::err is set)
constexpr unsigned kSlantSpinLimit = 1u << 22;

// PF: steps of data loads in flight per compute wave; CR: phases of hand-off
// granule loads in flight in the courier.
//
// Memory-instruction hygiene (as the other passes): every
// load and store of the steady-state loops is unconditional -- addresses are
// clamped into the volume, inactive lanes and steps write to a dummy word --
// so hipcc's waitcnt pass keeps exact vmcnt counts and the prefetch rings stay
// in flight across steps (a data-dependent branch around any memory
// instruction makes it wait for everything outstanding).
template <int V, bool FULL, int NW, int PF, int CR>
__global__ __launch_bounds__(64 * (NW + 1)) void slant_up_kernel(SlantArgs a, Geom g) {
    __shared__ __attribute__((aligned(16))) SlantUpLds<V, NW> L;
    const int wave = wave_id(), lane = tid_x() & 63;
    const int H = g.H, W = g.W, D = g.D;
    const int e0 = lane * V;
    const bool dact = FULL || e0 < D;
    const int T = a.ntiles, total = T * a.nviews;
    const long long dstep = (long long)(W - 1) * D;  // one step up-right: -W*D + D
    if (tid_x() == 0)
        L.epoch = __hip_atomic_load(&a.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float p2v = to_vgpr(a.p2);

    for (;;) {
        __syncthreads();
        if (tid_x() == 0) L.ticket = (int)atomicAdd(&a.ctl->tickets, 1u);
        __syncthreads();
        const int r = __builtin_amdgcn_readfirstlane(L.ticket);
        const unsigned tag = __builtin_amdgcn_readfirstlane(L.epoch) + 1u;
        if (r >= total) break;
        const int view = a.nviews == 2 ? (r & 1) : 0;
        const int t = T - 1 - (a.nviews == 2 ? (r >> 1) : r);
        const SlantView &sv = a.v[view];
        const int u_lo = -(H - 1) + t * NW;
        const int s_begin = max(0, -(u_lo + NW - 1));
        const int s_end = min(H, W - u_lo);
        const int nsteps = s_end - s_begin;

        if (wave == NW) {
            // ------------------------------------------------ courier wave
            // Phase p = 0 .. nsteps (the prologue, then one per step; each
            // ends on the tile's barrier):
            //  * publishes this tile's exit states of step s_begin + p - 1
            //    (waves 0 and 1 wrote them to LDS in that step) as granules;
            //  * hands the next tile's exit states of step gs = s_begin - 1 + p
            //    to LDS parity gs & 1 (slots NW, NW+1), which step gs + 1
            //    reads.  Their granule loads run CR phases ahead; a phase
            //    re-polls only when the next tile is not that far ahead.
            auto gvalid = [&](int p) {
                return t + 1 < T && (p >= 1 || s_begin >= 1) && p < nsteps;
            };
            // granules of (tile t+1, step s_begin - 1 + p); a phase with
            // nothing to fetch loads (and ignores) tile t+1's first step, or
            // this tile's own when t + 1 == T: every load stays in the buffer
            auto gsrc = [&](int p) -> const unsigned long long * {
                const int gs = s_begin - 1 + p;
                const bool ok = gvalid(p);
                const int tt = uniform(ok ? t + 1 : t);
                const int ss = uniform(ok ? gs : s_begin);
                return sv.gran + gran_index(T, H, D, view, tt, ss, 0) + e0;
            };
            unsigned long long rq[CR][3][V];
            auto issue = [&](int slot, int p) {
                const unsigned long long *gb = gsrc(p);
#pragma unroll
                for (int x = 0; x < 3; ++x)
#pragma unroll
                    for (int v = 0; v < V; ++v)
                        rq[slot][x][v] = __hip_atomic_load(const_cast<unsigned long long *>(gb + x * D + v),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
#pragma unroll
            for (int q = 0; q < CR; ++q) issue(q, q);
            auto phase = [&](int slot, int p) {
                // 1) publish: this tile's step sp = s_begin + p - 1 (the
                // prologue phase republishes nothing new: it rewrites step
                // s_begin's slots, which step s_begin's phase overwrites)
                {
                    const int sp = uniform(p >= 1 ? s_begin + p - 1 : s_begin);
                    const int par = sp & 1;
                    float y0[V], y1[V], y2[V];
                    load_lds_v<V>(y0, &L.st[par][0][0][e0]);
                    load_lds_v<V>(y1, &L.st[par][0][1][e0]);
                    load_lds_v<V>(y2, &L.st[par][1][1][e0]);
                    unsigned long long *gb = sv.gran + gran_index(T, H, D, view, t, sp, 0) + e0;
                    if (p >= 1) {
                        store_granules<V>(gb, y0, tag);
                        store_granules<V>(gb + D, y1, tag);
                        store_granules<V>(gb + 2 * D, y2, tag);
                    }
                }
                // 2) receive tile t+1's step gs = s_begin - 1 + p
                const int gs = s_begin - 1 + p;
                const bool want = gvalid(p);
                const int c0 = u_lo + NW + gs;  // tile t+1's wave 0 column at step gs
                const bool n0 = want && c0 >= 0 && c0 < W, n1 = want && c0 + 1 >= 0 && c0 + 1 < W;
                bool ok = true;
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    ok &= !n0 || (unsigned)(rq[slot][0][v] >> 32) == tag;
                    ok &= !n0 || (unsigned)(rq[slot][1][v] >> 32) == tag;
                    ok &= !n1 || (unsigned)(rq[slot][2][v] >> 32) == tag;
                }
                if (!__all(ok || !dact)) {
                    // slow path: the next tile is not CR steps ahead
#ifdef SGM_SLANT_STAMPS
                    const long long sp0 = __builtin_amdgcn_s_memtime();
                    unsigned nsp = 0;
#endif
                    const unsigned long long *gb = sv.gran + gran_index(T, H, D, view, t + 1, gs, 0) + e0;
                    for (unsigned spins = 1;; ++spins) {
                        __builtin_amdgcn_s_sleep(1);
#pragma unroll
                        for (int x = 0; x < 3; ++x)
#pragma unroll
                            for (int v = 0; v < V; ++v)
                                rq[slot][x][v] = __hip_atomic_load(
                                    const_cast<unsigned long long *>(gb + x * D + v), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
                        ok = true;
#pragma unroll
                        for (int v = 0; v < V; ++v) {
                            ok &= !n0 || (unsigned)(rq[slot][0][v] >> 32) == tag;
                            ok &= !n0 || (unsigned)(rq[slot][1][v] >> 32) == tag;
                            ok &= !n1 || (unsigned)(rq[slot][2][v] >> 32) == tag;
                        }
#ifdef SLANT_PROBE_NOWAIT
                        ok = true;  // timing probe: no hand-off wait (wrong results)
#endif
#ifdef SGM_SLANT_STAMPS
                        nsp = spins;
#endif
                        if (__all(ok || !dact)) break;
                        if (spins >= kSlantSpinLimit) {
                            if (lane == 0) atomicOr(&a.ctl->err, 1u);
                            break;
                        }
                    }
#ifdef SGM_SLANT_STAMPS
                    if (lane == 0) {
                        SLANT_STAMP(1, 1);
                        SLANT_STAMP(2, nsp);
                        SLANT_STAMP(3, __builtin_amdgcn_s_memtime() - sp0);
                    }
#endif
                }
                // (phases with nothing wanted write slots no valid
                // predecessor reads)
                float x0[V], x1[V], x2[V];
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    x0[v] = dact ? __uint_as_float((unsigned)rq[slot][0][v]) : SGM_INF;
                    x1[v] = dact ? __uint_as_float((unsigned)rq[slot][1][v]) : SGM_INF;
                    x2[v] = dact ? __uint_as_float((unsigned)rq[slot][2][v]) : SGM_INF;
                }
                const int par = gs & 1;
                const float m0 = wave_min(lane_min(x0)), m1 = wave_min(lane_min(x1)),
                            m2 = wave_min(lane_min(x2));
                store_lds_v<V>(&L.st[par][NW][0][e0], x0);
                store_lds_v<V>(&L.st[par][NW][1][e0], x1);
                store_lds_v<V>(&L.st[par][NW + 1][1][e0], x2);
                if (lane == 0) {
                    L.pm[par][NW][0] = m0;
                    L.pm[par][NW][1] = m1;
                    L.pm[par][NW + 1][1] = m2;
                }
                issue(slot, p + CR);
                lds_barrier();
            };
            const int np = nsteps + 1;
            int p0 = 0;
            for (; p0 + CR <= np; p0 += CR) {
#pragma unroll
                for (int q = 0; q < CR; ++q) phase(q, p0 + q);
            }
#pragma unroll
            for (int q = 0; q < CR; ++q)
                if (p0 + q < np) phase(q, p0 + q);
            // the tile's last step, published after its barrier
            {
                const int sp = s_end - 1, par = sp & 1;
                float y0[V], y1[V], y2[V];
                load_lds_v<V>(y0, &L.st[par][0][0][e0]);
                load_lds_v<V>(y1, &L.st[par][0][1][e0]);
                load_lds_v<V>(y2, &L.st[par][1][1][e0]);
                unsigned long long *gb = sv.gran + gran_index(T, H, D, view, t, sp, 0) + e0;
                store_granules<V>(gb, y0, tag);
                store_granules<V>(gb + D, y1, tag);
                store_granules<V>(gb + 2 * D, y2, tag);
            }
            continue;
        }

        // ------------------------------------------------- compute waves
        const int k = wave;
        const int u = u_lo + k;
        // pixel of step s: row H-1-s, column u+s.  Steps where this wave's
        // pixel lies outside the image load a clamped (valid) pixel and
        // their results are never consumed: a valid predecessor is always
        // an active wave's pixel (DESIGN.md "Slanted tiles").
        const long long base = ((long long)(H - 1) * W + u) * D + e0;
        const int s_lo = max(s_begin, -u), s_hi = min(s_end - 1, W - 1 - u);
        const bool never = s_lo > s_hi;
        auto off_of = [&](int s) -> long long {
            const int sc = uniform(min(max(s, s_lo), s_hi));
            return never ? (long long)e0 : base - (long long)sc * dstep;
        };
        float cb[PF][V], sb[PF][V], lb[PF][V], tb[PF][V];
        int pfs = s_begin;  // step of the next ring refill
        auto refill = [&](int slot) {
            const long long o = off_of(pfs);
            load_v<V>(cb[slot], sv.cost + o, dact);
#ifndef SLANT_PROBE_NOLOADS
            load_v_nt<V>(sb[slot], sv.s12 + o, dact);
            load_v_nt<V>(lb[slot], sv.l3 + o, dact);
            load_v_nt<V>(tb[slot], sv.t56 + o, dact);
#else
            load_v<V>(sb[slot], sv.cost + o, dact);
            load_v<V>(lb[slot], sv.cost + o, dact);
            load_v<V>(tb[slot], sv.cost + o, dact);
#endif
            ++pfs;
        };
#pragma unroll
        for (int q = 0; q < PF; ++q) refill(q);
        float p7[V];
#pragma unroll
        for (int v = 0; v < V; ++v) p7[v] = 0.0f;
        float m7 = 0.0f;
        lds_barrier();  // the courier's prologue phase
#ifdef SGM_SLANT_STAMPS
        long long st_prev = __builtin_amdgcn_s_memtime(), st_work = 0, st_wait = 0;
        const long long tile_t0 = st_prev;
#endif

        auto step = [&](int q, int s) {
            const int j = u + s;
            const bool act = j >= 0 && j < W;
            const int pp = (s - 1) & 1, cp = s & 1;
            // path starts (SGM.cpp:205-214, :321-335): a zero state before the
            // first pixel makes the step yield L = C (P1, P2 >= 0)
            const bool v4 = s >= 1, v7 = s >= 1 && j >= 1, v8 = s >= 1 && j + 1 <= W - 1;
            float q4[V], q8[V], z7[V];
            load_lds_v<V>(q4, &L.st[pp][k + 1][0][e0]);
            load_lds_v<V>(q8, &L.st[pp][k + 2][1][e0]);
            // (uniform LDS words: into SGPRs, dp_step's scalar operand)
            float m4 = uni_f(L.pm[pp][k + 1][0]), m8 = uni_f(L.pm[pp][k + 2][1]);
#pragma unroll
            for (int v = 0; v < V; ++v) {
                q4[v] = v4 ? q4[v] : 0.0f;
                q8[v] = v8 ? q8[v] : 0.0f;
                z7[v] = v7 ? p7[v] : 0.0f;
            }
            m4 = v4 ? m4 : 0.0f;
            m8 = v8 ? m8 : 0.0f;
            const float mm7 = v7 ? m7 : 0.0f;
            float L4[V], L7[V], L8[V];
            dp_step<V>(q4, m4, cb[q], L4, a.p1, p2v);
            dp_step<V>(z7, mm7, cb[q], L7, a.p1, p2v);
            dp_step<V>(q8, m8, cb[q], L8, a.p1, p2v);
            const float n4 = wave_min(lane_min(L4)), n7 = wave_min(lane_min(L7)),
                        n8 = wave_min(lane_min(L8));
            float tot[V];
#pragma unroll
            for (int v = 0; v < V; ++v)
                tot[v] = ((sb[q][v] + lb[q][v]) + L4[v]) + ((tb[q][v] + L7[v]) + L8[v]);
            int d;
            float f;
#ifdef SLANT_PROBE_NOWTA
            d = 0;  // timing probe: no WTA (wrong results)
            f = tot[0];
#else
            wta_subpixel<V>(tot, D, a.uniq, d, f);
#endif
            store_lds_v<V>(&L.st[cp][k][0][e0], L4);
            store_lds_v<V>(&L.st[cp][k][1][e0], L8);
            if (lane == 0) {
                L.pm[cp][k][0] = n4;
                L.pm[cp][k][1] = n8;
            }
#pragma unroll
            for (int v = 0; v < V; ++v) p7[v] = L7[v];
            m7 = n7;
            // outputs: an inactive step writes the dummy word instead
            {
                const long long pix = (long long)(H - 1 - s) * W + j;
                float *fs = act ? sv.sub + pix : a.dummy;
                if (lane == 0) *fs = f;
                if (sv.disp) {
                    uint16_t *ds = act ? sv.disp + pix : reinterpret_cast<uint16_t *>(a.dummy + 1);
                    if (lane == 0) *ds = (uint16_t)d;
                }
            }
            refill(q);
#ifdef SGM_SLANT_STAMPS
            const long long tb0 = __builtin_amdgcn_s_memtime();
            st_work += tb0 - st_prev;
#endif
            lds_barrier();
#ifdef SGM_SLANT_STAMPS
            st_prev = __builtin_amdgcn_s_memtime();
            st_wait += st_prev - tb0;
#endif
        };
        int s0 = s_begin;
        for (; s0 + PF <= s_end; s0 += PF) {
#pragma unroll
            for (int q = 0; q < PF; ++q) step(q, s0 + q);
        }
#pragma unroll
        for (int q = 0; q < PF; ++q)
            if (s0 + q < s_end) step(q, s0 + q);
#ifdef SGM_SLANT_STAMPS
        if (k == 0 && lane == 0) {
            SLANT_STAMP(0, nsteps);
            SLANT_STAMP(4, st_work);
            SLANT_STAMP(5, st_wait);
            SLANT_STAMP(7, __builtin_amdgcn_s_memtime() - tile_t0);
            SLANT_STAMP(9, 1);
        }
#endif
    }
#ifdef SGM_SLANT_STAMPS
    if (tid_x() == 0) SLANT_STAMP(8, 1);
#endif
    // the last workgroup out resets the tickets and moves the epoch on (the
    // next launch's granule tag), so a replayed launch never reads this
    // launch's granules as its own
    if (tid_x() == 0) {
        const unsigned n = atomicAdd(&a.ctl->exits, 1u);
        if (n == (unsigned)a.grid - 1) {
            atomicExch(&a.ctl->exits, 0u);
            atomicExch(&a.ctl->tickets, 0u);
            atomicAdd(&a.ctl->epoch, 1u);
        }
    }
}

size_t slant_tiles(Geom g) { return (size_t)((g.W + g.H - 1 + kSlantNW - 1) / kSlantNW); }

size_t slant_gran_count(Geom g, int nviews) {
    return (size_t)nviews * slant_tiles(g) * g.H * 3 * g.D;
}

hipError_t launch_slant_up(const SlantArgs &a0, Geom g, hipStream_t st) {
    SlantArgs a = a0;
    a.ntiles = (int)slant_tiles(g);
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int total = a.ntiles * a.nviews;
    a.grid = total < cus ? total : cus;
    const dim3 grid(a.grid), block(64 * (kSlantNW + 1));
    if (g.D == 32) slant_up_kernel<1, false, kSlantNW, 8, 3><<<grid, block, 0, st>>>(a, g);
    else if (g.D == 64) slant_up_kernel<1, true, kSlantNW, 8, 3><<<grid, block, 0, st>>>(a, g);
    else if (g.D == 128) slant_up_kernel<2, true, kSlantNW, 8, 3><<<grid, block, 0, st>>>(a, g);
    else slant_up_kernel<4, true, kSlantNW, 4, 2><<<grid, block, 0, st>>>(a, g);
    return hipGetLastError();
}

}  // namespace sgm

#ifdef SGM_SLANT_STAMPS
extern "C" int sgm_debug_slant_stamps(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sgm::slant_stamps), sizeof(sgm::slant_stamps)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sgm::slant_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
