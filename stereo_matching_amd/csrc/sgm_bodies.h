// sgm_bodies.h -- per-path role bodies (one wavefront each) shared by the
// single-role kernels and the multi-role stage kernels (DESIGN.md "Frame
// schedule": independent roles share one launch so they run concurrently
// whatever HIP stream -> hardware queue mapping the runtime picks).
#pragma once

#include "sgm_device.h"

#include <type_traits>

namespace sgm {

// Segment length K (steps between checkpoints): seg_k_hd / seg_k_v
// (sgm_internal.h), the one definition the allocation and guards share.
template <int V>
constexpr int pair_k() { return seg_k_hd(V); }
template <int V>
constexpr int pair_kv() { return seg_k_v(V); }
template <int FAM, int V>
constexpr int family_k() { return FAM == PAIR_V ? pair_kv<V>() : pair_k<V>(); }

template <int V>
__device__ __forceinline__ float lane_min(const float (&x)[V]) {
    float m = x[0];
#pragma unroll
    for (int v = 1; v < V; ++v) m = fminf(m, x[v]);
    return m;
}

// -------------------------------------------------------- single sweeps

// One direction over one path, one wavefront; lane l holds disparities
// l*V .. l*V+V-1 (FULL: all 64 lanes hold data, i.e. D >= 64; D = 32 uses
// lanes 0..31 and +inf above).  Loads run PF steps ahead of the DP through a
// register ring.  Modes STORE_L / INIT / ACC (the final sweep has its own
// two-wave kernel).
#ifdef SGM_STAMPS
// per role (0-2 final producer/consumer/WTA, 3-4 H producer/consumer):
// work cycles, barrier-wait cycles, waves
static __device__ unsigned long long sgm_stamps[16][3];  // one copy per translation unit
__device__ __forceinline__ void stamp_flush(int role, long long t0) {
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((tid_x() & 63) == 0) {
        atomicAdd(&sgm_stamps[role][0], (unsigned long long)(t1 - t0));
        atomicAdd(&sgm_stamps[role][2], 1ull);
    }
}
#endif

// BAND: a.band's steps only (the backward diagonals DIR 6 / 7 of the
// backward bands, L5 (DIR 4) of the forward bands)
template <int DIR, int V, int MODE, bool FULL, int PF, bool BAND = false>
__device__ __forceinline__ void sweep_body(const SweepArgs &a, const Geom &g, int path) {
    static_assert(MODE != SWEEP_FINAL, "the final pass is pair_final_kernel");
#ifdef SGM_STAMPS
    const long long st_t0 = __builtin_amdgcn_s_memtime();
#endif
    const float p2v = to_vgpr(a.p2);  // dp_step's P2 operand
    const int lane = tid_x() & 63;
    const int H = g.H, W = g.W;
    const long long D = g.D, WD = (long long)g.W * g.D;
    const int n = DIR < 2 ? W : H;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;
    constexpr bool NEED_ACC = MODE == SWEEP_ACC;
    static_assert(!BAND || DIR >= 4, "bands of diagonal sweeps");
    constexpr bool BANDED = BAND;
    const int kb = BANDED ? a.band.kb : 0;
    const int ke = BANDED && a.band.ke > 0 ? a.band.ke : n;

    Cursor<DIR> cc, pc;
    if (BANDED) {
        cc.init_at(path, kb, H, W, g.D);
        pc.init_at(path, kb, H, W, g.D);
    } else {
        cc.init(path, H, W, g.D);
        pc.init(path, H, W, g.D);
    }

    float cb[PF][V], ab[PF][V];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        load_v<V>(cb[u], a.cost + pc.off + e0, active);
        if (NEED_ACC) load_v_nt<V>(ab[u], a.acc_in + pc.off + e0, active);
        pc.advance_upto(ke, W, D, WD);
    }

    float prev[V];
    float pmin = 0.0f;
    if (BANDED && kb > 0) {  // the chain state entering the band
        load_v<V>(prev, a.band.carry + (size_t)path * g.D + e0, active);
        pmin = wave_min(lane_min(prev));
    } else {
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = SGM_INF;
    }

    // One DP step on ring slot u; branch-free so the waitcnt pass can keep
    // exact counts (each slot's loads are waited for PF steps later).
    auto step = [&](int u, bool refill) {
        float c[V], ai[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            c[v] = cb[u][v];
            ai[v] = ab[u][v];
        }
        float L[V];
        dp_step<V>(prev, pmin, c, L, a.p1, p2v);
        const bool st = cc.start(W);
#pragma unroll
        for (int v = 0; v < V; ++v) L[v] = st ? c[v] : L[v];
        float lm = L[0];
#pragma unroll
        for (int v = 1; v < V; ++v) lm = fminf(lm, L[v]);
        const float nmin = wave_min(lm);

        if constexpr (MODE == SWEEP_STORE_L) {
            store_v_nt<V>(a.acc_out + cc.off + e0, L, active);
            if (lane == 0) a.min_out[cc.off / D] = nmin;
        } else if constexpr (MODE == SWEEP_INIT) {
            store_v_nt<V>(a.acc_out + cc.off + e0, L, active);
        } else {
            float o[V];
#pragma unroll
            for (int v = 0; v < V; ++v) o[v] = ai[v] + L[v];
            store_v_nt<V>(a.acc_out + cc.off + e0, o, active);
        }
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = L[v];
        pmin = nmin;
        cc.advance(W, D, WD);
        if (refill) {
            // refill this ring slot only after its old contents are dead, so
            // the new load lands in the same registers (no copy, no wait)
            load_v<V>(cb[u], a.cost + pc.off + e0, active);
            if (NEED_ACC) load_v_nt<V>(ab[u], a.acc_in + pc.off + e0, active);
            pc.advance_upto(ke, W, D, WD);
        }
    };

    int k0 = kb;
    for (; k0 + PF <= ke; k0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) step(u, true);
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (k0 + u < ke) step(u, false);
    if (BANDED && ke < n) store_v<V>(a.band.carry + (size_t)path * g.D + e0, prev, active);
#ifdef SGM_STAMPS
    stamp_flush(DIR == 4 ? 8 : (DIR == 7 ? 9 : 10), st_t0);
#endif
}

// A diagonal cursor on the VALU: the same walk as Cursor<DIR> (wrapped
// diagonals), with the column and offset held in VGPRs (wave-uniform values
// the compiler is kept from moving to SGPRs).
template <int DIR>
struct VCursor {
    int j, k;
    long long off;
    __device__ __forceinline__ void init(int path, int H, int W, int D, int lane) {
        int z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // an opaque per-lane zero
        (void)lane;
        k = z;
        j = path + z;
        const int i = (DIR == 4 || DIR == 5) ? 0 : H - 1;
        off = ((long long)i * W + j) * D;
    }
    __device__ __forceinline__ void advance(int W, long long D, long long WD) {
        ++k;
        if constexpr (DIR == 4 || DIR == 6) {
            const bool wrap = j == W - 1;
            off += (DIR == 4 ? WD : -WD) + (wrap ? -(long long)(W - 1) * D : D);
            j = wrap ? 0 : j + 1;
        } else {
            const bool wrap = j == 0;
            off += (DIR == 5 ? WD : -WD) + (wrap ? (long long)(W - 1) * D : -D);
            j = wrap ? W - 1 : j - 1;
        }
    }
    // advance only while k < n-1 (the load cursor stops on the last pixel)
    __device__ __forceinline__ void advance_upto(int n, int W, long long D, long long WD) {
        VCursor nx = *this;
        nx.advance(W, D, WD);
        const bool go = k < n - 1;
        j = go ? nx.j : j;
        off = go ? nx.off : off;
        k = go ? nx.k : k;
    }
};

// ------------------------------------------------- split diagonal sweeps
//
// The same sweep (diagonal DIR 4-7, MODE INIT or ACC) on two waves of one
// workgroup: wave 0 moves memory -- the cost and accumulator rows of block
// b+1 are loaded while block b is computed, written to an LDS ring, and the
// results of block b-2 go back to global memory -- and wave 1 runs only the
// DP, reading its inputs from and writing its outputs to LDS.  One LDS
// barrier per block of BK steps.  A single wave interleaving the DP chain
// with its own loads and stores reached 85% of the memory-only rate of the
// same walk; the split reaches ~100% (tools/layout_probe.hip).
template <int V, int BK>
struct SweepSplitLds {
    float c[3][BK][64 * V];  // costs
    float a[3][BK][64 * V];  // acc_in rows (ACC)
    float o[3][BK][64 * V];  // results
};

template <int DIR, int V, int MODE, bool FULL, int BK>
__device__ __forceinline__ void sweep_split_body(const SweepArgs &a, const Geom &g, int path,
                                                 SweepSplitLds<V, BK> &L) {
    static_assert(DIR >= 4 && (MODE == SWEEP_INIT || MODE == SWEEP_ACC), "diagonal INIT/ACC sweeps");
    constexpr bool NEED_ACC = MODE == SWEEP_ACC;
    const int wave = wave_id();
    const int lane = tid_x() & 63;
    const int H = g.H, W = g.W;
    const long long D = g.D, WD = (long long)g.W * g.D;
    const int n = H;
    const int nb = (n + BK - 1) / BK;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;
    if (wave == 0) {
        // ------------------------------------------------------ memory wave
        // Addresses walk on the VALU (this wave's vector pipe is otherwise
        // idle; scalar cursors here would compete with the DP waves' scalar
        // work): VCursor keeps the column and the offset in VGPRs.
        VCursor<DIR> pc, sc;  // next load, next store
        pc.init(path, H, W, g.D, lane);
        sc.init(path, H, W, g.D, lane);
        float lc[BK][V], la[BK][V];
        auto issue = [&] {
#pragma unroll
            for (int u = 0; u < BK; ++u) {
                load_v<V>(lc[u], a.cost + pc.off + e0, active);
                if (NEED_ACC) load_v_nt<V>(la[u], a.acc_in + pc.off + e0, active);
                pc.advance_upto(n, W, D, WD);
            }
        };
        issue();
        for (int it = 0; it < nb + 2; ++it) {
            if (it >= 2) {  // block it-2's results (written by the DP wave in iteration it-1)
                const int b = it - 2;
#pragma unroll
                for (int u = 0; u < BK; ++u) {
                    if (b * BK + u < n) {
                        float o[V];
                        load_lds_v<V>(o, &L.o[b % 3][u][e0]);
                        store_v_nt<V>(a.acc_out + sc.off + e0, o, active);
                        sc.advance(W, D, WD);
                    }
                }
            }
            if (it < nb) {
#pragma unroll
                for (int u = 0; u < BK; ++u) {
                    store_lds_v<V>(&L.c[it % 3][u][e0], lc[u]);
                    if (NEED_ACC) store_lds_v<V>(&L.a[it % 3][u][e0], la[u]);
                }
                if (it + 1 < nb) issue();
            }
            lds_barrier();
        }
    } else {
        // --------------------------------------------------------- DP wave
        __builtin_amdgcn_s_setprio(3);
        const float p2v = to_vgpr(a.p2);
        // the next step at which the wrapped chain meets the image edge and
        // restarts (Cursor::start: DIR 4/6 wrap to column 0, DIR 5/7 to column
        // W-1), then every W steps (frames taller than wide wrap repeatedly)
        int kw = (DIR == 4 || DIR == 6) ? W - path : path + 1;
        float prev[V];
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = SGM_INF;
        float pmin = 0.0f;
        for (int it = 0; it < nb + 2; ++it) {
            if (it >= 1 && it - 1 < nb) {
                const int b = it - 1;
                // steps past the chain's end (the last block's tail) run on
                // stale LDS slots; their results are never stored
#pragma unroll
                for (int u = 0; u < BK; ++u) {
                    const int k = b * BK + u;
                    {
                        float c[V], ai[V], Lr[V];
                        load_lds_v<V>(c, &L.c[b % 3][u][e0]);
                        if (NEED_ACC) load_lds_v<V>(ai, &L.a[b % 3][u][e0]);
                        dp_step<V>(prev, pmin, c, Lr, a.p1, p2v);
                        const bool st = k == 0 || k == kw;
                        kw = uniform(k == kw ? kw + W : kw);
#pragma unroll
                        for (int v = 0; v < V; ++v) Lr[v] = st ? c[v] : Lr[v];
                        pmin = wave_min(lane_min(Lr));
                        float o[V];
#pragma unroll
                        for (int v = 0; v < V; ++v) o[v] = NEED_ACC ? ai[v] + Lr[v] : Lr[v];
                        store_lds_v<V>(&L.o[b % 3][u][e0], o);
#pragma unroll
                        for (int v = 0; v < V; ++v) prev[v] = Lr[v];
                    }
                }
            }
            lds_barrier();
        }
    }
}

// --------------------------------------------------------------- pairs
//
// Two opposite directions on the same scanlines (L1/L2 rows, L3/L4 columns,
// L6/L7 wrapped anti-diagonals): the forward body stores its path state every
// K steps, the backward body recomputes each K-step segment of the forward
// costs from its checkpoint in registers (each cost is read once for both)
// and combines  S12 = L1 + L2,  T = (T5 + L6) + L7,  total = ((S12+L3)+L4)+T
// on the fly in the reference's association order (SGM.cpp:386-390).
// Segments are counted from the END of a chain of n steps: segment 0 covers
// [0, r0) with r0 = n - (nseg-1)*K, segment s >= 1 covers [r0+(s-1)K, r0+sK);
// checkpoint m (m < nseg-1) is the forward state after position r0-1 + mK and
// seeds segment m+1, so the backward pass meets full segments first.

// ------------------------------------------------------- forward passes

// Forward direction FD (0 = L1, 2 = L3, 5 = L6) over one chain: the DP of
// SGM.cpp:93-117 with the cost stream prefetched PF steps ahead; the only
// output is the checkpoint set.
// BAND (FD 5, the forward bands above the Infinity Cache): steps [kb, ke)
// of the chain, whole segments (kb, ke = r0 mod K, or ke = n), the state
// entering the band from a.band.carry and the state leaving it stored there.
template <int FD, int V, bool FULL, int PF, bool BAND = false, bool NTC = false>
__device__ __forceinline__ void pair_fwd_body(const PairArgs &a, const Geom &g, int path) {
#ifdef SGM_STAMPS
    const long long st_t0 = __builtin_amdgcn_s_memtime();
#endif
    constexpr int K = family_k<FD == 0 ? PAIR_H : (FD == 2 ? PAIR_V : PAIR_D2), V>();
    static_assert(PF % K == 0, "the ring covers whole checkpoint segments");
    constexpr bool DIAG = FD == 5;
    const float p2v = to_vgpr(a.p2);  // dp_step's P2 operand
    const int lane = tid_x() & 63;
    const int H = g.H, W = g.W;
    const long long D = g.D, WD = (long long)g.W * g.D;
    const int n = FD == 0 ? W : H;
    const int nseg = (n + K - 1) / K;
    const int r0 = n - (nseg - 1) * K;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;
    float *ck = a.ckpt + (size_t)path * nseg * g.D + e0;

    // The chain is walked from a virtual start vs = K - r0 steps before
    // position 0 so that checkpoint m (the state after position r0-1 + mK)
    // falls on the last step of every K-step block: the stores sit at fixed
    // places in the unrolled loop, with no branch.  Virtual positions read
    // zero costs from a.zero; with the state starting at L = 0, minL = 0 a
    // step on a zero cost keeps it at 0 (P1, P2 >= 0), and the first real step
    // then yields L = C, the reference's path start (SGM.cpp:93-98).  Block
    // nseg-1 stores into the unused last slot.
    const int vs = K - r0;
    static_assert(!BAND || FD == 5, "bands of the forward diagonal");
    const int kb = BAND ? a.band.kb : 0;
    const int ke = BAND && a.band.ke > 0 ? a.band.ke : n;
    // the first position walked: the virtual start, or the band's first step
    const int s0 = kb > 0 ? kb : -vs;
    Cursor<FD> cc, pc;
    if (BAND && kb > 0) {
        cc.init_at(path, kb, H, W, g.D);
        pc.init_at(path, kb, H, W, g.D);
    } else {
        cc.init(path, H, W, g.D);
        pc.init(path, H, W, g.D);
    }
    int ppos = s0;  // position of the next ring refill
    // rows (FD 0): a plain running pointer; positions past the row's end read
    // the next row or the volume guard (kVolGuard) and are never consumed
    const float *hrow = a.cost + (size_t)path * W * g.D;
    auto fetch = [&](float (&dst)[V]) {
        if constexpr (FD == 0) {
            const float *src = ppos >= 0 ? hrow + (size_t)ppos * g.D : a.zero;
            if constexpr (NTC) load_v_nt<V>(dst, src + e0, active);
            else load_v<V>(dst, src + e0, active);
        } else {
            const float *src = ppos >= 0 ? a.cost + pc.off : a.zero;
            load_v<V>(dst, src + e0, active);
            pc.advance_if(ppos >= 0 && pc.k < n - 1, W, D, WD);
        }
        ++ppos;
    };
    float cb[PF][V];
#pragma unroll
    for (int u = 0; u < PF; ++u) fetch(cb[u]);
    // in the main loop every refill position is >= PF - vs > 0
    const float *hnext = hrow + (size_t)ppos * g.D + e0;
    auto refetch = [&](float (&dst)[V]) {
        if constexpr (FD == 0) {
            if constexpr (NTC) load_v_nt<V>(dst, hnext, active);
            else load_v<V>(dst, hnext, active);
            hnext += g.D;
        } else {
            fetch(dst);
        }
    };
    float prev[V];
    float pmin = 0.0f;
    if (BAND && kb > 0) {  // the chain state entering the band
        load_v<V>(prev, a.band.carry + (size_t)path * g.D + e0, active);
        pmin = wave_min(lane_min(prev));
    } else {
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = 0.0f;
    }
    int cpos = s0;  // position of the next step

    auto step = [&](int u, bool refill) {
        float L[V];
        dp_step<V>(prev, pmin, cb[u], L, a.p1, p2v);
        if constexpr (DIAG) {
            // a wrapped diagonal restarts where it meets the image edge
            const bool st = cpos > 0 && cc.start(W);
#pragma unroll
            for (int v = 0; v < V; ++v) L[v] = st ? cb[u][v] : L[v];
        }
        const float nmin = wave_min(lane_min(L));
        if (u % K == K - 1) store_v<V>(ck + (size_t)((cpos - r0 + 1) / K) * g.D, L, active);
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = L[v];
        pmin = nmin;
        if constexpr (DIAG) cc.advance_if(cpos >= 0, W, D, WD);
        ++cpos;
        // Rows (FD 0) refill the ring in bursts of RB slots: every RB-th step
        // reloads the RB slots consumed since the last burst, one contiguous
        // RB * D-float block of the row (K128 stage A -2.5%, the frame
        // -0.6..-0.8% paired; HD/4K unchanged; diagonals in bursts were
        // slower: profiles/r06_experiments/r06t_row_bursts.txt)
        constexpr int RB = FD == 0 ? 8 : 1;
        static_assert(PF % RB == 0, "bursts of whole ring slots");
        if (refill && u % RB == RB - 1) {
#pragma unroll
            for (int q = RB - 1; q >= 0; --q) refetch(cb[u - q]);
        }
    };
    const int total = ke - s0;  // nseg * K for the whole chain
    int k0 = 0;
    for (; k0 + PF <= total; k0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) step(u, true);
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (k0 + u < total) step(u, false);
    if (BAND && ke < n) store_v<V>(a.band.carry + (size_t)path * g.D + e0, prev, active);
#ifdef SGM_STAMPS
    stamp_flush(FD == 0 ? 5 : (FD == 5 ? 6 : 7), st_t0);
#endif
}

// ------------------------------------------------------- backward pass

// tb/pb: the FINAL mode's LDS ring (two chunks of K total-cost rows and
// pixel positions), unused otherwise.
template <int FAM, int V, bool FULL, int MODE, bool BAND = false, bool NTC = false>
__device__ __forceinline__ void pair_bwd_body(const PairArgs &a, const Geom &g, int path,
                                              float (*tb)[family_k<FAM, V>()][tbuf_stride<V>()],
                                              long long (*pb)[family_k<FAM, V>()]) {
#ifdef SGM_STAMPS
    const long long st_t0 = __builtin_amdgcn_s_memtime();
#endif
    constexpr int FD = FAM == PAIR_H ? 0 : (FAM == PAIR_V ? 2 : 5);
    constexpr int BD = FAM == PAIR_H ? 1 : (FAM == PAIR_V ? 3 : 6);
    constexpr int K = family_k<FAM, V>();
    constexpr bool FINAL = MODE == PAIR_FINAL;
    constexpr bool NEED_ACC = MODE != PAIR_INIT2;
    constexpr bool NEED_S = FINAL;
    const int wave = wave_id();
    const float p2v = to_vgpr(a.p2);  // dp_step's P2 operand
    const int lane = tid_x() & 63;
    const int H = g.H, W = g.W;
    const long long D = g.D, WD = (long long)g.W * g.D;
    const int n = FAM == PAIR_H ? W : H;
    const int nseg = (n + K - 1) / K;
    const int r0 = n - (nseg - 1) * K;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;
    // band (PAIR_D2 ACC, the frame schedule's stage B): backward steps
    // [kb, ke) = segments s_lo .. s_hi (backward step block c is segment
    // nseg-1-c)
    static_assert(!BAND || (FAM == PAIR_D2 && MODE == PAIR_ACC), "bands of the diagonal pair");
    constexpr bool BANDED = BAND;
    const int kb = BANDED ? a.band.kb : 0;
    const int ke = BANDED && a.band.ke > 0 ? a.band.ke : n;
    const int s_hi = nseg - 1 - kb / K, s_lo = nseg - (ke + K - 1) / K;

    if constexpr (FINAL) {
        if (wave == 1) {  // WTA consumer, one chunk per segment
            lds_barrier();
            for (int c = 0; c < nseg; ++c) {
                wta_consume_chunk<V, K>(tb[c & 1], pb[c & 1], c == nseg - 1 ? r0 : K, lane,
                                        g.D, a.uniq, a.disp, a.sub);
                lds_barrier();
            }
            return;
        }
    }

    // the backward direction walks the same chain in reverse: for the wrapped
    // anti-diagonals chain g of L6 is chain (g - (H-1)) mod W of L7
    const int bpath = FAM == PAIR_D2 ? uniform(((path - (H - 1)) % W + W) % W) : path;
    const float *ck = a.ckpt + (size_t)path * nseg * g.D + e0;

    Cursor<BD> bc, pc;
    if (BANDED) {
        bc.init_at(bpath, kb, H, W, g.D);
        pc.init_at(bpath, kb, H, W, g.D);
    } else {
        bc.init(bpath, H, W, g.D);
        pc.init(bpath, H, W, g.D);
    }
    float ab[K][V], sb[K][V];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        if (NEED_ACC) load_v_nt<V>(ab[u], a.acc_in + pc.off + e0, active);
        if (NEED_S) load_v_nt<V>(sb[u], a.s_in + pc.off + e0, active);
        pc.advance_upto(ke, W, D, WD);
    }

    float c0[K + 1][V], c1[K + 1][V], lf[K][V];
    float prevb[V];
    float pminb = 0.0f;
    if (BANDED && kb > 0) {  // the chain state entering the band
        load_v<V>(prevb, a.band.carry + (size_t)path * g.D + e0, active);
        pminb = wave_min(lane_min(prevb));
    } else {
#pragma unroll
        for (int v = 0; v < V; ++v) prevb[v] = SGM_INF;
    }

    // costs of segment s into cs; array slot kk holds position
    // pos0 + kk - (K - cnt) (slots below K - cnt are unused for the partial
    // segment and load position pos0 again)
    auto load_seg = [&](float (&cs)[K + 1][V], int s) {
        const int cnt = s == 0 ? r0 : K;
        const int pos0 = s == 0 ? 0 : r0 + (s - 1) * K;
        Cursor<FD> fc;
        fc.init_at(path, pos0, H, W, g.D);
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
            if constexpr (NTC) load_v_nt<V>(cs[kk], a.cost + fc.off + e0, active);
            else load_v<V>(cs[kk], a.cost + fc.off + e0, active);
            fc.advance_if(kk >= K - cnt && fc.k < n - 1, W, D, WD);
        }
        // slot K: the checkpoint seeding the segment, fetched with its costs
        // so recomputation never waits on a load younger than the look-ahead
        load_v<V>(cs[K], ck + (size_t)(s > 0 ? s - 1 : 0) * g.D, active);
    };

    auto process_seg = [&](float (&cs)[K + 1][V], int s, auto full_tag) {
        constexpr bool FULLSEG = decltype(full_tag)::value;
        const int cnt = FULLSEG ? K : (s == 0 ? r0 : K);
        const int pos0 = s == 0 ? 0 : r0 + (s - 1) * K;
        const int skip = K - cnt;
        // 1) recompute the forward costs of this segment from its checkpoint
        float pf[V];
        float pminf = 0.0f;
        if constexpr (FULLSEG) {  // s >= 1
#pragma unroll
            for (int v = 0; v < V; ++v) pf[v] = cs[K][v];
            pminf = wave_min(lane_min(pf));
        } else {  // segment 0 starts the chain
#pragma unroll
            for (int v = 0; v < V; ++v) pf[v] = SGM_INF;
        }
        Cursor<FD> fc;
        fc.init_at(path, pos0, H, W, g.D);
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
            if (FULLSEG || kk >= skip) {
                float L[V];
                dp_step<V>(pf, pminf, cs[kk], L, a.p1, p2v);
                const bool st = fc.start(W);
#pragma unroll
                for (int v = 0; v < V; ++v) L[v] = st ? cs[kk][v] : L[v];
                pminf = wave_min(lane_min(L));
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    lf[kk][v] = L[v];
                    pf[v] = L[v];
                }
                fc.advance(W, D, WD);
            }
        }
        // 2) backward direction over the segment, combined on the fly
        const int buf = (nseg - 1 - s) & 1;
#pragma unroll
        for (int r = 0; r < K; ++r) {
            const int kk = K - 1 - r;
            if (FULLSEG || kk >= skip) {
                float L[V];
                dp_step<V>(prevb, pminb, cs[kk], L, a.p1, p2v);
                const bool st = bc.start(W);
#pragma unroll
                for (int v = 0; v < V; ++v) L[v] = st ? cs[kk][v] : L[v];
                const float nmin = wave_min(lane_min(L));
                if constexpr (MODE == PAIR_INIT2) {
                    float o[V];
#pragma unroll
                    for (int v = 0; v < V; ++v) o[v] = lf[kk][v] + L[v];
                    store_v_nt<V>(a.out + bc.off + e0, o, active);
                } else if constexpr (MODE == PAIR_ACC) {
                    float o[V];
#pragma unroll
                    for (int v = 0; v < V; ++v) o[v] = (ab[r][v] + lf[kk][v]) + L[v];
                    store_v_nt<V>(a.out + bc.off + e0, o, active);
                } else if constexpr (FINAL) {
                    float tot[V];
#pragma unroll
                    for (int v = 0; v < V; ++v) tot[v] = ((sb[r][v] + lf[kk][v]) + L[v]) + ab[r][v];
                    store_lds_v<V>(&tb[buf][r][e0], tot);
                    if (lane == 0) pb[buf][r] = (long long)bc.i * W + bc.j;
                }
#pragma unroll
                for (int v = 0; v < V; ++v) prevb[v] = L[v];
                pminb = nmin;
                bc.advance(W, D, WD);
                if (NEED_ACC) load_v_nt<V>(ab[r], a.acc_in + pc.off + e0, active);
                if (NEED_S) load_v_nt<V>(sb[r], a.s_in + pc.off + e0, active);
                pc.advance_upto(ke, W, D, WD);
            }
        }
        if (FINAL) lds_barrier();
    };

    // Full segments two at a time (branch-free bodies keep the wait counts
    // exact, so each segment's cost loads stay in flight during the previous
    // segment), then segment 0, which may be partial.
    using full_t = std::integral_constant<bool, true>;
    using part_t = std::integral_constant<bool, false>;
    // (a band ending above segment 0 ends on a full segment)
    auto last = [&](float (&cs)[K + 1][V]) {
        if (s_lo == 0) process_seg(cs, 0, part_t{});
        else process_seg(cs, s_lo, full_t{});
    };
    load_seg(c0, s_hi);
    int s = s_hi;
    for (; s >= s_lo + 2; s -= 2) {
        load_seg(c1, s - 1);
        process_seg(c0, s, full_t{});
        load_seg(c0, s - 2);
        process_seg(c1, s - 1, full_t{});
    }
    if (s == s_lo + 1) {
        load_seg(c1, s_lo);
        process_seg(c0, s_lo + 1, full_t{});
        last(c1);
    } else {
        last(c0);
    }
    if (BANDED && ke < n) store_v<V>(a.band.carry + (size_t)path * g.D + e0, prevb, active);
    if (FINAL) lds_barrier();
#ifdef SGM_STAMPS
    stamp_flush(FAM == PAIR_D2 ? 11 : (FAM == PAIR_H ? 13 : 14), st_t0);
#endif
}

// ------------------------------------------------- split pair backward
//
// The same backward pass with its two serial chains on two waves of one
// workgroup: wave 0 (producer) recomputes each forward segment from its
// checkpoint and writes the segment's costs and forward path costs to a
// double-buffered LDS ring; wave 1 (consumer) runs the backward direction over
// the previous segment and combines (INIT2 / ACC: stores the volume; FINAL:
// writes total-cost rows to a second LDS ring that wave 2 turns into WTA
// results).  One serial chain per wave: the pair costs one chain latency.
//
// Barrier schedule (every wave runs nseg + NW - 1 LDS barriers): in
// iteration t the producer fills chunk t, the consumer drains chunk t-1 and
// the WTA wave chunk t-2 (chunk c = segment nseg-1-c).

template <int K, int V>
struct SplitLds {
    float c[2][K][tbuf_stride<V>()];    // segment costs
    float l[2][K][tbuf_stride<V>()];    // recomputed forward path costs
};

template <int K, int V>
struct SplitFinalLds {
    SplitLds<K, V> s;
    float t[2][K][tbuf_stride<V>()];    // total costs for the WTA wave
    long long p[2][K];                  // their pixel positions
};

// NB: register buffers of segment costs in the producer (NB-1 segments of
// loads in flight while one is recomputed); RH: the consumer's ring of
// accumulator loads is RH*K steps deep (chunks processed RH at a time).
template <int FAM, int V, bool FULL, int MODE, int K, int NB = 2, int RH = 1, int NWTA = 1,
          bool BAND = false, bool NTC = false>
__device__ __forceinline__ void pair_split_body(const PairArgs &a, const Geom &g, int path,
                                                int wave, SplitLds<K, V> &L,
                                                SplitFinalLds<K, V> *F) {
#ifdef SGM_STAMPS
    long long st_prev = __builtin_amdgcn_s_memtime(), st_work = 0, st_wait = 0;
    auto bar = [&] {
        const long long t0 = __builtin_amdgcn_s_memtime();
        lds_barrier();
        const long long t1 = __builtin_amdgcn_s_memtime();
        st_work += t0 - st_prev;
        st_wait += t1 - t0;
        st_prev = t1;
    };
#else
    auto bar = [] { lds_barrier(); };
#endif

    static_assert(NB == 2 || NB == 3, "producer buffers");
    static_assert(RH == 1 || RH == 2, "consumer ring halves");
    // the final pass's WTA loads reach K-1 rows above row 0 of T: the guard
    // allocated before T (t_guard_rows, sgm_capi.hip) must cover them
    static_assert(MODE != PAIR_FINAL || K - 1 <= t_guard_rows(V == 4 ? 256 : (V == 2 ? 128 : 64)),
                  "T guard rows");
    constexpr int FD = FAM == PAIR_H ? 0 : (FAM == PAIR_V ? 2 : 5);
    constexpr int BD = FAM == PAIR_H ? 1 : (FAM == PAIR_V ? 3 : 6);
    constexpr bool FINAL = MODE == PAIR_FINAL;
    constexpr int NSTAGE = FINAL ? 3 : 2;  // pipeline stages (WTA waves share stage 3)
    // FINAL: the backward wave streams S12 through its ring and the WTA wave
    // adds T last (total = ((S12 + L3) + L4) + T), so each of the three waves
    // keeps one stream in flight
    constexpr bool NEED_ACC = MODE == PAIR_ACC;
    constexpr bool NEED_S = FINAL;
    const float p2v = to_vgpr(a.p2);  // dp_step's P2 operand
    const int lane = tid_x() & 63;
    const int H = g.H, W = g.W;
    const long long D = g.D, WD = (long long)g.W * g.D;
    const int n = FAM == PAIR_H ? W : H;
    const int nseg = (n + K - 1) / K;
    const int r0 = n - (nseg - 1) * K;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;
    using full_t = std::integral_constant<bool, true>;
    using part_t = std::integral_constant<bool, false>;
    // Rows and columns (LIN) are addressed by a base and a stride; a path
    // starts only at position 0, handled by a zero initial state (L = 0,
    // minL = 0 makes the first step yield L = C, P1, P2 >= 0).  Wrapped
    // diagonals keep the cursor and the per-step restart select.
    constexpr bool LIN = FAM != PAIR_D2;
    const long long lin_base = FAM == PAIR_H ? (long long)path * WD : (long long)path * D;
    const long long lin_st = FAM == PAIR_H ? D : WD;
    // band (PAIR_V): backward steps [kb, ke) = chunks [c_lo, c_hi) = segments
    // s_lo .. s_hi (chunk c is segment nseg-1-c)
    static_assert(!BAND || FAM == PAIR_V, "bands of the final pass");
    constexpr bool BANDED = BAND;
    const int kb = BANDED ? a.band.kb : 0;
    const int ke = BANDED && a.band.ke > 0 ? a.band.ke : n;
    const int c_lo = kb / K, c_hi = (ke + K - 1) / K;
    const int s_hi = nseg - 1 - c_lo, s_lo = nseg - c_hi;

    if (wave == 0) {
        // H rows: the recompute chain is the slower one; V: the backward one
        __builtin_amdgcn_s_setprio(FAM == PAIR_H ? 3 : 2);
        // ---------------------------------------------------- producer
        const float *ck = a.ckpt + (size_t)path * nseg * g.D + e0;
        float cb[NB][K + 1][V];
        // segment s (clamped at 0: look-ahead past the last segment reloads
        // segment 0 into a buffer nobody reads, keeping the loop branch-free);
        // slot K holds the checkpoint seeding the segment, fetched with its
        // costs so recomputation never waits on a load younger than the
        // look-ahead
        auto load_seg = [&](float (&cs)[K + 1][V], int s) {
            s = s < s_lo ? s_lo : s;
            const int cnt = s == 0 ? r0 : K;
            const int pos0 = s == 0 ? 0 : r0 + (s - 1) * K;
            if constexpr (LIN) {
                // slot kk holds position pos0 + max(kk - (K - cnt), 0)
                const float *p0 = a.cost + lin_base + (long long)pos0 * lin_st + e0;
                const int sh = K - cnt;
#pragma unroll
                for (int kk = 0; kk < K; ++kk) {
                    const int rel = kk - sh > 0 ? kk - sh : 0;
                    if constexpr (NTC) load_v_nt<V>(cs[kk], p0 + (long long)rel * lin_st, active);
                    else load_v<V>(cs[kk], p0 + (long long)rel * lin_st, active);
                }
            } else {
                Cursor<FD> fc;
                fc.init_at(path, pos0, H, W, g.D);
#pragma unroll
                for (int kk = 0; kk < K; ++kk) {
                    load_v<V>(cs[kk], a.cost + fc.off + e0, active);
                    fc.advance_if(kk >= K - cnt && fc.k < n - 1, W, D, WD);
                }
            }
            load_v<V>(cs[K], ck + (size_t)(s > 0 ? s - 1 : 0) * g.D, active);
        };
        auto produce = [&](float (&cs)[K + 1][V], int s, auto full_tag) {
            constexpr bool FULLSEG = decltype(full_tag)::value;
            const int cnt = FULLSEG ? K : (s == 0 ? r0 : K);
            const int pos0 = s == 0 ? 0 : r0 + (s - 1) * K;
            const int skip = K - cnt;
            const int buf = (nseg - 1 - s) & 1;
            float pf[V];
            float pminf = 0.0f;
            if constexpr (FULLSEG) {  // s >= 1
#pragma unroll
                for (int v = 0; v < V; ++v) pf[v] = cs[K][v];
                pminf = wave_min(lane_min(pf));
            } else {  // segment 0 starts the chain
#pragma unroll
                for (int v = 0; v < V; ++v) pf[v] = LIN ? 0.0f : SGM_INF;
            }
            Cursor<FD> fc;
            if constexpr (!LIN) fc.init_at(path, pos0, H, W, g.D);
#pragma unroll
            for (int kk = 0; kk < K; ++kk) {
                if (FULLSEG || kk >= skip) {
                    float Lr[V];
                    dp_step<V>(pf, pminf, cs[kk], Lr, a.p1, p2v);
                    if constexpr (!LIN) {
                        const bool st = fc.start(W);
#pragma unroll
                        for (int v = 0; v < V; ++v) Lr[v] = st ? cs[kk][v] : Lr[v];
                    }
                    pminf = wave_min(lane_min(Lr));
                    store_lds_v<V>(&L.c[buf][kk][e0], cs[kk]);
                    store_lds_v<V>(&L.l[buf][kk][e0], Lr);
#pragma unroll
                    for (int v = 0; v < V; ++v) pf[v] = Lr[v];
                    if constexpr (!LIN) fc.advance(W, D, WD);
                }
            }
            bar();
        };
        // buffer u holds segment s_hi-m for m = u (mod NB)
#pragma unroll
        for (int u = 0; u + 1 < NB; ++u) load_seg(cb[u], s_hi - u);
        int s = s_hi;
        // full segments NB at a time, each step first issuing the segment
        // NB-1 further down
        for (; s - (NB - 1) >= s_lo + 1; s -= NB) {
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                load_seg(cb[(u + NB - 1) % NB], s - u - (NB - 1));
                produce(cb[u], s - u, full_t{});
            }
        }
        // fewer than NB segments left (s + 1 of them, the last partial)
        auto tail = [&](auto u_tag) {
            constexpr int U = decltype(u_tag)::value;
            if constexpr (U < NB) {
                if (s >= s_lo + 1) {
                    load_seg(cb[(U + NB - 1) % NB], s - (NB - 1));
                    produce(cb[U], s, full_t{});
                    --s;
                }
            }
        };
        tail(std::integral_constant<int, 0>{});
        if constexpr (NB == 3) tail(std::integral_constant<int, 1>{});
        // segment s_lo is in buffer (s_hi - s_lo) % NB; only segment 0 is partial
        const int b0 = (s_hi - s_lo) % NB;
        auto last = [&](auto tag) {
            if (b0 == 0) produce(cb[0], s_lo, tag);
            else if (b0 == 1) produce(cb[1], s_lo, tag);
            else produce(cb[NB - 1], s_lo, tag);
        };
        if (!BANDED || s_lo == 0) last(part_t{});
        else last(full_t{});
#pragma unroll
        for (int t = 0; t < NSTAGE - 1; ++t) bar();
    } else if (wave == 1) {
        // the backward chain is the critical path of the pair: issue priority
        __builtin_amdgcn_s_setprio(3);
        // ---------------------------------------------------- consumer
        constexpr int RD = RH * K;
        const int bpath = FAM == PAIR_D2 ? uniform(((path - (H - 1)) % W + W) % W) : path;
        Cursor<BD> bc, pc;
        bc.init(bpath, H, W, g.D);
        pc.init(bpath, H, W, g.D);
        // LIN: running offsets of the step (bo) and of the ring refill (po,
        // position pp, held at position 0 past the chain's end)
        long long bo = lin_base + (long long)(n - 1 - kb) * lin_st, po = bo;
        int pp = n - 1 - kb;
        auto padv = [&] {
            if constexpr (LIN) {
                po -= pp > 0 ? lin_st : 0;
                pp = pp > 0 ? pp - 1 : 0;
            } else {
                pc.advance_upto(n, W, D, WD);
            }
        };
        auto poff = [&] { return LIN ? po : pc.off; };
        float ab[RD][V], sb[RD][V];
#pragma unroll
        for (int u = 0; u < RD; ++u) {
            if (NEED_ACC) load_v_nt<V>(ab[u], a.acc_in + poff() + e0, active);
            if (NEED_S) load_v_nt<V>(sb[u], a.s_in + poff() + e0, active);
            padv();
        }
        float prevb[V];
        float pminb = 0.0f;
        if (BANDED && kb > 0) {  // the chain state entering the band
            load_v<V>(prevb, a.band.carry + (size_t)path * g.D + e0, active);
            pminb = wave_min(lane_min(prevb));
        } else {
#pragma unroll
            for (int v = 0; v < V; ++v) prevb[v] = LIN ? 0.0f : SGM_INF;
        }
        auto consume = [&](int c, auto full_tag, auto half_tag) {
            constexpr bool FULLSEG = decltype(full_tag)::value;
            constexpr int HF = decltype(half_tag)::value;
            const int cnt = FULLSEG ? K : (c == nseg - 1 ? r0 : K);
            const int skip = K - cnt;
            const int buf = c & 1;
#pragma unroll
            for (int r = 0; r < K; ++r) {
                const int kk = K - 1 - r;
                if (FULLSEG || kk >= skip) {
                    const int q = HF * K + r;   // ring slot
                    float cs[V], lf[V];
                    load_lds_v<V>(cs, &L.c[buf][kk][e0]);
                    load_lds_v<V>(lf, &L.l[buf][kk][e0]);
                    float Lr[V];
                    dp_step<V>(prevb, pminb, cs, Lr, a.p1, p2v);
                    if constexpr (!LIN) {
                        const bool st = bc.start(W);
#pragma unroll
                        for (int v = 0; v < V; ++v) Lr[v] = st ? cs[v] : Lr[v];
                    }
                    const float nmin = wave_min(lane_min(Lr));
                    const long long boff = LIN ? bo : bc.off;
                    if constexpr (MODE == PAIR_INIT2) {
                        float o[V];
#pragma unroll
                        for (int v = 0; v < V; ++v) o[v] = lf[v] + Lr[v];
                        store_v_nt<V>(a.out + boff + e0, o, active);
                    } else if constexpr (MODE == PAIR_ACC) {
                        float o[V];
#pragma unroll
                        for (int v = 0; v < V; ++v) o[v] = (ab[q][v] + lf[v]) + Lr[v];
                        store_v_nt<V>(a.out + boff + e0, o, active);
                    } else {
                        // X = (S12 + L3) + L4
                        float x[V];
#pragma unroll
                        for (int v = 0; v < V; ++v) x[v] = (sb[q][v] + lf[v]) + Lr[v];
                        store_lds_v<V>(&F->t[buf][r][e0], x);
                    }
#pragma unroll
                    for (int v = 0; v < V; ++v) prevb[v] = Lr[v];
                    pminb = nmin;
                    if constexpr (LIN) bo -= lin_st;
                    else bc.advance(W, D, WD);
                    if (NEED_ACC) load_v_nt<V>(ab[q], a.acc_in + poff() + e0, active);
                    if (NEED_S) load_v_nt<V>(sb[q], a.s_in + poff() + e0, active);
                    padv();
                }
            }
            bar();
        };
        using h0 = std::integral_constant<int, 0>;
        using h1 = std::integral_constant<int, RH - 1>;
        bar();
        int c = c_lo;
        for (; c + RH <= c_hi - 1; c += RH) {
            consume(c, full_t{}, h0{});
            if constexpr (RH == 2) consume(c + 1, full_t{}, h1{});
        }
        if (RH == 2 && c < c_hi - 1) {
            consume(c, full_t{}, h0{});
            consume(c + 1, part_t{}, h1{});
        } else {
            consume(c, part_t{}, h0{});
        }
        if (BANDED && ke < n) store_v<V>(a.band.carry + (size_t)path * g.D + e0, prevb, active);
        if (FINAL) bar();
    } else if constexpr (FINAL) {
        __builtin_amdgcn_s_setprio(3);  // the WTA wave is the slowest stage of the final pipeline
        // ------------------------------------------------- WTA (wave 2)
        // total = X + T (X = (S12 + L3) + L4 from the LDS ring), then WTA,
        // uniqueness and sub-pixel over the chunk.  T rows for the next chunk
        // are loaded while this one is processed.  Chunk c, slot r is pixel
        // (H-1 - (cK + r), path): L4 walks the column upward.
        // NWTA waves split each chunk's K pixels (KP each)
        constexpr int KP = K / NWTA;
        constexpr int LPP = 64 / KP;                 // lanes per pixel
        constexpr int QQ = (FULL ? 64 * V : 32) / LPP;  // disparities per lane
        static_assert(QQ % 4 == 0, "T rows load as float4");
        const int half = wave - 2;
        const int px = lane / LPP, d0 = (lane - px * LPP) * QQ;
        const int slot = half * KP + px;
        // T rows of chunk c: slot r is row H-1 - (cK + r).  Addressed from the
        // chunk's top row (slot K-1; a wave-uniform pointer) plus this lane's
        // constant byte offset; the partial last chunk's unused slots point
        // into the volume's leading guard (kTGuardRows rows, never consumed).
        const unsigned t_off = (unsigned)((((size_t)(K - 1 - slot) * W) * D + d0) * sizeof(float));
        auto tload = [&](float (&t)[QQ], int c) {
            const long long top = (long long)(H - K - c * K) * W + path;
            const float *src = reinterpret_cast<const float *>(
                reinterpret_cast<const char *>(a.acc_in + top * D) + t_off);
#pragma unroll
            for (int k = 0; k < QQ; k += 4) {
#pragma unroll
                for (int e = 0; e < 4; ++e) t[k + e] = __builtin_nontemporal_load(src + k + e);
            }
        };
        // results of chunk c: pixel (H-1 - cK - half*KP - px, path) = the
        // wave's top pixel (px = KP-1) + (KP-1 - px) rows
        const unsigned o_off = (unsigned)((KP - 1 - px) * W);
        // the sub-pixel map: row-major like disp, or column-major (a.sub_cm:
        // a chunk's KP pixels are then contiguous, whole cache lines over
        // consecutive chunks instead of one partial line per pixel)
        const unsigned s_off = a.sub_cm ? (unsigned)(KP - 1 - px) : o_off;
        // T for chunk c+2 is issued while chunk c is consumed (3 buffers)
        auto chunk = [&](const float (&t)[QQ], float (&tn)[QQ], int c) {
            tload(tn, c + 2 < c_hi ? c + 2 : c_hi - 1);
            const int cnt_all = c == nseg - 1 ? r0 : K;
            const int cnt = cnt_all - half * KP < 0 ? 0 : (cnt_all - half * KP > KP ? KP : cnt_all - half * KP);
            // total = X + T in registers (the WTA's own lane layout); the row
            // goes back to LDS only for the sub-pixel's three neighbours
            float *row = &F->t[c & 1][slot][d0];
            float x[QQ];
#pragma unroll
            for (int k = 0; k < QQ; k += 4) {
                float4 x4 = *reinterpret_cast<float4 *>(row + k);
                x4.x = x4.x + t[k];
                x4.y = x4.y + t[k + 1];
                x4.z = x4.z + t[k + 2];
                x4.w = x4.w + t[k + 3];
                x[k] = x4.x; x[k + 1] = x4.y; x[k + 2] = x4.z; x[k + 3] = x4.w;
                if (px < cnt) *reinterpret_cast<float4 *>(row + k) = x4;
            }
            const long long row_top = H - c * K - (half + 1) * KP;
            wta_chunk_q<V, KP, QQ>(x, F->t[c & 1] + half * KP, row_top * W + path, o_off,
                                   a.sub_cm ? (long long)path * H + row_top : row_top * W + path,
                                   s_off, cnt, lane, g.D, a.uniq, a.disp, a.sub);
            bar();
        };
        float t0[QQ], t1[QQ], t2[QQ];
        tload(t0, c_lo);
        tload(t1, c_lo + 1 < c_hi ? c_lo + 1 : c_lo);
        bar();
        bar();
        int c = c_lo;
        for (; c + 2 < c_hi; c += 3) {
            chunk(t0, t2, c);
            chunk(t1, t0, c + 1);
            chunk(t2, t1, c + 2);
        }
        if (c < c_hi) chunk(t0, t2, c);
        if (c + 1 < c_hi) chunk(t1, t0, c + 1);
    }
#ifdef SGM_STAMPS
    if (lane == 0) {
        const int role = wave + (FAM == PAIR_V ? 0 : 3);
        atomicAdd(&sgm_stamps[role][0], (unsigned long long)st_work);
        atomicAdd(&sgm_stamps[role][1], (unsigned long long)st_wait);
        atomicAdd(&sgm_stamps[role][2], 1ull);
    }
#endif
}

// ------------------------------------------------------ vertical pass

// cost_vertical_filter (Solver.cpp:333-368) fused with the L3 forward pass
// (SGM.cpp:161-199): one wave per column, lane l owning the V vertical IIR
// chains d = l*V .. l*V+V-1.  Row i of the final cost is produced, stored,
// and fed straight into the L3 DP; L3 is checkpointed for the PAIR_V
// backward kernel.  The raw rows the IIR adds (raw[i + WIN/2 + 1]) stream
// through a register ring PF rows ahead.
// BAND (the forward bands above the Infinity Cache): rows [a.band.kb,
// a.band.ke) only, the filter's running sum, its last output and the L3 state
// entering the band read from a.band.carry (3 D-vectors per column) and the
// state leaving it written back there.
// L3OUT (the slanted schedule, sgm_slant.hip): every row's L3 goes to a.out
// (a full HWD volume, streamed) instead of checkpoints.
template <int V, bool FULL, int WIN, int PF, bool BAND = false, bool L3OUT = false>
__device__ __forceinline__ void vfwd_body(const float *__restrict__ in, float *__restrict__ out,
                                          const PairArgs &a, const Geom &g, int j, int lane) {
    constexpr int K = pair_kv<V>();
    constexpr int HALF = WIN / 2, LAG = WIN - HALF - 1, LA = HALF + 1;
    const float p2v = to_vgpr(a.p2);  // dp_step's P2 operand
    const int H = g.H;
    const size_t stride = (size_t)g.W * g.D;
    const int e0 = lane * V;
    const bool active = FULL || e0 < g.D;
    const float *col = in + (size_t)j * g.D + e0;
    float *ocol = out + (size_t)j * g.D + e0;
    const int nseg = (H + K - 1) / K;
    const int r0 = H - (nseg - 1) * K;
    float *ck = a.ckpt + (size_t)j * nseg * g.D + e0;
    const int rb = BAND ? a.band.kb : 0;
    const int re = BAND && a.band.ke > 0 ? a.band.ke : H;
    // checkpoints sit after rows r0-1 + mK; the first one at or after rb
    int ck_i = rb <= r0 - 1 ? 0 : (rb - r0 + K) / K;
    int next_ck = r0 - 1 + ck_i * K;
    const int T = H - 2 * HALF;
    float *cy = BAND ? a.band.carry + (size_t)j * 3 * g.D + e0 : nullptr;

    float raw0[V], rawl[V], sum[V], o1[V];
    load_v_nt<V>(raw0, col, active);
    load_v_nt<V>(rawl, col + (size_t)(H - 1) * stride, active);  // the only row below LAG+T (WIN=3)
    float prev[V];
    float pmin = 0.0f;
    if (BAND && rb > 0) {  // the filter and path state entering the band
        load_v<V>(sum, cy, active);
        load_v<V>(o1, cy + g.D, active);
        load_v<V>(prev, cy + 2 * g.D, active);
        pmin = wave_min(lane_min(prev));
    } else {
#pragma unroll
        for (int v = 0; v < V; ++v) sum[v] = 0.0f;
#pragma unroll
        for (int k = 0; k < WIN; ++k) {
            float r[V];
            load_v_nt<V>(r, col + (size_t)k * stride, active);
#pragma unroll
            for (int v = 0; v < V; ++v) sum[v] += r[v];
        }
#pragma unroll
        for (int v = 0; v < V; ++v) o1[v] = 0.0f;
        // L = 0, minL = 0 before row 0 makes the first step yield L = C (the
        // path start, SGM.cpp:161-170) without a per-row select (P1, P2 >= 0)
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = 0.0f;
    }
    float ring[PF][V];
#pragma unroll
    for (int u = 0; u < PF; ++u)
        load_v_nt<V>(ring[u], col + (size_t)min(rb + LA + u, H - 1) * stride, active);

    auto row = [&](int i, int u, bool refill) {
        float c[V];
        if (i < LAG) {
            // row 0 stays raw; it is also what step t = 0 subtracts, kept in
            // o1 (and so in a band's carry) rather than re-read from `in`,
            // whose row 0 the forward bands overwrite with T (T aliases the
            // horizontally filtered volume) before the next band starts
#pragma unroll
            for (int v = 0; v < V; ++v) c[v] = raw0[v];
#pragma unroll
            for (int v = 0; v < V; ++v) o1[v] = c[v];
        } else if (i >= LAG + T) {
#pragma unroll
            for (int v = 0; v < V; ++v) c[v] = rawl[v];
        } else {
            const int t = i - LAG;
#pragma unroll
            for (int v = 0; v < V; ++v) c[v] = div_win<WIN>(sum[v]);
            if (t < T - 1) {
#pragma unroll
                for (int v = 0; v < V; ++v) {
                    const float sub = LAG == 0 ? c[v] : o1[v];
                    sum[v] = (sum[v] + ring[u][v]) - sub;
                }
            }
#pragma unroll
            for (int v = 0; v < V; ++v) o1[v] = c[v];
        }
        // the slanted schedule's C (L3OUT: above the Infinity Cache) streams
        // past L2 like L3 does (paired A/B r05: -0.6% HD256, -0.5% 4K256);
        // the whole-volume schedules keep the default policy, their C is
        // re-read from the cache
        if constexpr (L3OUT) store_v_nt<V>(ocol + (size_t)i * stride, c, active);
        else store_v<V>(ocol + (size_t)i * stride, c, active);
        // L3 forward step on the freshly filtered row
        float L[V];
        dp_step<V>(prev, pmin, c, L, a.p1, p2v);
        const float nmin = wave_min(lane_min(L));
        if constexpr (L3OUT) {
            store_v_nt<V>(a.out + (size_t)j * g.D + e0 + (size_t)i * stride, L, active);
        } else if (i == next_ck && ck_i < nseg - 1) {
            store_v<V>(ck + (size_t)ck_i * g.D, L, active);
            ++ck_i;
            next_ck += K;
        }
#pragma unroll
        for (int v = 0; v < V; ++v) prev[v] = L[v];
        pmin = nmin;
        if (refill) load_v_nt<V>(ring[u], col + (size_t)min(i + LA + PF, H - 1) * stride, active);
    };
    int i0 = rb;
    for (; i0 + PF <= re; i0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) row(i0 + u, u, true);
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (i0 + u < re) row(i0 + u, u, false);
    if (BAND && re < H) {  // the state leaving the band
        store_v<V>(cy, sum, active);
        store_v<V>(cy + g.D, o1, active);
        store_v<V>(cy + 2 * g.D, prev, active);
    }
}

}  // namespace sgm
