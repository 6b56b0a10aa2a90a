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
// take them from the next tile (t+1), whose waves 0 and 1 store them after
// each step as self-tagged 8-byte granules (16-byte sc1 stores of two; no
// flag, no fence: the data is the flag, cdna_hip_programming.md Guideline 16,
// R2), polled by this tile's receiver wave.  All dependencies point from
// tile t+1 to tile t, so tiles claimed in the order t = T-1, T-2, ... never
// wait on a tile no workgroup holds: no deadlock for any grid size, and a
// tile may run any number of steps behind its right neighbour.
//
// Two passes share the kernel (slant_kernel<UP, ...>):
//  * top-down (UP = false; tiles lean along L5, whose chains stay in a wave,
//    L6 comes from wave k+2): T56 = L5 + L6 (SGM.cpp:247-305; the first
//    association of SGM.cpp:389), reading C and writing T56: 8 B per element
//    instead of the two diagonal sweeps' 20;
//  * bottom-up (UP = true; tiles lean along L7, L4 from wave k+1, L8 from
//    wave k+2): L4 (SGM.cpp:201-239), L7, L8 (:311-369),
//      total = ((S12 + L3) + L4) + ((T56 + L7) + L8)   (SGM.cpp:386-390)
//    and the WTA + uniqueness + sub-pixel (SGM.cpp:372-418, Solver.cpp:
//    569-597), reading C, S12 = L1+L2, L3 and T56 once each: 16 B per
//    element instead of the 36.75 of stage B's diagonal pair + L8 + the final
//    pass.
#include "sgm_bodies.h"

#include <cstdlib>

namespace sgm {

// LDS exchange of one tile: the exchanged chain states (NE per wave:
// bottom-up L4 and L8, top-down L6) and their minima in a ring of R steps
// (step s in slot s & (R-1)); slots NW and NW+1 hold the next tile's wave 0 /
// wave 1 states, put there by the receiver wave.  No workgroup barrier per
// step: done[w + 2] is the last step whose states wave w (0..NW-1) has
// published, done[NW + 2] = done[NW + 3] the receiver's; done[0], done[1]
// stand for waves -2 and -1, which consume nothing (DESIGN.md 5e "Dataflow").
template <int V, int NW, int NE, int R>
struct SlantLds {
    float st[R][NW + 2][NE][64 * V];
    float pm[R][NW + 2][NE];
    int done[NW + 4];
    int ticket;
    unsigned epoch;
};

// granule index of (view, tile, step, slot 0..2, disparity).  Bottom-up:
// slot 0 = wave 0's L4, 1 = wave 0's L8, 2 = wave 1's L8; top-down: 0 = wave
// 0's L6, 1 = wave 1's L6.  The two passes share the buffer: their tags
// differ in parity.
__device__ __forceinline__ size_t gran_index(int T, int H, int D, int view, int t, int s, int slot) {
    return ((((size_t)view * T + t) * H + s) * 3 + slot) * D;
}

// A granule carries one float with a 16-bit tag in EACH 4-byte half:
// {tag:16 | lo16} {tag:16 | hi16}.  An 8-byte store is observed untorn on
// gfx950 (not an architectural guarantee, cdna_hip_programming.md Guideline
// 16); with the tag in both halves a torn read -- one half of this launch's
// store, one of an older one (the other pass shares the buffer) -- fails the
// check instead of passing a value that was never written.
__device__ __forceinline__ unsigned long long granule(float x, unsigned tag) {
    const unsigned b = __float_as_uint(x), t = tag << 16;
    return ((unsigned long long)(t | (b >> 16)) << 32) | (t | (b & 0xffffu));
}
// (bitwise, no short circuit: a branch here would make the waitcnt pass
// drain every load in flight before the next use of the ring)
__device__ __forceinline__ unsigned granule_ok(unsigned long long q, unsigned tag) {
    return (unsigned)((unsigned)(q >> 48) == tag) & (unsigned)(((unsigned)q >> 16) == tag);
}
__device__ __forceinline__ float granule_value(unsigned long long q) {
    return __uint_as_float(((unsigned)(q >> 16) & 0xffff0000u) | ((unsigned)q & 0xffffu));
}

// One tile's granules (H steps x 3 slots x D) as a buffer resource, moved by
// sc1 (write-through) buffer stores and loads: 16 bytes (two granules) per
// lane and instruction where a lane holds two or more (D >= 128), else 8.  A
// lane's V granules as separate 8-byte sc1 stores cost ~2.7x the 16-byte
// form per byte (MI355X_MICROARCH.md "stores of each flavour",
// cdna_hip_programming.md Guideline 16 pitfall 7).  A slot's D granules sit
// in access order: instruction k (of V/2) of lane l at byte (64k + l) * 16.  Two granules in one
// 16-byte access stay independently checkable: each 4-byte half carries the
// tag.  A resource with 0 records drops every access through it (the range
// check): waves without exit states store through one, so every compute wave
// runs the same instruction stream.
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
typedef unsigned v2u32 __attribute__((ext_vector_type(2)));
constexpr int kGranAux = 16;           // cache policy: sc1
constexpr int kGranOff = 0x40000000;   // an offset past every tile's records
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gran_rsrc(unsigned long long *tile_base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(tile_base, 0, bytes, 0x00020000);
}
template <int V>
__device__ __forceinline__ void store_granules(__amdgpu_buffer_rsrc_t rs, int off, const float (&x)[V],
                                               unsigned tag) {
    if constexpr (V == 1) {
        const unsigned long long g0 = granule(x[0], tag);
        const v2u32 q = {(unsigned)g0, (unsigned)(g0 >> 32)};
        __builtin_amdgcn_raw_buffer_store_b64(q, rs, off, 0, kGranAux);
    } else {
#pragma unroll
        for (int v = 0; v < V; v += 2) {
            const unsigned long long g0 = granule(x[v], tag), g1 = granule(x[v + 1], tag);
            const v4u32 q = {(unsigned)g0, (unsigned)(g0 >> 32), (unsigned)g1, (unsigned)(g1 >> 32)};
            __builtin_amdgcn_raw_buffer_store_b128(q, rs, off + (v / 2) * 1024, 0, kGranAux);
        }
    }
}
template <int V>
__device__ __forceinline__ void load_granules(unsigned long long (&g)[V], __amdgpu_buffer_rsrc_t rs, int off) {
    if constexpr (V == 1) {
        const v2u32 q = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, kGranAux);
        g[0] = ((unsigned long long)q[1] << 32) | q[0];
    } else {
#pragma unroll
        for (int v = 0; v < V; v += 2) {
            const v4u32 q = __builtin_amdgcn_raw_buffer_load_b128(rs, off + (v / 2) * 1024, 0, kGranAux);
            g[v] = ((unsigned long long)q[1] << 32) | q[0];
            g[v + 1] = ((unsigned long long)q[3] << 32) | q[2];
        }
    }
}

__device__ __forceinline__ float uni_f(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

#ifdef SGM_SLANT_STAMPS
// [0] tile-steps (compute wave 0)  [1] receiver phases that re-polled
// [2] receiver re-polls  [3] receiver cycles in re-polls  [4] compute wave 0
// cycles between barriers  [5] compute wave 0 cycles in barriers
// [7] cycles inside tiles (wave 0)  [8] workgroups  [9] tiles
// (the top-down pass's at [0, 16), the bottom-up pass's at [16, 32))
static __device__ unsigned long long slant_stamps[32];
#define SLANT_STAMP(i, v) atomicAdd(&slant_stamps[(UP ? 16 : 0) + (i)], (unsigned long long)(v))
#endif

#ifdef SGM_SLANT_HOPS
// Hop timeline (tools/slant_hops.py): per pass and (view, tile, step), in
// s_memrealtime ticks (100 MHz, chip-wide), low 32 bits: [0] compute wave 0
// issued this tile's exit-state stores of the step, [1] the receiver started
// the phase that needs the next tile's states of the step, [2] it held them,
// [3] compute wave 0 left the barrier that ends the step.
constexpr size_t kHopN = (size_t)1 << 21;
static __device__ unsigned slant_hops[2][4][kHopN];
__device__ __forceinline__ void hop_mark(int pass, int what, int T, int H, int view, int t, int s) {
    const size_t i = ((size_t)view * T + t) * H + s;
    if (s >= 0 && i < kHopN) slant_hops[pass][what][i] = (unsigned)__builtin_amdgcn_s_memrealtime();
}
#endif

// Exit states of a tile per step, as (wave, exchanged-state index) pairs:
// bottom-up (w0 L4, w0 L8, w1 L8), top-down (w0 L6, w1 L6).
template <bool UP>
struct SlantExits {
    static constexpr int NX = UP ? 3 : 2;
    __device__ static constexpr int wave(int e) { return UP ? (e == 2 ? 1 : 0) : e; }
    __device__ static constexpr int kind(int e) { return UP ? (e == 0 ? 0 : 1) : 0; }
};

// PF: steps of data loads in flight per compute wave; CR: phases of hand-off
// granule loads in flight in the receiver; R: steps in the LDS state ring.
//
// Memory-instruction hygiene (as the other passes): every
// load and store of the steady-state loops is unconditional -- load
// addresses are clamped into the volume, inactive steps store to a dummy
// area -- so hipcc's waitcnt pass keeps exact vmcnt counts and the prefetch
// rings stay in flight across steps (a branch around a memory instruction
// makes later waits drain everything outstanding).
//
// Dataflow inside a tile (DESIGN.md 5e "Dataflow"): a compute wave's step s
// waits only for the states it reads -- wave k+1's (bottom-up) and k+2's of
// step s-1 -- and for the waves that read its own ring slot (k-1 bottom-up,
// k-2) to be past step s-R; the receiver waits only for waves NW-1 and NW-2.
// Waves 0 and 1, which produce the exit states, depend on the next tile's
// states of about 7 steps before (the k+2 family), so they run ahead of the
// receiver's hop instead of meeting it at a barrier every step.
#ifndef SLANT_POLL_GAP
#define SLANT_POLL_GAP 96
#endif
constexpr int kSlantPollGap = SLANT_POLL_GAP;  // sleeps (64 clocks) between the D = 256 re-polls
#ifndef SLANT_PUB_WAIT
#define SLANT_PUB_WAIT 1
#endif

// a step counter's wait: done[ia] and done[ib] >= thr_ab, done[ic] and
// done[id] >= thr_cd (wave-uniform indices and thresholds; INT_MIN: no
// condition).  Spins with a bounded count; returns false when it gave up (the
// caller reports it: the hang guard).
__device__ __forceinline__ int lds_word(const int *p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ bool flow_wait(const int *done, int ia, int ib, int thr_ab, int ic, int id,
                                          int thr_cd, unsigned limit) {
    for (unsigned spins = 0;; ++spins) {
        const int va = lds_word(done + ia), vb = lds_word(done + ib);
        const int vc = lds_word(done + ic), vd = lds_word(done + id);
        if (min(va, vb) >= thr_ab && min(vc, vd) >= thr_cd) break;
        if (spins >= limit) return false;
        __builtin_amdgcn_s_sleep(1);
    }
    // (the state reads that follow stay below the counter reads)
    asm volatile("" ::: "memory");
    return true;
}

// publish step s as done[idx] (lanes 0..n-1 store idx .. idx+n-1): after this
// wave's LDS stores of the step (LDS executes a wave's DS instructions in
// order; SLANT_PUB_WAIT also waits for their completion first)
__device__ __forceinline__ void flow_publish(int *done, int idx, int n, int s, int lane) {
#if SLANT_PUB_WAIT
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: the prefetch ring stays in flight
#endif
    asm volatile("" ::: "memory");
    if (lane < n) __hip_atomic_store(done + idx + lane, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}

template <bool UP, int V, bool FULL, int NW, int PF, int CR, int R>
__global__ __launch_bounds__(64 * (NW + 1)) void slant_kernel(SlantArgs a, Geom g) {
    constexpr int NE = UP ? 2 : 1;         // states exchanged per wave
    constexpr int K2 = UP ? 1 : 0;         // index of the wave k+2 family (L8 / L6)
    static_assert(R >= 2 && (R & (R - 1)) == 0, "ring of a power of two steps");
    using X = SlantExits<UP>;
    constexpr int NX = X::NX;
    __shared__ __attribute__((aligned(16))) SlantLds<V, NW, NE, R> L;
    const int wave = wave_id(), lane = tid_x() & 63;
    const int H = g.H, W = g.W, D = g.D;
    const int e0 = lane * V;
    const bool dact = FULL || e0 < D;
    // byte offset of this lane's granules in a slot: lanes past D (D = 32)
    // get one past the buffer's records (their loads read 0, stores drop)
    // (V = 4: granule pair k of lane l at byte (k * 64 + l) * 16 of the
    // slot, so each 16-byte access instruction covers 1 KB contiguously --
    // lane-contiguous pairs would leave every 32-byte sector half written
    // per instruction, and the write-through sends each half on its own)
    const int goff = dact ? (V == 1 ? lane * 8 : lane * 16) : kGranOff;
    const int tile_bytes = H * 3 * D * 8;
    const int T = a.ntiles, total = T * a.nviews;
    SlantCtl *ctl = a.ctl + (UP ? 1 : 0);
    // one step: up-right (-W*D + D) bottom-up, down-right (W*D + D) top-down
    const long long dstep = UP ? -(long long)(W - 1) * D : (long long)(W + 1) * D;
    if (tid_x() == 0)
        L.epoch = __hip_atomic_load(&ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const float p2v = to_vgpr(a.p2);
    // an LDS wait never waits for anything outside the workgroup but the
    // receiver, whose polls are bounded (and which publishes after giving
    // up): this limit, far above the receiver's, only turns a bug into a
    // reported error instead of a hang
    const unsigned flow_limit = a.spin_limit > (0xffffffffu >> 8) ? 0xffffffffu : a.spin_limit << 8;
    // hang guard (receiver wave): once a poll of this launch gave up -- this
    // wave's, or any workgroup's (ctl->dead == this launch's id) -- later
    // polls skip their wait, so a neighbour that never stores costs one spin
    // limit per launch, not one per step (the frame's maps are invalid
    // anyway, and the host reports it: sgm_capi.hip check_slant_err)
    unsigned dead = 0;
    auto give_up = [&]() {
        const unsigned id = __builtin_amdgcn_readfirstlane(L.epoch) + 1u;
        const unsigned launch_id = id ? id : 1u;
        if (lane == 0) {
            atomicAdd(&ctl->err, 1u);
            atomicExch(&ctl->dead, launch_id);
            // (the host reports it: sgm_capi.hip check_slant_err)
            __hip_atomic_store(a.err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        dead = 1u;
    };

    for (;;) {
        __syncthreads();
        if (tid_x() == 0) L.ticket = (int)atomicAdd(&ctl->tickets, 1u);
        __syncthreads();
        const int r = __builtin_amdgcn_readfirstlane(L.ticket);
        // 16-bit tags, never 0 (the zeroed buffer): 1 + (2 * epoch + pass) mod
        // 65535, so consecutive launches and the two passes of a frame differ
        const unsigned tag =
            1u + (2u * __builtin_amdgcn_readfirstlane(L.epoch) + (UP ? 1u : 0u)) % 65535u;
        if (r >= total) break;
        const int view = a.nviews == 2 ? (r & 1) : 0;
        const int t = T - 1 - (a.nviews == 2 ? (r >> 1) : r);
        const SlantView &sv = a.v[view];
        const int u_lo = -(H - 1) + t * NW;
        const int s_begin = max(0, -(u_lo + NW - 1));
        const int s_end = min(H, W - u_lo);
        const int nsteps = s_end - s_begin;
        // the tile's counters: every compute wave "published" step s_begin-1
        // (never read by an active pixel: a path start zeroes it, and the only
        // active pixel of a step s_begin > 0 is wave NW-1's, which reads the
        // receiver's slots); the receiver's prologue phase publishes s_begin-1
        if (wave == 0 && lane < NW + 4)
            L.done[lane] = lane < 2 ? INT_MAX : (lane < NW + 2 ? s_begin - 1 : s_begin - 2);
        __syncthreads();
#ifdef SGM_SLANT_DEBUG
        const unsigned stall = (unsigned)(UP && view == 0 && t == a.stall_tile);
#endif

        if (wave == NW) {
            // ----------------------------------------------- receiver wave
            // the receiver's phases feed the tile's last two waves: issue
            // priority over the compute waves (HD256 slant_up -7%, 4K256
            // -4..7%: profiles/r05_experiments/r05d_ab_*.txt)
#ifndef SLANT_RECV_PRIO
#define SLANT_RECV_PRIO 3
#endif
            __builtin_amdgcn_s_setprio(SLANT_RECV_PRIO);
            // Phase p = 0 .. nsteps (the prologue, then one per step) hands
            // the next tile's exit states of step gs = s_begin - 1 + p to ring
            // slot gs & (R-1) (slots NW, NW+1), which waves NW-1 and NW-2 read
            // in their step gs + 1.  Their granule loads run CR phases ahead;
            // a phase re-polls only when the next tile is not that far ahead.
            auto gvalid = [&](int p) {
                return t + 1 < T && (p >= 1 || s_begin >= 1) && p < nsteps;
            };
            // granules of (tile t+1, step s_begin - 1 + p), through tile
            // t+1's resource; a phase with nothing to fetch loads (and
            // ignores) step s_begin's, and the last tile reads its own
            const auto rrs = gran_rsrc(sv.gran + gran_index(T, H, D, view, t + 1 < T ? t + 1 : t, 0, 0), tile_bytes);
            auto gstep = [&](int p) { return uniform(gvalid(p) ? s_begin - 1 + p : s_begin); };
            unsigned long long rq[CR][NX][V];
            auto issue = [&](int slot, int p) {
                const int ss = gstep(p);
#pragma unroll
                for (int x = 0; x < NX; ++x) load_granules<V>(rq[slot][x], rrs, (ss * 3 + x) * D * 8 + goff);
            };
#pragma unroll
            for (int q = 0; q < CR; ++q) issue(q, q);
            // ring reuse: waves NW-2 and NW-1 (done[NW], done[NW+1]) read the
            // slot a phase overwrites
#ifdef SGM_SLANT_STAMPS
            long long rw = 0, rb = 0, rt = __builtin_amdgcn_s_memtime();
            long long rp_phases = 0, rp_polls = 0, rp_ticks = 0;  // added once per tile
#endif
            auto phase = [&](int slot, int p) {
                const int gs = s_begin - 1 + p;
                const bool want = gvalid(p);
#ifdef SGM_SLANT_HOPS
                if (lane == 0 && want) hop_mark(UP, 1, T, H, view, t, gs);
#endif
                const int c0 = u_lo + NW + gs;  // tile t+1's wave 0 column at step gs
                bool need[NX];
#pragma unroll
                for (int x = 0; x < NX; ++x) {
                    const int c = c0 + X::wave(x);
                    need[x] = want && c >= 0 && c < W;
                }
                // decode and check every granule of the slot unconditionally
                // (bitwise flags): the ring's waits stay exact
                float y[NX][V];
                auto decode_from = [&](const unsigned long long (&buf)[NX][V]) -> bool {
                    unsigned ok = 1u;
#pragma unroll
                    for (int x = 0; x < NX; ++x)
#pragma unroll
                        for (int v = 0; v < V; ++v) {
                            const unsigned long long q = buf[x][v];
                            y[x][v] = granule_value(q);
                            ok &= (unsigned)!need[x] | granule_ok(q, tag);
                        }
#ifdef SGM_SLANT_DEBUG
                    ok &= stall ^ 1u;
#endif
                    return (ok | (unsigned)!dact) != 0u;
                };
                auto decode = [&]() -> bool { return decode_from(rq[slot]); };
                if (!__all(decode())) {
                    // slow path: the next tile is not CR steps ahead
#ifdef SGM_SLANT_STAMPS
                    const long long sp0 = __builtin_amdgcn_s_memtime();
                    unsigned nsp = 0;
#endif
                    {
                        const unsigned id = __builtin_amdgcn_readfirstlane(L.epoch) + 1u;
                        const unsigned launch_id = id ? id : 1u;
                        dead |= (unsigned)(__builtin_amdgcn_readfirstlane(__hip_atomic_load(
                                               &ctl->dead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == launch_id);
                    }
                    // give-up after the spin limit (the hang guard above)
                    auto spin_check = [&](unsigned spins) {
                        if (spins >= a.spin_limit) give_up();
                    };
                    if constexpr (V >= 4) {
                        // D = 256: two re-polls in flight, the second issued
                        // kSlantPollGap sleeps after the first, each re-issued
                        // as soon as it has been checked.  Polls one after
                        // the other (each waits its load's full latency before
                        // the next is issued) hold the states half a loaded
                        // round trip later on average; with the first
                        // prefetch one step ahead (CR = 1) this frees the
                        // registers the second poll needs (HD256 frame
                        // -3.1%, 4K256 -1%, profiles/r05_experiments/
                        // r05y_ab_poll*.txt)
                        unsigned long long qb[NX][V];
                        auto repoll = [&](unsigned long long (&buf)[NX][V]) {
                            asm volatile("" ::: "memory");
#pragma unroll
                            for (int x = 0; x < NX; ++x) load_granules<V>(buf[x], rrs, (gs * 3 + x) * D * 8 + goff);
                        };
                        if (!dead) {
                            repoll(rq[slot]);
                            // (s_sleep takes 7 bits: at most 64 x 64 clocks a call)
#pragma unroll
                            for (int k = 0; k < kSlantPollGap / 64; ++k) __builtin_amdgcn_s_sleep(64);
                            if constexpr (kSlantPollGap % 64 != 0) __builtin_amdgcn_s_sleep(kSlantPollGap % 64);
                            repoll(qb);
                        }
                        for (unsigned spins = 1; !dead; ++spins) {
#ifdef SGM_SLANT_STAMPS
                            nsp = spins;
#endif
                            if (__all(decode())) break;
                            repoll(rq[slot]);
                            if (__all(decode_from(qb))) break;
                            repoll(qb);
                            spin_check(spins);
                        }
                    } else {
                        for (unsigned spins = 1; !dead; ++spins) {
                            __builtin_amdgcn_s_sleep(1);
                            // (a compiler barrier: the re-poll loads stay inside the loop)
                            asm volatile("" ::: "memory");
#pragma unroll
                            for (int x = 0; x < NX; ++x) load_granules<V>(rq[slot][x], rrs, (gs * 3 + x) * D * 8 + goff);
#ifdef SGM_SLANT_STAMPS
                            nsp = spins;
#endif
                            if (__all(decode())) break;
                            spin_check(spins);
                        }
                    }
#ifdef SGM_SLANT_STAMPS
                    rp_phases += 1;
                    rp_polls += nsp;
                    rp_ticks += __builtin_amdgcn_s_memtime() - sp0;
#endif
                }
#ifdef SGM_SLANT_HOPS
                if (lane == 0 && want) hop_mark(UP, 2, T, H, view, t, gs);
#endif
                // (a phase with nothing wanted writes slots that no valid
                // successor reads)
                const int par = gs & (R - 1);
#ifdef SGM_SLANT_STAMPS
                const long long t0_ = __builtin_amdgcn_s_memtime();
                rw += t0_ - rt;
#endif
                if (!flow_wait(L.done, NW, NW + 1, gs - R + 1, NW, NW + 1, INT_MIN, flow_limit)) give_up();
#ifdef SGM_SLANT_STAMPS
                rt = __builtin_amdgcn_s_memtime();
                rb += rt - t0_;
#endif
                // the states to LDS, then their minima, all NX reductions
                // interleaved (this phase sits on the tile-to-tile hop,
                // DESIGN.md 5e)
                float mx[NX];
#pragma unroll
                for (int x = 0; x < NX; ++x) {
                    float yy[V];
#pragma unroll
                    for (int v = 0; v < V; ++v) yy[v] = dact ? y[x][v] : SGM_INF;
                    mx[x] = lane_min(yy);
                    store_lds_v<V>(&L.st[par][NW + X::wave(x)][X::kind(x)][e0], yy);
                }
                wave_min_n<NX>(mx);
                if (lane == 0) {
#pragma unroll
                    for (int x = 0; x < NX; ++x) L.pm[par][NW + X::wave(x)][X::kind(x)] = mx[x];
                }
                flow_publish(L.done, NW + 2, 2, gs, lane);
                issue(slot, p + CR);
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
#ifdef SGM_SLANT_STAMPS
            if (lane == 0) {
                SLANT_STAMP(10, rw);
                SLANT_STAMP(11, rb);
                SLANT_STAMP(1, rp_phases);
                SLANT_STAMP(2, rp_polls);
                SLANT_STAMP(3, rp_ticks);
            }
#endif
            continue;
        }

        // ------------------------------------------------- compute waves
        const int k = wave;
        const int u = u_lo + k;
        // exit states (this tile's waves 0 and 1, read by tile t-1's
        // receiver): stored as granules right after each step's DP.  Bottom-
        // up, wave 0 stores L4 (slot 0) and L8 (slot 1), wave 1 L8 (slot 2);
        // top-down, wave k < 2 stores L6 (slot k).  The other waves store
        // through a resource with no records (dropped).
        const auto xrs_a = gran_rsrc(sv.gran + gran_index(T, H, D, view, t, 0, 0), k < 2 ? tile_bytes : 0);
        const auto xrs_b = gran_rsrc(sv.gran + gran_index(T, H, D, view, t, 0, 0), UP && k == 0 ? tile_bytes : 0);
        const int xslot_a = UP ? (k == 0 ? 0 : 2) : (k < 2 ? k : 0);
        // pixel of step s: row H-1-s (bottom-up) or s (top-down), column u+s.
        // Steps where this wave's pixel lies outside the image load a clamped
        // (valid) pixel, store to the dummy area, and their states are never
        // consumed: a valid predecessor is always an active wave's pixel
        // (DESIGN.md "Slanted tiles").
        const long long base = ((long long)(UP ? H - 1 : 0) * W + u) * D + e0;
        const int s_lo = max(s_begin, -u), s_hi = min(s_end - 1, W - 1 - u);
        const bool never = s_lo > s_hi;
        auto off_of = [&](int s) -> long long {
            const int sc = uniform(min(max(s, s_lo), s_hi));
            return never ? (long long)e0 : base + (long long)sc * dstep;
        };
        // the step counters this wave waits on (done[w + 2] is wave w's): its
        // producers k+1 (bottom-up L4) and k+2 need step s-1, its ring slot's
        // readers k-1 (bottom-up) and k-2 step s-R+1 (top-down: k+2 and k-2
        // only, each index given twice)
        const int i_p1 = UP ? k + 3 : k + 4, i_r1 = UP ? k + 1 : k;
        constexpr int NS = UP ? 4 : 1;  // streams: C (+ S12, L3, T56)
        float rb[NS][PF][V];
        int pfs = s_begin;  // step of the next ring refill
        auto refill = [&](int slot) {
            const long long o = off_of(pfs);
            // the bottom-up pass is C's last reader: non-temporal like its
            // other streams (slant_up -0.9% at HD256, -0.4% at 4K256; the
            // top-down pass's C reads stay default-policy, measured slower
            // non-temporal: profiles/r06_experiments/r06y_slant_nt.txt)
            if constexpr (UP) {
                load_v_nt<V>(rb[0][slot], sv.cost + o, dact);
                load_v_nt<V>(rb[1][slot], sv.s12 + o, dact);
                load_v_nt<V>(rb[2][slot], sv.l3 + o, dact);
                load_v_nt<V>(rb[3][slot], sv.t56 + o, dact);
            } else {
                load_v<V>(rb[0][slot], sv.cost + o, dact);
            }
            ++pfs;
        };
#pragma unroll
        for (int q = 0; q < PF; ++q) refill(q);
        float po[V];  // the own (leaning) chain: L7 bottom-up, L5 top-down
#pragma unroll
        for (int v = 0; v < V; ++v) po[v] = 0.0f;
        float mo = 0.0f;
        // the WTA of step s runs in step s + 1, after that step's DP chains
        // and its publish (it feeds no chain).  ptot / pstep: the deferred
        // step's totals and pixel (pstep < 0: none yet).
        float ptot[V];
#pragma unroll
        for (int v = 0; v < V; ++v) ptot[v] = 0.0f;
        int pstep = -1;
        auto wta_out = [&](const float (&tt)[V], int ps) {
            int d;
            float f;
            wta_subpixel<V>(tt, D, a.uniq, d, f);
            // outputs: an inactive step writes the dummy words instead
            const int j = u + ps;
            const bool act = ps >= 0 && j >= 0 && j < W;
            const long long pix = (long long)(H - 1 - ps) * W + j;
            float *fs = act ? sv.sub + pix : a.dummy + 256;
            if (lane == 0) *fs = f;
            if (sv.disp) {
                uint16_t *ds = act ? sv.disp + pix : reinterpret_cast<uint16_t *>(a.dummy + 257);
                if (lane == 0) *ds = (uint16_t)d;
            }
        };
#ifdef SGM_SLANT_STAMPS
        long long st_prev = __builtin_amdgcn_s_memtime(), st_work = 0, st_wait = 0;
        const long long tile_t0 = st_prev;
#endif

        auto step = [&](int q, int s) {
            const int j = u + s;
            const bool act = j >= 0 && j < W;
            const int pp = (s - 1) & (R - 1), cp = s & (R - 1);
#ifdef SGM_SLANT_STAMPS
            const long long tw0 = __builtin_amdgcn_s_memtime();
            st_work += tw0 - st_prev;
#endif
            if (!flow_wait(L.done, i_p1, k + 4, s - 1, i_r1, k, s - R + 1, flow_limit)) give_up();
#ifdef SGM_SLANT_STAMPS
            st_prev = __builtin_amdgcn_s_memtime();
            st_wait += st_prev - tw0;
#endif
            // path starts (SGM.cpp:93-98, :165-170, :205-214, :259-276,
            // :321-335): a zero state before the first pixel makes the step
            // yield L = C (P1, P2 >= 0)
            const bool v1 = s >= 1, vo = s >= 1 && j >= 1, v2 = s >= 1 && j + 1 <= W - 1;
            const float(&c)[V] = rb[0][q];
            // The exit states first (bottom-up L4 and L8, top-down L6): the
            // next tile's step waits for them, so they are computed and
            // stored before the own chain and the minima
            float Lo[V], L2[V], L4[V];
            if constexpr (UP) {
                float q1[V];
                load_lds_v<V>(q1, &L.st[pp][k + 1][0][e0]);
                // (uniform LDS words: into SGPRs, dp_step's scalar operand)
                float m1 = uni_f(L.pm[pp][k + 1][0]);
#pragma unroll
                for (int v = 0; v < V; ++v) q1[v] = v1 ? q1[v] : 0.0f;
                m1 = v1 ? m1 : 0.0f;
                dp_step<V>(q1, m1, c, L4, a.p1, p2v);
            }
            {
                float q2[V];
                load_lds_v<V>(q2, &L.st[pp][k + 2][K2][e0]);
                float m2 = uni_f(L.pm[pp][k + 2][K2]);
#pragma unroll
                for (int v = 0; v < V; ++v) q2[v] = v2 ? q2[v] : 0.0f;
                m2 = v2 ? m2 : 0.0f;
                dp_step<V>(q2, m2, c, L2, a.p1, p2v);
            }
            if constexpr (UP) {
                float xa[V];
#pragma unroll
                for (int v = 0; v < V; ++v) xa[v] = k == 0 ? L4[v] : L2[v];
                store_granules<V>(xrs_a, (s * 3 + xslot_a) * D * 8 + goff, xa, tag);
                store_granules<V>(xrs_b, (s * 3 + 1) * D * 8 + goff, L2, tag);
#ifdef SGM_SLANT_HOPS
                if (k == 0 && lane == 0) hop_mark(1, 0, T, H, view, t, s);
#endif
            } else {
                store_granules<V>(xrs_a, (s * 3 + xslot_a) * D * 8 + goff, L2, tag);
#ifdef SGM_SLANT_HOPS
                if (k == 0 && lane == 0) hop_mark(0, 0, T, H, view, t, s);
#endif
            }
            float zo[V];
#pragma unroll
            for (int v = 0; v < V; ++v) zo[v] = vo ? po[v] : 0.0f;
            const float mmo = vo ? mo : 0.0f;
            dp_step<V>(zo, mmo, c, Lo, a.p1, p2v);
            float no;
            if constexpr (UP) {
                float mm[3] = {lane_min(L4), lane_min(L2), lane_min(Lo)};
                wave_min_n<3>(mm);
                no = mm[2];
                // the exchanged states out first: the waves below wait for them
                store_lds_v<V>(&L.st[cp][k][0][e0], L4);
                store_lds_v<V>(&L.st[cp][k][K2][e0], L2);
                if (lane == 0) {
                    L.pm[cp][k][0] = mm[0];
                    L.pm[cp][k][K2] = mm[1];
                }
                flow_publish(L.done, k + 2, 1, s, lane);
                // ((S12 + L3) + L4) + ((T56 + L7) + L8)
                float tot[V];
#pragma unroll
                for (int v = 0; v < V; ++v)
                    tot[v] = ((rb[1][q][v] + rb[2][q][v]) + L4[v]) + ((rb[3][q][v] + Lo[v]) + L2[v]);
                wta_out(ptot, pstep);
#pragma unroll
                for (int v = 0; v < V; ++v) ptot[v] = tot[v];
                pstep = s;
            } else {
                float mm[2] = {lane_min(L2), lane_min(Lo)};
                wave_min_n<2>(mm);
                no = mm[1];
                store_lds_v<V>(&L.st[cp][k][K2][e0], L2);
                if (lane == 0) L.pm[cp][k][K2] = mm[0];
                flow_publish(L.done, k + 2, 1, s, lane);
                // T56 = L5 + L6 (streamed: the bottom-up pass reads it once)
                float o[V];
#pragma unroll
                for (int v = 0; v < V; ++v) o[v] = Lo[v] + L2[v];
                float *dst = act ? sv.t56w + off_of(s) : a.dummy + e0;
                store_v_nt<V>(dst, o, dact);
            }
#ifdef SGM_SLANT_HOPS
            if (k == 0 && lane == 0) hop_mark(UP, 3, T, H, view, t, s);
#endif
#pragma unroll
            for (int v = 0; v < V; ++v) po[v] = Lo[v];
            mo = no;
            refill(q);
        };
        int s0 = s_begin;
        for (; s0 + PF <= s_end; s0 += PF) {
#pragma unroll
            for (int q = 0; q < PF; ++q) step(q, s0 + q);
        }
#pragma unroll
        for (int q = 0; q < PF; ++q)
            if (s0 + q < s_end) step(q, s0 + q);
        if constexpr (UP) wta_out(ptot, pstep);
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
        const unsigned n = atomicAdd(&ctl->exits, 1u);
        if (n == (unsigned)a.grid - 1) {
            atomicExch(&ctl->exits, 0u);
            atomicExch(&ctl->tickets, 0u);
            atomicAdd(&ctl->epoch, 1u);
        }
    }
}

size_t slant_tiles(Geom g, int nw) { return (size_t)((g.W + g.H - 1 + nw - 1) / nw); }

size_t slant_gran_count(Geom g, int nviews) {
    // (both passes share the buffer: the narrower tiles' count)
    return (size_t)nviews * slant_tiles(g, kSlantNW < kSlantNWUp ? kSlantNW : kSlantNWUp) * g.H * 3 * g.D;
}

template <bool UP>
static hipError_t launch_slant_t(const SlantArgs &a0, Geom g, hipStream_t st) {
    SlantArgs a = a0;
    constexpr int NW = UP ? kSlantNWUp : kSlantNW;
    a.ntiles = (int)slant_tiles(g, NW);
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const int total = a.ntiles * a.nviews;
    a.grid = total < cus ? total : cus;
    if (a.max_grid > 0 && a.max_grid < a.grid) a.grid = a.max_grid;
    a.spin_limit = kSlantSpinLimit;
    a.stall_tile = -1;
#ifdef SGM_SLANT_DEBUG
    if (const char *e = getenv("SGM_SLANT_GRID")) a.grid = atoi(e) > 0 && atoi(e) < a.grid ? atoi(e) : a.grid;
    if (const char *e = getenv("SGM_SLANT_SPIN_LIMIT")) a.spin_limit = atoi(e) > 0 ? (unsigned)atoi(e) : a.spin_limit;
    if (const char *e = getenv("SGM_SLANT_STALL")) a.stall_tile = *e ? atoi(e) : -1;
#endif
    const dim3 grid(a.grid), block(64 * (NW + 1));
#ifndef SLANT_PF_UP4
#define SLANT_PF_UP4 4
#endif
#ifndef SLANT_PF_DN4
#define SLANT_PF_DN4 8
#endif
    // (the hand-off loads of the receiver queue behind the compute waves'
    // stream loads in the CU's memory pipeline: deeper rings hide more
    // stream latency but lengthen every tile-to-tile hop)
    constexpr int PF4 = UP ? SLANT_PF_UP4 : SLANT_PF_DN4, PF = UP ? 8 : 16;
    size_t pad = 0;
#ifdef SGM_SLANT_DEBUG
    if (const char *e = getenv("SGM_SLANT_LDSPAD")) pad = (size_t)atoi(e) * 1024;
#endif
    // R: the LDS state ring (steps a wave may run ahead of the waves that
    // read its states): 2 bottom-up, 4 top-down (HD256 paired: R = 2 for both
    // made slant_up 2.4% faster and the top-down pass beside the H pair 6%
    // slower; profiles/r06_experiments/r06n_knobs_ab.txt)
#ifndef SLANT_RING_UP
#define SLANT_RING_UP 2
#endif
#ifndef SLANT_RING_DN
#define SLANT_RING_DN 4
#endif
    constexpr int R = UP ? SLANT_RING_UP : SLANT_RING_DN;
    if (g.D == 32) slant_kernel<UP, 1, false, NW, PF, 8, R><<<grid, block, pad, st>>>(a, g);
    else if (g.D == 64) slant_kernel<UP, 1, true, NW, PF, 8, R><<<grid, block, pad, st>>>(a, g);
    else if (g.D == 128) slant_kernel<UP, 2, true, NW, PF, 6, R><<<grid, block, pad, st>>>(a, g);
#ifndef SLANT_CR4
#define SLANT_CR4 1
#endif
    else slant_kernel<UP, 4, true, NW, PF4, SLANT_CR4, R><<<grid, block, 0, st>>>(a, g);
    return hipGetLastError();
}

hipError_t launch_slant_up(const SlantArgs &a, Geom g, hipStream_t st) { return launch_slant_t<true>(a, g, st); }
hipError_t launch_slant_down(const SlantArgs &a, Geom g, hipStream_t st) { return launch_slant_t<false>(a, g, st); }

}  // namespace sgm

#ifdef SGM_SLANT_HOPS
// the hop timeline of both passes (tools/slant_hops.py): out holds
// 2 x 4 x n words (n <= 2^21, entries (view * T + t) * H + s); reset clears it
extern "C" int sgm_debug_slant_hops(unsigned *out, size_t n, int reset) {
    if (n > sgm::kHopN) return -1;
    for (int p = 0; p < 2; ++p)
        for (int w = 0; w < 4; ++w) {
            const size_t off = ((size_t)p * 4 + w) * sgm::kHopN * sizeof(unsigned);
            if (out && hipMemcpyFromSymbol(out + ((size_t)p * 4 + w) * n, HIP_SYMBOL(sgm::slant_hops),
                                           n * sizeof(unsigned), off) != hipSuccess)
                return -1;
        }
    if (reset) {
        void *ptr = nullptr;
        if (hipGetSymbolAddress(&ptr, HIP_SYMBOL(sgm::slant_hops)) != hipSuccess ||
            hipMemset(ptr, 0, sizeof(sgm::slant_hops)) != hipSuccess)
            return -1;
    }
    return 0;
}
#endif

#ifdef SGM_SLANT_STAMPS
extern "C" int sgm_debug_slant_stamps(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sgm::slant_stamps), sizeof(sgm::slant_stamps)) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sgm::slant_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
