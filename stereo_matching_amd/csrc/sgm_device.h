// sgm_device.h -- device-side building blocks shared by the gfx950 kernels:
// DPP / permlane wave reductions, path cursors, the DP step of SGM.cpp:93-117
// and the WTA of SGM.cpp:376-418 + Solver.cpp:577-593.
#pragma once

#include "sgm_internal.h"

#include <float.h>
#include <limits.h>

namespace sgm {

#define SGM_INF __builtin_inff()

// ---------------------------------------------------------------- helpers

// Work-item / workgroup ids straight from the hardware registers.  blockIdx /
// threadIdx go through the device library (__ockl_get_group_id, ...), which
// is compiled without -mno-amdgpu-ieee and therefore never inlined into these
// kernels: every id would come back from a call, in a VGPR, and everything
// derived from it (scanline cursors, addresses) would run on the VALU.
__device__ __forceinline__ int bid_x() { return (int)__builtin_amdgcn_workgroup_id_x(); }
__device__ __forceinline__ int bid_y() { return (int)__builtin_amdgcn_workgroup_id_y(); }
__device__ __forceinline__ int tid_x() { return (int)__builtin_amdgcn_workitem_id_x(); }
// index of the calling wave in its workgroup, as a scalar (role dispatch on it
// must be a uniform branch, not an exec-masked one)
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(tid_x() >> 6); }

// Block b -> column so that each XCD takes one contiguous range of columns.
// Blocks are dealt round-robin over the 8 XCDs (b and b + 8 share one;
// MI355X_MICROARCH.md "Workgroup dispatch"), so the plain b -> column map puts
// neighbouring columns on different XCDs, and a row-major output row's 128-B
// line is written 4 bytes at a time from 8 L2s, each writing back its own
// partial line.  With this map the 32 columns of a line share one L2, which
// merges their stores before the line leaves.  A bijection on [0, n).
__device__ __forceinline__ int xcd_column(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Hamming distance of two census words as an exact float.  Two 32-bit counts
// (v_bcnt_u32_b32 accumulates) keep the conversion a single v_cvt_f32_i32;
// a 64-bit popcount is converted through the u64 -> f32 sequence.
__device__ __forceinline__ float hamming(uint64_t a, uint64_t b) {
    const uint64_t x = a ^ b;
    return (float)(int)(__builtin_popcount((uint32_t)x) + __builtin_popcount((uint32_t)(x >> 32)));
}

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

// Minimum over the 64 lanes as a wave-uniform value (an SGPR, usable as the
// scalar operand of the next step's VALU ops): quad, half-row and row mirrors
// give every lane its 16-lane row minimum; row_bcast:15 folds row 0 into 1
// and 2 into 3, row_bcast:31 folds lane 31 into rows 2-3, so lane 63 holds
// the minimum (GFX9 DPP, valid on gfx950).  The row_bcast steps keep the
// unmasked rows' values, which the compiler cannot express as a fused
// v_min_f32_dpp, hence the inline asm; the s_nop covers the VALU-write ->
// DPP-read hazard the hazard recognizer does not see inside asm.
__device__ __forceinline__ float wave_min(float x) {
    x = fminf(x, movdppf<DPP_QP_1032>(x));
    x = fminf(x, movdppf<DPP_QP_2301>(x));
    x = fminf(x, movdppf<DPP_HALF_MIRROR>(x));
    x = fminf(x, movdppf<DPP_MIRROR>(x));
    asm("s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\tv_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "+v"(x));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

// Same value (kept for call sites that want the name).
__device__ __forceinline__ float wave_min_u(float x) { return wave_min(x); }

// wave_min of N independent values, stage by stage: each DPP stage of one
// value issues between two of another's, so the VALU-write -> DPP-read wait
// states are filled with work instead of s_nop (one reduction's latency for N
// results).  Exact like wave_min: min is exact, so the order is free.
template <int N>
__device__ __forceinline__ void wave_min_n(float (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = fminf(x[i], movdppf<DPP_QP_1032>(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = fminf(x[i], movdppf<DPP_QP_2301>(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = fminf(x[i], movdppf<DPP_HALF_MIRROR>(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = fminf(x[i], movdppf<DPP_MIRROR>(x[i]));
    static_assert(N == 2 || N == 3, "wave_min_n: 2 or 3 values");
    // (N >= 2 instructions between a value's two row_bcast steps give its
    // second read one wait state; the s_nop 0 adds the other)
    if constexpr (N == 2)
        asm("s_nop 1\n\t"
            "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "v_min_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "s_nop 0\n\t"
            "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
            "v_min_f32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf"
            : "+v"(x[0]), "+v"(x[1]));
    else
        asm("s_nop 1\n\t"
            "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "v_min_f32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "v_min_f32_dpp %2, %2, %2 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
            "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
            "v_min_f32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
            "v_min_f32_dpp %2, %2, %2 row_bcast:31 row_mask:0xc bank_mask:0xf"
            : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]));
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[i]), 63));
}

// min(src of the neighbouring lane, a): SHR reads lane l-1, SHL lane l+1.
// The edge lane (0 for SHR, 63 for SHL) has no source: with bound_ctrl off
// the DPP op is disabled there and the tied destination keeps a.
template <int CTRL>
__device__ __forceinline__ float nbmin(float src, float a) {
    float d = a;
    if constexpr (CTRL == DPP_WAVE_SHR1)
        asm("s_nop 1\n\tv_min_f32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf"
            : "+v"(d)
            : "v"(src));
    else
        asm("s_nop 1\n\tv_min_f32_dpp %0, %1, %0 wave_shl:1 row_mask:0xf bank_mask:0xf"
            : "+v"(d)
            : "v"(src));
    return d;
}

// A uniform value copied into a VGPR (once, outside a chain's loop).
__device__ __forceinline__ float to_vgpr(float x) {
    float v;
    asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}

// min(x of the neighbouring lane, x) in place (the edge lane keeps x)
template <int CTRL>
__device__ __forceinline__ float nbmin_self(float x) {
    if constexpr (CTRL == DPP_WAVE_SHR1)
        asm("s_nop 1\n\tv_min_f32_dpp %0, %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x));
    else
        asm("s_nop 1\n\tv_min_f32_dpp %0, %0, %0 wave_shl:1 row_mask:0xf bank_mask:0xf" : "+v"(x));
    return x;
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

// ------------------------------------------------------------- sweeps

// Position of one path along its scanline.  Horizontal paths are rows;
// vertical and diagonal paths are indexed by a column g and visit row k at
// column g (vertical) or (g +/- k) mod W (diagonal): when the column wraps the
// chain meets the image edge, which is exactly where the reference restarts
// a diagonal path (SGM.cpp:266,282,330,346), so W chains of H steps cover
// every pixel once per direction.  `off` is the element offset (i*W + j)*D of
// the pixel's disparity vector; everything here is wave-uniform (SALU).
// Correctly rounded x / WIN for the cost filters' window sizes (Solver.cpp:319,
// 357: sum / win_size).  For WIN = 3 and 5, q0 = x*RN(1/WIN) corrected by one
// FMA residual step equals IEEE division bit-for-bit for EVERY non-negative
// finite float (exhaustive GPU check, tools/verify_div.hip; negative x follows
// by symmetry, and -0 cannot occur in the filters); 3 VALU ops instead of the
// ~10-op div_scale/div_fmas/div_fixup sequence.
template <int WIN>
__device__ __forceinline__ float div_win(float x) {
    if constexpr (WIN == 1) {
        return x;
    } else if constexpr (WIN == 2) {
        return x * 0.5f;
    } else {
        constexpr float r = 1.0f / WIN;
        const float q0 = x * r;
        const float e = __builtin_fmaf(-q0, (float)WIN, x);
        return __builtin_fmaf(e, r, q0);
    }
}

// Integer division has no scalar instruction, so hipcc computes % in VALU
// and then treats the (uniform) result as divergent; pin it back to an SGPR.
__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

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
    // Position the cursor at step k of chain `path` (L1 row walk, L3 column
    // walk, L5 / L6 wrapped diagonals; the backward walks L2, L4, L7, L8 for
    // bands).
    __device__ __forceinline__ void init_at(int path, int kk, int H, int W, int D) {
        k = kk;
        if (DIR == 0) { i = path; j = kk; }
        else if (DIR == 1) { i = path; j = W - 1 - kk; }
        else if (DIR == 2) { i = kk; j = path; }
        else if (DIR == 3) { i = H - 1 - kk; j = path; }
        else if (DIR == 4) { i = kk; j = uniform((path + kk) % W); }
        else if (DIR == 5) { i = kk; j = uniform(((path - kk) % W + W) % W); }
        else if (DIR == 6) { i = H - 1 - kk; j = uniform((path + kk) % W); }
        else { i = H - 1 - kk; j = uniform(((path - kk) % W + W) % W); }  // DIR 7
        off = ((long long)i * W + j) * D;
    }
    __device__ __forceinline__ bool start(int W) const {
        if (k == 0) return true;
        if (DIR == 4 || DIR == 6) return j == 0;
        if (DIR == 5 || DIR == 7) return j == W - 1;
        return false;
    }
    __device__ __forceinline__ void advance(int W, long long D, long long WD) {
        // branch-free (scalar selects): a branch here makes hipcc duplicate
        // the surrounding loads into both arms and lose exact wait counts
        ++k;
        switch (DIR) {
        case 0: ++j; off += D; break;
        case 1: --j; off -= D; break;
        case 2: ++i; off += WD; break;
        case 3: --i; off -= WD; break;
        case 4:
        case 6: {
            const long long di = DIR == 4 ? WD : -WD;
            const bool wrap = j == W - 1;
            off += di + (wrap ? -(long long)(W - 1) * D : D);
            // pinned to an SGPR: left alone hipcc carries j in a VGPR and
            // spends VALU ops on every step's wrap test and select
            j = uniform(wrap ? 0 : j + 1);
            i += DIR == 4 ? 1 : -1;
            break;
        }
        default: {
            const long long di = DIR == 5 ? WD : -WD;
            const bool wrap = j == 0;
            off += di + (wrap ? (long long)(W - 1) * D : -D);
            j = uniform(wrap ? W - 1 : j - 1);
            i += DIR == 5 ? 1 : -1;
            break;
        }
        }
    }
    // advance only while k < n-1 (prefetch cursors stop on the last pixel)
    __device__ __forceinline__ void advance_upto(int n, int W, long long D, long long WD) {
        advance_if(k < n - 1, W, D, WD);
    }
    // predicated advance, select-based (no branch)
    __device__ __forceinline__ void advance_if(bool go, int W, long long D, long long WD) {
        Cursor nx = *this;
        nx.advance(W, D, WD);
        i = go ? nx.i : i;
        j = go ? nx.j : j;
        off = go ? nx.off : off;
        k = go ? nx.k : k;
    }
};

template <int V>
__device__ __forceinline__ void load_v(float (&dst)[V], const float *p, bool active) {
    if constexpr (V == 4) {
        float4 t = active ? *reinterpret_cast<const float4 *>(p) : make_float4(SGM_INF, SGM_INF, SGM_INF, SGM_INF);
        dst[0] = t.x; dst[1] = t.y; dst[2] = t.z; dst[3] = t.w;
    } else if constexpr (V == 2) {
        float2 t = active ? *reinterpret_cast<const float2 *>(p) : make_float2(SGM_INF, SGM_INF);
        dst[0] = t.x; dst[1] = t.y;
    } else {
        dst[0] = active ? *p : SGM_INF;
    }
}

// Streaming (non-temporal) variants for the partial-sum volumes (S12, T5, T)
// and the horizontally filtered cost, each read or written once per frame:
// they then do not allocate in the 256 MB Infinity Cache, so the cost volume
// C -- read by six passes -- can stay resident there at K128 (238.5 MB).
// Measured (tools/mall_probe.hip): five 2R1W passes over C + streams ran
// 467 us with non-temporal streams against 704 us with the default policy.
template <int V>
__device__ __forceinline__ void load_v_nt(float (&dst)[V], const float *p, bool active) {
#pragma unroll
    for (int v = 0; v < V; ++v) dst[v] = active ? __builtin_nontemporal_load(p + v) : SGM_INF;
}

template <int V>
__device__ __forceinline__ void store_v_nt(float *p, const float (&v)[V], bool active) {
    if (!active) return;
#pragma unroll
    for (int k = 0; k < V; ++k) __builtin_nontemporal_store(v[k], p + k);
}

// V consecutive floats from LDS
template <int V>
__device__ __forceinline__ void load_lds_v(float (&t)[V], const float *src) {
    if constexpr (V == 4) {
        const float4 x = *reinterpret_cast<const float4 *>(src);
        t[0] = x.x; t[1] = x.y; t[2] = x.z; t[3] = x.w;
    } else if constexpr (V == 2) {
        const float2 x = *reinterpret_cast<const float2 *>(src);
        t[0] = x.x; t[1] = x.y;
    } else {
        t[0] = src[0];
    }
}

// V consecutive floats to LDS (16-byte aligned rows)
template <int V>
__device__ __forceinline__ void store_lds_v(float *dst, const float (&t)[V]) {
    if constexpr (V == 4) *reinterpret_cast<float4 *>(dst) = make_float4(t[0], t[1], t[2], t[3]);
    else if constexpr (V == 2) *reinterpret_cast<float2 *>(dst) = make_float2(t[0], t[1]);
    else dst[0] = t[0];
}

template <int V>
__device__ __forceinline__ void store_v(float *p, const float (&v)[V], bool active) {
    if (!active) return;
    if constexpr (V == 4) *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
    else if constexpr (V == 2) *reinterpret_cast<float2 *>(p) = make_float2(v[0], v[1]);
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
    typedef float f2 __attribute__((ext_vector_type(2)));
    // callers pass P2 as a VGPR (to_vgpr, once per chain): minLp (an SGPR) +
    // P2 is then one VALU op (a VALU op reads at most one SGPR)
    const float pmin_p2 = pmin + p2;
    if constexpr (V == 1) {
        // neighbour minima min(L[d-1], L[d+1]) (d = lane)
        const float right = dppf<DPP_WAVE_SHL1>(SGM_INF, prev[0]);
        const float nb = nbmin<DPP_WAVE_SHR1>(prev[0], right);
        const float m = fminf(fminf(prev[0], nb + p1), pmin_p2);
        L[0] = m + (c[0] - pmin);
    } else {
        // q = Lp + P1 first (rounding is monotone, so min(a, b) + P1 ==
        // min(a + P1, b + P1) bit for bit), then the neighbour minima of q
        // in place: each q value that feeds a cross-lane minimum is dead
        // after it, so the DPP op can overwrite it (its edge lane keeps the
        // in-lane neighbour) and no copies are needed
        float q[V];
#pragma unroll
        for (int v = 0; v < V; v += 2) {
            const f2 t = f2{prev[v], prev[v + 1]} + p1;
            q[v] = t.x;
            q[v + 1] = t.y;
        }
        float t[V];
        if constexpr (V == 2) {
            // t0 = min(q1[l-1], q1), t1 = min(q0, q0[l+1])
            t[0] = nbmin_self<DPP_WAVE_SHR1>(q[1]);
            t[1] = nbmin_self<DPP_WAVE_SHL1>(q[0]);
        } else {
            // t0 = min(q3[l-1], q1), t1 = min(q0, q2), t2 = min(q1, q3), t3 = min(q2, q0[l+1])
            t[1] = fminf(q[0], q[2]);
            t[2] = fminf(q[1], q[3]);
            t[0] = nbmin<DPP_WAVE_SHR1>(q[3], q[1]);
            t[3] = nbmin<DPP_WAVE_SHL1>(q[0], q[2]);
        }
#pragma unroll
        for (int v = 0; v < V; v += 2) {
            const f2 d = f2{c[v], c[v + 1]} - pmin;
            f2 m;
            m.x = fminf(fminf(prev[v], t[v]), pmin_p2);
            m.y = fminf(fminf(prev[v + 1], t[v + 1]), pmin_p2);
            const f2 r = m + d;
            L[v] = r.x;
            L[v + 1] = r.y;
        }
    }
}

// x[d] of a wave-spread vector (lane d / V, slot d % V) for a wave-uniform d:
// V readlanes and scalar selects.  (A select chain on the slot in VALU
// registers, pick() below, is lowered by hipcc to a dynamically indexed
// private array: scratch stores and loads, whose vmcnt waits then also wait
// for every prefetch load in flight.)
template <int V>
__device__ __forceinline__ float wave_pick(const float (&x)[V], int d) {
    const int l = d / V, v = d - l * V;
    float r = readlane_f(x[0], l);
#pragma unroll
    for (int k = 1; k < V; ++k) {
        const float t = readlane_f(x[k], l);
        r = v == k ? t : r;
    }
    return r;
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
        const float a = wave_pick<V>(tot, d - 1);
        const float b = wave_pick<V>(tot, d + 1);
        const float c = wave_pick<V>(tot, d);
        const float x = d + (a - b) / (2 * (a + b - 2 * c));
        const float lim = (D - 1) * 1.f;
        f = (lim < x) ? lim : x;  // std::min(x, lim)
    }
    disp_out = d;
    sub_out = f;
}

// LDS-only workgroup barrier: waits for this wave's LDS traffic, not for its
// global loads (the prefetch ring stays in flight across the barrier).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // keep the scheduler from hoisting work of the next segment (and the
    // waits its loads need) above the barrier
    __builtin_amdgcn_sched_barrier(0);
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
    // branch-free selects (a pointer-select here made hipcc spill to scratch)
    const bool a_lt = A.m < B.m, b_lt = B.m < A.m;
    Wta r;
    r.m = fminf(A.m, B.m);
    r.i = a_lt ? A.i : (b_lt ? B.i : min(A.i, B.i));
    const float c1 = b_lt ? B.s : A.s;
    const int j1 = b_lt ? B.si : A.si;
    const float c2 = a_lt ? B.m : (b_lt ? A.m : B.s);
    const int j2 = a_lt ? B.i : (b_lt ? A.i : B.si);
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

// Merge with the lane 16 apart inside each 32-lane half (ds_swizzle bit mode,
// xor_mask 0x10): the cross-row step when a pixel spans 32 lanes.
__device__ __forceinline__ Wta wta_swz16(const Wta &x) {
    constexpr int PAT = 0x1F | (0x10 << 10);
    Wta y;
    y.m = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x.m), PAT));
    y.s = __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x.s), PAT));
    y.i = __builtin_amdgcn_ds_swizzle(x.i, PAT);
    y.si = __builtin_amdgcn_ds_swizzle(x.si, PAT);
    return wta_merge(x, y);
}

// LDS image of one chunk: PF pixels x D total costs, rows padded by 16 bytes
// so the consumer's per-pixel reads spread over all banks.
template <int V>
constexpr int tbuf_stride() { return 64 * V + 4; }

// WTA + uniqueness + sub-pixel (SGM.cpp:376-418, Solver.cpp:577-593) for
// `cnt` <= PF pixels whose total cost vectors sit in LDS rows tb[0..cnt), all
// at once: 64/PF lanes per pixel, each scanning D*PF/64 costs in ascending d,
// the partial states merged with DPP.  Pixel positions come from pb.
template <int V, int PF>
__device__ __forceinline__ void wta_consume_chunk_at(const float (*tb)[tbuf_stride<V>()],
                                                     long long pix0, long long pix_step, int cnt,
                                                     int lane, int Dn, float uniq,
                                                     uint16_t *disp, float *sub) {
    constexpr int LPP = 64 / PF;  // lanes per pixel
    const int Q = Dn / LPP;       // disparities per lane (>= 8)
    const int px = lane / LPP, q = lane - px * LPP;
    const int d0 = q * Q;
    const float *row = tb[px < cnt ? px : 0];
    Wta w;
    w.m = SGM_INF; w.s = SGM_INF; w.i = INT_MAX; w.si = INT_MAX;
    for (int k = 0; k < Q; k += 4) {
        const float4 x4 = *reinterpret_cast<const float4 *>(row + d0 + k);
        const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float x = xs[e];
            const int d = d0 + k + e;
            const bool lt = x < w.m;
            const bool sec = !lt && x != w.m && x < w.s;
            w.s = lt ? w.m : (sec ? x : w.s);
            w.si = lt ? w.i : (sec ? d : w.si);
            w.m = lt ? x : w.m;
            w.i = lt ? d : w.i;
        }
    }
    w = wta_dpp<DPP_QP_1032>(w);
    w = wta_dpp<DPP_QP_2301>(w);
    if (LPP >= 8) w = wta_dpp<DPP_HALF_MIRROR>(w);
    if (LPP >= 16) w = wta_dpp<DPP_MIRROR>(w);
    if (LPP >= 32) w = wta_swz16(w);
    static_assert(LPP <= 32, "a pixel spans at most 32 lanes");
    int d = w.i;
    if (w.s != SGM_INF && w.m / w.s > uniq && abs(w.i - w.si) > 1) d = Dn + 1;
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
        const long long pix = pix0 + px * pix_step;
        disp[pix] = (uint16_t)d;
        sub[pix] = f;
    }
}

// Minimum over an LPP-lane group (LPP = 4..32 consecutive lanes), in every
// lane of the group: quad, half-row and row mirrors, then the 16-apart
// swizzle for 32-lane groups.
template <int LPP>
__device__ __forceinline__ float group_min(float x) {
    x = fminf(x, movdppf<DPP_QP_1032>(x));
    x = fminf(x, movdppf<DPP_QP_2301>(x));
    if constexpr (LPP >= 8) x = fminf(x, movdppf<DPP_HALF_MIRROR>(x));
    if constexpr (LPP >= 16) x = fminf(x, movdppf<DPP_MIRROR>(x));
    if constexpr (LPP >= 32)
        x = fminf(x, __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x1F | (0x10 << 10))));
    return x;
}
template <int LPP>
__device__ __forceinline__ int group_min_i(int x) {
    x = min(x, movdpp<DPP_QP_1032>(x));
    x = min(x, movdpp<DPP_QP_2301>(x));
    if constexpr (LPP >= 8) x = min(x, movdpp<DPP_HALF_MIRROR>(x));
    if constexpr (LPP >= 16) x = min(x, movdpp<DPP_MIRROR>(x));
    if constexpr (LPP >= 32) x = min(x, __builtin_amdgcn_ds_swizzle(x, 0x1F | (0x10 << 10)));
    return x;
}

// The same WTA + uniqueness + sub-pixel for `cnt` <= PF pixels of a chunk,
// with the disparities per lane (QQ) known at compile time: instead of a
// running (min, index, second, index) state merged across lanes (about 15
// VALU ops per disparity and per merge step), two group minima of the values
// and two of the first indices holding them:
//   m  = min_d S[d],                     min_d = min { d : S[d] == m }
//   s  = min { S[d] : S[d] != m },       sec_d = min { d : S[d] == s }
// (SGM.cpp:383-408: the first strict minimum, the smallest other value and
// its first index).
// x: this lane's QQ total costs (disparities d0 .. d0+QQ-1 of pixel px); the
// LDS rows tb[] hold the same totals for the sub-pixel's neighbours.  The
// results go to pixel pix_top + pix_off: a wave-uniform index (SGPRs) plus
// this lane's constant offset (>= 0), so the stores need no per-lane 64-bit
// address arithmetic.
// sub goes to sub_top + sub_off (its own layout: column-major maps of the
// two-view frames), disp to pix_top + pix_off (row-major).
template <int V, int PF, int QQ>
__device__ __forceinline__ void wta_chunk_q(const float (&x)[QQ], const float (*tb)[tbuf_stride<V>()],
                                            long long pix_top, unsigned pix_off, long long sub_top,
                                            unsigned sub_off, int cnt, int lane, int Dn, float uniq,
                                            uint16_t *disp, float *sub) {
    constexpr int LPP = 64 / PF;  // lanes per pixel
    static_assert(QQ % 4 == 0 && LPP <= 32, "QQ a multiple of 4, at most 32 lanes per pixel");
    const int px = lane / LPP, q = lane - px * LPP;
    const int d0 = q * QQ;
    const float *row = tb[px < cnt ? px : 0];
    float lm = x[0];
#pragma unroll
    for (int k = 1; k < QQ; ++k) lm = fminf(lm, x[k]);
    const float m = group_min<LPP>(lm);
    // first index of m in this lane (QQ: none), and the lane's smallest value != m
    int li = QQ;
    float ls = SGM_INF;
#pragma unroll
    for (int k = QQ - 1; k >= 0; --k) {
        const bool eq = x[k] == m;
        li = eq ? k : li;
        ls = eq ? ls : fminf(ls, x[k]);
    }
    const int mi = group_min_i<LPP>(li < QQ ? d0 + li : INT_MAX);
    const float sec = group_min<LPP>(ls);
    int d = mi;
    if (sec != SGM_INF) {  // a second distinct value exists (else sec = FLT_MAX: ratio ~ 0)
        int lj = QQ;
#pragma unroll
        for (int k = QQ - 1; k >= 0; --k) lj = x[k] == sec ? k : lj;
        const int si = group_min_i<LPP>(lj < QQ ? d0 + lj : INT_MAX);
        if (m / sec > uniq && abs(mi - si) > 1) d = Dn + 1;
    }
    float f;
    if (d > Dn - 1) {
        f = (float)(Dn + 1);
    } else if (d == 0 || d == Dn - 1) {
        f = (float)d;
    } else {
        const float av = row[d - 1], bv = row[d + 1], cv = row[d];
        const float xx = d + (av - bv) / (2 * (av + bv - 2 * cv));
        const float lim = (Dn - 1) * 1.f;
        f = (lim < xx) ? lim : xx;  // std::min(x, lim)
    }
    if (q == 0 && px < cnt) {
        // disp: only when the frame hands out its raw WTA map (else null:
        // these one-pixel-per-row stores are partial cache lines, ~5% of the
        // final pass at K128 for both maps, profiles/r03_experiments/final_stores.txt)
        if (disp) (disp + pix_top)[pix_off] = (uint16_t)d;
        (sub + sub_top)[sub_off] = f;
    }
}

template <int V, int PF>
__device__ __forceinline__ void wta_consume_chunk(const float (*tb)[tbuf_stride<V>()],
                                                  const long long *pb, int cnt, int lane,
                                                  int Dn, float uniq, uint16_t *disp,
                                                  float *sub) {
    // pixels of a chunk are equally spaced along the scanline
    const long long step = cnt > 1 ? pb[1] - pb[0] : 0;
    wta_consume_chunk_at<V, PF>(tb, pb[0], step, cnt, lane, Dn, uniq, disp, sub);
}

}  // namespace sgm
