// sgm_post.hip -- post_filter() (src/Solver.cpp:600-649) on the GPU, bit-exact
// against its single-thread semantics (DESIGN.md "Post filter").
//
// 1. Median fill (Solver.cpp:604-630).  The reference walks the interior in
//    raster order and writes filled values back in place, so a pixel's 5x5
//    window sees FINAL values in the 12 cells before it (rows i-2, i-1 and
//    (i, j-2), (i, j-1)) and ORIGINAL values in the 12 cells after it.  Only
//    pixels that were invalid on entry can change.  The result is the unique
//    solution of that dependency DAG; it is computed here by
//      * 64x4 or 64x8 tiles (by frame size), one wave per tile, rows in order
//        inside the tile with the tile's window grid in LDS, and the in-row
//        chain (j-1, j-2) resolved by iterating the row to its fixed point
//        with lane shuffles;
//      * chaotic relaxation across tiles: a tile reads its neighbours' border
//        cells from the working map as they are and keeps a snapshot of what
//        it read; in the next launch it recomputes only if one of those cells
//        has changed since.  A launch in which no tile changes anything proves
//        the fixed point (every tile's output is then its function of the
//        stable state), so the host launches until a launch's change counter
//        is zero.
// 2. Speckle removal (speckle_filter_new, Solver.cpp:514-566): its output is
//    determined by the 4-connected components of |a-b| < 2 and their sizes,
//    computed with a lock-free union-find: per-tile labelling in LDS, hooks
//    across tile borders in global memory (ECL-CC style: CAS on roots, pointer
//    jumping on non-roots, larger root linked under smaller), per-tile counts
//    folded into the roots' areas, then the area test.
#include <cstdlib>

#include "sgm_device.h"

namespace sgm {
namespace {

constexpr int kMW = 64;        // median tile width: one lane per column
constexpr int kLW = kMW + 4;   // LDS row: two halo columns each side
constexpr int kNoSample = 0x7fff;  // encodes an invalid sample (above any disparity)
// working-map cells a tile of MH rows reads (200 at MH = 16)
constexpr int snap_n(int MH) { return 2 * kMW + 8 + 4 * MH; }

// Batcher's odd-even merge sort for 32 inputs, pruned to 22 (a comparator
// touching a +inf pad is a no-op): 119 compare-exchanges, checked on all
// 2^22 0/1 inputs (0-1 principle).
__device__ __forceinline__ void sort22(int (&f)[22]) {
#define CE(i, j)                              \
    {                                         \
        const int a_ = f[i], b_ = f[j];       \
        f[i] = a_ < b_ ? a_ : b_;             \
        f[j] = a_ < b_ ? b_ : a_;             \
    }
    CE(0, 1);
    CE(2, 3);
    CE(0, 2);
    CE(1, 3);
    CE(1, 2);
    CE(4, 5);
    CE(6, 7);
    CE(4, 6);
    CE(5, 7);
    CE(5, 6);
    CE(0, 4);
    CE(2, 6);
    CE(2, 4);
    CE(1, 5);
    CE(3, 7);
    CE(3, 5);
    CE(1, 2);
    CE(3, 4);
    CE(5, 6);
    CE(8, 9);
    CE(10, 11);
    CE(8, 10);
    CE(9, 11);
    CE(9, 10);
    CE(12, 13);
    CE(14, 15);
    CE(12, 14);
    CE(13, 15);
    CE(13, 14);
    CE(8, 12);
    CE(10, 14);
    CE(10, 12);
    CE(9, 13);
    CE(11, 15);
    CE(11, 13);
    CE(9, 10);
    CE(11, 12);
    CE(13, 14);
    CE(0, 8);
    CE(4, 12);
    CE(4, 8);
    CE(2, 10);
    CE(6, 14);
    CE(6, 10);
    CE(2, 4);
    CE(6, 8);
    CE(10, 12);
    CE(1, 9);
    CE(5, 13);
    CE(5, 9);
    CE(3, 11);
    CE(7, 15);
    CE(7, 11);
    CE(3, 5);
    CE(7, 9);
    CE(11, 13);
    CE(1, 2);
    CE(3, 4);
    CE(5, 6);
    CE(7, 8);
    CE(9, 10);
    CE(11, 12);
    CE(13, 14);
    CE(16, 17);
    CE(18, 19);
    CE(16, 18);
    CE(17, 19);
    CE(17, 18);
    CE(20, 21);
    CE(16, 20);
    CE(18, 20);
    CE(17, 21);
    CE(19, 21);
    CE(17, 18);
    CE(19, 20);
    CE(18, 20);
    CE(19, 21);
    CE(17, 18);
    CE(19, 20);
    CE(0, 16);
    CE(8, 16);
    CE(4, 20);
    CE(12, 20);
    CE(4, 8);
    CE(12, 16);
    CE(2, 18);
    CE(10, 18);
    CE(6, 10);
    CE(14, 18);
    CE(2, 4);
    CE(6, 8);
    CE(10, 12);
    CE(14, 16);
    CE(18, 20);
    CE(1, 17);
    CE(9, 17);
    CE(5, 21);
    CE(13, 21);
    CE(5, 9);
    CE(13, 17);
    CE(3, 19);
    CE(11, 19);
    CE(7, 11);
    CE(15, 19);
    CE(3, 5);
    CE(7, 9);
    CE(11, 13);
    CE(15, 17);
    CE(19, 21);
    CE(1, 2);
    CE(3, 4);
    CE(5, 6);
    CE(7, 8);
    CE(9, 10);
    CE(11, 12);
    CE(13, 14);
    CE(15, 16);
    CE(17, 18);
    CE(19, 20);
#undef CE
}

// k-th smallest (0-based) of the sorted fixed samples f and two more, a <= b:
// the merged order is f[0..ra), a, f[ra..rb), b, f[rb..) with ra = #(f < a),
// rb = #(f < b).  Invalid samples (kNoSample) sort last; k < #valid, so the
// answer is always a valid sample.  sf: this lane's column of the sorted
// samples in LDS (sf[q * 64] = f[q]), read at the three candidate ranks.
__device__ __forceinline__ int kth_merged(const int (&f)[22], const int *sf, int a, int b, int k) {
    int ra = 0, rb = 0;
#pragma unroll
    for (int q = 0; q < 22; ++q) {
        ra += f[q] < a;
        rb += f[q] < b;
    }
    const int x0 = sf[k * 64], x1 = sf[(k - 1) * 64], x2 = sf[(k - 2) * 64];
    return k < ra ? x0 : (k == ra ? a : (k <= rb ? x1 : (k == rb + 1 ? b : x2)));
}

// std::vector<int> v.push_back(float) truncates (Solver.cpp:605,619)
__device__ __forceinline__ int sample(float x, float dmax) { return x <= dmax ? (int)x : kNoSample; }

__device__ __forceinline__ float shfl_up(float x, int d) {
    const int lane = tid_x() & 63;
    return __int_as_float(__builtin_amdgcn_ds_bpermute((lane - d) << 2, __float_as_int(x)));
}

__device__ __forceinline__ int halo_col(int k) { return k < 2 ? k : kMW + k; }  // 0,1,66,67

// MH tile rows (4, 8 or 16; median_rows_default): the tile's rows run in
// order, so a launch's latency is MH row steps per round of resident tiles.
template <int MH>
__global__ __launch_bounds__(64) void median_fill_kernel(const float *__restrict__ orig,
                                                        float *__restrict__ F, int H, int W,
                                                        float dmax, int iter, float *snap,
                                                        int *changes) {
    static_assert(MH >= 2 && 4 * MH <= 64, "halo cells: one lane each");
    constexpr int NOH = 4 * (MH + 2);      // original-map halo cells (4 columns x MH+2 rows)
    __shared__ float O[MH + 4][kLW];       // window grid (rows r0-2 .. r0+MH+1)
    __shared__ float FL[MH][2], FR[MH][2];  // working-map halo columns of the tile rows
    __shared__ float FC[MH][kMW];           // the working map's tile cells (change test)
    __shared__ int SF[22][kMW];             // each lane's sorted fixed samples of the row
    if (iter > 0 && changes[iter - 1] == 0) return;  // the last launch proved the fixed point
    const int tx = bid_x(), ty = bid_y(), ntx = (int)gridDim.x;
    const int tile = ty * ntx + tx;
    const int lane = tid_x();
    const int r0 = ty * MH, c0 = tx * kMW;
    const float out = dmax + 2.f;  // outside the frame: never a sample of an interior window
    auto at = [=](const float *m, int i, int j) {  // branch-free clamped load
        const float v = m[(size_t)clampi(i, 0, H - 1) * W + clampi(j, 0, W - 1)];
        return (i >= 0 && i < H && j >= 0 && j < W) ? v : out;
    };
    // 1. What this tile reads from the working map (raster-earlier cells):
    //    rows r0-2, r0-1 across c0-2..c0+65, and the halo columns c0-2, c0-1,
    //    c0+64, c0+65 of the tile rows.  Unchanged since this tile's last
    //    launch (the snapshot) => its output is still its function of them.
    const int hk = lane & 3;
    const bool hs_lane = lane < 4 * MH;  // lanes holding a tile-row halo cell
    const float h0 = at(F, r0 - 2, c0 + lane), h1 = at(F, r0 - 1, c0 + lane);
    const float hx = at(F, r0 - 2 + ((lane >> 2) & 1), c0 - 2 + halo_col(hk));  // lanes 0..7
    const float hs = at(F, r0 + (lane >> 2), c0 - 2 + halo_col(hk));
    float *sn = snap + (size_t)tile * snap_n(MH);
    if (iter > 0) {
        bool same = __float_as_uint(sn[lane]) == __float_as_uint(h0) &&
                    __float_as_uint(sn[64 + lane]) == __float_as_uint(h1);
        if (hs_lane) same = same && __float_as_uint(sn[136 + lane]) == __float_as_uint(hs);
        if (lane < 8) same = same && __float_as_uint(sn[128 + lane]) == __float_as_uint(hx);
        if (!__ballot(!same)) return;
    }
    sn[lane] = h0;
    sn[64 + lane] = h1;
    if (hs_lane) sn[136 + lane] = hs;
    if (lane < 8) sn[128 + lane] = hx;
    // 2. The tile rows and the two rows below start as the original map
    //    (raster-later cells), plus the working map's own cells.
    float ov[MH + 2], fc[MH], oh[2];
#pragma unroll
    for (int r = 0; r < MH + 2; ++r) ov[r] = at(orig, r0 + r, c0 + lane);
#pragma unroll
    for (int r = 0; r < MH; ++r) fc[r] = at(F, r0 + r, c0 + lane);
#pragma unroll
    for (int q = 0; q < 2; ++q)  // 4 halo columns x MH+2 rows
        oh[q] = at(orig, r0 + (lane + 64 * q) / 4, c0 - 2 + halo_col(hk));
    O[0][lane + 2] = h0;
    O[1][lane + 2] = h1;
    if (lane < 8) O[lane >> 2][halo_col(hk)] = hx;
    if (hs_lane) {
        if (hk < 2) FL[lane >> 2][hk] = hs; else FR[lane >> 2][hk - 2] = hs;
    }
#pragma unroll
    for (int r = 0; r < MH + 2; ++r) O[r + 2][lane + 2] = ov[r];
#pragma unroll
    for (int r = 0; r < MH; ++r) FC[r][lane] = fc[r];
#pragma unroll
    for (int q = 0; q < 2; ++q)
        if (lane + 64 * q < NOH) O[2 + (lane + 64 * q) / 4][halo_col(hk)] = oh[q];
    __syncthreads();

    const int j = c0 + lane, lc = lane + 2;
    bool changed_any = false;
    for (int r = 0; r < MH; ++r) {
        const int i = r0 + r, lr = r + 2;
        if (i >= H) break;
        if (lane < 2) O[lr][lane] = FL[r][lane];   // (i, c0-2..c0-1) precede (i, c0)
        __syncthreads();
        const float own = O[lr][lc];
        const bool active = i >= 2 && i <= H - 3 && j >= 2 && j <= W - 3 && !(own <= dmax);
        float cur = own;
        if (__ballot(active)) {
            int fixed[22];
#pragma unroll
            for (int dr = 0; dr < 5; ++dr) {
                if (dr == 2) continue;
#pragma unroll
                for (int dc = 0; dc < 5; ++dc)
                    fixed[(dr < 2 ? dr : dr - 1) * 5 + dc] = sample(O[lr - 2 + dr][lc - 2 + dc], dmax);
            }
            fixed[20] = sample(O[lr][lc + 1], dmax);
            fixed[21] = sample(O[lr][lc + 2], dmax);
            const float halo1 = O[lr][lc - 1], halo2 = O[lr][lc - 2];  // used by lanes 0, 1
            int nfixed = 0;
#pragma unroll
            for (int q = 0; q < 22; ++q) nfixed += fixed[q] != kNoSample;
            // a fill needs more than 12 samples: with at most 2 chained ones,
            // lanes with <= 10 fixed samples can never fill
            if (__ballot(active && nfixed > 10)) {
                sort22(fixed);
#pragma unroll
                for (int q = 0; q < 22; ++q) SF[q][lane] = fixed[q];
            }
            // the in-row chain: iterate the row to its fixed point
            for (int it = 0; it <= kMW; ++it) {
                const float u1 = shfl_up(cur, 1), u2 = shfl_up(cur, 2);
                const float l1 = lane >= 1 ? u1 : halo1;
                const float l2 = lane >= 2 ? u2 : halo2;
                const int s1 = sample(l1, dmax), s2 = sample(l2, dmax);
                const int cnt = nfixed + (s1 != kNoSample) + (s2 != kNoSample);
                float nv = own;
                if (active && cnt > 12)
                    nv = (float)kth_merged(fixed, &SF[0][lane], s1 < s2 ? s1 : s2,
                                           s1 < s2 ? s2 : s1, cnt / 2);
                const bool diff = __float_as_uint(nv) != __float_as_uint(cur);
                cur = nv;
                if (!__ballot(diff)) break;
            }
        }
        if (lane < kMW) O[lr][lc] = cur;
        if (lane < 2) O[lr][kMW + 2 + lane] = FR[r][lane];  // row i now precedes row i+1
        if (active) {
            if (__float_as_uint(FC[r][lane]) != __float_as_uint(cur)) {
                F[(size_t)i * W + j] = cur;
                changed_any = true;
            }
        }
        __syncthreads();
    }
    const bool any = __ballot(changed_any) != 0;  // whole wave: not under the lane test
    if (lane == 0 && any) atomicAdd(changes + iter, 1);
}

// ------------------------------------------------------------ speckle / CC

constexpr int kCW = 64, kCH = 16, kCN = kCW * kCH;  // CC tile: 64 x 16 pixels, 256 threads

__device__ __forceinline__ bool joined(float a, float b) { return fabsf(a - b) < 2.f; }  // :527-543

// Roots are the smallest index of their tree (the larger root is linked under
// the smaller), so path rewrites are atomicMin and only ever move an entry
// towards its root (see g_find).
__device__ int lds_find(int *lab, int x) {
    int cur = __atomic_load_n(lab + x, __ATOMIC_RELAXED);
    if (cur != x) {
        int prev = x, next;
        while (cur > (next = __atomic_load_n(lab + cur, __ATOMIC_RELAXED))) {
            atomicMin(lab + prev, next);
            prev = cur;
            cur = next;
        }
    }
    return cur;
}

__device__ void lds_union(int *lab, int a, int b) {
    for (;;) {
        a = lds_find(lab, a);
        b = lds_find(lab, b);
        if (a == b) return;
        if (a > b) { const int t = a; a = b; b = t; }
        const int old = atomicMin(lab + b, a);  // link the larger root under the smaller
        if (old == b) return;
        b = old;
    }
}

// Root of x with intermediate pointer jumping (ECL-CC): only non-root entries
// are rewritten, each to one of its ancestors.  A root is the smallest index
// of its tree (hooks link the larger root under the smaller), so every
// rewrite is an atomicMin: concurrent jumps and the final flattening can only
// lower an entry towards its root, never raise it back above.
__device__ int g_find(int *L, int x) {
    int cur = __atomic_load_n(L + x, __ATOMIC_RELAXED);
    if (cur != x) {
        int prev = x, next;
        while (cur > (next = __atomic_load_n(L + cur, __ATOMIC_RELAXED))) {
            atomicMin(L + prev, next);
            prev = cur;
            cur = next;
        }
    }
    return cur;
}

__device__ void g_hook(int *L, int a, int b) {
    a = g_find(L, a);
    b = g_find(L, b);
    while (a != b) {
        if (a < b) {
            const int ret = atomicCAS(L + b, b, a);
            if (ret == b) return;
            b = ret;
        } else {
            const int ret = atomicCAS(L + a, a, b);
            if (ret == a) return;
            a = ret;
        }
        a = g_find(L, a);
        b = g_find(L, b);
    }
}

// Per-tile labelling: L[k] = global index of k's tile-local root, cnt[k] =
// pixels under k if k is a tile-local root, else 0.  Each wave labels whole
// tile rows (lane = column): the joined-with-left mask is one ballot and a
// pixel's run start is the highest run break at or below its lane, so row runs
// need no union at all; runs of adjacent rows are then joined once per
// contiguous overlap.
__global__ __launch_bounds__(256) void cc_local_kernel(const float *__restrict__ F, int H, int W,
                                                      int *__restrict__ L, int *__restrict__ cnt,
                                                      int *__restrict__ area) {
    __shared__ int lab[kCN];
    __shared__ int num[kCN];
    __shared__ float val[kCN];
    __shared__ unsigned long long hjoin[kCH];  // bit l: (row, l) joined with (row, l-1)
    const int r0 = bid_y() * kCH, c0 = bid_x() * kCW, t = tid_x();
    const int lane = t & 63, wave = t >> 6;
    const int j = c0 + lane;
    for (int r = wave; r < kCH; r += 4) {
        const int i = r0 + r, p = r * kCW + lane;
        val[p] = (i < H && j < W) ? F[(size_t)i * W + j] : 0.f;
        num[p] = 0;
        if (i < H && j < W) area[(size_t)i * W + j] = 0;  // areas are indexed by root pixel
    }
    __syncthreads();
    for (int r = wave; r < kCH; r += 4) {
        const int i = r0 + r, p = r * kCW + lane;
        const bool in = i < H && j < W;
        const bool jl = in && lane > 0 && joined(val[p], val[p - 1]);
        const unsigned long long m = __ballot(jl);
        const unsigned long long brk = ~m & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
        lab[p] = r * kCW + 63 - __builtin_clzll(brk);
        if (lane == 0) hjoin[r] = m;
    }
    __syncthreads();
    for (int r = wave; r < kCH; r += 4) {
        if (r == 0) continue;
        const int i = r0 + r, p = r * kCW + lane;
        if (i >= H || j >= W) continue;
        if (!joined(val[p], val[p - kCW])) continue;
        // the same pair of runs was joined one column to the left
        const unsigned long long bit = 1ull << lane;
        if (lane > 0 && (hjoin[r] & bit) && (hjoin[r - 1] & bit) &&
            joined(val[p - 1], val[p - 1 - kCW]))
            continue;
        lds_union(lab, p, p - kCW);
    }
    __syncthreads();
    for (int r = wave; r < kCH; r += 4) {
        const int i = r0 + r, p = r * kCW + lane;
        if (i >= H || j >= W) continue;
        const int root = lds_find(lab, p);
        atomicAdd(num + root, 1);
        L[(size_t)i * W + j] = (r0 + root / kCW) * W + c0 + root % kCW;
    }
    __syncthreads();
    for (int r = wave; r < kCH; r += 4) {
        const int i = r0 + r, p = r * kCW + lane;
        if (i < H && j < W) cnt[(size_t)i * W + j] = num[p];
    }
}

// Hooks across the tile's left and top borders.
__global__ __launch_bounds__(128) void cc_merge_kernel(const float *__restrict__ F, int H, int W,
                                                      int *L) {
    const int r0 = bid_y() * kCH, c0 = bid_x() * kCW, t = tid_x();
    // A hook is skipped when the previous pixel pair along the border was
    // joined across it and each side is joined to it inside its own tile:
    // both sides then already belong to the hooked pair's components.
    if (t < kCW) {  // top border: (r0-1, j) -- (r0, j)
        const int j = c0 + t;
        if (r0 > 0 && j < W) {
            const int a = (r0 - 1) * W + j, b = r0 * W + j;
            if (joined(F[a], F[b]) &&
                !(t > 0 && joined(F[a - 1], F[b - 1]) && joined(F[a - 1], F[a]) &&
                  joined(F[b - 1], F[b])))
                g_hook(L, a, b);
        }
    } else if (t < kCW + kCH) {  // left border: (i, c0-1) -- (i, c0)
        const int r = t - kCW, i = r0 + r;
        if (c0 > 0 && i < H) {
            const int b = i * W + c0, a = b - 1;
            if (joined(F[a], F[b]) &&
                !(r > 0 && joined(F[a - W], F[b - W]) && joined(F[a - W], F[a]) &&
                  joined(F[b - W], F[b])))
                g_hook(L, a, b);
        }
    }
}

// Tile-local roots: flatten to the final root and add their pixel counts.
// Only area <= max_size matters to the test (cc_apply_kernel), and an area
// only grows, so a root already read above max_size (even through a stale
// line: a stale value is an older, smaller one) takes no more adds: the tile
// roots of a frame-wide component (a road) no longer all add into one word.
__global__ __launch_bounds__(256) void cc_count_kernel(int *L, const int *__restrict__ cnt,
                                                      int *area, int n, int max_size) {
    const int k = bid_x() * 256 + tid_x();
    if (k >= n) return;
    const int c = cnt[k];
    if (c == 0) return;
    const int root = g_find(L, k);
    atomicMin(L + k, root);
    if (__hip_atomic_load(area + root, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= max_size)
        atomicAdd(area + root, c);
}

// speckle_filter_new's last loop (:556-565): components of at most max_size
// pixels become `value` (invalid_disp).
__global__ __launch_bounds__(256) void cc_apply_kernel(const float *__restrict__ F,
                                                      const int *__restrict__ L,
                                                      const int *__restrict__ area, int n, int W,
                                                      int max_size, float value,
                                                      float *__restrict__ out, int out_pitch) {
    const int k = bid_x() * 256 + tid_x();
    if (k >= n) return;
    const int root = L[L[k]];  // L[k] is a (former) tile-local root, now flattened
    out[(size_t)(k / W) * out_pitch + k % W] = area[root] <= max_size ? value : F[k];
}

// Entry of a post filter: the map (pitched) into the original and working
// copies, and the fill's per-launch change counters zeroed.
__global__ __launch_bounds__(256) void pf_prep_kernel(const float *__restrict__ map, int pitch,
                                                     int H, int W, float *__restrict__ orig,
                                                     float *__restrict__ F, int *changes,
                                                     int nchanges) {
    const int k = bid_x() * 256 + tid_x();
    if (k < nchanges) changes[k] = 0;
    if (k >= H * W) return;
    const float v = map[(size_t)(k / W) * pitch + k % W];
    orig[k] = v;
    F[k] = v;
}

}  // namespace

// Tile rows of the fill (read when a handle is created).  A launch takes
// about MH row steps per round of tiles the chip holds at once (one wave each,
// ~4k resident), so short tiles pay while their count stays within a round:
// 4 rows when ceil(W/64) x ceil(H/4) <= 4096 tiles (K128: 43 vs 58 us at 8
// rows per frame), else 8 (4K: 121 us; 150 at 4 rows, 149 at 16;
// profiles/r03_experiments/median_tiles.txt).  SGM_MF_ROWS=4/8/16 forces it.
int median_rows_default(Geom g) {
    const char *e = std::getenv("SGM_MF_ROWS");
    const int r = e ? std::atoi(e) : 0;
    if (r == 4 || r == 8 || r == 16) return r;
    return (size_t)((g.W + kMW - 1) / kMW) * ((g.H + 3) / 4) <= 4096 ? 4 : 8;
}

size_t post_snapshot_floats(Geom g) {  // enough for any tile height
    const size_t tx = (size_t)(g.W + kMW - 1) / kMW;
    size_t n = 0;
    for (int mh : {4, 8, 16}) {
        const size_t m = tx * ((g.H + mh - 1) / mh) * snap_n(mh);
        n = m > n ? m : n;
    }
    return n;
}

template <int MH>
static void launch_mf(const float *orig, float *F, int iter, float *snap, int *changes, Geom g,
                      hipStream_t st) {
    median_fill_kernel<MH><<<dim3((g.W + kMW - 1) / kMW, (g.H + MH - 1) / MH), 64, 0, st>>>(
        orig, F, g.H, g.W, (float)(g.D - 1), iter, snap, changes);
}

hipError_t launch_median_fill(const float *orig, float *F, int iter, float *snap, int *changes,
                              int rows, Geom g, hipStream_t st) {
    if (rows == 16) launch_mf<16>(orig, F, iter, snap, changes, g, st);
    else if (rows == 4) launch_mf<4>(orig, F, iter, snap, changes, g, st);
    else launch_mf<8>(orig, F, iter, snap, changes, g, st);
    return hipGetLastError();
}

hipError_t launch_pf_prep(const float *map, int pitch, float *orig, float *F, int *changes,
                          int nchanges, Geom g, hipStream_t st) {
    const int n = g.H * g.W > nchanges ? g.H * g.W : nchanges;
    hipLaunchKernelGGL(pf_prep_kernel, dim3((n + 255) / 256), dim3(256), 0, st, map, pitch, g.H,
                       g.W, orig, F, changes, nchanges);
    return hipGetLastError();
}

hipError_t launch_cc_local(const float *F, int *L, int *cnt, int *area, Geom g, hipStream_t st) {
    const dim3 grid((g.W + kCW - 1) / kCW, (g.H + kCH - 1) / kCH);
    hipLaunchKernelGGL(cc_local_kernel, grid, dim3(256), 0, st, F, g.H, g.W, L, cnt, area);
    return hipGetLastError();
}

hipError_t launch_cc_merge(const float *F, int *L, Geom g, hipStream_t st) {
    const dim3 grid((g.W + kCW - 1) / kCW, (g.H + kCH - 1) / kCH);
    hipLaunchKernelGGL(cc_merge_kernel, grid, dim3(128), 0, st, F, g.H, g.W, L);
    return hipGetLastError();
}

hipError_t launch_cc_count(int *L, const int *cnt, int *area, int max_size, Geom g,
                           hipStream_t st) {
    const int n = g.H * g.W;
    hipLaunchKernelGGL(cc_count_kernel, dim3((n + 255) / 256), dim3(256), 0, st, L, cnt, area, n,
                       max_size);
    return hipGetLastError();
}

hipError_t launch_cc_apply(const float *F, const int *L, const int *area, int max_size,
                           float value, float *out, int out_pitch, Geom g, hipStream_t st) {
    const int n = g.H * g.W;
    hipLaunchKernelGGL(cc_apply_kernel, dim3((n + 255) / 256), dim3(256), 0, st, F, L, area, n,
                       g.W, max_size, value, out, out_pitch);
    return hipGetLastError();
}

}  // namespace sgm
