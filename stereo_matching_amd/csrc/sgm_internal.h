// sgm_internal.h -- kernel launchers shared by the C-ABI (sgm_capi.hip) and
// the kernels (sgm_kernels.hip).  Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sgm {

// Floats of slack after the final cost volume: row-walking prefetch rings may
// read up to 64 positions (x D <= 256) past the last row's end.
constexpr size_t kVolGuard = 64 * 256 + 256;

// Disparities per lane of a wave64 chain (lane l holds d = l*V .. l*V+V-1).
constexpr int vals_per_lane(int D) { return D >= 256 ? 4 : (D >= 128 ? 2 : 1); }

// Segment lengths K (chain steps between checkpoints) of the pair families,
// by values per lane.  The one definition: the kernels' pair_k<V>() /
// pair_kv<V>() (sgm_bodies.h), the checkpoint allocation (pair_ckpt_floats)
// and the guard below all derive from these.  The vertical family's final
// kernel holds five K x V register arrays, so it uses a shorter K to stay at
// <= 128 VGPRs (four waves per SIMD).
constexpr int seg_k_hd(int V) { return V >= 4 ? 8 : 16; }   // PAIR_H, PAIR_D2
constexpr int seg_k_v(int V) { return V >= 4 ? 4 : 8; }     // PAIR_V

// Rows of slack before the T volume read by the final pass (pair_split_body's
// WTA waves load a chunk from its top row; the partial last chunk's top lies
// up to K-1 rows above row 0, K = the vertical family's segment length).
constexpr int t_guard_rows(int D) { return seg_k_v(vals_per_lane(D)) - 1; }

// Geometry of one frame on the working (decimated) grid.
struct Geom {
    int H, W, D;   // rows, cols, disparities
    int scale;     // 1 or 2
};

// What a sweep does with its path costs L_r ("Sweeps").
enum SweepMode {
    SWEEP_STORE_L = 0,  // write L_r and minL_r (parity tests)
    SWEEP_INIT = 1,     // acc_out = L_r
    SWEEP_ACC = 2,      // acc_out = acc_in + L_r   (acc_in may alias acc_out)
    SWEEP_FINAL = 3     // (retired: the final pass is the PAIR_V backward kernel)
};

// A band of a backward pass: chain steps [kb, ke) of every chain (the rows
// H-ke .. H-1-kb of the walks that start at the bottom row), the chain state
// entering the band read from carry (kb > 0) and the state leaving it written
// there (ke < chain length; carry holds D floats per chain).  ke = 0: the
// whole chain.  The backward phase (stage B's diagonal pair, L8, final) runs
// band by band above the Infinity Cache, so that a band's cost volume and T
// stay cached from one pass to the next (DESIGN.md "Bands").
// Forward passes run bands too (rows [kb, ke) walked down, top band first:
// vfwd, L5, L6), with the same edges.
struct Band {
    int kb, ke;
    float *carry;
};

struct SweepArgs {
    const float *cost;   // HWD
    const float *acc_in; // HWD (ACC: chain state; FINAL: T chain)
    float *acc_out;      // HWD (STORE_L: L_r)
    const float *s_in;   // HWD (FINAL: S chain)
    float *min_out;      // HW  (STORE_L: minL_r)
    uint16_t *disp;      // HW  (FINAL)
    float *sub;          // HW  (FINAL)
    float p1, p2, uniq;
    Band band;           // backward diagonal sweeps (DIR 6, 7: the L8 pass)
};

// Scanline families fused into forward/backward pairs (DESIGN.md "Pairs"):
// the forward direction stores its path state every K steps (checkpoints),
// the backward kernel recomputes each K-step segment of the forward costs from
// its checkpoint in registers and combines both on the fly.
enum PairFamily {
    PAIR_H = 0,   // L1 (->) forward, L2 (<-) backward, one chain per row
    PAIR_V = 1,   // L3 (down) forward, L4 (up) backward, one chain per column
    PAIR_D2 = 2   // L6 (down-left) forward, L7 (up-right) backward, wrapped anti-diagonals
};
enum PairMode {
    PAIR_INIT2 = 0,  // out = Lf + Lb                         (S12 = L1 + L2)
    PAIR_ACC = 1,    // out = (acc_in + Lf) + Lb              (T = (T5 + L6) + L7)
    PAIR_FINAL = 2   // total = ((s_in + Lf) + Lb) + acc_in   (S + T) -> WTA, sub-pixel
};

struct PairArgs {
    const float *cost;
    const float *acc_in;
    const float *s_in;
    float *out;
    float *ckpt;
    uint16_t *disp;      // FINAL: raw WTA map, row-major (null: not wanted)
    float *sub;          // FINAL: sub-pixel map, row-major or (sub_cm) column-major
    int sub_cm;          // 1: sub[col * H + row] (two-view frames: lr_cm_kernel reads it)
    const float *zero;   // >= 256 zero floats: the cost of the virtual positions
                         // that align forward passes with their checkpoints
    float p1, p2, uniq;
    Band band;           // backward passes (D2 ACC, V FINAL): steps in whole segments
    int nt_cost;         // V FINAL (whole volume): read C by non-temporal loads -- the
                         // last read of a view's C when the other view's follows
};

// floats of checkpoint storage a family needs
size_t pair_ckpt_floats(int family, Geom g);
hipError_t launch_pair_fwd(int family, const PairArgs &a, Geom g, hipStream_t st);
hipError_t launch_pair_bwd(int family, int mode, const PairArgs &a, Geom g, hipStream_t st);
// both views' vfwd writing C and L3 (the slanted schedule), workgroup y = view
hipError_t launch_vfwd2_l3(const float *const *in, float *const *out, float *const *l3, const PairArgs *a,
                           Geom g, hipStream_t st);
// both views' vfwd (C and the L3 checkpoints, a[v].ckpt) in one launch
hipError_t launch_vfwd2(const float *const *in, float *const *out, const PairArgs *a, Geom g, hipStream_t st);
// the PAIR_V/PAIR_FINAL pass of two views in one launch
hipError_t launch_final2(const PairArgs &a0, const PairArgs &a1, Geom g, hipStream_t st);
// cost_vertical_filter (Solver.cpp:333-368) fused with the L3 forward pass:
// in = horizontally filtered volume, out = final cost volume, a.ckpt = L3
// checkpoints.
// Multi-role launches of the frame schedule (sgm_pair.hip); banded stage B
// launches (d7.band) run no H rows (the banded schedule's H pair is its own
// launch)
hipError_t launch_stage_a(const PairArgs &h1, const SweepArgs &l5, const PairArgs &d6, Geom g,
                          hipStream_t st);
hipError_t launch_stage_b(const PairArgs &h2, const PairArgs &d7, Geom g, hipStream_t st);
// both views' stage A / stage B / L8 sweep in one launch each (grid.y = view;
// arrays of two)
hipError_t launch_stage_a2(const PairArgs *h1, const SweepArgs *l5, const PairArgs *d6, Geom g,
                           hipStream_t st);
hipError_t launch_stage_b2(const PairArgs *h2, const PairArgs *d7, Geom g, hipStream_t st);
hipError_t launch_sweep2_l8(const SweepArgs &a0, const SweepArgs &a1, Geom g, hipStream_t st);
// the forward bands (DESIGN.md "Bands"): the whole H pair (L1 fwd, then L2
// bwd -> h2[v].out) of nviews views as one launch, and one band (l5.band, d6.band)
// of stage A's diagonal roles (L5 -> T5, L6 fwd)
hipError_t launch_stage_a_hpair(const PairArgs *h1, const PairArgs *h2, int nviews, Geom g,
                                hipStream_t st);
hipError_t launch_stage_a_band(const SweepArgs &l5, const PairArgs &d6, Geom g, hipStream_t st);
hipError_t launch_vfwd(const float *in, float *out, const PairArgs &a, Geom g, hipStream_t st);
// the same vertical IIR + L3, writing every row's L3 to the volume l3 (the
// slanted schedule's bottom-up pass reads it) instead of checkpoints
hipError_t launch_vfwd_l3(const float *in, float *out, float *l3, const PairArgs &a, Geom g,
                          hipStream_t st);

// ----------------------------------------------- slanted tiles (sgm_slant.hip)
// Compute waves per tile; one more wave per workgroup, the receiver, turns
// the next tile's exit-state granules into LDS states (the compute waves 0
// and 1 store this tile's own exit states themselves).
// The bottom-up pass's tiles are 15 columns wide (16 waves, the workgroup
// maximum): its hand-off granules cost 3 / NW of a tile-step's bytes, and
// slant_up ran 3.9-4.0% faster at HD256 with 15 than with 14; the top-down
// pass keeps 14 (with 15 the H pair beside it lost more than it gained,
// profiles/r06_experiments/r06l_tile_width.txt).
constexpr int kSlantNW = 14;     // top-down
constexpr int kSlantNWUp = 15;   // bottom-up
// Polls before a receiver gives up on a hand-off (a hang guard: seconds).
constexpr unsigned kSlantSpinLimit = 1u << 22;
// Launch bookkeeping of one slanted pass kind, in device memory (zeroed at
// create): tickets claim tiles, the last workgroup out resets tickets/exits
// and advances epoch (the hand-off granules' tag), err counts hang-guard
// give-ups, dead = epoch + 1 of the last launch in which a receiver gave up
// (every later poll of that launch skips its wait, so one dead neighbour
// costs one spin limit, not one per step).
struct SlantCtl {
    unsigned tickets, exits, epoch, err, dead;
};
struct SlantView {
    const float *cost, *s12, *l3, *t56;  // HWD: C, L1+L2, L3, L5+L6 (bottom-up reads)
    float *t56w;                         // HWD: L5+L6 (the top-down pass writes it)
    float *sub;                          // HW sub-pixel map, row-major
    uint16_t *disp;                      // HW raw WTA map (null: not wanted)
    unsigned long long *gran;            // hand-off granules, slant_gran_count
};
struct SlantArgs {
    SlantView v[2];
    SlantCtl *ctl;
    const float *zero;  // >= 256 zero floats
    float *dummy;       // >= 258 words: the target of inactive steps' stores
    float p1, p2, uniq;
    int nviews;
    int ntiles, grid;   // set by the launcher
    int max_grid;       // workgroups at most (0: one per CU)
    unsigned *err_host; // host-mapped word set to 1 when a hand-off poll gives up
    unsigned spin_limit;  // polls before giving up (kSlantSpinLimit; SGM_SLANT_DEBUG:
                          // SGM_SLANT_SPIN_LIMIT)
    int stall_tile;       // SGM_SLANT_DEBUG only (SGM_SLANT_STALL): the bottom-up pass's
                          // receiver of this tile of view 0 never accepts a granule, to
                          // exercise the give-up path; -1: none
};
size_t slant_tiles(Geom g, int nw);
// granules (8 B each) of nviews views' hand-offs
size_t slant_gran_count(Geom g, int nviews);
// both views' (a.nviews) bottom-up slanted pass: L4 + L7 + L8 + WTA (ctl[1])
hipError_t launch_slant_up(const SlantArgs &a, Geom g, hipStream_t st);
// both views' top-down slanted pass: T56 = L5 + L6 (ctl[0])
hipError_t launch_slant_down(const SlantArgs &a, Geom g, hipStream_t st);

// bm_rows: BM.cpp:24-25 decimation (rows not strided by the scale); src2/ct2:
// a second image censused in the same launch
hipError_t launch_census(const uint8_t *src, int pitch, Geom g, int blur, uint64_t *ct,
                         hipStream_t st, bool bm_rows = false, const uint8_t *src2 = nullptr,
                         uint64_t *ct2 = nullptr);
// BM's WTA (BM.cpp:53-85) over the filtered cost: raw disparity + its float copy
hipError_t launch_bm_wta(const float *cost, float uniq, uint16_t *disp, float *out, int out_pitch,
                         Geom g, hipStream_t st);
// both views' DSI + horizontal IIR in one launch (both sky masks or neither);
// cost_h2_supported: false when rows do not fit the staged kernel
bool cost_h2_supported(Geom g, bool sky);
hipError_t launch_cost_h2(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky0,
                          const uint8_t *sky1, int sky_pitch, Geom g, float *out0, float *out1,
                          hipStream_t st);
hipError_t launch_cost_h(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
                         int sky_pitch, int view, int filter, Geom g, float *out,
                         hipStream_t st);
// The strip schedule of the slanted frames' cost stage (sgm_vstrip.hip):
// a checkpoint pass of the horizontal IIR (launch_cost_ck, sgm_cost.hip),
// then one pass writing C and the L3 volume (launch_vstrip).  kVStripNC
// columns per strip; checkpoints: H x strips x 3 x D floats per view.
#ifndef VSTRIP_NC
#define VSTRIP_NC 16
#endif
constexpr int kVStripNC = VSTRIP_NC;
struct VStripArgs {
    const uint64_t *ctl, *ctr;  // census words (left, right image)
    const uint64_t *skw0, *skw1; // per view slot: sky flags, one word per pixel (null: no mask)
    int dsi0, dsi1;             // slot's DSI: 0 left view, 1 right view
    const float *ck0, *ck1;     // checkpoints (launch_cost_ck)
    float *c0, *c1;             // final cost C
    float *l30, *l31;           // L3 volume
    float *dummy;               // >= 256 floats: the target of idle stores
    float p1, p2;
};
size_t vstrip_strips(Geom g);
size_t vstrip_ck_floats(Geom g);
bool vstrip_supported(Geom g, bool sky);
hipError_t launch_cost_ck(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky0,
                          const uint8_t *sky1, int sky_pitch, int dsi0, int dsi1, int nviews, Geom g,
                          float *ck0, float *ck1, hipStream_t st);
hipError_t launch_vstrip(const VStripArgs &a, int nviews, Geom g, hipStream_t st);
// the sky mask as 0/1 words (the strip pass stages 8-byte words only), kept
// in the Ch buffer after the checkpoints (offset in floats)
size_t vstrip_sky_words_offset(Geom g);
hipError_t launch_sky_words(const uint8_t *sky, int pitch, Geom g, uint64_t *out, hipStream_t st);
hipError_t launch_copy(const float *in, float *out, Geom g, hipStream_t st);
hipError_t launch_sweep(int dir, int mode, const SweepArgs &a, Geom g, hipStream_t st);
// post_filter (sgm_post.hip)
size_t post_snapshot_floats(Geom g);
int median_rows_default(Geom g);
hipError_t launch_median_fill(const float *orig, float *F, int iter, float *snap, int *changes,
                              int rows, Geom g, hipStream_t st);
hipError_t launch_pf_prep(const float *map, int pitch, float *orig, float *F, int *changes,
                          int nchanges, Geom g, hipStream_t st);
hipError_t launch_cc_local(const float *F, int *L, int *cnt, int *area, Geom g, hipStream_t st);
hipError_t launch_cc_merge(const float *F, int *L, Geom g, hipStream_t st);
hipError_t launch_cc_count(int *L, const int *cnt, int *area, int max_size, Geom g,
                           hipStream_t st);
hipError_t launch_cc_apply(const float *F, const int *L, const int *area, int max_size,
                           float value, float *out, int out_pitch, Geom g, hipStream_t st);
// LKRefine (sgm_lk.hip): left/right full-size images (decimated by g.scale on
// the fly), din the working-grid map, dout (pitched) the refined map.
hipError_t launch_lk_refine(const uint8_t *left, const uint8_t *right, int pitch, const float *din,
                            float *dout, int out_pitch, Geom g, hipStream_t st);
// SkyAreaDetector::detect (sgm_sky.hip) on nviews (1 or 2) images at once:
// img[v] full-size (decimated by g.scale), mask[v] on the working grid;
// scratch of nviews * sky_scratch_bytes(g) bytes.
size_t sky_scratch_bytes(Geom g);
hipError_t launch_sky_detect(const uint8_t *const *img, int pitch, uint8_t *const *mask,
                             int mask_pitch, void *scratch, int nviews, Geom g, hipStream_t st);
// consumers (sgm_consumers.hip): Solver::colormap and the node's point cloud
hipError_t launch_colormap(const float *disp, int pitch, uint8_t *bgr, int bgr_pitch, Geom g,
                           hipStream_t st);
hipError_t launch_point_cloud(const float *disp, int pitch, const uint8_t *img, int img_pitch,
                              float fx, float fy, float cx, float cy, double baseline,
                              float max_range, int *counts, double *xyz, uint8_t *pixel,
                              int *total, Geom g, hipStream_t st);
hipError_t launch_lr(const float *fl, int fl_pitch, const float *fr, int fr_pitch, float *out,
                     int out_pitch, float lr, Geom g, hipStream_t st);
// the same LR check on COLUMN-major maps fl_cm, fr_cm (x[col * H + row], as
// the two-view frame's final passes write them), row-major out
hipError_t launch_lr_cm(const float *fl_cm, const float *fr_cm, float *out, int out_pitch, float lr,
                        Geom g, hipStream_t st);

}  // namespace sgm
