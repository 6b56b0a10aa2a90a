// sgm_capi.hip -- the C-ABI of libsgm_hip.so (include/sgm_hip.h).
//
// Host orchestration of one view (DESIGN.md "Frame schedule"), 73.5 B of HBM
// traffic per pixel-disparity, six launches on one stream:
//
//   census L,R -> cost_h -> vfwd (vertical IIR + L3 checkpoints)
//   -> stage A (L1 fwd | L5 | L6 fwd) -> stage B (L2 bwd | L7 bwd) -> L8
//   -> final (L4 bwd recomputing L3, sum, WTA, sub-pixel)
//
// Concurrency between independent roles comes from sharing a launch (stage
// A/B), not from streams (the runtime may map streams onto one hardware
// queue).  The right view runs on a second stream; then the LR check.
// All device memory is allocated at sgm_create (the reference allocates its
// scratch in the constructors, Solver.cpp:18-27 and SGM.cpp:7-24).
#include "../../include/sgm_hip.h"
#include "sgm_internal.h"

#include <algorithm>
#include <float.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <new>
#include <vector>

using sgm::Geom;
using sgm::SweepArgs;

struct sgm_handle {
    sgm_params p;
    Geom g;
    int device;
    int nviews;
    size_t bytes;
    hipStream_t st;       // the handle's own stream (host API, stages)
    hipEvent_t ev_pf;     // the post filter's convergence readback
    hipEvent_t ev_last;   // the end of the last call's work on last_st (StreamScope)
    hipStream_t last_st;  // the stream of the last entry point's work (null: none yet)
    bool last_recorded;   // ev_last was recorded at the end of that call (a caller's stream)
    uint8_t *d_in[2];     // full-size input staging (host API)
    uint8_t *d_sky[2];    // working-grid sky masks (host API / stages)
    uint64_t *d_ct[2];    // census words
    float *d_ch[2];       // horizontally filtered cost; reused as the T chain
    float *d_ch_base[2];  // its allocation: d_ch is preceded by t_guard_rows rows (final pass)
    float *d_c[2];        // final cost volume (+ kVolGuard: row-walking prefetch rings)
    float *d_s[2];        // S chain
    uint16_t *d_disp[2];  // WTA disparity
    float *d_sub[2];      // sub-pixel disparity
    float *d_out;         // LR-checked output (host API)
    float *d_min;         // minL (stage_path)
    float *d_zero;        // 256 zero floats (PairArgs::zero)
    float *d_ck[2][3];    // checkpoints per view and pair family (H, V, D2)
    float *d_carry[2][3]; // banded backward passes: chain state at band edges (L7, L8, L4)
    bool slant;           // the slanted-tile schedule (sgm_slant.hip, DESIGN.md "Slanted tiles")
    bool vstrip;          //   its cost stage as checkpoints + strips (sgm_vstrip.hip; SGM_VSTRIP=0: off)
    float *d_l3[2];       // slant: the full L3 volume per view
    unsigned long long *d_gran;  // slant: hand-off granules (both views)
    sgm::SlantCtl *d_slant_ctl;  // slant: launch bookkeeping of the passes
    float *d_slant_dummy;        // slant: the target of inactive lanes' stores
    int band_rows;        // rows per band of the backward phase (0: whole volume)
    int mf_rows;          // median fill tile rows (4 or 8 by frame size; SGM_MF_ROWS)
    // post_filter scratch (sgm_post.hip)
    float *d_pf_orig;     // the map as it entered the median fill
    float *d_pf_work;     // contiguous working map (pitched callers)
    int *d_pf_label;      // union-find parents
    int *d_pf_count;      // pixels under each tile-local root
    int *d_pf_area;       // component sizes
    float *d_pf_snap;     // per median tile: the working-map cells it last read
    int *d_pf_changes;    // per median launch: tiles that changed a pixel
    int *h_pf_changes;    // pinned readback of one counter
    unsigned *h_slant_err;  // slant: host-mapped hang-guard word (SlantArgs::err_host)
    hipStream_t st_h;       // slant: the H pair's stream, beside the top-down pass
    hipEvent_t ev_fork, ev_join;  //   its fork from / join into the frame's stream
    unsigned *d_slant_err;  //   its device-side address
    int pf_iters;         // median launches of the last post filter
    float *d_lk_in;       // LKRefine input copy (the kernel refines the map in place)
    uint8_t *d_sky_scratch;  // sky detector scratch (sgm_sky.hip)
    int *d_cloud_counts;  // point cloud: per-row counts -> offsets, then the total
    uint8_t *h_pin;       // pinned host staging for sgm_process (allocated on first use)
    size_t h_pin_bytes;
    char err[512];
    // profiling (sgm_set_profiling)
    int profiling;
    std::vector<hipEvent_t> ev_pool;
    struct Pending { int cls; double elems; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<sgm_kernel_stat> stats;
    std::vector<double> stat_elems;  // elements of the class's launches since the last readout
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Every entry point's work shares the handle's scratch (cost volumes,
// checkpoints, post-filter and LKRefine buffers), whichever stream the caller
// passes.
// Orders calls on different streams (they share the handle's scratch).  A
// call on a CALLER's stream records ev_last on that stream as it returns,
// while the stream certainly exists (a rocprof trace shows the record as a
// ~5 us gap before the next kernel; frame loops can run on the handle's own
// stream, sgm_get_stream, instead); a call on the handle's own stream
// records nothing (the same-stream path stays free of event records) and a later
// call on another stream records ev_last on the handle's stream, which the
// handle owns.  So no stream handle of the caller is kept past the call that
// used it.  Entry points construct the scope after their argument checks, so
// a call rejected before enqueueing anything leaves the state untouched.
struct StreamScope {
    sgm_handle *h;
    hipStream_t st;
    StreamScope(sgm_handle *handle, void *stream)
        : h(handle), st(stream ? (hipStream_t)stream : handle->st) {
        if (h->last_st && h->last_st != st) {
            if (h->last_recorded)
                (void)hipStreamWaitEvent(st, h->ev_last, 0);
            else if (hipEventRecord(h->ev_last, h->last_st) == hipSuccess)
                (void)hipStreamWaitEvent(st, h->ev_last, 0);
        }
    }
    ~StreamScope() {
        h->last_st = st;
        h->last_recorded = st != h->st && hipEventRecord(h->ev_last, st) == hipSuccess;
    }
};

int set_err(sgm_handle *h, int code, const char *fmt, ...) {
    if (h) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(h->err, sizeof(h->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(h, expr)                                                                      \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err((h), e_ == hipErrorOutOfMemory ? SGM_ERR_OUT_OF_MEMORY : SGM_ERR_HIP, \
                           "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,   \
                           __LINE__);                                                        \
    } while (0)

bool valid_params(const sgm_params *p, char *why, size_t n) {
    if (!p) { snprintf(why, n, "params is NULL"); return false; }
    // Solver.cpp:6-10 (d widened to 256), plus the filter windows' minimum size.
    if (p->height <= 0 || p->width <= 0 || p->scale <= 0 || p->max_disp <= 0) {
        snprintf(why, n, "h, w, s, d must be > 0 (Solver.cpp:6)");
        return false;
    }
    if (p->scale != 1 && p->scale != 2) { snprintf(why, n, "scale must be 1 or 2 (Solver.cpp:8)"); return false; }
    if (p->max_disp != 32 && p->max_disp != 64 && p->max_disp != 128 && p->max_disp != 256) {
        snprintf(why, n, "max_disp must be 32, 64, 128 or 256 (Solver.cpp:10, widened)");
        return false;
    }
    const int H = p->height / p->scale, W = p->width / p->scale;
    if (W < 5 || H < 3) { snprintf(why, n, "working size %dx%d below the 5x3 cost window", H, W); return false; }
    if (p->views != 1 && p->views != 2) { snprintf(why, n, "views must be 1 or 2"); return false; }
    // SGM.cpp:374-408 keeps the previous pixel's sec_min_d when a pixel has no
    // second distinct cost; that stale index decides a pixel when
    // min/FLT_MAX > UNIQUE_RATIO.  A path cost is at most C + P2 (SGM.cpp:
    // 93-117: L = min(...) + C - minLp <= P2 + C), C at most 999999 (the sky
    // override, Solver.cpp:167-176), so min <= 8 (P2 + 999999); a ratio above
    // that / FLT_MAX can never see the stale index, which this build's WTA
    // does not keep.  Ratios at or below it (0 and negatives included) are
    // rejected.
    if (!(p->uniqueness > 0.0f) ||
        (double)p->uniqueness * FLT_MAX <= 8.0 * ((double)p->p2 + 999999.0)) {
        snprintf(why, n, "uniqueness must be > 8*(p2 + 999999)/FLT_MAX (SGM.cpp:392-408 would read "
                         "the previous pixel's sec_min_d)");
        return false;
    }
    if (p->view != SGM_VIEW_LEFT && p->view != SGM_VIEW_RIGHT) {
        snprintf(why, n, "view must be SGM_VIEW_LEFT or SGM_VIEW_RIGHT");
        return false;
    }
    if (p->view == SGM_VIEW_RIGHT &&
        (p->views != 1 || p->solver != SGM_SOLVER_SGM || p->post_filter || p->lk_refine)) {
        snprintf(why, n, "SGM_VIEW_RIGHT needs views == 1, the SGM solver and no post_filter/lk_refine");
        return false;
    }
    // the sky detector keeps a row of borders (W <= 8192) and the top half of a
    // 64-column strip (H/2 + 2 rows of 68 B <= ~159 KiB) in LDS (sgm_sky.hip)
    if (p->sky_detect && (W > 8192 || (size_t)(H / 2 + 2) * 68 > 160 * 1024 - 1024)) {
        snprintf(why, n, "sky_detect supports working grids up to 8192 x %d", 2 * ((160 * 1024 - 1024) / 68 - 2));
        return false;
    }
    if (p->solver != SGM_SOLVER_SGM && p->solver != SGM_SOLVER_BM) {
        snprintf(why, n, "solver must be SGM_SOLVER_SGM or SGM_SOLVER_BM");
        return false;
    }
    // the path DP's start handling relies on non-negative penalties (SGM.cpp:27-28 uses 10, 100)
    if (p->p1 < 0 || p->p2 < 0) { snprintf(why, n, "p1 and p2 must be >= 0"); return false; }
    if ((size_t)H * W > (size_t)0x7fffffff) { snprintf(why, n, "image too large"); return false; }
    return true;
}

template <typename T>
int dalloc(sgm_handle *h, T **p, size_t count) {
    *p = nullptr;
    if (count == 0) return SGM_OK;
    HIPCHK(h, hipMalloc((void **)p, count * sizeof(T)));
    h->bytes += count * sizeof(T);
    return SGM_OK;
}

void free_all(sgm_handle *h) {
    for (int v = 0; v < 2; ++v) {
        (void)hipFree(h->d_in[v]); (void)hipFree(h->d_sky[v]); (void)hipFree(h->d_ct[v]);
        (void)hipFree(h->d_ch_base[v]); (void)hipFree(h->d_c[v]); (void)hipFree(h->d_s[v]);
        for (auto &c : h->d_carry[v]) (void)hipFree(c);
        (void)hipFree(h->d_l3[v]);
        (void)hipFree(h->d_disp[v]); (void)hipFree(h->d_sub[v]);
    }
    (void)hipFree(h->d_out);
    (void)hipFree(h->d_gran);
    (void)hipFree(h->d_slant_ctl);
    (void)hipFree(h->d_slant_dummy);
    (void)hipFree(h->d_pf_orig); (void)hipFree(h->d_pf_work); (void)hipFree(h->d_pf_label);
    (void)hipFree(h->d_pf_count); (void)hipFree(h->d_pf_area); (void)hipFree(h->d_pf_snap);
    (void)hipFree(h->d_pf_changes);
    (void)hipFree(h->d_lk_in);
    (void)hipFree(h->d_sky_scratch);
    (void)hipFree(h->d_cloud_counts);
    if (h->h_pf_changes) (void)hipHostFree(h->h_pf_changes);
    h->h_pf_changes = nullptr;
    if (h->h_slant_err) (void)hipHostFree(h->h_slant_err);
    h->h_slant_err = nullptr;
    (void)hipFree(h->d_min);
    (void)hipFree(h->d_zero);
    if (h->h_pin) (void)hipHostFree(h->h_pin);
    h->h_pin = nullptr;
    for (auto &v : h->d_ck)
        for (auto p : v) (void)hipFree(p);
    if (h->st) (void)hipStreamDestroy(h->st);
    if (h->st_h) (void)hipStreamDestroy(h->st_h);
    hipEvent_t evs[] = {h->ev_pf, h->ev_last, h->ev_fork, h->ev_join};
    for (auto e : evs) if (e) (void)hipEventDestroy(e);
    for (auto &p : h->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : h->ev_pool) (void)hipEventDestroy(e);
    h->pending.clear();
    h->ev_pool.clear();
}

hipEvent_t pool_event(sgm_handle *h) {
    if (!h->ev_pool.empty()) {
        hipEvent_t e = h->ev_pool.back();
        h->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

int stat_class(sgm_handle *h, const char *name, double elems) {
    for (size_t k = 0; k < h->stats.size(); ++k)
        if (!strncmp(h->stats[k].name, name, sizeof(h->stats[k].name))) return (int)k;
    sgm_kernel_stat st{};
    snprintf(st.name, sizeof(st.name), "%s", name);
    st.elems = elems;
    h->stats.push_back(st);
    h->stat_elems.push_back(0.0);
    return (int)h->stats.size() - 1;
}

// Launch `fn` on `st`; with profiling on, bracket it with pooled events.
template <typename F>
hipError_t timed(sgm_handle *h, const char *name, double elems, hipStream_t st, F &&fn) {
    if (!h->profiling) return fn();
    hipEvent_t a = pool_event(h), b = pool_event(h);
    if (!a || !b) return hipErrorOutOfMemory;
    hipError_t e = hipEventRecord(a, st);
    if (e == hipSuccess) e = fn();
    if (e == hipSuccess) e = hipEventRecord(b, st);
    h->pending.push_back({stat_class(h, name, elems), elems, a, b});
    return e;
}

// Upper bound on median-fill launches of one post filter: the fill reaches its
// fixed point in 2-3 launches on stereo output; the bound only stops a runaway.
constexpr int kMedianMaxLaunches = 4096;

const char *kDirName[8] = {"L1", "L2", "L3", "L4", "L5", "L6", "L7", "L8"};
const char *kModeName[4] = {"store", "init", "acc", "final"};

hipError_t sweep(sgm_handle *h, int dir, int mode, const SweepArgs &a, hipStream_t st) {
    char name[32];
    snprintf(name, sizeof(name), "sweep_%s_%s", kDirName[dir], kModeName[mode]);
    const double elems = (double)h->g.H * h->g.W * h->g.D;
    return timed(h, name, elems, st, [&] { return sgm::launch_sweep(dir, mode, a, h->g, st); });
}

SweepArgs sweep_args(const sgm_handle *h) {
    SweepArgs a{};
    a.p1 = (float)h->p.p1;
    a.p2 = (float)h->p.p2;
    a.uniq = h->p.uniqueness;
    return a;
}

sgm::PairArgs pair_args(const sgm_handle *h) {
    sgm::PairArgs a{};
    a.zero = h->d_zero;
    a.p1 = (float)h->p.p1;
    a.p2 = (float)h->p.p2;
    a.uniq = h->p.uniqueness;
    return a;
}

hipError_t pair_fwd(sgm_handle *h, int fam, const sgm::PairArgs &a, hipStream_t st) {
    static const char *names[3] = {"pair_fwd_L1", "pair_fwd_L3", "pair_fwd_L6"};
    const double elems = (double)h->g.H * h->g.W * h->g.D;
    return timed(h, names[fam], elems, st, [&] { return sgm::launch_pair_fwd(fam, a, h->g, st); });
}

hipError_t pair_bwd(sgm_handle *h, int fam, int mode, const sgm::PairArgs &a, hipStream_t st) {
    static const char *names[3] = {"pair_bwd_L2_init2", "pair_bwd_L4_final", "pair_bwd_L7_acc"};
    const double elems = (double)h->g.H * h->g.W * h->g.D;
    return timed(h, names[fam], elems, st,
                 [&] { return sgm::launch_pair_bwd(fam, mode, a, h->g, st); });
}

// The slanted-tile schedule replaces the bands (above the Infinity Cache)
// where it was measured faster (tools/slant_sizes.py,
// profiles/r04_experiments/slant.txt, with the H pair beside the top-down
// pass): at D = 256 once views * W >= 0.5 * NW * CUs, i.e. half a full-height
// tile of work per workgroup (round 6; 0.7 before), at D = 128 from 0.9
// (round 4 at 0.7: HD256 two views -18.6%, 4K256 one view -20%,
// two views -24%, 720p D = 256 two views -9.4%, HD128 two views -9.6%,
// 4K128 two views -18.8%; HD256 one view +2.0%, HD128 one view +24.9%,
// 1056x512 D = 128 two views +10.3%); never at D = 64 (HD64 two views
// +16.8%, 4K64 +4.2%; round 5: +11.4%, +2.2%).  Below that the tile-to-tile
// hand-off chain, not the bytes, sets the passes' time.  At D = 128 the
// threshold is 0.9 tiles per workgroup (below).
bool slant_default(Geom g, int nviews) {
    const double vol = (double)g.W * g.H * g.D * sizeof(float);
    if (vol <= 256.0 * 1024 * 1024 || g.D < 128) return false;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    // round 5 re-sweep with the prioritised receiver (profiles/r05_experiments/
    // r05m_slant_sizes.txt): 720p D = 256 two views (0.71 tiles per
    // workgroup) -6.2%, but 720p D = 128 two views (0.71) +7.7%: at D = 128
    // the crossover lies between 0.71 and HD128's 1.07 (-9.6%).  Round 6's
    // dataflow passes (profiles/r06_experiments/r06c_sizes_sweep.txt,
    // r06f_share_order_sweep.txt) moved D = 256 down: HD256 one view (0.54)
    // -5.0..-9.7%; at D = 128, 720p two views (0.71) stays +5.3%, HD128 one
    // view (0.54) +24%
    return 10LL * nviews * g.W >= (g.D >= 256 ? 5LL : 9LL) * sgm::kSlantNW * cus;
}

// Rows per band of the backward phase (stage B's diagonal pair, the L8
// sweep, the final pass) for cost volumes above the 256 MB Infinity Cache:
// about 192 MB of cost volume per band, so that a band's C and T stay in the
// cache from one pass to the next (tools/band_probe.hip: 1.27-1.35x for the
// three passes' streams alone; in the frame HD256 -3.5%, 4K256 -5%; 94-126 MB
// bands gain less).  A volume the cache already holds (K128) loses by it.
// Band edges sit on multiples of 16 rows from the bottom: whole segments of
// every pair family.
// SGM_BAND_ROWS overrides (0: whole-volume passes).
int band_rows_for(Geom g) {
    const char *e = getenv("SGM_BAND_ROWS");
    const double row_bytes = (double)g.W * g.D * sizeof(float);
    int rows;
    if (e && *e) {
        rows = atoi(e);
    } else {
#ifdef SGM_NO_BANDS
        return 0;
#endif
        if (row_bytes * g.H <= 256.0 * 1024 * 1024) return 0;
        rows = (int)(192.0 * 1024 * 1024 / row_bytes);
    }
    rows -= rows % 16;
    return rows <= 0 || rows >= g.H ? 0 : rows;
}

// The 8-path aggregation of one view, given the final cost volume and the L3
// checkpoints (written by vfwd, or by the PAIR_V forward pass here when
// `need_v_ckpt`), as three launches on one stream:
//   stage A: L1 fwd (ckpt) | L5 -> T5 | L6 fwd (ckpt)
//   stage B: L2 bwd: S12 = L1 + L2 | L7 bwd: T = (T5 + L6) + L7
//   L8:      T += L8
//   final:   L4 bwd recomputing L3: total = ((S12 + L3) + L4) + T -> WTA
// (the reference's order, SGM.cpp:386-390).  T may alias the dead
// horizontally filtered volume.
// Banded frames (cost volumes above the Infinity Cache): the view's vertical
// filter + L3 forward pass (vfwd, from the horizontally filtered volume T)
// and stage A's diagonal roles run in forward bands first, top band first, so
// that each band's final cost stays in the Infinity Cache from vfwd to L5 and
// L6; the whole H pair follows as its own launch; then the backward bands
// (DESIGN.md "Bands").  need_v_ckpt (the parity stage, from a final cost
// volume) runs whole-volume passes.
// part AGG_FWD stops after the forward bands and leaves the H pair's
// arguments in hp[0..1] (the caller launches both views' H pairs at once);
// AGG_BWD then runs the rest.
enum AggPart { AGG_ALL = 0, AGG_FWD = 1, AGG_BWD = 2 };
// the view's final cost volume C and its T chain (T reuses the horizontally
// filtered volume, dead once vfwd has read it; an in-place vfwd with T in the
// second volume measured no faster, profiles/r03_experiments/inplace_c.txt)
inline float *cost_buf(sgm_handle *h, int v) { return h->d_c[v]; }
inline float *t_buf(sgm_handle *h, int v) { return h->d_ch[v]; }
int aggregate_view(sgm_handle *h, int view, const float *cost, float *S, float *T, uint16_t *disp,
                   float *sub, hipStream_t st, bool need_v_ckpt, sgm::PairArgs *defer_final = nullptr,
                   int part = AGG_ALL, sgm::PairArgs *hp = nullptr, int sub_cm = 0) {
    float **ck = h->d_ck[view];
    const double elems = (double)h->g.H * h->g.W * h->g.D;
    sgm::PairArgs pa = pair_args(h);
    pa.cost = cost;
    if (need_v_ckpt) {
        pa.ckpt = ck[sgm::PAIR_V];
        HIPCHK(h, pair_fwd(h, sgm::PAIR_V, pa, st));
    }
    sgm::PairArgs h1 = pa, d6 = pa;
    h1.ckpt = ck[sgm::PAIR_H];
    d6.ckpt = ck[sgm::PAIR_D2];
    SweepArgs l5 = sweep_args(h);
    l5.cost = cost;
    l5.acc_out = T;
    sgm::PairArgs h2 = h1, d7 = d6;
    h2.out = S;
    d7.acc_in = T;
    d7.out = T;
    const int H = h->g.H;
    const bool banded = h->band_rows > 0 && !defer_final && !need_v_ckpt;
    const int BR = banded ? h->band_rows : 0;
    if (part == AGG_BWD) {
        // stage A ran (AGG_FWD + the caller's H pair launch)
    } else if (banded) {
        sgm::PairArgs va = pair_args(h);
        va.ckpt = ck[sgm::PAIR_V];
        // band edges at H - m*BR (multiples of 16 rows from the bottom, as
        // the backward bands): whole segments of every family
        const int FR = BR;
        const int nb = (H + FR - 1) / FR;
        for (int m = nb - 1; m >= 0; --m) {
            const int rb = H - (m + 1) * FR > 0 ? H - (m + 1) * FR : 0, re = H - m * FR;
            const double be = (double)(re - rb) / H * elems;
            va.band = {rb, re, h->d_carry[view][2]};
            HIPCHK(h, timed(h, "vfwd", be, st, [&] {
                       return sgm::launch_vfwd(h->d_ch[view], cost_buf(h, view), va, h->g, st);
                   }));
            l5.band = {rb, re, h->d_carry[view][0]};
            d6.band = {rb, re, h->d_carry[view][1]};
            HIPCHK(h, timed(h, "stage_a_d", be, st,
                            [&] { return sgm::launch_stage_a_band(l5, d6, h->g, st); }));
        }
        if (part == AGG_FWD) {
            hp[0] = h1;
            hp[1] = h2;
            return SGM_OK;
        }
        HIPCHK(h, timed(h, "stage_a_h", elems, st,
                        [&] { return sgm::launch_stage_a_hpair(&h1, &h2, 1, h->g, st); }));
    } else {
        HIPCHK(h, timed(h, "stage_a", elems, st,
                        [&] { return sgm::launch_stage_a(h1, l5, d6, h->g, st); }));
    }
    if (!banded)
        HIPCHK(h, timed(h, "stage_b", elems, st,
                        [&] { return sgm::launch_stage_b(h2, d7, h->g, st); }));
    SweepArgs l8 = sweep_args(h);
    l8.cost = cost;
    l8.acc_in = T;
    l8.acc_out = T;
    pa.ckpt = ck[sgm::PAIR_V];
    pa.s_in = S;
    pa.acc_in = T;
    pa.disp = disp;
    pa.sub = sub;
    pa.sub_cm = sub_cm;
    if (banded) {
        // bottom band first: the backward passes walk up
        for (int kb = 0; kb < H; kb += BR) {
            const int ke = kb + BR < H ? kb + BR : H;
            const double be = (double)(ke - kb) / H * elems;
            d7.band = {kb, ke, h->d_carry[view][0]};
            HIPCHK(h, timed(h, "stage_b_d2", be, st,
                            [&] { return sgm::launch_stage_b(h2, d7, h->g, st); }));
            l8.band = {kb, ke, h->d_carry[view][1]};
            pa.band = {kb, ke, h->d_carry[view][2]};
            HIPCHK(h, timed(h, "sweep_L8_acc", be, st,
                            [&] { return sgm::launch_sweep(SGM_DIR_L8, sgm::SWEEP_ACC, l8, h->g, st); }));
            HIPCHK(h, timed(h, "pair_bwd_L4_final", be, st, [&] {
                       return sgm::launch_pair_bwd(sgm::PAIR_V, sgm::PAIR_FINAL, pa, h->g, st);
                   }));
        }
        return SGM_OK;
    }
    HIPCHK(h, sweep(h, SGM_DIR_L8, sgm::SWEEP_ACC, l8, st));
    if (defer_final) {  // the caller launches this view's final pass with the other view's
        *defer_final = pa;
        return SGM_OK;
    }
    // two views: each final pass is the last read of its view's C, and the
    // other view's volume follows it into the Infinity Cache, so C goes by
    // non-temporal loads (K128 two views -1.0% paired).  With one view the
    // next frame's stage A loses what the final pass gains, with one C buffer
    // or two used alternately (profiles/r06_experiments/r06aa_final_nt.txt,
    // r06bb_c_alternate.txt), so one-view frames keep default loads
    pa.nt_cost = h->nviews == 2;
    HIPCHK(h, pair_bwd(h, sgm::PAIR_V, sgm::PAIR_FINAL, pa, st));
    return SGM_OK;
}

// Both views' aggregation as joint launches (grid.y = view): stage A, stage
// B, the L8 sweep and the final pass each take both views at once.  For frames
// whose two cost volumes fit the 256 MB Infinity Cache together (K64: 2 x 119
// MB), where one view's launches hold too few chains to fill the chip (the
// reference runs the views back to back, SGM.cpp:32-801; the results are the
// same per view).
int aggregate_joint(sgm_handle *h, float *sub0, uint16_t *raw, int cm, hipStream_t st) {
    const double elems2 = 2.0 * h->g.H * h->g.W * h->g.D;
    sgm::PairArgs h1[2], d6[2], h2[2], d7[2], fin[2];
    SweepArgs l5[2], l8[2];
    for (int v = 0; v < 2; ++v) {
        float **ck = h->d_ck[v];
        sgm::PairArgs pa = pair_args(h);
        pa.cost = cost_buf(h, v);
        h1[v] = pa;
        h1[v].ckpt = ck[sgm::PAIR_H];
        d6[v] = pa;
        d6[v].ckpt = ck[sgm::PAIR_D2];
        h2[v] = h1[v];
        h2[v].out = h->d_s[v];
        d7[v] = d6[v];
        d7[v].acc_in = t_buf(h, v);
        d7[v].out = t_buf(h, v);
        l5[v] = sweep_args(h);
        l5[v].cost = cost_buf(h, v);
        l5[v].acc_out = t_buf(h, v);
        l8[v] = l5[v];
        l8[v].acc_in = t_buf(h, v);
        fin[v] = pa;
        fin[v].ckpt = ck[sgm::PAIR_V];
        fin[v].s_in = h->d_s[v];
        fin[v].acc_in = t_buf(h, v);
        fin[v].disp = v ? nullptr : raw;
        fin[v].sub = v ? h->d_sub[1] : sub0;
        fin[v].sub_cm = cm;
    }
    const Geom g = h->g;
    HIPCHK(h, timed(h, "stage_a", elems2, st, [&] { return sgm::launch_stage_a2(h1, l5, d6, g, st); }));
    HIPCHK(h, timed(h, "stage_b", elems2, st, [&] { return sgm::launch_stage_b2(h2, d7, g, st); }));
    HIPCHK(h, timed(h, "sweep_L8_acc", elems2, st,
                    [&] { return sgm::launch_sweep2_l8(l8[0], l8[1], g, st); }));
    HIPCHK(h, timed(h, "pair_bwd_L4_final", elems2, st,
                    [&] { return sgm::launch_final2(fin[0], fin[1], g, st); }));
    return SGM_OK;
}

// build_dsi_from_table[_beta] (dsi 0 / 1) + horizontal IIR (cost_h), then
// the vertical IIR fused with the L3 forward pass (vfwd), into view slot
// `view`'s buffers.
int vfwd_view(sgm_handle *h, int view, hipStream_t st);
int cost_view(sgm_handle *h, int view, int dsi, const uint8_t *sky, int sky_pitch, hipStream_t st,
              bool vfwd = true) {
    const double elems = (double)h->g.H * h->g.W * h->g.D;
    HIPCHK(h, timed(h, "cost_h", elems, st, [&] {
               return sgm::launch_cost_h(h->d_ct[0], h->d_ct[1], sky, sky_pitch, dsi, 1, h->g,
                                         h->d_ch[view], st);
           }));
    return vfwd ? vfwd_view(h, view, st) : SGM_OK;
}

int vfwd_view(sgm_handle *h, int view, hipStream_t st) {
    const double elems = (double)h->g.H * h->g.W * h->g.D;
    sgm::PairArgs pa = pair_args(h);
    pa.ckpt = h->d_ck[view][sgm::PAIR_V];
    HIPCHK(h, timed(h, "vfwd", elems, st, [&] {
               return sgm::launch_vfwd(h->d_ch[view], cost_buf(h, view), pa, h->g, st);
           }));
    return SGM_OK;
}

int post_filter(sgm_handle *h, float *d_map, int pitch, hipStream_t st, bool to_lk = false);
int lk_refine(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
              float *d_map, int map_pitch, hipStream_t st, bool staged = false);

// BM::process (src/BM.cpp:9-97): census with BM's row decimation, the left
// DSI + both cost filters (the vertical filter's fused L3 checkpoints are
// simply not used), the filtered-cost WTA, then post_filter (:88).
int bm_frame(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
             const uint8_t *d_sky_l, int sky_pitch, float *d_out, int out_pitch, uint16_t *d_raw,
             hipStream_t st) {
    const Geom g = h->g;
    const double npx = (double)g.H * g.W, elems = npx * g.D;
    if (h->p.sky_detect) {
        HIPCHK(h, timed(h, "sky_detect", npx, st, [&] {
                   return sgm::launch_sky_detect(&d_left, pitch, h->d_sky, g.W, h->d_sky_scratch, 1,
                                                 g, st);
               }));
        d_sky_l = h->d_sky[0];
        sky_pitch = g.W;
    }
    HIPCHK(h, timed(h, "census", 2 * npx, st, [&] {
               return sgm::launch_census(d_left, pitch, g, h->p.blur, h->d_ct[0], st, true, d_right,
                                         h->d_ct[1]);
           }));
    int rc;
    if ((rc = cost_view(h, 0, 0, d_sky_l, sky_pitch, st)) != SGM_OK) return rc;
    HIPCHK(h, timed(h, "bm_wta", elems, st, [&] {
               return sgm::launch_bm_wta(cost_buf(h, 0), h->p.uniqueness, h->d_disp[0], d_out, out_pitch,
                                         g, st);
           }));
    if (d_raw && d_raw != h->d_disp[0])  // (the host API passes d_disp[0] itself)
        HIPCHK(h, hipMemcpyAsync(d_raw, h->d_disp[0], (size_t)g.H * g.W * sizeof(uint16_t),
                                 hipMemcpyDeviceToDevice, st));
    if (h->p.post_filter) return post_filter(h, d_out, out_pitch, st);
    return SGM_OK;
}

int finish_frame(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
                 float *d_out, int out_pitch, hipStream_t st);

// The slanted-tile schedule of the aggregation (DESIGN.md "Slanted tiles"),
// after the cost stage left each view's horizontally filtered volume in d_ch:
//   vfwd_l3 (per view): vertical IIR -> C, and the full L3 volume
//   slant_down (both views): T56 = L5 + L6 (SGM.cpp:389's first association)
//     into the dead horizontally filtered volume
//   H pair (both views): S12 = L1 + L2
//   slant_up (both views): L4, L7, L8 walking up, total
//     ((S12 + L3) + L4) + ((T56 + L7) + L8), WTA, sub-pixel (row-major maps)
// the top-down pass's share of the CUs (eighths) while the H pair runs
// beside it.  Round 6 (dataflow passes, profiles/r06_experiments/
// r06f_share_order_sweep.txt, best of 3): the top-down pass alone now takes
// 1.9 ms at HD256 (it took the whole 4.7 ms region before), so the share
// that balances the two moved: 4/8 for D = 256 frames below 2e9 elements
// (HD256 V=2 10.83 ms vs 11.12 at 8/8, HD256 V=1, 720p256 V=2), the whole
// chip otherwise (4K256 V=1/V=2, HD128 and 4K128 V=2 within 0.5% of their
// best at 8/8).  Launching the H pair first was no better at any share.
int slant_down_grid_eighths(Geom g, int nviews) {
#ifdef SGM_SLANT_DEBUG
    if (const char *e = getenv("SGM_SLANT_DOWN_EIGHTHS"))  // share sweeps (tools/slant_share.sh)
        if (atoi(e) >= 1 && atoi(e) <= 8) return atoi(e);
#endif
    const double elems = (double)nviews * g.H * g.W * g.D;
    return g.D >= 256 && elems < 2e9 ? 4 : 8;
}
int slant_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    return cus;
}

// have_c: the strip pass already wrote C and the L3 volumes (run_frame)
int slant_views(sgm_handle *h, float *sub0, uint16_t *raw, hipStream_t st, bool have_c) {
    const Geom g = h->g;
    const int nv = h->nviews;
    const double elems = (double)g.H * g.W * g.D;
    sgm::PairArgs hp1[2], hp2[2];
    sgm::SlantArgs sa{};
    if (have_c) {
    } else if (nv == 2) {  // both views in one launch
        const sgm::PairArgs pa[2] = {pair_args(h), pair_args(h)};
        const float *in[2] = {h->d_ch[0], h->d_ch[1]};
        float *out[2] = {h->d_c[0], h->d_c[1]}, *l3[2] = {h->d_l3[0], h->d_l3[1]};
        HIPCHK(h, timed(h, "vfwd_l3", 2 * elems, st, [&] { return sgm::launch_vfwd2_l3(in, out, l3, pa, g, st); }));
    } else {
        const sgm::PairArgs pa = pair_args(h);
        HIPCHK(h, timed(h, "vfwd_l3", elems, st, [&] {
                   return sgm::launch_vfwd_l3(h->d_ch[0], h->d_c[0], h->d_l3[0], pa, g, st);
               }));
    }
    for (int v = 0; v < nv; ++v) {
        hp1[v] = pair_args(h);
        hp1[v].cost = h->d_c[v];
        hp1[v].ckpt = h->d_ck[v][sgm::PAIR_H];
        hp2[v] = hp1[v];
        hp2[v].out = h->d_s[v];
        sa.v[v] = {h->d_c[v], h->d_s[v], h->d_l3[v], t_buf(h, v), t_buf(h, v),
                   v ? h->d_sub[1] : sub0, v ? nullptr : raw, h->d_gran};
    }
    sa.ctl = h->d_slant_ctl;
    sa.zero = h->d_zero;
    sa.dummy = h->d_slant_dummy;
    sa.p1 = (float)h->p.p1;
    sa.p2 = (float)h->p.p2;
    sa.uniq = h->p.uniqueness;
    sa.nviews = nv;
    sa.err_host = h->d_slant_err;
#ifdef SGM_SLANT_DEBUG
    if (getenv("SGM_SLANT_T56SWEEP")) {  // T56 by the two diagonal sweeps instead
        for (int v = 0; v < nv; ++v) {
            SweepArgs l5 = sweep_args(h);
            l5.cost = h->d_c[v];
            l5.acc_out = t_buf(h, v);
            HIPCHK(h, sgm::launch_sweep(SGM_DIR_L5, sgm::SWEEP_INIT, l5, g, st));
            SweepArgs l6 = l5;
            l6.acc_in = t_buf(h, v);
            HIPCHK(h, sgm::launch_sweep(SGM_DIR_L6, sgm::SWEEP_ACC, l6, g, st));
        }
    } else
#endif
    // The H pair and the top-down pass both only read C: the H pair runs on
    // its own stream beside the top-down pass, which keeps half of the CUs
    // (its workgroups are persistent and claim tiles in order, so any grid
    // is correct).  Each is bound by latency as much as by bytes (long H
    // chains; the tile-to-tile hand-off chain), so together they fill the
    // memory system better than one after the other: HD256 13.44 -> 12.72,
    // 4K256 48.03 -> 46.31 ms per frame (profiles/r04_experiments/slant.txt).
    // (profiled as one more entry, "slant_down_hpair": fork to join on the
    // frame's stream, the pair's wall time; the two launches' own entries
    // overlap in time)
    sa.max_grid = slant_down_grid_eighths(g, nv) * slant_cus() / 8;
#ifdef SGM_SLANT_DEBUG
    // timing probes (wrong maps): SGM_SLANT_SOLO=down|hpair runs that launch
    // alone on all CUs; =seq runs both, one after the other
    if (const char *solo = getenv("SGM_SLANT_SOLO")) {
        sa.max_grid = 0;
        if (strcmp(solo, "hpair") != 0)
            HIPCHK(h, timed(h, "slant_down", nv * elems, st, [&] { return sgm::launch_slant_down(sa, g, st); }));
        if (strcmp(solo, "down") != 0)
            HIPCHK(h, timed(h, "stage_a_h", nv * elems, st,
                            [&] { return sgm::launch_stage_a_hpair(hp1, hp2, nv, g, st); }));
        HIPCHK(h, timed(h, "slant_up", nv * elems, st, [&] { return sgm::launch_slant_up(sa, g, st); }));
        return SGM_OK;
    }
#endif
    HIPCHK(h, timed(h, "slant_down_hpair", nv * elems, st, [&] {
        hipError_t e = hipEventRecord(h->ev_fork, st);
        if (e == hipSuccess) e = hipStreamWaitEvent(h->st_h, h->ev_fork, 0);
        if (e == hipSuccess)
            e = timed(h, "slant_down", nv * elems, st, [&] { return sgm::launch_slant_down(sa, g, st); });
        if (e == hipSuccess)
            e = timed(h, "stage_a_h", nv * elems, h->st_h,
                      [&] { return sgm::launch_stage_a_hpair(hp1, hp2, nv, g, h->st_h); });
        if (e == hipSuccess) e = hipEventRecord(h->ev_join, h->st_h);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, h->ev_join, 0);
        return e;
    }));
    sa.max_grid = 0;
    HIPCHK(h, timed(h, "slant_up", nv * elems, st, [&] { return sgm::launch_slant_up(sa, g, st); }));
    return SGM_OK;
}

int run_frame(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
              const uint8_t *d_sky_l, const uint8_t *d_sky_r, int sky_pitch, float *d_out,
              int out_pitch, uint16_t *d_raw, hipStream_t st) {
    const Geom g = h->g;
    int rc;
    // Everything runs on one stream.  Two-view frames keep each view's cost
    // volume resident in the 256 MB Infinity Cache through its readers by
    // running the views' aggregation back to back (K128: 238.5 MB per view;
    // concurrent views measured 1.627 vs 1.589 ms per pair), unless both
    // volumes fit together (K64: joint launches) or neither fits (HD/4K:
    // bands, or the slanted schedule).
    if (h->p.solver == SGM_SOLVER_BM)
        return bm_frame(h, d_left, d_right, pitch, d_sky_l, sky_pitch, d_out, out_pitch, d_raw, st);
    const double npx = (double)g.H * g.W;
    const double vol_bytes = npx * g.D * sizeof(float);
    // a right-view handle (SGM_VIEW_RIGHT) runs the right view in slot 0
    const bool right_only = h->p.view == SGM_VIEW_RIGHT;
    if (h->p.sky_detect) {  // node.cpp:80-93: detect on both inputs, then process with the masks
        const uint8_t *imgs[2] = {right_only ? d_right : d_left, d_right};
        HIPCHK(h, timed(h, "sky_detect", npx, st, [&] {
                   return sgm::launch_sky_detect(imgs, pitch, h->d_sky, g.W, h->d_sky_scratch,
                                                 h->nviews, g, st);
               }));
        d_sky_l = h->d_sky[0];
        d_sky_r = right_only ? h->d_sky[0] : h->nviews == 2 ? h->d_sky[1] : nullptr;
        sky_pitch = g.W;
    }
    HIPCHK(h, timed(h, "census", 2 * npx, st, [&] {  // both images, one launch
               return sgm::launch_census(d_left, pitch, g, h->p.blur, h->d_ct[0], st, false,
                                         d_right, h->d_ct[1]);
           }));
    // two views: both DSIs + horizontal IIRs in one launch (a view's H*D
    // serial chains alone leave most SIMDs idle at KITTI sizes)
    const bool both_h = h->nviews == 2 && (d_sky_l == nullptr) == (d_sky_r == nullptr) &&
                        sgm::cost_h2_supported(g, d_sky_l != nullptr);
    // banded frames run vfwd in forward bands inside aggregate_view; the
    // slanted schedule runs its own vertical pass
    const bool banded = h->band_rows > 0;
    const bool vfwd_here = !banded && !h->slant;
    // the slanted schedule's cost stage as checkpoints + strips (sgm_vstrip.hip):
    // C and the L3 volumes in one pass, 9 B per element instead of cost_h's
    // 4 and vfwd_l3's 12
    const uint8_t *sky0 = right_only ? d_sky_r : d_sky_l;
    const bool vstrip = h->slant && h->vstrip && sgm::vstrip_supported(g, sky0 != nullptr) &&
                        (h->nviews == 1 || (sky0 == nullptr) == (d_sky_r == nullptr));
    // (a masked frame's sky flags go to the strip pass as words, after the
    // checkpoints in the Ch buffer: 3/16 + 2/D of its floats at most)
    if (vstrip) {
        const int dsi0 = right_only ? 1 : 0;
        HIPCHK(h, timed(h, "cost_ck", h->nviews * npx * g.D, st, [&] {
                   return sgm::launch_cost_ck(h->d_ct[0], h->d_ct[1], sky0, d_sky_r, sky_pitch, dsi0, 1,
                                              h->nviews, g, h->d_ch[0], h->d_ch[1], st);
               }));
        sgm::VStripArgs va{};
        va.ctl = h->d_ct[0];
        va.ctr = h->d_ct[1];
        if (sky0) {
            const uint8_t *skm[2] = {sky0, d_sky_r};
            uint64_t *skw[2] = {nullptr, nullptr};
            for (int v = 0; v < h->nviews; ++v) {
                skw[v] = reinterpret_cast<uint64_t *>(h->d_ch[v] + sgm::vstrip_sky_words_offset(g));
                HIPCHK(h, timed(h, "sky_words", npx, st,
                                [&] { return sgm::launch_sky_words(skm[v], sky_pitch, g, skw[v], st); }));
            }
            va.skw0 = skw[0];
            va.skw1 = skw[1];
        }
        va.dsi0 = dsi0;
        va.dsi1 = 1;
        va.ck0 = h->d_ch[0];  // (the checkpoints sit in the dead Ch volumes)
        va.ck1 = h->d_ch[1];
        va.c0 = h->d_c[0];
        va.c1 = h->d_c[1];
        va.l30 = h->d_l3[0];
        va.l31 = h->d_l3[1];
        va.dummy = h->d_slant_dummy;
        va.p1 = (float)h->p.p1;
        va.p2 = (float)h->p.p2;
        HIPCHK(h, timed(h, "vstrip", h->nviews * npx * g.D, st,
                        [&] { return sgm::launch_vstrip(va, h->nviews, g, st); }));
    } else if (both_h) {
        HIPCHK(h, timed(h, "cost_h", 2.0 * npx * g.D, st, [&] {
                   return sgm::launch_cost_h2(h->d_ct[0], h->d_ct[1], d_sky_l, d_sky_r, sky_pitch, g,
                                              h->d_ch[0], h->d_ch[1], st);
               }));
        if (vfwd_here) {
            // both views' vertical passes in one launch: W chains per view
            // leave the CUs under-filled at KITTI (K64 2 x 69.7 -> 90.7 us,
            // frame -3.9%; K128 two views 177 -> 166 us)
            sgm::PairArgs pa[2] = {pair_args(h), pair_args(h)};
            // (view 1's columns first, view 0's last, as the per-view passes
            // ran: stage A then finds more of view 0 in the cache, K64 stage
            // A -3 us, profiles/r05_experiments/r05s_ab_vfwd2.txt)
            const int v0 = 1, v1 = 0;
            pa[0].ckpt = h->d_ck[v0][sgm::PAIR_V];
            pa[1].ckpt = h->d_ck[v1][sgm::PAIR_V];
            const float *in[2] = {h->d_ch[v0], h->d_ch[v1]};
            float *out[2] = {cost_buf(h, v0), cost_buf(h, v1)};
            HIPCHK(h, timed(h, "vfwd", 2.0 * npx * g.D, st, [&] { return sgm::launch_vfwd2(in, out, pa, g, st); }));
        }
    } else {
        if (h->nviews == 2 && (rc = cost_view(h, 1, 1, d_sky_r, sky_pitch, st, vfwd_here)) != SGM_OK)
            return rc;
        if ((rc = cost_view(h, 0, right_only ? 1 : 0, right_only ? d_sky_r : d_sky_l, sky_pitch,
                            st, vfwd_here)) != SGM_OK)
            return rc;
    }
    // one view with a dense output map: the final pass writes the sub-pixel
    // map straight into it (no device copy after the frame)
    const bool direct_out = h->nviews == 1 && out_pitch == g.W;
    float *sub0 = direct_out ? d_out : h->d_sub[0];
    // two views: the final passes write column-major sub-pixel maps (whole
    // cache lines; lr_cm_kernel reads them through LDS tiles); the slanted
    // pass writes row-major ones
    const bool cm = h->nviews == 2 && !h->slant;
    if (h->slant) {
        if ((rc = slant_views(h, sub0, d_raw, st, vstrip)) != SGM_OK) return rc;
    } else if (h->nviews == 2 && !banded && 2.0 * vol_bytes <= 256.0 * 1024 * 1024) {
        // both volumes fit the Infinity Cache together: joint launches
        if ((rc = aggregate_joint(h, sub0, d_raw, 1, st)) != SGM_OK) return rc;
    } else if (h->nviews == 2 && banded) {
        // both views' forward bands, then both H pairs in one launch, then
        // each view's backward bands
        sgm::PairArgs hp[2][2];
        for (int v = 0; v < 2; ++v)
            if ((rc = aggregate_view(h, v, cost_buf(h, v), h->d_s[v], t_buf(h, v), v ? nullptr : d_raw,
                                     v ? h->d_sub[1] : sub0, st, false, nullptr, AGG_FWD,
                                     hp[v])) != SGM_OK)
                return rc;
        const sgm::PairArgs h1[2] = {hp[0][0], hp[1][0]}, h2[2] = {hp[0][1], hp[1][1]};
        HIPCHK(h, timed(h, "stage_a_h", 2.0 * npx * g.D, st,
                        [&] { return sgm::launch_stage_a_hpair(h1, h2, 2, g, st); }));
        for (int v = 0; v < 2; ++v)
            if ((rc = aggregate_view(h, v, cost_buf(h, v), h->d_s[v], t_buf(h, v), v ? nullptr : d_raw,
                                     v ? h->d_sub[1] : sub0, st, false, nullptr, AGG_BWD, nullptr,
                                     1)) != SGM_OK)
                return rc;
    } else if (h->nviews == 2 && vol_bytes > 256.0 * 1024 * 1024) {
        // whole-volume passes above the Infinity Cache (SGM_BAND_ROWS=0):
        // nothing is gained by finishing the left view first, so both
        // views' final passes run as one launch (fewer workgroup rounds)
        sgm::PairArgs fin[2];
        for (int v = 0; v < 2; ++v)
            if ((rc = aggregate_view(h, v, cost_buf(h, v), h->d_s[v], t_buf(h, v), v ? nullptr : d_raw,
                                     v ? h->d_sub[1] : sub0, st, false, &fin[v], AGG_ALL, nullptr,
                                     1)) != SGM_OK)
                return rc;
        HIPCHK(h, timed(h, "pair_bwd_L4_final", 2.0 * npx * g.D, st,
                        [&] { return sgm::launch_final2(fin[0], fin[1], g, st); }));
    } else {
        for (int v = 0; v < h->nviews; ++v)
            if ((rc = aggregate_view(h, v, cost_buf(h, v), h->d_s[v], t_buf(h, v), v ? nullptr : d_raw,
                                     v ? h->d_sub[1] : sub0, st, false, nullptr, AGG_ALL, nullptr,
                                     cm ? 1 : 0)) != SGM_OK)
                return rc;
    }
    if (h->nviews == 2) {
        HIPCHK(h, timed(h, "lr", npx, st, [&] {
                   return cm ? sgm::launch_lr_cm(h->d_sub[0], h->d_sub[1], d_out, out_pitch,
                                                 h->p.lr_max_diff, g, st)
                             : sgm::launch_lr(h->d_sub[0], g.W, h->d_sub[1], g.W, d_out, out_pitch,
                                              h->p.lr_max_diff, g, st);
               }));
    } else if (!direct_out) {
        HIPCHK(h, hipMemcpy2DAsync(d_out, (size_t)out_pitch * sizeof(float), h->d_sub[0],
                                   (size_t)g.W * sizeof(float), (size_t)g.W * sizeof(float), g.H,
                                   hipMemcpyDeviceToDevice, st));
    }
    // (the raw WTA map, when asked for, was written straight into d_raw by the
    // left view's final pass; the right view's is never written)
    return finish_frame(h, d_left, d_right, pitch, d_out, out_pitch, st);
}

// post_filter and LKRefine at the end of a frame (SGM.cpp:821-824)
int finish_frame(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
                 float *d_out, int out_pitch, hipStream_t st) {
    int rc;
    // with LKRefine next, the post filter's last kernel writes LKRefine's
    // input copy instead of the map (no device copy in between)
    const bool pf_to_lk = h->p.post_filter && h->p.lk_refine;
    if (h->p.post_filter && (rc = post_filter(h, d_out, out_pitch, st, pf_to_lk)))  // SGM.cpp:821
        return rc;
    if (h->p.lk_refine)  // SGM.cpp:824
        return lk_refine(h, d_left, d_right, pitch, d_out, out_pitch, st, pf_to_lk);
    return SGM_OK;
}

// Pinned staging for the host-buffer API: user rows are packed into pinned
// memory on the CPU, so every host<->device transfer is one contiguous DMA
// (pageable 2-D copies went through the runtime's staging path at a fraction
// of PCIe bandwidth).  Layout: left | right | sky_l | sky_r | out f32 | raw u16.
int ensure_pinned(sgm_handle *h) {
    const size_t nin = (size_t)h->p.height * h->p.width, npx = (size_t)h->g.H * h->g.W;
    const size_t need = 2 * nin + 2 * npx + npx * sizeof(float) + npx * sizeof(uint16_t) + 64;
    if (h->h_pin && h->h_pin_bytes >= need) return SGM_OK;
    if (h->h_pin) (void)hipHostFree(h->h_pin);
    h->h_pin = nullptr;
    HIPCHK(h, hipHostMalloc((void **)&h->h_pin, need, hipHostMallocDefault));
    h->h_pin_bytes = need;
    return SGM_OK;
}

int copy_in_image(sgm_handle *h, uint8_t *dst, const uint8_t *src, int pitch) {
    HIPCHK(h, hipMemcpy2DAsync(dst, (size_t)h->p.width, src, (size_t)pitch, (size_t)h->p.width,
                               (size_t)h->p.height, hipMemcpyHostToDevice, h->st));
    return SGM_OK;
}

void pack_rows(uint8_t *dst, const uint8_t *src, size_t row_bytes, int rows, size_t pitch) {
    if (pitch == row_bytes) {
        memcpy(dst, src, row_bytes * rows);
        return;
    }
    for (int i = 0; i < rows; ++i) memcpy(dst + i * row_bytes, src + i * pitch, row_bytes);
}

// post_filter() (Solver.cpp:600-649) in place on a device map (sgm_post.hip):
// median-fill launches until one changes nothing, then the speckle removal.
// The fill works on a separate map and the component kernels write the
// caller's map from it, so they are enqueued before the host reads the fill's
// convergence counter (the GPU keeps working through that round trip); in the
// rare case the fill had not converged, more fill launches run and the
// component kernels are enqueued again.
// to_lk: write the filtered map to d_lk_in (contiguous) instead of d_map, for
// lk_refine(..., staged = true) to read.
int post_filter(sgm_handle *h, float *d_map, int pitch, hipStream_t st, bool to_lk) {
    const Geom g = h->g;
    // The number of median-fill launches depends on a counter read back to
    // the host each round; under stream capture that copy never runs, so a
    // captured graph would replay a fixed, possibly unconverged, fill.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPCHK(h, hipStreamIsCapturing(st, &cap));
    if (cap != hipStreamCaptureStatusNone)
        return set_err(h, SGM_ERR_INVALID_ARG,
                       "post_filter cannot be captured into a HIP graph (its median-fill launch "
                       "count is read back to the host); capture frames with post_filter = 0");
    const double dnpx = (double)g.H * g.W;
    float *F = h->d_pf_work;
    HIPCHK(h, timed(h, "post_prep", dnpx, st, [&] {
               return sgm::launch_pf_prep(d_map, pitch, h->d_pf_orig, F, h->d_pf_changes,
                                          kMedianMaxLaunches, g, st);
           }));
    auto components = [&]() -> int {
        HIPCHK(h, timed(h, "post_cc_local", dnpx, st, [&] {
                   return sgm::launch_cc_local(F, h->d_pf_label, h->d_pf_count, h->d_pf_area, g, st);
               }));
        HIPCHK(h, timed(h, "post_cc_merge", dnpx, st,
                        [&] { return sgm::launch_cc_merge(F, h->d_pf_label, g, st); }));
        HIPCHK(h, timed(h, "post_cc_count", dnpx, st, [&] {
                   return sgm::launch_cc_count(h->d_pf_label, h->d_pf_count, h->d_pf_area, 1000 / g.scale,
                                               g, st);
               }));
        // speckle_filter_new(filtered_disp, invalid_disp, SPECKLE_SIZE/scale, SPECKLE_DIS), :645
        HIPCHK(h, timed(h, "post_cc_apply", dnpx, st, [&] {
                   return sgm::launch_cc_apply(F, h->d_pf_label, h->d_pf_area, 1000 / g.scale,
                                               (float)(g.D + 1), to_lk ? h->d_lk_in : d_map,
                                               to_lk ? g.W : pitch, g, st);
               }));
        return SGM_OK;
    };
    int k = 0, rc;
    for (;;) {
        // a fill usually settles in 2 launches and the 3rd proves it
        const int batch = k == 0 ? 3 : 2;
        for (int b = 0; b < batch; ++b, ++k)
            HIPCHK(h, timed(h, "post_median", dnpx, st, [&] {
                       return sgm::launch_median_fill(h->d_pf_orig, F, k, h->d_pf_snap,
                                                      h->d_pf_changes, h->mf_rows, g, st);
                   }));
        HIPCHK(h, hipMemcpyAsync(h->h_pf_changes, h->d_pf_changes + k - 1, sizeof(int),
                                 hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipEventRecord(h->ev_pf, st));
        if ((rc = components())) return rc;
        HIPCHK(h, hipEventSynchronize(h->ev_pf));
        if (*h->h_pf_changes == 0) break;
        if (k + 2 > kMedianMaxLaunches)
            return set_err(h, SGM_ERR_HIP, "post_filter: median fill did not converge in %d launches",
                           k);
    }
    h->pf_iters = k;
    return SGM_OK;
}

// LKRefine (sgm_lk.hip) in place on a device map: the kernel reads a
// contiguous copy of the map and writes the refined values back.
// staged: d_lk_in already holds the map (post_filter(..., to_lk = true))
int lk_refine(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
              float *d_map, int map_pitch, hipStream_t st, bool staged) {
    const Geom g = h->g;
    const size_t row = (size_t)g.W * sizeof(float);
    if (!staged)
        HIPCHK(h, hipMemcpy2DAsync(h->d_lk_in, row, d_map, (size_t)map_pitch * sizeof(float), row,
                                   g.H, hipMemcpyDeviceToDevice, st));
    HIPCHK(h, timed(h, "lk_refine", (double)g.H * g.W, st, [&] {
               return sgm::launch_lk_refine(d_left, d_right, pitch, h->d_lk_in, d_map, map_pitch, g,
                                            st);
           }));
    return SGM_OK;
}

}  // namespace

extern "C" {

int sgm_default_params(sgm_params *p, int h, int w, int s, int d) {
    if (!p) return SGM_ERR_INVALID_ARG;
    p->height = h;
    p->width = w;
    p->scale = s;
    p->max_disp = d;
    p->p1 = 10;              // SGM.cpp:27
    p->p2 = 100;             // SGM.cpp:28
    p->uniqueness = 0.7f;    // inc/Solver.h:14
    p->lr_max_diff = 1.0f;   // inc/Solver.h:16
    p->blur = 1;             // Solver.cpp:124-125
    p->views = 2;            // SGM.cpp:448-818
    p->post_filter = 0;      // out = LR-checked map (SGM.cpp:818); 1: + post_filter (:821)
    p->lk_refine = 0;        // 1: + LKRefine (SGM.cpp:824, commented out in the reference)
    p->sky_detect = 0;       // 1: masks from SkyAreaDetector::detect on the GPU (node.cpp:80-93)
    p->solver = SGM_SOLVER_SGM;
    p->aux_only = 0;
    p->view = SGM_VIEW_LEFT;
    return SGM_OK;
}

int sgm_create(const sgm_params *p, int device, sgm_handle **out) {
    if (!out) return SGM_ERR_INVALID_ARG;
    *out = nullptr;
    char why[256];
    if (!valid_params(p, why, sizeof(why))) {
        fprintf(stderr, "sgm_create: %s\n", why);
        return SGM_ERR_INVALID_ARG;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SGM_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(device);

    sgm_handle *h = new (std::nothrow) sgm_handle();
    if (!h) return SGM_ERR_OUT_OF_MEMORY;
    h->p = *p;
    h->device = device;
    h->g.scale = p->scale;
    h->g.H = p->height / p->scale;
    h->g.W = p->width / p->scale;
    h->g.D = p->max_disp;
    h->nviews = p->views;
    const size_t npx = (size_t)h->g.H * h->g.W;
    const size_t nvol = npx * h->g.D;
    const size_t nin = (size_t)p->height * p->width;
    h->mf_rows = sgm::median_rows_default(h->g);
    int rc = SGM_OK;
    do {
        if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) { rc = SGM_ERR_HIP; break; }
        hipEvent_t *evs[] = {&h->ev_pf, &h->ev_last};
        for (auto e : evs) {
            // stream-to-stream ordering on this device needs no system-scope
            // fence (L2 writeback/invalidate); the post filter's host
            // readback (ev_pf) keeps it
            const unsigned fl = hipEventDisableTiming | (e == &h->ev_pf ? 0u : hipEventDisableSystemFence);
            if (hipEventCreateWithFlags(e, fl) != hipSuccess) { rc = SGM_ERR_HIP; break; }
        }
        if (rc) break;
        for (int v = 0; v < 2 && !rc; ++v) {
            if ((rc = dalloc(h, &h->d_in[v], nin))) break;
            if ((rc = dalloc(h, &h->d_sky[v], npx))) break;
            if ((rc = dalloc(h, &h->d_ct[v], npx))) break;
        }
        for (int v = 0; v < (p->aux_only ? 0 : h->nviews) && !rc; ++v) {
            // the final pass addresses T (which reuses d_ch) in chunks from
            // their top row, which for the partial last chunk lies up to K-1
            // rows above row 0: d_ch carries that guard in front; the
            // row-walking passes prefetch up to PF positions past the end of
            // the last row of C (never consumed): both carry kVolGuard behind
            const size_t guard = (size_t)sgm::t_guard_rows(h->g.D) * h->g.W * h->g.D;
            if ((rc = dalloc(h, &h->d_ch_base[v], guard + nvol + sgm::kVolGuard))) break;
            h->d_ch[v] = h->d_ch_base[v] + guard;
            if ((rc = dalloc(h, &h->d_c[v], nvol + sgm::kVolGuard))) break;
            if ((rc = dalloc(h, &h->d_s[v], nvol))) break;
            if ((rc = dalloc(h, &h->d_disp[v], npx))) break;
            if ((rc = dalloc(h, &h->d_sub[v], npx))) break;
            for (int f = 0; f < 3 && !rc; ++f)
                rc = dalloc(h, &h->d_ck[v][f], sgm::pair_ckpt_floats(f, h->g));
            // slot 2 also holds vfwd's forward-band state (3 D-vectors per column)
            for (int f = 0; f < 3 && !rc; ++f)
                rc = dalloc(h, &h->d_carry[v][f], (size_t)h->g.W * h->g.D * (f == 2 ? 3 : 1));
        }
        h->band_rows = band_rows_for(h->g);
        if (!rc && p->aux_only) {  // the side stages' maps (stage_lr, the raw map copy)
            for (int v = 0; v < 2 && !rc; ++v) {
                if ((rc = dalloc(h, &h->d_disp[v], npx))) break;
                rc = dalloc(h, &h->d_sub[v], npx);
            }
        } else if (!rc && h->nviews == 1) {  // stage_lr needs a second sub-pixel map
            rc = dalloc(h, &h->d_sub[1], npx);
        }
        if (!rc) rc = dalloc(h, &h->d_cloud_counts, (size_t)h->g.H + 1);
        if (!rc) rc = dalloc(h, &h->d_out, npx);
        if (!rc) rc = dalloc(h, &h->d_min, npx);
        if (!rc) rc = dalloc(h, &h->d_zero, 256);
        if (!rc) rc = dalloc(h, &h->d_pf_orig, npx);
        if (!rc) rc = dalloc(h, &h->d_pf_work, npx);
        if (!rc) rc = dalloc(h, &h->d_pf_label, npx);
        if (!rc) rc = dalloc(h, &h->d_pf_count, npx);
        if (!rc) rc = dalloc(h, &h->d_pf_area, npx);
        if (!rc) rc = dalloc(h, &h->d_pf_snap, sgm::post_snapshot_floats(h->g));
        if (!rc) rc = dalloc(h, &h->d_lk_in, npx);
        if (!rc) rc = dalloc(h, &h->d_sky_scratch, 2 * sgm::sky_scratch_bytes(h->g));
        if (!rc) rc = dalloc(h, &h->d_pf_changes, (size_t)kMedianMaxLaunches);
        if (!rc && hipHostMalloc((void **)&h->h_pf_changes, sizeof(int), hipHostMallocDefault) !=
                       hipSuccess)
            rc = set_err(h, SGM_ERR_HIP, "hipHostMalloc of the post-filter counter failed");
        if (!rc && hipMemset(h->d_zero, 0, 256 * sizeof(float)) != hipSuccess)
            rc = set_err(h, SGM_ERR_HIP, "hipMemset of the zero page failed");
        bool slant_forced = false;
        {
            // the slanted schedule: by size (slant_default), SGM_SLANT=1/0
            // forces it on/off (the parity tests run it at every size)
            const char *e = getenv("SGM_SLANT");
            slant_forced = e && *e == '1';
            const bool want = e && *e ? slant_forced : slant_default(h->g, h->nviews);
            h->slant = !p->aux_only && p->solver == SGM_SOLVER_SGM && want;
            const char *ev = getenv("SGM_VSTRIP");
            h->vstrip = !(ev && *ev == '0');
        }
        const size_t ng = h->slant ? sgm::slant_gran_count(h->g, h->nviews) : 0;
        if (!rc && h->slant) {
            // its two large buffers: the L3 volumes and the hand-off granules
            // (about 28 GB for a 4K256 pair, whose whole handle is about 80 GB:
            // INTEGRATION.md 5), allocated after every common buffer, so that
            // the fallback below covers any shortage they cause
            int arc = SGM_OK;
            for (int v = 0; v < h->nviews && !arc; ++v) arc = dalloc(h, &h->d_l3[v], nvol);
            if (!arc) arc = dalloc(h, &h->d_gran, ng);
#ifdef SGM_SLANT_DEBUG
            if (!arc && getenv("SGM_SLANT_NO_MEMORY"))  // (tests the fallback below)
                arc = set_err(h, SGM_ERR_HIP, "hipMalloc: out of memory (forced, SGM_SLANT_NO_MEMORY)");
#endif
            if (arc && !slant_forced) {
                // chosen by size, not asked for: when the device cannot hold
                // them, the banded schedule (bit-identical maps, no extra
                // volume) instead of failing sgm_create
                for (int v = 0; v < 2; ++v) {
                    if (h->d_l3[v]) h->bytes -= nvol * sizeof(float);
                    (void)hipFree(h->d_l3[v]);
                    h->d_l3[v] = nullptr;
                }
                if (h->d_gran) h->bytes -= ng * sizeof(unsigned long long);
                (void)hipFree(h->d_gran);
                h->d_gran = nullptr;
                (void)hipGetLastError();  // (the failed hipMalloc's error is not the next launch's)
                h->err[0] = 0;
                h->slant = false;
            } else {
                rc = arc;
            }
        }
        if (!rc && h->slant) {
            if (!rc) rc = dalloc(h, &h->d_slant_ctl, 2);
            if (!rc) rc = dalloc(h, &h->d_slant_dummy, 512);
            if (!rc && (hipHostMalloc((void **)&h->h_slant_err, sizeof(unsigned), hipHostMallocMapped) != hipSuccess ||
                        hipHostGetDevicePointer((void **)&h->d_slant_err, h->h_slant_err, 0) != hipSuccess))
                rc = set_err(h, SGM_ERR_HIP, "hipHostMalloc of the slanted schedule's hang-guard word failed");
            if (!rc) *h->h_slant_err = 0;
            if (!rc && (hipStreamCreateWithFlags(&h->st_h, hipStreamNonBlocking) != hipSuccess ||
                        hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
                        hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess))
                rc = set_err(h, SGM_ERR_HIP, "creating the slanted schedule's H-pair stream failed");
            if (!rc && (hipMemset(h->d_gran, 0, ng * sizeof(unsigned long long)) != hipSuccess ||
                        hipMemset(h->d_slant_ctl, 0, 2 * sizeof(sgm::SlantCtl)) != hipSuccess))
                rc = set_err(h, SGM_ERR_HIP, "hipMemset of the slanted schedule's hand-off state failed");
        }
    } while (0);
    if (rc) {
        fprintf(stderr, "sgm_create: %s\n", h->err[0] ? h->err : "HIP stream/event creation failed");
        free_all(h);
        delete h;
        return rc;
    }
    *out = h;
    return SGM_OK;
}

int sgm_destroy(sgm_handle *h) {
    if (!h) return SGM_ERR_INVALID_ARG;
    {
        DeviceGuard guard(h->device);
        (void)hipDeviceSynchronize();
        free_all(h);
    }
    delete h;
    return SGM_OK;
}

const char *sgm_last_error(const sgm_handle *h) { return h ? h->err : "null handle"; }

int sgm_get_size(const sgm_handle *h, int *rows, int *cols, int *max_disp) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (rows) *rows = h->g.H;
    if (cols) *cols = h->g.W;
    if (max_disp) *max_disp = h->g.D;
    return SGM_OK;
}

size_t sgm_device_bytes(const sgm_handle *h) { return h ? h->bytes : 0; }

void *sgm_get_stream(const sgm_handle *h) { return h ? (void *)h->st : nullptr; }

// The slanted passes' hang guard (sgm_slant.hip): a receiver that polls a
// neighbouring tile's hand-off for seconds gives up, and that frame's maps
// are wrong.  It sets a host-mapped word; the next call on the handle (or
// sgm_process, after its own frame) reports it and clears it.
int check_slant_err(sgm_handle *h) {
    // read and clear in one step: a give-up stored by a frame still running
    // between a plain read and a plain clear would be lost
    if (!h->h_slant_err || !__atomic_exchange_n(h->h_slant_err, 0u, __ATOMIC_ACQ_REL)) return SGM_OK;
    return set_err(h, SGM_ERR_HIP, "slanted aggregation: a tile hand-off timed out; that frame's maps are invalid");
}

int sgm_check(sgm_handle *h) {
    if (!h) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    // the last call's work: on a caller's stream its end was recorded in
    // ev_last; on the handle's own stream, that stream (the H pair's stream
    // is joined into the frame's stream before the bottom-up pass)
    if (h->last_st && h->last_recorded) HIPCHK(h, hipEventSynchronize(h->ev_last));
    else if (!h->last_st || h->last_st == h->st) HIPCHK(h, hipStreamSynchronize(h->st));
    else HIPCHK(h, hipDeviceSynchronize());  // a caller's stream whose end could not be recorded
    return check_slant_err(h);
}

int sgm_process_device(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
                       const uint8_t *d_sky_l, const uint8_t *d_sky_r, int sky_pitch,
                       float *d_out, int out_pitch, uint16_t *d_raw_disp, void *stream) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (int rc = check_slant_err(h)) return rc;
    if (!d_left || !d_right || !d_out || pitch < h->p.width || out_pitch < h->g.W ||
        ((d_sky_l || d_sky_r) && sky_pitch < h->g.W))
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_process_device: bad pointer or pitch");
    if (h->p.aux_only)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_process_device: handle created with aux_only");
    DeviceGuard guard(h->device);
    StreamScope scope(h, stream);
    hipStream_t st = scope.st;
    return run_frame(h, d_left, d_right, pitch, d_sky_l, d_sky_r, sky_pitch, d_out, out_pitch,
                     d_raw_disp, st);
}

int sgm_process(sgm_handle *h, const uint8_t *left, const uint8_t *right, int pitch,
                const uint8_t *sky_l, const uint8_t *sky_r, int sky_pitch, float *out,
                int out_pitch, uint16_t *raw_disp) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (!left || !right || !out || pitch < h->p.width || out_pitch < h->g.W ||
        ((sky_l || sky_r) && sky_pitch < h->g.W))
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_process: bad pointer or pitch");
    if (h->p.aux_only)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_process: handle created with aux_only");
    int rc;
    if ((rc = check_slant_err(h))) return rc;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    if ((rc = ensure_pinned(h))) return rc;
    const size_t nin = (size_t)h->p.height * h->p.width, npx = (size_t)h->g.H * h->g.W;
    uint8_t *pl = h->h_pin, *pr = pl + nin, *psl = pr + nin, *psr = psl + npx;
    float *pout = reinterpret_cast<float *>(psr + npx + (16 - (size_t)(psr + npx) % 16) % 16);
    uint16_t *praw = reinterpret_cast<uint16_t *>(pout + npx);
    pack_rows(pl, left, h->p.width, h->p.height, pitch);
    pack_rows(pr, right, h->p.width, h->p.height, pitch);
    HIPCHK(h, hipMemcpyAsync(h->d_in[0], pl, nin, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, hipMemcpyAsync(h->d_in[1], pr, nin, hipMemcpyHostToDevice, h->st));
    if (sky_l) {
        pack_rows(psl, sky_l, h->g.W, h->g.H, sky_pitch);
        HIPCHK(h, hipMemcpyAsync(h->d_sky[0], psl, npx, hipMemcpyHostToDevice, h->st));
    }
    if (sky_r) {
        pack_rows(psr, sky_r, h->g.W, h->g.H, sky_pitch);
        HIPCHK(h, hipMemcpyAsync(h->d_sky[1], psr, npx, hipMemcpyHostToDevice, h->st));
    }
    if ((rc = run_frame(h, h->d_in[0], h->d_in[1], h->p.width, sky_l ? h->d_sky[0] : nullptr,
                        sky_r ? h->d_sky[1] : nullptr, h->g.W, h->d_out, h->g.W,
                        raw_disp ? h->d_disp[0] : nullptr, h->st)))
        return rc;
    HIPCHK(h, hipMemcpyAsync(pout, h->d_out, npx * sizeof(float), hipMemcpyDeviceToHost, h->st));
    if (raw_disp)
        HIPCHK(h, hipMemcpyAsync(praw, h->d_disp[0], npx * sizeof(uint16_t), hipMemcpyDeviceToHost,
                                 h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    if ((rc = check_slant_err(h))) return rc;
    for (int i = 0; i < h->g.H; ++i)
        memcpy(out + (size_t)i * out_pitch, pout + (size_t)i * h->g.W, h->g.W * sizeof(float));
    if (raw_disp) memcpy(raw_disp, praw, npx * sizeof(uint16_t));
    return SGM_OK;
}

#ifdef SGM_SLANT_DEBUG
// hang-guard give-ups of the slanted passes (SlantCtl::err), read and cleared
int sgm_debug_slant_err(sgm_handle *h, unsigned *down, unsigned *up) {
    if (!h || !h->d_slant_ctl) return SGM_ERR_INVALID_ARG;
    sgm::SlantCtl c[2];
    HIPCHK(h, hipDeviceSynchronize());
    HIPCHK(h, hipMemcpy(c, h->d_slant_ctl, sizeof(c), hipMemcpyDeviceToHost));
    *down = c[0].err;
    *up = c[1].err;
    c[0].err = c[1].err = 0;
    HIPCHK(h, hipMemcpy(h->d_slant_ctl, c, sizeof(c), hipMemcpyHostToDevice));
    return SGM_OK;
}
#endif

int sgm_set_profiling(sgm_handle *h, int enable) {
    if (!h) return SGM_ERR_INVALID_ARG;
    h->profiling = enable ? 1 : 0;
    return SGM_OK;
}

int sgm_get_profile(sgm_handle *h, sgm_kernel_stat *out, int max, int *count) {
    if (!h) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    HIPCHK(h, hipDeviceSynchronize());
    for (auto &p : h->pending) {
        float ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&ms, p.a, p.b));
        h->stats[p.cls].launches += 1;
        h->stats[p.cls].total_ms += ms;
        h->stat_elems[p.cls] += p.elems;
        h->ev_pool.push_back(p.a);
        h->ev_pool.push_back(p.b);
    }
    h->pending.clear();
    int n = 0;
    for (size_t k = 0; k < h->stats.size(); ++k) {
        sgm_kernel_stat &st = h->stats[k];
        if (st.launches == 0) continue;
        st.elems = h->stat_elems[k] / st.launches;  // banded launches differ in size
        if (out && n < max) out[n] = st;
        ++n;
    }
    if (count) *count = out ? (n < max ? n : max) : n;
    for (auto &st : h->stats) { st.launches = 0; st.total_ms = 0; }
    for (auto &e : h->stat_elems) e = 0.0;
    return SGM_OK;
}

// -------------------------------------------------------------- stages

int sgm_stage_census(sgm_handle *h, const uint8_t *img, int pitch, uint64_t *ct) {
    if (!h || !img || !ct || pitch < h->p.width) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    int rc;
    if ((rc = copy_in_image(h, h->d_in[0], img, pitch))) return rc;
    HIPCHK(h, sgm::launch_census(h->d_in[0], h->p.width, h->g, h->p.blur, h->d_ct[0], h->st));
    HIPCHK(h, hipMemcpyAsync(ct, h->d_ct[0], (size_t)h->g.H * h->g.W * sizeof(uint64_t),
                             hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

int sgm_stage_cost(sgm_handle *h, const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
                   int view, int filters, float *cost) {
    if (!h || !ctl || !ctr || !cost || (view != 0 && view != 1)) return SGM_ERR_INVALID_ARG;
    if (h->p.aux_only) return set_err(h, SGM_ERR_INVALID_ARG, "stage needs cost volumes (aux_only)");
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W, nvol = npx * h->g.D;
    HIPCHK(h, hipMemcpyAsync(h->d_ct[0], ctl, npx * 8, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, hipMemcpyAsync(h->d_ct[1], ctr, npx * 8, hipMemcpyHostToDevice, h->st));
    if (sky) HIPCHK(h, hipMemcpyAsync(h->d_sky[0], sky, npx, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, sgm::launch_cost_h(h->d_ct[0], h->d_ct[1], sky ? h->d_sky[0] : nullptr, h->g.W, view,
                                 filters & 1, h->g, h->d_ch[0], h->st));
    const float *res = h->d_ch[0];
    if (filters & 2) {  // the frame's own vfwd, in place when the frames run it so
        sgm::PairArgs pa = pair_args(h);
        pa.ckpt = h->d_ck[0][sgm::PAIR_V];
        HIPCHK(h, sgm::launch_vfwd(h->d_ch[0], cost_buf(h, 0), pa, h->g, h->st));
        res = cost_buf(h, 0);
    }
    HIPCHK(h, hipMemcpyAsync(cost, res, nvol * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

int sgm_stage_path(sgm_handle *h, int dir, const float *cost, float *L, float *minL) {
    if (!h || !cost || !L || dir < 0 || dir > 7) return SGM_ERR_INVALID_ARG;
    if (h->p.aux_only) return set_err(h, SGM_ERR_INVALID_ARG, "stage needs cost volumes (aux_only)");
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W, nvol = npx * h->g.D;
    HIPCHK(h, hipMemcpyAsync(h->d_c[0], cost, nvol * 4, hipMemcpyHostToDevice, h->st));
    SweepArgs a = sweep_args(h);
    a.cost = h->d_c[0];
    a.acc_out = h->d_s[0];
    a.min_out = h->d_min;
    HIPCHK(h, sgm::launch_sweep(dir, sgm::SWEEP_STORE_L, a, h->g, h->st));
    HIPCHK(h, hipMemcpyAsync(L, h->d_s[0], nvol * 4, hipMemcpyDeviceToHost, h->st));
    if (minL) HIPCHK(h, hipMemcpyAsync(minL, h->d_min, npx * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

int sgm_stage_aggregate(sgm_handle *h, const float *cost, uint16_t *disp, float *sub) {
    if (!h || !cost) return SGM_ERR_INVALID_ARG;
    if (h->p.aux_only) return set_err(h, SGM_ERR_INVALID_ARG, "stage needs cost volumes (aux_only)");
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W, nvol = npx * h->g.D;
    HIPCHK(h, hipMemcpyAsync(h->d_c[0], cost, nvol * 4, hipMemcpyHostToDevice, h->st));
    int rc = aggregate_view(h, 0, h->d_c[0], h->d_s[0], h->d_ch[0], h->d_disp[0], h->d_sub[0],
                            h->st, true);
    if (rc) return rc;
    if (disp) HIPCHK(h, hipMemcpyAsync(disp, h->d_disp[0], npx * 2, hipMemcpyDeviceToHost, h->st));
    if (sub) HIPCHK(h, hipMemcpyAsync(sub, h->d_sub[0], npx * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

int sgm_lr_check_device(sgm_handle *h, const float *d_fl, int fl_pitch, const float *d_fr,
                        int fr_pitch, float *d_out, int out_pitch, void *stream) {
    if (!h) return SGM_ERR_INVALID_ARG;
    const int W = h->g.W;
    if (!d_fl || !d_fr || !d_out || fl_pitch < W || fr_pitch < W || out_pitch < W)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_lr_check_device: bad pointer or pitch");
    if (d_out == d_fr)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_lr_check_device: d_out must not alias d_fr");
    DeviceGuard guard(h->device);
    StreamScope scope(h, stream);
    hipStream_t st = scope.st;
    HIPCHK(h, timed(h, "lr", (double)h->g.H * W, st, [&] {
               return sgm::launch_lr(d_fl, fl_pitch, d_fr, fr_pitch, d_out, out_pitch,
                                     h->p.lr_max_diff, h->g, st);
           }));
    return SGM_OK;
}

int sgm_post_filter_device(sgm_handle *h, float *d_disp, int pitch, void *stream) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (!d_disp || pitch < h->g.W)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_post_filter_device: bad pointer or pitch");
    DeviceGuard guard(h->device);
    StreamScope scope(h, stream);
    return post_filter(h, d_disp, pitch, scope.st);
}

int sgm_lk_refine_device(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
                         float *d_disp, int disp_pitch, void *stream) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (!d_left || !d_right || !d_disp || pitch < h->p.width || disp_pitch < h->g.W)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_lk_refine_device: bad pointer or pitch");
    DeviceGuard guard(h->device);
    StreamScope scope(h, stream);
    return lk_refine(h, d_left, d_right, pitch, d_disp, disp_pitch, scope.st);
}

int sgm_stage_lk_refine(sgm_handle *h, const uint8_t *left, const uint8_t *right, int pitch,
                        float *disp) {
    if (!h || !left || !right || !disp || pitch < h->p.width) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W;
    int rc;
    if ((rc = copy_in_image(h, h->d_in[0], left, pitch))) return rc;
    if ((rc = copy_in_image(h, h->d_in[1], right, pitch))) return rc;
    HIPCHK(h, hipMemcpyAsync(h->d_out, disp, npx * 4, hipMemcpyHostToDevice, h->st));
    if ((rc = lk_refine(h, h->d_in[0], h->d_in[1], h->p.width, h->d_out, h->g.W, h->st))) return rc;
    HIPCHK(h, hipMemcpyAsync(disp, h->d_out, npx * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

int sgm_sky_detect_device(sgm_handle *h, const uint8_t *d_img, int pitch, uint8_t *d_mask,
                          int mask_pitch, void *stream) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (!d_img || !d_mask || pitch < h->p.width || mask_pitch < h->g.W)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_sky_detect_device: bad pointer or pitch");
    DeviceGuard guard(h->device);
    StreamScope scope(h, stream);
    hipStream_t st = scope.st;
    HIPCHK(h, timed(h, "sky_detect", (double)h->g.H * h->g.W, st, [&] {
               return sgm::launch_sky_detect(&d_img, pitch, &d_mask, mask_pitch, h->d_sky_scratch,
                                             1, h->g, st);
           }));
    return SGM_OK;
}

int sgm_stage_sky_detect(sgm_handle *h, const uint8_t *img, int pitch, uint8_t *mask) {
    if (!h || !img || !mask || pitch < h->p.width) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W;
    int rc;
    if ((rc = copy_in_image(h, h->d_in[0], img, pitch))) return rc;
    if ((rc = sgm_sky_detect_device(h, h->d_in[0], h->p.width, h->d_sky[0], h->g.W, h->st)))
        return rc;
    HIPCHK(h, hipMemcpyAsync(mask, h->d_sky[0], npx, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

int sgm_colormap_device(sgm_handle *h, const float *d_disp, int pitch, uint8_t *d_bgr,
                        int bgr_pitch, void *stream) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (!d_disp || !d_bgr || pitch < h->g.W || bgr_pitch < 3 * h->g.W)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_colormap_device: bad pointer or pitch");
    DeviceGuard guard(h->device);
    StreamScope scope(h, stream);
    hipStream_t st = scope.st;
    HIPCHK(h, timed(h, "colormap", (double)h->g.H * h->g.W, st, [&] {
               return sgm::launch_colormap(d_disp, pitch, d_bgr, bgr_pitch, h->g, st);
           }));
    return SGM_OK;
}

int sgm_point_cloud_device(sgm_handle *h, const float *d_disp, int pitch, const uint8_t *d_img,
                           int img_pitch, const sgm_camera *cam, double *d_xyz,
                           uint8_t *d_pixel, int *d_count, void *stream) {
    if (!h) return SGM_ERR_INVALID_ARG;
    if (!d_disp || !d_img || !cam || !d_xyz || !d_pixel || !d_count || pitch < h->g.W ||
        img_pitch < h->g.W)
        return set_err(h, SGM_ERR_INVALID_ARG, "sgm_point_cloud_device: bad pointer or pitch");
    DeviceGuard guard(h->device);
    StreamScope scope(h, stream);
    hipStream_t st = scope.st;
    HIPCHK(h, timed(h, "point_cloud", (double)h->g.H * h->g.W, st, [&] {
               return sgm::launch_point_cloud(d_disp, pitch, d_img, img_pitch, cam->fx, cam->fy,
                                              cam->cx, cam->cy, cam->baseline, cam->max_range,
                                              h->d_cloud_counts, d_xyz, d_pixel, d_count, h->g,
                                              st);
           }));
    return SGM_OK;
}

int sgm_stage_colormap(sgm_handle *h, const float *disp, uint8_t *bgr) {
    if (!h || !disp || !bgr) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W;
    // staging: the map in d_out, the BGR image over the two working-grid sky masks' space
    uint8_t *d_bgr = nullptr;
    HIPCHK(h, hipMallocAsync((void **)&d_bgr, 3 * npx, h->st));
    HIPCHK(h, hipMemcpyAsync(h->d_out, disp, npx * 4, hipMemcpyHostToDevice, h->st));
    int rc = sgm_colormap_device(h, h->d_out, h->g.W, d_bgr, 3 * h->g.W, h->st);
    if (!rc) {
        HIPCHK(h, hipMemcpyAsync(bgr, d_bgr, 3 * npx, hipMemcpyDeviceToHost, h->st));
    }
    HIPCHK(h, hipFreeAsync(d_bgr, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return rc;
}

int sgm_stage_point_cloud(sgm_handle *h, const float *disp, const uint8_t *img, int img_pitch,
                          const sgm_camera *cam, double *xyz, uint8_t *pixel, int *count) {
    if (!h || !disp || !img || !cam || !xyz || !pixel || !count || img_pitch < h->g.W)
        return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W;
    const int rows_used = h->g.H;  // the node reads img(i, j) at working-grid indices
    uint8_t *d_img = nullptr, *d_pix = nullptr;
    double *d_xyz = nullptr;
    int *d_n = nullptr;
    HIPCHK(h, hipMallocAsync((void **)&d_img, (size_t)rows_used * img_pitch, h->st));
    HIPCHK(h, hipMallocAsync((void **)&d_pix, npx, h->st));
    HIPCHK(h, hipMallocAsync((void **)&d_xyz, 3 * npx * sizeof(double), h->st));
    HIPCHK(h, hipMallocAsync((void **)&d_n, sizeof(int), h->st));
    HIPCHK(h, hipMemcpyAsync(d_img, img, (size_t)rows_used * img_pitch, hipMemcpyHostToDevice,
                             h->st));
    HIPCHK(h, hipMemcpyAsync(h->d_out, disp, npx * 4, hipMemcpyHostToDevice, h->st));
    int rc = sgm_point_cloud_device(h, h->d_out, h->g.W, d_img, img_pitch, cam, d_xyz, d_pix, d_n,
                                    h->st);
    if (!rc) {
        HIPCHK(h, hipMemcpyAsync(count, d_n, sizeof(int), hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
        HIPCHK(h, hipMemcpyAsync(xyz, d_xyz, 3 * (size_t)*count * sizeof(double),
                                 hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipMemcpyAsync(pixel, d_pix, (size_t)*count, hipMemcpyDeviceToHost, h->st));
    }
    HIPCHK(h, hipFreeAsync(d_img, h->st));
    HIPCHK(h, hipFreeAsync(d_pix, h->st));
    HIPCHK(h, hipFreeAsync(d_xyz, h->st));
    HIPCHK(h, hipFreeAsync(d_n, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return rc;
}

int sgm_stage_post_filter(sgm_handle *h, float *disp) {
    if (!h || !disp) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W;
    HIPCHK(h, hipMemcpyAsync(h->d_out, disp, npx * 4, hipMemcpyHostToDevice, h->st));
    int rc = post_filter(h, h->d_out, h->g.W, h->st);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(disp, h->d_out, npx * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

int sgm_stage_lr(sgm_handle *h, const float *fl, const float *fr, float *out) {
    if (!h || !fl || !fr || !out) return SGM_ERR_INVALID_ARG;
    DeviceGuard guard(h->device);
    StreamScope scope(h, nullptr);
    const size_t npx = (size_t)h->g.H * h->g.W;
    HIPCHK(h, hipMemcpyAsync(h->d_sub[0], fl, npx * 4, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, hipMemcpyAsync(h->d_sub[1], fr, npx * 4, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, sgm::launch_lr(h->d_sub[0], h->g.W, h->d_sub[1], h->g.W, h->d_out, h->g.W,
                             h->p.lr_max_diff, h->g, h->st));
    HIPCHK(h, hipMemcpyAsync(out, h->d_out, npx * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return SGM_OK;
}

}  // extern "C"
