/*
 * sgm_oracle.h -- CPU restatement of hilbertw/stereo_matching's CPU SGM path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libsgm_hip.so, the
 * stereo_matching_amd package) may link, load or call this code.  It is used
 * by tests/ as the parity checker, by __graft_entry__.smoke() as the checker,
 * and by bench.py's cpu_baseline leg as the timed CPU baseline ("kind": "port",
 * orc_process_refplace: the reference's OpenMP placement).
 *
 * PARITY STATUS: "parity unpinned".  The reference (C++/OpenCV/ROS catkin
 * package) is unbuildable in this image: src/{Solver,SGM,cost}.cpp include
 * inc/global.h, which pulls OpenCV, ROS, cv_bridge and image_transport headers
 * (inc/global.h:11-20) that the image does not have, and the rules of this
 * build forbid writing stand-ins for them.  The reference ships no tests, no
 * fixtures and no golden vectors.  This restatement is
 * therefore cross-checked only against an independent pure-Python restatement
 * (tests/pyref.py) and hand-derived known-answer cases (tests/test_oracle.py).
 *
 * Every function cites the reference lines it restates.  Float arithmetic is
 * written in the reference's exact association order and must be compiled with
 * -ffp-contract=off and without -ffast-math (see oracle/Makefile).
 */
#ifndef SGM_ORACLE_H
#define SGM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Direction ids, numbered like the reference's L1..L8 (src/SGM.cpp:81-369). */
enum {
    ORC_L1 = 0, /* ->  predecessor (i, j-1)   src/SGM.cpp:81-119  */
    ORC_L2 = 1, /* <-  predecessor (i, j+1)   src/SGM.cpp:121-159 */
    ORC_L3 = 2, /* v   predecessor (i-1, j)   src/SGM.cpp:161-199 */
    ORC_L4 = 3, /* ^   predecessor (i+1, j)   src/SGM.cpp:201-239 */
    ORC_L5 = 4, /* \v  predecessor (i-1, j-1) src/SGM.cpp:247-305 */
    ORC_L6 = 5, /* /v  predecessor (i-1, j+1) src/SGM.cpp:247-305 */
    ORC_L7 = 6, /* /^  predecessor (i+1, j-1) src/SGM.cpp:311-369 */
    ORC_L8 = 7  /* \^  predecessor (i+1, j+1) src/SGM.cpp:311-369 */
};

/* Pinned stand-in for cv::GaussianBlur(img, out, Size(3,3), 2, 1)
 * (src/Solver.cpp:124-125): OpenCV 3.x CV_8U fixed-point separable filter,
 * kernels round(256*gauss) = [82,93,82] (sigma 2, x) and [70,116,70]
 * (sigma 1, y), BORDER_REFLECT_101, (acc + 2^15) >> 16, saturate to u8. */
void orc_blur(const uint8_t *src, uint8_t *dst, int H, int W);

/* CT_pts (src/cost.cpp:99-129) for one image: census word per pixel. */
void orc_census(const uint8_t *img, uint64_t *ct, int H, int W, int scale);

/* build_dsi_from_table (view 0, src/Solver.cpp:143-194) and
 * build_dsi_from_table_beta (view 1, src/Solver.cpp:197-248).
 * sky may be NULL (Solver.cpp:146). cost is HWD float32. */
void orc_dsi(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
             float *cost, int H, int W, int D, int scale, int view);

/* cost_horizontal_filter / cost_vertical_filter (src/Solver.cpp:296-368). */
void orc_hfilter(float *cost, int H, int W, int D, int win);
void orc_vfilter(float *cost, int H, int W, int D, int win);

/* One path direction: L (HWD) and minL (HW).  src/SGM.cpp:81-369. */
void orc_path(const float *cost, float *L, float *minL, int H, int W, int D,
              int dir, int P1, int P2);

/* Aggregation (src/SGM.cpp:386-390): S = ((L1+L2)+L3)+L4; S += ((L5+L6)+L7)+L8. */
void orc_aggregate(const float *const *L, float *S, int H, int W, int D);

/* WTA + uniqueness (src/SGM.cpp:376-418).  disp is int32 (invalid = D+1). */
void orc_wta(const float *S, int32_t *disp, int H, int W, int D, float uniq);

/* compute_subpixel (src/Solver.cpp:569-597). */
void orc_subpixel(const int32_t *disp, const float *S, float *out, int H, int W, int D);

/* LR check (src/SGM.cpp:803-818), in place on FL. */
void orc_lr_check(float *FL, const float *FR, int H, int W, int D, int scale, float lr_dis);

/* post_filter (src/Solver.cpp:600-649): 5x5 median fill + speckle removal
 * (speckle_filter_new, Solver.cpp:514-566) with its single-thread semantics. */
void orc_post_filter(float *F, int H, int W, int D, int scale);

/* LKRefine (LKRefine/LKSubPixelImpl.cpp:13-235) on working-grid images L, R
 * and a working-grid disparity map (refined in place); see sgm_oracle.c for
 * the pinned fp32 evaluation order of its Eigen expressions. */
void orc_lk_refine(const uint8_t *L, const uint8_t *R, float *disp, int H, int W, int D);

/* SkyAreaDetector::detect (sky_detector/imageSkyDetector.cpp:166-208) on a
 * single-channel h x w image (row pitch bytes) at scale s: mask on the
 * working grid (h/s x w/s), 255 = sky.  Pinned numerics: see sgm_oracle.c. */
void orc_sky_detect(const uint8_t *img, int h, int w, int pitch, int scale, uint8_t *mask);

/* BM::process (src/BM.cpp:9-97) on full-size inputs: raw WTA disparity of
 * the filtered cost, int32 rows x cols, invalid = D+1. */
int orc_bm_process(const uint8_t *left, const uint8_t *right, const uint8_t *sky,
                   int h, int w, int scale, int D, float uniq, int blur, int32_t *disp);

typedef struct orc_result {
    /* all optional (NULL = not wanted); sizes use the working (decimated) h, w */
    int32_t *disp;          /* left WTA disparity, HW */
    int32_t *disp_beta;     /* right WTA disparity, HW */
    float   *sub;           /* left sub-pixel disparity before LR check, HW */
    float   *sub_beta;      /* right sub-pixel disparity, HW */
    float   *lr;            /* left sub-pixel disparity after LR check, HW */
    float   *final_disp;    /* after post_filter, HW (what get_disp() returns) */
} orc_result;

/* The whole SGM::process (src/SGM.cpp:32-826) on full-size inputs h x w.
 * views = 1 stops after the left view (no right view, no LR, no post filter).
 * blur = 0 skips the pre-blur (census on raw pixels).  Returns 0 on success. */
int orc_process(const uint8_t *left, const uint8_t *right,
                const uint8_t *sky_l, const uint8_t *sky_r,
                int h, int w, int scale, int D, int P1, int P2,
                float uniq, float lr_dis, int blur, int views, orc_result *res);

/* The same outputs as orc_process from 3 cost-sized volumes instead of 10
 * (C, S = ((L1+L2)+L3)+L4, T = L5+L6; the paths stream their chain state and
 * add in the reference's association order).  Bit-identical to orc_process;
 * used where 10 volumes do not fit (4K256: 25.5 GB instead of 85 GB). */
int orc_process_lean(const uint8_t *left, const uint8_t *right,
                     const uint8_t *sky_l, const uint8_t *sky_r,
                     int h, int w, int scale, int D, int P1, int P2,
                     float uniq, float lr_dis, int blur, int views, orc_result *res);

/* The same outputs as orc_process with the reference's OpenMP placement and
 * memory (cost + 8 path volumes): parallel only where the reference has
 * `omp parallel for` (census and DSI rows, L1/L2 rows, L3/L4 columns, the
 * columns of each row of the L5/L6 and L7/L8 pair loops, sub-pixel rows, LR
 * rows); both cost filters and the fused aggregation + WTA sequential
 * (Solver.cpp:296-368, SGM.cpp:372-418).  bench.py's CPU baseline. */
int orc_process_refplace(const uint8_t *left, const uint8_t *right,
                         const uint8_t *sky_l, const uint8_t *sky_r,
                         int h, int w, int scale, int D, int P1, int P2,
                         float uniq, float lr_dis, int blur, int views, orc_result *res);

/* Threads the OpenMP regions will use (1 if built without OpenMP). */
int orc_max_threads(void);
void orc_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
