/*
 * sgm_hip.h -- C-ABI of libsgm_hip.so, the MI355X-native semi-global matcher.
 *
 * This library replaces the reference's dormant CUDA backend (gpu_sgm/,
 * class GPU_SGM, gpu_sgm/inc/SGM.cuh:23-62) and the CPU hot path it mirrors
 * (class SGM : Solver, inc/SGM.h:10-26, inc/Solver.h:23-70).  Plain C: plain
 * pointers and sizes, no STL, no OpenCV, no torch types.  The C++ class
 * surface with the reference's signatures (include/sgm_amd/SGM.h) and the
 * Python mirror (stereo_matching_amd/) are thin layers over these entry
 * points; INTEGRATION.md shows how the ROS node binds it.
 *
 * Semantics follow src/SGM.cpp / src/Solver.cpp bit-for-bit:
 * float32 costs, P1=10, P2=100, uniqueness 0.7, LR threshold 1.0, invalid
 * disparity D+1.  The reference's domain d in {32,64,128} (Solver.cpp:10) is
 * widened to 256; raw WTA disparities are therefore uint16 (the reference's
 * uchar would wrap D+1 = 257).
 *
 * Threading: a handle is bound to one device and is not thread-safe (one
 * frame at a time, like the reference object, Solver.h:29-30).  Use one
 * handle per device/thread.
 *
 * Stream arguments: NULL = the handle's own stream, created non-blocking (so
 * NOT ordered with the legacy default stream); hipStreamLegacy ((void *)1)
 * = the legacy default stream; otherwise a hipStream_t.
 *
 * Streams: every call on a handle uses the handle's device scratch (cost
 * volumes, checkpoints, post-filter and LKRefine buffers), so the library
 * orders calls made on different streams: a call whose stream differs from
 * the previous call's first makes its stream wait for the previous call's
 * work.  A call on a caller's stream records an event on that stream as it
 * returns (so the library keeps no caller stream past the call that used
 * it; a rocprof trace shows the record as a ~5 us gap before the next
 * kernel); calls on the handle's own stream (NULL, sgm_get_stream) record
 * nothing.  Device entry points return after
 * enqueueing, EXCEPT with post_filter: its median fill blocks the calling
 * host thread on an event once per two fill launches to read a convergence
 * counter (sgm_post_filter_device, and sgm_process_device with
 * params.post_filter), so those calls are not fully asynchronous.
 */
#ifndef SGM_HIP_H
#define SGM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGM_HIP_VERSION 1

/* Status codes (the reference only asserts, Solver.cpp:6-10; GPU errors were
 * printed and ignored, gpu_sgm/inc/cuda_inc.cuh:4-9 -- here they are returned). */
enum {
    SGM_OK = 0,
    SGM_ERR_INVALID_ARG = 1,   /* a reference assert would have fired */
    SGM_ERR_OUT_OF_MEMORY = 2,
    SGM_ERR_HIP = 3,           /* HIP runtime error; see sgm_last_error() */
    SGM_ERR_NO_DEVICE = 4
};

/* Path directions, numbered like the reference's L1..L8 (src/SGM.cpp:81-369). */
enum {
    SGM_DIR_L1 = 0, /* left -> right        */
    SGM_DIR_L2 = 1, /* right -> left        */
    SGM_DIR_L3 = 2, /* top -> down          */
    SGM_DIR_L4 = 3, /* down -> top          */
    SGM_DIR_L5 = 4, /* left-top -> right-down  */
    SGM_DIR_L6 = 5, /* right-top -> left-down  */
    SGM_DIR_L7 = 6, /* left-down -> right-top  */
    SGM_DIR_L8 = 7  /* right-down -> left-top  */
};

/* Matching algorithm: the Solver subclasses of the reference (node.cpp:49-50). */
enum {
    SGM_SOLVER_SGM = 0,  /* class SGM (inc/SGM.h:10-26, src/SGM.cpp) */
    SGM_SOLVER_BM = 1    /* class BM (inc/BM.h:6-19, src/BM.cpp): filtered-cost WTA, left view */
};

typedef struct sgm_params {
    int height;        /* input image rows (before decimation)      Solver(h,..) */
    int width;         /* input image cols                           Solver(.,w,..) */
    int scale;         /* 1 or 2: decimation (Solver.cpp:8,12-13; SGM.cpp:40-61) */
    int max_disp;      /* D in {32,64,128,256} (Solver.cpp:10, widened)          */
    int p1;            /* 10  (SGM.cpp:27) */
    int p2;            /* 100 (SGM.cpp:28) */
    float uniqueness;  /* 0.7 UNIQUE_RATIO (inc/Solver.h:14); must exceed 8*(p2+999999)/FLT_MAX
                          (about 2e-32): at or below it the reference's WTA would read the
                          previous pixel's sec_min_d (SGM.cpp:392-408), so sgm_create rejects it */
    float lr_max_diff; /* 1.0 LR_CHECK_DIS (inc/Solver.h:16) */
    int blur;          /* 1: pre-blur as Solver.cpp:124-125 (pinned formula); 0: off */
    int views;         /* 2: left+right views + LR check (SGM.cpp:32-818); 1: left view only */
    int post_filter;   /* 1: sgm_process[_device] output is post_filter()ed on the GPU
                          (Solver.cpp:600-649, what get_disp() returns, SGM.cpp:821);
                          0 (default): the LR-checked map (filtered_disp at SGM.cpp:818) */
    int lk_refine;     /* 1: then LKRefine on the GPU (LKSubPixelImpl.cpp:13-235; the call
                          at SGM.cpp:824 is commented out in the reference); 0 (default) */
    int sky_detect;    /* 1: the sky masks of both views come from SkyAreaDetector::detect
                          run on the GPU over the input images (node.cpp:80-93), replacing
                          any masks passed in; 0 (default): masks as passed (or none).
                          Working grid up to 8192 columns and 4784 rows */
    int solver;        /* SGM_SOLVER_SGM (default) or SGM_SOLVER_BM.  BM: out = the raw
                          WTA disparity as float (BM.cpp:53-85; post_filter()ed when
                          post_filter is set, BM.cpp:88), raw_disp = the same as u16;
                          views, lk_refine and the right sky mask are unused */
    int aux_only;      /* 1: a light handle for the per-frame side stages only (sky detector,
                          post_filter, LKRefine, colormap, point cloud): no cost volumes are
                          allocated and sgm_process[_device] refuse; 0 (default) */
    int view;          /* with views == 1: SGM_VIEW_LEFT (default), the left view
                          (SGM.cpp:32-445, disp/filtered_disp); or SGM_VIEW_RIGHT, the right
                          view alone (SGM.cpp:448-801: build_dsi_from_table_beta, the same
                          8 paths, disp_beta/filtered_disp_beta), so that a pair's two views
                          can run on two GPUs and meet in sgm_lr_check_device.
                          A right-view handle has no post_filter/lk_refine (they follow the
                          LR check on the left view's GPU) and uses sky_r (or the right image's
                          detected mask) */
} sgm_params;

enum { SGM_VIEW_LEFT = 0, SGM_VIEW_RIGHT = 1 };

/* Camera of the point cloud (CamIntrinsics, inc/utils.h:14-20, plus the two
 * constants of node.cpp:122-123). */
typedef struct sgm_camera {
    float fx, fy, cx, cy;
    double baseline;   /* 0.5 in node.cpp:123 */
    float max_range;   /* 100 in node.cpp:122 */
} sgm_camera;

typedef struct sgm_handle sgm_handle;

/* Fills p with the reference defaults for SGM(h, w, s, d) (node.cpp:49). */
int sgm_default_params(sgm_params *p, int h, int w, int s, int d);

/* Allocates every device buffer up front, as the reference constructors do
 * (Solver.cpp:18-27, SGM.cpp:7-24).  device = HIP ordinal.  Where the
 * slanted-tile schedule is chosen by size (HD/4K at D >= 128) and the device
 * cannot hold its extra buffers (a full L3 volume per view and the hand-off
 * granules, ~80 GB for a 4K256 pair), the handle takes the banded schedule
 * instead (the same maps, bit for bit); with SGM_SLANT=1 the allocation
 * failure is returned. */
int sgm_create(const sgm_params *p, int device, sgm_handle **out);
int sgm_destroy(sgm_handle *h);
const char *sgm_last_error(const sgm_handle *h);
/* Working (decimated) size: rows = height/scale, cols = width/scale. */
int sgm_get_size(const sgm_handle *h, int *rows, int *cols, int *max_disp);
/* Bytes of device memory the handle holds. */
size_t sgm_device_bytes(const sgm_handle *h);
/* The handle's own stream (a hipStream_t; what a NULL stream argument
 * means), valid until sgm_destroy; NULL for a NULL handle.  A caller that
 * runs its own work around the handle's calls can enqueue it on this stream
 * (e.g. as torch.cuda.ExternalStream) and pass NULL: calls on the handle's
 * stream record no events, while a call on a caller's stream records one as
 * it returns (see "Streams" above). */
void *sgm_get_stream(const sgm_handle *h);

/*
 * SGM::process(l, r, sky, sky_beta) (src/SGM.cpp:32-826, :829-834) up to and
 * including the LR check, on HOST buffers; synchronous.
 *   left/right : u8, height x width, row pitch in bytes
 *   sky_l/sky_r: u8 masks on the working grid (rows x cols), 255 = sky; may be
 *                NULL (Solver.cpp:146)
 *   out        : f32 rows x cols, LR-checked sub-pixel disparity
 *                (filtered_disp after SGM.cpp:818), invalid = D+1; with
 *                params.post_filter it is then post_filter()ed on the GPU
 *                (SGM.cpp:821, what get_disp() returns); with views == 1 it
 *                is the left sub-pixel map (SGM.cpp:443), or the right one
 *                (filtered_disp_beta, SGM.cpp:801) with params.view == SGM_VIEW_RIGHT
 *   raw_disp   : optional u16 rows x cols, left WTA disparity (SGM.cpp:411-415;
 *                disp_beta, SGM.cpp:755-795, with SGM_VIEW_RIGHT)
 */
int sgm_process(sgm_handle *h, const uint8_t *left, const uint8_t *right, int pitch,
                const uint8_t *sky_l, const uint8_t *sky_r, int sky_pitch,
                float *out, int out_pitch, uint16_t *raw_disp);

/* Same on DEVICE buffers, enqueued on `stream` (a hipStream_t; NULL = the
 * handle's own stream).  Returns after enqueueing; the caller synchronises.
 * With params.post_filter the call synchronises `stream` during the median
 * fill's convergence test (sgm_post_filter_device).
 * Volumes above the Infinity Cache may run the slanted-tile passes
 * (DESIGN.md 5e), whose tile-to-tile hand-offs poll with a bounded spin: a
 * frame in which a poll gave up (seconds without progress: a hung or
 * preempted neighbour; later polls of that launch then skip their wait) has
 * invalid maps.  sgm_check() reports it once the frame's work is done; the
 * NEXT sgm_process_device / sgm_process call on the handle also returns
 * SGM_ERR_HIP for it (sgm_process checks right after its own frame). */
int sgm_process_device(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
                       const uint8_t *d_sky_l, const uint8_t *d_sky_r, int sky_pitch,
                       float *d_out, int out_pitch, uint16_t *d_raw_disp, void *stream);

/* Post-sync validity check of the frames enqueued so far (the reference has
 * no asynchronous work to check: SGM::process is synchronous, SGM.cpp:32-826).
 * Waits for the handle's last call's work (its stream, or the event the call
 * recorded on the caller's stream), then returns SGM_ERR_HIP, with the
 * message in sgm_last_error, if any slanted-pass hand-off gave up since the
 * last report -- the maps of the frames in between are then invalid -- and
 * clears the report; else SGM_OK.  Frames replayed from a captured HIP graph
 * are not calls on the handle: synchronise the graph's stream first, then
 * call sgm_check.  A caller that gathers or times maps should call it after
 * synchronising and before trusting them. */
int sgm_check(sgm_handle *h);

/* The LR check of SGM.cpp:803-818 on DEVICE working-grid maps: out(i, j) =
 * fl(i, j), or D+1 where j >= fl and |fl - fr(i, (int)(j - fl/s))| > lr_max_diff.
 * fl is the left view's sub-pixel map (filtered_disp), fr the right view's
 * (filtered_disp_beta), e.g. from two SGM_VIEW_LEFT / SGM_VIEW_RIGHT handles on
 * two GPUs with fr copied over; pitches in floats; d_out may alias d_fl but not
 * d_fr.  Any handle of the working size (aux_only included) serves.  Enqueued
 * on `stream` (NULL = the handle's stream); sgm_post_filter_device and
 * sgm_lk_refine_device then complete get_disp()'s map. */
int sgm_lr_check_device(sgm_handle *h, const float *d_fl, int fl_pitch, const float *d_fr,
                        int fr_pitch, float *d_out, int out_pitch, void *stream);

/* post_filter() (Solver.cpp:600-649: median fill :604-630, speckle_filter_new
 * :514-566) on the GPU, bit-exact against its single-thread semantics, in
 * place on a DEVICE map of the handle's working size (rows x cols f32, row
 * pitch in floats), enqueued on `stream` (NULL = the handle's stream).  The
 * median fill iterates to a proven fixed point; the call synchronises
 * `stream` once per two fill launches to read the convergence counter, and
 * returns with the speckle kernels enqueued (the caller synchronises). */
int sgm_post_filter_device(sgm_handle *h, float *d_disp, int pitch, void *stream);

/* LKSubPixelImpl::LKRefine(img_l, img_r, disp_float) (LKRefine/LKSubPixelImpl.cpp:
 * 13-235) on the GPU: per-pixel Gauss-Newton refinement of the disparity over
 * a 7x7 window, interior pixels truncated first (:80), border pixels untouched.
 * d_left/d_right: DEVICE u8 images at the handle's full size (height x width,
 * row pitch in bytes), decimated by the scale as :29-44 does; d_disp: DEVICE
 * working-grid map (rows x cols f32, pitch in floats), refined in place.
 * Enqueued on `stream` (NULL = the handle's stream); the caller synchronises.
 * fp32 sums follow oracle/sgm_oracle.c:orc_lk_refine bit-for-bit (the
 * reference's Eigen reduction order is not pinned). */
int sgm_lk_refine_device(sgm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int pitch,
                         float *d_disp, int disp_pitch, void *stream);

/* SkyAreaDetector::detect(img, file, sky_label, scale) (sky_detector/
 * imageSkyDetector.cpp:166-208) on the GPU: d_img a DEVICE u8 image at the
 * handle's full size (height x width, pitch bytes); d_mask the DEVICE u8 mask
 * on the working grid (rows x cols, mask_pitch bytes), 255 = sky.  Four
 * launches on `stream` (NULL = the handle's stream), no host round trip.
 * Numerics pinned as oracle/sgm_oracle.c:orc_sky_detect (which reproduces
 * the reference's example/000017_14 mask exactly).  The debug image the
 * reference writes to `file` is not produced. */
int sgm_sky_detect_device(sgm_handle *h, const uint8_t *d_img, int pitch, uint8_t *d_mask,
                          int mask_pitch, void *stream);

/* Solver::colormap (src/Solver.cpp:652-707) of a DEVICE working-grid map
 * (rows x cols f32, pitch in floats) into DEVICE BGR (rows x cols x 3 u8,
 * bgr_pitch bytes): the image show_disp publishes (Solver.cpp:55-93). */
int sgm_colormap_device(sgm_handle *h, const float *d_disp, int pitch, uint8_t *d_bgr,
                        int bgr_pitch, void *stream);

/* The point cloud of node.cpp:119-143 from a DEVICE working-grid map: every
 * pixel with disp != D+1 and Z = (fx+fy)/2 * baseline / (disp + 1e-6) <=
 * max_range becomes (X, Y, Z) (doubles) and the gray value img(i, j) of the
 * DEVICE image d_img (img_pitch bytes; the node reads its full-size image
 * at working-grid indices, node.cpp:137), in row-major order.  d_xyz holds
 * up to rows*cols*3 doubles, d_pixel rows*cols bytes; *d_count (device int)
 * receives the number of points.  Enqueued on `stream`. */
int sgm_point_cloud_device(sgm_handle *h, const float *d_disp, int pitch, const uint8_t *d_img,
                           int img_pitch, const sgm_camera *cam, double *d_xyz,
                           uint8_t *d_pixel, int *d_count, void *stream);

/* ---- multi-GPU: pairs shard one per device, maps gathered to rank 0 ----
 *
 * stereo pairs are independent, so a batch runs one pair per
 * GPU (one sgm_handle per device) and the only collective is the gather of
 * the H x W disparity maps to rank 0: RCCL's ncclGather over xGMI (1.86 MB
 * per rank at K128).  The reference has no multi-GPU path; its per-pair call
 * is node.cpp:49,93 (SGM sgm(h, w, s, d); sgm.process(l, r)), which
 * include/sgm_amd/BatchSGM.h runs on every device of a batch, one host
 * thread per device.  RCCL is bound at run time on the first sgm_comm_*
 * call (an RCCL the process already holds, e.g. PyTorch's, is reused;
 * SGM_RCCL_LIB names another).  Errors before a communicator exists are
 * read with sgm_comm_last_error(NULL), per calling thread (as errno). */
typedef struct sgm_comm sgm_comm;

#define SGM_COMM_ID_BYTES 128  /* = sizeof(ncclUniqueId) */

/* Single process driving n devices, ranks 0..n-1 = devices[0..n-1]
 * (ncclCommInitAll).  Each device appears once. */
int sgm_comm_create(const int *devices, int n, sgm_comm **out);
/* One process per device (the torch.distributed.run layout): rank 0 makes an
 * id, every process receives it out of band and joins as `rank` of `nranks`
 * on `device` (ncclGetUniqueId / ncclCommInitRank; blocks until all joined). */
int sgm_comm_unique_id(char id[SGM_COMM_ID_BYTES]);
int sgm_comm_create_rank(const char id[SGM_COMM_ID_BYTES], int nranks, int rank, int device,
                         sgm_comm **out);
int sgm_comm_destroy(sgm_comm *c);
const char *sgm_comm_last_error(const sgm_comm *c);
/* ranks in the communicator, the first rank this object holds, and how many */
int sgm_comm_info(const sgm_comm *c, int *nranks, int *first_rank, int *nlocal);

/* Rank `rank`'s contribution to the gather (ncclGather, root 0): its DEVICE
 * map d_map (rows x cols f32, row pitch in floats >= cols; pitched maps are
 * packed first) lands at d_root_out + rank * rows * cols on rank 0's device
 * (nranks * rows * cols floats; ignored on other ranks).  Enqueued on
 * `stream`, a hipStream_t of the rank's device (NULL: the legacy default
 * stream), after the map's producer on that stream; returns after
 * enqueueing.  Every rank of the communicator must call it with the same
 * rows and cols: from its own host thread, or through sgm_batch_gather_all
 * when one thread drives all ranks.  Call sgm_check on the producing handle
 * first: a map from a frame sgm_check rejects is not valid.  A pitched map is
 * packed into one staging buffer per rank, so one rank's gathers go on one
 * stream (or are otherwise ordered). */
int sgm_batch_gather(sgm_comm *c, int rank, const float *d_map, int rows, int cols, int pitch,
                     float *d_root_out, void *stream);
/* The same for every rank this object holds, from one thread (one RCCL
 * group): d_maps[k] and streams[k] (NULL array: default streams) belong to
 * rank first_rank + k. */
int sgm_batch_gather_all(sgm_comm *c, const float *const *d_maps, int rows, int cols, int pitch,
                         float *d_root_out, void *const *streams);

/* ---- per-kernel timing (HIP events recorded around every launch) ---- */

typedef struct sgm_kernel_stat {
    char name[32];      /* kernel class, e.g. "sweep_L3_acc" */
    int launches;       /* completed launches since the last read */
    double total_ms;    /* sum of event-measured durations */
    double elems;       /* pixel-disparity elements touched per launch (mean over the launches) */
} sgm_kernel_stat;

/* enable != 0: every subsequent launch is bracketed by two HIP events on the
 * stream it runs on.  Off by default. */
int sgm_set_profiling(sgm_handle *h, int enable);
/* Synchronises the handle's device, folds all pending event pairs into the
 * per-class statistics, copies up to max entries to out, sets *count, and
 * resets the statistics. */
int sgm_get_profile(sgm_handle *h, sgm_kernel_stat *out, int max, int *count);

/* ---- stage entry points (host buffers, synchronous), for parity tests ---- */

/* Decimation + optional pre-blur + CT_pts on ONE image (cost.cpp:99-129).
 * img: height x width (full size, pitch bytes); ct: rows x cols u64. */
int sgm_stage_census(sgm_handle *h, const uint8_t *img, int pitch, uint64_t *ct);
/* build_dsi_from_table[_beta] + filters (Solver.cpp:143-248, 296-368).
 * view 0 = left, 1 = right; filters bit 1 = horizontal, bit 2 = vertical.
 * cost: rows x cols x D f32. */
int sgm_stage_cost(sgm_handle *h, const uint64_t *ctl, const uint64_t *ctr,
                   const uint8_t *sky, int view, int filters, float *cost);
/* One path DP over a cost volume (SGM.cpp:81-369): L (rows x cols x D) and
 * minL (rows x cols). */
int sgm_stage_path(sgm_handle *h, int dir, const float *cost, float *L, float *minL);
/* 8 paths + aggregation + WTA + uniqueness + sub-pixel (SGM.cpp:81-443). */
int sgm_stage_aggregate(sgm_handle *h, const float *cost, uint16_t *disp, float *sub);
/* LR check (SGM.cpp:803-818): out = checked copy of fl. */
int sgm_stage_lr(sgm_handle *h, const float *fl, const float *fr, float *out);
/* post_filter() (Solver.cpp:600-649) on a HOST rows x cols map, in place,
 * computed on the GPU (sgm_post_filter_device); synchronous. */
int sgm_stage_post_filter(sgm_handle *h, float *disp);
/* LKRefine (sgm_lk_refine_device) with HOST buffers: left/right full-size u8
 * images (pitch bytes), disp a rows x cols map refined in place; synchronous. */
int sgm_stage_lk_refine(sgm_handle *h, const uint8_t *left, const uint8_t *right, int pitch,
                        float *disp);
/* Sky detector (sgm_sky_detect_device) with HOST buffers: img full-size
 * (pitch bytes), mask rows x cols; synchronous. */
int sgm_stage_sky_detect(sgm_handle *h, const uint8_t *img, int pitch, uint8_t *mask);
/* colormap with HOST buffers: disp rows x cols, bgr rows x cols x 3. */
int sgm_stage_colormap(sgm_handle *h, const float *disp, uint8_t *bgr);
/* point cloud with HOST buffers: disp rows x cols, img the full-size image
 * (img_pitch bytes); xyz (3*rows*cols doubles) and pixel (rows*cols) receive
 * *count points. */
int sgm_stage_point_cloud(sgm_handle *h, const float *disp, const uint8_t *img, int img_pitch,
                          const sgm_camera *cam, double *xyz, uint8_t *pixel, int *count);

#ifdef __cplusplus
}
#endif
#endif
