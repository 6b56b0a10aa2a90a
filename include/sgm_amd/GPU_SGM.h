/*
 * sgm_amd/GPU_SGM.h -- the reference's CUDA backend class GPU_SGM
 * (gpu_sgm/inc/SGM.cuh:23-62, gpu_sgm/src/SGM.cu) over the C-ABI of
 * libsgm_hip.so, which replaces gpu_sgm/.  The ROS node carries its call site
 * commented out (node.cpp:10,50):
 *
 *   // #include "gpu_sgm/inc/SGM.cuh"
 *   // GSGMPtr gsv = std::make_shared<GPU_SGM>(g_img_h, g_img_w, g_scale, g_max_disp);
 *
 * With this header included instead (and `using namespace sgm_amd;`) both
 * lines compile unchanged.  Header-only, C++11.
 *
 *   GPU_SGM(h, w, s, d)   SGM.cu:4-57    working grid h/s x w/s, invalid = d+1
 *   process(l, r)         SGM.cu:105-232 the LEFT view only: census, Hamming
 *                         cost, the two cost filters, 8 paths, WTA +
 *                         uniqueness, sub-pixel (:207-217), then the median
 *                         fill and speckle removal (:218-225); no right view,
 *                         no LR check
 *   get_disp()            SGM.cuh:32     filtered_disp, CV_32FC1
 *   show_disp(view)       SGM.cu:236-262 sets filtered_disp[:, 0 .. d/s) to
 *                         invalid IN PLACE (as the reference does), then the
 *                         colormap (:265-330) under the left image
 *
 * Results follow the reference's CPU path that GPU_SGM was written to
 * accelerate (src/SGM.cpp:32-443 + Solver.cpp:569-649), bit for bit -- not
 * the CUDA tree's approximations (no pre-blur, diagonals truncated at the
 * left/right edges and stored as short, a parallel float median; SURVEY.md
 * 2.1).  process() returns with the map on the host (the CUDA version left
 * its device-to-host copy in flight, SGM.cu:230).
 */
#ifndef SGM_AMD_GPU_SGM_H
#define SGM_AMD_GPU_SGM_H

#include "SGM.h"

namespace sgm_amd {

// Not a Solver in the reference (gpu_sgm/inc/SGM.cuh:23): the class surface
// is its own; the left-view handle and the colormap are shared privately.
class GPU_SGM : private HipSolver {
public:
    explicit GPU_SGM(int h, int w, int s, int d) : HipSolver(h, w, s, d, SGM_SOLVER_SGM, 1) {}
    virtual ~GPU_SGM() = default;

    GPU_SGM(const GPU_SGM &) = delete;
    GPU_SGM &operator=(const GPU_SGM &) = delete;

    virtual void process(Mat &img_l, Mat &img_r) { HipSolver::process(img_l, img_r); }

    virtual void show_disp(Mat &debug_view) {
        // left border invalid (SGM.cu:238-246): columns without a full
        // disparity range
        const int cols = max_disp / scale < img_w ? max_disp / scale : img_w;
        for (int i = 0; i < filtered_disp.rows; ++i) {
            float *row = filtered_disp.template ptr<float>(i);
            for (int j = 0; j < cols; ++j) row[j] = (float)invalid_disp;
        }
        Solver::show_disp(debug_view);
    }
    virtual const Mat &get_disp() const { return filtered_disp; }

    using HipSolver::handle;
};

typedef std::shared_ptr<GPU_SGM> GSGMPtr;

}  // namespace sgm_amd

#endif
