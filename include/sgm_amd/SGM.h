/*
 * sgm_amd/SGM.h -- the reference's Solver / SGM class surface over the C-ABI.
 *
 * Same class names, signatures, ownership and error behaviour as the
 * reference (inc/Solver.h:23-70, inc/SGM.h:10-26), so the ROS node
 * (node.cpp:49,93,104,107) compiles against this header unchanged; the work
 * runs in libsgm_hip.so (include/sgm_hip.h) on one MI355X.  Header-only,
 * C++11.
 *
 *   SGM(h, w, s, d)              Solver.cpp:4-16   (asserts: h,w,s,d > 0,
 *                                s in {1,2}, d in {32,64,128} -- widened to 256)
 *   process(l, r)                SGM.cpp:32-826     (LR-checked, post-filtered)
 *   process(l, r, sky, sky_b)    SGM.cpp:829-834    (masks kept as members)
 *   BM(h, w, s, d)               BM.cpp:4-97        (filtered-cost WTA, post-filtered)
 *   get_disp()                   Solver.h:36        (CV_32FC1, invalid = d+1)
 *   show_disp(view)              Solver.cpp:55-93   (2h x w BGR, colormap :652-707)
 *
 * Mat is cv::Mat when OpenCV's core header is included first (or
 * SGM_AMD_USE_OPENCV is defined); otherwise a minimal row-major stand-in with
 * the members the class surface uses.  Errors abort with a message, like the
 * reference's asserts (define SGM_AMD_THROW to get std::runtime_error).
 */
#ifndef SGM_AMD_SGM_H
#define SGM_AMD_SGM_H

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "../sgm_hip.h"

#if defined(SGM_AMD_USE_OPENCV) || defined(OPENCV_CORE_HPP) || defined(__OPENCV_CORE_HPP__)
#include <opencv2/core/core.hpp>
namespace sgm_amd {
using cv::Mat;
typedef cv::Vec3b Vec3b;
}  // namespace sgm_amd
#define SGM_AMD_HAVE_OPENCV 1
#else
#ifndef CV_8UC1
#define CV_8UC1 0
#endif
#ifndef CV_32FC1
#define CV_32FC1 5
#endif
#ifndef CV_8UC3
#define CV_8UC3 16
#endif
namespace sgm_amd {
struct Vec3b {
    unsigned char v[3];
    unsigned char &operator[](int i) { return v[i]; }
    const unsigned char &operator[](int i) const { return v[i]; }
};
// Minimal cv::Mat stand-in: shallow copies share the buffer (as cv::Mat).
class Mat {
public:
    int rows = 0, cols = 0;
    size_t step = 0;  // bytes per row
    unsigned char *data = nullptr;

    Mat() = default;
    Mat(int r, int c, int t) { create(r, c, t); }
    void create(int r, int c, int t) {
        if (r == rows && c == cols && t == type_ && data) return;
        rows = r;
        cols = c;
        type_ = t;
        step = (size_t)c * elem_size(t);
        buf_.reset(new unsigned char[(size_t)r * step](), std::default_delete<unsigned char[]>());
        data = buf_.get();
    }
    void release() {
        buf_.reset();
        data = nullptr;
        rows = cols = 0;
        step = 0;
    }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    int type() const { return type_; }
    int channels() const { return type_ == CV_8UC3 ? 3 : 1; }
    Mat clone() const {  // packed copy (step = cols * elem), row by row as cv::Mat::clone
        Mat m(rows, cols, type_);
        for (int i = 0; i < rows && !empty(); ++i)
            std::memcpy(m.data + (size_t)i * m.step, data + (size_t)i * step, m.step);
        return m;
    }
    template <typename T> T *ptr(int i) { return reinterpret_cast<T *>(data + (size_t)i * step); }
    template <typename T> const T *ptr(int i) const {
        return reinterpret_cast<const T *>(data + (size_t)i * step);
    }
    template <typename T> T &at(int i, int j) { return ptr<T>(i)[j]; }
    template <typename T> const T &at(int i, int j) const { return ptr<T>(i)[j]; }

private:
    static size_t elem_size(int t) { return t == CV_32FC1 ? 4 : (t == CV_8UC3 ? 3 : 1); }
    int type_ = -1;
    std::shared_ptr<unsigned char> buf_;
};
}  // namespace sgm_amd
#endif

namespace sgm_amd {

inline void fail(const char *what, const char *detail) {
#ifdef SGM_AMD_THROW
    throw std::runtime_error(std::string(what) + ": " + (detail ? detail : ""));
#else
    std::fprintf(stderr, "sgm_amd: %s: %s\n", what, detail ? detail : "");
    std::abort();
#endif
}

// Solver (inc/Solver.h:23-70): geometry, result maps and the device handle.
class Solver {
public:
    explicit Solver(int h, int w, int s, int d) {
        if (!(h > 0 && w > 0 && s > 0 && d > 0) || !(s == 1 || s == 2) ||
            !(d == 32 || d == 64 || d == 128 || d == 256))
            fail("Solver", "h,w,s,d > 0, s in {1,2}, d in {32,64,128,256} (Solver.cpp:6-10)");
        img_h = h / s;
        img_w = w / s;
        scale = s;
        max_disp = d;
        invalid_disp = d + 1;
        in_h_ = h;
        in_w_ = w;
        filtered_disp.create(img_h, img_w, CV_32FC1);
        colored_disp.create(img_h, img_w, CV_8UC3);
    }
    virtual ~Solver() = default;

    Solver(const Solver &) = delete;
    Solver &operator=(Solver &) = delete;

    virtual void process(Mat &img_l, Mat &img_r) = 0;
    virtual void process(Mat &img_l, Mat &img_r, Mat &sky_mask, Mat &sky_mask_beta) = 0;

    // Solver.cpp:55-93: left image (BGR) above the colour-mapped disparity;
    // the lower tile starts at row img_h - 1 as in the reference.
    virtual void show_disp(Mat &debug_view) {
        colormap();
        debug_view.create(img_h * 2, img_w, CV_8UC3);
        std::memset(debug_view.data, 0, (size_t)debug_view.rows * debug_view.step);
        for (int i = 0; i < img_h && !img_l.empty(); ++i) {
            const unsigned char *src = img_l.template ptr<unsigned char>(i);
            Vec3b *dst = debug_view.template ptr<Vec3b>(i);
            for (int j = 0; j < img_w; ++j) dst[j][0] = dst[j][1] = dst[j][2] = src[j];
        }
        for (int i = 0; i < img_h; ++i)
            std::memcpy(debug_view.template ptr<Vec3b>(img_h - 1 + i),
                        colored_disp.template ptr<Vec3b>(i), (size_t)img_w * 3);
    }
    virtual const Mat &get_disp() const { return filtered_disp; }

protected:
    int img_h, img_w;
    int scale;
    int max_disp, invalid_disp;
    int in_h_, in_w_;

    Mat img_l, img_r;
    Mat filtered_disp;
    Mat colored_disp;
    Mat sky_mask, sky_mask_beta;

    // Solver.cpp:652-707
    void colormap() {
        for (int i = 0; i < img_h; ++i)
            for (int j = 0; j < img_w; ++j) {
                float v = filtered_disp.template at<float>(i, j);
                Vec3b &c = colored_disp.template at<Vec3b>(i, j);
                if (v > max_disp - 1) {
                    c[0] = c[1] = c[2] = 0;
                    continue;
                }
                v *= (256 / (max_disp));
                if (v <= 51) {
                    c[0] = 255; c[1] = (unsigned char)(v * 5); c[2] = 0;
                } else if (v <= 102) {
                    v -= 51;
                    c[0] = (unsigned char)(255 - v * 5); c[1] = 255; c[2] = 0;
                } else if (v <= 153) {
                    v -= 102;
                    c[0] = 0; c[1] = 255; c[2] = (unsigned char)(v * 5);
                } else if (v <= 204) {
                    v -= 153;
                    c[0] = 0; c[1] = (unsigned char)(255 - (unsigned char)(128.0 * v / 51.0 + 0.5)); c[2] = 255;
                } else {
                    v -= 204;
                    c[0] = 0; c[1] = (unsigned char)(127 - (unsigned char)(127.0 * v / 51.0 + 0.5)); c[2] = 255;
                }
            }
    }
};

typedef std::shared_ptr<Solver> SolverPtr;

// Common body of the two solvers: one libsgm_hip.so handle per object, the
// whole frame (and post_filter) on the GPU.
class HipSolver : public Solver {
public:
    virtual ~HipSolver() {
        if (handle_) sgm_destroy(handle_);
    }
    HipSolver(const HipSolver &) = delete;
    HipSolver &operator=(const HipSolver &) = delete;

    // SGM.cpp:829-834 / BM.cpp:91-96
    virtual void process(Mat &img_l, Mat &img_r, Mat &sky_mask, Mat &sky_mask_beta) {
        this->sky_mask = sky_mask;
        this->sky_mask_beta = sky_mask_beta;
        process(img_l, img_r);
    }
    virtual void process(Mat &img_l, Mat &img_r) {
        if (img_l.rows != img_r.rows || img_l.cols != img_r.cols || img_l.type() != img_r.type() ||
            img_l.type() != CV_8UC1 || img_l.rows != in_h_ || img_l.cols != in_w_)
            fail("process", "inputs must be CV_8UC1 of the constructed size (SGM.cpp:34-38)");
        this->img_l = img_l;  // shallow, as SGM.cpp:59-60 (decimated on the device)
        this->img_r = img_r;
        // Each mask applies on its own, as in the reference: sky_mask to the
        // left DSI (Solver.cpp:146-178), sky_mask_beta to the right one
        // (Solver.cpp:200-232); BM reads sky_mask only (BM.cpp:33-34).
        const bool sky_l = !sky_mask.empty();
        const bool sky_r = !bm_ && !sky_mask_beta.empty();
        if (sky_l) check_mask(sky_mask, "sky_mask");
        if (sky_r) check_mask(sky_mask_beta, "sky_mask_beta");
        // The C-ABI takes one pitch for both masks: copy to a common (packed)
        // pitch when the two masks' steps differ.
        Mat ml = sky_mask, mr = sky_mask_beta;
        if (sky_l && sky_r && ml.step != mr.step) {
            ml = sky_mask.clone();
            mr = sky_mask_beta.clone();
        }
        const int sky_pitch = sky_l ? (int)ml.step : sky_r ? (int)mr.step : 0;
        const int rc = sgm_process(handle_, img_l.data, img_r.data, (int)img_l.step,
                                   sky_l ? ml.data : nullptr, sky_r ? mr.data : nullptr, sky_pitch,
                                   filtered_disp.template ptr<float>(0),
                                   (int)(filtered_disp.step / sizeof(float)), nullptr);
        if (rc != SGM_OK) fail("process", sgm_last_error(handle_));
        if (scale > 1) decimate_left();
    }

    sgm_handle *handle() const { return handle_; }

protected:
    // views = 1: the left view alone (BM; GPU_SGM, gpu_sgm/src/SGM.cu:105-232)
    HipSolver(int h, int w, int s, int d, int solver, int views = 2)
        : Solver(h, w, s, d), bm_(solver == SGM_SOLVER_BM) {
        sgm_params p;
        if (sgm_default_params(&p, h, w, s, d) != SGM_OK) fail("Solver", "sgm_default_params");
        p.solver = solver;
        p.post_filter = 1;  // process() ends with post_filter(): SGM.cpp:821, BM.cpp:88 (on the GPU)
        p.views = bm_ ? 1 : views;
        const int rc = sgm_create(&p, device(), &handle_);
        if (rc != SGM_OK) fail("sgm_create", handle_ ? sgm_last_error(handle_) : "no device");
    }

private:
    sgm_handle *handle_ = nullptr;
    bool bm_;

    void check_mask(const Mat &m, const char *what) const {
        if (m.type() != CV_8UC1 || m.rows != img_h || m.cols != img_w)
            fail(what, "sky masks must be CV_8UC1 on the working grid (Solver.cpp:146,200)");
    }

    static int device() {
        const char *e = std::getenv("SGM_AMD_DEVICE");
        return e ? std::atoi(e) : 0;
    }
    // keep img_l on the working grid for show_disp: SGM.cpp:40-56 takes rows
    // i*scale, BM.cpp:20-31 rows i (both every scale-th column)
    void decimate_left() {
        Mat small(img_h, img_w, CV_8UC1);
        for (int i = 0; i < img_h; ++i) {
            const unsigned char *src = img_l.template ptr<unsigned char>(bm_ ? i : i * scale);
            unsigned char *dst = small.template ptr<unsigned char>(i);
            for (int j = 0; j < img_w; ++j) dst[j] = src[j * scale];
        }
        img_l = small;
    }
};

// SGM (inc/SGM.h:10-26): 8-path semi-global matching, both views, LR check,
// post_filter (SGM.cpp:32-826).
class SGM : public HipSolver {
public:
    explicit SGM(int h, int w, int s, int d) : HipSolver(h, w, s, d, SGM_SOLVER_SGM) {}
    SGM(const SGM &) = delete;
    SGM &operator=(const SGM &) = delete;
};

// BM (inc/BM.h:6-19): census cost, the two cost filters and a WTA on the
// filtered cost (BM.cpp:9-97).  get_disp() is the post-filtered integer
// disparity (the reference's BM::process never writes filtered_disp).
class BM : public HipSolver {
public:
    explicit BM(int h, int w, int s, int d) : HipSolver(h, w, s, d, SGM_SOLVER_BM) {}
    BM(const BM &) = delete;
    BM &operator=(const BM &) = delete;
};

typedef std::shared_ptr<BM> BMSolverPtr;
typedef std::shared_ptr<SGM> SGMSolverPtr;

}  // namespace sgm_amd

#endif
