/*
 * sgm_amd/LKSubPixel.h -- the reference's LKSubPixel (LKRefine/LKSubPixel.h:
 * 15-30, LKSubPixelImpl.cpp:13-235) over libsgm_hip.so: LKRefine runs on the
 * GPU (sgm_stage_lk_refine).  Header-only, C++11.
 *
 *   LKSubPixel::create(h, w, s, d)          LKSubPixel.cpp:17-20 (asserts :5-12)
 *   LKRefine(img_l, img_r, disp_float)      LKSubPixelImpl.cpp:13-54
 *     img_l, img_r  CV_8UC1, h x w (decimated by s inside, :29-44)
 *     disp_float    CV_32FC1, (h/s) x (w/s), refined in place
 *
 * The reference's LKRefine asserts img and disp have the same size (:21-26),
 * which contradicts its own decimation for s = 2; this wrapper takes the
 * full-size images for any s.
 */
#ifndef SGM_AMD_LK_SUBPIXEL_H
#define SGM_AMD_LK_SUBPIXEL_H

#include <memory>

#include "SGM.h"

namespace sgm_amd {

class LKSubPixel {
public:
    explicit LKSubPixel(int h, int w, int s, int d) : h_(h), w_(w), s_(s), d_(d) {
        if (!(h > 0 && w > 0 && s > 0 && d > 0) || (s != 1 && s != 2) ||
            (d != 32 && d != 64 && d != 128 && d != 256))
            fail("LKSubPixel", "h,w,s,d > 0, s in {1,2}, d in {32,64,128,256} (LKSubPixel.cpp:5-12)");
        sgm_params p;
        sgm_default_params(&p, h, w, s, d);
        p.aux_only = 1;
        const char *e = std::getenv("SGM_AMD_DEVICE");
        if (sgm_create(&p, e ? std::atoi(e) : 0, &handle_) != SGM_OK)
            fail("LKSubPixel", handle_ ? sgm_last_error(handle_) : "sgm_create failed");
    }
    virtual ~LKSubPixel() {
        if (handle_) sgm_destroy(handle_);
    }
    LKSubPixel(const LKSubPixel &) = delete;
    LKSubPixel &operator=(LKSubPixel &) = delete;

    static std::shared_ptr<LKSubPixel> create(int h, int w, int s, int d) {
        return std::make_shared<LKSubPixel>(h, w, s, d);
    }

    virtual void LKRefine(const Mat &img_l, const Mat &img_r, Mat &disp_float) {
        if (img_l.type() != CV_8UC1 || img_r.type() != CV_8UC1 || img_l.rows != h_ ||
            img_l.cols != w_ || img_r.rows != h_ || img_r.cols != w_ || img_l.step != img_r.step)
            fail("LKRefine", "images must be CV_8UC1 of the constructed size");
        if (disp_float.type() != CV_32FC1 || disp_float.rows != h_ / s_ ||
            disp_float.cols != w_ / s_ || disp_float.step != (size_t)disp_float.cols * 4)
            fail("LKRefine", "disp_float must be a continuous CV_32FC1 of the working size");
        if (sgm_stage_lk_refine(handle_, img_l.data, img_r.data, (int)img_l.step,
                                disp_float.template ptr<float>(0)) != SGM_OK)
            fail("LKRefine", sgm_last_error(handle_));
    }

private:
    int h_, w_, s_, d_;
    sgm_handle *handle_ = nullptr;
};

typedef std::shared_ptr<LKSubPixel> LKSubPixelPtr;

}  // namespace sgm_amd

#endif
