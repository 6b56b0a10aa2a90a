/*
 * sgm_amd/SkyAreaDetector.h -- the reference's sky_detector::SkyAreaDetector
 * (sky_detector/imageSkyDetector.h:17-73) over libsgm_hip.so: detect() runs
 * on the GPU (sgm_sky_detect_device), so node.cpp:51,83,86 compile and run
 * unchanged.  Header-only, C++11; include after sgm_amd/SGM.h's Mat choice
 * (cv::Mat when OpenCV's core header comes first).
 *
 *   detect(img, file_name, sky_label, scale)   imageSkyDetector.cpp:166-208
 *     img        CV_8UC1 (the node passes its gray frames), h x w
 *     sky_label  out: CV_8UC1, (h/scale) x (w/scale), 255 = sky
 *     file_name  the reference writes a debug overlay there with OpenCV's
 *                imwrite; this wrapper does not write files
 *
 * One light libsgm_hip handle (params.aux_only) per detector, created on the
 * first call and re-created when the frame geometry changes.
 */
#ifndef SGM_AMD_SKY_AREA_DETECTOR_H
#define SGM_AMD_SKY_AREA_DETECTOR_H

#include <string>

#include "SGM.h"

namespace sky_detector {

class SkyAreaDetector {
public:
    SkyAreaDetector() = default;
    ~SkyAreaDetector() { reset(); }
    SkyAreaDetector(const SkyAreaDetector &) {}  // thresholds are constants here
    SkyAreaDetector &operator=(const SkyAreaDetector &) { return *this; }

    void detect(const sgm_amd::Mat &img, const std::string file_name, sgm_amd::Mat &sky_label,
                int scale) {
        (void)file_name;
        if (img.empty() || img.type() != CV_8UC1 || (scale != 1 && scale != 2))
            sgm_amd::fail("SkyAreaDetector::detect", "img must be CV_8UC1, scale 1 or 2");
        ensure(img.rows, img.cols, scale);
        sky_label.create(img.rows / scale, img.cols / scale, CV_8UC1);
        if (sky_label.step != (size_t)sky_label.cols)
            sgm_amd::fail("SkyAreaDetector::detect", "sky_label must be continuous");
        if (sgm_stage_sky_detect(h_, img.data, (int)img.step, sky_label.data) != SGM_OK)
            sgm_amd::fail("SkyAreaDetector::detect", sgm_last_error(h_));
    }

private:
    sgm_handle *h_ = nullptr;
    int rows_ = 0, cols_ = 0, scale_ = 0;

    void reset() {
        if (h_) sgm_destroy(h_);
        h_ = nullptr;
    }
    void ensure(int rows, int cols, int scale) {
        if (h_ && rows == rows_ && cols == cols_ && scale == scale_) return;
        reset();
        sgm_params p;
        sgm_default_params(&p, rows, cols, scale, 32);
        p.aux_only = 1;
        const char *e = std::getenv("SGM_AMD_DEVICE");
        if (sgm_create(&p, e ? std::atoi(e) : 0, &h_) != SGM_OK)
            sgm_amd::fail("SkyAreaDetector", h_ ? sgm_last_error(h_) : "sgm_create failed");
        rows_ = rows;
        cols_ = cols;
        scale_ = scale;
    }
};

}  // namespace sky_detector

#endif
