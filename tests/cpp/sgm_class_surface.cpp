// Drives the reference's class surface (include/sgm_amd/SGM.h) the way the
// ROS node does (node.cpp:49,93,104,107): construct SGM(h, w, s, d), process
// a pair, read get_disp().
//   sgm_class_surface nodevice            -> argument asserts + no-device error
//   sgm_class_surface run L R H W D OUT   -> raw u8 pair in, f32 disparity out
//   sgm_class_surface runbm L R H W D OUT -> the same through BM(h, w, s, d)
//   sgm_class_surface rungpu L R H W S D OUT OUT2 -> GPU_SGM(h, w, s, d) as node.cpp:50
//                                         would build it: get_disp() to OUT, and to
//                                         OUT2 again after show_disp()
//   sgm_class_surface sky IMG H W S OUT   -> SkyAreaDetector::detect mask
//   sgm_class_surface lk L R DISP H W D OUT -> LKSubPixel::LKRefine of DISP
//   sgm_class_surface batch PREFIX N H W D OUT -> BatchSGM over the devices of
//                                         SGM_AMD_DEVICES (default "0"): pairs
//                                         PREFIX_l<k>.raw / PREFIX_r<k>.raw, k < N,
//                                         their get_disp() maps to OUT in pair order
#define SGM_AMD_THROW 1
#include "sgm_amd/BatchSGM.h"
#include "sgm_amd/SGM.h"
#include "sgm_amd/GPU_SGM.h"
#include "sgm_amd/LKSubPixel.h"
#include "sgm_amd/SkyAreaDetector.h"

#include <cstdio>
#include <fstream>
#include <vector>

using sgm_amd::Mat;

static int expect_throw(int h, int w, int s, int d) {
    try {
        sgm_amd::SGM sgm(h, w, s, d);
    } catch (const std::runtime_error &e) {
        std::printf("threw as expected (%d,%d,%d,%d): %s\n", h, w, s, d, e.what());
        return 0;
    }
    std::printf("did not throw (%d,%d,%d,%d)\n", h, w, s, d);
    return 1;
}

int main(int argc, char **argv) {
    if (argc >= 2 && std::string(argv[1]) == "nodevice") {
        int bad = 0;
        bad += expect_throw(375, 1242, 3, 128);  // s not in {1,2}   (Solver.cpp:8)
        bad += expect_throw(375, 1242, 1, 48);   // d not allowed    (Solver.cpp:10)
        bad += expect_throw(0, 1242, 1, 64);     // h > 0            (Solver.cpp:6)
        bad += expect_throw(375, 1242, 1, 64);   // valid, but no GPU in this container
        try {  // the multi-GPU batch: no device here either
            sgm_amd::BatchSGM batch(std::vector<int>{0}, 375, 1242, 1, 64);
            std::printf("BatchSGM did not throw\n");
            ++bad;
        } catch (const std::runtime_error &e) {
            std::printf("BatchSGM threw: %s\n", e.what());
        }
        // BatchSGM's round bookkeeping and argument checks (no device work):
        // 2N+1 pairs on N devices are rounds of N, N and 1
        using B = sgm_amd::BatchSGM;
        bad += B::round_count(9, 0, 4) != 4 || B::round_count(9, 4, 4) != 4 || B::round_count(9, 8, 4) != 1;
        bad += B::round_count(3, 0, 1) != 1 || B::round_count(3, 2, 1) != 1 || B::round_count(8, 0, 8) != 8;
        {
            std::vector<Mat> l2(2, Mat(6, 8, CV_8UC1)), r1(1, Mat(6, 8, CV_8UC1)), r2(2, Mat(6, 8, CV_8UC1));
            std::vector<Mat> wrong(2, Mat(6, 9, CV_8UC1)), f32(2, Mat(6, 8, CV_32FC1));
            const struct {
                const std::vector<Mat> &l, &r;
                const char *why;
            } cases[] = {{l2, r1, "counts differ"}, {l2, wrong, "constructed size"}, {f32, r2, "CV_8UC1"}};
            for (const auto &c : cases) {
                try {
                    B::check_batch(c.l, c.r, 6, 8);
                    std::printf("check_batch accepted a bad batch (%s)\n", c.why);
                    ++bad;
                } catch (const std::runtime_error &e) {
                    std::printf("check_batch threw: %s\n", e.what());
                }
            }
            B::check_batch(l2, r2, 6, 8);  // a valid batch passes
        }
        Mat m(4, 5, CV_32FC1);
        m.at<float>(3, 4) = 2.5f;
        Mat shallow = m;
        bad += shallow.at<float>(3, 4) != 2.5f;
        bad += m.clone().data == m.data;
        return bad;
    }
    if (argc == 8 && (std::string(argv[1]) == "run" || std::string(argv[1]) == "runbm")) {
        const int h = std::atoi(argv[4]), w = std::atoi(argv[5]), d = std::atoi(argv[6]);
        Mat l(h, w, CV_8UC1), r(h, w, CV_8UC1);
        std::ifstream fl(argv[2], std::ios::binary), fr(argv[3], std::ios::binary);
        fl.read(reinterpret_cast<char *>(l.data), (std::streamsize)h * w);
        fr.read(reinterpret_cast<char *>(r.data), (std::streamsize)h * w);
        if (!fl || !fr) return 2;
        sgm_amd::SolverPtr sgm;
        if (std::string(argv[1]) == "runbm")
            sgm = std::make_shared<sgm_amd::BM>(h, w, 1, d);
        else
            sgm = std::make_shared<sgm_amd::SGM>(h, w, 1, d);
        sgm->process(l, r);
        const Mat &disp = sgm->get_disp();
        Mat view;
        sgm->show_disp(view);
        if (view.rows != 2 * h || view.cols != w) return 3;
        std::ofstream fo(argv[7], std::ios::binary);
        for (int i = 0; i < disp.rows; ++i)
            fo.write(reinterpret_cast<const char *>(disp.ptr<float>(i)), (std::streamsize)w * 4);
        return fo ? 0 : 4;
    }
    if (argc == 8 && std::string(argv[1]) == "batch") {
        const std::string prefix = argv[2];
        const int n = std::atoi(argv[3]), h = std::atoi(argv[4]), w = std::atoi(argv[5]),
                  d = std::atoi(argv[6]);
        std::vector<int> devices;
        const char *env = std::getenv("SGM_AMD_DEVICES");
        for (const char *c = env && *env ? env : "0"; *c;) {
            devices.push_back(std::atoi(c));
            while (*c && *c != ',') ++c;
            if (*c == ',') ++c;
        }
        std::vector<Mat> ls, rs;
        for (int k = 0; k < n; ++k) {
            Mat l(h, w, CV_8UC1), r(h, w, CV_8UC1);
            std::ifstream fl(prefix + "_l" + std::to_string(k) + ".raw", std::ios::binary),
                fr(prefix + "_r" + std::to_string(k) + ".raw", std::ios::binary);
            fl.read(reinterpret_cast<char *>(l.data), (std::streamsize)h * w);
            fr.read(reinterpret_cast<char *>(r.data), (std::streamsize)h * w);
            if (!fl || !fr) return 2;
            ls.push_back(l);
            rs.push_back(r);
        }
        sgm_amd::BatchSGM batch(devices, h, w, 1, d);  // SGM(h, w, s, d) per device, node.cpp:49
        batch.process(ls, rs);                         // node.cpp:93 for every pair
        std::ofstream fo(argv[7], std::ios::binary);
        for (int k = 0; k < n; ++k) {
            const Mat &disp = batch.get_disp(k);       // node.cpp:104
            if (disp.rows != h || disp.cols != w) return 3;
            for (int i = 0; i < disp.rows; ++i)
                fo.write(reinterpret_cast<const char *>(disp.ptr<float>(i)), (std::streamsize)w * 4);
        }
        std::printf("batch of %d pairs on %zu device(s)\n", n, devices.size());
        return fo ? 0 : 4;
    }
    if (argc == 10 && std::string(argv[1]) == "rungpu") {
        const int h = std::atoi(argv[4]), w = std::atoi(argv[5]), s = std::atoi(argv[6]),
                  d = std::atoi(argv[7]);
        Mat l(h, w, CV_8UC1), r(h, w, CV_8UC1);
        std::ifstream fl(argv[2], std::ios::binary), fr(argv[3], std::ios::binary);
        fl.read(reinterpret_cast<char *>(l.data), (std::streamsize)h * w);
        fr.read(reinterpret_cast<char *>(r.data), (std::streamsize)h * w);
        if (!fl || !fr) return 2;
        using namespace sgm_amd;
        GSGMPtr gsv = std::make_shared<GPU_SGM>(h, w, s, d);  // node.cpp:50
        for (int frame = 0; frame < 2; ++frame) gsv->process(l, r);  // the handle is reused
        const Mat &disp = gsv->get_disp();
        std::ofstream fo(argv[8], std::ios::binary);
        for (int i = 0; i < disp.rows; ++i)
            fo.write(reinterpret_cast<const char *>(disp.ptr<float>(i)), (std::streamsize)disp.cols * 4);
        Mat view;
        gsv->show_disp(view);
        if (view.rows != 2 * (h / s) || view.cols != w / s) return 3;
        std::ofstream fo2(argv[9], std::ios::binary);
        for (int i = 0; i < disp.rows; ++i)
            fo2.write(reinterpret_cast<const char *>(disp.ptr<float>(i)), (std::streamsize)disp.cols * 4);
        return fo && fo2 ? 0 : 4;
    }
    if (argc == 10 && std::string(argv[1]) == "runsky") {
        // process(l, r, sky, sky_beta) with either mask possibly "-" (empty);
        // the beta mask is held with a wider row pitch than the left one
        const int h = std::atoi(argv[6]), w = std::atoi(argv[7]), d = std::atoi(argv[8]);
        Mat l(h, w, CV_8UC1), r(h, w, CV_8UC1), sl, sr;
        std::ifstream fl(argv[2], std::ios::binary), fr(argv[3], std::ios::binary);
        fl.read(reinterpret_cast<char *>(l.data), (std::streamsize)h * w);
        fr.read(reinterpret_cast<char *>(r.data), (std::streamsize)h * w);
        if (!fl || !fr) return 2;
        if (std::string(argv[4]) != "-") {
            sl.create(h, w, CV_8UC1);
            std::ifstream f(argv[4], std::ios::binary);
            f.read(reinterpret_cast<char *>(sl.data), (std::streamsize)h * w);
            if (!f) return 2;
        }
        if (std::string(argv[5]) != "-") {
            sr.create(h, w + 24, CV_8UC1);
            sr.cols = w;  // a pitched view: step = w + 24 bytes
            std::ifstream f(argv[5], std::ios::binary);
            for (int i = 0; i < h; ++i) f.read(reinterpret_cast<char *>(sr.ptr<unsigned char>(i)), w);
            if (!f) return 2;
        }
        sgm_amd::SGM sgm(h, w, 1, d);
        sgm.process(l, r, sl, sr);
        const Mat &disp = sgm.get_disp();
        std::ofstream fo(argv[9], std::ios::binary);
        for (int i = 0; i < disp.rows; ++i)
            fo.write(reinterpret_cast<const char *>(disp.ptr<float>(i)), (std::streamsize)w * 4);
        return fo ? 0 : 4;
    }
    if (argc == 7 && std::string(argv[1]) == "sky") {
        const int h = std::atoi(argv[3]), w = std::atoi(argv[4]), s = std::atoi(argv[5]);
        Mat img(h, w, CV_8UC1), mask;
        std::ifstream fi(argv[2], std::ios::binary);
        fi.read(reinterpret_cast<char *>(img.data), (std::streamsize)h * w);
        if (!fi) return 2;
        sky_detector::SkyAreaDetector det;
        det.detect(img, "unused.png", mask, s);
        det.detect(img, "unused.png", mask, s);  // the handle is reused
        if (mask.rows != h / s || mask.cols != w / s || mask.type() != CV_8UC1) return 3;
        std::ofstream fo(argv[6], std::ios::binary);
        fo.write(reinterpret_cast<const char *>(mask.data), (std::streamsize)mask.rows * mask.cols);
        return fo ? 0 : 4;
    }
    if (argc == 9 && std::string(argv[1]) == "lk") {
        const int h = std::atoi(argv[5]), w = std::atoi(argv[6]), d = std::atoi(argv[7]);
        Mat l(h, w, CV_8UC1), r(h, w, CV_8UC1), disp(h, w, CV_32FC1);
        std::ifstream fl(argv[2], std::ios::binary), fr(argv[3], std::ios::binary),
            fd(argv[4], std::ios::binary);
        fl.read(reinterpret_cast<char *>(l.data), (std::streamsize)h * w);
        fr.read(reinterpret_cast<char *>(r.data), (std::streamsize)h * w);
        fd.read(reinterpret_cast<char *>(disp.data), (std::streamsize)h * w * 4);
        if (!fl || !fr || !fd) return 2;
        sgm_amd::LKSubPixelPtr lk = sgm_amd::LKSubPixel::create(h, w, 1, d);
        lk->LKRefine(l, r, disp);
        std::ofstream fo(argv[8], std::ios::binary);
        fo.write(reinterpret_cast<const char *>(disp.data), (std::streamsize)h * w * 4);
        return fo ? 0 : 4;
    }
    std::fprintf(stderr, "usage: %s nodevice | run|runbm L R H W D OUT | sky IMG H W S OUT | "
                 "lk L R DISP H W D OUT\n", argv[0]);
    return 2;
}
