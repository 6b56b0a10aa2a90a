// stereo_node.cpp -- the reference ROS node's per-frame flow (node.cpp:25-151)
// on libsgm_hip.so through the drop-in headers, without ROS or OpenCV:
//
//   images (8-bit PGM)            node.cpp:69-70   imread(..., IMREAD_GRAYSCALE)
//   sky masks, both views         node.cpp:80-87   SkyAreaDetector::detect
//   SGM(h, w, s, d).process       node.cpp:49,93   (both views, LR check, post_filter)
//   get_disp()                    node.cpp:104     -> OUT_disp.f32 (raw float32 rows)
//   show_disp(debug_view)         node.cpp:107-110 -> OUT_debug.ppm (the node's imwrite)
//   point cloud                   node.cpp:113-143 -> OUT_cloud.bin (N x 3 float64 + N u8)
//
// The node's resize to the configured size (node.cpp:75-76) is left out: the
// configured size is the images' size.  The calibration (read_calib,
// utils.cpp:59-89) comes from the command line.  Every stage runs on the GPU.
//
// usage: stereo_node LEFT.pgm RIGHT.pgm OUT_PREFIX [scale] [max_disp] [fx fy cx cy]
#include "sgm_amd/SGM.h"
#include "sgm_amd/SkyAreaDetector.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

using sgm_amd::Mat;
typedef std::shared_ptr<sky_detector::SkyAreaDetector> SkyDetPtr;  // node.cpp:8

// binary PGM (P5, maxval 255) -> CV_8UC1
static bool read_pgm(const std::string &path, Mat &img) {
    std::ifstream f(path, std::ios::binary);
    std::string magic;
    int w = 0, h = 0, maxval = 0;
    if (!(f >> magic >> w >> h >> maxval) || magic != "P5" || maxval != 255 || w <= 0 || h <= 0)
        return false;
    f.get();  // the single whitespace after maxval
    img.create(h, w, CV_8UC1);
    for (int i = 0; i < h; ++i) f.read(reinterpret_cast<char *>(img.ptr<unsigned char>(i)), w);
    return (bool)f;
}

static bool write_ppm(const std::string &path, const Mat &bgr) {
    std::ofstream f(path, std::ios::binary);
    f << "P6\n" << bgr.cols << " " << bgr.rows << "\n255\n";
    std::vector<unsigned char> row((size_t)bgr.cols * 3);
    for (int i = 0; i < bgr.rows; ++i) {
        const unsigned char *p = bgr.ptr<unsigned char>(i);
        for (int j = 0; j < bgr.cols; ++j) {  // BGR -> RGB
            row[3 * j] = p[3 * j + 2];
            row[3 * j + 1] = p[3 * j + 1];
            row[3 * j + 2] = p[3 * j];
        }
        f.write(reinterpret_cast<const char *>(row.data()), (std::streamsize)row.size());
    }
    return (bool)f;
}

int main(int argc, char **argv) {
    if (argc != 4 && argc != 6 && argc != 10) {
        std::fprintf(stderr, "usage: %s LEFT.pgm RIGHT.pgm OUT_PREFIX [scale max_disp [fx fy cx cy]]\n",
                     argv[0]);
        return 2;
    }
    const std::string out = argv[3];
    const int scale = argc > 4 ? std::atoi(argv[4]) : 1;        // node.cpp:21 g_scale
    const int max_disp = argc > 5 ? std::atoi(argv[5]) : 128;   // node.cpp:22 g_max_disp
    sgm_camera cam;                                             // KITTI image_0 defaults
    cam.fx = argc > 6 ? (float)std::atof(argv[6]) : 721.5377f;
    cam.fy = argc > 7 ? (float)std::atof(argv[7]) : 721.5377f;
    cam.cx = argc > 8 ? (float)std::atof(argv[8]) : 609.5593f;
    cam.cy = argc > 9 ? (float)std::atof(argv[9]) : 172.854f;
    cam.baseline = 0.5;    // node.cpp:123
    cam.max_range = 100;   // node.cpp:122

    Mat img_l, img_r;
    if (!read_pgm(argv[1], img_l) || !read_pgm(argv[2], img_r) || img_l.rows != img_r.rows ||
        img_l.cols != img_r.cols) {
        std::fprintf(stderr, "cannot read two 8-bit PGM images of one size\n");
        return 2;
    }
    const int h = img_l.rows, w = img_l.cols;
    std::printf("left size: %d, %d\nright size: %d, %d\n", h, w, img_r.rows, img_r.cols);

    // node.cpp:49-51
    sgm_amd::SolverPtr sv = std::make_shared<sgm_amd::SGM>(h, w, scale, max_disp);
    SkyDetPtr sky_det = std::make_shared<sky_detector::SkyAreaDetector>();

    Mat sky_mask, sky_mask_beta;  // node.cpp:80-87 (no debug image is written)
    sky_det->detect(img_l, out + "_sky.png", sky_mask, scale);
    sky_det->detect(img_r, out + "_sky2.png", sky_mask_beta, scale);

    const auto be = std::chrono::steady_clock::now();
    sv->process(img_l, img_r, sky_mask, sky_mask_beta);  // node.cpp:93
    const auto en = std::chrono::steady_clock::now();
    std::printf("stereo matching done\ntime cost: %lf ms\n",
                std::chrono::duration<double, std::milli>(en - be).count());

    const Mat &disp = sv->get_disp();  // node.cpp:104
    {
        std::ofstream f(out + "_disp.f32", std::ios::binary);
        for (int i = 0; i < disp.rows; ++i)
            f.write(reinterpret_cast<const char *>(disp.ptr<float>(i)), (std::streamsize)disp.cols * 4);
    }
    Mat debug_view;  // node.cpp:107-110
    sv->show_disp(debug_view);
    if (!write_ppm(out + "_debug.ppm", debug_view)) return 3;

    // node.cpp:113-143: the cloud in row-major push_back order, on the GPU
    // (sgm_stage_point_cloud) through the solver's handle
    const size_t npx = (size_t)disp.rows * disp.cols;
    std::vector<double> xyz(3 * npx);
    std::vector<unsigned char> pix(npx);
    int n = 0;
    Mat packed = disp.clone();
    const int rc = sgm_stage_point_cloud(static_cast<sgm_amd::SGM *>(sv.get())->handle(),
                                         packed.ptr<float>(0), img_l.data, (int)img_l.step, &cam,
                                         xyz.data(), pix.data(), &n);
    if (rc != SGM_OK) {
        std::fprintf(stderr, "point cloud: %s\n",
                     sgm_last_error(static_cast<sgm_amd::SGM *>(sv.get())->handle()));
        return 4;
    }
    std::printf("pointcloud size: %d, %d\n", n, n);
    std::ofstream f(out + "_cloud.bin", std::ios::binary);
    f.write(reinterpret_cast<const char *>(xyz.data()), (std::streamsize)n * 3 * sizeof(double));
    f.write(reinterpret_cast<const char *>(pix.data()), (std::streamsize)n);
    return f ? 0 : 3;
}
