// sgm_consumers.hip -- the per-pixel consumers of the disparity map:
//   * Solver::colormap (src/Solver.cpp:652-707): the BGR rendering show_disp
//     publishes (node.cpp:107);
//   * the point cloud of node.cpp:119-143: back-projection of every valid
//     pixel with Z <= max_range, in row-major order (the reference's
//     push_back order), as an ordered compaction: per-row counts, one scan,
//     per-row writes at ballot-ranked positions.
// Both match the reference's float/double evaluation exactly.
#include "sgm_device.h"

namespace sgm {
namespace {

__global__ __launch_bounds__(256) void colormap_kernel(const float *__restrict__ disp, int pitch,
                                                      int H, int W, int D,
                                                      uint8_t *__restrict__ bgr, int bgr_pitch) {
    const int j = bid_x() * 64 + (tid_x() & 63), i = bid_y() * 4 + (tid_x() >> 6);
    if (i >= H || j >= W) return;
    float v = disp[(size_t)i * pitch + j];
    uint8_t b = 0, g = 0, r = 0;
    if (!(v > D - 1)) {
        v *= (256 / D);  // integer 256 / max_disp (:666)
        if (v <= 51) {
            b = 255; g = (uint8_t)(v * 5); r = 0;
        } else if (v <= 102) {
            v -= 51;
            b = (uint8_t)(255 - v * 5); g = 255; r = 0;
        } else if (v <= 153) {
            v -= 102;
            b = 0; g = 255; r = (uint8_t)(v * 5);
        } else if (v <= 204) {
            v -= 153;
            b = 0; g = (uint8_t)(255 - (uint8_t)(128.0 * v / 51.0 + 0.5)); r = 255;
        } else {
            v -= 204;
            b = 0; g = (uint8_t)(127 - (uint8_t)(127.0 * v / 51.0 + 0.5)); r = 255;
        }
    }
    uint8_t *p = bgr + (size_t)i * bgr_pitch + 3 * j;
    p[0] = b;
    p[1] = g;
    p[2] = r;
}

// node.cpp:125-140 for one pixel: is it a point, and where.
struct CloudArgs {
    float fx, fy, cx, cy, max_range;
    double baseline;
    float invalid;
    int scale;
};

__device__ __forceinline__ bool cloud_point(const CloudArgs &a, float d, int i, int j, double &X,
                                            double &Y, double &Z) {
    if (d == a.invalid) return false;                                   // :128
    Z = (a.fx + a.fy) / 2.0 * a.baseline / (d + 1e-6);                  // :130
    if (Z > a.max_range) return false;                                  // :131
    X = (j * a.scale - a.cx) * Z / a.fx;                                // :133
    Y = (i * a.scale - a.cy) * Z / a.fy;                                // :134
    return true;
}

// one wave per row: the row's point count
__global__ __launch_bounds__(64) void cloud_count_kernel(const float *__restrict__ disp, int pitch,
                                                        int H, int W, CloudArgs a,
                                                        int *__restrict__ counts) {
    const int i = bid_x(), lane = tid_x();
    int n = 0;
    for (int j0 = 0; j0 < W; j0 += 64) {
        const int j = j0 + lane;
        double X, Y, Z;
        const bool ok = j < W && cloud_point(a, disp[(size_t)i * pitch + j], i, j, X, Y, Z);
        n += __popcll(__ballot(ok));
    }
    if (lane == 0) counts[i] = n;
}

// exclusive scan of the row counts (one workgroup), total in counts[H]
__global__ __launch_bounds__(1024) void cloud_scan_kernel(int *counts, int H, int *total) {
    __shared__ int part[1024];
    const int t = tid_x();
    const int per = (H + 1023) / 1024, b = t * per;
    int s = 0;
    for (int k = 0; k < per && b + k < H; ++k) s += counts[b + k];
    part[t] = s;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan of the chunk sums
        const int v = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = t ? part[t - 1] : 0;
    for (int k = 0; k < per && b + k < H; ++k) {
        const int c = counts[b + k];
        counts[b + k] = run;
        run += c;
    }
    if (t == 1023) *total = part[1023];
}

__global__ __launch_bounds__(64) void cloud_write_kernel(const float *__restrict__ disp, int pitch,
                                                        const uint8_t *__restrict__ img,
                                                        int img_pitch, int H, int W, CloudArgs a,
                                                        const int *__restrict__ offsets,
                                                        double *__restrict__ xyz,
                                                        uint8_t *__restrict__ pixel) {
    const int i = bid_x(), lane = tid_x();
    int base = offsets[i];
    for (int j0 = 0; j0 < W; j0 += 64) {
        const int j = j0 + lane;
        double X = 0, Y = 0, Z = 0;
        const bool ok = j < W && cloud_point(a, disp[(size_t)i * pitch + j], i, j, X, Y, Z);
        const unsigned long long m = __ballot(ok);
        if (ok) {
            const int k = base + __popcll(m & ((1ull << lane) - 1));
            xyz[3 * (size_t)k + 0] = X;
            xyz[3 * (size_t)k + 1] = Y;
            xyz[3 * (size_t)k + 2] = Z;
            // img_l.at<uchar>(i, j) on the node's full-size image (:137)
            pixel[k] = img[(size_t)i * img_pitch + j];
        }
        base += __popcll(m);
    }
}

}  // namespace

hipError_t launch_colormap(const float *disp, int pitch, uint8_t *bgr, int bgr_pitch, Geom g,
                           hipStream_t st) {
    hipLaunchKernelGGL(colormap_kernel, dim3((g.W + 63) / 64, (g.H + 3) / 4), dim3(256), 0, st,
                       disp, pitch, g.H, g.W, g.D, bgr, bgr_pitch);
    return hipGetLastError();
}

hipError_t launch_point_cloud(const float *disp, int pitch, const uint8_t *img, int img_pitch,
                              float fx, float fy, float cx, float cy, double baseline,
                              float max_range, int *counts, double *xyz, uint8_t *pixel,
                              int *total, Geom g, hipStream_t st) {
    CloudArgs a{fx, fy, cx, cy, max_range, baseline, (float)(g.D + 1), g.scale};
    hipLaunchKernelGGL(cloud_count_kernel, dim3(g.H), dim3(64), 0, st, disp, pitch, g.H, g.W, a,
                       counts);
    hipLaunchKernelGGL(cloud_scan_kernel, dim3(1), dim3(1024), 0, st, counts, g.H, total);
    hipLaunchKernelGGL(cloud_write_kernel, dim3(g.H), dim3(64), 0, st, disp, pitch, img, img_pitch,
                       g.H, g.W, a, counts, xyz, pixel);
    return hipGetLastError();
}

}  // namespace sgm
