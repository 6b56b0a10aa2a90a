// sgm_internal.h -- kernel launchers shared by the C-ABI (sgm_capi.hip) and
// the kernels (sgm_kernels.hip).  Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace sgm {

// Geometry of one frame on the working (decimated) grid.
struct Geom {
    int H, W, D;   // rows, cols, disparities
    int scale;     // 1 or 2
};

// What a sweep does with its path costs L_r ("Sweeps").
enum SweepMode {
    SWEEP_STORE_L = 0,  // write L_r and minL_r (parity tests)
    SWEEP_INIT = 1,     // acc_out = L_r
    SWEEP_ACC = 2,      // acc_out = acc_in + L_r   (acc_in may alias acc_out)
    SWEEP_FINAL = 3     // total = S + (T + L_r) -> WTA, uniqueness, sub-pixel
};

struct SweepArgs {
    const float *cost;   // HWD
    const float *acc_in; // HWD (ACC: chain state; FINAL: T chain)
    float *acc_out;      // HWD (STORE_L: L_r)
    const float *s_in;   // HWD (FINAL: S chain)
    float *min_out;      // HW  (STORE_L: minL_r)
    uint16_t *disp;      // HW  (FINAL)
    float *sub;          // HW  (FINAL)
    float p1, p2, uniq;
};

hipError_t launch_census(const uint8_t *src, int pitch, Geom g, int blur, uint64_t *ct,
                         hipStream_t st);
hipError_t launch_cost_h(const uint64_t *ctl, const uint64_t *ctr, const uint8_t *sky,
                         int sky_pitch, int view, int filter, Geom g, float *out,
                         hipStream_t st);
hipError_t launch_cost_v(const float *in, float *out, int filter, Geom g, hipStream_t st);
hipError_t launch_sweep(int dir, int mode, const SweepArgs &a, Geom g, hipStream_t st);
hipError_t launch_lr(const float *fl, const float *fr, float *out, int out_pitch, float lr,
                     Geom g, hipStream_t st);

}  // namespace sgm
