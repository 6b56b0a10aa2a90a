// dp_bfly.hip -- development probe: the DP step with the wave minimum taken
// by a full butterfly (four DPP row stages, then v_permlane16_swap and
// v_permlane32_swap, gfx950) so that every lane holds minLp in a VGPR, against
// the production dp_step + wave_min (row_bcast stages, v_readlane to an SGPR).
// Checks that both give the same path costs bit for bit and measures cycles
// per step for a lone chain and chain-steps per second at 375 / 1242 / 4096
// chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../stereo_matching_amd/csrc/sgm_device.h"

using namespace sgm;
typedef float f2 __attribute__((ext_vector_type(2)));

// minimum over the 64 lanes, in every lane (VGPR)
__device__ __forceinline__ float wave_min_all(float x) {
    x = fminf(x, movdppf<DPP_QP_1032>(x));
    x = fminf(x, movdppf<DPP_QP_2301>(x));
    x = fminf(x, movdppf<DPP_HALF_MIRROR>(x));
    x = fminf(x, movdppf<DPP_MIRROR>(x));
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
    x = fminf(__int_as_float(r[0]), __int_as_float(r[1]));
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(x), false, false);
    return fminf(__int_as_float(s[0]), __int_as_float(s[1]));
}

// dp_step<2> with minLp in a VGPR (every lane the same value)
__device__ __forceinline__ void dp_step_v(const float (&prev)[2], float pmin, const float (&c)[2],
                                          float (&L)[2], float p1, float p2) {
    const float pmin_p2 = pmin + p2;
    const f2 qq = f2{prev[0], prev[1]} + p1;
    float q0 = qq.x, q1 = qq.y;
    const float t0 = nbmin_self<DPP_WAVE_SHR1>(q1);
    const float t1 = nbmin_self<DPP_WAVE_SHL1>(q0);
    const f2 d = f2{c[0], c[1]} - f2{pmin, pmin};
    f2 m;
    m.x = fminf(fminf(prev[0], t0), pmin_p2);
    m.y = fminf(fminf(prev[1], t1), pmin_p2);
    const f2 r = m + d;
    L[0] = r.x;
    L[1] = r.y;
}

template <int MODE>
__global__ __launch_bounds__(64) void chain(const float *__restrict__ cin, float *out, long long *cyc,
                                            int nsteps) {
    const int lane = tid_x();
    float c[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < 2; ++v) c[k][v] = cin[((bid_x() & 7) * 4 * 64 + k * 64 + lane) * 2 + v];
    float L[2] = {c[0][0], c[0][1]};
    float pmin = 0.0f;
    const float p2v = to_vgpr(20.0f);
    const long long t0 = clock64();
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float N[2];
            if constexpr (MODE == 0) {
                dp_step<2>(L, pmin, c[k], N, 3.0f, p2v);
                pmin = wave_min(fminf(N[0], N[1]));
            } else {
                dp_step_v(L, pmin, c[k], N, 3.0f, 20.0f);
                pmin = wave_min_all(fminf(N[0], N[1]));
            }
            L[0] = N[0];
            L[1] = N[1];
        }
    }
    const long long t1 = clock64();
    out[(bid_x() * 64 + lane) * 3 + 0] = L[0];
    out[(bid_x() * 64 + lane) * 3 + 1] = L[1];
    out[(bid_x() * 64 + lane) * 3 + 2] = pmin;
    if (lane == 0) cyc[bid_x()] = t1 - t0;
}

template <int MODE>
static double run(int nblocks, int nsteps, const float *dc, float *dout, long long *dcyc, double *clk) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    chain<MODE><<<nblocks, 64>>>(dc, dout, dcyc, nsteps);
    (void)hipEventRecord(e0);
    chain<MODE><<<nblocks, 64>>>(dc, dout, dcyc, nsteps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long cyc = 0;
    (void)hipMemcpy(&cyc, dcyc, sizeof(cyc), hipMemcpyDeviceToHost);
    *clk = (double)cyc / nsteps;
    return ms * 1e6 / nsteps;
}

int main() {
    const int NC = 8 * 4 * 64 * 2;
    float *dc, *dout;
    long long *dcyc;
    (void)hipMalloc(&dc, NC * sizeof(float));
    (void)hipMalloc(&dout, 4096 * 64 * 3 * sizeof(float));
    (void)hipMalloc(&dcyc, 4096 * sizeof(long long));
    float *hc = (float *)malloc(NC * sizeof(float));
    srand(7);
    for (int i = 0; i < NC; ++i) hc[i] = (float)(rand() % 6200) / 100.0f + (rand() % 3 == 0 ? 0.2f : 0.0f);
    (void)hipMemcpy(dc, hc, NC * sizeof(float), hipMemcpyHostToDevice);
    const int NO = 4096 * 64 * 3;
    float *a = (float *)malloc(NO * 4), *b = (float *)malloc(NO * 4);
    double clk;
    for (int nsteps : {4, 64, 1024}) {
        run<0>(64, nsteps, dc, dout, dcyc, &clk);
        (void)hipMemcpy(a, dout, 64 * 64 * 3 * 4, hipMemcpyDeviceToHost);
        run<1>(64, nsteps, dc, dout, dcyc, &clk);
        (void)hipMemcpy(b, dout, 64 * 64 * 3 * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 64 * 64 * 3; ++i) bad += memcmp(&a[i], &b[i], 4) != 0;
        printf("nsteps %5d: %d mismatches of %d (e.g. %g vs %g)\n", nsteps, bad, 64 * 64 * 3, a[0], b[0]);
    }
    for (int nb : {1, 375, 1242, 2484, 4096}) {
        double c0, c1;
        const double t0 = run<0>(nb, 4096, dc, dout, dcyc, &c0);
        const double t1 = run<1>(nb, 4096, dc, dout, dcyc, &c1);
        printf("chains %5d: readlane %6.1f clk/step %7.2f ns/step | butterfly %6.1f clk/step %7.2f ns/step | ratio %.3f\n",
               nb, c0, t0, c1, t1, t0 / t1);
    }
    return 0;
}
