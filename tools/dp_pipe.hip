// dp_pipe.hip -- development probe: a DP step whose wave minimum of the
// previous path costs is reduced at the start of the step, interleaved with
// the part of the step that does not need it (neighbour minima, + P1, the
// min with Lp[d]), against the production dp_step + wave_min at the end of
// each step.  Checks bit-exactness and prints cycles per step for one chain
// (latency) and for K128-like chain counts.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I.. tools/dp_pipe.hip -o tools/dp_pipe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../stereo_matching_amd/csrc/sgm_device.h"

using namespace sgm;
typedef float f2 __attribute__((ext_vector_type(2)));

// fused step, all in C++ (the compiler schedules the reduction and the
// pmin-free part freely; row_bcast steps as a DPP move + min)
__device__ __forceinline__ void step_fused_cpp(float (&L)[2], const float (&c)[2], float p1, float p2) {
    float x = fminf(L[0], L[1]);
    const float nb0 = fminf(dppf<DPP_WAVE_SHR1>(L[1], L[1]), L[1]);
    const float nb1 = fminf(dppf<DPP_WAVE_SHL1>(L[0], L[0]), L[0]);
    x = fminf(x, movdppf<DPP_QP_1032>(x));
    x = fminf(x, movdppf<DPP_QP_2301>(x));
    const f2 t = f2{nb0, nb1} + p1;
    const float m0 = fminf(L[0], t.x), m1 = fminf(L[1], t.y);
    x = fminf(x, movdppf<DPP_HALF_MIRROR>(x));
    x = fminf(x, movdppf<DPP_MIRROR>(x));
    x = fminf(x, dppf<DPP_BCAST15, 0xA>(x, x));
    x = fminf(x, dppf<DPP_BCAST31, 0xC>(x, x));
    const float pmin = readlane_f(x, 63);
    const float pp = pmin + p2;
    const f2 d = f2{c[0], c[1]} - pmin;
    const f2 r = f2{fminf(m0, pp), fminf(m1, pp)} + d;
    L[0] = r.x;
    L[1] = r.y;
}

// fused step with the DPP parts as asm, interleaved by hand
__device__ __forceinline__ void step_fused_asm(float (&L)[2], const float (&c)[2], float p1, float p2) {
    float x, n0, n1;
    asm volatile(
        "v_min_f32 %0, %3, %4\n\t"
        "v_mov_b32 %1, %4\n\t"
        "v_mov_b32 %2, %3\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_min_f32_dpp %1, %4, %1 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %2, %3, %2 wave_shl:1 row_mask:0xf bank_mask:0xf\n\t"
        "v_min_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32 %1, %5, %1\n\t"
        "v_add_f32 %2, %5, %2\n\t"
        "v_min_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_min_f32 %1, %3, %1\n\t"
        "v_min_f32 %2, %4, %2\n\t"
        "v_min_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_min_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
        : "=&v"(x), "=&v"(n0), "=&v"(n1)
        : "v"(L[0]), "v"(L[1]), "s"(p1));
    // n0, n1 now hold m' = min(Lp[d], min(Lp[d-1], Lp[d+1]) + P1)
    const float pmin = readlane_f(x, 63);
    const float pp = pmin + p2;
    const f2 d = f2{c[0], c[1]} - pmin;
    const f2 r = f2{fminf(n0, pp), fminf(n1, pp)} + d;
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
    float pmin = wave_min(fminf(L[0], L[1]));
    const long long t0 = clock64();
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (MODE == 0) {
                float N[2];
                dp_step<2>(L, pmin, c[k], N, 3.0f, 20.0f);
                pmin = wave_min(fminf(N[0], N[1]));
                L[0] = N[0];
                L[1] = N[1];
            } else if constexpr (MODE == 1) {
                step_fused_cpp(L, c[k], 3.0f, 20.0f);
            } else {
                step_fused_asm(L, c[k], 3.0f, 20.0f);
            }
        }
    }
    const long long t1 = clock64();
    out[(bid_x() * 64 + lane) * 2 + 0] = L[0];
    out[(bid_x() * 64 + lane) * 2 + 1] = L[1];
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
    (void)hipMalloc(&dout, 4096 * 64 * 2 * sizeof(float));
    (void)hipMalloc(&dcyc, 4096 * sizeof(long long));
    float *hc = (float *)malloc(NC * sizeof(float));
    srand(7);
    for (int i = 0; i < NC; ++i) hc[i] = (float)(rand() % 6200) / 100.0f + (rand() % 3 == 0 ? 0.2f : 0.0f);
    (void)hipMemcpy(dc, hc, NC * sizeof(float), hipMemcpyHostToDevice);
    const int NO = 64 * 64 * 2;
    float *a = (float *)malloc(NO * 4), *b = (float *)malloc(NO * 4), *e = (float *)malloc(NO * 4);
    double clk;
    for (int nsteps : {4, 64, 1024}) {
        run<0>(64, nsteps, dc, dout, dcyc, &clk);
        (void)hipMemcpy(a, dout, NO * 4, hipMemcpyDeviceToHost);
        run<1>(64, nsteps, dc, dout, dcyc, &clk);
        (void)hipMemcpy(b, dout, NO * 4, hipMemcpyDeviceToHost);
        run<2>(64, nsteps, dc, dout, dcyc, &clk);
        (void)hipMemcpy(e, dout, NO * 4, hipMemcpyDeviceToHost);
        int bad1 = 0, bad2 = 0;
        for (int i = 0; i < NO; ++i) {
            bad1 += memcmp(&a[i], &b[i], 4) != 0;
            bad2 += memcmp(&a[i], &e[i], 4) != 0;
        }
        printf("nsteps %5d: fused_cpp %d, fused_asm %d mismatches of %d (e.g. %g %g %g)\n", nsteps, bad1,
               bad2, NO, a[0], b[0], e[0]);
    }
    for (int nb : {1, 375, 1242, 2484, 4096}) {
        double c0, c1, c2;
        const double t0 = run<0>(nb, 4096, dc, dout, dcyc, &c0);
        const double t1 = run<1>(nb, 4096, dc, dout, dcyc, &c1);
        const double t2 = run<2>(nb, 4096, dc, dout, dcyc, &c2);
        printf("blocks %5d: production %6.1f clk %6.2f ns | fused_cpp %6.1f clk %6.2f ns | fused_asm %6.1f clk %6.2f ns per step\n",
               nb, c0, t0, c1, t1, c2, t2);
    }
    return 0;
}
