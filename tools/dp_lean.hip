// dp_lean.hip -- development probe: bit-exactness and cost of a leaner DP
// step (packed f32 adds, DPP-fused neighbour minima, row_bcast reduction to
// an SGPR) against the production dp_step + wave_min.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../stereo_matching_amd/csrc/sgm_device.h"

using namespace sgm;
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void dp_lean2(f2 &prev, float &pmin, f2 c, float p1, float p2) {
    const float pv[2] = {prev.x, prev.y}, cv[2] = {c.x, c.y};
    float L[2];
    dp_step<2>(pv, pmin, cv, L, p1, p2);
    pmin = wave_min(fminf(L[0], L[1]));
    prev = f2{L[0], L[1]};
}

template <int LEAN>
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
    f2 Lp = {c[0][0], c[0][1]};
    const long long t0 = clock64();
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (LEAN) {
                dp_lean2(Lp, pmin, f2{c[k][0], c[k][1]}, 3.0f, 20.0f);
            } else {
                float N[2];
                dp_step<2>(L, pmin, c[k], N, 3.0f, 20.0f);
                pmin = wave_min(fminf(N[0], N[1]));
                L[0] = N[0];
                L[1] = N[1];
            }
        }
    }
    const long long t1 = clock64();
    if (LEAN) { L[0] = Lp.x; L[1] = Lp.y; }
    out[(bid_x() * 64 + lane) * 3 + 0] = L[0];
    out[(bid_x() * 64 + lane) * 3 + 1] = L[1];
    out[(bid_x() * 64 + lane) * 3 + 2] = pmin;
    if (lane == 0) cyc[bid_x()] = t1 - t0;
}

// NCH independent chains interleaved in one wave
template <int NCH>
__global__ __launch_bounds__(64) void chain_multi(const float *__restrict__ cin, float *out, long long *cyc,
                                                  int nsteps) {
    const int lane = tid_x();
    float c[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < 2; ++v) c[k][v] = cin[((bid_x() & 7) * 4 * 64 + k * 64 + lane) * 2 + v];
    f2 Lp[NCH];
    float pmin[NCH];
#pragma unroll
    for (int q = 0; q < NCH; ++q) { Lp[q] = f2{c[q & 3][0] + q, c[q & 3][1]}; pmin[q] = 0.0f; }
    const long long t0 = clock64();
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int q = 0; q < NCH; ++q) dp_lean2(Lp[q], pmin[q], f2{c[k][0], c[k][1]}, 3.0f, 20.0f);
    }
    const long long t1 = clock64();
    float acc = 0;
#pragma unroll
    for (int q = 0; q < NCH; ++q) acc += Lp[q].x + Lp[q].y + pmin[q];
    out[bid_x() * 64 + lane] = acc;
    if (lane == 0) cyc[bid_x()] = t1 - t0;
}

template <int NCH>
static void run_multi(int nblocks, const float *dc, float *dout, long long *dcyc) {
    const int nsteps = 4096;
    chain_multi<NCH><<<nblocks, 64>>>(dc, dout, dcyc, nsteps);
    (void)hipDeviceSynchronize();
    long long cyc = 0;
    (void)hipMemcpy(&cyc, dcyc, sizeof(cyc), hipMemcpyDeviceToHost);
    printf("chains/wave %d blocks %5d: %6.1f clk per step of all chains, %6.1f per chain-step\n", NCH,
           nblocks, (double)cyc / nsteps, (double)cyc / nsteps / NCH);
}

template <int LEAN>
static double run(int nblocks, int nsteps, const float *dc, float *dout, long long *dcyc, double *clk) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    chain<LEAN><<<nblocks, 64>>>(dc, dout, dcyc, nsteps);
    (void)hipEventRecord(e0);
    chain<LEAN><<<nblocks, 64>>>(dc, dout, dcyc, nsteps);
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
    for (int nb : {1, 1242, 4096}) {
        double c0, c1;
        const double t0 = run<0>(nb, 4096, dc, dout, dcyc, &c0);
        const double t1 = run<1>(nb, 4096, dc, dout, dcyc, &c1);
        printf("blocks %5d: current %6.1f clk/step %7.2f ns/step | lean %6.1f clk/step %7.2f ns/step\n",
               nb, c0, t0, c1, t1);
    }
    for (int nb : {1, 375}) {
        run_multi<1>(nb, dc, dout, dcyc);
        run_multi<2>(nb, dc, dout, dcyc);
        run_multi<3>(nb, dc, dout, dcyc);
        run_multi<4>(nb, dc, dout, dcyc);
    }
    return 0;
}
