// sgm_bm.hip -- the WTA of BM::process (src/BM.cpp:53-85): winner-take-all
// straight on the filtered cost volume (no path aggregation), uniqueness
// min/sec > 0.7 with |min_d - sec_min_d| > 2.  Census, DSI and both cost
// filters are the SGM kernels (census with BM's row decimation, BM.cpp:24-25).
//
// One wave per pixel at a time, lane l holding d = l*V .. l*V+V-1 (V = D/64,
// or one d on lanes < D when D = 32): the pixel's D floats are one coalesced
// read; minima are wave reductions and first indices ballots (sgm_device.h).
// HBM-bound: 4 B per element read once.
#include "sgm_device.h"

namespace sgm {
namespace {

constexpr int kBmPixPerWave = 16;

template <int V>
__global__ __launch_bounds__(256) void bm_wta_kernel(const float *__restrict__ cost, int npx, int W,
                                                    int D, float uniq, uint16_t *__restrict__ disp,
                                                    float *__restrict__ out, int out_pitch) {
    const int lane = tid_x() & 63;
    const int wave = bid_x() * 4 + wave_id();
    const int p0 = wave * kBmPixPerWave;
    for (int q = 0; q < kBmPixPerWave; ++q) {
        const int p = p0 + q;
        if (p >= npx) break;
        const float *c = cost + (size_t)p * D;
        float tot[V];
#pragma unroll
        for (int v = 0; v < V; ++v) {
            const int d = lane * V + v;
            tot[v] = d < D ? __builtin_nontemporal_load(c + d) : SGM_INF;
        }
        float lm = tot[0];
#pragma unroll
        for (int v = 1; v < V; ++v) lm = fminf(lm, tot[v]);
        const float m = wave_min_u(lm);
        float ls = SGM_INF;
#pragma unroll
        for (int v = 0; v < V; ++v) ls = fminf(ls, tot[v] != m ? tot[v] : SGM_INF);
        const float sec = wave_min_u(ls);
        int d = first_index<V>(tot, m);
        if (sec != SGM_INF) {  // else sec_min_cost stays FLT_MAX: ratio ~ 0, never rejected
            const int sd = first_index<V>(tot, sec);
            if (m / sec > uniq && abs(d - sd) > 2) d = D + 1;
        }
        if (lane == 0) {
            disp[p] = (uint16_t)d;
            out[(size_t)(p / W) * out_pitch + p % W] = (float)d;
        }
    }
}

}  // namespace

hipError_t launch_bm_wta(const float *cost, float uniq, uint16_t *disp, float *out, int out_pitch,
                         Geom g, hipStream_t st) {
    const int npx = g.H * g.W;
    const int waves = (npx + kBmPixPerWave - 1) / kBmPixPerWave;
    const dim3 grid((waves + 3) / 4);
    switch (g.D) {
        case 32:
        case 64: hipLaunchKernelGGL(bm_wta_kernel<1>, grid, dim3(256), 0, st, cost, npx, g.W, g.D,
                                    uniq, disp, out, out_pitch); break;
        case 128: hipLaunchKernelGGL(bm_wta_kernel<2>, grid, dim3(256), 0, st, cost, npx, g.W, g.D,
                                     uniq, disp, out, out_pitch); break;
        case 256: hipLaunchKernelGGL(bm_wta_kernel<4>, grid, dim3(256), 0, st, cost, npx, g.W, g.D,
                                     uniq, disp, out, out_pitch); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sgm
