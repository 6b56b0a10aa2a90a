// dp_ilp.hip -- development probe: NCH independent scanline chains
// interleaved in one wave (the production dp_step + wave_min each), against
// one chain per wave, at equal numbers of chains.  Tells whether the s_nop
// hazard pads of a lone chain's step cost the SIMD issue cycles that other
// waves could use (interleaving fills them with the other chain's work).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../stereo_matching_amd/csrc/sgm_device.h"

using namespace sgm;

template <int NCH, int XN = 0>
__global__ __launch_bounds__(64) void chains(const float *__restrict__ cin, float *out, int nsteps) {
    const int lane = tid_x();
    float c[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < 2; ++v) c[k][v] = cin[((bid_x() & 7) * 4 * 64 + k * 64 + lane) * 2 + v];
    const float p2v = to_vgpr(20.0f);
    float L[NCH][2], pmin[NCH];
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
        L[q][0] = c[q & 3][0] + q;
        L[q][1] = c[q & 3][1];
        pmin[q] = 0.0f;
    }
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int q = 0; q < NCH; ++q) {
                float N[2];
                dp_step<2>(L[q], pmin[q], c[k], N, 3.0f, p2v);
                pmin[q] = wave_min(fminf(N[0], N[1]));
                if constexpr (XN > 0) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
                L[q][0] = N[0];
                L[q][1] = N[1];
            }
        }
    }
    float acc = 0.0f;
#pragma unroll
    for (int q = 0; q < NCH; ++q) acc += L[q][0] + L[q][1] + pmin[q];
    out[bid_x() * 64 + lane] = acc;
}

template <int NCH, int XN = 0>
static double ns_per_chain_step(int nchains, const float *dc, float *dout, int nsteps) {
    const int nb = (nchains + NCH - 1) / NCH;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    chains<NCH, XN><<<nb, 64>>>(dc, dout, nsteps);
    (void)hipEventRecord(e0);
    chains<NCH, XN><<<nb, 64>>>(dc, dout, nsteps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e6 / ((double)nb * NCH * nsteps);
}

int main() {
    const int NC = 8 * 4 * 64 * 2;
    float *dc, *dout;
    (void)hipMalloc(&dc, NC * sizeof(float));
    (void)hipMalloc(&dout, 16384 * 64 * sizeof(float));
    float *hc = (float *)malloc(NC * sizeof(float));
    srand(7);
    for (int i = 0; i < NC; ++i) hc[i] = (float)(rand() % 6200) / 100.0f + (rand() % 3 == 0 ? 0.2f : 0.0f);
    (void)hipMemcpy(dc, hc, NC * sizeof(float), hipMemcpyHostToDevice);
    const int nsteps = 2048;
    printf("ns per chain-step (lower is better), %d steps\n", nsteps);
    for (int nch : {375, 1242, 2484, 4096, 8192, 16384}) {
        const double a = ns_per_chain_step<1>(nch, dc, dout, nsteps);
        const double b = ns_per_chain_step<2>(nch, dc, dout, nsteps);
        const double c = ns_per_chain_step<4>(nch, dc, dout, nsteps);
        const double d = ns_per_chain_step<1, 1>(nch, dc, dout, nsteps);
        printf("chains %6d: 1/wave %7.3f | 2/wave %7.3f | 4/wave %7.3f | 1/wave + 4 x s_nop 7 per step %7.3f\n", nch, a, b, c, d);
    }
    return 0;
}
