// dp_latency.hip -- cycles per DP step of one scanline chain (dp_step + the
// 64-lane minimum that feeds the next step) for several reduction schemes.
// Development probe; build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off
//   -fno-honor-nans -mno-amdgpu-ieee -I../include -o dp_latency dp_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../stereo_matching_amd/csrc/sgm_device.h"

using namespace sgm;

// row (16-lane) minimum in every lane
__device__ __forceinline__ float row_min(float x) {
    x = fminf(x, movdppf<DPP_QP_1032>(x));
    x = fminf(x, movdppf<DPP_QP_2301>(x));
    x = fminf(x, movdppf<DPP_HALF_MIRROR>(x));
    x = fminf(x, movdppf<DPP_MIRROR>(x));
    return x;
}

__device__ __forceinline__ uint32_t umin_s(uint32_t a, uint32_t b) { return a < b ? a : b; }

template <int R>
__device__ __forceinline__ float reduce(float x) {
    if constexpr (R == 0) {
        return wave_min(x);
    } else if constexpr (R == 1) {  // GCN row_bcast chain, lane 63 -> SGPR
        x = row_min(x);
        x = fminf(x, __int_as_float(movdpp<DPP_BCAST15, 0xA>(__float_as_int(x))));
        x = fminf(x, __int_as_float(movdpp<DPP_BCAST31, 0xC>(__float_as_int(x))));
        return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
    } else if constexpr (R == 2) {  // row minima -> 4 readlanes -> SALU
        x = row_min(x);
        const uint32_t a = __builtin_amdgcn_readlane(__float_as_uint(x), 0);
        const uint32_t b = __builtin_amdgcn_readlane(__float_as_uint(x), 16);
        const uint32_t c = __builtin_amdgcn_readlane(__float_as_uint(x), 32);
        const uint32_t d = __builtin_amdgcn_readlane(__float_as_uint(x), 48);
        return __uint_as_float(umin_s(umin_s(a, b), umin_s(c, d)));
    } else if constexpr (R == 3) {  // permlane swaps, then readfirstlane
        return wave_min_u(x);
    } else {  // no reduction (dp_step latency alone)
        return 0.0f;
    }
}

template <int V, int R>
__global__ __launch_bounds__(64) void chain(const float *__restrict__ cin, float *out,
                                            long long *cyc, int nsteps) {
    const int lane = threadIdx.x;
    float c[4][V];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < V; ++v) c[k][v] = cin[(k * 64 + lane) * V + v];
    float L[V];
#pragma unroll
    for (int v = 0; v < V; ++v) L[v] = c[0][v];
    float pmin = 0.0f;
    const long long t0 = clock64();
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float N[V];
            dp_step<V>(L, pmin, c[k], N, 3.0f, 20.0f);
            float m = N[0];
#pragma unroll
            for (int v = 1; v < V; ++v) m = fminf(m, N[v]);
            pmin = R == 4 ? pmin : reduce<R>(m);
#pragma unroll
            for (int v = 0; v < V; ++v) L[v] = N[v];
        }
    }
    const long long t1 = clock64();
    float acc = pmin;
#pragma unroll
    for (int v = 0; v < V; ++v) acc += L[v];
    out[blockIdx.x * 64 + lane] = acc;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V, int R>
static void run(const char *name, int nblocks, const float *dc, float *dout, long long *dcyc) {
    const int nsteps = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    chain<V, R><<<nblocks, 64>>>(dc, dout, dcyc, nsteps);
    hipEventRecord(e0);
    chain<V, R><<<nblocks, 64>>>(dc, dout, dcyc, nsteps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    long long cyc = 0;
    hipMemcpy(&cyc, dcyc, sizeof(cyc), hipMemcpyDeviceToHost);
    printf("V=%d %-28s blocks=%5d  %7.1f clk/step (lane0 clock64)  %7.2f ns/step (event)\n", V,
           name, nblocks, (double)cyc / nsteps, ms * 1e6 / nsteps);
}

int main() {
    float *dc, *dout;
    long long *dcyc;
    hipMalloc(&dc, 4 * 64 * 4 * sizeof(float));
    hipMalloc(&dout, 4096 * 64 * sizeof(float));
    hipMalloc(&dcyc, 4096 * sizeof(long long));
    float hc[4 * 64 * 4];
    for (int i = 0; i < 4 * 64 * 4; ++i) hc[i] = (float)((i * 37) % 61);
    hipMemcpy(dc, hc, sizeof(hc), hipMemcpyHostToDevice);
    for (int nb : {1, 1242, 4096}) {
        run<2, 0>("wave_min (permlane swaps)", nb, dc, dout, dcyc);
        run<2, 1>("row_bcast + readlane63", nb, dc, dout, dcyc);
        run<2, 2>("row_min + 4 readlane + SALU", nb, dc, dout, dcyc);
        run<2, 3>("permlane + readfirstlane", nb, dc, dout, dcyc);
        run<2, 4>("dp_step only", nb, dc, dout, dcyc);
    }
    run<4, 0>("wave_min (permlane swaps)", 1, dc, dout, dcyc);
    run<4, 1>("row_bcast + readlane63", 1, dc, dout, dcyc);
    run<4, 2>("row_min + 4 readlane + SALU", 1, dc, dout, dcyc);
    run<1, 0>("wave_min (permlane swaps)", 1, dc, dout, dcyc);
    run<1, 2>("row_min + 4 readlane + SALU", 1, dc, dout, dcyc);
    return 0;
}
