// dp_half.hip -- development probe: two scanline chains per wave (lanes 0-31
// and 32-63, four disparities per lane at D = 128) against the production
// layout (one chain per wave, two disparities per lane).  Checks that both
// give the same path costs bit for bit and measures chain-steps per second
// with the GPU filled to 1-4 chains' worth of waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "../stereo_matching_amd/csrc/sgm_device.h"

using namespace sgm;
typedef float f2 __attribute__((ext_vector_type(2)));

// one chain per wave (production dp_step + wave_min)
__global__ __launch_bounds__(64) void chain1(const float *__restrict__ cin, float *out, int nsteps) {
    const int lane = tid_x();
    const int ch = bid_x();
    float c[4][2];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < 2; ++v) c[k][v] = cin[((ch & 63) * 4 * 128) + k * 128 + lane * 2 + v];
    float L[2] = {0.0f, 0.0f};
    float pmin = 0.0f;
    const float p2v = to_vgpr(20.0f);
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float N[2];
            dp_step<2>(L, pmin, c[k], N, 3.0f, p2v);
            pmin = wave_min(fminf(N[0], N[1]));
            L[0] = N[0];
            L[1] = N[1];
        }
    }
    out[(ch * 128) + lane * 2] = L[0];
    out[(ch * 128) + lane * 2 + 1] = L[1];
}

// Half-wave minimum: every lane gets the minimum of its 32-lane half.
__device__ __forceinline__ float half_min(float x) {
    x = fminf(x, movdppf<DPP_QP_1032>(x));
    x = fminf(x, movdppf<DPP_QP_2301>(x));
    x = fminf(x, movdppf<DPP_HALF_MIRROR>(x));
    x = fminf(x, movdppf<DPP_MIRROR>(x));
    // rows 0<->1 and 2<->3 (v_permlane16_swap of a register with itself)
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
    return fminf(__int_as_float(r[0]), __int_as_float(r[1]));
}

// two chains per wave: lane l < 32 holds chain A's d = 4l .. 4l+3, lane
// l >= 32 chain B's d = 4(l-32) .. +3
__global__ __launch_bounds__(64) void chain2(const float *__restrict__ cin, float *out, int nsteps) {
    const int lane = tid_x();
    const int hl = lane & 31, ch = bid_x() * 2 + (lane >> 5);
    float c[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int v = 0; v < 4; ++v) c[k][v] = cin[((ch & 63) * 4 * 128) + k * 128 + hl * 4 + v];
    float L[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    float pmin = 0.0f;  // per half, in a VGPR
    const float p1 = 3.0f, p2 = 20.0f;
    // lanes whose wave_shr / wave_shl source is the other chain's edge
    const bool first = hl == 0, last = hl == 31;
    for (int s = 0; s < nsteps; s += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float q[4];
            {
                const f2 a = f2{L[0], L[1]} + p1, b = f2{L[2], L[3]} + p1;
                q[0] = a.x; q[1] = a.y; q[2] = b.x; q[3] = b.y;
            }
            float t[4];
            t[1] = fminf(q[0], q[2]);
            t[2] = fminf(q[1], q[3]);
            t[0] = nbmin<DPP_WAVE_SHR1>(q[3], q[1]);
            t[3] = nbmin<DPP_WAVE_SHL1>(q[0], q[2]);
            t[0] = first ? q[1] : t[0];
            t[3] = last ? q[2] : t[3];
            const float pp2 = pmin + p2;
            float N[4];
            const f2 d01 = f2{c[k][0], c[k][1]} - pmin, d23 = f2{c[k][2], c[k][3]} - pmin;
            f2 m01, m23;
            m01.x = fminf(fminf(L[0], t[0]), pp2);
            m01.y = fminf(fminf(L[1], t[1]), pp2);
            m23.x = fminf(fminf(L[2], t[2]), pp2);
            m23.y = fminf(fminf(L[3], t[3]), pp2);
            const f2 r01 = m01 + d01, r23 = m23 + d23;
            N[0] = r01.x; N[1] = r01.y; N[2] = r23.x; N[3] = r23.y;
            pmin = half_min(fminf(fminf(N[0], N[1]), fminf(N[2], N[3])));
#pragma unroll
            for (int v = 0; v < 4; ++v) L[v] = N[v];
        }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) out[(ch * 128) + hl * 4 + v] = L[v];
}

static float time_it(void (*launch)(int, const float *, float *, int), int nb, const float *dc,
                     float *dout, int nsteps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    launch(nb, dc, dout, nsteps);
    (void)hipEventRecord(e0);
    launch(nb, dc, dout, nsteps);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

static void l1(int nb, const float *dc, float *dout, int n) { chain1<<<nb, 64>>>(dc, dout, n); }
static void l2(int nb, const float *dc, float *dout, int n) { chain2<<<nb, 64>>>(dc, dout, n); }

int main() {
    const int NC = 64 * 4 * 128;
    float *dc, *d1, *d2;
    (void)hipMalloc(&dc, NC * sizeof(float));
    (void)hipMalloc(&d1, 8192 * 128 * sizeof(float));
    (void)hipMalloc(&d2, 8192 * 128 * sizeof(float));
    float *hc = (float *)malloc(NC * sizeof(float));
    srand(11);
    for (int i = 0; i < NC; ++i) hc[i] = (float)(rand() % 6200) / 100.0f + (rand() % 3 == 0 ? 0.2f : 0.0f);
    (void)hipMemcpy(dc, hc, NC * sizeof(float), hipMemcpyHostToDevice);
    // bit-exactness: the same 128 chains both ways
    for (int nsteps : {4, 64, 1024}) {
        chain1<<<128, 64>>>(dc, d1, nsteps);
        chain2<<<64, 64>>>(dc, d2, nsteps);
        (void)hipDeviceSynchronize();
        static float a[128 * 128], b[128 * 128];
        (void)hipMemcpy(a, d1, sizeof(a), hipMemcpyDeviceToHost);
        (void)hipMemcpy(b, d2, sizeof(b), hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i < 128 * 128; ++i) bad += memcmp(&a[i], &b[i], 4) != 0;
        printf("nsteps %5d: %d mismatches of %d (e.g. %g vs %g)\n", nsteps, bad, 128 * 128, a[5], b[5]);
    }
    const int nsteps = 4096;
    for (int chains : {375, 1024, 2048, 3072, 4096, 6144}) {
        const float t1 = time_it(l1, chains, dc, d1, nsteps);
        const float t2 = time_it(l2, (chains + 1) / 2, dc, d2, nsteps);
        printf("chains %5d: one per wave %7.2f us (%6.3f ns/chain-step) | two per wave %7.2f us (%6.3f ns/chain-step) | ratio %.3f\n",
               chains, t1 * 1e3, t1 * 1e6 / ((double)chains * nsteps), t2 * 1e3,
               t2 * 1e6 / ((double)chains * nsteps), t1 / t2);
    }
    return 0;
}
