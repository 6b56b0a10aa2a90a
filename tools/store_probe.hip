// store_probe.hip -- development probe: the write rate of cost_h's store
// pattern against alternatives, on a KITTI-sized (375 x 1242 x 128 f32)
// volume written row-major (i, j, d), non-temporal.  Each "chain" walks its
// row's W columns and stores at every step; DELAY dependent VALU ops per step
// stand in for the IIR's serial work.
//   A: cost_h today: lane = d, 64 disparities per wave, two waves per row
//      (a 256 B store per wave-step, the pixel's other half from the other wave)
//   B: one wave per row, two disparities per lane: one 512 B dwordx2 store per step
//   C: like A, but both waves of a row in one workgroup of one row only
//   D: like A, but every 4 steps one dwordx4 store per lane (16 lanes per
//      pixel's 64 disparities, 4 pixels per 1 KB wave-instruction), the
//      4x64 block transposed through LDS
//   E: A with default-policy (cached) stores
//   F: the flat float4 stream (grid-stride), the volume's write ceiling
// Usage: hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o /tmp/store_probe && /tmp/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int H = 375, W = 1242, D = 128;
constexpr long long N = (long long)H * W * D;

template <int DELAY>
__device__ __forceinline__ float work(float x) {
#pragma unroll
    for (int k = 0; k < DELAY; ++k) x = x * 1.0001f + 0.5f;
    return x;
}

// A / C: R rows per workgroup, D threads per row (lane = d)
template <int DELAY>
__global__ __launch_bounds__(256) void pat_a(float *__restrict__ o, int R) {
    const int r = threadIdx.x / D, d = threadIdx.x % D;
    const int i = blockIdx.x * R + r;
    if (i >= H) return;
    float x = (float)d;
    float *p = o + (long long)i * W * D + d;
    for (int j = 0; j < W; ++j) {
        x = work<DELAY>(x);
        __builtin_nontemporal_store(x, p + (long long)j * D);
    }
}

// B: one wave per row, lane holds d = 2*lane, 2*lane+1
template <int DELAY>
__global__ __launch_bounds__(64) void pat_b(float *__restrict__ o) {
    const int lane = threadIdx.x, i = blockIdx.x;
    float x = (float)lane, y = x + 1.f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 *p = reinterpret_cast<f2 *>(o + (long long)i * W * D) + lane;
    for (int j = 0; j < W; ++j) {
        x = work<DELAY>(x);
        y = work<DELAY>(y);
        f2 v = {x, y};
        __builtin_nontemporal_store(v, p + (long long)j * (D / 2));
    }
}

// D: lane = d for the chain; every 4 steps a 64 x 4 block goes through LDS
template <int DELAY>
__global__ __launch_bounds__(256) void pat_d(float *__restrict__ o) {
    __shared__ float tile[4][4][68];  // per wave: 4 steps x 64 d (+pad)
    const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int r = threadIdx.x / D, d = threadIdx.x % D;
    const int i = blockIdx.x * 2 + r;
    if (i >= H) return;
    float x = (float)d;
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int dbase = d - lane;  // 0 or 64
    float *prow = o + (long long)i * W * D + dbase + 4 * (lane % 16);
    for (int j = 0; j + 4 <= W; j += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            x = work<DELAY>(x);
            tile[wv][u][lane] = x;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        const int u = lane / 16, q = 4 * (lane % 16);
        f4 v = {tile[wv][u][q], tile[wv][u][q + 1], tile[wv][u][q + 2], tile[wv][u][q + 3]};
        __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(prow + (long long)(j + u) * D));
        __builtin_amdgcn_wave_barrier();
    }
}

template <int DELAY>
__global__ __launch_bounds__(256) void pat_e(float *__restrict__ o, int R) {
    const int r = threadIdx.x / D, d = threadIdx.x % D;
    const int i = blockIdx.x * R + r;
    if (i >= H) return;
    float x = (float)d;
    float *p = o + (long long)i * W * D + d;
    for (int j = 0; j < W; ++j) {
        x = work<DELAY>(x);
        p[(long long)j * D] = x;
    }
}

__global__ __launch_bounds__(256) void pat_f(float *__restrict__ o) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 *p = reinterpret_cast<f4 *>(o);
    const long long n4 = N / 4;
    for (long long k = blockIdx.x * 256ll + threadIdx.x; k < n4; k += (long long)gridDim.x * 256) {
        f4 v = {(float)k, 1.f, 2.f, 3.f};
        __builtin_nontemporal_store(v, p + k);
    }
}

template <typename F>
static float time_it(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) f();
    hipEventRecord(a);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / reps;
}

template <int DELAY>
static void run(float *o) {
    const double bytes = (double)N * 4;
    const float ta2 = time_it([&] { pat_a<DELAY><<<(H + 1) / 2, 2 * D>>>(o, 2); });
    const float ta1 = time_it([&] { pat_a<DELAY><<<H, D>>>(o, 1); });
    const float tb = time_it([&] { pat_b<DELAY><<<H, 64>>>(o); });
    const float td = time_it([&] { pat_d<DELAY><<<(H + 1) / 2, 2 * D>>>(o); });
    const float te = time_it([&] { pat_e<DELAY><<<(H + 1) / 2, 2 * D>>>(o, 2); });
    printf("delay %3d  D (dwordx4 via LDS) %7.1f us %5.2f TB/s | E (A, cached) %7.1f us %5.2f TB/s\n",
           DELAY, td, bytes / td / 1e6, te, bytes / te / 1e6);
    printf("delay %3d  A (2 rows/WG, 4 waves, 256 B/store) %7.1f us %5.2f TB/s | "
           "C (1 row/WG) %7.1f us %5.2f TB/s | B (1 wave/row, 512 B dwordx2) %7.1f us %5.2f TB/s\n",
           DELAY, ta2, bytes / ta2 / 1e6, ta1, bytes / ta1 / 1e6, tb, bytes / tb / 1e6);
}

int main() {
    float *o;
    if (hipMalloc(&o, N * sizeof(float)) != hipSuccess) return 1;
    const float tf = time_it([&] { pat_f<<<4096, 256>>>(o); });
    printf("F (flat float4 nt stream) %7.1f us %5.2f TB/s\n", tf, (double)N * 4 / tf / 1e6);
    run<0>(o);
    run<4>(o);
    run<8>(o);
    run<16>(o);
    hipFree(o);
    return 0;
}
