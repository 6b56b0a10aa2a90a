// store_probe.hip -- development probe: the write rate of cost_h's store
// pattern against alternatives, on a KITTI-sized (375 x 1242 x 128 f32)
// volume written row-major (i, j, d), non-temporal.  Each "chain" walks its
// row's W columns and stores at every step; DELAY dependent VALU ops per step
// stand in for the IIR's serial work.
//   A: cost_h today: lane = d, 64 disparities per wave, two waves per row
//      (a 256 B store per wave-step, the pixel's other half from the other wave)
//   B: one wave per row, two disparities per lane: one 512 B dwordx2 store per step
//   C: like A, but both waves of a row in one workgroup of one row only
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
    printf("delay %3d  A (2 rows/WG, 4 waves, 256 B/store) %7.1f us %5.2f TB/s | "
           "C (1 row/WG) %7.1f us %5.2f TB/s | B (1 wave/row, 512 B dwordx2) %7.1f us %5.2f TB/s\n",
           DELAY, ta2, bytes / ta2 / 1e6, ta1, bytes / ta1 / 1e6, tb, bytes / tb / 1e6);
}

int main() {
    float *o;
    if (hipMalloc(&o, N * sizeof(float)) != hipSuccess) return 1;
    run<0>(o);
    run<4>(o);
    run<8>(o);
    run<16>(o);
    hipFree(o);
    return 0;
}
