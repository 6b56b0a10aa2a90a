// bw_probe.hip -- development probe: HBM bandwidth the scanline access
// patterns of the aggregation kernels can reach with no arithmetic, against
// plain coalesced streams.  Volumes are KITTI-sized (375 x 1242 x 128 f32).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int H = 375, W = 1242, D = 128;
constexpr long long N = (long long)H * W * D;

__global__ __launch_bounds__(256) void stream_copy(const float4 *__restrict__ a,
                                                   const float4 *__restrict__ b,
                                                   float4 *__restrict__ o, long long n4, int rd2) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        float4 x = a[i];
        if (rd2) {
            const float4 y = b[i];
            x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
        }
        o[i] = x;
    }
}

__global__ __launch_bounds__(256) void stream_read(const float4 *__restrict__ a, float *o, long long n4) {
    float s = 0;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 x = a[i];
        s += x.x + x.y + x.z + x.w;
    }
    if (s == 12345.f) o[0] = s;
}

// one wave per chain, chain walks DIR: 0 = column (down), 1 = diagonal up-left (wrapping),
// 2 = row; per step: read a (and b), write o; 512 B (D floats) per access; PF-deep ring
template <int DIR, int NRD, int PF>
__global__ __launch_bounds__(64) void chain_walk(const float *__restrict__ a, const float *__restrict__ b,
                                                 float *__restrict__ o, float *sink) {
    const int lane = threadIdx.x, g = blockIdx.x;
    const int n = DIR == 2 ? W : H;
    auto off_at = [&](int k) -> long long {
        int i, j;
        if (DIR == 0) { i = k; j = g; }
        else if (DIR == 1) { i = H - 1 - k; j = ((g - k) % W + W) % W; }
        else { i = g; j = k; }
        return ((long long)i * W + j) * D + lane * 2;
    };
    float2 ra[PF], rb[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        const long long off = off_at(u < n ? u : n - 1);
        ra[u] = *reinterpret_cast<const float2 *>(a + off);
        if (NRD > 1) rb[u] = *reinterpret_cast<const float2 *>(b + off);
    }
    float acc = 0;
    for (int k0 = 0; k0 < n; k0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int k = k0 + u;
            if (k < n) {
                float2 x = ra[u];
                if (NRD > 1) { x.x += rb[u].x; x.y += rb[u].y; }
                acc += x.x;
                if (o) *reinterpret_cast<float2 *>(o + off_at(k)) = x;
                const int kn = k + PF < n ? k + PF : n - 1;
                const long long off = off_at(kn);
                ra[u] = *reinterpret_cast<const float2 *>(a + off);
                if (NRD > 1) rb[u] = *reinterpret_cast<const float2 *>(b + off);
            }
        }
    }
    if (acc == 12345.f) sink[0] = acc;
}

template <typename F>
static float timeit(F f, int reps = 5) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    f();
    (void)hipEventRecord(e0);
    for (int r = 0; r < reps; ++r) f();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    float *a, *b, *o, *sink;
    (void)hipMalloc(&a, N * 4);
    (void)hipMalloc(&b, N * 4);
    (void)hipMalloc(&o, N * 4);
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(a, 0, N * 4);
    (void)hipMemset(b, 0, N * 4);
    const double MB = N * 4 / 1e6;
    const long long n4 = N / 4;
    float t;
    t = timeit([&] { stream_read<<<4096, 256>>>((const float4 *)a, sink, n4); });
    printf("stream read 1 vol           %7.1f us  %6.2f TB/s\n", t * 1e3, MB / t / 1e6);
    t = timeit([&] { stream_copy<<<4096, 256>>>((const float4 *)a, (const float4 *)b, (float4 *)o, n4, 0); });
    printf("stream 1R 1W                %7.1f us  %6.2f TB/s\n", t * 1e3, 2 * MB / t / 1e6);
    t = timeit([&] { stream_copy<<<4096, 256>>>((const float4 *)a, (const float4 *)b, (float4 *)o, n4, 1); });
    printf("stream 2R 1W                %7.1f us  %6.2f TB/s\n", t * 1e3, 3 * MB / t / 1e6);
    t = timeit([&] { chain_walk<0, 1, 16><<<W, 64>>>(a, b, nullptr, sink); });
    printf("column walk 1R   PF16       %7.1f us  %6.2f TB/s\n", t * 1e3, MB / t / 1e6);
    t = timeit([&] { chain_walk<0, 2, 16><<<W, 64>>>(a, b, o, sink); });
    printf("column walk 2R1W PF16       %7.1f us  %6.2f TB/s\n", t * 1e3, 3 * MB / t / 1e6);
    t = timeit([&] { chain_walk<1, 2, 16><<<W, 64>>>(a, b, o, sink); });
    printf("diag walk   2R1W PF16       %7.1f us  %6.2f TB/s\n", t * 1e3, 3 * MB / t / 1e6);
    t = timeit([&] { chain_walk<1, 2, 32><<<W, 64>>>(a, b, o, sink); });
    printf("diag walk   2R1W PF32       %7.1f us  %6.2f TB/s\n", t * 1e3, 3 * MB / t / 1e6);
    t = timeit([&] { chain_walk<1, 1, 16><<<W, 64>>>(a, b, o, sink); });
    printf("diag walk   1R1W PF16       %7.1f us  %6.2f TB/s\n", t * 1e3, 2 * MB / t / 1e6);
    t = timeit([&] { chain_walk<2, 2, 32><<<H, 64>>>(a, b, o, sink); });
    printf("row walk    2R1W PF32 (375) %7.1f us  %6.2f TB/s\n", t * 1e3, 3 * MB / t / 1e6);
    return 0;
}
