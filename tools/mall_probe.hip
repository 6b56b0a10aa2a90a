// mall_probe.hip -- development probe: can a 238 MB cost volume stay resident
// in the 256 MB Infinity Cache while other volumes stream past it, if the
// streaming accesses use non-temporal loads/stores?  Each "pass" reads C plus
// A and writes B (2R1W, like an accumulating sweep); five passes back to back.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr long long N = 375LL * 1242 * 128;  // K128 volume, floats

template <bool NT>
__global__ __launch_bounds__(256) void pass(const float4 *__restrict__ c, const float4 *__restrict__ a,
                                            float4 *__restrict__ b, long long n4) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 x = c[i];
        float4 y;
        if (NT) {
            y.x = __builtin_nontemporal_load(&a[i].x); y.y = __builtin_nontemporal_load(&a[i].y);
            y.z = __builtin_nontemporal_load(&a[i].z); y.w = __builtin_nontemporal_load(&a[i].w);
        } else {
            y = a[i];
        }
        float4 z = {x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w};
        if (NT) {
            __builtin_nontemporal_store(z.x, &b[i].x); __builtin_nontemporal_store(z.y, &b[i].y);
            __builtin_nontemporal_store(z.z, &b[i].z); __builtin_nontemporal_store(z.w, &b[i].w);
        } else {
            b[i] = z;
        }
    }
}

int main() {
    float *c, *bufs[6];
    (void)hipMalloc(&c, N * 4);
    for (auto &p : bufs) { (void)hipMalloc(&p, N * 4); (void)hipMemset(p, 0, N * 4); }
    (void)hipMemset(c, 0, N * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const long long n4 = N / 4;
    for (int nt = 0; nt < 2; ++nt) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int p = 0; p < 5; ++p) {
                const float4 *a = (const float4 *)bufs[(2 * p) % 6];
                float4 *b = (float4 *)bufs[(2 * p + 1) % 6];
                if (nt) pass<true><<<4096, 256>>>((const float4 *)c, a, b, n4);
                else pass<false><<<4096, 256>>>((const float4 *)c, a, b, n4);
            }
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double bytes = 5.0 * 3 * N * 4;
            printf("%s streams: 5 passes %.1f us  (%.2f TB/s of algorithmic bytes)\n",
                   nt ? "non-temporal" : "default     ", ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
