// band_probe.hip -- development probe: upside of running the backward phase
// of the frame (D2 pair, L8 sweep, final pass: three passes that all read the
// cost volume C and carry the accumulator T) band by band at 4K / HD sizes,
// so that C(band) and T(band) stay in the 256 MB Infinity Cache between the
// three passes, against three whole-volume passes.  Memory traffic only
// (coalesced streams, no DP):
//   pass 1: T = f(C, T5)        (D2 pair:  read C, T5 (nt), write T)
//   pass 2: T = f(C, T)         (L8 sweep: read C, T, write T)
//   pass 3: sink(C, S12, T)     (final:    read C, S12 (nt), T)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void p1(const float4 *__restrict__ c, const float *__restrict__ t5,
                                          float4 *__restrict__ t, long long n4) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 x = c[i];
        float4 y;
        y.x = __builtin_nontemporal_load(t5 + 4 * i);
        y.y = __builtin_nontemporal_load(t5 + 4 * i + 1);
        y.z = __builtin_nontemporal_load(t5 + 4 * i + 2);
        y.w = __builtin_nontemporal_load(t5 + 4 * i + 3);
        t[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
    }
}

__global__ __launch_bounds__(256) void p2(const float4 *__restrict__ c, float4 *__restrict__ t, long long n4) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 x = c[i], y = t[i];
        t[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
    }
}

__global__ __launch_bounds__(256) void p3(const float4 *__restrict__ c, const float *__restrict__ s12,
                                          const float4 *__restrict__ t, long long n4, float *sink) {
    float acc = 0.f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
        const float4 x = c[i], y = t[i];
        const float s = __builtin_nontemporal_load(s12 + 4 * i) + __builtin_nontemporal_load(s12 + 4 * i + 3);
        acc += x.x + y.y + s;
    }
    if (acc == -1.f) sink[0] = acc;
}

static double run(int H, int W, int D, int band_rows, float *C, float *T5, float *S12, float *T, float *sink) {
    const long long row = (long long)W * D;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        // bottom band first (the backward phase walks up)
        for (int i1 = H; i1 > 0; i1 -= band_rows) {
            const int i0 = i1 - band_rows > 0 ? i1 - band_rows : 0;
            const long long off = (long long)i0 * row, n4 = (long long)(i1 - i0) * row / 4;
            const int grid = 2048;
            p1<<<grid, 256>>>((const float4 *)(C + off), T5 + off, (float4 *)(T + off), n4);
            p2<<<grid, 256>>>((const float4 *)(C + off), (float4 *)(T + off), n4);
            p3<<<grid, 256>>>((const float4 *)(C + off), S12 + off, (const float4 *)(T + off), n4, sink);
        }
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    return best;
}

int main() {
    struct Cfg { const char *name; int H, W, D; };
    for (Cfg cfg : {Cfg{"K128", 375, 1242, 128}, Cfg{"4K256", 2160, 3840, 256}, Cfg{"HD256", 1080, 1920, 256}}) {
        const long long n = (long long)cfg.H * cfg.W * cfg.D;
        float *C, *T5, *S12, *T, *sink;
        if (hipMalloc(&C, n * 4) || hipMalloc(&T5, n * 4) || hipMalloc(&S12, n * 4) || hipMalloc(&T, n * 4) ||
            hipMalloc(&sink, 64)) {
            printf("alloc failed\n");
            return 1;
        }
        (void)hipMemset(C, 0, n * 4);
        (void)hipMemset(T5, 0, n * 4);
        (void)hipMemset(S12, 0, n * 4);
        (void)hipMemset(T, 0, n * 4);
        const double bytes = 10.0 * n * 4;  // 3 + 3 + 3 reads, 2 writes ... (C,T5,T | C,T,T | C,S12,T) = 10 streams
        const double rowmb = (double)cfg.W * cfg.D * 4 / 1e6;
        const double whole = run(cfg.H, cfg.W, cfg.D, cfg.H, C, T5, S12, T, sink);
        printf("%s whole volume: %8.3f ms  %.2f TB/s of stream bytes\n", cfg.name, whole, bytes / (whole * 1e-3) / 1e12);
        for (int mb : {32, 48, 64, 96, 128, 192}) {
            int rows = (int)(mb / rowmb);
            if (rows < 1) rows = 1;
            const double t = run(cfg.H, cfg.W, cfg.D, rows, C, T5, S12, T, sink);
            printf("%s bands of %4d rows (%6.1f MB of C per band): %8.3f ms  %.2f TB/s  x%.3f\n", cfg.name, rows,
                   rows * rowmb, t, bytes / (t * 1e-3) / 1e12, whole / t);
        }
        (void)hipFree(C);
        (void)hipFree(T5);
        (void)hipFree(S12);
        (void)hipFree(T);
        (void)hipFree(sink);
    }
    return 0;
}
