// layout_probe.hip -- development probe: memory-only scanline walks in the
// production lane layout (one chain per wave, 8 B per lane: float2 loads,
// 512 B per wave-instruction) against a half-wave layout (two chains per
// wave, 32 lanes x 16 B each: float4 loads, two pixels per wave-instruction),
// same bytes, same wrapped-diagonal walk (the L8 sweep's: read C, read T,
// write T; C kept resident in the Infinity Cache, T streamed non-temporal)
// and the same column walk.  Tells whether the per-CU memory rate the K128
// passes run at is bound by wave-instructions or by bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../stereo_matching_amd/csrc/sgm_device.h"

using namespace sgm;
constexpr int H = 375, W = 1242, D = 128;
constexpr long long N = (long long)H * W * D;

template <int DIR, int PF, bool WRITE>
__global__ __launch_bounds__(64) void walk64(const float *__restrict__ c, float *t, float *sink) {
    const int lane = threadIdx.x, g = blockIdx.x;
    auto off_at = [&](int k) -> long long {
        const int i = H - 1 - k;
        const int j = DIR == 0 ? g : ((g - k) % W + W) % W;
        return ((long long)i * W + j) * D + lane * 2;
    };
    float2 rc[PF], rt[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        const long long off = off_at(u);
        rc[u] = *reinterpret_cast<const float2 *>(c + off);
        rt[u].x = __builtin_nontemporal_load(t + off);
        rt[u].y = __builtin_nontemporal_load(t + off + 1);
    }
    float acc = 0.f;
    for (int k0 = 0; k0 < H; k0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int k = k0 + u;
            if (k < H) {
                const float2 x = make_float2(rc[u].x + rt[u].x, rc[u].y + rt[u].y);
                acc += x.x;
                if (WRITE) {
                    const long long o = off_at(k);
                    __builtin_nontemporal_store(x.x, t + o);
                    __builtin_nontemporal_store(x.y, t + o + 1);
                }
                const long long off = off_at(k + PF < H ? k + PF : H - 1);
                rc[u] = *reinterpret_cast<const float2 *>(c + off);
                rt[u].x = __builtin_nontemporal_load(t + off);
                rt[u].y = __builtin_nontemporal_load(t + off + 1);
            }
        }
    }
    if (acc == 12345.f) sink[g] = acc;
}

// two chains per wave: lanes 0-31 chain 2b, lanes 32-63 chain 2b+1
template <int DIR, int PF, bool WRITE>
__global__ __launch_bounds__(64) void walk32(const float *__restrict__ c, float *t, float *sink) {
    const int lane = threadIdx.x, g = blockIdx.x * 2 + (lane >> 5), hl = lane & 31;
    const int gg = g < W ? g : W - 1;
    auto off_at = [&](int k) -> long long {
        const int i = H - 1 - k;
        const int j = DIR == 0 ? gg : ((gg - k) % W + W) % W;
        return ((long long)i * W + j) * D + hl * 4;
    };
    float4 rc[PF], rt[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        const long long off = off_at(u);
        rc[u] = *reinterpret_cast<const float4 *>(c + off);
        rt[u].x = __builtin_nontemporal_load(t + off);
        rt[u].y = __builtin_nontemporal_load(t + off + 1);
        rt[u].z = __builtin_nontemporal_load(t + off + 2);
        rt[u].w = __builtin_nontemporal_load(t + off + 3);
    }
    float acc = 0.f;
    for (int k0 = 0; k0 < H; k0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int k = k0 + u;
            if (k < H) {
                const float4 x = make_float4(rc[u].x + rt[u].x, rc[u].y + rt[u].y, rc[u].z + rt[u].z,
                                             rc[u].w + rt[u].w);
                acc += x.x;
                if (WRITE && g < W) {
                    const long long o = off_at(k);
                    __builtin_nontemporal_store(x.x, t + o);
                    __builtin_nontemporal_store(x.y, t + o + 1);
                    __builtin_nontemporal_store(x.z, t + o + 2);
                    __builtin_nontemporal_store(x.w, t + o + 3);
                }
                const long long off = off_at(k + PF < H ? k + PF : H - 1);
                rc[u] = *reinterpret_cast<const float4 *>(c + off);
                rt[u].x = __builtin_nontemporal_load(t + off);
                rt[u].y = __builtin_nontemporal_load(t + off + 1);
                rt[u].z = __builtin_nontemporal_load(t + off + 2);
                rt[u].w = __builtin_nontemporal_load(t + off + 3);
            }
        }
    }
    if (acc == 12345.f) sink[g] = acc;
}


// walk64 with the L8 sweep's DP on the loaded costs (T += L8): compute + memory
template <int PF>
__global__ __launch_bounds__(64) void walk64dp(const float *__restrict__ c, float *t, float *sink) {
    const int lane = threadIdx.x, g = blockIdx.x;
    auto off_at = [&](int k) -> long long {
        const int i = H - 1 - k;
        const int j = ((g - k) % W + W) % W;
        return ((long long)i * W + j) * D + lane * 2;
    };
    const float p2v = to_vgpr(100.0f);
    float2 rc[PF], rt[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        const long long off = off_at(u);
        rc[u] = *reinterpret_cast<const float2 *>(c + off);
        rt[u].x = __builtin_nontemporal_load(t + off);
        rt[u].y = __builtin_nontemporal_load(t + off + 1);
    }
    float prev[2] = {0.f, 0.f}, pmin = 0.f;
    for (int k0 = 0; k0 < H; k0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int k = k0 + u;
            if (k < H) {
                const float cc[2] = {rc[u].x, rc[u].y};
                float L[2];
                dp_step<2>(prev, pmin, cc, L, 10.0f, p2v);
                pmin = wave_min(fminf(L[0], L[1]));
                prev[0] = L[0];
                prev[1] = L[1];
                const long long o = off_at(k);
                __builtin_nontemporal_store(rt[u].x + L[0], t + o);
                __builtin_nontemporal_store(rt[u].y + L[1], t + o + 1);
                const long long off = off_at(k + PF < H ? k + PF : H - 1);
                rc[u] = *reinterpret_cast<const float2 *>(c + off);
                rt[u].x = __builtin_nontemporal_load(t + off);
                rt[u].y = __builtin_nontemporal_load(t + off + 1);
            }
        }
    }
    if (pmin == 12345.f) sink[g] = pmin;
}

// the same split over two waves of one workgroup: wave 0 moves memory
// (global -> LDS ring, LDS -> global), wave 1 runs the DP from LDS; one LDS
// barrier per block of BK steps (ring of 3 blocks)
template <int BK>
__global__ __launch_bounds__(128) void walk_split(const float *__restrict__ c, float *t, float *sink) {
    __shared__ float2 sc[3][BK][64], st[3][BK][64], so[3][BK][64];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = blockIdx.x;
    auto off_at = [&](int k) -> long long {
        const int i = H - 1 - k;
        const int j = ((g - k) % W + W) % W;
        return ((long long)i * W + j) * D + lane * 2;
    };
    const int nb = (H + BK - 1) / BK;
    if (wave == 0) {
        // block b: loads issued in iteration b, landed in LDS in iteration b+1,
        // consumed by the DP wave in iteration b+2, its results stored to
        // global memory in iteration b+3
        float2 lc[BK], lt[BK];
        auto issue = [&](int b) {
#pragma unroll
            for (int u = 0; u < BK; ++u) {
                int k = b * BK + u;
                k = k < H ? k : H - 1;
                const long long off = off_at(k);
                lc[u] = *reinterpret_cast<const float2 *>(c + off);
                lt[u].x = __builtin_nontemporal_load(t + off);
                lt[u].y = __builtin_nontemporal_load(t + off + 1);
            }
        };
        issue(0);
        for (int it = 0; it < nb + 3; ++it) {
            // results of block it-3 (written by the DP wave in iteration it-1)
            if (it >= 3) {
                const int b = it - 3;
#pragma unroll
                for (int u = 0; u < BK; ++u) {
                    const int k = b * BK + u;
                    if (k < H) {
                        const float2 x = so[b % 3][u][lane];
                        const long long o = off_at(k);
                        __builtin_nontemporal_store(x.x, t + o);
                        __builtin_nontemporal_store(x.y, t + o + 1);
                    }
                }
            }
            if (it < nb) {
#pragma unroll
                for (int u = 0; u < BK; ++u) {
                    sc[it % 3][u][lane] = lc[u];
                    st[it % 3][u][lane] = lt[u];
                }
                if (it + 1 < nb) issue(it + 1);
            }
            __syncthreads();
        }
    } else {
        const float p2v = to_vgpr(100.0f);
        float prev[2] = {0.f, 0.f}, pmin = 0.f;
        for (int it = 0; it < nb + 3; ++it) {
            if (it >= 1 && it - 1 < nb) {
                const int b = it - 1;
#pragma unroll
                for (int u = 0; u < BK; ++u) {
                    const float2 x = sc[b % 3][u][lane], y = st[b % 3][u][lane];
                    const float cc[2] = {x.x, x.y};
                    float L[2];
                    dp_step<2>(prev, pmin, cc, L, 10.0f, p2v);
                    pmin = wave_min(fminf(L[0], L[1]));
                    prev[0] = L[0];
                    prev[1] = L[1];
                    so[b % 3][u][lane] = make_float2(y.x + L[0], y.y + L[1]);
                }
            }
            __syncthreads();
        }
        if (pmin == 12345.f) sink[g] = pmin;
    }
}

template <typename F>
static float timeit(F f, int reps = 10) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    f();
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
    float *c, *t, *sink;
    (void)hipMalloc(&c, N * 4);
    (void)hipMalloc(&t, N * 4);
    (void)hipMalloc(&sink, W * 8);
    (void)hipMemset(c, 0, N * 4);
    (void)hipMemset(t, 0, N * 4);
    const double MB = N * 4 / 1e6;
    float a, b;
    for (int rep = 0; rep < 2; ++rep) {
        a = timeit([&] { walk64dp<16><<<W, 64>>>(c, t, sink); });
        b = timeit([&] { walk_split<4><<<W, 128>>>(c, t, sink); });
        const float b8 = timeit([&] { walk_split<8><<<W, 128>>>(c, t, sink); });
        printf("diag 2R1W + DP: one wave  %7.1f us | memory wave + DP wave (LDS ring) BK4 %7.1f us BK8 %7.1f us\n", a * 1e3, b * 1e3, b8 * 1e3);
        a = timeit([&] { walk64<1, 16, true><<<W, 64>>>(c, t, sink); });
        b = timeit([&] { walk32<1, 16, true><<<(W + 1) / 2, 64>>>(c, t, sink); });
        printf("diag 2R1W  64-lane %7.1f us %5.2f TB/s | 32-lane %7.1f us %5.2f TB/s\n", a * 1e3,
               3 * MB / a / 1e6, b * 1e3, 3 * MB / b / 1e6);
        a = timeit([&] { walk64<1, 16, false><<<W, 64>>>(c, t, sink); });
        b = timeit([&] { walk32<1, 16, false><<<(W + 1) / 2, 64>>>(c, t, sink); });
        printf("diag 2R    64-lane %7.1f us %5.2f TB/s | 32-lane %7.1f us %5.2f TB/s\n", a * 1e3,
               2 * MB / a / 1e6, b * 1e3, 2 * MB / b / 1e6);
        a = timeit([&] { walk64<0, 16, true><<<W, 64>>>(c, t, sink); });
        b = timeit([&] { walk32<0, 16, true><<<(W + 1) / 2, 64>>>(c, t, sink); });
        printf("col  2R1W  64-lane %7.1f us %5.2f TB/s | 32-lane %7.1f us %5.2f TB/s\n", a * 1e3,
               3 * MB / a / 1e6, b * 1e3, 3 * MB / b / 1e6);
    }
    return 0;
}
