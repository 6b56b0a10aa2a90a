// Exhaustive check (all non-negative finite floats) that
//   q0 = x * r;  e = fma(-q0, c, x);  q = fma(e, r, q0)      (r = RN(1/c))
// equals the correctly rounded x / c for the IIR window constants c = 3, 5.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__global__ void check(float c, float r, uint32_t base, unsigned long long *bad, unsigned long long *first) {
    const uint32_t bits = base + blockIdx.x * blockDim.x + threadIdx.x;
    if (bits >= 0x7f800000u) return;  // +inf / NaN excluded
    const float x = __uint_as_float(bits);
    const float want = x / c;
    const float q0 = x * r;
    const float e = __builtin_fmaf(-q0, c, x);
    const float q = __builtin_fmaf(e, r, q0);
    if (__float_as_uint(q) != __float_as_uint(want)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, (unsigned long long)bits);
    }
}

int main() {
    const float cs[2] = {3.0f, 5.0f};
    unsigned long long *bad, *first;
    hipMalloc(&bad, 8); hipMalloc(&first, 8);
    for (float c : cs) {
        const float r = 1.0f / c;
        hipMemset(bad, 0, 8);
        unsigned long long ff = ~0ull;
        hipMemcpy(first, &ff, 8, hipMemcpyHostToDevice);
        for (uint64_t base = 0; base < 0x7f800000ull; base += (1ull << 28))
            check<<<(1u << 28) / 256, 256>>>(c, r, (uint32_t)base, bad, first);
        unsigned long long nb = 0, f = 0;
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        hipMemcpy(&f, first, 8, hipMemcpyDeviceToHost);
        printf("c=%g: %llu mismatches over [0, +inf); first bits 0x%llx (%g)\n", c, nb, f,
               nb ? (double)__builtin_bit_cast(float, (uint32_t)f) : 0.0);
    }
    return 0;
}
