// Which HIP stream kinds run concurrently (i.e. land on different hardware
// queues)?  Launch one ~2 ms spin kernel on each of two streams of a kind and
// compare the wall time with one kernel's.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <stdio.h>
#include <vector>

__global__ void spin(long long cycles, int *sink) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {}
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(sink, 1);
}

static double run(hipStream_t a, hipStream_t b, int *sink, long long cycles) {
    hipDeviceSynchronize();
    auto t0 = std::chrono::steady_clock::now();
    spin<<<64, 64, 0, a>>>(cycles, sink);
    if (b) spin<<<64, 64, 0, b>>>(cycles, sink);
    hipDeviceSynchronize();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
    int *sink;
    hipMalloc(&sink, 4);
    const long long cycles = 4000000;  // ~2 ms at ~2 GHz
    std::vector<hipStream_t> plain(6);
    for (auto &s : plain) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int lo, hi;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStream_t p_hi, p_lo;
    hipStreamCreateWithPriority(&p_hi, hipStreamNonBlocking, hi);
    hipStreamCreateWithPriority(&p_lo, hipStreamNonBlocking, lo);
    uint32_t mask[8];
    for (auto &m : mask) m = 0xffffffffu;
    hipStream_t cm1, cm2;
    hipExtStreamCreateWithCUMask(&cm1, 8, mask);
    hipExtStreamCreateWithCUMask(&cm2, 8, mask);
    run(plain[0], nullptr, sink, cycles);  // warm up
    printf("one kernel                 : %.2f ms\n", run(plain[0], nullptr, sink, cycles));
    for (int k = 1; k < 6; ++k)
        printf("plain stream 0 + plain %d   : %.2f ms\n", k, run(plain[0], plain[k], sink, cycles));
    printf("priority hi + lo           : %.2f ms (range %d..%d)\n", run(p_hi, p_lo, sink, cycles), lo, hi);
    printf("priority hi + plain 0      : %.2f ms\n", run(p_hi, plain[0], sink, cycles));
    printf("cu-mask + cu-mask          : %.2f ms\n", run(cm1, cm2, sink, cycles));
    printf("cu-mask + plain 0          : %.2f ms\n", run(cm1, plain[0], sink, cycles));
    printf("null + plain 0             : %.2f ms\n", run(0, plain[0], sink, cycles));
    return 0;
}
