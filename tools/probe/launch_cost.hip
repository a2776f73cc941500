// Host-side cost of the calls on the update path (A/B probe, not part of the engine): hipSetDevice,
// and hipLaunchKernelGGL of an empty kernel with 16-byte and 1144-byte (FrRolloutArgs) arguments.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
struct Big { double d[143]; };
__global__ void k_small(int *p) { if (p && threadIdx.x == 9999) p[0] = 1; }
__global__ void k_big(Big b) { if (b.d[0] == 12345.0 && threadIdx.x == 9999) ((int *)nullptr)[0] = 1; }
int main()
{
    hipSetDevice(0);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    Big b{};
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b);
    hipStreamSynchronize(s);
    const int N = 2000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) hipSetDevice(0);
    auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) { hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, nullptr); if (i % 100 == 99) hipStreamSynchronize(s); }
    hipStreamSynchronize(s);
    auto t2 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) { hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b); if (i % 100 == 99) hipStreamSynchronize(s); }
    hipStreamSynchronize(s);
    auto t3 = std::chrono::steady_clock::now();
    // idle-queue latency: launch, then wait for completion, one at a time
    auto t4 = std::chrono::steady_clock::now();
    for (int i = 0; i < 200; i++) { hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, b); hipStreamSynchronize(s); }
    auto t5 = std::chrono::steady_clock::now();
    auto us = [](auto a, auto b, int n) { return std::chrono::duration<double, std::micro>(b - a).count() / n; };
    std::printf("hipSetDevice %.3f us; launch 16 B args %.3f us; launch 1144 B args %.3f us (host call, queue busy); launch+sync idle %.2f us\n",
                us(t0, t1, N), us(t1, t2, N), us(t2, t3, N), us(t4, t5, 200));
    return 0;
}
