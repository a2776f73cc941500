// The gap between two updates split into its parts (probe, not part of the engine).  Kernel A
// stands for the finish kernel: it stamps s_memrealtime and then publishes a flag in mapped host
// memory (system-scope stores, as the engine's publish does).  The host spins on the flag and then
// launches kernel B, which stamps s_memrealtime at its first instruction; B stands for the next
// rollout launch.  Optionally kernel T, queued right behind A, spins for a few microseconds, as
// rank_draw_kernel runs behind the publish.  Per variant, medians of
//   gpu gap   B's start - A's stamp (device clock, 100 MHz)
//   call      the host's launch call for B (steady_clock)
//   detect    the flag seen - A's stamp is not measurable across clocks; instead B's start minus
//             the time the call returned is bounded by gpu gap - call
// Variants: B with 16-byte or 800-byte arguments, with and without T (5 us).
// Build: hipcc -O2 --offload-arch=gfx950 gap_probe.hip -o gap_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct Big { double d[100]; };

__global__ void k_pub(unsigned long long *stamp, volatile double *flag, double seq)
{
    if (threadIdx.x == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_store(stamp, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_waitcnt(0);
        __hip_atomic_store((double *)flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_tail(unsigned ticks)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
}

__global__ void k_small(unsigned long long *stamp)
{
    if (threadIdx.x == 0) __hip_atomic_store(stamp, (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_big(unsigned long long *stamp, Big b)
{
    if (threadIdx.x == 0) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_store(stamp, t + (b.d[7] == 12345.0 ? 1ull : 0ull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

int main()
{
    hipSetDevice(0);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned long long *h_st = nullptr, *d_st = nullptr;
    double *h_flag = nullptr, *d_flag = nullptr;
    hipHostMalloc((void **)&h_st, 64 * sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent);
    hipHostMalloc((void **)&h_flag, 16 * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent);
    hipHostGetDevicePointer((void **)&d_st, h_st, 0);
    hipHostGetDevicePointer((void **)&d_flag, h_flag, 0);
    h_flag[0] = 0.0;
    Big b{};
    const int N = 400;
    double seq = 0.0;
    for (int variant = 0; variant < 4; variant++) {
        const bool big = variant & 1, tail = variant & 2;
        std::vector<double> gap, call;
        for (int i = 0; i < N + 50; i++) {
            seq += 1.0;
            hipLaunchKernelGGL(k_pub, dim3(1), dim3(64), 0, s, d_st, d_flag, seq);
            if (tail) hipLaunchKernelGGL(k_tail, dim3(1), dim3(64), 0, s, 500u);   // 5 us
            while (*(volatile double *)h_flag != seq) {
            }
            const auto c0 = std::chrono::steady_clock::now();
            if (big) hipLaunchKernelGGL(k_big, dim3(1), dim3(64), 0, s, d_st + 8, b);
            else hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d_st + 8);
            const auto c1 = std::chrono::steady_clock::now();
            hipStreamSynchronize(s);
            if (i < 50) continue;   // warm-up
            const double g = (double)(h_st[8] - h_st[0]) * 0.01;   // us (100 MHz)
            gap.push_back(g);
            call.push_back(std::chrono::duration<double, std::micro>(c1 - c0).count());
        }
        std::printf("B %s, %s: gpu gap (A's stamp -> B's start) median %.2f us; launch call median %.2f us\n",
                    big ? "800-B args" : "16-B args", tail ? "a 5-us kernel behind A" : "nothing behind A", median(gap),
                    median(call));
    }
    // the same, but the host launches B without waiting for the flag (B queued behind A already):
    // the dispatch of a queued kernel behind a running one
    {
        std::vector<double> gap;
        for (int i = 0; i < N + 50; i++) {
            seq += 1.0;
            hipLaunchKernelGGL(k_pub, dim3(1), dim3(64), 0, s, d_st, d_flag, seq);
            hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s, d_st + 8);
            hipStreamSynchronize(s);
            if (i >= 50) gap.push_back((double)(h_st[8] - h_st[0]) * 0.01);
        }
        std::printf("B queued behind A: gpu gap median %.2f us\n", median(gap));
    }
    return 0;
}
