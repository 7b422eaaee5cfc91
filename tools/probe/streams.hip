// Probe: how many HIP streams run kernels concurrently on this device/runtime
// (GPU_MAX_HW_QUEUES hardware queues per process): S streams each launch one
// single-wave kernel that spins for ~T ms (s_memrealtime, no inter-kernel
// dependency, so it can never deadlock); the wall time is T if every stream
// has its own queue and k*T if up to k streams share one.
//   hipcc --offload-arch=gfx950 -O2 tools/probe/streams.hip -o /tmp/streams && /tmp/streams
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

int main() {
    const unsigned long long ticks = 100ULL * 20000;   // 100 MHz: 20 ms
    for (int S = 1; S <= 8; S++) {
        hipStream_t st[8];
        for (int i = 0; i < S; i++) hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
        for (int i = 0; i < S; i++) spin<<<1, 64, 0, st[i]>>>(ticks / 10);   // warm
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < S; i++) spin<<<1, 64, 0, st[i]>>>(ticks);
        hipDeviceSynchronize();
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        printf("streams=%d wall=%.1f ms (one kernel = 20 ms)\n", S, ms);
        for (int i = 0; i < S; i++) hipStreamDestroy(st[i]);
    }
    return 0;
}
