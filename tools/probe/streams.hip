// Probe: how many HIP streams run kernels concurrently on this device/runtime
// (GPU_MAX_HW_QUEUES hardware queues per process): S streams each launch one
// single-wave kernel that spins for ~T ms (s_memrealtime, no inter-kernel
// dependency, so it can never deadlock); the wall time is T if every stream
// has its own queue and k*T if up to k streams share one.
// Part 2: CU-masked streams (hipExtStreamCreateWithCUMask): where the
// workgroups of each stream land (XCC / SE / CU from the hardware ID
// registers) and whether a consumer kernel on one masked stream sees a flag a
// producer kernel on the other sets -- with a bounded wait, so serialised
// streams show up as a timeout, never as a hang.
//   hipcc --offload-arch=gfx950 -O2 tools/probe/streams.hip -o tools/probe/streams && tools/probe/streams
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <set>
#include <vector>

__global__ void spin(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

__device__ unsigned hw_id() {
    unsigned v, x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    // xcc:4 | se:3 | sh:1 | cu:4
    return ((x & 15) << 8) | (((v >> 13) & 7) << 5) | (((v >> 12) & 1) << 4) | ((v >> 8) & 15);
}

// every workgroup records where it ran, then spins ~ticks
__global__ void where(unsigned *ids, unsigned long long ticks) {
    if (threadIdx.x == 0) ids[blockIdx.x] = hw_id();
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

// producer: after `delay` ticks, set the flag (vector store + release)
__global__ void producer(int *flag, unsigned long long delay) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < delay) __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// consumer: wait for the flag at most `limit` ticks; out = ticks waited, or ~0 on timeout
__global__ void consumer(const int *flag, unsigned long long limit, unsigned long long *out) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long dt = 0;
    for (;;) {
        if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        dt = __builtin_amdgcn_s_memrealtime() - t0;
        if (dt > limit) { dt = ~0ULL; break; }
        __builtin_amdgcn_s_sleep(20);
    }
    if (threadIdx.x == 0) *out = dt;
}

static void summarize(const char *name, const std::vector<unsigned> &ids) {
    std::set<unsigned> cu, xcc;
    for (unsigned v : ids) { cu.insert(v); xcc.insert(v >> 8); }
    printf("%s: %zu workgroups on %zu distinct CUs over %zu XCCs\n", name, ids.size(), cu.size(), xcc.size());
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

    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int n_cu = p.multiProcessorCount;
    printf("CUs: %d\n", n_cu);
    // mask A: the first 32 logical CUs; mask B: the rest
    std::vector<uint32_t> ma((n_cu + 31) / 32, 0), mb((n_cu + 31) / 32, 0);
    for (int c = 0; c < n_cu; c++) (c < 32 ? ma : mb)[c / 32] |= 1u << (c % 32);
    hipStream_t sa, sb;
    if (hipExtStreamCreateWithCUMask(&sa, (uint32_t)ma.size(), ma.data()) != hipSuccess ||
        hipExtStreamCreateWithCUMask(&sb, (uint32_t)mb.size(), mb.data()) != hipSuccess) {
        printf("hipExtStreamCreateWithCUMask failed\n");
        return 0;
    }
    const int na = 256, nb = 2048;
    unsigned *ia, *ib;
    hipMalloc(&ia, na * 4);
    hipMalloc(&ib, nb * 4);
    where<<<na, 64, 0, sa>>>(ia, 100ULL * 2000);
    where<<<nb, 64, 0, sb>>>(ib, 100ULL * 2000);
    hipDeviceSynchronize();
    std::vector<unsigned> ha(na), hb(nb);
    hipMemcpy(ha.data(), ia, na * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hb.data(), ib, nb * 4, hipMemcpyDeviceToHost);
    summarize("mask A (32 CUs)", ha);
    summarize("mask B (rest)", hb);
    std::set<unsigned> sa_ids(ha.begin(), ha.end());
    int overlap = 0;
    for (unsigned v : std::set<unsigned>(hb.begin(), hb.end())) overlap += sa_ids.count(v);
    printf("CUs used by both masks: %d\n", overlap);

    // consumer launched first on A, producer on B: does A see B's flag?
    int *flag;
    unsigned long long *out;
    hipMalloc(&flag, 4);
    hipMalloc(&out, 8);
    for (int rep = 0; rep < 3; rep++) {
        hipMemset(flag, 0, 4);
        hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        consumer<<<1, 64, 0, sa>>>(flag, 100ULL * 50000, out);       // at most 50 ms
        producer<<<1, 64, 0, sb>>>(flag, 100ULL * 5000);             // sets it after 5 ms
        hipDeviceSynchronize();
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        unsigned long long w = 0;
        hipMemcpy(&w, out, 8, hipMemcpyDeviceToHost);
        if (w == ~0ULL) printf("cross-stream flag: TIMEOUT (streams serialised), wall %.1f ms\n", ms);
        else printf("cross-stream flag: seen after %.2f ms, wall %.1f ms\n", w / 100000.0, ms);
    }
    // the same with plain (unmasked) streams, 4 of them busy as in a check call
    hipStream_t q[4];
    for (int i = 0; i < 4; i++) hipStreamCreateWithFlags(&q[i], hipStreamNonBlocking);
    hipMemset(flag, 0, 4);
    hipDeviceSynchronize();
    consumer<<<1, 64, 0, q[1]>>>(flag, 100ULL * 50000, out);
    producer<<<1, 64, 0, q[0]>>>(flag, 100ULL * 5000);
    hipDeviceSynchronize();
    unsigned long long w = 0;
    hipMemcpy(&w, out, 8, hipMemcpyDeviceToHost);
    if (w == ~0ULL) printf("plain streams flag: TIMEOUT\n");
    else printf("plain streams flag: seen after %.2f ms\n", w / 100000.0);
    return 0;
}
