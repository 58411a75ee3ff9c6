// Host-path latency calibration (diagnostic, not product): what one synchronous
// host-buffer codec call pays besides its kernels on this box. Each row is the
// median of 200 repetitions (us):
//   sync_idle       hipStreamSynchronize on an idle stream
//   launch_sync     empty kernel launch + hipStreamSynchronize
//   h2d_64k_sync    hipMemcpyAsync H2D 64 KiB (registered) + sync
//   h2d_1m_sync     hipMemcpyAsync H2D 1 MiB (registered) + sync
//   d2h_128_sync    hipMemcpyAsync D2H 128 B into pinned memory + sync
//   chain4_sync     H2D 1 MiB + empty kernel + empty kernel + D2H 128 B + sync
//   kernel_flag_spin  empty kernel that writes a flag into mapped pinned memory,
//                   host spins on the flag (no stream sync)
//   zc_read_1m_spin kernel reading 1 MiB of mapped pinned host memory (zero copy,
//                   256 WGs) and writing a flag, host spins on the flag
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

__global__ void k_empty() {}
__global__ void k_flag(volatile uint32_t *flag, uint32_t v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __threadfence_system();
        *flag = v;
    }
}
__global__ void k_zc_read(const uint4 *p, uint64_t n16, uint32_t *acc, volatile uint32_t *flag, uint32_t v,
                          uint32_t *done) {
    uint32_t x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        uint4 q = p[i];
        x ^= q.x ^ q.y ^ q.z ^ q.w;
    }
    if (x == 0x12345678) acc[0] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(done, 1u) == gridDim.x - 1) {
            *done = 0;
            __threadfence_system();
            *flag = v;
        }
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const size_t M = 1 << 20;
    uint8_t *h = (uint8_t *)aligned_alloc(4096, M);
    memset(h, 1, M);
    hipHostRegister(h, M, hipHostRegisterMapped);
    uint8_t *hd = nullptr;
    hipHostGetDevicePointer((void **)&hd, h, 0);
    uint8_t *d;
    hipMalloc(&d, M);
    uint32_t *acc, *done;
    hipMalloc(&acc, 64);
    hipMalloc(&done, 64);
    hipMemset(done, 0, 64);
    void *pin;
    hipHostMalloc(&pin, 4096, hipHostMallocMapped);
    volatile uint32_t *flag = (volatile uint32_t *)pin;
    uint32_t *dflag;
    hipHostGetDevicePointer((void **)&dflag, pin, 0);
    auto run = [&](const char *name, auto fn) {
        std::vector<double> t;
        for (int i = 0; i < 20; ++i) fn(i);
        for (int i = 0; i < 200; ++i) {
            double t0 = now_us();
            fn(i);
            t.push_back(now_us() - t0);
        }
        std::sort(t.begin(), t.end());
        printf("{\"row\": \"%s\", \"median_us\": %.1f, \"p10_us\": %.1f, \"p90_us\": %.1f}\n", name, t[100], t[20], t[180]);
    };
    run("sync_idle", [&](int) { hipStreamSynchronize(s); });
    run("launch_sync", [&](int) { hipLaunchKernelGGL(k_empty, 1, 64, 0, s); hipStreamSynchronize(s); });
    run("h2d_64k_sync", [&](int) { hipMemcpyAsync(d, h, 65536, hipMemcpyHostToDevice, s); hipStreamSynchronize(s); });
    run("h2d_1m_sync", [&](int) { hipMemcpyAsync(d, h, M, hipMemcpyHostToDevice, s); hipStreamSynchronize(s); });
    run("d2h_128_sync", [&](int) { hipMemcpyAsync((uint8_t *)pin + 1024, d, 128, hipMemcpyDeviceToHost, s); hipStreamSynchronize(s); });
    run("chain4_sync", [&](int) {
        hipMemcpyAsync(d, h, M, hipMemcpyHostToDevice, s);
        hipLaunchKernelGGL(k_empty, 255, 320, 0, s);
        hipLaunchKernelGGL(k_empty, 4, 512, 0, s);
        hipMemcpyAsync((uint8_t *)pin + 1024, d, 128, hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
    });
    uint32_t seq = 0;
    run("kernel_flag_spin", [&](int) {
        const uint32_t v = ++seq;
        hipLaunchKernelGGL(k_flag, 1, 64, 0, s, (volatile uint32_t *)dflag, v);
        while (*flag != v) {}
    });
    run("zc_read_1m_spin", [&](int) {
        const uint32_t v = ++seq;
        hipLaunchKernelGGL(k_zc_read, 256, 256, 0, s, (const uint4 *)hd, (uint64_t)(M / 16), acc,
                           (volatile uint32_t *)dflag, v, done);
        while (*flag != v) {}
    });
    run("zc_read_1m_sync", [&](int) {
        const uint32_t v = ++seq;
        hipLaunchKernelGGL(k_zc_read, 256, 256, 0, s, (const uint4 *)hd, (uint64_t)(M / 16), acc,
                           (volatile uint32_t *)dflag, v, done);
        hipStreamSynchronize(s);
    });
    hipStreamSynchronize(s);
    return 0;
}
