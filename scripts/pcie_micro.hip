// Diagnostic only: how fast do workgroups read a small registered host record in place
// over the host link (the resident service's hashing stage at C1)? One
// launch reads B bytes of mapped pinned host memory with G workgroups of 256 threads,
// every lane issuing all of its 16-B loads before using any; in-kernel wall clock
// (s_memrealtime, 100 MHz) from the first workgroup's start to the last one's end.
// build: hipcc --offload-arch=gfx950 -O3 -o scripts/pcie_micro scripts/pcie_micro.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <algorithm>
#include <vector>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

// per thread: up to 32 chunks of 16 B, chunk c = tid + 256 k of the workgroup's slice
__global__ __launch_bounds__(256) void k_read(const uint4 *__restrict__ src, uint64_t n16, uint64_t *t, uint32_t *sink) {
    const uint64_t t0 = now();
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = blockIdx.x * per, hi = min(lo + per, n16);
    uint4 v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint64_t c = lo + threadIdx.x + 256ull * k;
        v[k] = c < hi ? src[c] : make_uint4(0, 0, 0, 0);
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 32; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    __syncthreads();
    const uint64_t t1 = now();
    if (x == 0x12345678u) sink[0] = x;
    if (threadIdx.x == 0) {
        atomicMin((unsigned long long *)&t[0], (unsigned long long)t0);
        atomicMax((unsigned long long *)&t[1], (unsigned long long)t1);
    }
}

int main() {
    std::vector<uint64_t> sizes = {4608, 38912, 304128, 1048576};
    std::vector<int> grids = {1, 2, 4, 8, 16, 32, 64, 128};
    // three kinds of host memory: hipHostMalloc coherent / non-coherent, and a
    // hipHostRegister'ed malloc range (what iggy_codec_host_register makes)
    uint8_t *hm[3];
    CK(hipHostMalloc((void **)&hm[0], 1 << 22, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&hm[1], 1 << 22, hipHostMallocMapped | hipHostMallocNonCoherent));
    hm[2] = (uint8_t *)aligned_alloc(4096, 1 << 22);
    CK(hipHostRegister(hm[2], 1 << 22, hipHostRegisterMapped));
    const char *kind[3] = {"coherent", "noncoherent", "registered"};
    uint64_t *t;
    uint32_t *sink;
    CK(hipMalloc(&t, 16));
    CK(hipMalloc(&sink, 16));
    printf("{\"unit\": \"us, in-kernel first start to last end, median of 30\", \"rows\": [\n");
    bool first = true;
    for (int km = 0; km < 3; ++km) {
    uint8_t *h = hm[km], *hd;
    for (int i = 0; i < (1 << 22); ++i) h[i] = (uint8_t)(i * 31 + 7);
    CK(hipHostGetDevicePointer((void **)&hd, h, 0));
    for (uint64_t B : sizes) {
        for (int G : grids) {
            const uint64_t n16 = B / 16;
            if ((n16 + G - 1) / G > 256 * 32) continue;  // one load round per lane
            std::vector<double> us;
            for (int r = 0; r < 33; ++r) {
                const uint64_t init[2] = {~0ull, 0};
                CK(hipMemcpy(t, init, 16, hipMemcpyHostToDevice));
                hipLaunchKernelGGL(k_read, dim3(G), dim3(256), 0, 0, (const uint4 *)hd, n16, t, sink);
                CK(hipDeviceSynchronize());
                uint64_t o[2];
                CK(hipMemcpy(o, t, 16, hipMemcpyDeviceToHost));
                if (r >= 3) us.push_back((o[1] - o[0]) / 100.0);
            }
            std::sort(us.begin(), us.end());
            const double med = us[us.size() / 2];
            printf("%s{\"mem\": \"%s\", \"bytes\": %llu, \"wgs\": %d, \"us\": %.2f, \"GBps\": %.1f}", first ? "" : ",\n",
                   kind[km], (unsigned long long)B, G, med, B / med / 1e3);
            fflush(stdout);
            first = false;
        }
    }
    }
    printf("\n]}\n");
    return 0;
}
