// Diagnostic only (scripts/mall_micro.py): is a chunk that a copy kernel has just
// written read back from the 256-MiB Infinity Cache, and at what rate, with and
// without XXH3-shaped arithmetic per 16-B piece? The question behind a copy-then-hash
// C3 encode. Not part of the codec.
// build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/_mall_micro.so scripts/mall_micro.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint64_t n16) {
    constexpr int U = 4;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + 256 * u < n16) v[u] = s[i + 256 * u];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + 256 * u < n16) d[i + 256 * u] = v[u];
    }
}

__device__ __forceinline__ uint64_t mul32x32(uint64_t x) { return (uint64_t)(uint32_t)x * (x >> 32); }

// H = 0: xor-reduce; H = 1: XXH3-stripe-shaped accumulate (two 32x32->64 products per 16 B)
template <int H>
__global__ __launch_bounds__(256) void k_read(const u32x4 *__restrict__ s, uint64_t n16, uint64_t *out) {
    constexpr int U = 8;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    uint64_t a0 = threadIdx.x, a1 = 0;
    const uint64_t s0 = 0x1cad21f72c81017cull ^ threadIdx.x, s1 = 0xdb979083e96dd4deull;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = (i + 256 * u < n16) ? s[i + 256 * u] : u32x4{0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t w0 = (uint64_t)v[u].x | ((uint64_t)v[u].y << 32);
            const uint64_t w1 = (uint64_t)v[u].z | ((uint64_t)v[u].w << 32);
            if (H) {
                a0 += mul32x32(w0 ^ s0) + w1;
                a1 += mul32x32(w1 ^ s1) + w0;
            } else {
                a0 ^= w0;
                a1 ^= w1;
            }
        }
    }
    if ((a0 ^ a1) == 0x123456789ull) out[0] = a0;  // keeps the loads
}

extern "C" int mm_copy(const void *src, void *dst, uint64_t nbytes, int wgs, hipStream_t st) {
    hipLaunchKernelGGL(k_copy, dim3(wgs), dim3(256), 0, st, (const u32x4 *)src, (u32x4 *)dst, nbytes / 16);
    return (int)hipGetLastError();
}
extern "C" int mm_read(const void *src, uint64_t nbytes, int hash, int wgs, void *out, hipStream_t st) {
    if (hash)
        hipLaunchKernelGGL(k_read<1>, dim3(wgs), dim3(256), 0, st, (const u32x4 *)src, nbytes / 16, (uint64_t *)out);
    else
        hipLaunchKernelGGL(k_read<0>, dim3(wgs), dim3(256), 0, st, (const u32x4 *)src, nbytes / 16, (uint64_t *)out);
    return (int)hipGetLastError();
}
