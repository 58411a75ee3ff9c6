// Diagnostic only (scripts/copy_bound.py): plain device copies at the C3 encode's
// size, the read-once / write-once bound for DESIGN §4.4. Not part of the codec.
// build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o scripts/_copy_kernel.so scripts/copy_kernel.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// variant 0: 16-B loads and stores, U per thread per round, grid-stride
// variant 1: the same with nontemporal stores
// variant 2: destination shifted by one byte (unaligned 16-B stores, like the encode's frames)
template <int V, int U>
__global__ __launch_bounds__(256) void k_copy(const u32x4 *__restrict__ s, uint8_t *__restrict__ d, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + 256 * u < n16) v[u] = s[i + 256 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (i + 256 * u >= n16) break;
            if (V == 0) ((u32x4 *)d)[i + 256 * u] = v[u];
            if (V == 1) __builtin_nontemporal_store(v[u], (u32x4 *)d + i + 256 * u);
            if (V == 2) *(u32x4 *)(d + 1 + 16 * (i + 256 * u)) = v[u];
        }
    }
}

extern "C" int copy_launch(const void *src, void *dst, uint64_t nbytes, int variant, int wgs, hipStream_t st) {
    const uint64_t n16 = nbytes / 16;
    if (variant == 0) hipLaunchKernelGGL((k_copy<0, 4>), dim3(wgs), dim3(256), 0, st, (const u32x4 *)src, (uint8_t *)dst, n16);
    else if (variant == 1) hipLaunchKernelGGL((k_copy<1, 4>), dim3(wgs), dim3(256), 0, st, (const u32x4 *)src, (uint8_t *)dst, n16);
    else if (variant == 2) hipLaunchKernelGGL((k_copy<2, 4>), dim3(wgs), dim3(256), 0, st, (const u32x4 *)src, (uint8_t *)dst, n16);
    else return -1;
    return (int)hipGetLastError();
}
