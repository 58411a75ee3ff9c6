// copy_align_micro.hip — diagnostic: device copy bandwidth of 16-B-per-lane
// copies by source / destination alignment (the encode's frame copy moves each
// payload from an arbitrary SoA offset to an arbitrary frame offset).
// usage: ./copy_align_micro  -> one line per variant (GB/s = read + write bytes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct __attribute__((packed, aligned(1))) u128_ua { uint4 v; };

__global__ void k_copy(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, uint64_t n16) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = tid; i < n16; i += nth) {
        uint4 v = ((const u128_ua *)(src + 16 * i))->v;
        ((u128_ua *)(dst + 16 * i))->v = v;
    }
}

// destination-aligned: each lane loads its 16 B as two aligned-down pieces of
// the misaligned source and funnels them (v_alignbyte) before an aligned store
__global__ void k_copy_funnel(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, uint64_t n16, uint32_t r) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    const uint8_t *s4 = src - (r & 3);
    for (uint64_t i = tid; i < n16; i += nth) {
        const uint4 w = ((const u128_ua *)(s4 + 16 * i))->v;
        const uint32_t nx = *(const uint32_t *)(s4 + 16 * i + 16);
        const uint32_t q = r & 3;
        uint4 o = make_uint4(__builtin_amdgcn_alignbyte(w.y, w.x, q), __builtin_amdgcn_alignbyte(w.z, w.y, q),
                             __builtin_amdgcn_alignbyte(w.w, w.z, q), __builtin_amdgcn_alignbyte(nx, w.w, q));
        *(uint4 *)(dst + 16 * i) = o;
    }
}

int main() {
    const uint64_t bytes = 2ull << 30;
    uint8_t *a, *b;
    hipMalloc(&a, bytes + 4096);
    hipMalloc(&b, bytes + 4096);
    hipMemset(a, 1, bytes + 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const uint64_t n16 = bytes / 16;
    struct V { const char *name; uint32_t so, dof; int funnel; } vs[] = {
        {"aligned", 0, 0, 0}, {"src+5", 5, 0, 0}, {"dst+3", 0, 3, 0}, {"src+5,dst+3", 5, 3, 0},
        {"src+8,dst+8", 8, 8, 0}, {"src+4,dst+0", 4, 0, 0}, {"funnel src+5->dst aligned", 5, 0, 1}};
    for (int grid_mult : {4, 8, 16}) {
        for (const V &v : vs) {
            const int grid = ncu * grid_mult;
            float best = 1e9f;
            for (int it = 0; it < 6; ++it) {
                hipEventRecord(e0);
                if (v.funnel)
                    hipLaunchKernelGGL(k_copy_funnel, dim3(grid), dim3(256), 0, 0, a + v.so, b + v.dof, n16, v.so);
                else
                    hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a + v.so, b + v.dof, n16);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms = 0;
                hipEventElapsedTime(&ms, e0, e1);
                if (it > 0 && ms < best) best = ms;
            }
            printf("grid %2dx%d %-28s %.3f ms  %.0f GB/s (read+write)\n", grid_mult, ncu, v.name, best,
                   2.0 * bytes / best / 1e6);
        }
    }
    return 0;
}
