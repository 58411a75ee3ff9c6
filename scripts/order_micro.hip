// Diagnostic (not product): the uniform decode's LDS-DMA load shape (8 lanes per
// frame, 8 frames per wave-instruction, 16 B per lane, explicit vmcnt ring) with
// no compute, under several frame -> (wave, step) orders and step sizes, on the
// C2 record shape (1 M frames of 1072 B). Answers: does the order in which the
// 1020 producer waves sweep the record change the streaming rate, and what do a
// 9-load step (stored checksum folded into the last-stripe load) and a 3-slot
// ring cost?
//   ORDER 0 "unit64"   : wave gw owns 64-frame units gw, gw+nw, ... (the product)
//   ORDER 1 "chunk-il" : WG g owns 256-frame chunks g, g+nWG, ...; its 4 waves
//                        interleave over the chunk's 32 groups (4 consecutive
//                        groups per step per WG)
//   ORDER 2 "unit8"    : group k*nw + gw (one contiguous front for the chip)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

template <bool NT>
__device__ __forceinline__ void glds(const void *g, uint32_t lds) {
    if (NT)
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt"
                     :: "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                     :: "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void wvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int ORDER, int LOADS, int SLOTS, bool NT = false>
__global__ __launch_bounds__(256, 1) void k_order(const uint8_t *__restrict__ blob, uint64_t S, uint64_t N,
                                                  uint64_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nwg = gridDim.x, g = blockIdx.x;
    const uint64_t gw = g * 4 + wave, nw = nwg * 4;
    constexpr uint32_t kStep = LOADS * 1024;
    const uint32_t ring = wave * SLOTS * kStep;
    const int l = lane & 7, fg = lane >> 3, m = l >> 1, par = l & 1;
    const uint32_t poff = 16 * (m + 4 * par);
    const uint64_t ngroups = (N + 7) / 8;
    auto group_of = [&](uint64_t k) -> uint64_t {
        if (ORDER == 0) return (gw + (k / 8) * nw) * 8 + (k % 8);
        if (ORDER == 1) return (g + (k / 8) * nwg) * 32 + (k % 8) * 4 + wave;
        if (ORDER == 3) return (g + (k / 4) * nwg) * 16 + (k % 4) * 4 + wave;  // 128-frame blocks per WG
        return k * nw + gw;
    };
    uint64_t mine = 0;
    while (group_of(mine) < ngroups) ++mine;  // (all orders visit groups in increasing k)
    auto issue = [&](uint64_t k) {
        const uint64_t f = group_of(k) * 8 + fg;
        const uint8_t *fb = blob + (f < N ? f : 0) * S;
        const uint32_t slot = ring + (uint32_t)(k % SLOTS) * kStep;
#pragma unroll
        for (int q = 0; q < 8; ++q) glds<NT>(fb + 8 + 128 * q + poff, slot + 1024 * q);
        if (LOADS == 10) {
            glds<NT>(fb + 8 + 1000 + 16 * m, slot + 8192);
            glds<NT>(fb, slot + 9216);
        } else {  // 9 loads: even lanes the last-stripe piece, odd lanes the stored checksum
            glds<NT>(par ? fb : fb + 8 + 1000 + 16 * m, slot + 8192);
        }
    };
    uint32_t x = 0;
    uint64_t issued = 0;
    for (; issued < SLOTS && issued < mine; ++issued) issue(issued);
    for (uint64_t k = 0; k < mine; ++k) {
        if (k + SLOTS <= mine) wvm<LOADS * (SLOTS - 1)>();
        else wvm<0>();
        const uint8_t *p = smem + ring + (k % SLOTS) * kStep + 16 * lane;
        uint4 v = *(const uint4 *)p;
        x ^= v.x ^ v.w;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (issued < mine) { issue(issued); ++issued; }
    }
    wvm<0>();
    if (x == 0x12345678) out[0] = x;
}

__global__ void fill_random(uint64_t *p, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull + 0x1234567;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main() {
    const uint64_t N = 1 << 20, S = 1072, L = 256 + N * S;
    uint8_t *d;
    uint64_t *o;
    if (hipMalloc(&d, L + 4096) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    hipLaunchKernelGGL(fill_random, 4096, 256, 0, 0, (uint64_t *)d, (L + 4096) / 8);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, const void *fn, uint32_t lds) {
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        const uint8_t *b = d + 256;
        uint64_t s_ = S, n_ = N;
        void *args[] = {(void *)&b, (void *)&s_, (void *)&n_, (void *)&o};
        for (int w = 0; w < 3; ++w) hipLaunchKernel(fn, dim3(255), dim3(256), args, lds, 0);
        hipDeviceSynchronize();
        const int reps = 20;
        float best = 1e9, sum = 0;
        for (int r = 0; r < reps; ++r) {
            hipEventRecord(e0);
            hipLaunchKernel(fn, dim3(255), dim3(256), args, lds, 0);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("%-34s avg %.4f ms (%.1f GB/s)  best %.4f ms (%.1f GB/s)\n", name, sum / reps,
               L / (sum / reps * 1e-3) / 1e9, best, L / (best * 1e-3) / 1e9);
    };
    for (int rep = 0; rep < 2; ++rep) {
        timeit("unit8     9 loads 4 slots", (const void *)k_order<2, 9, 4>, 4 * 4 * 9216);
        timeit("block128  9 loads 4 slots", (const void *)k_order<3, 9, 4>, 4 * 4 * 9216);
        timeit("unit8     9 loads 4 slots nt", (const void *)k_order<2, 9, 4, true>, 4 * 4 * 9216);
        timeit("block128  9 loads 4 slots nt", (const void *)k_order<3, 9, 4, true>, 4 * 4 * 9216);
        timeit("block128  9 loads 3 slots nt", (const void *)k_order<3, 9, 3, true>, 4 * 3 * 9216);
        timeit("unit64   10 loads 4 slots", (const void *)k_order<0, 10, 4>, 4 * 4 * 10240);
    }
    return 0;
}
