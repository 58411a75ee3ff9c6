// Diagnostic (not product): the lane-group decode step in isolation -- LDS-DMA
// staging of 8 frames x (8 x 128 B + last stripe + stored checksum) per step,
// with (HASH=1) or without the per-frame XXH3 -- to price hashing and traversal
// against scripts/bw_micro.hip's pure streaming rates. Reads a C2-shaped record
// (argv[1], or random bytes: then the mismatch count is just every frame).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../iggy_amd/csrc/codec_common.hpp"
using namespace iggy;

__device__ __forceinline__ void glds(const void *g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}
template <int N> __device__ __forceinline__ void wvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int C> __device__ __forceinline__ uint64_t dpp64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, C, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), C, 0xF, 0xF, false);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint64_t swz4(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)x, 0x101F);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(x >> 32), 0x101F);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ void piece(uint64_t &a0, uint64_t &a1, uint4 p, uint64_t s0, uint64_t s1) {
    const uint64_t w0 = (uint64_t)p.x | ((uint64_t)p.y << 32), w1 = (uint64_t)p.z | ((uint64_t)p.w << 32);
    a0 += mul32x32(w0 ^ s0) + w1;
    a1 += mul32x32(w1 ^ s1) + w0;
}

// groups of 8 frames; wave's k-th group = (k / per) * nw * per + gw * per + k % per
template <int UNIT, int SLOTS, int HASH, int PUB = 0, int POLL = 0>
__global__ __launch_bounds__(256, 1) void lg_hash(const uint8_t *__restrict__ blob, uint64_t S, uint64_t N,
                                                  uint64_t *out, uint64_t *pubbuf = nullptr) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *exited = (uint32_t *)(out + 4);
    if (POLL) {
        if (blockIdx.x == 0) {  // the product's consumer WG: wave 0 waits for every producer wave
            if (wave == 0) {
                // POLL 1: sc1 load + s_sleep 4 + s_memrealtime bound (the product's form)
                // POLL 2: sc1 load + s_sleep 4, iteration-count bound
                // POLL 3: s_memrealtime only in the loop, no memory poll (exits on a fixed time)
                // POLL 4: sc1 load + s_sleep 127, iteration-count bound
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                uint64_t it = 0;
                while (true) {
                    if (POLL != 3 &&
                        __hip_atomic_load(exited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 4 * (gridDim.x - 1))
                        break;
                    if (POLL == 4) __builtin_amdgcn_s_sleep(127); else __builtin_amdgcn_s_sleep(4);
                    if (POLL == 1 || POLL == 3) {
                        if (__builtin_amdgcn_s_memrealtime() - t0 > (POLL == 3 ? 17000ull : 400000000ull)) break;
                    } else if (++it > 200000ull) break;
                }
                if (POLL != 3 && lane == 0)
                    __hip_atomic_fetch_sub(exited, 4 * (gridDim.x - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }
    }
    const uint64_t gw = (uint64_t)(blockIdx.x - (POLL ? 1 : 0)) * 4 + wave,
                   nw = (uint64_t)(gridDim.x - (POLL ? 1 : 0)) * 4;
    const uint32_t ring = wave * SLOTS * 10240;
    const uint32_t l = lane & 7, fg = lane >> 3, m = l >> 1, par = l & 1;
    const uint32_t poff = 16 * (m + 4 * par);
    const uint64_t L = S - 8;
    uint64_t s0[8], s1[8];
    for (int q = 0; q < 8; ++q) { s0[q] = kSecretW8[2 * q + par + 2 * m]; s1[q] = kSecretW8[2 * q + par + 2 * m + 1]; }
    const uint64_t key0 = kSecretW8[16 + 2 * m], key1 = kSecretW8[17 + 2 * m];
    const uint64_t init0 = par ? 0 : kAccInit[2 * m], init1 = par ? 0 : kAccInit[2 * m + 1];
    const uint64_t last0 = kSecretLast[2 * m], last1 = kSecretLast[2 * m + 1];
    const uint64_t mrg0 = kSecretMerge[2 * m], mrg1 = kSecretMerge[2 * m + 1];
    const uint64_t ngroups = (N + 7) / 8;
    constexpr uint64_t per = UNIT / 8;
    auto group_of = [&](uint64_t k) -> uint64_t { return (k / per) * nw * per + gw * per + (k % per); };
    uint64_t mine = 0;
    while (group_of(mine) < ngroups) ++mine;
    auto issue = [&](uint64_t k) {
        const uint64_t f = group_of(k) * 8 + fg;
        const uint8_t *fb = blob + (f < N ? f : 0) * S;
        const uint32_t slot = ring + (uint32_t)(k % SLOTS) * 10240;
        for (int q = 0; q < 8; ++q) glds(fb + 8 + 128 * q + poff, slot + 1024 * q);
        glds(fb + 8 + L - 64 + 16 * m, slot + 8192);
        glds(fb, slot + 9216);
    };
    uint32_t x = 0;
    uint64_t bad = 0;
    for (uint64_t k = 0; k < SLOTS && k < mine; ++k) issue(k);
    for (uint64_t k = 0; k < mine; ++k) {
        // PUB: every 8th step publishes like the product (5 store instructions);
        // PUB == 2 widens the following waits by those 5 younger stores
        if (k + SLOTS <= mine) {
            if (PUB == 2 && (k & 7) >= 1 && (k & 7) <= SLOTS) wvm<10 * (SLOTS - 1) + 5>();
            else wvm<10 * (SLOTS - 1)>();
        } else wvm<0>();
        const uint8_t *p = smem + ring + (k % SLOTS) * 10240 + 16 * lane;
        uint4 v[8];
        for (int q = 0; q < 8; ++q) v[q] = *(const uint4 *)(p + 1024 * q);
        const uint4 lastp = *(const uint4 *)(p + 8192);
        const uint64_t stored = *(const uint64_t *)(p + 9216);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (k + SLOTS < mine) issue(k + SLOTS);
        if (HASH) {
            uint64_t a0 = init0, a1 = init1, p0[4] = {0, 0, 0, 0}, p1[4] = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < 8; ++q) piece(p0[q & 3], p1[q & 3], v[q], s0[q], s1[q]);
            a0 += (p0[0] + p0[1]) + (p0[2] + p0[3]);
            a1 += (p1[0] + p1[1]) + (p1[2] + p1[3]);
            a0 += dpp64<0xB1>(a0); a1 += dpp64<0xB1>(a1);
            a0 = scramble1(a0, key0); a1 = scramble1(a1, key1);
            if (par) { a0 = 0; a1 = 0; }
            a0 += dpp64<0xB1>(a0); a1 += dpp64<0xB1>(a1);
            piece(a0, a1, lastp, last0, last1);
            uint64_t t = fold64(a0 ^ mrg0, a1 ^ mrg1);
            t += dpp64<0x4E>(t);
            t += swz4(t);
            const uint64_t h = avalanche(L * P64_1 + t);
            const uint64_t f = group_of(k) * 8 + fg;
            bad += (f < N && h != stored && l == 0) ? 1 : 0;
            if (PUB && (k & 7) == 0) {
                uint64_t *pb = pubbuf + (gw * 64 + (k >> 3)) * 64;
                if (lane < 8) {
                    __hip_atomic_store(pb + 2 * lane, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(pb + 2 * lane + 1, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                if (lane == 0) __hip_atomic_store(pb + 16, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 63) __hip_atomic_store(pb + 17, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                pb[20 + lane] = h;
            }
        } else {
            for (int q = 0; q < 8; ++q) x ^= v[q].x ^ v[q].w;
            x ^= lastp.y ^ (uint32_t)stored;
        }
    }
    wvm<0>();
    if (POLL && POLL != 3 && lane == 0) __hip_atomic_fetch_add(exited, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (x == 0x12345678 || bad) atomicAdd((unsigned long long *)out, (unsigned long long)(bad + (x == 0x12345678)));
}

int main(int argc, char **argv) {
    const uint64_t N = 1 << 20, S = 1072, L = 256 + N * S;
    std::vector<uint8_t> h(L);
    FILE *f = argc > 1 ? fopen(argv[1], "rb") : nullptr;
    if (f) {
        if (fread(h.data(), 1, L, f) != L) { printf("short read\n"); return 1; }
        fclose(f);
    } else {
        uint64_t z = 1;
        for (uint64_t i = 0; i < L; ++i) { z = z * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint8_t)(z >> 56); }
    }
    uint8_t *d;
    uint64_t *o;
    (void)hipMalloc(&d, L + 4096);
    (void)hipMalloc(&o, 64);
    (void)hipMemcpy(d, h.data(), L, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        (void)hipDeviceSynchronize();
        (void)hipMemset(o, 0, 64);
        (void)hipEventRecord(e0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        uint64_t bad = 0;
        (void)hipMemcpy(&bad, o, 8, hipMemcpyDeviceToHost);
        fflush(stdout); printf("%-28s %8.4f ms  %7.1f GB/s  mismatches/rep=%lu\n", name, ms, L / (ms * 1e-3) / 1e9,
               (unsigned long)(bad / reps));
    };
#define RUN(U, SL, H)                                                                                          \
    (void)hipFuncSetAttribute((const void *)lg_hash<U, SL, H>, hipFuncAttributeMaxDynamicSharedMemorySize,    \
                              163840);                                                                         \
    timeit("unit" #U " slots" #SL " hash" #H,                                                                  \
           [&] { hipLaunchKernelGGL((lg_hash<U, SL, H>), 255, 256, 163840, 0, d + 256, S, N, o); });
    uint64_t *pub;
    (void)hipMalloc(&pub, 1020ull * 64 * 64 * 8);
#define RUNP(U, SL, P)                                                                                         \
    (void)hipFuncSetAttribute((const void *)lg_hash<U, SL, 1, P>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              163840);                                                                         \
    timeit("unit" #U " slots" #SL " hash1 pub" #P,                                                            \
           [&] { hipLaunchKernelGGL((lg_hash<U, SL, 1, P>), 255, 256, 163840, 0, d + 256, S, N, o, pub); });
#define RUNQ(U, SL, Q, G)                                                                                      \
    (void)hipFuncSetAttribute((const void *)lg_hash<U, SL, 0, 0, Q>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                              163840);                                                                         \
    timeit("unit" #U " slots" #SL " hash0 poll" #Q " grid" #G,                                                 \
           [&] { hipLaunchKernelGGL((lg_hash<U, SL, 0, 0, Q>), G, 256, 163840, 0, d + 256, S, N, o, pub); });
    (void)hipMemset(o, 0, 64);
    for (int rep = 0; rep < 2; ++rep) {
        RUN(8, 4, 0) RUN(8, 4, 1) RUN(64, 4, 0) RUN(64, 4, 1) RUN(8, 3, 1) RUN(16, 4, 1)
        RUNP(64, 4, 1) RUNP(64, 4, 2) RUNP(8, 3, 1) RUNP(8, 3, 2)
        RUNQ(64, 4, 0, 256) RUNQ(64, 4, 1, 256) RUNQ(64, 4, 2, 256) RUNQ(64, 4, 3, 256) RUNQ(64, 4, 4, 256)
    }
    return 0;
}
