// HBM read-bandwidth calibration (diagnostic, not product): how fast can this
// box stream a ~1.1 GB device buffer with (a) coalesced global_load_dwordx4 into
// VGPRs, (b) 8 lanes x 16 B per frame-segment at a 1072-B stride (the
// lane-group frame layout), at several grid shapes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void rd_coalesced(const uint4 *__restrict__ p, uint64_t n16, uint64_t *out, int unroll) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t x = 0;
    for (; i + 7 * stride < n16; i += 8 * stride) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[i + k * stride];
#pragma unroll
        for (int k = 0; k < 8; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < n16; i += stride) { uint4 v = p[i]; x ^= v.x ^ v.y ^ v.z ^ v.w; }
    if (x == 0x12345678) out[0] = x;
}

// wave = 8 frame groups of 8 lanes; each lane loads 16 B at frame + 8 + 128 q + 16 (l%8).
// UNIT = frames a wave walks before jumping by nw*UNIT (8: 17 MB window, 64: 139 MB window)
template <int DEPTH, int UNIT = 8>
__global__ void rd_frames(const uint8_t *__restrict__ blob, uint64_t S, uint64_t N, uint64_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t gw = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t nseg = (uint32_t)((S - 8 + 127) / 128);
    uint32_t x = 0;
    for (uint64_t ff = 0; ff < N; ff += 8) {
        const uint64_t f0 = (ff / UNIT) * nw * UNIT + gw * UNIT + (ff % UNIT);
        if (f0 >= N) break;
        const uint64_t f = f0 + (lane >> 3);
        const uint8_t *base = blob + f * S + 8 + 16 * (lane & 7);
        const bool ok = f < N;
        for (uint32_t q = 0; q < nseg; q += DEPTH) {
            uint4 v[DEPTH];
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) {
                const uint64_t off = 128ull * (q + d);
                v[d] = (ok && q + d < nseg && off + 16 * (lane & 7) + 24 <= S)
                           ? *(const uint4 *)(base + off) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int d = 0; d < DEPTH; ++d) x ^= v[d].x ^ v[d].y ^ v[d].z ^ v[d].w;
        }
    }
    if (x == 0x12345678) out[0] = x;
}


// ---- LDS-DMA staging variants (no compute): 4 waves per WG, SLOTS x 10 x 1 KiB ring per wave
__device__ __forceinline__ void glds(const void *g, uint32_t lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 :: "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}
__device__ __forceinline__ void wvm(int n) {
    if (n >= 30) asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
    else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (n >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// MODE 0: segment pattern (lane group = frame, 8 frames x 128 B per instruction), 8 seg + 2 extra loads/step
// MODE 1: per-frame contiguous blocks (instruction k = frame k's 1 KiB), 8 + 1 loads/step
// UNIT: frames per wave-unit before jumping (64 or 8)
template <int MODE, int UNIT, int SLOTS>
__global__ __launch_bounds__(256, 1) void lds_frames(const uint8_t *__restrict__ blob, uint64_t S, uint64_t N, uint64_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t gw = (uint64_t)blockIdx.x * 4 + wave, nw = (uint64_t)gridDim.x * 4;
    const uint32_t ring = wave * SLOTS * 10240;
    const int l = lane & 7, fg = lane >> 3, m = l >> 1, par = l & 1;
    const uint32_t poff = 16 * (m + 4 * par);
    uint64_t issued = 0, done = 0;
    const uint64_t nsteps_total = (N + 7) / 8;  // groups
    // group sequence for this wave
    auto group_of = [&](uint64_t k) -> uint64_t {  // k-th group of this wave
        const uint64_t per = UNIT / 8;
        return (k / per) * nw * per + gw * per + (k % per);
    };
    auto issue = [&](uint64_t k) {
        const uint64_t grp = group_of(k);
        const uint32_t slot = ring + (uint32_t)(k % SLOTS) * 10240;
        if (MODE == 0) {
            const uint64_t f = grp * 8 + fg;
            const uint8_t *fb = blob + (f < N ? f : 0) * S;
            for (int q = 0; q < 8; ++q) glds(fb + 8 + 128 * q + poff, slot + 1024 * q);
            glds(fb + 8 + 1000 + 16 * m, slot + 8192);
            glds(fb, slot + 9216);
        } else {
            for (int k2 = 0; k2 < 8; ++k2) {
                const uint64_t f = grp * 8 + k2;
                const uint8_t *fb = blob + (f < N ? f : 0) * S;
                glds(fb + 8 + 16 * lane, slot + 1040 * k2);
            }
            const uint64_t f = grp * 8 + fg;
            const uint8_t *fb = blob + (f < N ? f : 0) * S;
            glds(l < 4 ? fb + 8 + 1000 + 16 * l : fb, slot + 8320);
        }
    };
    uint32_t x = 0;
    uint64_t mine = 0;
    while (group_of(mine) < nsteps_total) ++mine;
    for (; issued < SLOTS && issued < mine; ++issued) issue(issued);
    for (uint64_t k = 0; k < mine; ++k) {
        const int ahead = (int)(issued - 1 - k);
        wvm((MODE == 0 ? 10 : 9) * ahead >= 30 ? 30 : (MODE == 0 ? 10 : 9) * ahead >= 20 ? 20 : (MODE == 0 ? 10 : 9) * ahead >= 10 ? 10 : 0);
        const uint8_t *p = smem + ring + (k % SLOTS) * 10240 + 16 * lane;
        uint4 v = *(const uint4 *)p;
        x ^= v.x ^ v.w;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (issued < mine) { issue(issued); ++issued; }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (x == 0x12345678) out[0] = x;
}

// The C2 producers' order (decode_uniform.hip produce_lg), staging only: WG g of NP takes
// 128-frame blocks g, g + NP, ...; at step k its wave w loads unit k & 3 (32 frames) of
// block k >> 2, frame group w of it (frames 32 u - 6 + 8 w + fg), 9 loads per step, a
// SLOTS ring per wave and a constant vmcnt (SLOTS - 1 steps in flight).
// ORDER 1: the same blocks, but the chip's units in step order (unit-major: at step k all
// WGs read unit k & 3 of ONE window of NP blocks -- the product); ORDER 2: a contiguous
// window per step (WG g reads unit g & 3 of block 4 * (k div ... )): see issue()
template <int SLOTS, int ORDER>
__global__ __launch_bounds__(256, 1) void lds_blocks(const uint8_t *__restrict__ blob, uint64_t S, uint64_t N, uint64_t *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t ring = wave * SLOTS * 9216;
    const int l = lane & 7, fg = lane >> 3, m = l >> 1, par = l & 1;
    const uint32_t poff = 16 * (m + 4 * par);
    const uint64_t NP = gridDim.x, g = blockIdx.x;
    const uint64_t blocks = (N + 6 + 127) / 128;
    const uint64_t units = 4 * blocks;
    // unit of step k for this WG
    auto unit_of = [&](uint64_t k) -> uint64_t {
        if (ORDER == 1) return 4 * (g + NP * (k >> 2)) + (k & 3);
        // ORDER 2: at step k the NP WGs read NP consecutive units (a contiguous window);
        // WG g's unit sequence still covers whole blocks? no: staging-only bound
        return NP * k + g;
    };
    uint64_t mine = 0;
    while (unit_of(mine) < units) ++mine;
    auto issue = [&](uint64_t k) {
        const uint64_t u = unit_of(k);
        const int64_t i = (int64_t)(32 * u) - 6 + 8 * (int64_t)wave + fg;
        const bool valid = i >= 0 && (uint64_t)i < N;
        const uint8_t *fb = blob + (valid ? (uint64_t)i : 0) * S;
        const uint32_t slot = ring + (uint32_t)(k % SLOTS) * 9216;
        for (int q = 0; q < 8; ++q) glds(fb + 8 + 128 * q + poff, slot + 1024 * q);
        glds(!par ? fb + 8 + 1000 + 16 * m : (m == 1 ? fb + S : fb), slot + 8192);
    };
    uint32_t x = 0;
    uint64_t issued = 0;
    for (; issued < SLOTS && issued < mine; ++issued) issue(issued);
    for (uint64_t k = 0; k < mine; ++k) {
        if (issued - 1 - k >= (uint64_t)SLOTS - 1) {
            if (SLOTS == 4) asm volatile("s_waitcnt vmcnt(27)" ::: "memory");
            else if (SLOTS == 3) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint8_t *p = smem + ring + (k % SLOTS) * 9216 + 16 * lane;
        uint4 v = *(const uint4 *)p;
        x ^= v.x ^ v.w;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (issued < mine) { issue(issued); ++issued; }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
    hipMalloc(&d, L + 4096);
    hipMalloc(&o, 64);
    if (getenv("BW_RANDOM")) {  // random bytes (the product reads random payloads)
        hipLaunchKernelGGL(fill_random, 4096, 256, 0, 0, (uint64_t *)d, (L + 4096) / 8);
        hipDeviceSynchronize();
    } else {
        hipMemset(d, 0x5a, L + 4096);
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char *name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-40s %8.4f ms  %7.1f GB/s\n", name, ms, L / (ms * 1e-3) / 1e9);
    };
    char nm[128];
    if (getenv("BW_ORDER")) {  // the C2 producers' block order vs a contiguous window, staging only
        hipFuncSetAttribute((const void *)lds_blocks<4, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
        hipFuncSetAttribute((const void *)lds_blocks<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
        hipFuncSetAttribute((const void *)lds_blocks<3, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
        hipFuncSetAttribute((const void *)lds_frames<0, 8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
        for (int rep = 0; rep < 2; ++rep) {
            for (int np : {249, 255, 256}) {
                snprintf(nm, sizeof nm, "blocks(product order) 4slot np=%d", np);
                timeit(nm, [&] { hipLaunchKernelGGL((lds_blocks<4, 1>), np, 256, 4 * 4 * 9216, 0, d + 256, S, N, o); });
                snprintf(nm, sizeof nm, "blocks(product order) 3slot np=%d", np);
                timeit(nm, [&] { hipLaunchKernelGGL((lds_blocks<3, 1>), np, 256, 4 * 3 * 9216, 0, d + 256, S, N, o); });
                snprintf(nm, sizeof nm, "units(contiguous window) 4slot np=%d", np);
                timeit(nm, [&] { hipLaunchKernelGGL((lds_blocks<4, 2>), np, 256, 4 * 4 * 9216, 0, d + 256, S, N, o); });
            }
            timeit("ldsdma seg unit8 4slot (round 1)", [&] { hipLaunchKernelGGL((lds_frames<0, 8, 4>), 255, 256, 163840, 0, d + 256, S, N, o); });
        }
        return 0;
    }
    if (getenv("BW_MISALIGN")) {  // the same frame-segment reads with 16-B / 4-B / 1-B aligned frame starts
        for (uint64_t S2 : {1072ull, 1076ull, 1073ull}) {
            for (uint64_t base : {256ull, 257ull}) {
                const uint64_t N2 = (L - 512) / S2;
                snprintf(nm, sizeof nm, "frames d9 unit8 S=%llu base=%llu", (unsigned long long)S2,
                         (unsigned long long)base);
                timeit(nm, [&] { hipLaunchKernelGGL((rd_frames<9, 8>), 255, 512, 0, 0, d + base, S2, N2, o); });
            }
        }
        return 0;
    }
    hipFuncSetAttribute((const void *)lds_frames<0, 64, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    hipFuncSetAttribute((const void *)lds_frames<0, 8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    hipFuncSetAttribute((const void *)lds_frames<1, 64, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    hipFuncSetAttribute((const void *)lds_frames<1, 8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    hipFuncSetAttribute((const void *)lds_frames<0, 64, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    timeit("ldsdma seg unit64 4slot", [&] { hipLaunchKernelGGL((lds_frames<0, 64, 4>), 255, 256, 163840, 0, d + 256, S, N, o); });
    timeit("ldsdma seg unit8 4slot", [&] { hipLaunchKernelGGL((lds_frames<0, 8, 4>), 255, 256, 163840, 0, d + 256, S, N, o); });
    timeit("ldsdma contig unit64 4slot", [&] { hipLaunchKernelGGL((lds_frames<1, 64, 4>), 255, 256, 163840, 0, d + 256, S, N, o); });
    timeit("ldsdma contig unit8 4slot", [&] { hipLaunchKernelGGL((lds_frames<1, 8, 4>), 255, 256, 163840, 0, d + 256, S, N, o); });
    timeit("ldsdma seg unit64 3slot", [&] { hipLaunchKernelGGL((lds_frames<0, 64, 3>), 255, 256, 163840, 0, d + 256, S, N, o); });
    for (int blocks : {255}) {
        timeit("frames d9 unit64 grid=255 x 512", [&] { hipLaunchKernelGGL((rd_frames<9, 64>), 255, 512, 0, 0, d + 256, S, N, o); });
        timeit("frames d9 unit8 grid=255 x 512", [&] { hipLaunchKernelGGL((rd_frames<9, 8>), 255, 512, 0, 0, d + 256, S, N, o); });
        timeit("frames d4 unit64 grid=255 x 512", [&] { hipLaunchKernelGGL((rd_frames<4, 64>), 255, 512, 0, 0, d + 256, S, N, o); });
        timeit("frames d9 unit64 grid=255 x 1024", [&] { hipLaunchKernelGGL((rd_frames<9, 64>), 255, 1024, 0, 0, d + 256, S, N, o); });
    }
    for (int blocks : {256, 1024}) {
        for (int th : {256, 512}) {
            snprintf(nm, sizeof nm, "coalesced grid=%d x %d", blocks, th);
            timeit(nm, [&] { hipLaunchKernelGGL(rd_coalesced, blocks, th, 0, 0, (const uint4 *)d, L / 16, o, 8); });
        }
    }
    for (int blocks : {256, 1024}) {
        for (int th : {512}) {
            snprintf(nm, sizeof nm, "frames d4 grid=%d x %d", blocks, th);
            timeit(nm, [&] { hipLaunchKernelGGL(rd_frames<4>, blocks, th, 0, 0, d + 256, S, N, o); });
            snprintf(nm, sizeof nm, "frames d9 grid=%d x %d", blocks, th);
            timeit(nm, [&] { hipLaunchKernelGGL(rd_frames<9>, blocks, th, 0, 0, d + 256, S, N, o); });
        }
    }
    return 0;
}
