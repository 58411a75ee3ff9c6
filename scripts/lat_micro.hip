// Dependent-latency micro-benchmark of the VALU instructions on the batch-checksum
// chain's critical path (diagnostic, not product). One wave; each kernel runs a loop of
// 16 dependent instructions of one kind; ns per instruction from HIP events.
// Also whole chain-step variants (hand-written asm) checked against a host reference.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <vector>

constexpr uint32_t P = 0x9E3779B1u;
constexpr int kIters = 4096;

#define REP16(x) x x x x x x x x x x x x x x x x

__global__ void l_add_u32(uint32_t *out, uint32_t a) {
    uint32_t v = threadIdx.x;
    for (int i = 0; i < kIters; ++i) asm volatile(REP16("v_add_u32 %0, %0, %1\n\t") : "+v"(v) : "v"(a));
    out[threadIdx.x] = v;
}
__global__ void l_xor(uint32_t *out, uint32_t a) {
    uint32_t v = threadIdx.x;
    for (int i = 0; i < kIters; ++i) asm volatile(REP16("v_xor_b32 %0, %0, %1\n\t") : "+v"(v) : "v"(a));
    out[threadIdx.x] = v;
}
__global__ void l_mul_lo(uint32_t *out, uint32_t a) {
    uint32_t v = threadIdx.x;
    for (int i = 0; i < kIters; ++i) asm volatile(REP16("v_mul_lo_u32 %0, %0, %1\n\t") : "+v"(v) : "v"(a));
    out[threadIdx.x] = v;
}
__global__ void l_mul_u24(uint32_t *out, uint32_t a) {
    uint32_t v = threadIdx.x;
    for (int i = 0; i < kIters; ++i) asm volatile(REP16("v_mul_u32_u24 %0, %0, %1\n\t") : "+v"(v) : "v"(a));
    out[threadIdx.x] = v;
}
__global__ void l_mul_hi(uint32_t *out, uint32_t a) {
    uint32_t v = threadIdx.x;
    for (int i = 0; i < kIters; ++i) asm volatile(REP16("v_mul_hi_u32 %0, %0, %1\n\t") : "+v"(v) : "v"(a));
    out[threadIdx.x] = v;
}
__global__ void l_lshl_add_u64(uint64_t *out, uint64_t a) {
    uint64_t v = threadIdx.x;
    for (int i = 0; i < kIters; ++i) asm volatile(REP16("v_lshl_add_u64 %0, %0, 0, %1\n\t") : "+v"(v) : "v"(a));
    out[threadIdx.x] = v;
}
__global__ void l_add_co(uint64_t *out, uint64_t a) {  // 64-bit add as add_co + addc
    uint32_t lo = threadIdx.x, hi = 0;
    const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32);
    for (int i = 0; i < kIters; ++i)
        asm volatile(REP16("v_add_co_u32 %0, s[20:21], %0, %2\n\tv_addc_co_u32 %1, s[20:21], %1, %3, s[20:21]\n\t")
                     : "+v"(lo), "+v"(hi) : "v"(alo), "v"(ahi) : "s20", "s21");
    out[threadIdx.x] = ((uint64_t)hi << 32) | lo;
}
// mad_u64_u32 chained through its 32-bit source (the lo path of a chain step)
__global__ void l_mad_src(uint64_t *out, uint64_t a) {
    uint64_t v = threadIdx.x;
    for (int i = 0; i < kIters; ++i)
        asm volatile("v_lshl_add_u64 v[50:51], %0, 0, 0\n\t" REP16("v_mad_u64_u32 v[50:51], s[20:21], v50, %1, %2\n\t")
                     "v_lshl_add_u64 %0, v[50:51], 0, 0\n\t"
                     : "+v"(v) : "v"(P), "v"(a) : "s20", "s21", "v50", "v51");
    out[threadIdx.x] = v;
}
// mad_u64_u32 chained through its 64-bit addend
__global__ void l_mad_add(uint64_t *out, uint64_t a) {
    uint64_t v = threadIdx.x;
    const uint32_t x = (uint32_t)a;
    for (int i = 0; i < kIters; ++i)
        asm volatile(REP16("v_mad_u64_u32 %0, s[20:21], %1, %2, %0\n\t") : "+v"(v) : "v"(x), "v"(P) : "s20", "s21");
    out[threadIdx.x] = v;
}

// ---- whole chain steps over nb blocks of sums (8 chains, lanes 0..7 meaningful)
// current product form (decode_uniform.hip chain_step, as compiled)
__global__ void c_v1(const uint64_t *sums, uint64_t nb, const uint64_t *keys, uint64_t *out) {
    const int j = threadIdx.x & 7;
    const uint64_t key = keys[j];
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    uint64_t y = 0x1234 + j + sums[j];
    for (uint64_t b = 0; b < nb; b += 8) {
        uint64_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = (b + k + 1 < nb) ? sums[(b + k + 1) * 8 + j] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t hi = (uint32_t)(y >> 32);
            const uint32_t lo = (uint32_t)y ^ (hi >> 15) ^ klo;
            const uint32_t h2 = hi ^ khi;
            uint64_t t = (uint64_t)lo * P + ((uint64_t)(h2 * P) << 32);
            asm volatile("" : "+v"(t));
            y = t + v[k];
        }
    }
    out[threadIdx.x] = y;
}
// split, asm: mad(lo', P, s) then hi += (h ^ khi) * P
#define SPLIT(VK)                                       \
    "v_lshrrev_b32 v42, 15, v41\n\t"                    \
    "v_xor_b32 v43, %2, v41\n\t"                        \
    "v_bitop3_b32 v42, v40, v42, %1 bitop3:0x96\n\t"    \
    "v_mul_lo_u32 v43, v43, %3\n\t"                     \
    "v_mad_u64_u32 v[40:41], s[20:21], v42, %3, " VK "\n\t" \
    "v_add_u32 v41, v41, v43\n\t"
// split with 24-bit multiplies for the hi product
#define SPLIT24(VK)                                     \
    "v_xor_b32 v43, %2, v41\n\t"                        \
    "v_lshrrev_b32 v42, 15, v41\n\t"                    \
    "v_and_b32 v44, 0xffff, v43\n\t"                    \
    "v_lshrrev_b32 v45, 16, v43\n\t"                    \
    "v_bitop3_b32 v42, v40, v42, %1 bitop3:0x96\n\t"    \
    "v_mul_u32_u24 v46, v44, %4\n\t"                    \
    "v_mul_u32_u24 v44, v44, %5\n\t"                    \
    "v_mul_u32_u24 v45, v45, %4\n\t"                    \
    "v_mad_u64_u32 v[40:41], s[20:21], v42, %3, " VK "\n\t" \
    "v_add_u32 v44, v44, v45\n\t"                       \
    "v_lshl_add_u32 v43, v44, 16, v46\n\t"              \
    "v_add_u32 v41, v41, v43\n\t"
#define CHAIN_KERNEL(NAME, STEP, EXTRA_IN, EXTRA_CLOB)                                                        \
    __global__ void NAME(const uint64_t *sums, uint64_t nb, const uint64_t *keys, uint64_t *out) {           \
        const int j = threadIdx.x & 7;                                                                         \
        const uint64_t key = keys[j];                                                                          \
        const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);                                     \
        const uint32_t pl = P & 0xffff, ph = P >> 16;                                                          \
        uint64_t y = 0x1234 + j + sums[j];                                                                     \
        for (uint64_t b = 0; b < nb; b += 8) {                                                                 \
            uint64_t v[8];                                                                                     \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) v[k] = (b + k + 1 < nb) ? sums[(b + k + 1) * 8 + j] : 0; \
            asm volatile("v_lshl_add_u64 v[40:41], %0, 0, 0\n\t" STEP("%6") STEP("%7") STEP("%8") STEP("%9")     \
                         STEP("%10") STEP("%11") STEP("%12") STEP("%13") "v_lshl_add_u64 %0, v[40:41], 0, 0\n\t" \
                         : "+v"(y)                                                                             \
                         : "v"(klo), "v"(khi), "v"(P), "v"(pl), "v"(ph), "v"(v[0]), "v"(v[1]), "v"(v[2]),      \
                           "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7])                               \
                         : "s20", "s21", "v40", "v41", "v42", "v43", "v44", "v45", "v46");                     \
        }                                                                                                      \
        out[threadIdx.x] = y;                                                                                  \
    }
CHAIN_KERNEL(c_split, SPLIT, , )
CHAIN_KERNEL(c_split24, SPLIT24, , )


// ---- chain steps fed from registers (16 sums cycled: the step's own latency, no load)
__device__ __forceinline__ uint64_t regsum(int k, int j) { return 0x9E3779B97F4A7C15ull * (uint64_t)(16 * j + k + 1); }
__global__ void r_v1(uint64_t nb, const uint64_t *keys, uint64_t *out) {
    const int j = threadIdx.x & 7;
    const uint64_t key = keys[j];
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    uint64_t v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { v[k] = regsum(k, j); asm volatile("" : "+v"(v[k])); }
    uint64_t y = 0x1234 + j + v[0];
    for (uint64_t b = 0; b < nb; b += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t hi = (uint32_t)(y >> 32);
            const uint32_t lo = (uint32_t)y ^ (hi >> 15) ^ klo;
            const uint32_t h2 = hi ^ khi;
            uint64_t t = (uint64_t)lo * P + ((uint64_t)(h2 * P) << 32);
            asm volatile("" : "+v"(t));
            y = t + v[(k + 1) & 15];
        }
    }
    out[threadIdx.x] = y;
}
#define RCHAIN_KERNEL(NAME, STEP)                                                                              \
    __global__ void NAME(uint64_t nb, const uint64_t *keys, uint64_t *out) {                                   \
        const int j = threadIdx.x & 7;                                                                         \
        const uint64_t key = keys[j];                                                                          \
        const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);                                     \
        const uint32_t pl = P & 0xffff, ph = P >> 16;                                                          \
        uint64_t v[16];                                                                                        \
        _Pragma("unroll") for (int k = 0; k < 16; ++k) { v[k] = regsum(k, j); asm volatile("" : "+v"(v[k])); } \
        uint64_t y = 0x1234 + j + v[0];                                                                        \
        for (uint64_t b = 0; b < nb; b += 16) {                                                                \
            asm volatile("v_lshl_add_u64 v[40:41], %0, 0, 0\n\t" STEP("%7") STEP("%8") STEP("%9") STEP("%10") \
                         STEP("%11") STEP("%12") STEP("%13") STEP("%14") STEP("%15") STEP("%16") STEP("%17")   \
                         STEP("%18") STEP("%19") STEP("%20") STEP("%21") STEP("%6")                            \
                         "v_lshl_add_u64 %0, v[40:41], 0, 0\n\t"                                               \
                         : "+v"(y)                                                                             \
                         : "v"(klo), "v"(khi), "v"(P), "v"(pl), "v"(ph), "v"(v[0]), "v"(v[1]), "v"(v[2]),      \
                           "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "v"(v[8]), "v"(v[9]),        \
                           "v"(v[10]), "v"(v[11]), "v"(v[12]), "v"(v[13]), "v"(v[14]), "v"(v[15])              \
                         : "s20", "s21", "v40", "v41", "v42", "v43", "v44", "v45", "v46");                     \
        }                                                                                                      \
        out[threadIdx.x] = y;                                                                                  \
    }
// the product form as the compiler emits it: y = mad(lo', P, {0, h2 * P}) + s
#define V1ASM(VK)                                       \
    "v_lshrrev_b32 v42, 15, v41\n\t"                    \
    "v_xor_b32 v43, v41, %2\n\t"                        \
    "v_bitop3_b32 v42, v40, v42, %1 bitop3:0x96\n\t"    \
    "v_mul_lo_u32 v45, v43, %3\n\t"                     \
    "v_mov_b32 v44, 0\n\t"                              \
    "v_mad_u64_u32 v[40:41], s[20:21], v42, %3, v[44:45]\n\t" \
    "v_lshl_add_u64 v[40:41], v[40:41], 0, " VK "\n\t"
RCHAIN_KERNEL(r_split, SPLIT)
RCHAIN_KERNEL(r_split24, SPLIT24)
RCHAIN_KERNEL(r_v1asm, V1ASM)
static uint64_t host_ref_reg(uint64_t nb, const uint64_t *keys, int j) {
    uint64_t acc = 0x1234 + j;
    for (uint64_t b = 0; b < nb; ++b) {
        uint64_t x = acc + 0x9E3779B97F4A7C15ull * (uint64_t)(16 * j + (b & 15) + 1);
        x ^= x >> 47;
        x ^= keys[j];
        acc = x * P;
    }
    return acc + 0x9E3779B97F4A7C15ull * (uint64_t)(16 * j + 1);  // y after the last step adds v[0] again
}

static uint64_t host_ref(const std::vector<uint64_t> &s, uint64_t nb, const uint64_t *keys, int j) {
    uint64_t acc = 0x1234 + j;
    for (uint64_t b = 0; b < nb; ++b) {
        uint64_t x = acc + s[b * 8 + j];
        x ^= x >> 47;
        x ^= keys[j];
        acc = x * P;
    }
    return acc;
}

template <class K, class... A>
static float timeit(K k, A... a) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, 1, 64, 0, 0, a...);
    hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL(k, 1, 64, 0, 0, a...);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    uint64_t *d64;
    hipMalloc(&d64, 4096);
    const double ninst = (double)kIters * 16;
    struct { const char *n; float ms; } r[] = {
        {"v_add_u32", timeit(l_add_u32, (uint32_t *)d64, 3u)},
        {"v_xor_b32", timeit(l_xor, (uint32_t *)d64, 3u)},
        {"v_mul_lo_u32", timeit(l_mul_lo, (uint32_t *)d64, 3u)},
        {"v_mul_u32_u24", timeit(l_mul_u24, (uint32_t *)d64, 3u)},
        {"v_mul_hi_u32", timeit(l_mul_hi, (uint32_t *)d64, 3u)},
        {"v_lshl_add_u64", timeit(l_lshl_add_u64, d64, (uint64_t)3)},
        {"v_add_co+addc (pair)", timeit(l_add_co, d64, (uint64_t)3)},
        {"v_mad_u64_u32 via src", timeit(l_mad_src, d64, (uint64_t)3)},
        {"v_mad_u64_u32 via addend", timeit(l_mad_add, d64, (uint64_t)3)},
    };
    for (auto &x : r) printf("%-28s %.3f ns per dependent instruction\n", x.n, x.ms * 1e6 / ninst);

    const uint64_t nb = 8192;
    std::vector<uint64_t> hs(nb * 8);
    uint64_t q = 1;
    for (auto &v : hs) { q = q * 6364136223846793005ull + 1442695040888963407ull; v = q; }
    uint64_t keys[8];
    for (int j = 0; j < 8; ++j) keys[j] = 0xA5A5A5A5DEADBEEFull * (j + 3);
    uint64_t *ds, *dk, *dout;
    hipMalloc(&ds, hs.size() * 8);
    hipMalloc(&dk, 64);
    hipMalloc(&dout, 512);
    hipMemcpy(ds, hs.data(), hs.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dk, keys, 64, hipMemcpyHostToDevice);
    struct { const char *n; void (*k)(const uint64_t *, uint64_t, const uint64_t *, uint64_t *); } cs[] = {
        {"chain v1 (product form)", c_v1}, {"chain split (mad addend = next sum)", c_split},
        {"chain split, 24-bit hi product", c_split24}};
    for (int rep = 0; rep < 2; ++rep)
        for (auto &c : cs) {
            hipMemset(dout, 0, 512);
            const float ms = timeit(c.k, (const uint64_t *)ds, nb, (const uint64_t *)dk, dout);
            uint64_t o[64];
            hipMemcpy(o, dout, 512, hipMemcpyDeviceToHost);
            bool ok = true;
            // y after the last block is acc_nb (the "next sum" after the last block is 0)
            for (int j = 0; j < 8; ++j) ok &= o[j] == host_ref(hs, nb, keys, j);
            printf("%-40s %.1f ns/step ok=%d\n", c.n, ms * 1e6 / nb, ok);
        }
    struct { const char *n; void (*k)(uint64_t, const uint64_t *, uint64_t *); } rs[] = {
        {"reg-fed v1 (product form, compiler)", r_v1}, {"reg-fed v1 asm", r_v1asm},
        {"reg-fed split", r_split}, {"reg-fed split24", r_split24}};
    for (int rep = 0; rep < 2; ++rep)
        for (auto &c : rs) {
            hipMemset(dout, 0, 512);
            const float ms = timeit(c.k, nb, (const uint64_t *)dk, dout);
            uint64_t o[64];
            hipMemcpy(o, dout, 512, hipMemcpyDeviceToHost);
            bool ok = true;
            for (int j = 0; j < 8; ++j) ok &= o[j] == host_ref_reg(nb, keys, j);
            printf("%-40s %.1f ns/step ok=%d\n", c.n, ms * 1e6 / nb, ok);
        }
    return 0;
}
