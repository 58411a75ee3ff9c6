// batch_checksum.hip — calculate_batch_checksum (core/binary_protocol/src/batch.rs:439-459)
// for a record whose walked frames are known: XXH3-64 streamed over the 44
// header-field bytes followed by every frame's stored 8-byte checksum.
//
// The input is 44 + 8N bytes; as XXH3 "long" input it is 1024-B blocks whose
// 16 stripe contributions commute (computed in parallel, one wave per block,
// k_bsum_blocks) chained by one scramble per block (k_bsum_chain: one wave chains,
// lane j carries accumulator j; a second wave stages its sums through LDS). Word m of the input (8 bytes at 8m):
//   m < 5  : partition_id, base_offset, base_timestamp, origin_timestamp, batch_length
//   m == 5 : message_count | lo32(cs_0) << 32
//   m >= 6 : hi32(cs_{m-6}) | lo32(cs_{m-5}) << 32
#include "codec_common.hpp"

namespace iggy {

// where the frame checksums come from
struct CsSource {
    const uint64_t *cs;     // dense array (decode general / encode), or
    const uint8_t *blob;    // gathered at blob + fpos[i]
    const uint64_t *fpos;
    const uint64_t *first = nullptr;  // device-resident index of fpos[0] (a slice), applied per kernel
    __device__ __forceinline__ uint64_t operator()(uint64_t i) const {
        return cs ? cs[i] : ld64_any(blob + fpos[i]);
    }
};

struct CsPlan {
    uint64_t n, nb, Mreg;
    bool long_cs;
};
__device__ __forceinline__ CsPlan cs_plan(uint64_t nframes) {
    CsPlan p;
    p.n = 44 + 8 * nframes;
    p.long_cs = p.n > 240;
    p.nb = 0;
    p.Mreg = 0;
    if (p.long_cs) {
        p.nb = (p.n - 1) / 1024;
        const uint64_t ns = ((p.n - 1) - 1024 * p.nb) / 64;
        p.Mreg = 8 * (16 * p.nb + ns);
    }
    return p;
}

__device__ __forceinline__ uint64_t cs_word(uint64_t m, const iggy_batch_header &h,
                                            const CsSource &src) {
    switch (m) {
        case 0: return h.partition_id;
        case 1: return h.base_offset;
        case 2: return h.base_timestamp;
        case 3: return h.origin_timestamp;
        case 4: return h.batch_length;
        case 5: return (uint64_t)h.message_count | (src(0) << 32);
        default: return (src(m - 6) >> 32) | (src(m - 5) << 32);
    }
}

// One XXH3 scramble of accumulator lane j (key = secret word 16 + j) in the
// 32-bit-piece form measured fastest on gfx950 (scripts/chain_micro.hip); the
// empty asm keeps the next block sum out of the multiply-add's addend.
__device__ __forceinline__ uint64_t scramble_fast(uint64_t y, uint32_t klo, uint32_t khi) {
    const uint32_t hi = (uint32_t)(y >> 32);
    const uint32_t lo = (uint32_t)y ^ (hi >> 15) ^ klo;
    const uint32_t h2 = hi ^ khi;
    uint64_t t = (uint64_t)lo * P32_1 + ((uint64_t)(h2 * P32_1) << 32);
    asm volatile("" : "+v"(t));
    return t;
}

// The serial part of a long XXH3 input: acc_j over nb full blocks whose stripe
// sums are bsums[8b + j] (one wave, lane j & 7 carries accumulator j). Groups of
// 16 sums rotate through three register sets (no copies of in-flight loads), so
// every group's loads were issued two groups (~32 steps) before it is chained.
__device__ __forceinline__ void chain_load16(const uint64_t *bsums, uint64_t nb, uint64_t g, int j,
                                             uint64_t (&v)[16]) {
    const uint64_t last = 8 * nb - 8 + j;  // clamp: past-the-end groups re-read a valid sum
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint64_t ix = 8 * (16 * g + k) + j;
        v[k] = bsums[ix < 8 * nb ? ix : last];
    }
}
__device__ __forceinline__ uint64_t chain_run16(uint64_t acc, const uint64_t (&v)[16], uint32_t klo, uint32_t khi) {
#pragma unroll
    for (int k = 0; k < 16; ++k) acc = scramble_fast(acc + v[k], klo, khi);
    return acc;
}
__device__ inline uint64_t chain_blocks(const uint64_t *bsums, uint64_t nb, int lane,
                                       const uint64_t *acc_in = nullptr) {
    const int j = lane & 7;
    uint64_t acc = acc_in ? acc_in[j] : kAccInit[j];
    const uint64_t key = kSecretW8[16 + j];
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    if (nb == 0) return acc;
    const uint64_t ng = nb / 16;  // full groups
    uint64_t A[16], B[16], C[16];
    chain_load16(bsums, nb, 0, j, A);
    chain_load16(bsums, nb, 1, j, B);
    chain_load16(bsums, nb, 2, j, C);
    uint64_t g = 0;
    for (; g + 3 <= ng; g += 3) {
        acc = chain_run16(acc, A, klo, khi);
        chain_load16(bsums, nb, g + 3, j, A);
        acc = chain_run16(acc, B, klo, khi);
        chain_load16(bsums, nb, g + 4, j, B);
        acc = chain_run16(acc, C, klo, khi);
        chain_load16(bsums, nb, g + 5, j, C);
    }
    if (g < ng) { acc = chain_run16(acc, A, klo, khi); ++g; }
    if (g < ng) { acc = chain_run16(acc, B, klo, khi); ++g; }
    for (uint64_t b = 16 * ng; b < nb; ++b) acc = scramble_fast(acc + bsums[8 * b + j], klo, khi);
    return acc;
}

// The same chain handed between two waves of a workgroup whose other waves do
// something else (the general decode's verify): the stager wave copies chunks of
// kChainChunk block sums into an LDS double buffer, the chain wave consumes them.
// Reading its sums straight from global memory beside the verify stream, the
// chain wave waited microseconds per prefetch group (C3: 53-56 ns per step). LDS
// flags: [0], [1] = chunk index + 1 staged in buffer 0 / 1, [2] = chunks consumed.
// Every wait is bounded (the waiter gives up after kSpinLimitTicks).
constexpr uint32_t kChainChunk = 512;  // blocks per staged chunk (32 KiB)
__device__ inline void chain_stager(const uint64_t *bsums, uint64_t nb, uint64_t *buf, uint32_t *flags, int lane,
                                    uint64_t t0) {
    const uint64_t nch = (nb + kChainChunk - 1) / kChainChunk;
    const uint4 *src = (const uint4 *)bsums;
    for (uint64_t c = 0; c < nch; ++c) {
        // buffer c & 1 is free once chunk c - 2 is consumed
        while (c >= 2 && __hip_atomic_load(&flags[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) + 2 <= c) {
            __builtin_amdgcn_s_sleep(1);
            if (rt_now() - t0 > kSpinLimitTicks) return;
        }
        uint4 *dst = (uint4 *)(buf + (c & 1) * kChainChunk * 8);
        const uint64_t q0 = 4 * kChainChunk * c, q1 = min(q0 + 4 * kChainChunk, 4 * nb);
        for (uint32_t h = 0; h < 2; ++h) {  // two rounds of 16 loads per lane
            uint4 r[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const uint64_t q = q0 + 1024u * h + lane + 64u * u;
                r[u] = q < q1 ? src[q] : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const uint64_t q = q0 + 1024u * h + lane + 64u * u;
                if (q < q1) dst[q - q0] = r[u];
            }
        }
        __hip_atomic_store(&flags[c & 1], (uint32_t)(c + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
// the chain over nb blocks from the stager's buffer (false: gave up waiting)
__device__ inline bool chain_staged(uint64_t nb, const uint64_t *buf, uint32_t *flags, int lane, uint64_t t0,
                                    uint64_t &acc) {
    const int j = lane & 7;
    acc = kAccInit[j];
    const uint64_t key = kSecretW8[16 + j];
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    const uint64_t nch = (nb + kChainChunk - 1) / kChainChunk;
    for (uint64_t c = 0; c < nch; ++c) {
        while (__hip_atomic_load(&flags[c & 1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != c + 1) {
            __builtin_amdgcn_s_sleep(1);
            if (rt_now() - t0 > kSpinLimitTicks) return false;
        }
        const uint64_t *b = buf + (c & 1) * kChainChunk * 8;
        const uint32_t kend = (uint32_t)min<uint64_t>(kChainChunk, nb - kChainChunk * c);
        uint32_t k = 0;
        uint64_t va[16], vb[16];
        if (kend >= 16) {
#pragma unroll
            for (int x = 0; x < 16; ++x) va[x] = b[8 * x + j];
            while (true) {
                const bool more = k + 32 <= kend;
                if (more) {
#pragma unroll
                    for (int x = 0; x < 16; ++x) vb[x] = b[8 * (k + 16 + x) + j];
                }
                acc = chain_run16(acc, va, klo, khi);
                k += 16;
                if (!more) break;
                const bool more2 = k + 32 <= kend;
                if (more2) {
#pragma unroll
                    for (int x = 0; x < 16; ++x) va[x] = b[8 * (k + 16 + x) + j];
                }
                acc = chain_run16(acc, vb, klo, khi);
                k += 16;
                if (!more2) break;
            }
        }
        for (; k < kend; ++k) acc = scramble_fast(acc + b[8 * k + j], klo, khi);
        __hip_atomic_store(&flags[2], (uint32_t)(c + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    return true;
}

// Header fields (by value) and the frame count (by value, or from a device word an
// earlier kernel on the stream wrote, e.g. a decode's frame_count) into the device
// words the checksum kernels read: no host copy on the enqueue path.
__global__ void k_put_header(iggy_batch_header h, uint64_t n, const uint64_t *n_dev, iggy_batch_header *dh,
                             uint64_t *dn) {
    if (threadIdx.x == 0) {
        *dh = h;
        *dn = n_dev ? *n_dev : n;
    }
}

// admit_wire_request's stamped header (server_common/src/send_messages.rs:529-537):
// the decoded header with the namespace partition id and a zero checksum field;
// nothing is hashed unless the decode succeeded.
__global__ void k_admit_header(const iggy_decode_result *res, uint64_t partition_id, iggy_batch_header *dh,
                               uint64_t *dn) {
    if (threadIdx.x == 0) {
        iggy_batch_header h = res->header;
        h.partition_id = partition_id;
        h.batch_checksum = 0;
        *dh = h;
        *dn = res->error.kind == IGGY_OK ? res->frame_count : 0;
    }
}

// header and frame count come from device memory (written by an earlier kernel
// on the stream) so nothing has to travel back to the host in between.
__global__ __launch_bounds__(256) void k_bsum_blocks(const iggy_batch_header *hp,
                                                     const uint64_t *nframes_p, CsSource src,
                                                     uint64_t *bsums, const uint32_t *skip) {
    if (skip && *skip) return;
    const iggy_batch_header h = *hp;
    const CsPlan pl = cs_plan(*nframes_p);
    if (!pl.long_cs) return;
    if (src.first) src.fpos += *src.first;
    const int lane = threadIdx.x & 63;
    const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t sec[2] = {block_word_secret(0, lane), block_word_secret(1, lane)};
    for (uint64_t b = wid; b <= pl.nb; b += nwaves) {
        uint64_t x = 0, y = 0;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const uint64_t m = 128 * b + 64 * half + lane;
            if (m < pl.Mreg) {
                const uint64_t v = cs_word(m, h, src);
                y += v;
                x += mul32x32(v ^ sec[half]);
            }
        }
        x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
        x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
        x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
        const uint64_t t8 = x + __shfl_xor(y, 1);
        if (lane < 8) bsums[b * 8 + lane] = t8;
    }
}

// one wave: out[0] = batch checksum. `small` >= 240 B scratch for short inputs.
// two waves: wave 0 chains, wave 1 stages the block sums through LDS (chain_stager)
__global__ __launch_bounds__(128) void k_bsum_chain(const iggy_batch_header *hp,
                                                    const uint64_t *nframes_p, CsSource src,
                                                    const uint64_t *bsums, uint8_t *small,
                                                    uint64_t *out, const uint32_t *skip) {
    if (skip && *skip) return;
    const iggy_batch_header h = *hp;
    const uint64_t N = *nframes_p;
    if (src.first) src.fpos += *src.first;
    const CsPlan pl = cs_plan(N);
    const int lane = threadIdx.x & 63;
    __shared__ uint64_t s_cbuf[2 * kChainChunk * 8];
    __shared__ uint32_t s_cflags[3];
    if (threadIdx.x < 3) s_cflags[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t t0 = rt_now();
    if (threadIdx.x >= 64) {
        if (pl.long_cs) chain_stager(bsums, pl.nb, s_cbuf, s_cflags, lane, t0);
        return;
    }
    if (pl.long_cs) {
        const int j = lane & 7;
        uint64_t acc = 0;
        if (!chain_staged(pl.nb, s_cbuf, s_cflags, lane, t0, acc)) acc = 0;  // bug guard (4 s): a wrong checksum
        acc += bsums[pl.nb * 8 + j];
        const uint64_t v = src(N - 8 + j);
        acc += __shfl_xor(v, 1);
        acc += mul32x32(v ^ kSecretLast[j]);
        uint64_t a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
        uint64_t r = pl.n * P64_1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
        if (lane == 0) *out = avalanche(r);
    } else if (lane == 0) {
        for (uint64_t m = 0; m < 5; ++m) st64_any(small + 8 * m, cs_word(m, h, src));
        *(uint32_t *)(small + 40) = h.message_count;
        for (uint64_t i = 0; i < N; ++i) st64_any(small + 44 + 8 * i, src(i));
        *out = xxh3_64_lane(small, pl.n);
    }
}

// ---- the same checksum in segments, so its serial chain can run beside the
// kernels still producing later frame checksums (encode: k_enc_lanes by frame
// range). Blocks [b_lo, b_hi) of the nb full blocks + the last partial block.
__global__ __launch_bounds__(256) void k_bsum_blocks_range(const iggy_batch_header *hp,
                                                           const uint64_t *nframes_p, CsSource src,
                                                           uint64_t *bsums, uint64_t b_lo, uint64_t b_hi) {
    const iggy_batch_header h = *hp;
    const CsPlan pl = cs_plan(*nframes_p);
    if (!pl.long_cs) return;
    const int lane = threadIdx.x & 63;
    const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t hi = b_hi < pl.nb + 1 ? b_hi : pl.nb + 1;
    const uint64_t sec[2] = {block_word_secret(0, lane), block_word_secret(1, lane)};
    for (uint64_t b = b_lo + wid; b < hi; b += nwaves) {
        uint64_t x = 0, y = 0;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const uint64_t m = 128 * b + 64 * half + lane;
            if (m < pl.Mreg) {
                const uint64_t v = cs_word(m, h, src);
                y += v;
                x += mul32x32(v ^ sec[half]);
            }
        }
        x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
        x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
        x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
        const uint64_t t8 = x + __shfl_xor(y, 1);
        if (lane < 8) bsums[b * 8 + lane] = t8;
    }
}

// full blocks [b_lo, min(b_hi, nb)) of the chain; state[8] carries the
// accumulators between segments (b_lo == 0 starts from the XXH3 init)
// Blocks [b_lo, b_hi) of the chain, carried in `state` (8 words). Beside a
// streaming kernel the chain wave's global loads come back after microseconds, so
// three register groups of prefetch (48 blocks, ~1.5 us of chain) starved it: a
// segment chain beside k_enc_lanes took 70-130 ns per step. Here waves 1..3 stage
// chunks of kChainChunk block sums into an LDS double buffer, one chunk ahead of
// wave 0, which chains from LDS (two register groups in flight).
__global__ __launch_bounds__(256) void k_chain_partial(const uint64_t *nframes_p, const uint64_t *bsums,
                                                       uint64_t *state, uint64_t b_lo, uint64_t b_hi) {
    const CsPlan pl = cs_plan(*nframes_p);
    if (!pl.long_cs) return;
    const uint64_t hi = b_hi < pl.nb ? b_hi : pl.nb;
    if (b_lo >= hi) return;
    __shared__ uint4 buf[2][kChainChunk * 4];  // 8 u64 (4 x 16 B) per block
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t nbk = hi - b_lo;
    const uint64_t nch = (nbk + kChainChunk - 1) / kChainChunk;
    const uint4 *src = (const uint4 *)(bsums + 8 * b_lo);
    auto stage = [&](uint64_t c, uint32_t t0, uint32_t nt) {  // chunk c by threads t0.. (nt of them)
        const uint64_t q0 = 4 * kChainChunk * c, q1 = min(q0 + 4 * kChainChunk, 4 * nbk);
        constexpr int kU = 11;  // ceil(4 * kChainChunk / 192): every load of a chunk in flight at once
        uint4 r[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t q = q0 + threadIdx.x - t0 + (uint64_t)u * nt;
            r[u] = q < q1 ? src[q] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const uint64_t q = q0 + threadIdx.x - t0 + (uint64_t)u * nt;
            if (q < q1) buf[c & 1][q - q0] = r[u];
        }
    };
    if (threadIdx.x >= 64) stage(0, 64, 192);
    __syncthreads();
    const int j = lane & 7;
    uint64_t acc = b_lo ? state[j] : kAccInit[j];
    const uint64_t key = kSecretW8[16 + j];
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    for (uint64_t c = 0; c < nch; ++c) {
        if (wave != 0) {
            if (c + 1 < nch) stage(c + 1, 64, 192);
        } else {
            const uint64_t *b = (const uint64_t *)buf[c & 1];
            const uint32_t kend = (uint32_t)min<uint64_t>(kChainChunk, nbk - kChainChunk * c);
            uint32_t k = 0;
            uint64_t va[16], vb[16];
            if (kend >= 16) {
#pragma unroll
                for (int x = 0; x < 16; ++x) va[x] = b[8 * x + j];
                while (true) {
                    const bool more = k + 32 <= kend;
                    if (more) {
#pragma unroll
                        for (int x = 0; x < 16; ++x) vb[x] = b[8 * (k + 16 + x) + j];
                    }
                    acc = chain_run16(acc, va, klo, khi);
                    k += 16;
                    if (!more) break;
                    const bool more2 = k + 32 <= kend;
                    if (more2) {
#pragma unroll
                        for (int x = 0; x < 16; ++x) va[x] = b[8 * (k + 16 + x) + j];
                    }
                    acc = chain_run16(acc, vb, klo, khi);
                    k += 16;
                    if (!more2) break;
                }
            }
            for (; k < kend; ++k) acc = scramble_fast(acc + b[8 * k + j], klo, khi);
        }
        __syncthreads();
    }
    if (threadIdx.x < 8) state[threadIdx.x] = acc;
}

// last partial block, last stripe and merge after the segments (or the whole
// short-input form); out[0] = the batch checksum
__global__ __launch_bounds__(64) void k_chain_finish(const iggy_batch_header *hp, const uint64_t *nframes_p,
                                                     CsSource src, const uint64_t *bsums, const uint64_t *state,
                                                     uint8_t *small, uint64_t *out) {
    const iggy_batch_header h = *hp;
    const uint64_t N = *nframes_p;
    const CsPlan pl = cs_plan(N);
    const int lane = threadIdx.x & 63;
    if (pl.long_cs) {
        const int j = lane & 7;
        uint64_t acc = pl.nb ? state[j] : kAccInit[j];
        acc += bsums[pl.nb * 8 + j];
        const uint64_t v = src(N - 8 + j);
        acc += __shfl_xor(v, 1);
        acc += mul32x32(v ^ kSecretLast[j]);
        uint64_t a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
        uint64_t r = pl.n * P64_1;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
        if (lane == 0) *out = avalanche(r);
    } else if (lane == 0) {
        for (uint64_t m = 0; m < 5; ++m) st64_any(small + 8 * m, cs_word(m, h, src));
        *(uint32_t *)(small + 40) = h.message_count;
        for (uint64_t i = 0; i < N; ++i) st64_any(small + 44 + 8 * i, src(i));
        *out = xxh3_64_lane(small, pl.n);
    }
}

// XXH3-64 of independent ranges, one lane per range (calculate_checksum,
// common/src/utils/checksum.rs:20, applied to many buffers at once).
__global__ __launch_bounds__(256) void k_xxh3_ranges(const uint8_t *data, const uint64_t *offs,
                                                     const uint32_t *lens, uint64_t n,
                                                     uint64_t *out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = xxh3_64_lane(data + offs[i], lens[i]);
}

// one-shot XXH3-64 of a single large device buffer: per-block stripe sums in
// parallel, then the scramble chain (same split as the batch checksum).
__global__ __launch_bounds__(256) void k_xxh3_big_blocks(const uint8_t *p, uint64_t len,
                                                         uint64_t *bsums) {
    const int lane = threadIdx.x & 63;
    const uint64_t nb = (len - 1) / 1024;
    const uint64_t ns = ((len - 1) - 1024 * nb) / 64;
    const uint64_t Mreg = 8 * (16 * nb + ns);
    const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t sec[2] = {block_word_secret(0, lane), block_word_secret(1, lane)};
    for (uint64_t b = wid; b <= nb; b += nwaves) {
        uint64_t x = 0, y = 0;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const uint64_t m = 128 * b + 64 * half + lane;
            if (m < Mreg) {
                const uint64_t v = ld64_any(p + 8 * m);
                y += v;
                x += mul32x32(v ^ sec[half]);
            }
        }
        x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
        x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
        x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
        const uint64_t t8 = x + __shfl_xor(y, 1);
        if (lane < 8) bsums[b * 8 + lane] = t8;
    }
}

__global__ __launch_bounds__(64) void k_xxh3_big_chain(const uint8_t *p, uint64_t len,
                                                       const uint64_t *bsums, uint64_t *out) {
    const int lane = threadIdx.x & 63;
    if (len <= 240) {
        if (lane == 0) *out = xxh3_64_lane(p, len);
        return;
    }
    const uint64_t nb = (len - 1) / 1024;
    const int j = lane & 7;
    uint64_t acc = chain_blocks(bsums, nb, lane);
    acc += bsums[nb * 8 + j];
    const uint64_t v = ld64_any(p + len - 64 + 8 * j);
    acc += __shfl_xor(v, 1);
    acc += mul32x32(v ^ kSecretLast[j]);
    uint64_t a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
    uint64_t r = len * P64_1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
    if (lane == 0) *out = avalanche(r);
}

// stamp_prepare_for_persistence (server_common/src/send_messages.rs:642-663):
// header fields -> record bytes (batch.rs:138-150 encode_into)
__global__ void k_write_header(uint8_t *rec, const iggy_batch_header *hp, const uint64_t *cs) {
    const int t = threadIdx.x;  // 64 threads x 4 bytes
    iggy_batch_header h = *hp;
    if (cs) h.batch_checksum = *cs;
    uint32_t w = 0;
    const uint32_t off = 4 * t;
    if (off < 48) {
        const uint64_t f[6] = {h.partition_id, h.base_offset, h.base_timestamp,
                               h.origin_timestamp, h.batch_length, h.batch_checksum};
        const uint64_t v = f[off / 8];
        w = (off & 4) ? (uint32_t)(v >> 32) : (uint32_t)v;
    } else if (off == 48) {
        w = h.message_count;
    }
    *(u32_ua *)(rec + off) = w;
}

}  // namespace iggy
