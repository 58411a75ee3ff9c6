// decode_stream.hip — DIAGNOSTIC BUILD ONLY (next-round candidate; the product
// library runs decode_general.hip). decode_batch_slice_with (batch.rs:391-527) for
// records with arbitrary frame sizes in ONE streaming pass over the record, where
// decode_general.hip walks it twice (a latency-bound locate, then the verify
// stream) with five grid barriers in between.
//
// The algorithm is scripts/stream_model.py, step for step; tests/test_stream_model_cpu.py
// checks that model against the oracle (clean records, every corruption kind,
// deliberately wrong entries, a starved link). Roles:
//   workers (every wave of members 1.., waves 4-7 of member 0): tile t = w + j W of
//     kStT bytes plus a kStE-byte overhang is DMA'd into the wave's LDS window
//     (global_load_lds_dwordx4, 16-B aligned source, no VGPRs); the entry is picked
//     and the frames walked in LDS; every listed frame hashed from LDS (8 lanes per
//     frame above 240 hashed bytes, one lane below; a frame that runs past the
//     window is hashed from global memory by one lane) and compared; the tile's
//     summary (entry, exit, count, list, stored checksums, first mismatch) published
//     with write-through stores; the group's last tile folds the group summary
//     (decode_general.hip phase B1). Between tiles a worker does the deferred work of
//     its earlier tiles whose group is linked: frame positions and stored checksums
//     scattered to walk order, the first mismatch mapped to its walk index, and the
//     tile's words of the batch-checksum input added to per-block sums and counts;
//   the link (member 0 wave 2): decode_general.hip phase B2 over the groups that are
//     ready, in order, publishing each group's base and mode;
//   the chain (member 0 waves 0-1): a stager copies blocks whose 128 words are all
//     in (a complete block is always a full block of the final input) into an LDS
//     ring; the chain wave scrambles them;
//   after the one grid barrier: the partial block, the last stripe, the merge and
//     the precedence (batch.rs:395-421, 461-506).
// Cross-workgroup data is written with relaxed agent-scope atomic stores
// (write-through) and read with atomic loads; a flag is raised only after the
// writer's vmcnt drain (the uniform kernel's publication rule, no L2 writeback).
#include "codec_common.hpp"

namespace iggy {

constexpr uint32_t kStT = 12288;                                     // tile bytes
constexpr uint32_t kStE = 4608;                                      // overhang staged with a tile
constexpr uint32_t kStLoads = (kStT + kStE + 16 + 1023) / 1024;      // LDS-DMA instructions per tile (1 KiB each)
constexpr uint32_t kStWin = kStLoads * 1024;                         // window bytes
constexpr uint32_t kStSlack = 32;                                    // reads never leave the wave's region
constexpr uint32_t kStListCap = kStT / kFrameHdr + 2;                // frames starting in a tile
constexpr uint32_t kStAccBlocks = 5;                                 // checksum blocks one tile's words touch
constexpr uint32_t kStListOff = kStWin + kStSlack;
constexpr uint32_t kStAccOff = kStListOff + 4 * kStListCap;          // u64 [kStAccBlocks][8]
constexpr uint32_t kStCntOff = kStAccOff + 64 * kStAccBlocks;        // u32 [kStAccBlocks]
constexpr uint32_t kStWaveBytes = (kStCntOff + 4 * kStAccBlocks + 15) & ~15u;
constexpr uint32_t kStThreads = 512;
constexpr uint32_t kStRing = 1024;                                   // chain ring (member 0), blocks
constexpr uint32_t kStRingFlags = kStRing * 64;                      // staged, consumed (u32)
constexpr uint32_t kStMemOff = 8 * kStWaveBytes;                     // join words
constexpr uint32_t kStLds = kStMemOff + 64;
static_assert(kStLds <= 160 * 1024, "LDS budget");
static_assert(kStRingFlags + 16 <= 4 * kStWaveBytes, "member 0's ring below its worker waves 4-7");
static_assert(kStT % kTileMin == 0, "tiles are whole kTileMin units (scratch sizing)");

struct StreamScratch {
    uint32_t *tile_bad;    // [ntiles] first mismatching listed frame (~0: none)
    uint32_t *tile_flags;  // [ntiles] 1: re-walked by the link (its hashes are re-done)
    uint32_t *grp_done;    // [ngroups] tiles finished
    uint32_t *grp_ready;   // [ngroups] summary published
    uint32_t *grp_linked;  // [ngroups] base and mode published
    uint32_t *blk_count;   // [nblocks] checksum words added
    uint32_t *final_flag;  // [1] the link ended: misc[0] = frames, misc[1] = end (| stop)
    uint32_t *timed_out;   // [1] a bounded wait gave up
};

// ---- publication helpers (write-through stores, coherent loads)
__device__ __forceinline__ void st_pub64(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_pub32(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_pub64(const uint64_t *p) {
    return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_pub32(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- wave reductions
__device__ __forceinline__ uint64_t wmin64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(v, d);
        v = o < v ? o : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wmax64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(v, d);
        v = o > v ? o : v;
    }
    return v;
}

// ---- reads of the LDS window at any byte offset: dword-aligned reads, realigned
__device__ __forceinline__ uint32_t st_rd32(const uint8_t *win, uint32_t w) { return *(const uint32_t *)(win + w); }
__device__ __forceinline__ uint4 st_rd16(const uint8_t *win, uint32_t w) {
    const uint32_t a = w & ~3u, r = w & 3u;
    const uint32_t d0 = st_rd32(win, a), d1 = st_rd32(win, a + 4), d2 = st_rd32(win, a + 8), d3 = st_rd32(win, a + 12),
                   d4 = st_rd32(win, a + 16);
    return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, r), __builtin_amdgcn_alignbyte(d2, d1, r),
                      __builtin_amdgcn_alignbyte(d3, d2, r), __builtin_amdgcn_alignbyte(d4, d3, r));
}
__device__ __forceinline__ uint64_t st_rd8(const uint8_t *win, uint32_t w) {
    const uint32_t a = w & ~3u, r = w & 3u;
    const uint32_t d0 = st_rd32(win, a), d1 = st_rd32(win, a + 4), d2 = st_rd32(win, a + 8);
    return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, r) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, r) << 32);
}

// XXH3-64 of a 17..240-byte stream in the window (xxh3_device.hpp's ladder)
__device__ inline uint64_t st_xxh3_short(const uint8_t *win, uint32_t w0, uint64_t len) {
    auto mix16 = [&](uint64_t off, uint64_t s0, uint64_t s1) {
        return fold64(st_rd8(win, w0 + (uint32_t)off) ^ s0, st_rd8(win, w0 + (uint32_t)off + 8) ^ s1);
    };
    if (len <= 128) {
        uint64_t acc = len * P64_1;
        if (len > 32) {
            if (len > 64) {
                if (len > 96) {
                    acc += mix16(48, Secret::w(96), Secret::w(104));
                    acc += mix16(len - 64, Secret::w(112), Secret::w(120));
                }
                acc += mix16(32, Secret::w(64), Secret::w(72));
                acc += mix16(len - 48, Secret::w(80), Secret::w(88));
            }
            acc += mix16(16, Secret::w(32), Secret::w(40));
            acc += mix16(len - 32, Secret::w(48), Secret::w(56));
        }
        acc += mix16(0, Secret::w(0), Secret::w(8));
        acc += mix16(len - 16, Secret::w(16), Secret::w(24));
        return avalanche(acc);
    }
    uint64_t acc = len * P64_1;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += mix16(16 * i, Secret::w(16 * i), Secret::w(16 * i + 8));
    acc = avalanche(acc);
    const uint32_t rounds = (uint32_t)(len / 16);
#pragma unroll
    for (int i = 8; i < 15; ++i)
        if ((uint32_t)i < rounds) acc += mix16(16 * i, Secret::w(16 * (i - 8) + 3), Secret::w(16 * (i - 8) + 11));
    acc += mix16(len - 16, Secret::w(119), Secret::w(127));
    return avalanche(acc);
}

struct StTile {  // one worker's view of its current tile
    uint64_t t, lo, hi;
    uint32_t d;      // the window starts d bytes before lo (16-B aligned source)
    uint8_t *win;    // the wave's LDS window
    __device__ __forceinline__ uint32_t W(uint64_t x) const { return (uint32_t)(x - lo + d); }
};

// a valid frame header at blob offset p (inside the window): reserved zero, fits
__device__ __forceinline__ bool st_valid(const StTile &tl, uint64_t bl, uint64_t p, uint64_t &e) {
    if (p + kFrameHdr > bl) return false;
    const uint4 w = st_rd16(tl.win, tl.W(p) + 32);
    if ((w.z | w.w) != 0) return false;
    e = p + kFrameHdr + (uint64_t)w.x + w.y;
    return e <= bl;
}

// The speculative entry of tile (lo, hi): candidates from the zero dwords of the
// window (8 zero reserved bytes at p + 40 contain an aligned zero dword), tested
// 64 dwords a round; the first confirmed candidate (its successor is a valid header
// inside the tile), moved to the last confirmed one within 16 B; failing that the
// valid candidate with the nearest exit, else the first valid. Only speed depends on
// the pick (the link re-walks a tile whose entry disagrees).
__device__ inline uint64_t st_pick(const StTile &tl, uint64_t bl, int lane) {
    const uint32_t w_first = (40u + tl.d) & ~3u;
    const uint32_t w_last = tl.W(tl.hi) + 43u;
    uint64_t clean_p = kNoStart, clean_x = ~0ull, first_valid = kNoStart;
    for (uint32_t w0 = w_first; w0 <= w_last; w0 += 256) {
        const uint32_t wd = w0 + 4u * (uint32_t)lane;
        uint64_t fconf = kNoStart, lconf = 0, fval = kNoStart, cp = kNoStart, cx = ~0ull;
        if (wd <= w_last && st_rd32(tl.win, wd) == 0) {
            const uint64_t ga = (uint64_t)wd + tl.lo - tl.d;  // blob offset of the zero dword
#pragma unroll
            for (int dd = 3; dd >= 0; --dd) {  // ascending p
                if (ga < 40u + (uint64_t)dd) continue;
                const uint64_t p = ga - 40 - dd;
                if (p < tl.lo || p >= tl.hi) continue;
                uint64_t e;
                if (!st_valid(tl, bl, p, e)) continue;
                if (fval == kNoStart) fval = p;
                if (e < tl.hi) {
                    uint64_t e2;
                    if (st_valid(tl, bl, e, e2)) {
                        if (fconf == kNoStart) fconf = p;
                        lconf = p;
                    }
                } else if (e < cx) {
                    cx = e;
                    cp = p;
                }
            }
        }
        const uint64_t fc = wmin64(fconf);
        if (fc != kNoStart) return wmax64((fconf != kNoStart && lconf <= fc + 16) ? lconf : 0);
        const uint64_t fv = wmin64(fval);
        if (first_valid == kNoStart) first_valid = fv;
        const uint64_t bx = wmin64(cx);
        if (bx < clean_x) {
            clean_x = bx;
            clean_p = wmin64(cx == bx ? cp : kNoStart);
        }
    }
    return clean_p != kNoStart ? clean_p : first_valid;
}

// decode_general.hip phase B1 for one group (one wave, 4 tiles per lane), reading
// the published tile summaries and publishing the group's and the tiles' prefixes
__device__ inline void st_group_fold(const GeneralScratch &gs, uint64_t g, uint64_t ntiles, uint64_t T, uint64_t bl,
                                     int lane) {
    const uint64_t tb = (uint64_t)kGrpTiles * g + 4 * lane;
    bool lhas = false, lok = true, lterm = false;
    uint64_t ls = kNoStart, lx = 0, lhi = 0;
    uint32_t lc = 0, pre[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t t = tb + i;
        pre[i] = kNotLive;
        if (t >= ntiles || lterm) continue;
        const uint64_t s = ld_pub64(gs.tile_s + t), x = ld_pub64(gs.tile_x + t);
        const uint32_t c = ld_pub32(gs.tile_cnt + t);
        const uint64_t hi_t = min((t + 1) * T, bl);
        lhi = hi_t;
        if (s != kNoStart && !(lhas && lx >= hi_t)) {
            if (lhas) lok &= s == lx;
            else ls = s;
            lhas = true;
            pre[i] = lc;
            lc += c;
            lx = x;
            lterm = (x & kStopBit) || x >= bl;
        } else if (lhas) {
            lok &= lx >= hi_t;
        }
    }
    const uint64_t termmask = __ballot(lhas && lterm);
    const int last = termmask ? __builtin_ctzll(termmask) : 63;
    const bool live = lhas && lane <= last;
    const uint64_t hasmask = __ballot(live);
    uint64_t S = kNoStart, X = 0, CNT = 0, flags = kGrpOk;
    uint32_t lpre = 0;
    if (hasmask) {
        const int f0 = __builtin_ctzll(hasmask);
        const int lh = 63 - __builtin_clzll(hasmask);
        uint64_t pm = live ? lx : 0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o = __shfl_up(pm, d);
            if (lane >= d) pm = max(pm, o);
        }
        const uint64_t pred = __shfl_up(pm, 1);
        const bool okl = lane < f0 || lane > last || lhi == 0 ||
                         (lok && (lane == f0 || (lhas ? ls == pred : pred >= lhi)));
        if (__ballot(!okl)) flags = 0;
        const uint64_t c = live ? lc : 0;
        uint64_t inc = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o = __shfl_up(inc, d);
            if (lane >= d) inc += o;
        }
        lpre = (uint32_t)(inc - c);
        S = __shfl(ls, f0);
        X = __shfl(lx, lh);
        CNT = __shfl(inc, 63);
        if (termmask) flags |= kGrpTerm;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t t = tb + i;
        if (t < ntiles) st_pub32(gs.tile_pre + t, (live && pre[i] != kNotLive) ? lpre + pre[i] : kNotLive);
    }
    if (lane == 0) {
        uint64_t *q = gs.grp + kGrpWords * g;
        st_pub64(q + 0, S);
        st_pub64(q + 1, X);
        st_pub64(q + 2, CNT);
        st_pub64(q + 3, flags);
    }
}

// the candidate chain from p while p < hi, published (the link's re-walk)
__device__ inline uint32_t st_walk_pub(const uint8_t *blob, uint64_t bl, uint64_t p, uint64_t hi, uint64_t lo,
                                       uint32_t *list, uint64_t *lcs, uint64_t *x_out) {
    uint32_t cnt = 0;
    while (p < hi) {
        if (p >= bl || bl - p < kFrameHdr) break;
        const uint4 w = ld128_any(blob + p + 32);
        const uint64_t c = ld64_any(blob + p);
        const uint64_t e = p + kFrameHdr + (uint64_t)w.x + w.y;
        if ((w.z | w.w) != 0 || e > bl) break;
        st_pub32(list + cnt, (uint32_t)(p - lo));
        st_pub64(lcs + cnt, c);
        ++cnt;
        p = e;
    }
    *x_out = p < hi ? (p | kStopBit) : p;
    return cnt;
}

struct StCtx {
    const uint8_t *body, *blob, *body_end;
    uint64_t bl, ntiles, ngroups, lcap, cap, nblk;
    uint64_t *frame_pos;
    iggy_batch_header h;
    GeneralScratch gs;
    StreamScratch ss;
    uint64_t t0;
};

// ---------------------------------------------------------------- worker: one tile
template <bool VERIFY>
__device__ inline void st_tile(const StCtx &cx, StTile &tl, uint32_t *lst, int lane) {
    const GeneralScratch &gs = cx.gs;
    const uint64_t bl = cx.bl, t = tl.t;
    // 1. entry and walk (lane 0 walks; the list goes to LDS and, published, to global)
    const uint64_t s = t == 0 ? 0 : st_pick(tl, bl, lane);
    uint32_t cnt = 0;
    uint64_t x = kNoStart;
    if (s != kNoStart && lane == 0) {
        uint64_t p = s;
        uint32_t *gl = gs.tile_list + t * cx.lcap;
        uint64_t *gc = gs.tile_lcs + t * cx.lcap;
        while (p < tl.hi) {
            uint64_t e;
            if (!st_valid(tl, bl, p, e)) break;
            lst[cnt] = (uint32_t)(p - tl.lo);
            st_pub32(gl + cnt, (uint32_t)(p - tl.lo));
            st_pub64(gc + cnt, st_rd8(tl.win, tl.W(p)));
            ++cnt;
            p = e;
        }
        x = p < tl.hi ? (p | kStopBit) : p;
    }
    cnt = (uint32_t)__shfl((int)cnt, 0);
    x = __shfl(x, 0);
    if (lane == 0) {
        st_pub64(gs.tile_s + t, s);
        st_pub64(gs.tile_x + t, x);
        st_pub32(gs.tile_cnt + t, cnt);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // lane 0's list in LDS, for every lane
    // 2. every listed frame hashed and compared
    uint32_t badk = ~0u;
    if (VERIFY && cnt) {
        const uint64_t xe = x & ~kStopBit;
        auto frame = [&](uint32_t k, uint64_t &p, uint64_t &L, bool &inw) {
            p = tl.lo + lst[k];
            const uint64_t end = k + 1 < cnt ? tl.lo + lst[k + 1] : xe;
            L = end - p - 8;
            inw = (uint64_t)tl.W(end) + 4 <= kStWin;
        };
        // one lane per frame: hashed length <= 240, or running past the window
        for (uint32_t k = (uint32_t)lane; k < cnt; k += 64) {
            uint64_t p, L;
            bool inw;
            frame(k, p, L, inw);
            uint64_t hsh;
            if (!inw) hsh = xxh3_64_lane(cx.blob + p + 8, L);
            else if (L <= 240) hsh = st_xxh3_short(tl.win, tl.W(p + 8), L);
            else continue;
            if (hsh != st_rd8(tl.win, tl.W(p))) badk = min(badk, k);
        }
        // eight lanes per frame (decode_general.hip verify_frames' lane groups, from LDS)
        const uint32_t l = lane & 7, m = l >> 1, par = l & 1, fg = (uint32_t)lane >> 3;
        const uint32_t poff = 16 * (m + 4 * par);
        uint64_t s0[8], s1[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            s0[q] = kSecretW8[2 * q + par + 2 * m];
            s1[q] = kSecretW8[2 * q + par + 2 * m + 1];
        }
        const uint64_t key0 = kSecretW8[16 + 2 * m], key1 = kSecretW8[17 + 2 * m];
        const uint64_t init0 = par ? 0 : kAccInit[2 * m], init1 = par ? 0 : kAccInit[2 * m + 1];
        const uint64_t last0 = kSecretLast[2 * m], last1 = kSecretLast[2 * m + 1];
        const uint64_t mrg0 = kSecretMerge[2 * m], mrg1 = kSecretMerge[2 * m + 1];
        auto next_long = [&](uint32_t k) -> uint32_t {
            for (; k < cnt; k += 8) {
                uint64_t p, L;
                bool inw;
                frame(k, p, L, inw);
                if (inw && L > 240) break;
            }
            return k;
        };
        uint32_t k = next_long(fg), b = 0, wH = 0;
        uint64_t L = 0, nbF = 0, ns = 0, a0 = 0, a1 = 0, stored = 0;
        uint32_t nsteps = 1;
        uint4 lastp = make_uint4(0, 0, 0, 0);
        auto setup = [&]() {
            if (k >= cnt) return;
            uint64_t p;
            bool inw;
            frame(k, p, L, inw);
            wH = tl.W(p + 8);
            nbF = (L - 1) / 1024;
            ns = ((L - 1) - 1024 * nbF) / 64;
            nsteps = (uint32_t)(nbF + (ns > 0));
            b = 0;
            a0 = init0;
            a1 = init1;
            lastp = st_rd16(tl.win, wH + (uint32_t)L - 64 + 16 * m);
            stored = st_rd8(tl.win, tl.W(p));
        };
        setup();
        while (__ballot(k < cnt)) {
            if (k < cnt) {
                uint4 pc[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const bool use = b < nbF || (uint64_t)(2 * q + par) < ns;
                    pc[q] = use ? st_rd16(tl.win, wH + 1024 * b + 128 * q + poff) : make_uint4(0, 0, 0, 0);
                }
                if (b < nbF) {
                    uint64_t p0[4] = {0, 0, 0, 0}, p1[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int q = 0; q < 8; ++q) piece(p0[q & 3], p1[q & 3], pc[q], s0[q], s1[q]);
                    a0 += (p0[0] + p0[1]) + (p0[2] + p0[3]);
                    a1 += (p1[0] + p1[1]) + (p1[2] + p1[3]);
                    a0 += gdpp64<0xB1>(a0);
                    a1 += gdpp64<0xB1>(a1);
                    a0 = scramble1(a0, key0);
                    a1 = scramble1(a1, key1);
                    if (par) { a0 = 0; a1 = 0; }
                } else {
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        if ((uint64_t)(2 * q + par) < ns) piece(a0, a1, pc[q], s0[q], s1[q]);
                }
                if (b + 1 == nsteps) {
                    a0 += gdpp64<0xB1>(a0);
                    a1 += gdpp64<0xB1>(a1);
                    piece(a0, a1, lastp, last0, last1);
                    uint64_t tt = fold64(a0 ^ mrg0, a1 ^ mrg1);
                    tt += gdpp64<0x4E>(tt);
                    tt += gswz_xor4(tt);
                    if (avalanche(L * P64_1 + tt) != stored) badk = min(badk, k);
                    k = next_long(k + 8);
                    setup();
                } else {
                    ++b;
                }
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) badk = min(badk, (uint32_t)__shfl_xor((int)badk, d));
    }
    if (lane == 0) st_pub32(cx.ss.tile_bad + t, badk);
    // 3. publish; the group's last tile folds the group summary
    vm_drain();
    const uint64_t g = t / kGrpTiles;
    const uint32_t in_group = (uint32_t)min<uint64_t>(kGrpTiles, cx.ntiles - (uint64_t)kGrpTiles * g);
    uint32_t old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(cx.ss.grp_done + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = (uint32_t)__shfl((int)old, 0);
    if (old + 1 == in_group) {
        st_group_fold(gs, g, cx.ntiles, kStT, bl, lane);
        vm_drain();
        if (lane == 0) st_pub32(cx.ss.grp_ready + g, 1u);
    }
}

// ------------------------------------------------- worker: deferred work of a tile
// false: the tile's group is not linked yet
template <bool VERIFY>
__device__ inline bool st_deferred(const StCtx &cx, uint64_t t, uint8_t *wl, int lane) {
    const GeneralScratch &gs = cx.gs;
    const uint64_t g = t / kGrpTiles;
    if (!ld_pub32(cx.ss.grp_linked + g)) return false;
    const uint64_t *q = gs.grp + kGrpWords * g;
    const uint64_t mode = ld_pub64(q + 5), gbase = ld_pub64(q + 4);
    uint64_t base = 0;
    bool live = false;
    if (mode == 1) {
        const uint32_t pre = ld_pub32(gs.tile_pre + t);
        live = pre != kNotLive;
        base = gbase + pre;
    } else if (mode == 2) {
        live = ld_pub64(gs.tile_e + t) != ~0ull;
        base = ld_pub64(gs.tile_base + t);
    }
    if (!live) return true;
    const uint32_t cnt = ld_pub32(gs.tile_cnt + t);
    const uint64_t x = ld_pub64(gs.tile_x + t);
    const uint64_t lo = t * kStT, bl = cx.bl;
    const uint32_t *gl = gs.tile_list + t * cx.lcap;
    const uint64_t *gc = gs.tile_lcs + t * cx.lcap;
    uint64_t *acc = (uint64_t *)(wl + kStAccOff);
    uint32_t *acnt = (uint32_t *)(wl + kStCntOff);
    const uint64_t b_lo = base == 0 ? 0 : (base + 6) >> 7;
    uint64_t cs0 = 0;
    for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
        const uint32_t k = k0 + (uint32_t)lane;
        const bool inr = k < cnt;
        const uint32_t off = inr ? ld_pub32(gl + k) : 0;
        const uint64_t c = inr ? ld_pub64(gc + k) : 0;
        const uint64_t f = base + k;
        if (inr) {
            gs.fpos[f] = lo + off;
            gs.cs[f] = c;
            if (cx.frame_pos && f < cx.cap) cx.frame_pos[f] = lo + off;
        }
        if (k0 == 0) cs0 = __shfl(c, 0);
        if (VERIFY) {
            // word f + 6 = hi32(cs_f) | lo32(cs_{f+1}) << 32; the tile's last frame takes
            // the next frame's checksum at its exit (the record's last one has no word)
            uint64_t nx = __shfl_down(c, 1);
            bool has = inr && k + 1 < cnt;
            if (inr && lane == 63 && k + 1 < cnt) nx = ld_pub64(gc + k + 1);
            if (inr && k + 1 == cnt && !(x & kStopBit) && x + 8 <= bl) {
                nx = ld64_any(cx.blob + x);
                has = true;
            }
            if (has) {
                const uint64_t m = f + 6, v = (c >> 32) | (nx << 32);
                const uint32_t j = (uint32_t)(m & 7), bi = (uint32_t)((m >> 7) - b_lo);
                atomicAdd((unsigned long long *)&acc[8 * bi + j],
                          (unsigned long long)mul32x32(v ^ kSecretW8[((m >> 3) & 15) + j]));
                atomicAdd((unsigned long long *)&acc[8 * bi + (j ^ 1)], (unsigned long long)v);
                atomicAdd(&acnt[bi], 1u);
            }
        }
    }
    if (VERIFY) {
        if (base == 0 && lane < 6) {  // words 0..5: header fields, count | lo32(cs_0)
            const iggy_batch_header &h = cx.h;
            const uint64_t v = lane == 0 ? h.partition_id : lane == 1 ? h.base_offset : lane == 2 ? h.base_timestamp
                             : lane == 3 ? h.origin_timestamp : lane == 4 ? h.batch_length
                                         : (uint64_t)h.message_count | (cs0 << 32);
            const uint32_t j = (uint32_t)lane;
            atomicAdd((unsigned long long *)&acc[j], (unsigned long long)mul32x32(v ^ kSecretW8[j]));
            atomicAdd((unsigned long long *)&acc[j ^ 1], (unsigned long long)v);
            atomicAdd(&acnt[0], 1u);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // the first mismatch: the tile's own (hashed with its list), or re-hashed when
        // the link re-walked the tile
        uint32_t bad = ~0u;
        if (ld_pub32(cx.ss.tile_flags + t)) {
            for (uint32_t k = (uint32_t)lane; k < cnt; k += 64) {
                const uint64_t p = lo + ld_pub32(gl + k);
                const uint64_t end = k + 1 < cnt ? lo + ld_pub32(gl + k + 1) : (x & ~kStopBit);
                if (xxh3_64_lane(cx.blob + p + 8, end - p - 8) != ld_pub64(gc + k)) bad = min(bad, k);
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) bad = min(bad, (uint32_t)__shfl_xor((int)bad, d));
        } else {
            bad = ld_pub32(cx.ss.tile_bad + t);
        }
        if (lane == 0 && bad != ~0u && bad < cnt)
            atomicMax((unsigned long long *)&gs.misc[2], (unsigned long long)~(base + bad));
        // the tile's block partials, then (after they land) the blocks' word counts
        const uint64_t nbt = min<uint64_t>(kStAccBlocks, ((base + cnt + 5) >> 7) - b_lo + 1);
        if ((uint64_t)lane < 8 * nbt) {
            const uint64_t v = acc[lane];
            if (v) atomicAdd((unsigned long long *)&gs.bsums[8 * b_lo + lane], (unsigned long long)v);
        }
        vm_drain();
        if ((uint64_t)lane < nbt && acnt[lane])
            __hip_atomic_fetch_add(cx.ss.blk_count + b_lo + lane, acnt[lane], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        // re-zero the partials for the next tile
        if (lane < (int)(8 * kStAccBlocks)) acc[lane] = 0;
        if (lane < (int)kStAccBlocks) acnt[lane] = 0;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return true;
}

template <bool VERIFY>
__device__ inline void st_worker(const StCtx &cx, uint8_t *smem, uint32_t wave, uint64_t wid, uint64_t W, int lane,
                                 bool &ok) {
    uint8_t *wl = smem + wave * kStWaveBytes;
    const uint32_t wl_lds = wave * kStWaveBytes;  // LDS byte address of the window (dynamic LDS only)
    uint32_t *lst = (uint32_t *)(wl + kStListOff);
    if (lane < (int)(8 * kStAccBlocks)) ((uint64_t *)(wl + kStAccOff))[lane] = 0;
    if (lane < (int)kStAccBlocks) ((uint32_t *)(wl + kStCntOff))[lane] = 0;
    const uint64_t ntiles = cx.ntiles;
    const uint64_t jn = wid < ntiles ? (ntiles - wid + W - 1) / W : 0;
    uint64_t jd = 0;
    for (uint64_t j = 0; j < jn; ++j) {
        StTile tl;
        tl.t = wid + j * W;
        tl.lo = tl.t * kStT;
        tl.hi = min(tl.lo + kStT, cx.bl);
        const uint8_t *a0 = (const uint8_t *)((uintptr_t)(cx.blob + tl.lo) & ~(uintptr_t)15);
        tl.d = (uint32_t)((cx.blob + tl.lo) - a0);
        tl.win = wl;
        // the window's DMA; then, while it flies, the deferred work of earlier tiles
#pragma unroll
        for (uint32_t i = 0; i < kStLoads; ++i) {
            const uint8_t *src = a0 + 1024u * i + 16u * (uint32_t)lane;
            glds16(src + 16 <= cx.body_end ? src : a0, wl_lds + 1024u * i);
        }
        while (jd < j && st_deferred<VERIFY>(cx, wid + jd * W, wl, lane)) ++jd;
        vm_drain();
        st_tile<VERIFY>(cx, tl, lst, lane);
    }
    while (jd < jn) {
        if (st_deferred<VERIFY>(cx, wid + jd * W, wl, lane)) {
            ++jd;
            continue;
        }
        __builtin_amdgcn_s_sleep(2);
        if (rt_now() - cx.t0 > kSpinLimitTicks) {
            ok = false;
            return;
        }
    }
}

// ------------------------------------------------------------------ the link
__device__ inline void st_publish_linked(const StCtx &cx, uint64_t g) { st_pub32(cx.ss.grp_linked + g, 1u); }

template <bool VERIFY>
__device__ inline void st_linker(const StCtx &cx, int lane, bool &ok) {
    const GeneralScratch &gs = cx.gs;
    const uint64_t ngroups = cx.ngroups, ntiles = cx.ntiles, T = kStT, bl = cx.bl, lcap = cx.lcap;
    uint64_t e = 0, total = 0, G0 = 0;
    bool ended = false;
    while (G0 < ngroups) {
        if (ended) {  // the walk ended: no later group holds frames
            for (uint64_t g = G0 + lane; g < ngroups; g += 64) st_pub64(gs.grp + kGrpWords * g + 5, 0);
            vm_drain();
            for (uint64_t g = G0 + lane; g < ngroups; g += 64) st_publish_linked(cx, g);
            break;
        }
        const uint64_t g = G0 + lane;
        const bool inr = g < ngroups;
        const uint64_t rmask = __ballot(inr && ld_pub32(cx.ss.grp_ready + g));
        const uint32_t nready = (uint32_t)min<uint64_t>(rmask == ~0ull ? 64 : __builtin_ctzll(~rmask), ngroups - G0);
        if (nready == 0) {
            __builtin_amdgcn_s_sleep(2);
            if (rt_now() - cx.t0 > kSpinLimitTicks) {
                ok = false;
                break;
            }
            continue;
        }
        const bool in = (uint32_t)lane < nready;
        uint64_t *q = gs.grp + kGrpWords * g;
        const uint64_t S = in ? ld_pub64(q + 0) : kNoStart, X = in ? ld_pub64(q + 1) : 0;
        const uint64_t CNT = in ? ld_pub64(q + 2) : 0, flags = in ? ld_pub64(q + 3) : 0;
        const bool has = S != kNoStart;
        const uint64_t ghi = min(min((uint64_t)kGrpTiles * (g + 1), ntiles) * T, bl);
        const uint64_t termmask = __ballot(in && has && (flags & kGrpTerm));
        const int last = termmask ? __builtin_ctzll(termmask) : 63;
        uint64_t pm = (in && has && lane <= last) ? X : 0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o = __shfl_up(pm, d);
            if (lane >= d) pm = max(pm, o);
        }
        uint64_t pred = __shfl_up(pm, 1);
        if (lane == 0) pred = 0;
        pred = max(pred, e);
        const bool okl = !in || lane > last || ((flags & kGrpOk) && (has ? S == pred : pred >= ghi));
        const uint64_t badmask = __ballot(!okl);
        const uint32_t nacc = (uint32_t)min<uint64_t>(badmask ? __builtin_ctzll(badmask) : 64, nready);
        if (nacc > 0) {
            const bool acc = (uint32_t)lane < nacc;
            const uint64_t c = (acc && has && lane <= last) ? CNT : 0;
            uint64_t inc = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(inc, d);
                if (lane >= d) inc += o;
            }
            if (acc) {
                st_pub64(q + 4, total + inc - c);
                st_pub64(q + 5, (has && lane <= last) ? 1 : 0);
            }
            total += __shfl(inc, 63);
            if (termmask && (uint32_t)last < nacc) {
                e = __shfl(X, last);
                ended = true;
            } else {
                e = max(e, __shfl(pm, (int)nacc - 1));
            }
            vm_drain();
            if (acc) st_publish_linked(cx, g);
            G0 += nacc;
        }
        if (ended || nacc == nready) continue;
        // group G0 exactly (decode_general.hip phase B2's single-group path)
        const uint64_t gg = G0;
        const uint32_t ln = nacc;  // its lane in this step
        const uint64_t Sl = __shfl(S, (int)ln), Xl = __shfl(X, (int)ln), Cl = __shfl(CNT, (int)ln);
        const uint64_t Fl = __shfl(flags, (int)ln), ghl = __shfl(ghi, (int)ln);
        uint64_t *ql = gs.grp + kGrpWords * gg;
        G0 = gg + 1;
        if ((Fl & kGrpOk) && Sl != kNoStart && Sl == e) {
            if (lane == 0) { st_pub64(ql + 4, total); st_pub64(ql + 5, 1); }
            total += Cl;
            e = Xl;
            if (Fl & kGrpTerm) ended = true;
            vm_drain();
            if (lane == 0) st_publish_linked(cx, gg);
            continue;
        }
        if ((Fl & kGrpOk) && Sl == kNoStart && e >= ghl) {
            if (lane == 0) st_pub64(ql + 5, 0);  // one frame spans the whole group
            vm_drain();
            if (lane == 0) st_publish_linked(cx, gg);
            continue;
        }
        // tile by tile: lane l holds tiles 4l..4l+3 of the group
        uint64_t ts[4], tx[4];
        uint32_t tc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint64_t t = (uint64_t)kGrpTiles * gg + 4 * lane + i;
            const bool tin = t < ntiles;
            ts[i] = tin ? ld_pub64(gs.tile_s + t) : kNoStart;
            tx[i] = tin ? ld_pub64(gs.tile_x + t) : 0;
            tc[i] = tin ? ld_pub32(gs.tile_cnt + t) : 0;
        }
        const uint64_t gt0 = (uint64_t)kGrpTiles * gg;
        uint32_t k0 = 0;
        while (!ended && k0 < kGrpTiles && gt0 + k0 < ntiles) {
            bool seen = false, lterm = false;
            uint64_t lx = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t k = 4 * lane + i;
                const uint64_t t = gt0 + k;
                if (k < k0 || t >= ntiles || lterm || ts[i] == kNoStart) continue;
                const uint64_t hi = min((t + 1) * T, bl);
                if (seen && lx >= hi) continue;
                seen = true;
                lx = tx[i];
                lterm = (lx & kStopBit) || lx >= bl;
            }
            const uint64_t tm = __ballot(seen && lterm);
            const int tl = tm ? __builtin_ctzll(tm) : 63;
            uint64_t pmx = (seen && lane <= tl) ? lx : 0;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(pmx, d);
                if (lane >= d) pmx = max(pmx, o);
            }
            uint64_t r = __shfl_up(pmx, 1);
            if (lane == 0) r = 0;
            r = max(r, e);
            uint32_t kbad = kGrpTiles;
            uint64_t ebad = 0;
            bool aseen = false, stop = false;
            uint64_t ax = 0;
            uint32_t livem = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t k = 4 * lane + i;
                const uint64_t t = gt0 + k;
                if (k < k0 || t >= ntiles || stop || kbad != kGrpTiles || lane > tl) continue;
                const uint64_t hi = min((t + 1) * T, bl);
                const bool hs = ts[i] != kNoStart;
                const bool assumed = hs && (!aseen || ax < hi);
                const bool fail = r >= hi ? assumed : (!hs || ts[i] != r || !assumed);
                if (fail) {
                    kbad = k;
                    ebad = r;
                    continue;
                }
                if (assumed) {
                    aseen = true;
                    ax = tx[i];
                    livem |= 1u << i;
                    r = tx[i];
                    stop = (r & kStopBit) || r >= bl;
                }
            }
            uint32_t kb = kbad;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) kb = min(kb, (uint32_t)__shfl_xor((int)kb, d));
            uint64_t c = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (((livem >> i) & 1) && 4 * (uint32_t)lane + i < kb) c += tc[i];
            uint64_t inc = c;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t o = __shfl_up(inc, d);
                if (lane >= d) inc += o;
            }
            uint64_t run = total + inc - c;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t k = 4 * lane + i;
                const uint64_t t = gt0 + k;
                if (k < k0 || k >= kb || t >= ntiles) continue;
                const bool lv = (livem >> i) & 1;
                st_pub64(gs.tile_e + t, lv ? ts[i] : ~0ull);
                if (lv) {
                    st_pub64(gs.tile_base + t, run);
                    run += tc[i];
                }
            }
            total += __shfl(inc, 63);
            if (kb == kGrpTiles) {
                if (tm) {
                    e = __shfl(lx, tl);
                    ended = true;
                } else {
                    e = max(e, __shfl(pmx, 63));
                }
                k0 = kGrpTiles;
                break;
            }
            // re-walk tile kb from its true entry (no frames when the entry spans it)
            const uint32_t owner = kb >> 2;
            const uint64_t eb = __shfl(ebad, (int)owner);
            const uint64_t t = gt0 + kb;
            const uint64_t lo = t * T, hi = min(lo + T, bl);
            uint64_t x2 = 0;
            uint32_t c2 = 0;
            if (lane == 0) {
                c2 = st_walk_pub(cx.blob, bl, eb, hi, lo, gs.tile_list + t * lcap, gs.tile_lcs + t * lcap, &x2);
                st_pub32(gs.tile_cnt + t, c2);
                st_pub64(gs.tile_x + t, x2);
                st_pub64(gs.tile_e + t, c2 ? eb : ~0ull);
                st_pub64(gs.tile_base + t, total);
                st_pub32(cx.ss.tile_flags + t, 1u);
            }
            x2 = __shfl(x2, 0);
            c2 = (uint32_t)__shfl((int)c2, 0);
            total += c2;
            e = x2;
            if ((e & kStopBit) || e >= bl) ended = true;
            k0 = kb + 1;
        }
        if (ended) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t k = 4 * lane + i;
                if (k >= k0 && gt0 + k < ntiles) st_pub64(gs.tile_e + gt0 + k, ~0ull);
            }
        }
        if (lane == 0) st_pub64(ql + 5, 2);
        vm_drain();
        if (lane == 0) st_publish_linked(cx, gg);
    }
    if (lane == 0) {
        st_pub64(&gs.misc[0], total);
        st_pub64(&gs.misc[1], e);
    }
    vm_drain();
    if (lane == 0) st_pub32(cx.ss.final_flag, 1u);
}

// ------------------------------------------------------------------ the chain
// full blocks of the checksum input of a walk of n frames
__device__ __forceinline__ uint64_t st_full_blocks(uint64_t nwalk) {
    const uint64_t n = 44 + 8 * nwalk;
    return n > 240 ? (n - 1) / 1024 : 0;
}
__device__ inline void st_stager(const StCtx &cx, uint8_t *smem, int lane, bool &ok) {
    uint64_t *ring = (uint64_t *)smem;
    uint32_t *flags = (uint32_t *)(smem + kStRingFlags);  // [0] staged, [1] consumed
    uint64_t b0 = 0;
    while (true) {
        uint64_t nbf = ~0ull;
        if (ld_pub32(cx.ss.final_flag)) nbf = st_full_blocks(ld_pub64(&cx.gs.misc[0]));
        if (b0 >= nbf) break;
        const uint32_t consumed = __hip_atomic_load(&flags[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t room = kStRing - (b0 - consumed);
        const uint64_t b = b0 + lane;
        const bool cand = (uint64_t)lane < room && b < nbf && b < cx.nblk;
        const bool full = cand && ld_pub32(cx.ss.blk_count + b) == 128;
        const uint64_t fm = __ballot(full);
        const uint32_t k = fm == ~0ull ? 64 : __builtin_ctzll(~fm);
        if (k == 0) {
            __builtin_amdgcn_s_sleep(1);
            if (rt_now() - cx.t0 > kSpinLimitTicks) {
                ok = false;
                break;
            }
            continue;
        }
        if ((uint32_t)lane < k) {
            const uint64_t *src = cx.gs.bsums + 8 * b;
            uint64_t *dst = ring + 8 * (b % kStRing);
#pragma unroll
            for (int j = 0; j < 8; ++j) dst[j] = ld_pub64(src + j);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        b0 += k;
        if (lane == 0) __hip_atomic_store(&flags[0], (uint32_t)b0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
// lane j & 7 carries accumulator j over every full block; false: gave up waiting
__device__ inline uint64_t st_chain(const StCtx &cx, uint8_t *smem, int lane, bool &ok) {
    const uint64_t *ring = (const uint64_t *)smem;
    uint32_t *flags = (uint32_t *)(smem + kStRingFlags);
    const int j = lane & 7;
    uint64_t acc = kAccInit[j];
    const uint64_t key = kSecretW8[16 + j];
    const uint32_t klo = (uint32_t)key, khi = (uint32_t)(key >> 32);
    uint64_t b = 0;
    while (true) {
        const uint32_t staged = __hip_atomic_load(&flags[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (b < staged) {
            for (; b < staged; ++b) acc = scramble_fast(acc + ring[8 * (b % kStRing) + j], klo, khi);
            if (lane == 0) __hip_atomic_store(&flags[1], (uint32_t)b, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            continue;
        }
        if (ld_pub32(cx.ss.final_flag) && b >= st_full_blocks(ld_pub64(&cx.gs.misc[0]))) break;
        __builtin_amdgcn_s_sleep(1);
        if (rt_now() - cx.t0 > kSpinLimitTicks) {
            ok = false;
            break;
        }
    }
    return acc;
}

// ------------------------------------------------------------------ kernel
template <bool VERIFY>
__global__ __launch_bounds__(kStThreads) void k_decode_stream(const uint8_t *__restrict__ body, uint64_t len,
                                                              uint64_t *frame_pos, uint64_t cap,
                                                              iggy_decode_result *result, GeneralScratch gs,
                                                              StreamScratch ss) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // the uniform kernel of this decode has completed (stream order): re-arm its sync words
        __hip_atomic_store(gs.u_exited, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gs.u_first_bad, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gs.u_spec_fail, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (__hip_atomic_load(&result->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kStatusNeedGeneral) return;
    StCtx cx;
    cx.t0 = rt_now();
    uint32_t *s_mem = (uint32_t *)(smem + kStMemOff);
    join_members(gs, cx.t0, s_mem);
    const uint32_t member = s_mem[0];
    if (member == kNotMember) return;
    const uint32_t nwg = s_mem[1];
    cx.body = body;
    cx.blob = body + kHdr;
    cx.body_end = body + len;
    cx.h = result->header;
    cx.bl = cx.h.batch_length - kHdr;
    cx.ntiles = (cx.bl + kStT - 1) / kStT;
    cx.ngroups = (cx.ntiles + kGrpTiles - 1) / kGrpTiles;
    cx.lcap = tile_list_cap(kStT);
    cx.cap = cap;
    cx.frame_pos = frame_pos;
    cx.nblk = (44 + 8 * (cx.bl / kFrameHdr + 1)) / 1024 + 2;
    cx.gs = gs;
    cx.ss = ss;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    bool ok = true;
    // zero the counters and the block sums (every member), one barrier
    {
        const uint64_t gt = (uint64_t)member * blockDim.x + threadIdx.x, gn = (uint64_t)nwg * blockDim.x;
        for (uint64_t i = gt; i < cx.ntiles; i += gn) ss.tile_flags[i] = 0;
        for (uint64_t i = gt; i < cx.ngroups; i += gn) {
            ss.grp_done[i] = 0;
            ss.grp_ready[i] = 0;
            ss.grp_linked[i] = 0;
        }
        for (uint64_t i = gt; i < cx.nblk; i += gn) ss.blk_count[i] = 0;
        for (uint64_t i = gt; i < 8 * cx.nblk; i += gn) gs.bsums[i] = 0;
        if (gt == 0) {
            *ss.final_flag = 0;
            *ss.timed_out = 0;
        }
        if (member == 0 && threadIdx.x < 2) ((uint32_t *)(smem + kStRingFlags))[threadIdx.x] = 0;
    }
    ok &= grid_barrier2(gs.bar2, member, nwg, 1, cx.t0);
    const uint64_t W = 8ull * (nwg - 1) + 4;
    uint64_t acc = 0;
    if (member == 0 && wave == 0) {
        if (VERIFY) acc = st_chain(cx, smem, lane, ok);
    } else if (member == 0 && wave == 1) {
        if (VERIFY) st_stager(cx, smem, lane, ok);
    } else if (member == 0 && wave == 2) {
        st_linker<VERIFY>(cx, lane, ok);
    } else if (member == 0 && wave == 3) {
        // idle (its LDS holds the chain ring)
    } else {
        const uint64_t wid = member == 0 ? 8ull * (nwg - 1) + (wave - 4) : (uint64_t)wave * (nwg - 1) + (member - 1);
        st_worker<VERIFY>(cx, smem, wave, wid, W, lane, ok);
    }
    if (!ok) __hip_atomic_store(ss.timed_out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ok &= grid_barrier2(gs.bar2, member, nwg, 2, cx.t0);

    // ---------------- resolution (wave 0 of member 0): partial block, last stripe, precedence
    if (member != 0 || wave != 0) return;
    const uint64_t nwalk = __hip_atomic_load(&gs.misc[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t end = __hip_atomic_load(&gs.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t n = 44 + 8 * nwalk;
    const bool long_cs = VERIFY && n > 240;
    const iggy_batch_header h = cx.h;
    uint64_t computed = 0;
    if (long_cs) {
        const uint64_t nb = (n - 1) / 1024, ns = ((n - 1) - 1024 * nb) / 64, Mreg = 8 * (16 * nb + ns);
        const int j = lane & 7;
        uint64_t x = 0, y = 0;
        for (int half = 0; half < 2; ++half) {  // the partial block nb (words < Mreg)
            const uint64_t mw = 128 * nb + 64 * half + lane;
            if (mw < Mreg) {
                const uint64_t v = mw < 5 ? (mw == 0 ? h.partition_id : mw == 1 ? h.base_offset
                                              : mw == 2 ? h.base_timestamp : mw == 3 ? h.origin_timestamp
                                                                                   : h.batch_length)
                                 : mw == 5 ? ((uint64_t)h.message_count | (gs.cs[0] << 32))
                                           : ((gs.cs[mw - 6] >> 32) | (gs.cs[mw - 5] << 32));
                y += v;
                x += mul32x32(v ^ block_word_secret(half, lane));
            }
        }
        x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
        x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
        x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
        acc += x + __shfl_xor(y, 1);
        const uint64_t v = gs.cs[nwalk - 8 + j];  // the last stripe: the last 8 stored checksums
        acc += __shfl_xor(v, 1);
        acc += mul32x32(v ^ kSecretLast[j]);
        uint64_t a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
        uint64_t r = n * P64_1;
#pragma unroll
        for (int i = 0; i < 4; ++i) r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
        computed = avalanche(r);
    } else if (VERIFY && lane == 0) {
        uint8_t *s = gs.small;
        const uint64_t w[5] = {h.partition_id, h.base_offset, h.base_timestamp, h.origin_timestamp, h.batch_length};
        for (int i = 0; i < 5; ++i)
            for (int k = 0; k < 8; ++k) s[8 * i + k] = (uint8_t)(w[i] >> (8 * k));
        for (int k = 0; k < 4; ++k) s[40 + k] = (uint8_t)(h.message_count >> (8 * k));
        for (uint64_t i = 0; i < nwalk; ++i)
            for (int k = 0; k < 8; ++k) s[44 + 8 * i + k] = (uint8_t)(gs.cs[i] >> (8 * k));
        computed = xxh3_64_lane(s, n);
    }
    if (lane != 0) return;
    const uint8_t *blob = cx.blob;
    const uint64_t bl = cx.bl;
    HeaderInfo hi;
    hi.h = h;
    const uint64_t fb_enc = __hip_atomic_load(&gs.misc[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t kind = IGGY_OK, reason = 0;
    uint64_t a = 0, b = 0, c = 0;
    if (!ok || __hip_atomic_load(ss.timed_out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        kind = IGGY_ERR_TIMEOUT;
    } else if (VERIFY && fb_enc != 0) {
        const uint64_t i = ~fb_enc, p = gs.fpos[i];
        const uint64_t L = 40 + (uint64_t)ld32_any(blob + p + 36) + ld32_any(blob + p + 32);
        kind = IGGY_ERR_INVALID_MESSAGE_CHECKSUM;
        a = gs.cs[i];
        b = xxh3_64_lane(blob + p + 8, L);
        c = sat_add(h.base_offset, ld32_any(blob + p + 24));
    } else if (nwalk != (uint64_t)h.message_count || (end & kStopBit) || end != bl) {
        kind = IGGY_ERR_VALIDATION;
        reason = IGGY_V_FRAMES_DO_NOT_TILE;
    } else if (VERIFY && computed != h.batch_checksum) {
        kind = IGGY_ERR_INVALID_BATCH_CHECKSUM;
        a = h.batch_checksum; b = computed; c = h.base_offset;
    }
    write_result(result, hi, kind, reason, a, b, c, nwalk, computed, 3, kStatusDone, end & ~kStopBit);
}

template __global__ void k_decode_stream<true>(const uint8_t *__restrict__, uint64_t, uint64_t *, uint64_t,
                                               iggy_decode_result *, GeneralScratch, StreamScratch);
template __global__ void k_decode_stream<false>(const uint8_t *__restrict__, uint64_t, uint64_t *, uint64_t,
                                                iggy_decode_result *, GeneralScratch, StreamScratch);

}  // namespace iggy
