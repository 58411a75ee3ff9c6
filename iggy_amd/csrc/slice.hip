// slice.hip — the poll path's per-batch selection on a decoded, device-resident
// record: select_batch_slice (core/partitions/src/journal.rs:1025-1086) and the
// rewritten header push_selected_batch_fragments serves a partial selection with
// (journal.rs:1096-1137: clamped length and count, batch checksum recomputed over
// the selected frames via checksum_for_blob, batch.rs:174-176).
//
// The reference walks the frames serially. Here:
//  k_slice_stop  : first frame whose offset (base_offset + offset_delta) exceeds the
//                  ceiling (the walk breaks there, journal.rs:1048-1050);
//  k_slice_count : selected frames (before the stop) per 1024-frame tile;
//  k_slice_pick  : one WG: the first selected frame and the frame at which the
//                  running count reaches `remaining` (journal.rs:1075-1077), by a
//                  serial scan of the tile counts and a block scan inside two tiles;
//  then the batch checksum kernels over frames first..last (CsSource.first) and
//  k_slice_finish writes the result and the 256 header bytes.
// Frames between the first and last selected ones that are not selected
// themselves (non-monotone offsets) stay inside the byte range and the checksum
// but not in matched_messages, exactly as in the reference loop.
#include "codec_common.hpp"

namespace iggy {

constexpr uint32_t kSliceTile = 1024;

struct SliceScratch {
    uint64_t *stop;          // [1] min index of a frame above the ceiling (~0 = none); reset per call
    uint32_t *tile_cnt;      // [ntiles]
    iggy_batch_header *hdr;  // header the checksum covers (rewritten)
    uint64_t *nsel;          // [1] frames walked inside the slice
    uint64_t *first;         // [1] first frame of the slice
    uint32_t *skip;          // [1] 1 = no checksum to compute (none selected, or full body)
    uint64_t *computed;      // [1]
};

__device__ __forceinline__ uint64_t slice_offset(const uint8_t *blob, const uint64_t *pos, uint64_t base,
                                                 uint64_t i) {
    return base + (uint64_t)ld32_any(blob + pos[i] + 24);  // wrapping add, as in release Rust
}
__device__ __forceinline__ bool slice_selected(const iggy_slice_query &q, uint64_t off, uint64_t base_ts) {
    return q.kind == IGGY_LOOKUP_OFFSET ? off >= q.value : base_ts >= q.value;  // journal.rs:1052-1065
}

// `gate` (nullable, device): 1 = this batch is not selected from at all (a chunk
// walk that already stopped); `d_matched` (nullable, device) replaces
// q.already_matched with the running count of a chunk walk.
__global__ __launch_bounds__(256) void k_slice_stop(const uint8_t *rec, const uint64_t *pos, uint64_t n,
                                                    iggy_slice_query q, uint64_t *stop, const uint32_t *gate) {
    if (gate && *gate) return;
    const uint64_t base = ld64_any(rec + 8);
    const uint8_t *blob = rec + kHdr;
    uint64_t mine = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        if (slice_offset(blob, pos, base, i) > q.ceiling) { mine = i; break; }  // ascending per thread
    for (int d = 32; d; d >>= 1) {
        const uint64_t o = __shfl_xor(mine, d);
        mine = o < mine ? o : mine;
    }
    if ((threadIdx.x & 63) == 0 && mine != ~0ull) atomicMin((unsigned long long *)stop, (unsigned long long)mine);
}

__global__ __launch_bounds__(256) void k_slice_count(const uint8_t *rec, const uint64_t *pos, uint64_t n,
                                                     iggy_slice_query q, const uint64_t *stop, uint32_t *tile_cnt,
                                                     const uint32_t *gate) {
    if (gate && *gate) return;
    __shared__ uint32_t part[4];
    const uint64_t base = ld64_any(rec + 8), bts = ld64_any(rec + 16);
    const uint8_t *blob = rec + kHdr;
    const uint64_t lim = *stop < n ? *stop : n;
    const uint64_t t0 = (uint64_t)blockIdx.x * kSliceTile;
    uint32_t c = 0;
    for (uint32_t k = threadIdx.x; k < kSliceTile; k += 256) {
        const uint64_t i = t0 + k;
        if (i < lim && slice_selected(q, slice_offset(blob, pos, base, i), bts)) ++c;
    }
    for (int d = 32; d; d >>= 1) c += __shfl_xor(c, d);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// index of the `need`-th (1-based) selected frame of tile t, whole WG
__device__ uint64_t slice_nth(const uint8_t *blob, const uint64_t *pos, uint64_t lim, const iggy_slice_query &q,
                              uint64_t base, uint64_t bts, uint64_t t, uint32_t need, uint32_t *sh) {
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = t * kSliceTile + 4ull * tid;  // 4 consecutive frames per thread
    bool sel[4];
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t i = i0 + k;
        sel[k] = i < lim && slice_selected(q, slice_offset(blob, pos, base, i), bts);
        c += sel[k];
    }
    sh[tid] = c;
    __syncthreads();
    for (uint32_t d = 1; d < 256; d <<= 1) {  // inclusive scan
        const uint32_t v = tid >= d ? sh[tid - d] : 0;
        __syncthreads();
        sh[tid] += v;
        __syncthreads();
    }
    const uint32_t incl = sh[tid], excl = incl - c;
    __syncthreads();
    if (excl < need && need <= incl) {
        uint32_t r = excl;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (sel[k] && ++r == need) sh[256] = (uint32_t)(4 * tid + k);
    }
    __syncthreads();
    const uint64_t idx = t * kSliceTile + sh[256];
    __syncthreads();
    return idx;
}

__global__ __launch_bounds__(256) void k_slice_pick(const uint8_t *rec, const uint64_t *pos, uint64_t n,
                                                    iggy_slice_query q, const uint32_t *tile_cnt, uint64_t ntiles,
                                                    SliceScratch ss, iggy_slice_result *res, const uint32_t *gate,
                                                    const uint32_t *d_matched) {
    __shared__ uint32_t sh[257];
    if (gate && *gate) {
        if (threadIdx.x == 0) {
            *res = iggy_slice_result{};
            *ss.skip = 1;
            *ss.nsel = 0;
            *ss.first = 0;
        }
        return;
    }
    if (d_matched) q.already_matched = *d_matched;
    __shared__ uint64_t plan[5];  // first tile, last tile, need in the last tile, matched, status
    const uint8_t *blob = rec + kHdr;
    iggy_batch_header h{};
    h.partition_id = ld64_any(rec + 0);
    h.base_offset = ld64_any(rec + 8);
    h.base_timestamp = ld64_any(rec + 16);
    h.origin_timestamp = ld64_any(rec + 24);
    h.batch_length = ld64_any(rec + 32);
    h.batch_checksum = ld64_any(rec + 40);
    h.message_count = ld32_any(rec + 48);
    const uint64_t lim = *ss.stop < n ? *ss.stop : n;
    const uint32_t remaining = q.count > q.already_matched ? q.count - q.already_matched : 0;  // journal.rs:1030
    if (threadIdx.x == 0) {
        uint64_t ft = ~0ull, tt = ~0ull, need = 0, acc = 0;
        if (remaining != 0 && h.message_count != 0) {  // journal.rs:1032-1034
            uint64_t lt = ~0ull, lt_cnt = 0;
            for (uint64_t t = 0; t < ntiles && t * kSliceTile < lim; ++t) {
                const uint32_t c = tile_cnt[t];
                if (!c) continue;
                if (ft == ~0ull) ft = t;
                if (acc + c >= remaining) { tt = t; need = remaining - acc; acc = remaining; break; }
                acc += c;
                lt = t;
                lt_cnt = c;
            }
            if (tt == ~0ull && lt != ~0ull) { tt = lt; need = lt_cnt; }  // fewer than remaining: last selected
        }
        plan[0] = ft; plan[1] = tt; plan[2] = need; plan[3] = acc; plan[4] = ft != ~0ull;
    }
    __syncthreads();
    if (!plan[4]) {  // None (journal.rs:1080-1085: `start?`)
        if (threadIdx.x == 0) {
            iggy_slice_result r{};
            r.header = h;
            *res = r;
            *ss.skip = 1;
            *ss.nsel = 0;
            *ss.first = 0;
            *ss.hdr = h;
        }
        return;
    }
    const uint64_t base = h.base_offset, bts = h.base_timestamp;
    const uint64_t first = slice_nth(blob, pos, lim, q, base, bts, plan[0], 1, sh);
    const uint64_t last = slice_nth(blob, pos, lim, q, base, bts, plan[1], (uint32_t)plan[2], sh);
    if (threadIdx.x == 0) {
        const uint64_t start = pos[first], lp = pos[last];
        const uint64_t end = lp + kFrameHdr + ld32_any(blob + lp + 36) + ld32_any(blob + lp + 32);
        const uint64_t blob_len = h.batch_length - kHdr;
        iggy_slice_result r{};
        r.selected = 1;
        r.full_body = start == 0 && end == blob_len;  // journal.rs:1105
        r.start = start;
        r.end = end;
        r.matched_messages = (uint32_t)plan[3];
        r.last_matching_offset = slice_offset(blob, pos, base, last);
        iggy_batch_header w = h;
        if (!r.full_body) {  // journal.rs:1114-1124
            w.batch_length = kHdr + (end - start);
            w.message_count = r.matched_messages;
        }
        r.header = w;
        *res = r;
        *ss.hdr = w;
        *ss.first = first;
        *ss.nsel = last - first + 1;
        *ss.skip = r.full_body ? 1u : 0u;
    }
}

__global__ void k_slice_finish(const uint8_t *rec, SliceScratch ss, iggy_slice_result *res, uint8_t *header_out) {
    const int t = threadIdx.x;  // 64 threads x 4 header bytes
    if (!res->selected) return;
    iggy_batch_header h = res->header;
    if (!*ss.skip) h.batch_checksum = *ss.computed;
    if (header_out) {
        uint32_t w;
        if (res->full_body) {
            w = ld32_any(rec + 4 * t);  // the record's own header bytes
        } else {
            w = 0;
            const uint32_t off = 4 * t;
            if (off < 48) {
                const uint64_t f[6] = {h.partition_id, h.base_offset, h.base_timestamp,
                                       h.origin_timestamp, h.batch_length, h.batch_checksum};
                const uint64_t v = f[off / 8];
                w = (off & 4) ? (uint32_t)(v >> 32) : (uint32_t)v;
            } else if (off == 48) {
                w = h.message_count;
            }
        }
        *(u32_ua *)(header_out + 4 * t) = w;
    }
    __syncthreads();
    if (t == 0) res->header.batch_checksum = h.batch_checksum;
}

// stamp_prepare_for_persistence (server_common/src/send_messages.rs:642-663): the
// header the checksum covers, from the record's own fields and the new base values
__global__ void k_stamp_prep(const uint8_t *rec, uint64_t base_offset, uint64_t base_timestamp, uint64_t nframes,
                             iggy_batch_header *hdr, uint64_t *nframes_out) {
    if (threadIdx.x != 0) return;
    iggy_batch_header h{};
    h.partition_id = ld64_any(rec + 0);
    h.base_offset = base_offset;
    h.base_timestamp = base_timestamp;
    h.origin_timestamp = ld64_any(rec + 24);
    h.batch_length = ld64_any(rec + 32);
    h.batch_checksum = 0;
    h.message_count = ld32_any(rec + 48);
    *hdr = h;
    *nframes_out = nframes;
}

__global__ void k_stamp_finish(uint8_t *rec, const iggy_batch_header *hdr, const uint64_t *cs,
                               iggy_batch_header *out) {
    const int t = threadIdx.x;  // 64 threads x 4 bytes of the 52 header bytes that change
    iggy_batch_header h = *hdr;
    h.batch_checksum = *cs;
    const uint32_t off = 4 * t;
    if (off < 48) {
        const uint64_t f[6] = {h.partition_id, h.base_offset, h.base_timestamp,
                               h.origin_timestamp, h.batch_length, h.batch_checksum};
        const uint64_t v = f[off / 8];
        *(u32_ua *)(rec + off) = (off & 4) ? (uint32_t)(v >> 32) : (uint32_t)v;
    }
    if (t == 0 && out) *out = h;
}

// ---- walk_disk_chunk (core/partitions/src/poll_plan.rs:950-1011): the walk's
// state lives on the device so that every batch of a chunk is verified, gated and
// selected in one enqueue (the running match count feeds the next selection).
struct ChunkState {
    uint32_t stopped, corrupt, matched, nfrag;
    uint64_t consumed, last_matching_offset, has_last, batches;
    iggy_wire_error error;
};

__global__ void k_chunk_init(ChunkState *st, uint32_t already_matched) {
    if (threadIdx.x == 0) {
        ChunkState z{};
        z.matched = already_matched;
        *st = z;
    }
}

// before batch k: the loop condition (:963) and the decode verdict (:964-988)
__global__ void k_chunk_gate(const iggy_decode_result *res, uint64_t pos, uint32_t count, ChunkState *st,
                             uint32_t *gate) {
    if (threadIdx.x != 0) return;
    uint32_t g = 1;
    if (!st->stopped) {
        if (st->matched >= count) {
            st->stopped = 1;
            st->consumed = pos;
        } else if (res->error.kind != IGGY_OK) {
            // InvalidBatchChecksum: damaged at rest (:966-983); anything else: incomplete tail (:984-987)
            st->stopped = 1;
            st->consumed = pos;
            st->corrupt = res->error.kind == IGGY_ERR_INVALID_BATCH_CHECKSUM ? 1u : 0u;
            st->error = res->error;
        } else {
            g = 0;
        }
    }
    *gate = g;
}

// after batch k's selection: push_selected_batch_fragments (journal.rs:1096-1137)
// and the cursor advance (:1003)
__global__ void k_chunk_after(const iggy_slice_result *sr, const uint8_t *hdr_bytes, uint64_t pos, uint64_t total,
                              ChunkState *st, const uint32_t *gate, iggy_chunk_fragment *frags, uint8_t *headers,
                              uint64_t cap) {
    if (*gate) return;
    const int t = threadIdx.x;  // 64 threads
    const uint32_t idx = st->nfrag;
    const bool sel = sr->selected != 0;
    __syncthreads();
    if (sel && idx < cap) {
        if (headers) *(u32_ua *)(headers + 256ull * idx + 4 * t) = *(const u32_ua *)(hdr_bytes + 4 * t);
        if (t == 0) {
            iggy_chunk_fragment f{};
            f.batch_pos = pos;
            f.full_body = sr->full_body;
            f.matched_messages = sr->matched_messages;
            f.body_start = sr->full_body ? pos : pos + kHdr + sr->start;
            f.body_end = sr->full_body ? pos + total : pos + kHdr + sr->end;
            f.last_matching_offset = sr->last_matching_offset;
            frags[idx] = f;
        }
    }
    if (t == 0) {
        if (sel) {
            st->nfrag = idx + 1;
            st->matched += sr->matched_messages;
            st->last_matching_offset = sr->last_matching_offset;
            st->has_last = 1;
        }
        st->consumed = pos + total;
        st->batches += 1;
    }
}


// ---- walk_disk_chunk in ONE launch after the chunk's batches are decoded by
// k_decode_records (decode_records.hip): one workgroup per batch. Each computes
// what it can alone (the ceiling stop and the selected-frame counts), then takes
// the walk state after batch k - 1 from its predecessor (decoupled look-back on a
// published, epoch-tagged link: workgroups are dispatched in order, so the one
// waited on is always resident or done), applies the loop condition and the
// decode verdict (poll_plan.rs:963-988), selects (journal.rs:1025-1086),
// recomputes a partial selection's batch checksum (batch.rs:439-450 via
// checksum_for_blob), pushes the fragment (journal.rs:1096-1137) and publishes
// the walk state after batch k.
struct ChunkCand {
    uint64_t pos;    // chunk offset of the batch header
    uint64_t bl;     // batch_length (0: the header did not decode or the batch does not fit)
    uint64_t pbase;  // its frame positions: pos_all[pbase + i]
    uint64_t bbase;  // its block-sum scratch: bsums[8 * (bbase + b) + j]
};
struct ChunkLink {
    ChunkState st;  // the walk state after this batch
    uint32_t ready; // == epoch once st is published
    uint32_t _pad[7];
};
constexpr uint32_t kChunkThreads = 256;
// Host callers may pass cands in host-mapped memory and frags / headers / out_state
// there too; the last batch's workgroup then raises host_flag (launch completion
// without a stream sync or a D2H copy).

__global__ __launch_bounds__(kChunkThreads) void k_chunk_walk(const uint8_t *__restrict__ chunk,
                                                              const ChunkCand *__restrict__ cands, uint32_t K,
                                                              const iggy_decode_result *__restrict__ dres,
                                                              const uint64_t *__restrict__ pos_all,
                                                              iggy_slice_query q, uint32_t epoch, ChunkLink *links,
                                                              ChunkState *out_state, iggy_chunk_fragment *frags,
                                                              uint8_t *headers, uint64_t cap, uint64_t *bsums_all,
                                                              uint32_t *host_flag, uint32_t flag_value) {
    __shared__ uint64_t s_red[kChunkThreads / 64];
    __shared__ uint32_t s_cnt[kChunkThreads];
    __shared__ ChunkState s_st;
    __shared__ uint64_t s_sel[4];  // first, last, matched, selected
    __shared__ uint8_t s_small[256];
    const uint32_t k = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    const int lane = tid & 63;
    const ChunkCand cd = cands[k];
    const iggy_decode_result res = dres[k];
    const bool ok = res.error.kind == IGGY_OK && res.status == kStatusDone && cd.bl != 0;
    const uint8_t *rec = chunk + cd.pos;
    const uint8_t *blob = rec + kHdr;
    const uint64_t *pos = pos_all + cd.pbase;
    const uint64_t nf = ok ? res.frame_count : 0;
    const iggy_batch_header h = res.header;
    auto wmin = [&](uint64_t v) -> uint64_t {
        for (int d = 32; d; d >>= 1) {
            const uint64_t o = __shfl_xor(v, d);
            v = o < v ? o : v;
        }
        if (lane == 0) s_red[tid >> 6] = v;
        __syncthreads();
        uint64_t m = s_red[0];
        for (uint32_t w = 1; w < kChunkThreads / 64; ++w) m = s_red[w] < m ? s_red[w] : m;
        __syncthreads();
        return m;
    };
    // 1. alone: the first frame above the ceiling (the walk breaks there, journal.rs:1048-1050)
    //    and the selected frames before it, a contiguous range per thread
    uint64_t mine = ~0ull;
    for (uint64_t i = tid; i < nf; i += kChunkThreads)
        if (slice_offset(blob, pos, h.base_offset, i) > q.ceiling) { mine = i; break; }
    const uint64_t stop = wmin(mine);
    const uint64_t lim = stop < nf ? stop : nf;
    const uint64_t F = (lim + kChunkThreads - 1) / kChunkThreads;
    const uint64_t r0 = min((uint64_t)tid * F, lim), r1 = min(r0 + F, lim);
    uint32_t c = 0;
    for (uint64_t i = r0; i < r1; ++i) c += slice_selected(q, slice_offset(blob, pos, h.base_offset, i), h.base_timestamp);
    s_cnt[tid] = c;
    __syncthreads();
    for (uint32_t d = 1; d < kChunkThreads; d <<= 1) {  // inclusive scan of the per-thread counts
        const uint32_t v = tid >= d ? s_cnt[tid - d] : 0;
        __syncthreads();
        s_cnt[tid] += v;
        __syncthreads();
    }
    const uint32_t incl = s_cnt[tid], excl = incl - c, total = s_cnt[kChunkThreads - 1];
    // 2. the walk state after batch k - 1
    if (tid == 0) {
        ChunkState st{};
        if (k == 0) {
            st.matched = q.already_matched;
        } else {
            const uint64_t t0 = rt_now();
            bool timed_out = false;
            while (__hip_atomic_load(&links[k - 1].ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
                __builtin_amdgcn_s_sleep(1);
                if (rt_now() - t0 > kSpinLimitTicks) { timed_out = true; break; }
            }
            if (timed_out) {
                st.stopped = 1;
                st.error.kind = IGGY_ERR_TIMEOUT;
            } else {
                st = links[k - 1].st;
            }
        }
        s_st = st;
    }
    __syncthreads();
    ChunkState st = s_st;
    bool sel_live = false;
    uint32_t remaining = 0;
    if (!st.stopped) {  // the loop condition and the decode verdict (poll_plan.rs:963-988)
        if (st.matched >= q.count) {
            st.stopped = 1;
            st.consumed = cd.pos;
        } else if (!ok) {
            st.stopped = 1;
            st.consumed = cd.pos;
            st.corrupt = res.error.kind == IGGY_ERR_INVALID_BATCH_CHECKSUM ? 1u : 0u;
            st.error = res.error;
            if (res.status != kStatusDone) st.error.kind = IGGY_ERR_PENDING;  // host re-walks (general record)
        } else {
            remaining = q.count > st.matched ? q.count - st.matched : 0;  // journal.rs:1030
            sel_live = remaining != 0 && h.message_count != 0 && total != 0;  // :1032-1034, `start?`
        }
    }
    // 3. selection: the first selected frame and the min(remaining, total)-th
    if (tid == 0) s_sel[3] = 0;
    __syncthreads();
    if (sel_live) {
        const uint32_t need = remaining < total ? remaining : total;
        if (c && excl == 0) {  // the first selected frame
            for (uint64_t i = r0; i < r1; ++i)
                if (slice_selected(q, slice_offset(blob, pos, h.base_offset, i), h.base_timestamp)) { s_sel[0] = i; break; }
        }
        if (c && excl < need && need <= incl) {
            uint32_t r = excl;
            for (uint64_t i = r0; i < r1; ++i)
                if (slice_selected(q, slice_offset(blob, pos, h.base_offset, i), h.base_timestamp) && ++r == need) {
                    s_sel[1] = i;
                    break;
                }
        }
        if (tid == 0) { s_sel[2] = need; s_sel[3] = 1; }
    }
    __syncthreads();
    iggy_chunk_fragment fr{};
    bool pushed = false;
    iggy_batch_header w = h;
    if (s_sel[3]) {
        const uint64_t first = s_sel[0], last = s_sel[1];
        const uint64_t start = pos[first], lp = pos[last];
        const uint64_t end = lp + kFrameHdr + ld32_any(blob + lp + 36) + ld32_any(blob + lp + 32);
        const uint64_t blob_len = h.batch_length - kHdr;
        const bool full = start == 0 && end == blob_len;  // journal.rs:1105
        if (!full) {  // journal.rs:1114-1124: clamped length and count, checksum over the slice
            w.batch_length = kHdr + (end - start);
            w.message_count = (uint32_t)s_sel[2];
            const uint64_t nsel = last - first + 1;
            const CsSource src{nullptr, blob, pos + first};
            const CsPlan cp = cs_plan(nsel);
            uint64_t computed = 0;
            if (cp.long_cs) {
                uint64_t *bs = bsums_all + 8 * cd.bbase;
                const uint64_t sec[2] = {block_word_secret(0, lane), block_word_secret(1, lane)};
                for (uint64_t b = tid >> 6; b <= cp.nb; b += kChunkThreads / 64) {
                    uint64_t x = 0, y = 0;
#pragma unroll
                    for (int half = 0; half < 2; ++half) {
                        const uint64_t m = 128 * b + 64 * half + lane;
                        if (m < cp.Mreg) {
                            const uint64_t v = cs_word(m, w, src);
                            y += v;
                            x += mul32x32(v ^ sec[half]);
                        }
                    }
                    x += __shfl_xor(x, 8); y += __shfl_xor(y, 8);
                    x += __shfl_xor(x, 16); y += __shfl_xor(y, 16);
                    x += __shfl_xor(x, 32); y += __shfl_xor(y, 32);
                    const uint64_t t8 = x + __shfl_xor(y, 1);
                    if (lane < 8) bs[b * 8 + lane] = t8;
                }
                __syncthreads();  // (workgroup-scope fence: the block sums are visible to wave 0)
                if (tid < 64) {
                    const int j = lane & 7;
                    uint64_t acc = chain_blocks(bs, cp.nb, lane);
                    acc += bs[cp.nb * 8 + j];
                    const uint64_t v = src(nsel - 8 + j);
                    acc += __shfl_xor(v, 1);
                    acc += mul32x32(v ^ kSecretLast[j]);
                    uint64_t a[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) a[i] = __shfl(acc, i);
                    uint64_t r = cp.n * P64_1;
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        r += fold64(a[2 * i] ^ Secret::w(11 + 16 * i), a[2 * i + 1] ^ Secret::w(19 + 16 * i));
                    computed = avalanche(r);
                }
            } else if (tid == 0) {
                for (uint64_t m = 0; m < 5; ++m) st64_any(s_small + 8 * m, cs_word(m, w, src));
                *(u32_ua *)(s_small + 40) = w.message_count;
                for (uint64_t i = 0; i < nsel; ++i) st64_any(s_small + 44 + 8 * i, src(i));
                computed = xxh3_64_lane(s_small, cp.n);
            }
            w.batch_checksum = computed;  // (thread 0's value is the one used below)
        }
        fr.batch_pos = cd.pos;
        fr.full_body = full ? 1u : 0u;
        fr.matched_messages = (uint32_t)s_sel[2];
        fr.body_start = full ? cd.pos : cd.pos + kHdr + start;
        fr.body_end = full ? cd.pos + h.batch_length : cd.pos + kHdr + end;
        fr.last_matching_offset = slice_offset(blob, pos, h.base_offset, last);
        pushed = true;
        // the header bytes served with the fragment: the record's own (full body) or rewritten
        const uint32_t idx = st.nfrag;
        if (headers && idx < cap && tid < 64) {
            const uint64_t wcs = __shfl(w.batch_checksum, 0);
            uint32_t word;
            const uint32_t off = 4 * tid;
            if (full) {
                word = ld32_any(rec + off);
            } else {
                word = 0;
                const uint64_t f[6] = {w.partition_id, w.base_offset, w.base_timestamp,
                                       w.origin_timestamp, w.batch_length, wcs};
                if (off < 48) word = (off & 4) ? (uint32_t)(f[off / 8] >> 32) : (uint32_t)f[off / 8];
                else if (off == 48) word = w.message_count;
            }
            *(u32_ua *)(headers + 256ull * idx + off) = word;
        }
    }
    if (host_flag) __threadfence_system();  // every wave's header bytes, before thread 0 publishes
    __syncthreads();
    if (tid != 0) return;
    if (!st.stopped) {  // push_selected_batch_fragments and the cursor advance (:1003)
        if (pushed) {
            if (st.nfrag < cap) frags[st.nfrag] = fr;
            st.nfrag += 1;
            st.matched += fr.matched_messages;
            st.last_matching_offset = fr.last_matching_offset;
            st.has_last = 1;
        }
        st.consumed = cd.pos + cd.bl;
        st.batches += 1;
    }
    links[k].st = st;
    // frags / headers / out_state may be host-mapped memory: system scope before the
    // link, so the last workgroup's flag covers every earlier workgroup's writes
    if (host_flag) __threadfence_system();
    __hip_atomic_store(&links[k].ready, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    if (k + 1 == K) {
        *out_state = st;
        if (host_flag) {
            __threadfence_system();
            __hip_atomic_store(host_flag, flag_value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

}  // namespace iggy
