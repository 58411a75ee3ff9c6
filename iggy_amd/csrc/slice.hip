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

}  // namespace iggy
