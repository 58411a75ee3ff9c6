// host_slice.hpp -- poll-path slicing, the disk-chunk walk and the device stamp
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

extern "C" {

// ------------------------------------------------- poll-path slicing / stamp
// select_batch_slice + served header on a decoded device record (gate / d_matched:
// chunk walks, see k_chunk_gate)
static int enqueue_select(iggy_codec_ctx *c, const uint8_t *d_record, const uint64_t *d_frame_pos, uint64_t nframes,
                          const iggy_slice_query &qq, iggy_slice_result *d_out, uint8_t *d_header_out, hipStream_t s,
                          const uint32_t *gate = nullptr, const uint32_t *d_matched = nullptr) {
    const uint64_t ntiles = (nframes + kSliceTile - 1) / kSliceTile;
    int r = c->sl.ensure(512 + ntiles * 4);
    r |= c->gbsums.ensure(((44 + 8 * nframes) / 1024 + 2) * 64);
    if (r) return IGGY_ERR_DEVICE;
    SliceScratch ss;
    ss.stop = c->sl.as<uint64_t>(0);
    ss.nsel = c->sl.as<uint64_t>(8);
    ss.first = c->sl.as<uint64_t>(16);
    ss.computed = c->sl.as<uint64_t>(24);
    ss.skip = c->sl.as<uint32_t>(32);
    ss.hdr = c->sl.as<iggy_batch_header>(64);
    ss.tile_cnt = c->sl.as<uint32_t>(512);
    HIP_OK(hipMemsetAsync(ss.stop, 0xff, 8, s));
    if (nframes) {
        const uint32_t g = (uint32_t)std::min<uint64_t>((nframes + 255) / 256, (uint64_t)c->ncu * 8);
        hipLaunchKernelGGL(k_slice_stop, dim3(g), dim3(256), 0, s, d_record, d_frame_pos, nframes, qq, ss.stop, gate);
        hipLaunchKernelGGL(k_slice_count, dim3((uint32_t)ntiles), dim3(256), 0, s, d_record, d_frame_pos, nframes, qq,
                           (const uint64_t *)ss.stop, ss.tile_cnt, gate);
    }
    hipLaunchKernelGGL(k_slice_pick, dim3(1), dim3(256), 0, s, d_record, d_frame_pos, nframes, qq,
                       (const uint32_t *)ss.tile_cnt, ntiles, ss, d_out, gate, d_matched);
    CsSource src{nullptr, d_record + kHdr, d_frame_pos, ss.first};
    hipLaunchKernelGGL(k_bsum_blocks, dim3(bsum_grid(c, nframes)), dim3(256), 0, s, (const iggy_batch_header *)ss.hdr,
                       (const uint64_t *)ss.nsel, src, c->gbsums.as<uint64_t>(), (const uint32_t *)ss.skip);
    hipLaunchKernelGGL(k_bsum_chain, dim3(1), dim3(128), 0, s, (const iggy_batch_header *)ss.hdr,
                       (const uint64_t *)ss.nsel, src, (const uint64_t *)c->gbsums.as<uint64_t>(),
                       c->sl.as<uint8_t>(128), ss.computed, (const uint32_t *)ss.skip);
    hipLaunchKernelGGL(k_slice_finish, dim3(1), dim3(64), 0, s, d_record, ss, d_out, d_header_out);
    HIP_OK(hipGetLastError());
    return 0;
}

int iggy_codec_select_slice_device(iggy_codec_ctx *c, const uint8_t *d_record, const uint64_t *d_frame_pos,
                                   uint64_t nframes, const iggy_slice_query *q, iggy_slice_result *d_out,
                                   uint8_t *d_header_out, void *stream) {
    if (!c || !d_record || !q || !d_out || (nframes && !d_frame_pos)) return IGGY_ERR_INVALID_ARGUMENT;
    if (q->kind != IGGY_LOOKUP_OFFSET && q->kind != IGGY_LOOKUP_TIMESTAMP) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    hipStream_t s = bind(c, stream);
    return enqueue_select(c, d_record, d_frame_pos, nframes, *q, d_out, d_header_out, s);
}

// The per-batch form of the chunk walk: every batch's decode, gate, selection and
// fragment push enqueued one after the other (~11 stream operations per batch). Used
// for chunks holding a batch that is not single-stride, or that the one-launch form
// (below) found to need the general walk.
static int walk_chunk_per_batch(iggy_codec_ctx *c, const uint8_t *chunk, uint64_t len, const iggy_slice_query *q,
                                int integrity, iggy_chunk_fragment *frags, uint8_t *headers, uint64_t cap,
                                iggy_chunk_walk *out) {
    memset(out, 0, sizeof(*out));
    // the batch extents follow from the 256-B headers alone (host); a header that does
    // not decode or a batch that does not fit is the last candidate (its decode fails)
    struct Cand { uint64_t pos, bl, nframes, pbase; };
    std::vector<Cand> cand;
    uint64_t cursor = 0, pwords = 0, maxn = 0;
    while (cursor + 256 <= len) {
        iggy_batch_header h;
        iggy_wire_error he;
        const bool ok = iggy_batch_header_decode(chunk + cursor, len - cursor, &h, &he) == 0;
        const bool fits = ok && h.batch_length <= len - cursor;
        const uint64_t nf = fits ? (h.batch_length - 256) / 48 + 1 : 1;
        cand.push_back({cursor, fits ? h.batch_length : 0, fits ? (uint64_t)h.message_count : 0, pwords});
        pwords += nf;
        maxn = std::max(maxn, nf);
        if (!fits) break;
        cursor += h.batch_length;
    }
    const uint64_t K = cand.size();
    // device: the chunk once; per batch its Verify / LayoutOnly decode, the gate, the
    // selection (match count from the previous batch) and the fragment push; one sync
    const uint64_t kState = 256, kSlot = 512;
    int r = c->din.ensure(len + 16);
    r |= c->dpos.ensure((pwords + 1) * 8);
    r |= c->pres.ensure((K + 1) * sizeof(iggy_decode_result));
    r |= c->cwk.ensure(kState + K * (kSlot + 8) + cap * (sizeof(iggy_chunk_fragment) + 256) + 64);
    if (!r) r = ensure_decode_scratch(c, len);
    if (r) return IGGY_ERR_DEVICE;
    hipStream_t s = c->stream;
    ChunkState *st = c->cwk.as<ChunkState>(0);
    uint32_t *gates = c->cwk.as<uint32_t>(kState);
    uint8_t *slots = c->cwk.as<uint8_t>(kState + K * 8);
    iggy_chunk_fragment *d_frags = c->cwk.as<iggy_chunk_fragment>(kState + K * (kSlot + 8));
    uint8_t *d_hdrs = (uint8_t *)(d_frags + cap);
    r = put_host(c, c->din.p, chunk, len, s);
    if (r) return r;
    hipLaunchKernelGGL(k_chunk_init, dim3(1), dim3(64), 0, s, st, q->already_matched);
    iggy_decode_result *d_res = c->pres.as<iggy_decode_result>();
    for (uint64_t k = 0; k < K; ++k) {
        const Cand &cd = cand[k];
        const uint8_t *rec = c->din.as<uint8_t>(cd.pos);
        uint64_t *pos = c->dpos.as<uint64_t>(8 * cd.pbase);
        r = enqueue_decode(c, rec, len - cd.pos, integrity, pos, cd.bl ? (cd.bl - 256) / 48 + 1 : 0, d_res + k, s);
        if (r) return r;
        hipLaunchKernelGGL(k_chunk_gate, dim3(1), dim3(64), 0, s, (const iggy_decode_result *)(d_res + k), cd.pos,
                           q->count, st, gates + k);
        if (!cd.bl) break;  // its decode failed (the gate stops the walk there)
        iggy_slice_result *sr = (iggy_slice_result *)(slots + k * kSlot);
        uint8_t *hb = slots + k * kSlot + 256;
        r = enqueue_select(c, rec, pos, cd.nframes, *q, sr, hb, s, gates + k, &st->matched);
        if (r) return r;
        hipLaunchKernelGGL(k_chunk_after, dim3(1), dim3(64), 0, s, (const iggy_slice_result *)sr,
                           (const uint8_t *)hb, cd.pos, cd.bl, st, (const uint32_t *)(gates + k), d_frags, d_hdrs, cap);
    }
    HIP_OK(hipGetLastError());
    ChunkState hs{};
    r = get_host(c, &hs, st, sizeof(hs), s);
    if (r) return r;
    const uint64_t nf = std::min<uint64_t>(hs.nfrag, cap);
    if (nf) {
        r = get_host(c, frags, d_frags, nf * sizeof(iggy_chunk_fragment), s);
        if (!r && headers) r = get_host(c, headers, d_hdrs, nf * 256, s);
        if (r) return r;
    }
    if (hs.error.kind == IGGY_ERR_TIMEOUT) {  // a bug guard fired, not a verdict on the chunk
        reset_after_timeout(c);
        return IGGY_ERR_TIMEOUT;
    }
    out->consumed = std::min<uint64_t>(hs.consumed, len);
    out->corrupt = hs.corrupt;
    out->matched = hs.matched;
    out->last_matching_offset = hs.last_matching_offset;
    out->has_last_matching_offset = (uint32_t)hs.has_last;
    out->fragments = hs.nfrag;
    out->error = hs.error;
    out->batches = hs.batches;
    return hs.nfrag > cap ? IGGY_ERR_CAPACITY : 0;
}

int iggy_codec_walk_disk_chunk(iggy_codec_ctx *c, const uint8_t *chunk, uint64_t len, const iggy_slice_query *q,
                               int integrity, iggy_chunk_fragment *frags, uint8_t *headers, uint64_t cap,
                               iggy_chunk_walk *out) {
    if (!c || !q || !out || (!chunk && len) || (cap && !frags)) return IGGY_ERR_INVALID_ARGUMENT;
    if (q->kind != IGGY_LOOKUP_OFFSET && q->kind != IGGY_LOOKUP_TIMESTAMP) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    memset(out, 0, sizeof(*out));
    // the batch extents follow from the 256-B headers alone (host); a header that does
    // not decode or a batch that does not fit is the last candidate (its decode fails)
    std::vector<ChunkCand> cand;
    uint64_t cursor = 0, pwords = 0, nbb = 0;
    bool one_launch = true;
    while (cursor + 256 <= len) {
        iggy_batch_header h;
        iggy_wire_error he;
        const bool ok = iggy_batch_header_decode(chunk + cursor, len - cursor, &h, &he) == 0;
        const bool fits = ok && h.batch_length <= len - cursor;
        uint64_t nfp = 0;
        if (!rec_plan(chunk + cursor, len - cursor, &nfp)) one_launch = false;
        const uint64_t nf = fits ? (h.batch_length - 256) / 48 + 1 : 1;
        cand.push_back({cursor, fits ? h.batch_length : 0, pwords, nbb});
        pwords += nf;
        nbb += rec_blocks(nfp) + 2;
        if (!fits) break;
        cursor += h.batch_length;
    }
    const uint64_t K = cand.size();
    if (K == 0) {  // no header fits: the loop does not run (poll_plan.rs:963)
        out->matched = q->already_matched;
        return 0;
    }
    if (!one_launch) return walk_chunk_per_batch(c, chunk, len, q, integrity, frags, headers, cap, out);
    // One copy of the chunk, ONE multi-record decode launch, ONE k_chunk_walk launch
    // (one workgroup per batch: gate, selection, partial checksum, fragment push, the
    // match count handed batch to batch). The tables are read and the outputs written
    // by the kernels in host-mapped memory; the host spins on the completion flag.
    const uint64_t capk = std::min<uint64_t>(cap, K);  // at most one fragment per batch
    const size_t res_bytes = 256 + capk * (sizeof(iggy_chunk_fragment) + 256);
    const size_t cand_bytes = K * sizeof(ChunkCand), link_bytes = K * sizeof(ChunkLink);
    int r = c->din.ensure(len + 16);
    r |= c->dpos.ensure((pwords + 1) * 8);
    r |= c->pres.ensure((K + 1) * sizeof(iggy_decode_result));
    r |= c->sl.ensure(nbb * 64 + 64);
    r |= c->cmap.ensure(cand_bytes);
    r |= c->omap.ensure(64 + res_bytes);
    // the links live in a buffer of their own that only ever holds links: a stale one
    // carries an older epoch, never the current one (zeroed whenever it is new)
    const size_t links_cap_before = c->clinks.cap;
    r |= c->clinks.ensure(link_bytes);
    if (r) return IGGY_ERR_DEVICE;
    hipStream_t s = c->stream;
    // the chunk is copied (read in place over the host link, a registered 1 MiB chunk
    // walked 98-103 us against 90-93 us copied, Verify, same box: k_chunk_walk's
    // scattered reads pay a link round trip each)
    r = put_host(c, c->din.p, chunk, len, s);
    if (r) return r;
    const uint8_t *d_chunk = c->din.as<uint8_t>();
    std::vector<RecIn> rin(K);
    for (uint64_t k = 0; k < K; ++k)
        rin[k] = RecIn{cand[k].pos, len - cand[k].pos, cand[k].pbase, cand[k].bl ? (cand[k].bl - 256) / 48 + 1 : 0, 0};
    iggy_decode_result *d_res = c->pres.as<iggy_decode_result>();
    std::vector<size_t> single;
    r = enqueue_records(c, d_chunk, chunk, rin.data(), K, integrity, c->dpos.as<uint64_t>(), nullptr,
                        d_res, &single);
    if (r) return r;
    memcpy(c->cmap.h, cand.data(), cand_bytes);
    uint8_t *pin_res = c->omap.hp<uint8_t>(64);
    ChunkState *d_state = c->omap.dp<ChunkState>(64);
    iggy_chunk_fragment *d_frags = c->omap.dp<iggy_chunk_fragment>(64 + 256);
    uint8_t *d_hdrs = c->omap.dp<uint8_t>(64 + 256 + capk * sizeof(iggy_chunk_fragment));
    ChunkLink *d_links = c->clinks.as<ChunkLink>();
    if (++c->chunk_epoch == 0 || c->clinks.cap != links_cap_before) {  // new buffer or wrapped tags
        if (c->chunk_epoch == 0) c->chunk_epoch = 1;
        HIP_OK(hipMemsetAsync(c->clinks.p, 0, c->clinks.cap, s));
    }
    const uint32_t v = next_flag(c);
    hipLaunchKernelGGL(k_chunk_walk, dim3((uint32_t)K), dim3(kChunkThreads), 0, s, d_chunk,
                       c->cmap.dp<const ChunkCand>(), (uint32_t)K, (const iggy_decode_result *)d_res,
                       (const uint64_t *)c->dpos.as<uint64_t>(), *q, c->chunk_epoch, d_links, d_state, d_frags,
                       headers ? d_hdrs : nullptr, capk, c->sl.as<uint64_t>(), c->omap.dp<uint32_t>(), v);
    HIP_OK(hipGetLastError());
    r = wait_host_flag(c, v);
    if (!r) r = xfer_settle(c);
    if (r) return r;
    ChunkState hs;
    memcpy(&hs, pin_res, sizeof(hs));
    if (hs.error.kind == IGGY_ERR_PENDING)  // a batch needs the general walk: the per-batch form
        return walk_chunk_per_batch(c, chunk, len, q, integrity, frags, headers, cap, out);
    if (hs.error.kind == IGGY_ERR_TIMEOUT) {  // a bug guard fired, not a verdict on the chunk
        reset_after_timeout(c);
        return IGGY_ERR_TIMEOUT;
    }
    const uint64_t nf = std::min<uint64_t>(hs.nfrag, capk);
    if (nf) {
        memcpy(frags, pin_res + 256, nf * sizeof(iggy_chunk_fragment));
        if (headers) memcpy(headers, pin_res + 256 + capk * sizeof(iggy_chunk_fragment), nf * 256);
    }
    out->consumed = std::min<uint64_t>(hs.consumed, len);
    out->corrupt = hs.corrupt;
    out->matched = hs.matched;
    out->last_matching_offset = hs.last_matching_offset;
    out->has_last_matching_offset = (uint32_t)hs.has_last;
    out->fragments = hs.nfrag;
    out->error = hs.error;
    out->batches = hs.batches;
    return hs.nfrag > cap ? IGGY_ERR_CAPACITY : 0;
}

int iggy_codec_select_slice(iggy_codec_ctx *c, const uint8_t *record, uint64_t len, const iggy_slice_query *q,
                            iggy_slice_result *out, uint8_t *header_out, iggy_wire_error *err) {
    if (!c || !q || !out || (!record && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    set_err(err, IGGY_OK);
    const uint64_t cap = len / kFrameHdr + 1;
    int r = c->din.ensure(len + 16);
    r |= c->dpos.ensure((cap + 1) * 8);
    r |= c->slres.ensure(512);
    if (r) return IGGY_ERR_DEVICE;
    r = put_host(c, c->din.p, record, len, c->stream);
    if (r) return r;
    // the reference selects on a decoded batch: decode it (layout) first
    iggy_decode_result *d_res = c->dresult.as<iggy_decode_result>();
    r = enqueue_decode(c, c->din.as<uint8_t>(), len, IGGY_INTEGRITY_LAYOUT_ONLY, c->dpos.as<uint64_t>(), cap, d_res,
                       c->stream);
    if (r) return r;
    iggy_decode_result *h_res = (iggy_decode_result *)c->h_pinned;
    HIP_OK(hipMemcpyAsync(h_res, d_res, sizeof(*h_res), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    const iggy_decode_result res = *h_res;
    if (res.error.kind == IGGY_ERR_TIMEOUT) reset_after_timeout(c);
    if (res.error.kind != IGGY_OK) {
        fill_err(err, res.error);
        return (int)res.error.kind;
    }
    iggy_slice_result *d_out = c->slres.as<iggy_slice_result>(0);
    uint8_t *d_hdr = c->slres.as<uint8_t>(256);
    r = iggy_codec_select_slice_device(c, c->din.as<uint8_t>(), c->dpos.as<uint64_t>(), res.frame_count, q, d_out,
                                       d_hdr, c->stream);
    if (r) return r;
    uint8_t *h = (uint8_t *)c->h_pinned + 1024;
    HIP_OK(hipMemcpyAsync(h, d_out, 512, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    memcpy(out, h, sizeof(*out));
    if (header_out && out->selected) memcpy(header_out, h + 256, 256);
    return 0;
}

int iggy_codec_stamp_batch_device(iggy_codec_ctx *c, uint8_t *d_record, const uint64_t *d_frame_pos,
                                  uint64_t nframes, uint64_t base_offset, uint64_t base_timestamp,
                                  iggy_batch_header *d_header, void *stream) {
    if (!c || !d_record || (nframes && !d_frame_pos)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    hipStream_t s = bind(c, stream);
    int r = c->sl.ensure(512 + 4);
    r |= c->gbsums.ensure(((44 + 8 * nframes) / 1024 + 2) * 64);
    if (r) return IGGY_ERR_DEVICE;
    iggy_batch_header *dh = c->sl.as<iggy_batch_header>(64);
    uint64_t *dn = c->sl.as<uint64_t>(8), *dcs = c->sl.as<uint64_t>(24);
    hipLaunchKernelGGL(k_stamp_prep, dim3(1), dim3(64), 0, s, (const uint8_t *)d_record, base_offset, base_timestamp,
                       nframes, dh, dn);
    CsSource src{nullptr, d_record + kHdr, d_frame_pos};
    hipLaunchKernelGGL(k_bsum_blocks, dim3(bsum_grid(c, nframes)), dim3(256), 0, s, (const iggy_batch_header *)dh,
                       (const uint64_t *)dn, src, c->gbsums.as<uint64_t>(), nullptr);
    hipLaunchKernelGGL(k_bsum_chain, dim3(1), dim3(128), 0, s, (const iggy_batch_header *)dh, (const uint64_t *)dn,
                       src, (const uint64_t *)c->gbsums.as<uint64_t>(), c->sl.as<uint8_t>(128), dcs, nullptr);
    hipLaunchKernelGGL(k_stamp_finish, dim3(1), dim3(64), 0, s, d_record, (const iggy_batch_header *)dh,
                       (const uint64_t *)dcs, d_header);
    HIP_OK(hipGetLastError());
    return 0;
}

}  // extern "C"
