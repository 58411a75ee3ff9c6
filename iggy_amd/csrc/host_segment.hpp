// host_segment.hpp -- segment files: boot recovery walk, state-transfer walk, segment writes
// of device records
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

extern "C" {

// recover_segment_bounds' index-less walk (core/partitions/src/segment_recovery.rs:425-530).
// The chain of candidate batches depends on headers only (decode, extent, offset
// contiguity), so the host walks it first; every candidate is then verified on the
// GPU from one copy of the file (decodes queued back to back, one sync), and the
// first candidate that fails verification ends the accepted chain.
int iggy_codec_recover_segment(iggy_codec_ctx *c, const uint8_t *messages, uint64_t len,
                               uint64_t start_offset, iggy_segment_recovery *out) {
    if (!c || !out || (!messages && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    memset(out, 0, sizeof(*out));
    auto sat = [](uint64_t a, uint64_t b) { return a + b < a ? ~0ull : a + b; };
    struct Cand { uint64_t pos; iggy_batch_header h; };
    std::vector<Cand> cand;
    uint64_t pos = 0, expected = start_offset, maxlen = 0;
    while (pos < len) {
        iggy_batch_header h;
        iggy_wire_error e;
        if (len - pos < 256 || iggy_batch_header_decode(messages + pos, 256, &h, &e)) break;
        const uint64_t extent = sat(pos, h.batch_length);
        if (extent > len || h.base_offset != expected) break;
        cand.push_back({pos, h});
        maxlen = std::max(maxlen, h.batch_length);
        if (h.message_count > 0) expected = sat(sat(h.base_offset, (uint64_t)h.message_count - 1), 1);
        pos = extent;
    }
    size_t accepted = 0;
    if (!cand.empty()) {
        // one copy of the file, every candidate verified in one multi-record launch
        // (the single-record decode for the rest), one sync
        const uint64_t span = cand.back().pos + cand.back().h.batch_length;
        const size_t K = cand.size();
        if (c->din.ensure(span + 16)) return IGGY_ERR_DEVICE;
        (void)maxlen;
        int r = put_host(c, c->din.p, messages, span, c->stream);
        if (r) return r;
        std::vector<RecIn> recs(K);
        for (size_t k = 0; k < K; ++k) recs[k] = RecIn{cand[k].pos, cand[k].h.batch_length, 0, 0, 0};
        std::vector<iggy_decode_result> res(K);
        r = decode_records_to_host(c, c->din.as<uint8_t>(), messages, recs.data(), K, IGGY_INTEGRITY_VERIFY,
                                   res.data());
        if (r) return r;
        for (; accepted < K; ++accepted)
            if (res[accepted].error.kind != IGGY_OK) break;
    }
    uint64_t end_offset = start_offset, end_ts = 0, start_ts = 0, walked = 0;
    bool have_start = false;
    for (size_t k = 0; k < accepted; ++k) {
        const iggy_batch_header &h = cand[k].h;
        if (h.message_count > 0) {
            end_offset = sat(h.base_offset, (uint64_t)h.message_count - 1);
            end_ts = h.base_timestamp;
            if (!have_start) { start_ts = h.base_timestamp; have_start = true; }
        }
        walked = cand[k].pos + h.batch_length;
    }
    out->found = have_start ? 1 : 0;
    out->start_timestamp = start_ts;
    out->end_timestamp = end_ts;
    out->end_offset = end_offset;
    out->walked_bytes = walked;
    out->batches = accepted;
    return 0;
}

// walk_segment_payload (core/partitions/src/state_transfer.rs:715-833). The batch
// extents follow from the headers (host); every batch is Verify-decoded on the GPU
// (one copy, all queued, one sync); the verdicts and the header-level checks are
// then applied in walk order, so the first invalid byte decides, as in the reference.
int iggy_codec_walk_segment_payload(iggy_codec_ctx *c, const uint8_t *bytes, uint64_t len, uint64_t base_offset,
                                    uint8_t *index_out, uint64_t index_cap, iggy_segment_walk *out) {
    if (!c || !out || (!bytes && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    memset(out, 0, sizeof(*out));
    struct Cand { uint64_t pos; iggy_batch_header h; bool ok; };
    std::vector<Cand> cand;
    uint64_t pos = 0, maxlen = 256;
    while (pos < len) {
        iggy_batch_header h{};
        iggy_wire_error e;
        const bool ok = iggy_batch_header_decode(bytes + pos, len - pos, &h, &e) == 0 && h.batch_length <= len - pos;
        cand.push_back({pos, h, ok});
        if (!ok) break;  // its decode reports the error at this position
        maxlen = std::max(maxlen, h.batch_length);
        pos += h.batch_length;
    }
    std::vector<iggy_decode_result> res(cand.size());
    if (!cand.empty()) {
        // one copy, every batch in one multi-record launch (single-record decode for the
        // rest), one sync
        const size_t K = cand.size();
        if (c->din.ensure(len + 16)) return IGGY_ERR_DEVICE;
        (void)maxlen;
        int r = put_host(c, c->din.p, bytes, len, c->stream);
        if (r) return r;
        std::vector<RecIn> recs(K);
        for (size_t k = 0; k < K; ++k) recs[k] = RecIn{cand[k].pos, len - cand[k].pos, 0, 0, 0};
        r = decode_records_to_host(c, c->din.as<uint8_t>(), bytes, recs.data(), K, IGGY_INTEGRITY_VERIFY,
                                       res.data());
        if (r) return r;
    }
    uint64_t next_offset = base_offset, indexed = 0, nidx = 0;
    bool have_stats = false, have_index = false;
    for (size_t k = 0; k < cand.size(); ++k) {
        const iggy_decode_result &rs = res[k];
        const uint64_t position = cand[k].pos;
        if (rs.error.kind == IGGY_ERR_TIMEOUT) {
            reset_after_timeout(c);
            return IGGY_ERR_TIMEOUT;
        }
        if (rs.error.kind != IGGY_OK) {  // :750-755, batch_error's mapping
            out->error = IGGY_SEG_BATCH;
            out->position = position;
            out->source = rs.error;
            server_error((int)rs.error.kind, &out->source);
            return 0;
        }
        const iggy_batch_header &h = rs.header;
        if (!have_stats && h.base_offset != base_offset) {
            out->error = IGGY_SEG_BASE_OFFSET_MISMATCH;
            out->expected = base_offset;
            out->actual = h.base_offset;
            return 0;
        }
        if (h.base_offset != next_offset) {
            out->error = IGGY_SEG_NON_CONTIGUOUS;
            out->expected = next_offset;
            out->actual = h.base_offset;
            return 0;
        }
        if (h.message_count == 0) {
            out->error = IGGY_SEG_BATCH;
            out->position = position;
            set_err(&out->source, IGGY_ERR_INVALID_MESSAGES_COUNT);
            return 0;
        }
        const uint64_t add = (uint64_t)h.message_count - 1;
        if (h.base_offset > ~0ull - add) {
            out->error = IGGY_SEG_OFFSET_OVERFLOW;
            out->position = position;
            return 0;
        }
        const uint64_t batch_end = h.base_offset + add, ts = h.base_timestamp;
        if (!have_index || position - indexed >= 64 * 1024) {  // INDEX_STRIDE_BYTES (:2799)
            have_index = true;
            indexed = position;
            if (index_out && nidx < index_cap) {
                memcpy(index_out + 24 * nidx + 0, &h.base_offset, 8);
                memcpy(index_out + 24 * nidx + 8, &ts, 8);
                memcpy(index_out + 24 * nidx + 16, &position, 8);
            }
            ++nidx;
        }
        if (!have_stats) {
            out->start_timestamp = ts;
            out->max_timestamp = ts;
        } else if (ts > out->max_timestamp) {
            out->max_timestamp = ts;
        }
        have_stats = true;
        out->end_offset = batch_end;
        out->end_timestamp = ts;
        out->batches++;
        if (batch_end == ~0ull) {
            out->error = IGGY_SEG_OFFSET_OVERFLOW;
            out->position = position;
            return 0;
        }
        next_offset = batch_end + 1;
    }
    out->index_entries = nidx;
    if (!have_stats) {
        out->error = IGGY_SEG_EMPTY;
        return 0;
    }
    return nidx > index_cap && index_out ? IGGY_ERR_CAPACITY : 0;
}

int iggy_codec_segment_write_device(iggy_codec_ctx *c, int fd, uint64_t position, const uint8_t *d_bytes,
                                    uint64_t len, int fsync, uint64_t *written) {
    if (!c || fd < 0 || (!d_bytes && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    if (written) *written = 0;
    constexpr uint64_t kPiece = 8ull << 20;  // two 8 MiB pinned halves
    if (!c->wstage) {
        if (hipHostMalloc(&c->wstage, 2 * kPiece, hipHostMallocDefault) != hipSuccess) {
            c->wstage = nullptr;
            return IGGY_ERR_DEVICE;
        }
        for (auto &ev : c->wev)
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return IGGY_ERR_DEVICE;
    }
    const uint64_t npieces = (len + kPiece - 1) / kPiece;
    auto issue = [&](uint64_t k) -> int {
        const uint64_t off = k * kPiece, n = std::min(kPiece, len - off);
        HIP_OK(hipMemcpyAsync((uint8_t *)c->wstage + (k & 1) * kPiece, d_bytes + off, n, hipMemcpyDeviceToHost,
                              c->stream));
        HIP_OK(hipEventRecord(c->wev[k & 1], c->stream));
        return 0;
    };
    int r = npieces ? issue(0) : 0;
    for (uint64_t k = 0; k < npieces && !r; ++k) {
        HIP_OK(hipEventSynchronize(c->wev[k & 1]));
        if (k + 1 < npieces) r = issue(k + 1);  // the next piece's copy runs under this pwrite
        const uint64_t off = k * kPiece, n = std::min(kPiece, len - off);
        const uint8_t *src = (const uint8_t *)c->wstage + (k & 1) * kPiece;
        uint64_t done = 0;
        while (done < n) {
            const ssize_t w = pwrite(fd, src + done, n - done, (off_t)(position + off + done));
            if (w <= 0) {
                if (w < 0 && errno == EINTR) continue;
                (void)hipStreamSynchronize(c->stream);
                return IGGY_ERR_DEVICE;
            }
            done += (uint64_t)w;
        }
        if (written) *written += n;
    }
    if (r) return r;
    if (fsync && fdatasync(fd) != 0) return IGGY_ERR_DEVICE;
    return 0;
}

}  // extern "C"
