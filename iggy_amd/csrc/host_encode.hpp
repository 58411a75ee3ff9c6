// host_encode.hpp -- encode: SoA staging and the encode enqueue (segmented ring / lane-group
// kernels, batch-checksum chain on the side stream) behind the encode entry points
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

extern "C" {

// ---------------------------------------------------------------- encode
// A small encode's SoA input as device-visible host memory: every array read in place
// when all are registered (and non-empty), else all copied with one memcpy each into
// `stage` (mapped, every array 256-B aligned with 16 B of slack). dm: the result.
static int stage_soa(const iggy_raw_messages *m, uint64_t n, uint64_t spl, uint64_t suh, HostMap &stage,
                     iggy_raw_messages *dm) {
    const bool has_uh = m->user_headers_lengths != nullptr;
    struct Arr { const void *h; uint64_t len; const uint8_t *d; };
    Arr a[6] = {{m->ids, n * 16, nullptr}, {m->origin_timestamps, n * 8, nullptr},
                {m->payloads, spl, nullptr}, {m->payload_lengths, n * 4, nullptr},
                {has_uh ? m->user_headers : nullptr, has_uh ? suh : 0, nullptr},
                {has_uh ? m->user_headers_lengths : nullptr, has_uh ? n * 4 : 0, nullptr}};
    bool mapped = true;  // (an empty array takes the staging too: a valid address behind it)
    for (int i = 0; i < (has_uh ? 6 : 4); ++i)
        mapped &= a[i].len && (a[i].d = host_device_ptr(a[i].h, a[i].len)) != nullptr;
    if (!mapped) {
        uint64_t off[6], tot = 0;
        for (int i = 0; i < 6; ++i) {
            off[i] = tot;
            tot += (a[i].len + 16 + 255) & ~(uint64_t)255;
        }
        if (stage.ensure(tot)) return IGGY_ERR_DEVICE;
        for (int i = 0; i < 6; ++i) {
            if (a[i].len) memcpy(stage.hp<uint8_t>(off[i]), a[i].h, a[i].len);
            a[i].d = stage.d + off[i];
        }
    }
    dm->count = n;
    dm->ids = (const uint64_t *)a[0].d;
    dm->origin_timestamps = (const uint64_t *)a[1].d;
    dm->payloads = a[2].d;
    dm->payload_lengths = (const uint32_t *)a[3].d;
    dm->user_headers = has_uh ? a[4].d : nullptr;
    dm->user_headers_lengths = has_uh ? (const uint32_t *)a[5].d : nullptr;
    return 0;
}

static int enqueue_encode(iggy_codec_ctx *c, const iggy_raw_messages *dm, uint64_t partition_id,
                          uint8_t *d_out, uint64_t cap, iggy_encode_result *d_res, hipStream_t s,
                          EncOwn *own = nullptr) {
    // own (nullable): scratch of an asynchronous slot, so unsegmented encodes of
    // different slots run side by side on their own streams (else the context's)
    const uint64_t n = dm->count;
    DevBuf &epl = own ? own->epl : c->epl, &euh = own ? own->euh : c->euh, &etile = own ? own->etile : c->etile;
    DevBuf &ecs = own ? own->ecs : c->ecs, &emisc = own ? own->emisc : c->emisc, &bsums = own ? own->bsums : c->gbsums;
    const uint64_t ntiles = (n + kEncTile - 1) / kEncTile;
    int r = 0;
    r |= epl.ensure(n * 8);
    r |= euh.ensure(n * 8);
    r |= etile.ensure(ntiles * 24 + 64);
    r |= ecs.ensure(n * 8);
    r |= emisc.ensure(1024);  // misc | header | checksum | small | chain state (512)
    const uint64_t nbk = (44 + 8 * n) / 1024 + 2;
    r |= bsums.ensure(nbk * 64);
    if (r) return IGGY_ERR_DEVICE;
    EncScratch es;
    es.pl_local = epl.as<uint64_t>();
    es.uh_local = euh.as<uint64_t>();
    es.tile_pl = etile.as<uint64_t>();
    es.tile_uh = etile.as<uint64_t>(ntiles * 8);
    es.tile_min = etile.as<uint64_t>(ntiles * 16);
    es.cs = ecs.as<uint64_t>();
    es.misc = emisc.as<uint64_t>();
    es.hdr = emisc.as<iggy_batch_header>(128);
    es.dbg = diag_bits(c);
    iggy_raw_messages m = *dm;
    if (!own) prof_begin(c, 1, s);
    hipLaunchKernelGGL(k_enc_prep, dim3(ntiles), dim3(256), 0, s, m, es, partition_id, cap, (uint32_t)(ntiles == 1));
    if (ntiles != 1) hipLaunchKernelGGL(k_enc_scan, dim3(1), dim3(256), 0, s, ntiles, n, partition_id, cap, es);
    const uint64_t waves = std::min<uint64_t>(n, (uint64_t)c->ncu * 32);
    CsSource src{es.cs, nullptr, nullptr};
    // checksum blocks: 44 + 8n bytes; full blocks nb (the chain), then the last one
    const uint64_t csb = 44 + 8 * n;
    const uint64_t nb = csb > 240 ? (csb - 1) / 1024 : 0;
    bool segmented = false;
    if (!m.user_headers_lengths) {
        // no user headers: lane-group kernel (k_enc_frames only covers a < 16-B payload
        // area, and runs first so the segments' checksum chain sees its output)
        int nseg = 1;
        if (!own && n >= kEncSegMinFrames && nb >= 4 * kEncSegs && c->side) {
            nseg = kEncSegs;
            for (auto ev : c->seg_ev)
                if (!ev) nseg = 1;
        }
        segmented = nseg > 1;
        // frames of <= 240 hashed bytes (one lane each, latency-bound): segmented, they
        // run at the head of the side stream beside the first segment, ahead of every
        // block-sum range that reads their checksums; k_enc_lanes never writes their
        // checksum words. Unsegmented, the one k_enc_lanes launch hashes them after its
        // loop and runs the < 16-B payload-area fallback itself (own_tail).
        const bool ring = segmented && IGGY_ENC_RING;
        // writer waves beside the hashers (k_enc_ring<true>) when every frame's payload
        // keeps its source offset mod 16 in the output (P - out = 0 mod 16, encode.hip)
        const bool split = IGGY_ENC_SPLIT && ((((uintptr_t)m.payloads) - (uintptr_t)d_out) & 15) == 0;
        if (ring) {
            if (c->erec.ensure((n + 1) * 32) || c->esink.ensure(kErSinkBytes)) return IGGY_ERR_DEVICE;
            hipLaunchKernelGGL(k_enc_recs, dim3((uint32_t)std::min<uint64_t>((n + 256) / 256, (uint64_t)c->ncu * 8)),
                               dim3(256), 0, s, m, es, c->erec.as<uint4>());
        }
        if (segmented) {
            hipLaunchKernelGGL(k_enc_frames, dim3((waves + 3) / 4), dim3(256), 0, s, m, es, d_out, 1u);
            const dim3 sgrid((uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->ncu * 4));
            HIP_OK(hipEventRecord(c->seg_ev[kEncSegs + 1], s));
            HIP_OK(hipStreamWaitEvent(c->side, c->seg_ev[kEncSegs + 1], 0));
            hipLaunchKernelGGL(k_enc_short, sgrid, dim3(256), 0, c->side, m, es, d_out);
        }
        // one resident round of lane-group waves (2 WGs of 256 per CU at 240 VGPRs)
        // segmented: one CU stays free of lane-group waves, so the side stream's
        // single-wave chain (k_chain_partial) issues on a SIMD of its own (sharing one
        // with lane-group waves it ran 132 ns/step instead of ~31)
        const uint64_t lcu = (segmented && !(diag_bits(c) & 16384)) ? (uint64_t)c->ncu - 1 : (uint64_t)c->ncu;
        const uint64_t lwg = std::min<uint64_t>((n + 31) / 32, lcu * ((diag_bits(c) & 2048) ? 8 : 2));
        uint64_t *state = emisc.as<uint64_t>(512);
        for (int k = 0; k < nseg; ++k) {
            // blocks [B_k, B_k+1) need frames up to 128 B_k+1 - 6: segment k encodes
            // frames [F_k, F_k+1), F_k = 128 B_k - 5
            // uneven segments: the last one (whose chain cannot overlap) is ~6 % of the blocks
            // (same box: 60 / 30 / 8 / 2 % measured no better once the segment chains
            // stopped starving: 1.383-1.389 vs 1.376-1.386 ms)
            static const uint32_t kSegPermille[kEncSegs + 1] = {0, 400, 750, 940, 1000};
            auto bound = [&](int q) {
                if (nseg == 1) return q ? nb : (uint64_t)0;
                if (diag_bits(c) & 1024) return nb * q / nseg;  // diagnostics: even segments
                return nb * kSegPermille[q] / 1000;
            };
            const uint64_t B0 = bound(k), B1 = bound(k + 1);
            const uint64_t F0 = k == 0 ? 0 : std::min<uint64_t>(n, 128 * B0 - 5);
            const uint64_t F1 = k == nseg - 1 ? n : std::min<uint64_t>(n, 128 * B1 - 5);
            if (ring && split)
                hipLaunchKernelGGL(k_enc_ring<true>, dim3((uint32_t)std::min<uint64_t>((n + 63) / 64, lcu)),
                                   dim3(2 * kErThreads), kEsLds, s, m, es, d_out, F0, F1,
                                   (const uint4 *)c->erec.as<uint4>(), c->esink.as<uint8_t>());
            else if (ring)
                hipLaunchKernelGGL(k_enc_ring<false>, dim3((uint32_t)std::min<uint64_t>((n + 63) / 64, lcu)),
                                   dim3(kErThreads), kErLds, s, m, es, d_out, F0, F1,
                                   (const uint4 *)c->erec.as<uint4>(), c->esink.as<uint8_t>());
            else if (segmented)
                hipLaunchKernelGGL(k_enc_lanes<false>, dim3(lwg), dim3(256), 0, s, m, es, d_out, F0, F1);
            else
                hipLaunchKernelGGL(k_enc_lanes<true>, dim3(lwg), dim3(256), 0, s, m, es, d_out, F0, F1);
            if (segmented && k < nseg - 1) {
                HIP_OK(hipEventRecord(c->seg_ev[k], s));
                HIP_OK(hipStreamWaitEvent(c->side, c->seg_ev[k], 0));
                hipLaunchKernelGGL(k_bsum_blocks_range, dim3(c->ncu / 2), dim3(256), 0, c->side,
                                   (const iggy_batch_header *)es.hdr, (const uint64_t *)&es.misc[3], src,
                                   bsums.as<uint64_t>(), B0, B1);
                hipLaunchKernelGGL(k_chain_partial, dim3(1), dim3(256), 0, c->side, (const uint64_t *)&es.misc[3],
                                   (const uint64_t *)bsums.as<uint64_t>(), state, B0, B1);
            }
        }
        if (segmented) {
            // the last segment's blocks and the partial one, after every frame
            const uint64_t Bl = (diag_bits(c) & 1024) ? nb * (nseg - 1) / nseg : nb * 940 / 1000;  // last segment
            HIP_OK(hipEventRecord(c->seg_ev[kEncSegs], c->side));
            HIP_OK(hipStreamWaitEvent(s, c->seg_ev[kEncSegs], 0));
            hipLaunchKernelGGL(k_bsum_blocks_range, dim3(c->ncu), dim3(256), 0, s, (const iggy_batch_header *)es.hdr,
                               (const uint64_t *)&es.misc[3], src, bsums.as<uint64_t>(), Bl, nb + 1);
            hipLaunchKernelGGL(k_chain_partial, dim3(1), dim3(256), 0, s, (const uint64_t *)&es.misc[3],
                               (const uint64_t *)bsums.as<uint64_t>(), state, Bl, nb);
        }
    } else {
        hipLaunchKernelGGL(k_enc_frames, dim3((waves + 3) / 4), dim3(256), 0, s, m, es, d_out, 0u);
    }
    if (!own) prof_end(c, 1, s);
    uint64_t *dcs = emisc.as<uint64_t>(256);
    if (!segmented && nb + 1 <= kEncTailBlocks) {  // small batch: sums, chain and finish in one launch
        hipLaunchKernelGGL(k_enc_tail_small, dim3(1), dim3(256), 0, s, m, es, partition_id, cap,
                           emisc.as<uint8_t>(320), d_out, d_res);
        HIP_OK(hipGetLastError());
        return 0;
    }
    if (segmented) {
        hipLaunchKernelGGL(k_chain_finish, dim3(1), dim3(64), 0, s, (const iggy_batch_header *)es.hdr,
                           (const uint64_t *)&es.misc[3], src, (const uint64_t *)bsums.as<uint64_t>(),
                           (const uint64_t *)emisc.as<uint64_t>(512), emisc.as<uint8_t>(320), dcs);
    } else {
        hipLaunchKernelGGL(k_bsum_blocks, dim3(bsum_grid(c, n)), dim3(256), 0, s, (const iggy_batch_header *)es.hdr,
                           (const uint64_t *)&es.misc[3], src, bsums.as<uint64_t>(), nullptr);
        hipLaunchKernelGGL(k_bsum_chain, dim3(1), dim3(128), 0, s, (const iggy_batch_header *)es.hdr,
                           (const uint64_t *)&es.misc[3], src, (const uint64_t *)bsums.as<uint64_t>(),
                           emisc.as<uint8_t>(320) /* 192 B of small */, dcs, nullptr);
    }
    hipLaunchKernelGGL(k_enc_finish, dim3(1), dim3(64), 0, s, m, es, partition_id, cap,
                       (const uint64_t *)dcs, d_out, d_res);
    HIP_OK(hipGetLastError());
    return 0;
}

int iggy_codec_encode_batch(iggy_codec_ctx *c, const iggy_raw_messages *m, uint64_t partition_id,
                            uint8_t *out, uint64_t cap, uint64_t *out_len, iggy_wire_error *err) {
    if (!c || !m) return IGGY_ERR_INVALID_ARGUMENT;
    set_err(err, IGGY_OK);
    if (m->count == 0) {
        set_err(err, IGGY_ERR_VALIDATION, IGGY_V_EMPTY_BATCH);
        return IGGY_ERR_VALIDATION;
    }
    if (m->count > 0xFFFFFFFFull) {
        set_err(err, IGGY_ERR_PAYLOAD_TOO_LARGE, 0, m->count, 0xFFFFFFFFull);
        return IGGY_ERR_PAYLOAD_TOO_LARGE;
    }
    DevGuard dg(c->device);
    bind(c, nullptr);
    const uint64_t n = m->count;
    uint64_t spl = 0, suh = 0;
    for (uint64_t i = 0; i < n; ++i) {
        spl += m->payload_lengths[i];
        suh += m->user_headers_lengths ? m->user_headers_lengths[i] : 0;
    }
    const uint64_t need = 256 + 48 * n + spl + suh;
    if (cap < need || !out) {
        set_err(err, IGGY_ERR_CAPACITY, 0, need, cap);
        return IGGY_ERR_CAPACITY;
    }
    int r = 0;
    const uint64_t in_bytes = n * 28 + spl + (m->user_headers_lengths ? suh + n * 4 : 0);
    if (in_bytes <= kZeroCopyBytes && n < kEncSegMinFrames) {
        // a small batch in place (as encode_submit's): the SoA arrays read over the host
        // link, the wire bytes into the caller's registered `out` or the context's
        // mapped bounce, the verdict into mapped memory; one stream sync, no copy
        iggy_raw_messages dm;
        if (stage_soa(m, n, spl, suh, c->zin, &dm)) return IGGY_ERR_DEVICE;
        uint8_t *d_out = (uint8_t *)host_device_ptr(out, need);
        const bool bounce = !d_out;
        if (bounce) {
            if (c->zout.ensure(need + 16)) return IGGY_ERR_DEVICE;
            d_out = c->zout.d;
        }
        if (c->omap.ensure(64 + 256)) return IGGY_ERR_DEVICE;
        iggy_encode_result *d_res = c->omap.dp<iggy_encode_result>(64);
        hipStream_t s = c->stream;
        r = enqueue_encode(c, &dm, partition_id, d_out, need, d_res, s);
        if (r) return r;
        HIP_OK(hipStreamSynchronize(s));
        const iggy_encode_result res = *c->omap.hp<iggy_encode_result>(64);
        if (res.error.kind != IGGY_OK) {
            fill_err(err, res.error);
            return (int)res.error.kind;
        }
        if (bounce) memcpy(out, c->zout.h, need);
        if (out_len) *out_len = need;
        return 0;
    }
    r |= c->eids.ensure(n * 16);
    r |= c->eots.ensure(n * 8);
    r |= c->epay.ensure(spl + 16);
    r |= c->eplen.ensure(n * 4);
    r |= c->euhb.ensure(suh + 16);
    r |= c->euhl.ensure(n * 4);
    r |= c->dout.ensure(need + 16);
    if (r) return IGGY_ERR_DEVICE;
    hipStream_t s = c->stream;
    r |= put_host(c, c->eids.p, m->ids, n * 16, s);
    r |= put_host(c, c->eots.p, m->origin_timestamps, n * 8, s);
    r |= put_host(c, c->epay.p, m->payloads, spl, s);
    r |= put_host(c, c->eplen.p, m->payload_lengths, n * 4, s);
    const bool has_uh = m->user_headers_lengths != nullptr;
    if (has_uh) {
        r |= put_host(c, c->euhb.p, m->user_headers, suh, s);
        r |= put_host(c, c->euhl.p, m->user_headers_lengths, n * 4, s);
    }
    if (r) return IGGY_ERR_DEVICE;
    iggy_raw_messages dm;
    dm.count = n;
    dm.ids = c->eids.as<uint64_t>();
    dm.origin_timestamps = c->eots.as<uint64_t>();
    dm.payloads = c->epay.as<uint8_t>();
    dm.payload_lengths = c->eplen.as<uint32_t>();
    dm.user_headers = has_uh ? c->euhb.as<uint8_t>() : nullptr;
    dm.user_headers_lengths = has_uh ? c->euhl.as<uint32_t>() : nullptr;
    iggy_encode_result *d_res = c->dresult.as<iggy_encode_result>(512);
    r = enqueue_encode(c, &dm, partition_id, c->dout.as<uint8_t>(), need, d_res, s);
    if (r) return r;
    iggy_encode_result *h_res = (iggy_encode_result *)((uint8_t *)c->h_pinned + 512);
    HIP_OK(hipMemcpyAsync(h_res, d_res, sizeof(*h_res), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (h_res->error.kind != IGGY_OK) {
        fill_err(err, h_res->error);
        return (int)h_res->error.kind;
    }
    r = get_host(c, out, c->dout.p, need, s);
    if (r) return r;
    if (out_len) *out_len = need;
    return 0;
}

int iggy_codec_encode_batch_device(iggy_codec_ctx *c, const iggy_raw_messages *msgs,
                                   uint64_t partition_id, uint8_t *d_out, uint64_t cap,
                                   iggy_encode_result *d_result, void *stream) {
    if (!c || !msgs || !d_out || !d_result || msgs->count == 0 || msgs->count > 0xFFFFFFFFull)
        return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    // cap is checked on the device against the scanned batch length: a batch that
    // does not fit writes nothing and reports IGGY_ERR_CAPACITY in *d_result
    return enqueue_encode(c, msgs, partition_id, d_out, cap, d_result, bind(c, stream));
}

}  // extern "C"
