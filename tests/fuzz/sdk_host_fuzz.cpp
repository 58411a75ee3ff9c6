// Host sanitizer harness (TEST INFRASTRUCTURE): the host-pure half of
// iggy_amd/csrc/sdk.cpp (built with -DIGGY_HOST_ONLY) under
// -fsanitize=address,undefined, driven by tests/test_sdk_fuzz_cpu.py, which feeds
// random and mutated wire inputs on stdin and checks every printed result against
// oracle/sdk_ref.py. One command per line, one result line per decode:
//   M <hex>                      SendMessagesHeader decode (send_messages.rs:222-241)
//   B <hex>                      BatchHeader::decode (batch.rs:98-134)
//   F <cap> <max> <hex>          read_message + try_from over a socketpair (framing.rs:107-164);
//                                a frame above cap is finished in a grown buffer
//   P <batch_length> <batch_size> <direct>   a new producer, then
//   E <sk> <shex> <tk> <thex> <pk> <phex> <n> <pl,..> <uh,..|->   one append
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/iggy_codec.h"

static std::vector<uint8_t> unhex(const char *h) {
    std::vector<uint8_t> v;
    if (!h || h[0] == '-') return v;
    const size_t n = strlen(h);
    for (size_t i = 0; i + 1 < n; i += 2) {
        unsigned x;
        sscanf(h + i, "%2x", &x);
        v.push_back((uint8_t)x);
    }
    return v;
}

static void hexout(const uint8_t *p, uint64_t n) {
    if (!n) {
        fputs("-", stdout);
        return;
    }
    for (uint64_t i = 0; i < n; ++i) printf("%02x", p[i]);
}

static void errout(const iggy_wire_error &e) {
    printf("%u %u %llu %llu %llu", e.kind, e.reason, (unsigned long long)e.a, (unsigned long long)e.b,
           (unsigned long long)e.c);
}

static std::vector<uint32_t> ints(const char *s) {
    std::vector<uint32_t> v;
    if (!s || s[0] == '-') return v;
    const char *p = s;
    while (*p) {
        v.push_back((uint32_t)strtoul(p, (char **)&p, 10));
        if (*p == ',') ++p;
    }
    return v;
}

static void field(uint32_t kind, const std::vector<uint8_t> &v, uint32_t *k, uint32_t *l, uint8_t *val) {
    *k = kind;
    *l = (uint32_t)v.size();
    memset(val, 0, 256);
    if (!v.empty()) memcpy(val, v.data(), v.size() < 256 ? v.size() : 256);
}

int main() {
    std::string line;
    char buf[1 << 16];
    iggy_producer *prod = nullptr;
    std::vector<char> big;
    while (true) {
        std::string l;
        int c;
        while ((c = getchar()) != EOF && c != '\n') l.push_back((char)c);
        if (c == EOF && l.empty()) break;
        std::vector<char> w(l.begin(), l.end());
        w.push_back(0);
        std::vector<char *> tok;
        for (char *t = strtok(w.data(), " "); t; t = strtok(nullptr, " ")) tok.push_back(t);
        if (tok.empty()) continue;
        const char cmd = tok[0][0];
        if (cmd == 'M' && tok.size() >= 2) {
            const std::vector<uint8_t> in = unhex(tok[1]);
            // an exact-size heap copy: any read past the input is an ASan report
            uint8_t *p = in.empty() ? nullptr : (uint8_t *)malloc(in.size());
            if (p) memcpy(p, in.data(), in.size());
            iggy_send_messages_header h;
            iggy_wire_error e;
            uint64_t used = 0;
            const int rc = iggy_send_messages_header_decode(p, in.size(), &h, &used, &e);
            printf("M %d ", rc);
            errout(e);
            if (rc == 0) {
                printf(" %llu %u ", (unsigned long long)used, h.stream_id.kind);
                hexout(h.stream_id.value, h.stream_id.length);
                printf(" %u ", h.topic_id.kind);
                hexout(h.topic_id.value, h.topic_id.length);
                printf(" %u ", h.partitioning.kind);
                hexout(h.partitioning.value, h.partitioning.length);
                printf(" %u", h.messages_count);
            }
            putchar('\n');
            free(p);
        } else if (cmd == 'B' && tok.size() >= 2) {
            const std::vector<uint8_t> in = unhex(tok[1]);
            uint8_t *p = in.empty() ? nullptr : (uint8_t *)malloc(in.size());
            if (p) memcpy(p, in.data(), in.size());
            iggy_batch_header h;
            iggy_wire_error e;
            const int rc = iggy_batch_header_decode(p, in.size(), &h, &e);
            printf("B %d ", rc);
            errout(e);
            if (rc == 0)
                printf(" %llu %llu %llu %llu %llu %llu %u", (unsigned long long)h.partition_id,
                       (unsigned long long)h.base_offset, (unsigned long long)h.base_timestamp,
                       (unsigned long long)h.origin_timestamp, (unsigned long long)h.batch_length,
                       (unsigned long long)h.batch_checksum, h.message_count);
            putchar('\n');
            free(p);
        } else if (cmd == 'F' && tok.size() >= 4) {
            const uint64_t cap = strtoull(tok[1], nullptr, 10), mx = strtoull(tok[2], nullptr, 10);
            const std::vector<uint8_t> stream = unhex(tok[3]);
            int sv[2];
            if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 2;
            std::thread wr([&]() {
                size_t off = 0;
                while (off < stream.size()) {
                    const size_t k = stream.size() - off < 997 ? stream.size() - off : 997;
                    const ssize_t r = write(sv[0], stream.data() + off, k);
                    if (r <= 0) break;
                    off += (size_t)r;
                }
                shutdown(sv[0], SHUT_WR);
            });
            std::vector<uint8_t> fb(cap ? cap : 1);
            while (true) {
                uint64_t total = 0;
                iggy_wire_error e;
                int rc = iggy_frame_read(sv[1], fb.data(), cap, mx, &total, &e);
                const uint8_t *frame = fb.data();
                std::vector<uint8_t> grown;
                if (rc == IGGY_ERR_CAPACITY) {
                    printf("F %d -\n", rc);
                    grown.resize(total);  // exact size: an overrun is an ASan report
                    memcpy(grown.data(), fb.data(), IGGY_FRAME_HEADER_BYTES);
                    rc = iggy_frame_read_rest(sv[1], grown.data(), total, &e);
                    frame = grown.data();
                }
                printf("F %d ", rc);
                hexout(frame, rc == 0 ? total : 0);
                putchar('\n');
                if (rc == IGGY_ERR_CONNECTION_CLOSED || rc == IGGY_ERR_TCP_ERROR ||
                    (rc == IGGY_ERR_INVALID_COMMAND && total == 0))
                    break;
            }
            wr.join();
            close(sv[0]);
            close(sv[1]);
        } else if (cmd == 'P' && tok.size() >= 4) {
            if (prod) iggy_producer_destroy(prod);
            iggy_producer_config cfg;
            memset(&cfg, 0, sizeof(cfg));
            cfg.batch_length = strtoull(tok[1], nullptr, 10);
            cfg.batch_size = strtoull(tok[2], nullptr, 10);
            cfg.direct = (uint32_t)atoi(tok[3]);
            // the staging never touches the context in the host-only build
            prod = nullptr;
            const int rc = iggy_producer_create((iggy_codec_ctx *)&cfg, &cfg, &prod);
            printf("P %d\n", rc);
        } else if (cmd == 'E' && tok.size() >= 10 && prod) {
            iggy_identifier s, t;
            iggy_partitioning pt;
            field((uint32_t)atoi(tok[1]), unhex(tok[2]), &s.kind, &s.length, s.value);
            field((uint32_t)atoi(tok[3]), unhex(tok[4]), &t.kind, &t.length, t.value);
            field((uint32_t)atoi(tok[5]), unhex(tok[6]), &pt.kind, &pt.length, pt.value);
            const uint64_t n = strtoull(tok[7], nullptr, 10);
            std::vector<uint32_t> pl = ints(tok[8]), uh = ints(tok[9]);
            pl.resize(n, 0);
            const bool has_uh = tok[9][0] != '-';
            if (has_uh) uh.resize(n, 0);
            uint64_t spl = 0, suh = 0;
            for (uint64_t i = 0; i < n; ++i) {
                spl += pl[i];
                suh += has_uh ? uh[i] : 0;
            }
            std::vector<uint64_t> ids(2 * n + 1, 7), ots(n + 1, 1700000000000000ull);
            std::vector<uint8_t> pay(spl + 1, 0x61), uhb(suh + 1, 0x62);
            iggy_raw_messages m;
            m.count = n;
            m.ids = ids.data();
            m.origin_timestamps = ots.data();
            m.payloads = pay.data();
            m.payload_lengths = pl.data();
            m.user_headers = has_uh ? uhb.data() : nullptr;
            m.user_headers_lengths = has_uh ? uh.data() : nullptr;
            int due = -1;
            const int rc = iggy_producer_append(prod, &s, &t, &pt, &m, &due);
            uint64_t ne = 0, nb = 0, nm = 0;
            iggy_producer_pending(prod, &ne, &nb, &nm);
            printf("E %d %d %llu %llu %llu\n", rc, due, (unsigned long long)ne, (unsigned long long)nb,
                   (unsigned long long)nm);
        }
        fflush(stdout);
    }
    if (prod) iggy_producer_destroy(prod);
    (void)buf;
    (void)big;
    return 0;
}
