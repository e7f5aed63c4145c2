// gen.cpp -- synthetic masked-frame batches for the BASELINE configs
// (fws_gen_batch in include/fws_gpu.h). Host code, deterministic per seed.
//
// Frame layout written (client -> server, RFC 6455 §5.2, the layout the
// reference parses at net/w_socket.h:435-524):
//   [FIN|opcode] [0x80|len7] [ext len: 0 / 2 / 8 B big-endian] [key: 4 B] [payload ^ key]
// Two independent mt19937_64 streams: `meta` draws lengths, keys and
// injection sites; `data` draws plaintext payload bytes.
#include <math.h>
#include <string.h>

#include <random>

#include "fws_gpu.h"

namespace {

struct Gen {
    const fws_gen_params &p;
    std::mt19937_64 meta, data;
    uint64_t meta_draws = 0;
    explicit Gen(const fws_gen_params &pp)
        : p(pp), meta(pp.seed), data(pp.seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {}

    double uniform() { return (double)(meta() >> 11) * (1.0 / 9007199254740992.0); }

    // log-uniform integer in [lo, hi]
    uint64_t log_uniform(uint64_t lo, uint64_t hi) {
        double a = log2((double)lo), b = log2((double)hi + 1.0);
        uint64_t v = (uint64_t)exp2(a + (b - a) * uniform());
        if (v < lo) v = lo;
        if (v > hi) v = hi;
        return v;
    }
};

inline uint32_t hdr_len_for(uint64_t plen) { return plen < 126 ? 6u : (plen <= 65535 ? 8u : 14u); }

// Write header at w (returns header length).
uint32_t put_header(uint8_t *w, uint32_t opcode, uint32_t fin, uint64_t plen, uint32_t key) {
    uint32_t n = 0;
    w[n++] = (uint8_t)((fin << 7) | (opcode & 15u));
    if (plen < 126) {
        w[n++] = (uint8_t)(0x80u | plen);
    } else if (plen <= 65535) {
        w[n++] = 0x80u | 126u;
        w[n++] = (uint8_t)(plen >> 8);
        w[n++] = (uint8_t)plen;
    } else {
        w[n++] = 0x80u | 127u;
        for (int i = 7; i >= 0; --i) w[n++] = (uint8_t)(plen >> (8 * i));
    }
    memcpy(w + n, &key, 4);   // wire bytes = native LE u32 (w_socket.h:504)
    return n + 4;
}

void fill_random(std::mt19937_64 &r, uint8_t *p, uint64_t n) {
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v = r();
        memcpy(p + i, &v, 8);
    }
    if (i < n) {
        uint64_t v = r();
        memcpy(p + i, &v, n - i);
    }
}

void mask_in_place(uint8_t *p, uint64_t n, uint32_t key) {
    uint8_t kb[4];
    memcpy(kb, &key, 4);
    uint64_t k64 = ((uint64_t)key << 32) | key, i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t v;
        memcpy(&v, p + i, 8);
        v ^= k64;
        memcpy(p + i, &v, 8);
    }
    for (; i < n; ++i) p[i] ^= kb[i & 3];
}

// Encode code point cp as UTF-8 into out; returns bytes.
int utf8_encode(uint32_t cp, uint8_t *out) {
    if (cp < 0x80) { out[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { out[0] = 0xC0 | (cp >> 6); out[1] = 0x80 | (cp & 63); return 2; }
    if (cp < 0x10000) {
        out[0] = 0xE0 | (cp >> 12); out[1] = 0x80 | ((cp >> 6) & 63); out[2] = 0x80 | (cp & 63);
        return 3;
    }
    out[0] = 0xF0 | (cp >> 18); out[1] = 0x80 | ((cp >> 12) & 63);
    out[2] = 0x80 | ((cp >> 6) & 63); out[3] = 0x80 | (cp & 63);
    return 4;
}

// Valid UTF-8 text of exactly n bytes: a mix of 1-4 byte sequences.
void fill_utf8(std::mt19937_64 &r, uint8_t *p, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        uint64_t x = r();
        int cls = (int)(x & 3) + 1;
        uint32_t v = (uint32_t)(x >> 8);
        uint32_t cp;
        if (cls == 1) cp = v % 0x80;
        else if (cls == 2) cp = 0x80 + v % (0x800 - 0x80);
        else if (cls == 3) { cp = 0x800 + v % (0x10000 - 0x800 - 0x800); if (cp >= 0xD800) cp += 0x800; }
        else cp = 0x10000 + v % (0x110000 - 0x10000);
        uint8_t tmp[4];
        int k = utf8_encode(cp, tmp);
        if (i + (uint64_t)k > n) { p[i++] = (uint8_t)(0x20 + (x >> 40) % 0x5F); continue; }
        memcpy(p + i, tmp, (size_t)k);
        i += (uint64_t)k;
    }
}

// Overwrite with one always-invalid pattern (Unicode Table 3-7 violations).
void inject_invalid(Gen &g, uint8_t *p, uint64_t n) {
    static const uint8_t pats[6][4] = {{0xFF, 0, 0, 0}, {0xC0, 0x80, 0, 0}, {0xED, 0xA0, 0x80, 0},
                                       {0xC1, 0xBF, 0, 0}, {0xF4, 0x90, 0x80, 0x80}, {0xE2, 0x82, 0, 0}};
    static const int lens[6] = {1, 2, 3, 2, 4, 2};
    int k = (int)(g.meta() % 6);
    if (k == 5) {                      // truncated 3-byte sequence at the very end
        if (n >= 2) { p[n - 2] = 0xE2; p[n - 1] = 0x82; }
        else if (n == 1) p[0] = 0xFF;
        return;
    }
    if (n < (uint64_t)lens[k]) { if (n) p[0] = 0xFF; return; }
    uint64_t at = g.meta() % (n - (uint64_t)lens[k] + 1);
    memcpy(p + at, pats[k], (size_t)lens[k]);
}

}  // namespace

extern "C" int fws_gen_batch(const fws_gen_params *pp, uint8_t *wire, uint64_t cap, uint64_t *wire_len,
                             fws_frame_desc *descs, uint64_t descs_cap, uint64_t *n_frames,
                             uint8_t *utf8_ok) {
    if (!pp || !wire_len || !n_frames) return FWS_ERR_INVALID;
    const fws_gen_params &p = *pp;
    Gen g(p);
    uint64_t w = 0, nf = 0, total_pl = 0;
    const bool write = wire != nullptr;
    auto emit = [&](uint32_t opcode, uint32_t fin, uint64_t plen, int text_kind) -> int {
        uint32_t key = (uint32_t)g.meta();
        uint32_t hl = hdr_len_for(plen);
        bool bad = false;
        if (text_kind) bad = (g.meta() % 1000) < p.invalid_permille;
        if (write) {
            if (w + hl + plen > cap) return FWS_ERR_CAPACITY;
            put_header(wire + w, opcode, fin, plen, key);
            uint8_t *pl = wire + w + hl;
            if (text_kind) {
                fill_utf8(g.data, pl, plen);
                if (bad) inject_invalid(g, pl, plen);
            } else {
                fill_random(g.data, pl, plen);
            }
            mask_in_place(pl, plen, key);
            if (descs && nf < descs_cap) descs[nf] = fws_frame_desc{w + hl, plen, key, 0u};
            if (utf8_ok && nf < descs_cap) utf8_ok[nf] = (uint8_t)(text_kind && !bad);
        }   // size-only pass: lengths never depend on the data or injection draws
        w += hl + plen;
        total_pl += plen;
        ++nf;
        return 0;
    };
    int r = 0;
    switch (p.kind) {
    case 0:   // fixed-size frames (C2)
        for (uint64_t i = 0; i < p.n_frames && !r; ++i) r = emit(p.opcode, 1, p.payload_min, 0);
        break;
    case 1:   // log-uniform sizes until the payload total reaches target (C3)
        while (total_pl < p.target_bytes && !r)
            r = emit(p.opcode, 1, g.log_uniform(p.payload_min, p.payload_max), 0);
        break;
    case 2: { // one fragmented message of exactly target bytes (C4)
        bool first = true;
        while (total_pl < p.target_bytes && !r) {
            uint64_t len = g.log_uniform(p.payload_min, p.payload_max);
            uint64_t left = p.target_bytes - total_pl;
            if (len > left) len = left;
            bool last = len == left;
            r = emit(first ? p.opcode : 0u, last ? 1u : 0u, len, 0);
            first = false;
        }
        break;
    }
    case 3:   // UTF-8 TEXT frames (C5)
        for (uint64_t i = 0; i < p.n_frames && !r; ++i) r = emit(1u, 1, p.payload_min, 1);
        break;
    default:
        return FWS_ERR_INVALID;
    }
    *wire_len = w;
    *n_frames = nf;
    return r;
}
