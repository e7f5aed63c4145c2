// tools/utf8_lookup_check.c -- host proof that the table-lookup UTF-8 check
// (utf8_err in flashws_amd/csrc/fws_device.h, r05) flags exactly the bytes the
// r02-r04 SWAR form flagged. Both are written here with C emulations of the
// gfx950 instructions they use (v_perm_b32 on selectors 0..7, v_alignbit_b32,
// v_alignbyte_b32). Byte k of x is judged from (prev3, prev2, prev1, x_k); the
// check runs every (prev3, prev2) pair of a 48-byte boundary set against every
// (prev1, x_k) of all 256 x 256, at each of the 4 byte positions, then random
// dword pairs.   cc -O2 -o /tmp/u8c tools/utf8_lookup_check.c && /tmp/u8c
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint32_t alignbit(uint32_t a, uint32_t b, uint32_t s) {
    return (uint32_t)(((((uint64_t)a) << 32) | b) >> (s & 31u));
}
static uint32_t alignbyte(uint32_t a, uint32_t b, uint32_t s) { return alignbit(a, b, 8u * (s & 3u)); }
static uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {   // selector bytes 0..7 only
    const uint64_t d = (((uint64_t)s0) << 32) | s1;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xFFu;
        if (s > 7) { fprintf(stderr, "selector %u\n", s); exit(2); }
        r |= (uint32_t)((d >> (8 * s)) & 0xFFu) << (8 * i);
    }
    return r;
}

// r02-r04 form (bit 7 of each byte = error). shifted = 1: the same rules, except
// that an invalid byte (C0, C1, F5..FF) is flagged at the byte after it, which is
// where the lookup form flags it: a lead >= C0 followed by a non-continuation
// fails rule (A), followed by a continuation fails a table rule. The byte after
// is always judged (the walks run 3 zero bytes past every region's end), so the
// per-frame verdict is the same.
static uint32_t err_swar(uint32_t x, uint32_t p, int shifted) {
    const uint32_t H = 0x80808080u;
    const uint32_t x1 = x << 1, x2 = x << 2, x3 = x << 3;
    const uint32_t tx = x & x1, ux = tx & x2, wx = ux & x3;
    const uint32_t tp = p & (p << 1), up = tp & (p << 2), wp = up & (p << 3);
    const uint32_t req = alignbyte(tx, tp, 3u) | alignbyte(ux, up, 2u) | alignbyte(wx, wp, 1u);
    uint32_t err = (x & ~x1) ^ req;
    const uint32_t inv = (tx & ~((x & 0x3E3E3E3Eu) + 0x7E7E7E7Eu)) | (((x & 0x7F7F7F7Fu) + 0x0B0B0B0Bu) & x);
    if (shifted) {   // an invalid byte (C0, C1, F5..FF) flagged at the byte after it
        const uint32_t tp1 = p & (p << 1);
        const uint32_t invp = (tp1 & ~((p & 0x3E3E3E3Eu) + 0x7E7E7E7Eu)) | (((p & 0x7F7F7F7Fu) + 0x0B0B0B0Bu) & p);
        err |= alignbyte(inv, invp, 3u);
    } else {
        err |= inv;
    }
    const uint32_t e1 = alignbyte(ux, up, 3u);
    const uint32_t q = alignbyte(x, p, 3u) & 0x1F1F1F1Fu;
    const uint32_t nzE0 = q + 0x7F7F7F7Fu, nzED = (q ^ 0x0D0D0D0Du) + 0x7F7F7F7Fu;
    const uint32_t nzF0 = (q ^ 0x10101010u) + 0x7F7F7F7Fu, nzF4 = (q ^ 0x14141414u) + 0x7F7F7F7Fu;
    const uint32_t s5 = x2, s54 = x2 | x3;
    const uint32_t bE = (s5 & nzED) | (~s5 & nzE0);
    const uint32_t bF = (s54 & nzF4) | (~s54 & nzF0);
    err |= e1 & ~(bE & bF);
    return err & H;
}

// r05 form: tables as in fws_device.h (byte k nonzero = error)
#define TA0 0x00000000u
#define TA1 0xFE010000u
#define TB0 0x10000009u
#define TB1 0x8282C4A0u
#define TC0 0x828283ABu
#define TC1 0x868696C2u
#define T20 0x57574F2Fu
#define T21 0x00000000u
static uint32_t lead_tables(uint32_t x, uint32_t *ta) {
    const uint32_t m = 0x07070707u;
    *ta = perm(TA1, TA0, (x >> 5) & m);
    return *ta & perm(TB1, TB0, (x >> 2) & m) & perm(TC1, TC0, x & m);
}
static uint32_t err_lookup(uint32_t x, uint32_t p) {
    uint32_t tax, tap;
    const uint32_t b1x = lead_tables(x, &tax), b1p = lead_tables(p, &tap);
    const uint32_t x1 = x << 1, tx = x & x1, tp = p & (p << 1);
    const uint32_t req = alignbyte(tx, tp, 3u) | alignbyte(tax, tap, 2u) | alignbyte(b1x, b1p, 1u);
    const uint32_t ea = (x & ~x1) ^ req;
    const uint32_t b2 = perm(T21, T20, (x >> 4) & 0x07070707u);
    return (ea & 0x80808080u) | (alignbyte(b1x, b1p, 3u) & b2);
}

static uint64_t rs = 88172645463325252ull;
static uint32_t rnd(void) { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return (uint32_t)rs; }

int main(void) {
    static const uint8_t bnd[48] = {0x00, 0x0D, 0x20, 0x3F, 0x40, 0x41, 0x5F, 0x60, 0x68, 0x6D, 0x70, 0x74, 0x7F,
                                    0x80, 0x81, 0x8F, 0x90, 0x9F, 0xA0, 0xAF, 0xB0, 0xBF, 0xC0, 0xC1, 0xC2, 0xCF,
                                    0xD0, 0xDF, 0xE0, 0xE1, 0xE8, 0xEC, 0xED, 0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4,
                                    0xF5, 0xF7, 0xF8, 0xF9, 0xFB, 0xFC, 0xFD, 0xFE, 0xFF};
    uint64_t n = 0, bad = 0;
    for (int k = 0; k < 4; ++k)                      // position of the judged byte in x
        for (int i3 = 0; i3 < 48; ++i3)
            for (int i2 = 0; i2 < 48; ++i2)
                for (uint32_t p1 = 0; p1 < 256; ++p1)
                    for (uint32_t xk = 0; xk < 256; ++xk) {
                        uint8_t w[8];
                        for (int j = 0; j < 8; ++j) w[j] = (uint8_t)rnd();
                        w[4 + k] = (uint8_t)xk; w[3 + k] = (uint8_t)p1; w[2 + k] = bnd[i2]; w[1 + k] = bnd[i3];
                        const uint32_t p = w[0] | w[1] << 8 | w[2] << 16 | (uint32_t)w[3] << 24;
                        const uint32_t x = w[4] | w[5] << 8 | w[6] << 16 | (uint32_t)w[7] << 24;
                        const int a = (err_swar(x, p, 1) >> (8 * k + 7)) & 1;
                        const int b = ((err_lookup(x, p) >> (8 * k)) & 0xFFu) != 0;
                        ++n;
                        if (a != b && bad++ < 10)
                            printf("MISMATCH k=%d p=%08x x=%08x swar=%d lookup=%d\n", k, p, x, a, b);
                    }
    for (uint64_t i = 0; i < 400000000ull; ++i) {
        uint32_t x = rnd(), p = rnd();
        if (i & 1) { x &= 0xBFBFBFBFu | rnd(); p |= 0x80808080u & rnd(); }   // more continuation bytes
        const uint32_t s = err_swar(x, p, 1), l = err_lookup(x, p);
        for (int k = 0; k < 4; ++k) {
            const int a = (s >> (8 * k + 7)) & 1, b = ((l >> (8 * k)) & 0xFFu) != 0;
            if (a != b && bad++ < 20) printf("MISMATCH rnd p=%08x x=%08x k=%d\n", p, x, k);
        }
        n += 4;
    }
    printf("%llu byte verdicts compared, %llu mismatches\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
