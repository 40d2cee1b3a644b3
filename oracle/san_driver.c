/* TEST INFRASTRUCTURE ONLY — host sanitizer driver for the CPU oracle.
 *
 * Built by `make -C oracle san` with -fsanitize=address,undefined
 * -fno-sanitize-recover=all (an ASan/UBSan build of the CPU
 * side) and run by tests/test_sanitizers_cpu.py.  Every buffer is a heap
 * block of exactly the size the reference's contract allows (no slack), so a
 * read or write one element past it is an ASan report; UBSan covers shifts,
 * signed overflow and misaligned accesses.  The cases follow the shapes the
 * reference's own tests use (tests/roundtrip_test.cpp, error_code_test.cpp,
 * scratch_buffer_error_test.cpp, odd_symbol_count_test.cpp): round trips at
 * SF 5-12 with osr 1/2 and Hann windows, truncated and ragged sample counts,
 * capacity and scratch errors, garbage symbols, and the codec / LoRaWAN
 * helpers over ragged lengths.  Exit status 0 = every check held.
 */
#include "lphy_oracle.h"

#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int fails;
#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                     \
        }                                                                \
    } while (0)

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (uint32_t)(rs >> 11);
}
static void* xmalloc(size_t n) {
    void* p = malloc(n ? n : 1);
    if (!p) abort();
    return p;
}

/* encode -> modulate -> (mode A | dechirp + mode B) -> decode, exact-size buffers */
static void roundtrip(unsigned sf, unsigned bw, unsigned osr, int hann, size_t plen, float ampl) {
    uint8_t* pay = xmalloc(plen);
    for (size_t i = 0; i < plen; ++i) pay[i] = (uint8_t)rnd();
    const size_t ns = 2 * plen, N = (size_t)1 << sf, step = N * osr;
    uint16_t* syms = xmalloc(ns * sizeof(uint16_t));
    CHECK(orc_lora_encode(pay, plen, syms) == ns);
    uint8_t* dec = xmalloc(plen);
    uint8_t crc = 7;
    CHECK(orc_decode(syms, ns, dec, plen, &crc) == (ssize_t)plen);
    if (plen) CHECK(memcmp(dec, pay, plen) == 0);
    if (plen) CHECK(orc_decode(syms, ns, dec, plen - 1, &crc) == -ERANGE);
    if (ns) CHECK(orc_decode(syms, ns - 1, dec, plen, &crc) == -EINVAL);
    free(dec);
    /* symbols above the SF's alphabet cannot round trip: keep them in range */
    for (size_t i = 0; i < ns; ++i) syms[i] &= (uint16_t)(N - 1);
    const size_t count = (ns + 2) * step;
    float* iq = xmalloc(2 * count * sizeof(float));
    CHECK(orc_lora_modulate(syms, ns, iq, sf, osr, bw, ampl, 0x00) == count);
    /* (sync word 0: the estimate reads the two sync symbols, so a nonzero
     * one shifts every bin of an unimpaired frame) */

    uint16_t* out = xmalloc(ns * sizeof(uint16_t));
    float met[2];
    uint8_t sw = 0;
    CHECK(orc_demodulate(sf, bw, osr, hann, iq, count, out, ns, met, 0x12, &sw) == (ssize_t)ns);
    /* (mode A estimates on the raw chirps, phy.cpp:81-148, so an unimpaired
     * frame does not round trip through it; its symbols are not compared) */
    /* capacity one short: -ERANGE, nothing written past the buffer */
    if (ns) {
        uint16_t* small = xmalloc((ns - 1) * sizeof(uint16_t));
        CHECK(orc_demodulate(sf, bw, osr, hann, iq, count, small, ns - 1, met, 0, &sw) == -ERANGE);
        free(small);
    }
    /* ragged count: -EINVAL in mode A */
    if (count > 1) CHECK(orc_demodulate(sf, bw, osr, hann, iq, count - 1, out, ns, met, 0, &sw) == -EINVAL);

    if (osr == 1) {
        float* dch = xmalloc(2 * count * sizeof(float));
        orc_dechirp(iq, dch, count, sf, bw);
        uint8_t sync = 0;
        CHECK(orc_lora_demodulate(sf, hann, dch, count, out, 1, &sync, count, met) == (ssize_t)ns);
        if (sf >= 7 && !hann && ampl <= 1.0f) CHECK(memcmp(out, syms, ns * sizeof(uint16_t)) == 0);
        /* truncated by a partial symbol: the whole symbols only */
        if (count > N) {
            const size_t c2 = count - N / 2;
            const size_t tot = c2 / N;
            uint16_t* o2 = xmalloc((tot >= 2 ? tot - 2 : tot) * sizeof(uint16_t));
            const ssize_t r = orc_lora_demodulate(sf, hann, dch, c2, o2, 1, &sync, c2, met);
            CHECK(r == (ssize_t)(tot >= 2 ? tot - 2 : tot));
            free(o2);
        }
        /* amplitude above 1 with no scratch: -ERANGE (scratch_buffer_error_test) */
        for (size_t i = 0; i < 2 * count; ++i) dch[i] *= 4.0f;
        CHECK(orc_lora_demodulate(sf, hann, dch, count, out, 1, &sync, 0, met) == -ERANGE);
        CHECK(orc_lora_demodulate(sf, hann, dch, count, out, 1, &sync, count, met) == (ssize_t)ns);
        free(dch);
    }

    free(out);
    free(iq);
    free(syms);
    free(pay);
}

static void estimate_compensate(unsigned sf, unsigned osr) {
    const size_t N = (size_t)1 << sf, count = 5 * N * osr + (rnd() % N);
    float* iq = xmalloc(2 * count * sizeof(float));
    for (size_t i = 0; i < 2 * count; ++i) iq[i] = (float)((int)(rnd() % 2001) - 1000) / 1000.0f;
    float met[2] = {0.0f, 0.0f};
    orc_estimate_offsets(sf, osr, (int)(rnd() & 1), iq, count, met);
    orc_compensate_offsets(sf, osr, met[0], met[1], iq, count);
    orc_estimate_offsets(sf, osr, 0, iq, 0, met); /* empty: no-op */
    free(iq);
}

static void garbage_symbols(void) {
    for (int rep = 0; rep < 64; ++rep) {
        const size_t n = 2 * (rnd() % 300), cap = n / 2;
        uint16_t* s = xmalloc(n * sizeof(uint16_t));
        for (size_t i = 0; i < n; ++i) s[i] = (uint16_t)rnd();
        uint8_t* out = xmalloc(cap);
        uint8_t crc;
        CHECK(orc_decode(s, n, out, cap, &crc) == (ssize_t)cap);
        free(out);
        free(s);
    }
}

static void codecs(void) {
    for (int rep = 0; rep < 200; ++rep) {
        const size_t rdd = 1 + rnd() % 4, ppm = 5 + rnd() % 8, blocks = rnd() % 6;
        const size_t ncw = ppm * blocks, nsym = (4 + rdd) * blocks;
        uint8_t* cw = xmalloc(ncw);
        uint8_t* back = xmalloc(ncw);
        uint16_t* sy = xmalloc(nsym * sizeof(uint16_t));
        for (size_t i = 0; i < ncw; ++i) cw[i] = (uint8_t)(rnd() & ((1u << (4 + rdd)) - 1));
        orc_interleave(cw, ncw, sy, ppm, rdd);
        memset(back, 0, ncw);
        orc_deinterleave(sy, nsym, back, ppm, rdd);
        if (ncw) CHECK(memcmp(cw, back, ncw) == 0);
        const size_t len = rnd() % 70;
        uint8_t* w = xmalloc(len);
        for (size_t i = 0; i < len; ++i) w[i] = (uint8_t)rnd();
        for (int kind = 0; kind < 3; ++kind)
            orc_whiten(w, len, kind, (int)(rnd() % 40), (unsigned)(1 + rnd() % 4));
        if (len >= 2) {
            (void)orc_checksum(w, len, 0);
            (void)orc_checksum(w, len, 1);
        }
        for (int op = 0; op < 8; ++op) {
            uint8_t fl;
            (void)orc_hamming((uint8_t)rnd(), op, &fl);
        }
        (void)orc_gray((uint16_t)rnd(), (int)(rnd() & 1));
        free(w);
        free(sy);
        free(back);
        free(cw);
    }
}

static void lorawan(void) {
    uint8_t key[16];
    for (int i = 0; i < 16; ++i) key[i] = (uint8_t)rnd();
    for (size_t len = 0; len < 80; ++len) {
        uint8_t* b = xmalloc(len);
        for (size_t i = 0; i < len; ++i) b[i] = (uint8_t)rnd();
        (void)orc_lorawan_mic(key, (int)(len & 1), rnd(), rnd(), b, len);
        int64_t rec[10];
        orc_lorawan_parse(key, b, len, rec);
        free(b);
    }
}

int main(void) {
    for (unsigned sf = 5; sf <= 12; ++sf) {
        const size_t plen = sf >= 11 ? 4 + rnd() % 5 : rnd() % 33;
        roundtrip(sf, 125000, 1, 0, plen, 1.0f);
        roundtrip(sf, 250000, 1, 1, plen ? plen - 1 : 0, 0.5f);
        if (sf <= 10) roundtrip(sf, 125000, 2, 0, 3 + rnd() % 8, 1.0f);
        estimate_compensate(sf, 1);
        if (sf <= 9) estimate_compensate(sf, 2);
    }
    roundtrip(7, 500000, 1, 0, 0, 1.0f); /* header-only frame: 2 sync symbols */
    garbage_symbols();
    codecs();
    lorawan();
    if (fails) {
        fprintf(stderr, "%d checks failed\n", fails);
        return 1;
    }
    printf("oracle sanitizer driver: all checks held\n");
    return 0;
}
