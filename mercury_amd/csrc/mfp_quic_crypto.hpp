// mfp_quic_crypto.hpp -- the cryptography a QUIC Initial needs before its
// ClientHello can be fingerprinted, written for one lane per packet on gfx950
// (and compiled for the host by the crypto unit test, tests/c/quic_crypto_test.cc).
//
// The reference delegates all of it to OpenSSL (crypto_engine.h:59-148,
// 264-327; quic.h:916-1013): HKDF-Extract / HKDF-Expand-Label over HMAC-SHA256
// for the Initial secrets, AES-128-ECB for the header-protection mask and
// AES-128-GCM (with tag check) for the payload.  Here each is restated from its
// specification: SHA-256 (FIPS 180-4), HMAC (RFC 2104), HKDF (RFC 5869) with
// the TLS 1.3 label layout crypto_engine.h:271-277 builds, AES-128 (FIPS 197,
// the 32-bit T-table form: one 1 KiB table in LDS, its three rotations and the
// S-box derived from it), GCM (NIST SP 800-38D) with GHASH by Shoup's 4-bit
// table method (a 256-byte table per lane, in LDS).
//
// Everything a lane keeps is in registers (round keys, hash state) except the
// two tables; no step depends on another lane.
#pragma once
#include <stdint.h>

#ifndef QHD
#define QHD __host__ __device__ __forceinline__
#endif

namespace mfpq {

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4 §6.2)
// ---------------------------------------------------------------------------
constexpr uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2,
};

struct Sha256 {
    uint32_t h[8];
};

QHD uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

QHD void sha256_init(Sha256 &s) {
    s.h[0] = 0x6a09e667; s.h[1] = 0xbb67ae85; s.h[2] = 0x3c6ef372; s.h[3] = 0xa54ff53a;
    s.h[4] = 0x510e527f; s.h[5] = 0x9b05688c; s.h[6] = 0x1f83d9ab; s.h[7] = 0x5be0cd19;
}

// one 64-byte block, given as 16 big-endian words
QHD void sha256_block(Sha256 &s, const uint32_t in[16]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = in[i];
    uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
            const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
            const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
            wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + kSha256K[i] + wi;
        const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
        const uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
        const uint32_t t2 = S0 + maj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    s.h[0] += a; s.h[1] += b; s.h[2] += c; s.h[3] += d;
    s.h[4] += e; s.h[5] += f; s.h[6] += g; s.h[7] += h;
}

// big-endian word k of a byte string (bytes past len read as 0)
QHD uint32_t be_word(const uint8_t *p, uint32_t len, uint32_t k) {
    uint32_t w = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t i = 4 * k + j;
        w = (w << 8) | (i < len ? (uint32_t)p[i] : 0u);
    }
    return w;
}

// ---------------------------------------------------------------------------
// HMAC-SHA256 (RFC 2104) with the key's inner/outer states computed once
// ---------------------------------------------------------------------------
struct Hmac {
    Sha256 inner, outer;   // state after the ipad / opad block
};

// key given as big-endian words (klen <= 64 bytes, zero-padded words)
QHD void hmac_init_words(Hmac &m, const uint32_t *kw, uint32_t nkw) {
    uint32_t blk[16];
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) blk[i] = (i < nkw ? kw[i] : 0u) ^ 0x36363636u;
    sha256_init(m.inner);
    sha256_block(m.inner, blk);
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) blk[i] ^= 0x36363636u ^ 0x5c5c5c5cu;
    sha256_init(m.outer);
    sha256_block(m.outer, blk);
}

// HMAC(key, msg) for a message of at most 55 bytes given as 14 big-endian
// words (zero past len): one inner block, one outer block.  out: 8 words.
QHD void hmac_short(const Hmac &m, const uint32_t mw[14], uint32_t mlen, uint32_t out[8]) {
    uint32_t blk[16];
#pragma unroll
    for (uint32_t i = 0; i < 14; i++) blk[i] = mw[i];
    // the 0x80 terminator after the last message byte
    const uint32_t wi = mlen >> 2, sh = 24 - 8 * (mlen & 3);
#pragma unroll
    for (uint32_t i = 0; i < 14; i++)
        if (i == wi) blk[i] |= 0x80u << sh;
    blk[14] = 0;
    blk[15] = (64 + mlen) * 8;
    Sha256 s = m.inner;
    sha256_block(s, blk);
#pragma unroll
    for (int i = 0; i < 8; i++) blk[i] = s.h[i];
    blk[8] = 0x80000000u;
#pragma unroll
    for (int i = 9; i < 15; i++) blk[i] = 0;
    blk[15] = (64 + 32) * 8;
    Sha256 o = m.outer;
    sha256_block(o, blk);
#pragma unroll
    for (int i = 0; i < 8; i++) out[i] = o.h[i];
}

// HKDF-Expand-Label, single output block (length <= 32), the label layout of
// crypto_engine.h:271-277: {0x00, length, label_len, label..., 0x00} then the
// block counter 0x01.  `label` is the full label ("tls13 quic key"), up to 30
// bytes.
QHD void hkdf_expand_label(const Hmac &m, const char *label, uint32_t label_len, uint32_t length, uint32_t out[8]) {
    uint8_t info[56];
#pragma unroll
    for (int i = 0; i < 56; i++) info[i] = 0;
    info[0] = 0;
    info[1] = (uint8_t)length;
    info[2] = (uint8_t)label_len;
    for (uint32_t i = 0; i < label_len; i++) info[3 + i] = (uint8_t)label[i];
    info[3 + label_len] = 0;        // context length
    info[4 + label_len] = 1;        // T(1) counter
    const uint32_t mlen = 5 + label_len;
    uint32_t mw[14];
#pragma unroll
    for (uint32_t k = 0; k < 14; k++) mw[k] = be_word(info, mlen, k);
    hmac_short(m, mw, mlen, out);
}

// ---------------------------------------------------------------------------
// AES-128 (FIPS 197), T-table form
// ---------------------------------------------------------------------------
struct AesTables {
    uint32_t sbox[256];
    uint32_t te0[256];
};
constexpr uint32_t gf_xtime(uint32_t x) { return ((x << 1) ^ ((x & 0x80) ? 0x1b : 0)) & 0xff; }
constexpr uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) r ^= a;
        a = gf_xtime(a);
        b >>= 1;
    }
    return r;
}
constexpr uint32_t gf_inv(uint32_t x) {   // x^254
    uint32_t r = 1, b = x;
    uint32_t e = 254;
    while (e) {
        if (e & 1) r = gf_mul(r, b);
        b = gf_mul(b, b);
        e >>= 1;
    }
    return x ? r : 0;
}
constexpr uint32_t aes_sbox_entry(uint32_t x) {
    const uint32_t b = gf_inv(x);
    uint32_t s = b;
    for (int k = 1; k <= 4; k++) s ^= ((b << k) | (b >> (8 - k))) & 0xff;
    return (s ^ 0x63) & 0xff;
}
constexpr AesTables make_aes_tables() {
    AesTables t{};
    for (uint32_t x = 0; x < 256; x++) {
        const uint32_t s = aes_sbox_entry(x);
        t.sbox[x] = s;
        t.te0[x] = (gf_mul(s, 2) << 24) | (s << 16) | (s << 8) | gf_mul(s, 3);
    }
    return t;
}
constexpr AesTables kAes = make_aes_tables();
static_assert(kAes.sbox[0] == 0x63 && kAes.sbox[1] == 0x7c && kAes.sbox[0x53] == 0xed, "AES S-box");
static_assert(kAes.te0[0] == 0xc66363a5u, "AES T-table");

// te: the 256-entry T0 table (LDS on the device); S[x] = (te[x] >> 8) & 0xff
QHD uint32_t aes_sub_word(const uint32_t *te, uint32_t w) {
    return (((te[w >> 24] >> 8) & 0xff) << 24) | (((te[(w >> 16) & 0xff] >> 8) & 0xff) << 16) |
           (((te[(w >> 8) & 0xff] >> 8) & 0xff) << 8) | ((te[w & 0xff] >> 8) & 0xff);
}

// key schedule: 44 words from 4 big-endian key words
QHD void aes128_expand(const uint32_t *te, const uint32_t key[4], uint32_t rk[44]) {
    rk[0] = key[0]; rk[1] = key[1]; rk[2] = key[2]; rk[3] = key[3];
    uint32_t rcon = 0x01;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint32_t t = rk[4 * i + 3];
        const uint32_t rot = (t << 8) | (t >> 24);
        rk[4 * i + 4] = rk[4 * i] ^ aes_sub_word(te, rot) ^ (rcon << 24);
        rk[4 * i + 5] = rk[4 * i + 1] ^ rk[4 * i + 4];
        rk[4 * i + 6] = rk[4 * i + 2] ^ rk[4 * i + 5];
        rk[4 * i + 7] = rk[4 * i + 3] ^ rk[4 * i + 6];
        rcon = gf_xtime(rcon);
    }
}

QHD uint32_t ror8(uint32_t x) { return (x >> 8) | (x << 24); }
QHD uint32_t ror16(uint32_t x) { return (x >> 16) | (x << 16); }
QHD uint32_t ror24(uint32_t x) { return (x >> 24) | (x << 8); }

// one block: in/out as 4 big-endian words
QHD void aes128_encrypt(const uint32_t *te, const uint32_t rk[44], const uint32_t in[4], uint32_t out[4]) {
    uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < 10; r++) {
        const uint32_t t0 = te[s0 >> 24] ^ ror8(te[(s1 >> 16) & 0xff]) ^ ror16(te[(s2 >> 8) & 0xff]) ^ ror24(te[s3 & 0xff]) ^ rk[4 * r];
        const uint32_t t1 = te[s1 >> 24] ^ ror8(te[(s2 >> 16) & 0xff]) ^ ror16(te[(s3 >> 8) & 0xff]) ^ ror24(te[s0 & 0xff]) ^ rk[4 * r + 1];
        const uint32_t t2 = te[s2 >> 24] ^ ror8(te[(s3 >> 16) & 0xff]) ^ ror16(te[(s0 >> 8) & 0xff]) ^ ror24(te[s1 & 0xff]) ^ rk[4 * r + 2];
        const uint32_t t3 = te[s3 >> 24] ^ ror8(te[(s0 >> 16) & 0xff]) ^ ror16(te[(s1 >> 8) & 0xff]) ^ ror24(te[s2 & 0xff]) ^ rk[4 * r + 3];
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
#define MFPQ_SB(x) ((te[(x)] >> 8) & 0xff)
    out[0] = ((MFPQ_SB(s0 >> 24) << 24) | (MFPQ_SB((s1 >> 16) & 0xff) << 16) | (MFPQ_SB((s2 >> 8) & 0xff) << 8) | MFPQ_SB(s3 & 0xff)) ^ rk[40];
    out[1] = ((MFPQ_SB(s1 >> 24) << 24) | (MFPQ_SB((s2 >> 16) & 0xff) << 16) | (MFPQ_SB((s3 >> 8) & 0xff) << 8) | MFPQ_SB(s0 & 0xff)) ^ rk[41];
    out[2] = ((MFPQ_SB(s2 >> 24) << 24) | (MFPQ_SB((s3 >> 16) & 0xff) << 16) | (MFPQ_SB((s0 >> 8) & 0xff) << 8) | MFPQ_SB(s1 & 0xff)) ^ rk[42];
    out[3] = ((MFPQ_SB(s3 >> 24) << 24) | (MFPQ_SB((s0 >> 16) & 0xff) << 16) | (MFPQ_SB((s1 >> 8) & 0xff) << 8) | MFPQ_SB(s2 & 0xff)) ^ rk[43];
#undef MFPQ_SB
}

// ---------------------------------------------------------------------------
// GHASH (SP 800-38D §6.4) by 4-bit tables: M[i] = i * H for the 16 nibble
// values, in GCM's reflected bit order, as two 64-bit halves (big-endian
// halves of the 128-bit block).  The table lives in LDS, interleaved by lane:
// entry k of lane l at tab[k * stride + l] (k = 0..15 high halves, 16..31 low).
// ---------------------------------------------------------------------------
// r * (x^128 reduction for 4 shifted-out bits): the 16-entry table of the
// method, as its linear combination of the four single-bit values
QHD uint64_t ghash_rem4(uint32_t r) {
    uint32_t v = 0;
    v ^= (0u - (r & 1)) & 0x1c20u;
    v ^= (0u - ((r >> 1) & 1)) & 0x3840u;
    v ^= (0u - ((r >> 2) & 1)) & 0x7080u;
    v ^= (0u - ((r >> 3) & 1)) & 0xe100u;
    return (uint64_t)v << 48;
}

QHD void ghash_table(uint64_t *tab, uint32_t stride, uint32_t lane, uint64_t hh, uint64_t hl) {
    // nibble 8 (bit pattern 1000) is the field's 1: M[8] = H
    uint64_t H[16], L[16];
    H[0] = 0; L[0] = 0;
    H[8] = hh; L[8] = hl;
    uint64_t vh = hh, vl = hl;
#pragma unroll
    for (int i = 4; i > 0; i >>= 1) {     // M[4] = H*x, M[2] = H*x^2, M[1] = H*x^3
        const uint64_t t = (vl & 1) ? 0xe100000000000000ull : 0ull;
        vl = (vh << 63) | (vl >> 1);
        vh = (vh >> 1) ^ t;
        H[i] = vh; L[i] = vl;
    }
#pragma unroll
    for (int i = 2; i <= 8; i *= 2) {
#pragma unroll
        for (int j = 1; j < i; j++) { H[i + j] = H[i] ^ H[j]; L[i + j] = L[i] ^ L[j]; }
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        tab[(uint32_t)k * stride + lane] = H[k];
        tab[(uint32_t)(16 + k) * stride + lane] = L[k];
    }
}

// (xh:xl) <- (xh:xl) * H
QHD void ghash_mul(const uint64_t *tab, uint32_t stride, uint32_t lane, uint64_t &xh, uint64_t &xl) {
    uint64_t zh = 0, zl = 0;
    bool first = true;
#pragma unroll
    for (int i = 15; i >= 0; i--) {
        const uint32_t byte = (uint32_t)((i >= 8 ? xl >> (8 * (15 - i)) : xh >> (8 * (7 - i))) & 0xff);
        const uint32_t lo = byte & 0xf, hi = byte >> 4;
        if (first) {
            zh = tab[lo * stride + lane];
            zl = tab[(16 + lo) * stride + lane];
            first = false;
        } else {
            const uint32_t rem = (uint32_t)(zl & 0xf);
            zl = (zh << 60) | (zl >> 4);
            zh = (zh >> 4) ^ ghash_rem4(rem);
            zh ^= tab[lo * stride + lane];
            zl ^= tab[(16 + lo) * stride + lane];
        }
        const uint32_t rem = (uint32_t)(zl & 0xf);
        zl = (zh << 60) | (zl >> 4);
        zh = (zh >> 4) ^ ghash_rem4(rem);
        zh ^= tab[hi * stride + lane];
        zl ^= tab[(16 + hi) * stride + lane];
    }
    xh = zh; xl = zl;
}

QHD uint32_t bswap32_(uint32_t x) {
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

}  // namespace mfpq
