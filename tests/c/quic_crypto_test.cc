// quic_crypto_test.cc -- host build of the device cryptography in
// mercury_amd/csrc/mfp_quic_crypto.hpp, checked against known answers and
// against OpenSSL's libcrypto (test infrastructure only; the product runs
// these functions on the GPU, in k_quic).
//
//   RFC 9001 Appendix A.1 (also the reference's own unit test,
//   crypto_engine.h:334-495): client Initial secrets for DCID 8394c8f03e515708
//   RFC 9001 Appendix A.2: header-protection mask of the sample
//   random vectors: SHA-256 / HMAC / AES-128 / AES-128-GCM (encrypt with
//   OpenSSL, then GHASH + CTR as k_quic computes them)
//
// Build: g++ -O2 -std=c++17 -I mercury_amd/csrc tests/c/quic_crypto_test.cc -lcrypto
// Exit status 0 when every check passes.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/sha.h>

#define QHD inline
#include "mfp_quic_crypto.hpp"

using namespace mfpq;

static int fails = 0;
#define CHECK(c, ...)                                    \
    do {                                                 \
        if (!(c)) {                                      \
            fails++;                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                \
            fprintf(stderr, "\n");                       \
        }                                                \
    } while (0)

static std::vector<uint8_t> unhex(const char *h) {
    std::vector<uint8_t> v;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) {
        unsigned x;
        sscanf(h + i, "%2x", &x);
        v.push_back((uint8_t)x);
    }
    return v;
}
static void to_words(const uint8_t *b, size_t n, uint32_t *w, size_t nw) {
    for (size_t k = 0; k < nw; k++) w[k] = be_word(b, (uint32_t)n, (uint32_t)k);
}
static void words_to_bytes(const uint32_t *w, size_t n, uint8_t *b) {
    for (size_t i = 0; i < n; i++) b[i] = (uint8_t)(w[i / 4] >> (24 - 8 * (i % 4)));
}

// HKDF-Extract + the four Expand-Labels, as k_quic composes them
static void initial_keys(const uint8_t *salt, const uint8_t *dcid, size_t dl, const char *kl, const char *ivl,
                         const char *hpl, uint8_t csec[32], uint8_t key[16], uint8_t iv[12], uint8_t hp[16]) {
    uint32_t sw[5];
    to_words(salt, 20, sw, 5);
    Hmac m;
    hmac_init_words(m, sw, 5);
    uint32_t mw[14];
    to_words(dcid, dl, mw, 14);
    uint32_t sec[8];
    hmac_short(m, mw, (uint32_t)dl, sec);
    Hmac m2;
    hmac_init_words(m2, sec, 8);
    uint32_t cs[8];
    hkdf_expand_label(m2, "tls13 client in", 15, 32, cs);
    words_to_bytes(cs, 32, csec);
    Hmac m3;
    hmac_init_words(m3, cs, 8);
    uint32_t o[8];
    hkdf_expand_label(m3, kl, (uint32_t)strlen(kl), 16, o); words_to_bytes(o, 16, key);
    hkdf_expand_label(m3, ivl, (uint32_t)strlen(ivl), 12, o); words_to_bytes(o, 12, iv);
    hkdf_expand_label(m3, hpl, (uint32_t)strlen(hpl), 16, o); words_to_bytes(o, 16, hp);
}

static void aes_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    uint32_t kw[4], rk[44], iw[4], ow[4];
    to_words(key, 16, kw, 4);
    aes128_expand(kAes.te0, kw, rk);
    to_words(in, 16, iw, 4);
    aes128_encrypt(kAes.te0, rk, iw, ow);
    words_to_bytes(ow, 16, out);
}

// GCM decrypt + tag check, the composition k_quic uses
static bool gcm_open(const uint8_t key[16], const uint8_t iv[12], const uint8_t *aad, size_t al, const uint8_t *ct,
                     size_t cl, const uint8_t tag[16], uint8_t *pt) {
    uint32_t kw[4], rk[44];
    to_words(key, 16, kw, 4);
    aes128_expand(kAes.te0, kw, rk);
    uint32_t z[4] = {0, 0, 0, 0}, H[4];
    aes128_encrypt(kAes.te0, rk, z, H);
    uint64_t tab[32];
    ghash_table(tab, 1, 0, ((uint64_t)H[0] << 32) | H[1], ((uint64_t)H[2] << 32) | H[3]);
    uint64_t xh = 0, xl = 0;
    auto absorb = [&](const uint8_t *p, size_t n) {
        for (size_t b = 0; b < n; b += 16) {
            uint8_t blk[16] = {};
            memcpy(blk, p + b, n - b < 16 ? n - b : 16);
            uint32_t w[4];
            to_words(blk, 16, w, 4);
            xh ^= ((uint64_t)w[0] << 32) | w[1];
            xl ^= ((uint64_t)w[2] << 32) | w[3];
            ghash_mul(tab, 1, 0, xh, xl);
        }
    };
    absorb(aad, al);
    absorb(ct, cl);
    xl ^= (uint64_t)cl * 8;
    xh ^= (uint64_t)al * 8;
    ghash_mul(tab, 1, 0, xh, xl);
    uint32_t ivw[3];
    to_words(iv, 12, ivw, 3);
    for (size_t b = 0; b < cl; b += 16) {
        uint32_t cb[4] = {ivw[0], ivw[1], ivw[2], (uint32_t)(b / 16 + 2)}, ks[4];
        aes128_encrypt(kAes.te0, rk, cb, ks);
        uint8_t kb[16];
        words_to_bytes(ks, 16, kb);
        for (size_t j = 0; j < 16 && b + j < cl; j++) pt[b + j] = ct[b + j] ^ kb[j];
    }
    uint32_t j0[4] = {ivw[0], ivw[1], ivw[2], 1}, ej[4];
    aes128_encrypt(kAes.te0, rk, j0, ej);
    uint32_t t[4] = {(uint32_t)(xh >> 32) ^ ej[0], (uint32_t)xh ^ ej[1], (uint32_t)(xl >> 32) ^ ej[2], (uint32_t)xl ^ ej[3]};
    uint8_t tb[16];
    words_to_bytes(t, 16, tb);
    return memcmp(tb, tag, 16) == 0;
}

int main() {
    // ---- RFC 9001 A.1
    {
        const auto salt = unhex("38762cf7f55934b34d179ae6a4c80cadccbb7f0a");
        const auto dcid = unhex("8394c8f03e515708");
        uint8_t cs[32], key[16], iv[12], hp[16];
        initial_keys(salt.data(), dcid.data(), dcid.size(), "tls13 quic key", "tls13 quic iv", "tls13 quic hp", cs, key, iv,
                     hp);
        CHECK(!memcmp(cs, unhex("c00cf151ca5be075ed0ebfb5c80323c42d6b7db67881289af4008f1f6c357aea").data(), 32),
              "client_initial_secret");
        CHECK(!memcmp(key, unhex("1f369613dd76d5467730efcbe3b1a22d").data(), 16), "quic key");
        CHECK(!memcmp(iv, unhex("fa044b2f42a3fd3b46fb255c").data(), 12), "quic iv");
        CHECK(!memcmp(hp, unhex("9f50449e04a0e810283a1e9933adedd2").data(), 16), "quic hp");
        // ---- RFC 9001 A.2: mask = AES-ECB(hp, sample)
        uint8_t mask[16];
        aes_block(hp, unhex("d1b1c98dd7689fb8ec11d242b123dc9b").data(), mask);
        CHECK(!memcmp(mask, unhex("437b9aec36").data(), 5), "header protection mask");
    }
    std::mt19937_64 rng(0x5eed0009);
    auto fill = [&](uint8_t *p, size_t n) { for (size_t i = 0; i < n; i++) p[i] = (uint8_t)rng(); };
    // ---- SHA-256 / HMAC-SHA256 against libcrypto (short messages, keys of 5..64 bytes)
    for (int it = 0; it < 200; it++) {
        uint8_t k[64], msg[55], ref[32];
        const size_t kl = 5 + rng() % 60, ml = rng() % 56;
        fill(k, kl);
        fill(msg, ml);
        unsigned rl = 0;
        HMAC(EVP_sha256(), k, (int)kl, msg, ml, ref, &rl);
        uint32_t kw[16], mw[14], out[8];
        to_words(k, kl, kw, 16);
        to_words(msg, ml, mw, 14);
        Hmac m;
        hmac_init_words(m, kw, 16);
        hmac_short(m, mw, (uint32_t)ml, out);
        uint8_t ob[32];
        words_to_bytes(out, 32, ob);
        CHECK(!memcmp(ob, ref, 32), "hmac iteration %d (key %zu, msg %zu)", it, kl, ml);
    }
    // ---- AES-128 block against libcrypto
    for (int it = 0; it < 200; it++) {
        uint8_t key[16], in[16], ref[32], out[16];
        fill(key, 16);
        fill(in, 16);
        EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
        int l = 0;
        EVP_EncryptInit_ex(c, EVP_aes_128_ecb(), nullptr, key, nullptr);
        EVP_CIPHER_CTX_set_padding(c, 0);
        EVP_EncryptUpdate(c, ref, &l, in, 16);
        EVP_CIPHER_CTX_free(c);
        aes_block(key, in, out);
        CHECK(!memcmp(out, ref, 16), "aes iteration %d", it);
    }
    // ---- AES-128-GCM: seal with libcrypto, open with the k_quic composition
    for (int it = 0; it < 300; it++) {
        uint8_t key[16], iv[12], aad[96], pt[2048], ct[2048], tag[16], back[2048];
        const size_t al = 1 + rng() % 96, pl = rng() % 2033;
        fill(key, 16); fill(iv, 12); fill(aad, al); fill(pt, pl);
        EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
        int l = 0;
        EVP_EncryptInit_ex(c, EVP_aes_128_gcm(), nullptr, nullptr, nullptr);
        EVP_EncryptInit_ex(c, nullptr, nullptr, key, iv);
        EVP_EncryptUpdate(c, nullptr, &l, aad, (int)al);
        EVP_EncryptUpdate(c, ct, &l, pt, (int)pl);
        EVP_EncryptFinal_ex(c, ct + l, &l);
        EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_GET_TAG, 16, tag);
        EVP_CIPHER_CTX_free(c);
        const bool ok = gcm_open(key, iv, aad, al, ct, pl, tag, back);
        CHECK(ok, "gcm tag iteration %d (aad %zu, pt %zu)", it, al, pl);
        CHECK(!memcmp(back, pt, pl), "gcm plaintext iteration %d", it);
        if (pl) {
            ct[rng() % pl] ^= 1;
            CHECK(!gcm_open(key, iv, aad, al, ct, pl, tag, back), "gcm forged ciphertext accepted, iteration %d", it);
        }
    }
    if (fails) {
        fprintf(stderr, "%d checks failed\n", fails);
        return 1;
    }
    printf("quic crypto: all checks passed\n");
    return 0;
}
