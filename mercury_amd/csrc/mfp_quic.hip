// mfp_quic.hip -- QUIC Initial packets on the device.
//
// The reference (quic.h:405-1753, crypto_engine.h) turns a UDP payload that
// matches the QUIC long-header matcher (quic.h:544) into a quic_init:
//   1. parse the long header (quic_initial_packet::parse quic.h:421);
//   2. if the reserved bits of the (still protected) first byte are zero, try
//      the payload as plaintext frames (quic_init_decry::parse quic.h:1359);
//   3. otherwise derive the client Initial keys from the version's salt and
//      the DCID (HKDF), remove header protection (AES-ECB of a payload sample),
//      and AES-128-GCM-decrypt the payload, tag checked
//      (quic_crypto_engine::decrypt quic.h:806-1013);
//   4. walk the frames, gather CRYPTO frames into an 8 KiB buffer by offset
//      (cryptographic_buffer quic.h:1203-1294), and parse the buffer (or, when
//      frames are missing, the first frame) as a TLS handshake + ClientHello;
//   5. fingerprint "quic/[1/](version)(tls version)(ciphers)[extensions]"
//      (quic_init::compute_fingerprint quic.h:1702, quic_client_hello quic.h:1313).
//
// k_quic runs that per packet, one lane per packet (the work is sequential
// per packet: 16 SHA-256 blocks, ~80 AES blocks and ~80 GHASH products for a
// 1200-byte Initial, all independent across packets).  Each lane owns a
// scratch slot in HBM for the decrypted payload (2 KiB, the reference's
// pt_buf_len) and the CRYPTO buffer (8 KiB); the AES T-table and the lanes'
// GHASH tables sit in LDS.  The fingerprint is then written like
// k_fingerprint writes its strings (count pass, tile reservation, emission
// pass), followed by the string hash and a *sidecar* with the ClientHello's
// server name, QUIC user agent and ALPN list (they exist only in the
// decrypted payload, so the record's spans index the sidecar; the classifier
// reads them there).
#include <hip/hip_runtime.h>

#include "mfp_device.hpp"
#include "mfp_kphase.hpp"
#define QHD __device__ __forceinline__
#include "mfp_quic_crypto.hpp"

namespace mfp {

constexpr int QT = 128;                          // lanes per workgroup
constexpr uint32_t Q_PT = 2048;                  // decrypted payload (pt_buf_len, crypto_engine.h:30)
constexpr uint32_t Q_CB = 8192;                  // CRYPTO buffer (cryptographic_buffer::crypto_buf_len quic.h:1206)
constexpr uint32_t Q_SLOT = Q_PT + Q_CB + 64;    // per-lane scratch (the emitter may read an aligned word past the end)

// ---- the long header (quic_initial_packet::parse quic.h:421-522)
struct QHdr {
    uint32_t ci;                                 // connection_info (protected first byte)
    const uint8_t *ver;                          // 4 version bytes
    Cur dcid, payload;                           // payload = packet number + protected payload
    const uint8_t *aad_start, *aad_end;          // header bytes before the packet number
    bool valid;
};
DEV QHdr quic_hdr(Cur d) {
    QHdr h;
    h.valid = false; h.ci = 0; h.ver = nullptr;
    cset_null(h.dcid); cset_null(h.payload);
    h.aad_start = d.d; h.aad_end = nullptr;
    if (clen(d) < 1184) return h;                // min_len_pdu quic.h:525
    h.ci = rd_u8(d);
    Cur ver; cparse(ver, d, 4);
    h.ver = ver.d;
    const uint32_t dl = rd_u8(d);
    if (dl > 20) return h;
    cparse(h.dcid, d, (long)dl);
    const uint32_t sl = rd_u8(d);
    if (sl > 20) return h;
    Cur scid; cparse(scid, d, (long)sl);
    const uint64_t tl = vli_rd(d);
    Cur tok; cparse(tok, d, (long)tl);
    const uint64_t len = vli_rd(d);
    if (clen(d) < (long)len || len < 64) return h;   // min_len_pn_and_payload quic.h:524
    h.aad_end = d.d;
    cparse(h.payload, d, (long)len);
    if (!cnotempty(h.payload)) return h;
    h.valid = true;
    return h;
}

// ---- Initial parameters per version (quic_parameters quic.h:551-764):
// salt index, and whether the version uses the v2 labels and packet-type bits
DEV bool quic_version(uint32_t v, uint32_t &salt, bool &v2) {
    v2 = false;
    switch (v) {
    case 0xfaceb001u: case 0xff000016u: salt = 0; return true;
    case 0xfaceb002u: case 0xfaceb00eu: case 0xfaceb010u: case 0xfaceb011u: case 0xfaceb012u: case 0xfaceb013u:
    case 0xff000017u: case 0xff000018u: case 0xff000019u: case 0xff00001au: case 0xff00001bu: case 0xff00001cu:
        salt = 1; return true;
    case 0xff00001du: case 0xff00001eu: case 0xff00001fu: case 0xff000020u: salt = 2; return true;
    case 0xfacefeedu: case 0xff000021u: case 0xff000022u: case 0x00000001u: case 0xd4000400u: salt = 3; return true;
    case 0x709a50c4u: salt = 4; v2 = true; return true;
    case 0x6b3343cfu: salt = 5; v2 = true; return true;
    }
    return false;
}
// the six salts (quic.h:595-602) as big-endian words
constexpr uint32_t kSalt[6][5] = {
    {0x7fbcdb0e, 0x7c66bbe9, 0x193a96cd, 0x21519ebd, 0x7a02644a},
    {0xc3eef712, 0xc72ebb5a, 0x11a7d243, 0x2bb46365, 0xbef9f502},
    {0xafbfec28, 0x9993d24c, 0x9e9786f1, 0x9c6111e0, 0x4390a899},
    {0x38762cf7, 0xf55934b3, 0x4d179ae6, 0xa4c80cad, 0xccbb7f0a},
    {0xa707c203, 0xa59b4718, 0x4a1d62ca, 0x570406ea, 0x7ae3e5d3},
    {0x0dede3de, 0xf700a6db, 0x819381be, 0x6e269dcb, 0xf9bd2ed9},
};

// HKDF-Expand-Label messages ({0, length, label_len, label, 0, counter 1},
// crypto_engine.h:271-277) as big-endian words, built at compile time
struct LabelMsg {
    uint32_t w[14];
    uint32_t len;
};
constexpr LabelMsg make_label(const char *label, uint32_t length) {
    LabelMsg m{};
    uint32_t ll = 0;
    while (label[ll]) ll++;
    uint8_t b[56] = {};
    b[1] = (uint8_t)length;
    b[2] = (uint8_t)ll;
    for (uint32_t i = 0; i < ll; i++) b[3 + i] = (uint8_t)label[i];
    b[4 + ll] = 1;
    m.len = 5 + ll;
    for (int k = 0; k < 14; k++)
        m.w[k] = ((uint32_t)b[4 * k] << 24) | ((uint32_t)b[4 * k + 1] << 16) | ((uint32_t)b[4 * k + 2] << 8) | b[4 * k + 3];
    return m;
}
constexpr LabelMsg kClientIn = make_label("tls13 client in", 32);
constexpr LabelMsg kKey1 = make_label("tls13 quic key", 16), kKey2 = make_label("tls13 quicv2 key", 16);
constexpr LabelMsg kIv1 = make_label("tls13 quic iv", 12), kIv2 = make_label("tls13 quicv2 iv", 12);
constexpr LabelMsg kHp1 = make_label("tls13 quic hp", 16), kHp2 = make_label("tls13 quicv2 hp", 16);

DEV void expand(const mfpq::Hmac &m, const LabelMsg &a, const LabelMsg &b, bool use_b, uint32_t out[8]) {
    uint32_t w[14];
#pragma unroll
    for (int k = 0; k < 14; k++) w[k] = use_b ? b.w[k] : a.w[k];
    mfpq::hmac_short(m, w, use_b ? b.len : a.len, out);
}

// len bytes src -> dst (disjoint, any alignment) with 8-byte stores at dst's
// alignment, each word funnel-shifted from two aligned 8-byte loads of src
// (byte-wise moves of a lane's own scratch slot are one memory transaction per
// byte per lane); src may be read up to 7 bytes past its end
DEV void copy_bytes(uint8_t *dst, const uint8_t *src, uint32_t len) {
    uint32_t j = 0;
    while (j < len && (((uintptr_t)(dst + j)) & 7)) { dst[j] = src[j]; j++; }
    if (j + 8 <= len) {
        const uintptr_t a = (uintptr_t)(src + j);
        const uint64_t *q = (const uint64_t *)(a & ~(uintptr_t)7);
        const uint32_t sh = (uint32_t)(a & 7) * 8;
        uint64_t cur = q[0];
        for (; j + 8 <= len; j += 8) {
            const uint64_t nxt = *++q;
            *(uint64_t *)(dst + j) = sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
            cur = nxt;
        }
    }
    for (; j < len; j++) dst[j] = src[j];
}

// big-endian word of packet bytes p[0..n) (n <= 4), zero-padded
DEV uint32_t be_bytes(const uint8_t *p, uint32_t n) {
    return n == 0 ? 0u : ld_be32n(p, (int)n) << (8 * (4 - n));
}

DEV void ghash_block(const uint64_t *gh, uint32_t lane, uint64_t &xh, uint64_t &xl, uint32_t w0, uint32_t w1, uint32_t w2,
                     uint32_t w3) {
    xh ^= ((uint64_t)w0 << 32) | w1;
    xl ^= ((uint64_t)w2 << 32) | w3;
    mfpq::ghash_mul(gh, QT, lane, xh, xl);
}

// quic_crypto_engine::decrypt for the version's parameters (quic.h:806-866,
// 916-1013; crypto_engine.h:89-148).  Returns -2 when the first byte is not an
// Initial of this version (the reference then marks the packet invalid:
// quic.h:825-829), -1 when there is no plaintext (unknown version, reserved
// bits set after unmasking, AAD over 1 KiB), 0 with *pt_len bytes of plaintext
// in pt (0 when the tag does not verify).
DEV int quic_decrypt(const QHdr &h, uint8_t *pt, const uint32_t *te, uint64_t *gh, uint32_t lane, uint32_t &pt_len) {
    pt_len = 0;
    const uint32_t v = ld_be32n(h.ver, 4);
    uint32_t salt = 0;
    bool v2 = false;
    if (!quic_version(v, salt, v2)) return -1;
    if ((h.ci & 0xb0u) != (v2 ? 0x90u : 0x80u)) return -2;     // init_pkt_masks_values quic.h:668-671

    // Initial secrets: HKDF-Extract(salt, dcid), then Expand-Label
    uint32_t sec[8], key[8], iv[8], hp[8];
    {
        uint32_t sw[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            uint32_t x = kSalt[0][k];
            for (uint32_t s = 1; s < 6; s++) x = salt == s ? kSalt[s][k] : x;
            sw[k] = x;
        }
        mfpq::Hmac m;
        mfpq::hmac_init_words(m, sw, 5);
        const uint32_t dl = (uint32_t)clen(h.dcid);
        uint32_t mw[14];
#pragma unroll
        for (uint32_t k = 0; k < 14; k++) {
            const uint32_t lo = 4 * k;
            mw[k] = lo < dl ? be_bytes(h.dcid.d + lo, dl - lo < 4 ? dl - lo : 4u) : 0u;
        }
        mfpq::hmac_short(m, mw, dl, sec);
        mfpq::Hmac m2;
        mfpq::hmac_init_words(m2, sec, 8);
        expand(m2, kClientIn, kClientIn, false, sec);
        mfpq::Hmac m3;
        mfpq::hmac_init_words(m3, sec, 8);
        expand(m3, kKey1, kKey2, v2, key);
        expand(m3, kIv1, kIv2, v2, iv);
        expand(m3, kHp1, kHp2, v2, hp);
    }
    // header protection (RFC 9001 §5.4): mask = AES-ECB(hp, sample at pn + 4)
    uint32_t rk[44];
    uint32_t mask[4];
    {
        mfpq::aes128_expand(te, hp, rk);
        const uint8_t *sp = h.payload.d + 4;
        const uint32_t smp[4] = {ld_be32n(sp, 4), ld_be32n(sp + 4, 4), ld_be32n(sp + 8, 4), ld_be32n(sp + 12, 4)};
        mfpq::aes128_encrypt(te, rk, smp, mask);
    }
    const uint32_t unm = h.ci ^ ((mask[0] >> 24) & 0x0f);
    if (unm & 0x0c) return -1;                                  // quic.h:963-965
    const uint32_t pnl = (unm & 3) + 1;
    const uint32_t hdr_len = (uint32_t)(h.aad_end - h.aad_start);
    const uint32_t aad_len = hdr_len + pnl;
    if (aad_len > 1024) return -1;                              // data_buffer<1024> (quic.h:811, 982)
    // unprotected packet number bytes (big-endian in pnw's top bytes)
    const uint32_t pn_raw = ld_be32n(h.payload.d, 4);
    const uint32_t pnw = (pn_raw ^ ((mask[0] << 8) | (mask[1] >> 24))) & (0xffffffffu << (8 * (4 - pnl)));
    // AEAD nonce: iv with the packet number XORed into its last bytes (quic.h:988-990)
    {
        const uint64_t pn = (uint64_t)(pnw >> (8 * (4 - pnl)));
        const uint64_t lo = (((uint64_t)iv[1] << 32) | iv[2]) ^ pn;
        iv[1] = (uint32_t)(lo >> 32);
        iv[2] = (uint32_t)lo;
    }

    // AES-128-GCM (crypto_engine.h:89-148): the ciphertext is cut to pt_buf_len,
    // and its last 16 bytes are the tag
    const uint32_t plen = (uint32_t)clen(h.payload);
    const uint32_t cipher_len = (plen - pnl) & 0xffffu;          // uint16_t (quic.h:1004)
    const long ct_len = (long)(cipher_len < 2048u ? cipher_len : 2048u) - 16;
    if (ct_len < 0) return 0;
    const uint8_t *ct = h.payload.d + pnl;
    mfpq::aes128_expand(te, key, rk);
    uint32_t H[4];
    {
        const uint32_t z[4] = {0, 0, 0, 0};
        mfpq::aes128_encrypt(te, rk, z, H);
    }
    mfpq::ghash_table(gh, QT, lane, ((uint64_t)H[0] << 32) | H[1], ((uint64_t)H[2] << 32) | H[3]);
    uint64_t xh = 0, xl = 0;
    // AAD: unprotected first byte, header bytes up to the packet number, the packet number
    for (uint32_t b0 = 0; b0 < aad_len; b0 += 16) {
        uint32_t w[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            uint32_t x = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                const uint32_t a = b0 + 4 * k + j;
                uint32_t by = 0;
                if (a == 0) by = unm;
                else if (a < hdr_len) by = ld(h.aad_start + a);
                else if (a < aad_len) by = (pnw >> (24 - 8 * (a - hdr_len))) & 0xff;
                x = (x << 8) | by;
            }
            w[k] = x;
        }
        ghash_block(gh, lane, xh, xl, w[0], w[1], w[2], w[3]);
    }
    // ciphertext: GHASH over it, CTR keystream from counter 2 (J0 = iv || 1)
    const uint32_t nct = (uint32_t)ct_len;
    // the ciphertext through aligned 8-byte loads (two per block, the third
    // carried to the next block), bytes past ct_len masked off
    const uint64_t *cq = (const uint64_t *)((uintptr_t)ct & ~(uintptr_t)7);
    const uint32_t csh = (uint32_t)((uintptr_t)ct & 7) * 8;
    uint64_t cx0 = nct ? cq[0] : 0ull;
    for (uint32_t b0 = 0, ctr = 2; b0 < nct; b0 += 16, ctr++) {
        const uint32_t left = nct - b0;
        const uint64_t cx1 = cq[b0 / 8 + 1], cx2 = cq[b0 / 8 + 2];
        const uint64_t lo = csh ? (cx0 >> csh) | (cx1 << (64 - csh)) : cx0;
        const uint64_t hi = csh ? (cx1 >> csh) | (cx2 << (64 - csh)) : cx1;
        cx0 = cx2;
        uint32_t c[4] = {__builtin_bswap32((uint32_t)lo), __builtin_bswap32((uint32_t)(lo >> 32)),
                         __builtin_bswap32((uint32_t)hi), __builtin_bswap32((uint32_t)(hi >> 32))};
        if (left < 16) {
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t o = 4 * k, n = o < left ? (left - o < 4 ? left - o : 4u) : 0u;
                c[k] &= n == 0 ? 0u : 0xffffffffu << (8 * (4 - n));
            }
        }
        ghash_block(gh, lane, xh, xl, c[0], c[1], c[2], c[3]);
        const uint32_t cb[4] = {iv[0], iv[1], iv[2], ctr};
        uint32_t ks[4];
        mfpq::aes128_encrypt(te, rk, cb, ks);
        uint4 o4;
        o4.x = __builtin_bswap32(c[0] ^ ks[0]);
        o4.y = __builtin_bswap32(c[1] ^ ks[1]);
        o4.z = __builtin_bswap32(c[2] ^ ks[2]);
        o4.w = __builtin_bswap32(c[3] ^ ks[3]);
        *(uint4 *)(pt + b0) = o4;                               // bytes past ct_len are never read
    }
    ghash_block(gh, lane, xh, xl, 0u, aad_len * 8u, 0u, nct * 8u);
    uint32_t ej[4];
    {
        const uint32_t j0[4] = {iv[0], iv[1], iv[2], 1u};
        mfpq::aes128_encrypt(te, rk, j0, ej);
    }
    const uint8_t *tag = ct + nct;
    const bool ok = (((uint32_t)(xh >> 32) ^ ej[0]) == ld_be32n(tag, 4)) &&
                    (((uint32_t)xh ^ ej[1]) == ld_be32n(tag + 4, 4)) &&
                    (((uint32_t)(xl >> 32) ^ ej[2]) == ld_be32n(tag + 8, 4)) &&
                    (((uint32_t)xl ^ ej[3]) == ld_be32n(tag + 12, 4));
    pt_len = ok ? nct : 0u;
    return 0;
}

// ---- CRYPTO frame gathering (cryptographic_buffer quic.h:1203-1294)
struct CState {
    uint64_t buf_len, min_off, min_len, max_off, max_len;
    uint32_t total, count;
    bool first_ok;        // has_first_frame()
    Cur first;            // crypto_frames[first_frame_index].data()
    const uint8_t *cc;    // the last connection_close / ack (/ ack_ecn) frame's type byte (quic_init::cc)
};
DEV void cs_reset(CState &s) {
    s.buf_len = 0; s.min_off = ~0ull; s.min_len = ~0ull; s.max_off = 0; s.max_len = 0;
    s.total = 0; s.count = 0; s.first_ok = false; cset_null(s.first); s.cc = nullptr;
}
// extend() + update_crypto_frames(); cb[0, hw) holds this packet's bytes
// (written or zero: the reference's buffer starts zeroed for every packet)
DEV void cb_extend(CState &s, uint64_t off, uint64_t len, Cur data, uint8_t *cb, uint32_t &hw) {
    if (off > Q_CB || len > Q_CB || off + len > Q_CB) return;
    for (uint32_t j = hw; j < (uint32_t)off; j++) cb[j] = 0;
    copy_bytes(cb + off, data.d, (uint32_t)len);
    if (off + len > hw) hw = (uint32_t)(off + len);
    if (off + len > s.buf_len) s.buf_len = off + len;
    if (off == 0) { s.first_ok = s.count < 20; s.first = data; }
    if (off <= s.min_off) { s.min_off = off; s.min_len = len; }
    if (off >= s.max_off) { s.max_off = off; s.max_len = len; }
    s.total += (uint32_t)len;
    if (s.count < 20) s.count++;
}
// PADDING runs skipped word-wide in quic_frames (MI355X: k_quic 65.2 -> 51.9 ms per 2 M Initials, profiles/r04i_quic_*)
#ifndef MFP_QUIC_PADSKIP
#define MFP_QUIC_PADSKIP 1
#endif
// the end of a run of zero bytes from d (at most e): four aligned 8-byte
// loads per step, so an Initial's PADDING (hundreds of one-byte frames) costs a
// few dependent loads, not one per byte; reads only [d, e)
DEV const uint8_t *skip_zeros(const uint8_t *d, const uint8_t *e) {
    while (d < e && ((uintptr_t)d & 7)) { if (ld(d)) return d; d++; }
    while (d + 32 <= e) {
        const uint64_t *q = (const uint64_t *)d;
        const uint64_t w[4] = {q[0], q[1], q[2], q[3]};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (w[k]) return d + 8 * k + (__builtin_ctzll(w[k]) >> 3);
        }
        d += 32;
    }
    while (d < e) { if (ld(d)) return d; d++; }
    return e;
}

// the frame loop: strict = quic_init_decry::parse (quic.h:1369-1390: an invalid
// frame or a null cursor fails the whole payload), otherwise quic_init's loop
// (quic.h:1532-1552: stop at the first invalid frame).  Returns strict validity.
DEV bool quic_frames(Cur p, bool strict, CState &s, uint8_t *cb, uint32_t &hw) {
    while (cnotempty(p)) {
        const uint8_t *at = p.d;
        const uint32_t t = rd_u8(p);            // quic_frame ctor quic.h:1131-1152
#if MFP_QUIC_PADSKIP
        if (t == 0x00) {                        // PADDING: the zero bytes that follow are PADDING frames too
            p.d = skip_zeros(p.d, p.e);
            continue;
        }
#endif
        bool crypto = false;
        uint64_t off = 0, len = 0;
        Cur data; cset_null(data);
        if (t == 0x06) {                        // crypto quic.h:233
            off = vli_rd(p); len = vli_rd(p);
            cparse(data, p, (long)len);
            crypto = true;
        } else if (t == 0x1c) {                 // connection_close quic.h:354
            vli_rd(p); vli_rd(p);
            const uint64_t rl = vli_rd(p);
            Cur r; cparse(r, p, (long)rl);
        } else if (t == 0x02 || t == 0x03) {    // ack / ack_ecn quic.h:123-173
            vli_rd(p); vli_rd(p);
            const uint64_t rc = vli_rd(p);
            vli_rd(p);
            if (rc > 1000) cset_null(p);
            else for (uint64_t i = 0; i < rc && cnotempty(p); i++) { vli_rd(p); vli_rd(p); }
            if (t == 0x03) { vli_rd(p); vli_rd(p); vli_rd(p); }
        } else if (t != 0x00 && t != 0x01) {    // padding / ping carry nothing
            return !strict;
        }
        if (strict && cnull(p)) return false;
        if (crypto && cnotempty(data)) cb_extend(s, off, len, data, cb, hw);
        // cc = frame: connection_close or ack, and ack_ecn outside the
        // pre-decrypted parse (quic.h:1389-1391, 1550-1552)
        if (t == 0x1c || t == 0x02 || (t == 0x03 && !strict)) s.cc = at;
    }
    return true;
}

struct QRes {
    uint32_t flags;         // MFP_FLAG_EMIT | MFP_FLAG_TRUNCATED
    bool hello;             // quic_client_hello::is_not_empty()
    bool pre;               // pre_decrypted: fingerprinted with format 0 (quic.h:1455-1463)
    const uint8_t *ver;
    Ch ch;
    // what quic_init::write_json prints (quic.h:1662-1690, 1438-1452)
    Cur plain;              // the plaintext (decrypted payload, or the pre-decrypted frames)
    Cur hs;                 // the bytes the handshake was parsed from
    const uint8_t *cc;      // the cc frame's type byte in `plain`, or null
    uint32_t salt;          // salt of the decryption (0..5), 0xff none
    // reassembly inputs (process_quic_reassembly reassembly.hpp:895-1033)
    uint32_t more;          // additional_bytes_needed (quic.h:1628-1630)
    uint32_t min_off;       // get_min_crypto_offset (quic.h:1644-1646), ~0u without CRYPTO data
};

// quic_init ctor (quic.h:1513-1591)
DEV QRes quic_process(Cur pay, uint8_t *pt, uint8_t *cb, const uint32_t *te, uint64_t *gh, uint32_t lane) {
    QRes r;
    r.flags = 0; r.hello = false; r.pre = false; r.ver = nullptr;
    cset_null(r.ch.version); cset_null(r.ch.ciphers); cset_null(r.ch.compression); cset_null(r.ch.extensions);
    cset_null(r.plain); cset_null(r.hs); r.cc = nullptr; r.salt = 0xff;
    r.more = 0; r.min_off = ~0u;
    const QHdr h = quic_hdr(pay);
    if (!h.valid) return r;
    r.ver = h.ver;
    uint32_t hw = 0;
    CState s;
    cs_reset(s);
    bool use = false;
    if ((h.ci & 0x0c) == 0) {                   // already-decrypted Initial? (quic.h:1517-1523)
        const uint32_t pnl0 = (h.ci & 3) + 1;
        const Cur pl = cmk(h.payload.d + pnl0, h.payload.e);
        if (quic_frames(pl, true, s, cb, hw)) { r.pre = true; use = true; r.plain = pl; }
    }
    if (!use) {
        cs_reset(s);                            // crypto_buffer.reset(): the bytes stay
        uint32_t pt_len = 0;
        const int dr = quic_decrypt(h, pt, te, gh, lane, pt_len);
        if (dr == -2) return r;                 // not an Initial of its version: no record
        if (dr == 0 && pt_len) {
            r.plain = cmk(pt, pt + pt_len);
            bool v2 = false;
            quic_version(ld_be32n(h.ver, 4), r.salt, v2);   // quic_crypto_engine::salt_str (quic.h:821-842)
            quic_frames(r.plain, false, s, cb, hw);
        }
    }
    r.cc = s.cc;
    r.flags = MFP_FLAG_EMIT;                    // is_not_empty(): the header parsed (quic.h:1623)
    if (s.buf_len == 0) return r;               // crypto_buffer.is_valid()
    r.min_off = (uint32_t)s.min_off;
    Cur d;
    if ((uint64_t)s.total == s.max_off + s.max_len - s.min_off) {   // no missing frames (quic.h:1267-1272)
        d = cmk(cb, cb + s.buf_len);
    } else {
        if (!s.first_ok) return r;
        if (clen(s.first) < 10) {               // min_crypto_data: the buffer's first 10 bytes
            for (uint32_t j = hw; j < 10; j++) cb[j] = 0;
            if (hw < 10) hw = 10;
            d = cmk(cb, cb + 10);
        } else {
            d = s.first;
        }
    }
    r.hs = d;
    const Hs hs = tls_hs_parse(d);
    r.more = (uint32_t)hs.more;                 // more_bytes_needed (uint32_t)
    if (r.more) r.flags |= MFP_FLAG_TRUNCATED;
    r.ch = tls_ch_parse(hs.body);
    r.hello = cnotempty(r.ch.compression);
    return r;
}

// quic_init::compute_fingerprint + quic_client_hello::fingerprint
template <class E>
DEV void quic_fp(E &b, const QRes &q, uint32_t fmt) {
    fp_type_prefix(b, 12);
    if (fmt) { b.putc('0' + fmt); b.putc('/'); }   // set_type(quic, format) fingerprint.h:44-52
    b.putc('('); b.hex(q.ver, 4); b.putc(')');      // quic_hdr_fp quic.h:1301
    b.putc('('); b.hex(q.ch.version.d, clen(q.ch.version)); b.putc(')');
    b.putc('('); hex_degrease(b, q.ch.ciphers.d, clen(q.ch.ciphers)); b.putc(')');
    exts_fp12(b, q.ch.extensions, 0, (int)fmt + 1);   // fmt 0: fingerprint_quic_tls, 1: fingerprint_format2
}

// classifier inputs (tls_extensions::set_meta_data tls.h:1316-1370): server
// name, the QUIC user agent (transport parameter 0x3129 of extension 0xffa5)
// and the ALPN list; the last of each wins
struct QMeta { Cur sni, ua, alpn; };
DEV QMeta quic_meta(Cur exts) {
    QMeta m; cset_null(m.sni); cset_null(m.ua); cset_null(m.alpn);
    Cur p = exts;
    while (clen(p) > 0) {
        const uint8_t *start = p.d;
        uint64_t t, l;
        if (!rd_uint(p, 2, t)) break;
        if (!rd_uint(p, 2, l)) break;
        if (!cskip(p, (long)l)) break;
        if (t == 0) { Cur e = cmk(start, p.d); cskip(e, 9); m.sni = e; }
        if (t == 0xffa5) {
            Cur e = cmk(start, p.d);
            cskip(e, 4);
            while (clen(e) > 0) {                // quic_transport_parameter tls.h:1244
                Cur id; cparse(id, e, vli_len(look_u8(e)));
                const uint64_t vl = vli_rd(e);
                Cur val; cparse(val, e, (long)vl);
                if (vli_value(id) == 0x3129) m.ua = val;
            }
        }
        if (t == 16) {                           // protocol_name_list tls.h:1172-1176
            Cur e = cmk(start, p.d);
            cskip(e, 4);
            uint64_t al;
            if (rd_uint(e, 2, al) && (uint64_t)clen(e) >= al) m.alpn = cmk(e.d, e.d + al);
            else cset_null(m.alpn);
        }
    }
    return m;
}
DEV uint32_t span_len(Cur c) { return cnull(c) ? 0u : (uint32_t)clen(c); }

// ---- OpenVPN over TCP (openvpn_tcp openvpn.h:353-500)
// One record (openvpn_tcp_record openvpn.h:272-290 over openvpn_payload
// openvpn.h:116-246).  Only the fields the fingerprint needs are kept; the
// cursor advances over exactly what the reference reads (a record that is
// not P_CONTROL_V1 consumes its header only, not its length field's span).
struct OvRec { uint32_t opcode, key, hmac_len; Cur data; bool ctrl, valid; };
DEV OvRec ovpn_record(Cur &d) {
    OvRec r; r.hmac_len = 0; r.valid = false; cset_null(r.data);
    uint64_t len, code, t;
    rd_uint(d, 2, len);
    rd_uint(d, 1, code);
    r.opcode = (uint32_t)code >> 3;                      // code.slice<0,5>
    r.key = (uint32_t)code & 7;                          // code.slice<5,8>
    const uint32_t op = r.opcode;
    const int type = (op >= 1 && op <= 4) || op == 7 || op == 8 || op == 10 || op == 11 ? 1   // ctrl
                   : op == 5 ? 0 : (op == 6 || op == 9) ? 2 : 3;                            // ack, data, unknown
    r.ctrl = type == 1;
    const bool have_data = op == 4;
    // openvpn_payload::parse
    rd_uint(d, 8, t);                                    // session_id
    uint64_t hm = 0;
    { Cur la = d; rd_uint(la, 4, hm); }                  // lookahead: 0 when short
    uint32_t zeros = 0;
    for (int k = 0; k < 4; k++) zeros += ((hm >> (8 * k)) & 0xff) == 0;
    bool tls_auth = false;
    if (zeros <= 1) {                                    // valid_HMAC: entropy check
        if (clen(d) < 16) return r;
        // datum::find_delim(0x00 0x00) (datum.h:546-567): index just past the
        // first two zero bytes, or minus the bytes scanned; then - 2 as uint8_t
        long at = 0, m = 0;
        const long dl = clen(d);
        while (m < 2 && at < dl) { m = ld(d.d + at) == 0 ? m + 1 : 0; at++; }
        const long fd = m == 2 ? at : -at;
        const uint32_t hl = (uint32_t)(uint8_t)(fd - 2);
        if (hl < 16 || (long)hl >= clen(d)) return r;
        r.hmac_len = hl;
        cskip(d, (long)hl);
        tls_auth = true;
    }
    (void)tls_auth;
    rd_uint(d, 4, t);                                    // replay_pkt_id
    bool net_time = false;
    {
        Cur dc = d;
        const uint32_t b1 = rd_u8(dc), b2 = rd_u8(dc);
        if ((long)b1 * 4 > clen(dc) || b2) net_time = true;
    }
    if (net_time) rd_uint(d, 4, t);
    const uint32_t nid = rd_u8(d);                       // pkt_id_array_len
    if (clen(d) < 4 * (long)nid) return r;
    if (nid) { cskip(d, 4 * (long)nid); rd_uint(d, 8, t); }   // the array, remote_session_id
    if (r.ctrl) rd_uint(d, 4, t);                        // msg_pkt_id
    const uint32_t hdr = 1 + 8 + r.hmac_len + 4 + (net_time ? 4 : 0) + 1 + 4 * nid + (nid ? 8 : 0) + (r.ctrl ? 4 : 0);
    if (have_data) {
        if (hdr >= (uint32_t)len) return r;
        const long dl = (long)((uint32_t)len - hdr) & 0xffff;   // data_len is a uint16_t
        if (clen(d) < dl) return r;
        r.data = cmk(d.d, d.d + dl);
        cskip(d, dl);
    }
    r.valid = type != 3;
    return r;
}

struct OvRes { bool present, hello; uint32_t nctrl, opcode, key, hmac_len; Ch ch; };
// openvpn_tcp::openvpn_tcp: the records, then the control records' data
// gathered into an 800-byte buffer (data_buffer<800>, a copy that does not
// fit nulls it) and parsed as a TLS record + handshake + ClientHello
DEV OvRes ovpn_process(Cur d, uint8_t *buf) {
    OvRes v; v.present = false; v.hello = false; v.nctrl = 0; v.opcode = 0; v.key = 0; v.hmac_len = 0;
    uint32_t nrec = 0, used = 0;
    bool buf_null = false;
    while (clen(d) > 0) {
        const OvRec r = ovpn_record(d);
        if (cnull(d) || !r.valid) return v;
        if (r.ctrl) {
            if (v.nctrl == 0) { v.opcode = r.opcode; v.key = r.key; v.hmac_len = r.hmac_len; }
            v.nctrl++;
            if (!cnull(r.data) && !buf_null) {
                const long dl = clen(r.data);
                if (used + (uint32_t)dl > 800) buf_null = true;
                else { for (long j = 0; j < dl; j++) buf[used + j] = (uint8_t)ld(r.data.d + j); used += (uint32_t)dl; }
            }
        }
        nrec++;
    }
    v.present = (uint8_t)nrec != 0;                      // is_not_empty: valid && num_records (uint8_t)
    if (!v.present || v.nctrl == 0 || buf_null || used == 0) return v;
    Cur p = cmk(buf, buf + used);
    Cur frag = tls_record_fragment(p);
    Hs hs = tls_hs_parse(frag);
    v.ch = tls_ch_parse(hs.body);
    v.hello = cnotempty(v.ch.compression);
    return v;
}

// openvpn_tcp::fingerprint + tls_client_hello::fingerprint (format 0)
template <class E>
DEV void ovpn_fp(E &b, const OvRes &v) {
    fp_type_prefix(b, 14);
    b.lit("(06)");
    b.putc('('); b.hex8(v.nctrl & 0xff); b.putc(')');
    b.putc('('); b.hex8(v.opcode); b.hex8(v.key ? 1u : 0u); b.putc(')');
    b.putc('('); b.hex8(v.hmac_len); b.putc(')');
    tls_ch_fp(b, v.ch, 0);
}

#ifndef MFP_QUIC_MINW
#define MFP_QUIC_MINW 1
#endif
__global__ __launch_bounds__(QT, MFP_QUIC_MINW) void k_quic(KParams P, uint8_t *scratch, uint32_t quic_format) {
    __shared__ uint32_t s_te[256];
    __shared__ uint64_t s_gh[32 * QT];
    __shared__ uint64_t out_line[QT][8];
    __shared__ uint32_t wave_tot[QT / 64];
    __shared__ unsigned long long tile_base;
    const int tid = threadIdx.x;
    for (int k = tid; k < 256; k += QT) s_te[k] = mfpq::kAes.te0[k];
    __syncthreads();
    uint8_t *pt = scratch + ((uint64_t)blockIdx.x * QT + tid) * Q_SLOT;
    uint8_t *cb = pt + Q_PT;
    const uint64_t count = (uint64_t)__hip_atomic_load(P.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    KPH_DECL
    for (uint64_t tile = blockIdx.x; tile * QT < count; tile += gridDim.x) {
        const uint64_t t = tile * QT + tid;
        const bool live = t < count;
        const uint64_t i = live ? (uint64_t)P.idx[t] : 0;
        mfp_pkt_desc dsc;
        if (live) dsc = P.desc[i];
        else { dsc.offset = 0; dsc.caplen = 0; dsc.linktype = 0xffff; dsc.flags = 0; }
        const uint8_t *data = P.arena + dsc.offset;

        // link / IP / UDP walk to the payload (identification only)
        Out o;
        {
            Em<false> e;
            TlsPlan plan;
            e.plan = &plan;
            Cfg c = P.cfg;
            c.classify = 1;
            packet_walk(e, c, o, data, dsc.caplen, dsc.linktype);
        }
        KPH(0);
        QRes q;
        q.flags = 0; q.hello = false; q.pre = false; q.ver = nullptr; q.more = 0; q.min_off = ~0u;
        const bool ovpn = live && o.msg == MFP_MSG_OPENVPN;
        OvRes v; v.present = false; v.hello = false;
        if (live && o.msg == MFP_MSG_QUIC)
            q = quic_process(cmk(data + o.pay_off, data + o.pay_off + o.pay_len), pt, cb, s_te, s_gh, (uint32_t)tid);
        // a reassembled Initial (include/mfp.h MFP_DESC_QUIC_CRYPTO): the
        // ClientHello is parsed again from the reassembled CRYPTO data the
        // host put behind the packet (reparse_crypto_buf quic.h:1593-1598);
        // the pre-decrypted path keeps its own hello (get_tls_client_hello
        // quic.h:1655-1660), the packet's header, plaintext and truncation stay
        if (live && o.msg == MFP_MSG_QUIC && (dsc.flags & MFP_DESC_QUIC_CRYPTO) && (q.flags & MFP_FLAG_EMIT) && !q.pre) {
            const uint8_t *rb = data + ((dsc.caplen + 7) & ~7u);
            const uint32_t rl = (uint32_t)ld(rb) | (uint32_t)ld(rb + 1) << 8 | (uint32_t)ld(rb + 2) << 16 | (uint32_t)ld(rb + 3) << 24;
            Cur d = cmk(rb + 8, rb + 8 + (rl > Q_CB ? Q_CB : rl));
            q.hs = d;
            const Hs hs = tls_hs_parse(d);
            q.ch = tls_ch_parse(hs.body);
            q.hello = cnotempty(q.ch.compression);
        }
        if (ovpn) {
            v = ovpn_process(cmk(data + o.pay_off, data + o.pay_off + o.pay_len), pt);
            q.flags = v.present ? MFP_FLAG_EMIT : 0;
        }
        KPH(1);
        const uint32_t fmt = q.pre ? 0u : quic_format;
        // the string's slot: QUIC, from an upper bound (every byte of the
        // handshake yields at most 2.5 characters: a 4-byte extension header
        // 10, a transport parameter's 1-byte id and length 4), so the string is
        // written in one pass and its length known after; OpenVPN, exact (a
        // counting pass)
        uint32_t len = 0, fp_type = 0, bound = 0;
        QMeta m; cset_null(m.sni); cset_null(m.ua); cset_null(m.alpn);
        if (q.hello) {
            const uint32_t hb = 5 * span_len(q.hs) / 2 + 64;
            bound = hb < FP_MAX ? hb : FP_MAX;
            fp_type = 12;
            m = quic_meta(q.ch.extensions);
        } else if (v.hello) {
            Em<false> e;
            TlsPlan plan;
            e.plan = &plan;
            ovpn_fp(e, v);
            if (e.valid()) { len = e.n; bound = len; fp_type = 14; }
        }
        // the sidecar (include/mfp.h MFP_FLAG_SIDECAR): an 8-byte header, the
        // classifier inputs, and on the write_json path the bytes the JSON
        // writer needs for the record's "tls" and "quic" objects (quic.h:1662-1690),
        // present also when there is no fingerprint
        const bool quic = live && o.msg == MFP_MSG_QUIC && (q.flags & MFP_FLAG_EMIT);
        // with reassembly inputs requested: the plaintext of an Initial whose
        // CRYPTO data may take part in reassembly (its frames are walked again
        // by the host's flow table, mfp_reassembly.cpp quic_initial)
        const bool reasm = quic && P.seg != nullptr && cnotempty(q.plain) && q.min_off != ~0u && (q.more || q.min_off);
        const bool json = quic && (P.cfg.mode == MFP_MODE_WRITE_JSON || reasm);
        const uint32_t pt_n = json ? span_len(q.plain) : 0u;
        const uint32_t hs_n = json && q.hello && P.cfg.mode == MFP_MODE_WRITE_JSON ? span_len(q.hs) : 0u;
        const uint32_t meta = bound && !ovpn ? span_len(m.sni) + span_len(m.ua) + span_len(m.alpn) : 0u;
        const uint32_t jlen = json ? 16 + pt_n + hs_n : 0u;
        const uint32_t side = (bound && !ovpn) || json ? 8 + meta + jlen : 0u;

        // tile reservation of 64-byte slots: string (its bound), hash, sidecar
        const int lane = tid & 63, wid = tid >> 6;
        const uint32_t slot = bound || side ? (((bound + 7) & ~7u) + 8 + side + 63) & ~63u : 0u;
        uint32_t incl = slot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) wave_tot[wid] = incl;
        __syncthreads();
        uint32_t wbase = 0, total = 0;
#pragma unroll
        for (int w = 0; w < QT / 64; w++) {
            const uint32_t tt = wave_tot[w];
            if (w < wid) wbase += tt;
            total += tt;
        }
        const uint32_t excl = wbase + incl - slot;
        if (tid == 0) {
            unsigned long long b = total ? atomicAdd(&P.fp_used[0], (unsigned long long)total) : 0ull;
            if (b + total > P.fp_cap) { atomicExch(&P.fp_used[1], 1ull); b = ~0ull; }
            tile_base = b;
        }
        __syncthreads();
        const unsigned long long base = tile_base;
        const bool fits = base != ~0ull;

        KPH(2);
        uint32_t sni_off = 0, sni_len = 0xffff, ua_off = 0, ua_len = 0xffff;
        uint8_t *out = P.fp_arena + (fits ? base + excl : 0);
        uint8_t *sc = out;
        if (bound && fits) {
            Em<true> e;
            e.begin(out, out_line[tid]);
            e.out_end = out + ((bound + 7) & ~7u) + 8;   // (a final 16-byte store may cover the hash's place)
            if (ovpn) ovpn_fp(e, v); else quic_fp(e, q, fmt);
            e.finish();
            if (e.valid() && e.n <= bound) {
                len = e.n;
                *(uint64_t *)(out + ((len + 7) & ~7u)) = e.hash();
            } else {
                fp_type = 0;                               // fingerprint::final drops truncated strings
            }
        }
        sc = out + ((len + 7) & ~7u) + 8;
        {   // bytes written (fp_used[2]): the exact lengths
            uint32_t lsum = fits ? len : 0u;
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) lsum += __shfl_xor(lsum, d, 64);
            if (lane == 0 && lsum) atomicAdd(&P.fp_used[2], (unsigned long long)lsum);
        }
        KPH(3);
        if (side && fits) {
            // header: {u16 alpn_off, u16 alpn_len, u16 side_len, u16 json_off}, then
            // the server name, user agent and ALPN list (classifier inputs)
            uint32_t at = 8;
            const Cur parts[3] = {m.sni, m.ua, m.alpn};
            uint32_t offs[3], lens[3];
            for (int k = 0; k < 3; k++) {
                offs[k] = at;
                lens[k] = len && !cnull(parts[k]) ? (uint32_t)clen(parts[k]) : 0xffffu;
                const uint32_t sl = len ? span_len(parts[k]) : 0u;
                copy_bytes(sc + at, parts[k].d, sl);
                at += sl;
            }
            if (len) { sni_off = offs[0]; sni_len = lens[0]; ua_off = offs[1]; ua_len = lens[1]; }
            const uint32_t json_off = json ? at : 0u;
            if (json) {
                // the JSON block: {u16 payload offset, u16 payload length, u16 plaintext
                // length, u16 handshake length, u16 cc frame offset in the plaintext (0xffff
                // none), u8 bit 0 pre-decrypted / bit 1 hello, u8 salt (0xff none), u32 0},
                // the plaintext, the handshake bytes
                uint8_t hdr[16];
                const uint32_t cco = q.cc && cnotempty(q.plain) ? (uint32_t)(q.cc - q.plain.d) : 0xffffu;
                const uint32_t hv[5] = {o.pay_off, o.pay_len, pt_n, hs_n, cco};
                for (int k = 0; k < 5; k++) { hdr[2 * k] = (uint8_t)hv[k]; hdr[2 * k + 1] = (uint8_t)(hv[k] >> 8); }
                hdr[10] = (uint8_t)((q.pre ? 1u : 0u) | (q.hello ? 2u : 0u) | (reasm ? 4u : 0u));
                hdr[11] = (uint8_t)q.salt;
                hdr[12] = hdr[13] = hdr[14] = hdr[15] = 0;
                for (int k = 0; k < 16; k++) sc[at + k] = hdr[k];
                at += 16;
                copy_bytes(sc + at, q.plain.d, pt_n);
                at += pt_n;
                copy_bytes(sc + at, q.hs.d, hs_n);
                at += hs_n;
            }
            const uint32_t hv2[4] = {offs[2], lens[2], side, json_off};
            for (int k = 0; k < 4; k++) { sc[2 * k] = (uint8_t)hv2[k]; sc[2 * k + 1] = (uint8_t)(hv2[k] >> 8); }
        }
        // OpenVPN: the TCP payload, which the JSON writer re-reads for the "openvpn" object
        if (ovpn) { sni_off = o.pay_off; sni_len = o.pay_len; }
        if (live) {
            mfp_record r;
            r.fp_offset = fits && slot ? base + excl : 0;
            r.fp_len = fits ? len : 0;
            r.fp_type = (uint8_t)(fits ? fp_type : 0);
            r.msg = (uint8_t)o.msg;
            r.flags = (uint8_t)(q.flags | (o.flags & MFP_FLAG_ENCAP) | (fits && len ? MFP_FLAG_HASHED : 0) |
                                (fits && side ? MFP_FLAG_SIDECAR : 0));
            r.xflags = 0;
            r.sni_off = (uint16_t)(sni_len == 0xffff ? 0 : sni_off);
            r.sni_len = (uint16_t)sni_len;
            r.ua_off = (uint16_t)(ua_len == 0xffff ? 0 : ua_off);
            r.ua_len = (uint16_t)ua_len;
            r.src_port = (uint16_t)o.src_port;
            r.dst_port = (uint16_t)o.dst_port;
            r.net = o.net;
            P.rec[i] = r;
            if (quic) { o.seg_kind |= MFP_SEG_QUIC; o.more = q.more; }
            write_seg(P, i, o);
        }
        __syncthreads();   // tile_base / wave_tot reuse
        KPH(4);
    }
    KPH_FLUSH();
}

}  // namespace mfp

#include "mfp_internal.h"

extern "C" int mfp_launch_quic(const void *kparams, uint8_t *scratch, uint32_t quic_format, uint32_t grid,
                               hipStream_t stream, mfp_prof *prof) {
    const mfp::KParams &P = *(const mfp::KParams *)kparams;
    if (prof) mfp_prof_begin(prof, "k_quic", stream);
    hipLaunchKernelGGL(mfp::k_quic, dim3(grid), dim3(mfp::QT), 0, stream, P, scratch, quic_format);
    if (prof) mfp_prof_end(prof, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

KPH_READER(quic)

extern "C" size_t mfp_quic_scratch_bytes(uint32_t grid) { return (size_t)grid * mfp::QT * mfp::Q_SLOT + 64; }
