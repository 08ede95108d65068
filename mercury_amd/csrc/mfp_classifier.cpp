// mfp_classifier.cpp -- host side of the --analysis process classifier:
// reads the reference's resource archive (.tgz: VERSION, fingerprint_db.json,
// fp_prevalence_tls.txt, pyasn.db; analysis.h:821-980) and turns it into the
// flat device tables the classifier kernel (mfp_analysis.hip) reads.
//
// Model restated from the reference (file:line relative to
// /root/reference/src/libmerc/):
//   * fingerprint_data / naive_bayes_tls_quic_http ctor  analysis.h:143-218,
//     naive_bayes.hpp:710-750: per fingerprint, P processes, a prior vector
//     (add_class naive_bayes.hpp:657-663) and six categorical features whose
//     updates are precomputed as (log(count/total) - log(0.1/total)) * weight
//     (feature::add_update naive_bayes.hpp:103-118; domain/sni updates of the
//     same process combine, update::combine naive_bayes.hpp:34-40);
//   * classifier::process_fp_db_line analysis.h:646-743 (validate_fp
//     analysis.h:598-640, MALWARE_DB, feature_weights, str_repr_array);
//   * attribute name indices (attribute_names result.h:133-172, reserved in
//     the order of pkt_proc.h:72 and analysis.h:830).
// The loader runs once per context; the per-packet work is on the device.
#include <hip/hip_runtime.h>
#include <zlib.h>
#include <openssl/evp.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mfp.h"
#include "mfp_analysis.h"
#include "mfp_common.hpp"
#include "mfp_internal.h"
#include "mfp_lctrie.hpp"

namespace {

// ---------------------------------------------------------------------------
// minimal JSON (one fingerprint_db.json line at a time; keeps member order)
// ---------------------------------------------------------------------------
struct JV {
    enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
    bool b = false;
    std::string s;                       // string value, or the number's text
    double num = 0;
    bool is_uint = false;
    uint64_t u = 0;
    std::vector<JV> a;
    std::vector<std::pair<std::string, JV>> o;
    const JV *get(const char *k) const {
        for (auto &kv : o) if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

struct JP {
    const char *p, *e;
    bool ok = true;
    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
    bool str(std::string &out) {
        if (p >= e || *p != '"') return ok = false;
        p++;
        while (p < e && *p != '"') {
            if (*p == '\\') {
                p++;
                if (p >= e) return ok = false;
                char c = *p++;
                switch (c) {
                case 'n': out += '\n'; break;
                case 't': out += '\t'; break;
                case 'r': out += '\r'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'u': {
                    if (e - p < 4) return ok = false;
                    unsigned v = (unsigned)strtoul(std::string(p, 4).c_str(), nullptr, 16);
                    p += 4;
                    if (v >= 0xd800 && v < 0xdc00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        unsigned lo = (unsigned)strtoul(std::string(p + 2, 4).c_str(), nullptr, 16);
                        p += 6;
                        v = 0x10000 + ((v - 0xd800) << 10) + (lo - 0xdc00);
                    }
                    if (v < 0x80) out += (char)v;
                    else if (v < 0x800) { out += (char)(0xc0 | v >> 6); out += (char)(0x80 | (v & 63)); }
                    else if (v < 0x10000) { out += (char)(0xe0 | v >> 12); out += (char)(0x80 | (v >> 6 & 63)); out += (char)(0x80 | (v & 63)); }
                    else { out += (char)(0xf0 | v >> 18); out += (char)(0x80 | (v >> 12 & 63)); out += (char)(0x80 | (v >> 6 & 63)); out += (char)(0x80 | (v & 63)); }
                    break;
                }
                default: out += c;
                }
            } else {
                out += *p++;
            }
        }
        if (p >= e) return ok = false;
        p++;
        return true;
    }
    bool val(JV &v, int depth = 0) {
        if (depth > 64) return ok = false;
        ws();
        if (p >= e) return ok = false;
        char c = *p;
        if (c == '{') {
            v.t = JV::OBJ; p++; ws();
            if (p < e && *p == '}') { p++; return true; }
            while (true) {
                ws();
                std::string k;
                if (!str(k)) return false;
                ws();
                if (p >= e || *p != ':') return ok = false;
                p++;
                v.o.emplace_back(std::move(k), JV());
                if (!val(v.o.back().second, depth + 1)) return false;
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == '}') { p++; return true; }
                return ok = false;
            }
        }
        if (c == '[') {
            v.t = JV::ARR; p++; ws();
            if (p < e && *p == ']') { p++; return true; }
            while (true) {
                v.a.emplace_back();
                if (!val(v.a.back(), depth + 1)) return false;
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == ']') { p++; return true; }
                return ok = false;
            }
        }
        if (c == '"') { v.t = JV::STR; return str(v.s); }
        if (e - p >= 4 && !strncmp(p, "true", 4)) { v.t = JV::BOOL; v.b = true; p += 4; return true; }
        if (e - p >= 5 && !strncmp(p, "false", 5)) { v.t = JV::BOOL; v.b = false; p += 5; return true; }
        if (e - p >= 4 && !strncmp(p, "null", 4)) { v.t = JV::NUL; p += 4; return true; }
        const char *s = p;
        while (p < e && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E')) p++;
        if (p == s) return ok = false;
        v.t = JV::NUM;
        v.s.assign(s, p);
        v.num = strtod(v.s.c_str(), nullptr);
        bool integral = v.s.find_first_of(".eE-") == std::string::npos;
        if (integral) { v.is_uint = true; v.u = strtoull(v.s.c_str(), nullptr, 10); }
        return true;
    }
};

bool parse_json(const std::string &line, JV &out) {
    JP jp{line.data(), line.data() + line.size()};
    return jp.val(out) && jp.ok;
}

// ---------------------------------------------------------------------------
// .tgz reader (gzip via zlib, ustar headers): calls f(name, contents)
// ---------------------------------------------------------------------------
// encrypted_file (enc_file_reader.h:86-231): AES-128-CBC under the 16-byte
// key with a zero IV; the file's first block is the real IV, so the first
// plaintext block is discarded; PKCS#7 padding checked by the final block
bool decrypt_archive(const char *path, const uint8_t *key, std::string &out) {
    FILE *fp = fopen(path, "rb");
    if (!fp) return false;
    std::string ct;
    char buf[1 << 16];
    size_t r;
    while ((r = fread(buf, 1, sizeof buf, fp)) > 0) ct.append(buf, r);
    fclose(fp);
    EVP_CIPHER_CTX *ctx = EVP_CIPHER_CTX_new();
    if (!ctx) return false;
    const uint8_t iv[16] = {0};
    out.resize(ct.size() + 32);
    int n1 = 0, n2 = 0;
    bool ok = EVP_DecryptInit_ex(ctx, EVP_aes_128_cbc(), nullptr, key, iv) == 1 &&
              EVP_DecryptUpdate(ctx, (unsigned char *)&out[0], &n1, (const unsigned char *)ct.data(), (int)ct.size()) == 1 &&
              EVP_DecryptFinal_ex(ctx, (unsigned char *)&out[0] + n1, &n2) == 1;
    EVP_CIPHER_CTX_free(ctx);
    if (!ok || n1 + n2 < 16) return false;
    out.resize((size_t)(n1 + n2));
    out.erase(0, 16);
    return true;
}

// gzip stream in memory -> bytes
bool gunzip(const std::string &in, std::string &out) {
    z_stream z{};
    if (inflateInit2(&z, 16 + MAX_WBITS) != Z_OK) return false;
    z.next_in = (Bytef *)in.data();
    z.avail_in = (uInt)in.size();
    char buf[1 << 16];
    int r;
    do {
        z.next_out = (Bytef *)buf;
        z.avail_out = sizeof buf;
        r = inflate(&z, Z_NO_FLUSH);
        if (r != Z_OK && r != Z_STREAM_END) { inflateEnd(&z); return false; }
        out.append(buf, sizeof buf - z.avail_out);
    } while (r != Z_STREAM_END && (z.avail_in > 0 || z.avail_out == 0));
    inflateEnd(&z);
    return r == Z_STREAM_END;
}

template <class F>
bool read_tgz(const char *path, F f, const uint8_t *key = nullptr) {
    std::string all;
    bool keyed = false;
    if (key) for (int k = 0; k < 16; k++) keyed |= key[k] != 0;   // cryptovar::is_null: plain file
    if (keyed) {
        std::string gz;
        if (!decrypt_archive(path, key, gz) || !gunzip(gz, all)) return false;
    } else {
        gzFile gz = gzopen(path, "rb");
        if (!gz) return false;
        char buf[1 << 16];
        int r;
        while ((r = gzread(gz, buf, sizeof buf)) > 0) all.append(buf, r);
        gzclose(gz);
        if (r < 0) return false;
    }
    size_t off = 0;
    std::string longname;
    while (off + 512 <= all.size()) {
        const char *h = all.data() + off;
        if (h[0] == 0) break;
        std::string name(h, strnlen(h, 100));
        std::string prefix(h + 345, strnlen(h + 345, 155));
        if (!prefix.empty() && !memcmp(h + 257, "ustar", 5)) name = prefix + "/" + name;
        uint64_t size = strtoull(std::string(h + 124, 12).c_str(), nullptr, 8);
        char type = h[156];
        off += 512;
        if (off + size > all.size()) return false;
        if (type == 'L') {
            longname.assign(all.data() + off, strnlen(all.data() + off, size));
        } else {
            if (!longname.empty()) { name = longname; longname.clear(); }
            if (type == '0' || type == 0) {
                size_t sl = name.rfind('/');
                f(sl == std::string::npos ? name : name.substr(sl + 1), std::string(all.data() + off, size));
            }
        }
        off += (size + 511) / 512 * 512;
    }
    return true;
}

// the lines of an archive member as the reference's loader sees them:
// `while (archive.getline(line))` (analysis.h:859-930) strips the newline and
// stops at the first empty line (getline returns the length, archive.h:247-270)
template <class F>
void for_lines(const std::string &s, F f) {
    size_t a = 0;
    while (a < s.size()) {
        size_t b = s.find('\n', a);
        if (b == std::string::npos) b = s.size();
        if (b == a) break;
        std::string line = s.substr(a, b - a);
        f(line);
        a = b + 1;
    }
}

// ---------------------------------------------------------------------------
// host model
// ---------------------------------------------------------------------------
struct Upd { uint32_t idx; double val; };
struct FeatMap {
    std::map<std::string, std::vector<Upd>> by_str;     // ua, domain, sni
    std::map<uint64_t, std::vector<Upd>> by_int;        // asn, port, ipv4
    std::map<std::string, std::vector<Upd>> by_v6;      // 16-byte keys
};
struct Entry {
    std::vector<std::string> proc_name;
    std::vector<uint8_t> malware;
    std::vector<uint32_t> attr;
    std::vector<double> prior;
    std::vector<std::vector<std::pair<std::string, uint64_t>>> os;   // per process: os_info (archive order)
    bool malware_db = false;
    FeatMap f[7];
};

typedef unsigned __int128 u128;

// one domain-mappings.db prefix (subnet_data::domains_prefix, addr.cc:256-309)
struct DomPrefix {
    u128 addr;                  // host order, unmasked until process_domain_mappings_final
    int len;
    uint32_t type;              // MFP_DOM_MAPPING / MFP_DOM_EXCEPTION
    std::vector<uint8_t> idx;   // mapped domain indices, uint8_t as the reference stores them
};

struct Weights { double as, domain, port, ip, sni, ua; double sum() const { return as + domain + port + ip + sni + ua; } };
const Weights kDefaultWeights{0.13924, 0.15590, 0.00528, 0.56735, 0.96941, 1.0};   // naive_bayes.hpp:697-704

const char *kReservedAttrs[] = {   // pkt_proc.h:72 then analysis.h:830
    "residential_proxy", "exposed_credentials_plaintext", "exposed_credentials_token",
    "exposed_credentials_derived", "cnsa_2_0_non_conformant", "nist_sp_800_52_2_non_conformant",
    "encrypted_dns", "encrypted_channel", "domain_faking", "faketls",
};

}  // namespace

struct mfp_classifier_s {
    // host model
    std::vector<std::string> attr_names;
    bool accept_attr = true;
    std::vector<std::unique_ptr<Entry>> entries;
    std::unordered_map<std::string, uint32_t> fpdb;           // fingerprint string -> entry
    std::vector<std::string> fp_order;                         // strings in insertion order
    std::unordered_set<std::string> known_prevalence;
    std::vector<uint32_t> fp_types;
    std::map<std::string, std::pair<uint32_t, size_t>> fp_count_and_format;
    std::string version;
    bool malware_db = false;
    bool disabled = false;
    std::vector<std::pair<uint64_t, uint32_t>> asn4;           // (prefix<<8 | len, asn)
    std::vector<std::pair<std::string, uint32_t>> asn6;        // (16 bytes + len byte, asn)
    std::vector<std::string> proc_names;                       // global process-name table
    std::unordered_map<std::string, uint32_t> proc_name_id;
    // encrypted_dns: doh-watchlist.txt (watchlist::process_line watchlist.hpp:624-652)
    bool doh_enabled = false;
    std::unordered_set<std::string> doh_names;
    std::vector<uint32_t> doh_v4;
    std::vector<std::pair<uint64_t, uint64_t>> doh_v6;
    // domain_faking: domain-mappings.db (analysis.h:765-819, addr.cc:256-458)
    bool faking_enabled = false;
    std::unordered_map<std::string, uint32_t> dom_idx;         // subnet_data::domains_watchlist
    std::vector<std::pair<std::string, std::string>> dom_lines4, dom_lines6;   // (subnet, tag) per family
    std::vector<DomPrefix> dom4, dom6;
    // os_info per process slot (flattened like the device's prior array)
    std::vector<std::pair<uint32_t, uint32_t>> os_span;         // (first, count) into os_flat
    std::vector<std::pair<std::string, uint64_t>> os_flat;
    mfp_classifier_dev dev;                                    // device tables (mfp_analysis.h)
    uint64_t device_bytes = 0;                                 // their size in HBM
    int device = -1;
};

namespace {

int attr_index(mfp_classifier_s &c, const std::string &name) {   // attribute_names::get_index
    if (c.accept_attr) {
        c.attr_names.push_back(name);
        if (c.attr_names.size() > 16) throw std::runtime_error("too many attributes in attribute_names");
        return (int)c.attr_names.size() - 1;
    }
    for (size_t i = 0; i < c.attr_names.size(); i++) if (c.attr_names[i] == name) return (int)i;
    return -1;
}

std::string normalized_sni(const std::string &s) {
    char out[400];
    int n = mfpc::normalize_server_name((const uint8_t *)s.data(), (int)s.size(), out);
    return std::string(out, n);
}

bool ipv4_key(const std::string &s, uint32_t &key) {   // lookahead<ipv4_address_string> + normalize
    int pos = 0;
    uint32_t v;
    if (!mfpc::parse_ipv4((const uint8_t *)s.data(), (int)s.size(), pos, v)) return false;
    key = mfpc::normalize_ipv4(v);
    return true;
}

bool ipv6_key(const std::string &s, std::string &key) {
    int pos = 0;
    uint8_t a[16];
    if (!mfpc::parse_ipv6((const uint8_t *)s.data(), (int)s.size(), pos, a)) return false;
    mfpc::normalize_ipv6(a);
    key.assign((const char *)a, 16);
    return true;
}

uint64_t stoul_like(const std::string &s, uint64_t max) {   // feature<T>::convert
    char *end = nullptr;
    errno = 0;
    unsigned long long v = strtoull(s.c_str(), &end, 10);
    if (end == s.c_str()) return 0;
    if (v > max) return 0;
    return v;
}

void add_update(std::vector<Upd> &lst, uint32_t idx, uint64_t count, uint64_t total, double w) {
    double base_prior = log(0.1 / (double)total);
    lst.push_back(Upd{idx, (log((double)count / (double)total) - base_prior) * w});
}

// domain_name_model::add_domain_update / add_sni_update (naive_bayes.hpp:422-490)
void add_combining_update(std::vector<Upd> &lst, uint32_t idx, uint64_t count, uint64_t total, double w) {
    double base_prior = log(0.1 / (double)total);
    for (auto it = lst.rbegin(); it != lst.rend(); ++it) {
        if (it->idx == idx) {   // update::combine naive_bayes.hpp:34-40
            long double old_count = expl((long double)(it->val / w + base_prior)) * (long double)total;
            size_t old_int = (size_t)roundl(old_count);
            it->val = (log((double)(count + old_int) / (double)total) - base_prior) * w;
            return;
        }
    }
    lst.push_back(Upd{idx, (log((double)count / (double)total) - base_prior) * w});
}

uint32_t fp_type_code(const std::string &s) {   // classifier::get_fingerprint_type analysis.h:448
    if (s == "tls") return 1;
    if (s == "http") return 3;
    if (s == "quic") return 12;
    if (s == "stun") return 16;
    if (s == "tofsee") return 15;
    if (s == "ssh") return 5;
    return 0;
}

// get_fingerprint_type_and_version analysis.h:501-541
std::pair<uint32_t, size_t> type_and_version(const std::string &s) {
    size_t idx = s.find('/');
    if (idx == std::string::npos) return {0, 0};
    uint32_t t = fp_type_code(s.substr(0, idx));
    if (!t) return {0, 0};
    std::string tail = s.substr(idx + 1);
    if (tail.empty()) return {0, 0};
    if (tail[0] == '(' || tail.compare(0, 10, "randomized") == 0) return {t, 0};
    char *end = nullptr;
    long v = strtol(tail.c_str(), &end, 10);
    if (end == tail.c_str()) return {0, 0};
    return {t, (size_t)v};
}

bool validate_fp(mfp_classifier_s &c, std::string &fp, uint32_t code, const std::string &type_str) {
    if (fp.empty() || fp.size() >= 8192) return false;
    if (code == 1 && (fp[0] == '(' || fp == "randomized")) fp = "tls/" + fp;
    auto tv = type_and_version(fp);
    if (tv.first != code) return false;
    auto it = c.fp_count_and_format.find(type_str);
    if (it != c.fp_count_and_format.end()) {
        if (it->second.first == 1) it->second.second = tv.second;
        else if (tv.second != it->second.second) return false;
    }
    return true;
}

void process_fp_db_line(mfp_classifier_s &c, const std::string &line) {
    JV fp;
    if (!parse_json(line, fp) || fp.t != JV::OBJ) return;
    uint32_t code = 1;
    std::string type_str;
    if (const JV *t = fp.get("fp_type"); t && t->t == JV::STR) {
        type_str = t->s;
        code = fp_type_code(type_str);
        auto &cf = c.fp_count_and_format[type_str];
        cf.first++;
        if (cf.first == 1) cf.second = 0;
    }
    if (code && std::find(c.fp_types.begin(), c.fp_types.end(), code) == c.fp_types.end()) c.fp_types.push_back(code);
    uint64_t total = 0;
    if (const JV *t = fp.get("total_count"); t && t->t == JV::NUM && t->is_uint) total = t->u;
    Weights w = kDefaultWeights;
    if (const JV *fw = fp.get("feature_weights"); fw && fw->t == JV::OBJ) {
        for (auto &kv : fw->o) {
            double v = (double)(float)kv.second.num;   // rapidjson GetFloat()
            if (kv.first == "as") w.as = v;
            else if (kv.first == "domain") w.domain = v;
            else if (kv.first == "port") w.port = v;
            else if (kv.first == "ip") w.ip = v;
            else if (kv.first == "sni") w.sni = v;
            else if (kv.first == "ua") w.ua = v;
        }
    }
    const JV *pi = fp.get("process_info");
    if (!pi || pi->t != JV::ARR) return;
    if (!pi->a.empty()) {
        if (pi->a[0].get("malware")) c.malware_db = true;
    }
    if (total == 0) throw std::runtime_error("total_count==0 in naive_bayes");
    auto e = std::make_unique<Entry>();
    e->malware_db = c.malware_db;
    uint32_t idx = 0;
    for (auto &x : pi->a) {
        if (const JV *p = x.get("process"); p && p->t == JV::STR) e->proc_name.push_back(p->s);
        if (const JV *m = x.get("malware"); m && m->t == JV::BOOL) e->malware.push_back(m->b);
        uint32_t bits = 0;
        if (const JV *a = x.get("attributes"); a && a->t == JV::OBJ) {
            for (auto &kv : a->o) {
                int ai = attr_index(c, kv.first);
                if (ai < 0) throw std::runtime_error("unknown attribute " + kv.first);
                if (kv.second.t == JV::BOOL && kv.second.b) bits |= 1u << ai;
            }
            c.accept_attr = false;
        }
        e->attr.push_back(bits);
        // os_info (analysis.h:195-205; loaded whatever report_os says, reported only when it is on)
        e->os.emplace_back();
        if (const JV *oi = x.get("os_info"); oi && oi->t == JV::OBJ)
            for (auto &kv : oi->o)
                if (!kv.first.empty()) e->os.back().push_back({kv.first, kv.second.is_uint ? kv.second.u : 0});
        if (x.t == JV::OBJ) {
            // domain_name_model: sni (normalized keys) then domains
            const JV *sni = x.get("classes_hostname_sni");
            const JV *dom = x.get("classes_hostname_domains");
            const JV *port = x.get("classes_port_port");
            const JV *as = x.get("classes_ip_as");
            const JV *ua = x.get("classes_user_agent");
            const JV *ip = x.get("classes_ip_ip");
            if (!sni || !dom || !port || !as || !ip) throw std::runtime_error("missing feature in process_info");
            if (sni->t == JV::OBJ)
                for (auto &kv : sni->o)
                    if (kv.second.is_uint)
                        add_combining_update(e->f[mfpc::F_SNI].by_str[normalized_sni(kv.first)], idx, kv.second.u, total, w.sni);
            if (dom->t == JV::OBJ)
                for (auto &kv : dom->o)
                    if (kv.second.is_uint)
                        add_combining_update(e->f[mfpc::F_DOMAIN].by_str[kv.first], idx, kv.second.u, total, w.domain);
            if (port->t != JV::OBJ || as->t != JV::OBJ || ip->t != JV::OBJ) throw std::runtime_error("feature not an object");
            for (auto &kv : port->o) {
                if (!kv.second.is_uint) throw std::runtime_error("expected uint64");
                add_update(e->f[mfpc::F_PORT].by_int[stoul_like(kv.first, 65535)], idx, kv.second.u, total, w.port);
            }
            for (auto &kv : as->o) {
                if (!kv.second.is_uint) throw std::runtime_error("expected uint64");
                uint64_t k = kv.first == "unknown" ? 0 : stoul_like(kv.first, 0xffffffffULL);
                add_update(e->f[mfpc::F_ASN].by_int[k], idx, kv.second.u, total, w.as);
            }
            if (ua && ua->t == JV::OBJ) {
                for (auto &kv : ua->o) {
                    if (!kv.second.is_uint) throw std::runtime_error("expected uint64");
                    add_update(e->f[mfpc::F_UA].by_str[kv.first == "None" ? std::string() : kv.first], idx, kv.second.u,
                               total, w.ua);
                }
            }
            for (auto &kv : ip->o) {
                if (!kv.second.is_uint) throw std::runtime_error("expected uint64");
                uint32_t k4;
                std::string k6;
                if (ipv4_key(kv.first, k4)) add_update(e->f[mfpc::F_IPV4].by_int[k4], idx, kv.second.u, total, w.ip);
                else if (ipv6_key(kv.first, k6)) add_update(e->f[mfpc::F_IPV6].by_v6[k6], idx, kv.second.u, total, w.ip);
            }
        }
        // naive_bayes::add_class_from_count naive_bayes.hpp:665-680
        const JV *cnt = x.get("count");
        if (!cnt || !cnt->is_uint || cnt->u == 0) throw std::runtime_error("bad process count");
        double base_prior = log(0.1 / (double)total);
        double score = log((double)cnt->u / (double)total);
        e->prior.push_back(fmax(score, log(.1)) + base_prior * w.sum());
        idx++;
    }
    if (e->proc_name.size() != idx || e->malware.size() != idx) {
        // the reference asserts these; a DB without "malware" members gives
        // malware = false for every process in non-malware databases
        if (e->malware.size() != idx) e->malware.assign(idx, 0);
        if (e->proc_name.size() != idx) return;
    }
    uint32_t eid = (uint32_t)c.entries.size();
    bool used = false;
    if (const JV *s = fp.get("str_repr"); s && s->t == JV::STR) {
        std::string fs = s->s;
        if (!validate_fp(c, fs, code, type_str)) return;
        if (c.fpdb.count(fs)) return;
        c.fpdb[fs] = eid; c.fp_order.push_back(fs); used = true;
    }
    if (const JV *arr = fp.get("str_repr_array"); arr && arr->t == JV::ARR) {
        for (auto &x : arr->a) {
            if (x.t != JV::STR) continue;
            std::string fs = x.s;
            if (!validate_fp(c, fs, code, type_str)) { if (used) break; return; }
            if (c.fpdb.count(fs)) continue;
            c.fpdb[fs] = eid; c.fp_order.push_back(fs); used = true;
        }
    }
    if (used) c.entries.push_back(std::move(e));
}

// pyasn.db line: a '.' makes it IPv4 (analysis.h:896-905); parsed as
// lct_subnet_set_from_string does (lctrie_bgp.hpp:23-98): sscanf with "%hhu"
// octets (taken modulo 256) or an IPv6 text of at most 45 characters, a
// length in 1..32 / 1..128 and an ASN -- anything else is skipped
void process_asn_line(mfp_classifier_s &c, const std::string &line) {
    uint8_t len = 0;
    unsigned asn = 0;
    if (line.find('.') != std::string::npos) {
        uint32_t addr = 0;
        unsigned char *dq = (unsigned char *)&addr;   // host order, as the reference fills it
        if (sscanf(line.c_str(), "%hhu.%hhu.%hhu.%hhu/%hhu\t%u", dq + 3, dq + 2, dq + 1, dq, &len, &asn) != 6) return;
        if (len == 0 || len > 32) return;
        c.asn4.push_back({(uint64_t)addr << 8 | (uint64_t)len, (uint32_t)asn});
    } else {
        char a[46];
        if (sscanf(line.c_str(), "%45[^/]/%hhu\t%u", a, &len, &asn) != 3) return;
        if (len == 0 || len > 128) return;
        int pos = 0;
        uint8_t b[16];
        const int al = (int)strlen(a);
        if (!mfpc::parse_ipv6((const uint8_t *)a, al, pos, b) || pos != al) return;
        std::string k((const char *)b, 16);   // masked when the trie is built (subnet_mask_v6)
        k.push_back((char)len);
        c.asn6.push_back({k, (uint32_t)asn});
    }
}

// dns_string (watchlist.hpp:54-83): the host name at the start of s (labels
// of [A-Za-z0-9_-] separated by dots, an optional leading "*.", the last
// label holding a letter); trailing bytes are left unparsed
bool dns_prefix(const std::string &s, std::string &out) {
    size_t p = 0;
    const size_t n = s.size();
    if (p < n && s[p] == '*') {
        p++;
        if (p < n && s[p] == '.') p++;
        else return false;
    }
    long ls = -1, le = -1;
    while (p < n) {
        const size_t a = p;
        while (p < n && mfpc::is_label_char((uint8_t)s[p])) p++;
        if (p == a) break;
        ls = (long)a; le = (long)p;
        if (p < n && s[p] == '.') p++;
        else break;
    }
    bool alpha = false;
    for (long k = ls; k >= 0 && k < le; k++) alpha |= mfpc::is_alpha((uint8_t)s[k]);
    if (!alpha) return false;
    out = s.substr(0, (size_t)le);
    return true;
}

// watchlist::process_line (watchlist.hpp:624-652): an IPv4 address, else a
// DNS name, else an IPv6 address; '#' comments and empty lines are skipped,
// anything else is ignored (the loader drops process_line's false)
void process_doh_line(mfp_classifier_s &c, const std::string &line) {
    if (line.empty() || line[0] == '#') return;
    const uint8_t *s = (const uint8_t *)line.data();
    int pos = 0;
    uint32_t v4;
    if (mfpc::parse_ipv4(s, (int)line.size(), pos, v4)) { c.doh_v4.push_back(v4); return; }
    std::string name;
    if (dns_prefix(line, name)) { c.doh_names.insert(name); return; }
    pos = 0;
    uint8_t a[16];
    if (mfpc::parse_ipv6(s, (int)line.size(), pos, a)) {
        uint64_t hi = 0, lo = 0;
        for (int k = 0; k < 8; k++) { hi = hi << 8 | a[k]; lo = lo << 8 | a[8 + k]; }
        c.doh_v6.push_back({hi, lo});
    }
}

// classifier::process_domain_mapping_line (analysis.h:765-819): the subnet
// and its tag ("proxy"/"sinkhole" entries carry their type as the tag); a
// '.' in the subnet makes it IPv4
void process_domain_line(mfp_classifier_s &c, const std::string &line) {
    JV o;
    if (!parse_json(line, o) || o.t != JV::OBJ) return;
    const JV *sub = o.get("subnet"), *type = o.get("type"), *tag = o.get("tag");
    if (!sub || sub->t != JV::STR || !type || type->t != JV::STR || !tag || tag->t != JV::STR) return;
    std::string t;
    if (type->s == "domain_mapping") t = tag->s;
    else if (type->s == "proxy" || type->s == "sinkhole") t = type->s;
    else return;
    (sub->s.find('.') != std::string::npos ? c.dom_lines4 : c.dom_lines6).push_back({sub->s, t});
}

// subnet_data::lct_add_domain_mapping / lct_add_domain_exception (addr.cc:256-309,
// 350-403): a mapping whose exact (address, length) was seen before gains the
// domain index (its length differing: dropped); an exception is always a new
// prefix; indices are stored as uint8_t
template <class Map>
void add_domain_prefix(mfp_classifier_s &c, std::vector<DomPrefix> &v, Map &seen, u128 addr, int len,
                       const std::string &tag) {
    if (tag == "proxy" || tag == "sinkhole") {
        v.push_back(DomPrefix{addr, len, MFP_DOM_EXCEPTION, {}});
        return;
    }
    uint32_t idx;
    auto it = c.dom_idx.find(tag);
    if (it == c.dom_idx.end()) { idx = (uint32_t)c.dom_idx.size(); c.dom_idx[tag] = idx; }
    else idx = it->second;
    auto s = seen.find(addr);
    if (s != seen.end()) {
        DomPrefix &p = v[s->second];
        if (p.type == MFP_DOM_MAPPING && p.addr == addr && p.len == len) p.idx.push_back((uint8_t)idx);
        return;
    }
    seen[addr] = v.size();
    v.push_back(DomPrefix{addr, len, MFP_DOM_MAPPING, {(uint8_t)idx}});
}

struct U128Hash { size_t operator()(u128 x) const { return std::hash<uint64_t>()((uint64_t)x ^ (uint64_t)(x >> 64) * 31); } };

// process_domain_mapping_subnets[_v6] (addr.cc:311-348, 405-458): IPv4 lines
// first (their domains get the first indices), then IPv6
void build_domain_prefixes(mfp_classifier_s &c) {
    std::unordered_map<u128, size_t, U128Hash> seen4, seen6;
    for (auto &e : c.dom_lines4) {
        uint32_t addr = 0;
        unsigned char *dq = (unsigned char *)&addr;   // host order, as the reference fills it
        uint8_t len = 0;
        if (sscanf(e.first.c_str(), "%hhu.%hhu.%hhu.%hhu/%hhu", dq + 3, dq + 2, dq + 1, dq, &len) != 5) continue;
        if (len == 0 || len > 32) continue;
        add_domain_prefix(c, c.dom4, seen4, (u128)addr, len, e.second);
    }
    for (auto &e : c.dom_lines6) {
        char a[46];
        uint8_t len = 0;
        if (sscanf(e.first.c_str(), "%45[^/]/%hhu", a, &len) != 2) continue;
        if (len == 0 || len > 128) break;   // the reference abandons the rest of the IPv6 list
        int pos = 0;
        uint8_t b[16];
        if (!mfpc::parse_ipv6((const uint8_t *)a, (int)strlen(a), pos, b)) continue;
        u128 v = 0;
        for (int k = 0; k < 16; k++) v = v << 8 | b[k];
        add_domain_prefix(c, c.dom6, seen6, v, len, e.second);
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// C++ API used by mfp_host.cpp
// ---------------------------------------------------------------------------
mfp_classifier *mfp_classifier_load(const char *path, const uint8_t *enc_key) {
    auto c = std::make_unique<mfp_classifier_s>();
    for (const char *a : kReservedAttrs) attr_index(*c, a);
    bool got_db = false, got_prev = false, got_ver = false, got_asn = false;
    std::string db_text;
    try {
        bool ok = read_tgz(path, [&](const std::string &name, const std::string &data) {
            if (name == "fp_prevalence_tls.txt") {
                for_lines(data, [&](std::string l) {
                    if (!l.empty() && l.back() == '\n') l.pop_back();
                    if (l.empty()) return;
                    if (l[0] == '(') l = "tls/" + l;
                    c->known_prevalence.insert(l);
                });
                got_prev = true;
            } else if (name == "fingerprint_db.json") {
                db_text = data;
                got_db = true;
            } else if (name == "VERSION") {
                for_lines(data, [&](const std::string &l) { c->version += l; });
                got_ver = true;
            } else if (name == "pyasn.db") {
                for_lines(data, [&](const std::string &l) { process_asn_line(*c, l); });
                got_asn = true;
            } else if (name == "doh-watchlist.txt") {
                for_lines(data, [&](const std::string &l) { process_doh_line(*c, l); });
                c->doh_enabled = true;
            } else if (name == "domain-mappings.db") {
                for_lines(data, [&](const std::string &l) { process_domain_line(*c, l); });
                c->faking_enabled = true;
            }
        }, enc_key);
        if (!ok) { mfp_set_error("cannot read resource archive %s", path); return nullptr; }
        c->fp_types.push_back(1);   // tls is always expected (analysis.h:833)
        bool dual = c->version.find("dual") != std::string::npos, lite = c->version.find("lite") != std::string::npos,
             full = c->version.find("full") != std::string::npos;
        if (!dual && !lite && !full) c->disabled = true;   // legacy archive
        if (!c->disabled) for_lines(db_text, [&](const std::string &l) { if (!l.empty()) process_fp_db_line(*c, l); });
    } catch (const std::exception &ex) {
        mfp_set_error("resource archive %s: %s", path, ex.what());
        return nullptr;
    }
    if (std::count(c->version.begin(), c->version.end(), ';') != 1) c->disabled = true;
    if (!got_db || !got_prev || !got_ver || !got_asn) c->disabled = true;
    c->accept_attr = false;
    build_domain_prefixes(*c);
    // global process-name table; os_info per process slot
    for (auto &e : c->entries) {
        for (auto &n : e->proc_name)
            if (!c->proc_name_id.count(n)) {
                c->proc_name_id[n] = (uint32_t)c->proc_names.size();
                c->proc_names.push_back(n);
            }
        for (size_t i = 0; i < e->prior.size(); i++) {
            const auto &os = i < e->os.size() ? e->os[i] : std::vector<std::pair<std::string, uint64_t>>{};
            c->os_span.push_back({(uint32_t)c->os_flat.size(), (uint32_t)os.size()});
            c->os_flat.insert(c->os_flat.end(), os.begin(), os.end());
        }
    }
    return c.release();
}

int mfp_classifier_attr_count(const mfp_classifier *c) { return (int)c->attr_names.size(); }
const char *mfp_classifier_version(const mfp_classifier *c) { return c->version.c_str(); }
uint64_t mfp_classifier_device_bytes(const mfp_classifier *c) { return c->device_bytes; }

int mfp_classifier_os_info(const mfp_classifier *c, uint32_t slot, uint32_t k, const char **name, uint64_t *prev) {
    if (slot >= c->os_span.size()) return -1;
    const auto &sp = c->os_span[slot];
    if (k < sp.second) {
        if (name) *name = c->os_flat[sp.first + k].first.c_str();
        if (prev) *prev = c->os_flat[sp.first + k].second;
    }
    return (int)sp.second;
}

void mfp_classifier_free(mfp_classifier *c) {
    if (!c) return;
    mfp_classifier_free_device(c->dev);
    delete c;
}

int mfp_classifier_tls_format(const mfp_classifier *c) {
    auto it = c->fp_count_and_format.find("tls");
    return it == c->fp_count_and_format.end() ? 0 : (int)it->second.second;
}
// classifier::get_quic_fingerprint_format (analysis.h:488)
int mfp_classifier_quic_format(const mfp_classifier *c) {
    auto it = c->fp_count_and_format.find("quic");
    return it == c->fp_count_and_format.end() ? 0 : (int)it->second.second;
}
bool mfp_classifier_disabled(const mfp_classifier *c) { return c->disabled; }
const char *mfp_classifier_process_name(const mfp_classifier *c, uint32_t id) {
    return id < c->proc_names.size() ? c->proc_names[id].c_str() : nullptr;
}
const char *mfp_classifier_attr_name(const mfp_classifier *c, uint32_t i) {
    return i < c->attr_names.size() ? c->attr_names[i].c_str() : nullptr;
}
void mfp_classifier_stats(const mfp_classifier *c, uint64_t out[8]) {
    uint64_t procs = 0, upd = 0;
    for (auto &e : c->entries) {
        procs += e->prior.size();
        for (auto &f : e->f) {
            for (auto &kv : f.by_str) upd += kv.second.size();
            for (auto &kv : f.by_int) upd += kv.second.size();
            for (auto &kv : f.by_v6) upd += kv.second.size();
        }
    }
    out[0] = c->fpdb.size(); out[1] = c->entries.size(); out[2] = procs; out[3] = upd;
    out[4] = c->known_prevalence.size(); out[5] = c->asn4.size() + c->asn6.size();
    out[6] = c->disabled; out[7] = c->proc_names.size();
}

// ---------------------------------------------------------------------------
// flatten the model into device tables (layout: mfp_analysis.h)
// ---------------------------------------------------------------------------
namespace {

uint64_t pow2_at_least(uint64_t n) {
    uint64_t p = 16;
    while (p < n) p <<= 1;
    return p;
}


// ---------------------------------------------------------------------------
// the reference's LC-trie, built as it builds it (lctrie/lctrie.hpp,
// lctrie_ip.hpp, ipv6_lctrie.h), for a W-bit key (32: IPv4 in a1's low word;
// 128: IPv6 as (a0, a1) = (high, low) 64-bit halves, ip_address.hpp:775-814)
// ---------------------------------------------------------------------------
struct LNet {
    uint64_t a0 = 0, a1 = 0;
    uint8_t type = 0, len = 0;           // IP_BASE 0 / IP_PREFIX 1 / IP_PREFIX_FULL 2
    uint32_t prefix = MFP_LCT_NIL;
    uint32_t val = 0;
};
struct LTrie {
    std::vector<mfp_lct_node> node;      // empty: no table (lookups find nothing)
    std::vector<LNet> net;
};

template <int W> uint64_t l_ext(uint32_t pos, uint32_t num, const LNet &k) {
    if constexpr (W == 32) return lct_ext4(pos, num, (uint32_t)k.a1);
    else return lct_ext6(pos, num, k.a0, k.a1);
}
template <int W> uint64_t l_ext_idx(uint32_t pos, uint32_t num, const LNet &k) {
    if constexpr (W == 32) return lct_ext4(pos, num, (uint32_t)k.a1);
    else return lct_ext6_idx(pos, num, k.a0, k.a1);
}
// REMOVE (common.hpp:98-101, ipv6_lctrie.h:196-212)
template <int W> LNet l_remove(uint32_t p, const LNet &k) {
    LNet r;
    if constexpr (W == 32) {
        r.a1 = lct_shr32(lct_shl32((uint32_t)k.a1, p), p);
    } else if (p < 64) {
        r.a0 = lct_shr64(lct_shl64(k.a0, p), p); r.a1 = k.a1;
    } else {
        r.a1 = lct_shr64(lct_shl64(k.a1, p - 64), p - 64);
    }
    return r;
}
bool l_less(const LNet &x, const LNet &y) { return x.a0 != y.a0 ? x.a0 < y.a0 : x.a1 < y.a1; }

// subnet_isprefix (lctrie_ip.hpp:427-434)
template <int W> bool l_isprefix(const LNet &s, const LNet &t) {
    return s.len == 0 || (s.len <= t.len && l_ext<W>(0, s.len, s) == l_ext<W>(0, s.len, t));
}

// compute_skip (lctrie.hpp:87-109)
template <int W> uint8_t l_skip(const LTrie &T, const std::vector<uint32_t> &bases, uint32_t prefix, uint32_t first,
                                uint32_t num, uint32_t *newprefix) {
    if (prefix == 0 && first == 0) return 0;
    const LNet lo = l_remove<W>(prefix, T.net[bases[first]]), hi = l_remove<W>(prefix, T.net[bases[first + num - 1]]);
    uint32_t i = prefix;
    while (i < 2u * W && l_ext<W>(i, 1, lo) == l_ext<W>(i, 1, hi)) i++;
    *newprefix = i;
    return (uint8_t)(*newprefix - prefix);
}

// compute_branch (lctrie.hpp:111-159); FILLFACT 50, ROOT_BRANCH 16
template <int W> uint8_t l_branch(const LTrie &T, const std::vector<uint32_t> &bases, uint32_t prefix, uint32_t first,
                                  uint32_t num, uint32_t newprefix) {
    if (num == 2) return 1;
    if (prefix == 0 && first == 0) return 16;
    size_t bits = 1, count = 0;
    do {
        bits++;
        if (num < ((50u * (1u << bits)) / 100u) || (newprefix + bits) > (size_t)W) break;
        size_t i = first;
        count = 0;
        const uint64_t maxpat = (uint64_t)1 << bits;
        for (uint64_t pat = 0; pat < maxpat; pat++) {
            bool found = false;
            while (i < first + num && pat == l_ext<W>(newprefix, (uint32_t)bits, T.net[bases[i]])) { i++; found = true; }
            if (found) count++;
        }
    } while (count >= ((50u * (1u << bits)) / 100u));
    return (uint8_t)(bits - 1);
}

// build_inner (lctrie.hpp:161-248); node indices grow as the reference's do
template <int W> void l_build_inner(LTrie &T, const std::vector<uint32_t> &bases, uint32_t &ncount, uint32_t prefix,
                                    uint32_t first, uint32_t num, uint32_t pos) {
    if (T.node.size() < (size_t)ncount) T.node.resize(ncount);
    mfp_lct_node &nd0 = T.node[pos];
    if (num == 1) {
        nd0.branch = 0; nd0.skip = 0; nd0.index = first;
        return;
    }
    uint32_t newprefix = 0;
    const uint8_t skip = l_skip<W>(T, bases, prefix, first, num, &newprefix);
    const uint8_t branch = l_branch<W>(T, bases, prefix, first, num, newprefix);
    const uint32_t idx = ncount;
    T.node[pos].skip = skip; T.node[pos].branch = branch; T.node[pos].index = idx;
    ncount += 1u << branch;
    T.node.resize(ncount);
    // an empty slot's pattern compared through the 32-bit EXTRACT overload
    // (common.hpp:86): the uint64_t bit pattern does not convert to
    // ipv6_addr_lct (explicit constructor), so IPv6 builds take it too
    auto slot_bits = [&](uint64_t bitpat, uint32_t n) -> uint64_t {
        return lct_ext4((uint32_t)W - branch, n, (uint32_t)bitpat);
    };
    auto chain_match = [&](uint32_t base, uint64_t bitpat) -> uint32_t {
        uint32_t prep = T.net[base].prefix;
        while (prep != MFP_LCT_NIL) {
            const uint32_t len = T.net[prep].len;
            if (len > newprefix && l_ext_idx<W>(newprefix, len - newprefix, T.net[base]) == slot_bits(bitpat, len - newprefix))
                return len;
            prep = T.net[prep].prefix;
        }
        return 0;
    };
    size_t p = first;
    for (uint64_t bitpat = 0; bitpat < ((uint64_t)1 << branch); ++bitpat) {
        size_t k = 0;
        while (p + k < first + num && l_ext_idx<W>(newprefix, branch, T.net[bases[p + k]]) == bitpat) ++k;
        if (k == 0) {
            const uint32_t match1 = p > first ? chain_match(bases[p - 1], bitpat) : 0;
            const uint32_t match2 = p < first + num ? chain_match(bases[p], bitpat) : 0;
            if ((match1 > match2 && p > first) || p == first + num)
                l_build_inner<W>(T, bases, ncount, newprefix + branch, (uint32_t)p - 1, 1, idx + (uint32_t)bitpat);
            else
                l_build_inner<W>(T, bases, ncount, newprefix + branch, (uint32_t)p, 1, idx + (uint32_t)bitpat);
        } else if (k == 1 && (uint32_t)(T.net[bases[p]].len - newprefix) < (uint32_t)branch) {
            const size_t bits = branch - T.net[bases[p]].len + newprefix;
            for (uint32_t i = (uint32_t)bitpat; i < bitpat + (1u << bits); i++)
                l_build_inner<W>(T, bases, ncount, newprefix + branch, (uint32_t)p, 1, idx + i);
            bitpat = bitpat + (1u << bits) - 1;
        } else {
            l_build_inner<W>(T, bases, ncount, newprefix + branch, (uint32_t)p, (uint32_t)k, idx + (uint32_t)bitpat);
        }
        p += k;
    }
}

// subnet_data::process_final / process_final_v6 / process_domain_mappings_final[_v6]
// (addr.cc:460-705) over (address, length, value) entries in file order:
// subnet_mask_v4/_v6, qsort by (address, length) -- glibc's qsort is a stable
// merge sort here -- subnet_dedup kept literally (of two adjacent equal
// prefixes the first stays and the loop steps past the survivor), subnet_prefix
// with its UINT64_MAX size cap, the full-prefix check that abandons the table,
// then lct_build
template <int W> LTrie l_build(std::vector<LNet> v) {
    LTrie T;
    if (v.empty()) return T;
    for (auto &s : v) {
        if constexpr (W == 32) {
            const uint32_t mask = s.len >= 32 ? 0xffffffffu : ~(0xffffffffu >> s.len);
            s.a1 = (uint32_t)s.a1 & mask;
        } else {
            const u128 a = (u128)s.a0 << 64 | s.a1;
            const u128 mask = s.len >= 128 ? ~(u128)0 : ~(~(u128)0 >> s.len);
            s.a0 = (uint64_t)((a & mask) >> 64); s.a1 = (uint64_t)(a & mask);
        }
    }
    std::stable_sort(v.begin(), v.end(), [](const LNet &x, const LNet &y) {
        if (l_less(x, y)) return true;
        if (l_less(y, x)) return false;
        return x.len < y.len;
    });
    size_t size = v.size();
    for (size_t i = 0, j = 1; j < size; ++i, ++j)
        if (v[i].a0 == v[j].a0 && v[i].a1 == v[j].a1 && v[i].len == v[j].len) {
            v.erase(v.begin() + (long)j);
            --size;
        }
    // subnet_prefix (lctrie_ip.hpp:440-585)
    const size_t n = v.size();
    std::vector<uint64_t> sz(n), used(n, 0);
    for (size_t i = 0; i < n; ++i) v[i].prefix = MFP_LCT_NIL;
    for (size_t i = 0; i < n; ++i) {
        const size_t j = i + 1;
        if (j < n && l_isprefix<W>(v[i], v[j])) {
            v[j].prefix = (uint32_t)i;
            for (size_t k = j + 1; k < n && l_isprefix<W>(v[i], v[k]); ++k) v[k].prefix = (uint32_t)i;
            v[i].type = 1;
        } else {
            v[i].type = 0;
        }
        const unsigned host_bits = W - v[i].len;
        sz[i] = host_bits >= 64 ? UINT64_MAX : (uint64_t)1 << host_bits;
    }
    for (size_t i = 0; i < n; ++i)
        if (v[i].prefix != MFP_LCT_NIL) used[v[i].prefix] += sz[i];
    for (size_t i = 0; i < n; ++i)
        if (used[i] == sz[i]) v[i].type = 2;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t pr = v[i].prefix;
        if (pr != MFP_LCT_NIL && v[pr].type == 2) v[i].prefix = v[pr].prefix;
    }
    for (size_t i = 0; i < n; ++i)
        if (v[i].prefix != MFP_LCT_NIL && v[v[i].prefix].type == 2) return T;   // the reference returns unbuilt
    // lct_build (lctrie.hpp:262-319)
    std::vector<uint32_t> bases;
    for (size_t i = 0; i < n; ++i)
        if (v[i].type == 0) bases.push_back((uint32_t)i);
    if (bases.empty()) return T;
    T.net = std::move(v);
    T.node.assign(1, mfp_lct_node{0, 0, 0, 0});
    uint32_t ncount = 1;
    l_build_inner<W>(T, bases, ncount, 0, 0, (uint32_t)bases.size(), 0);
    T.node.resize(ncount);
    for (auto &nd : T.node)
        if (nd.branch == 0) nd.index = bases[nd.index];   // leaves hold the net index
    return T;
}

LNet lnet4(uint32_t addr_host, int len, uint32_t val) { LNet s; s.a1 = addr_host; s.len = (uint8_t)len; s.val = val; return s; }
LNet lnet6(u128 addr, int len, uint32_t val) {
    LNet s; s.a0 = (uint64_t)(addr >> 64); s.a1 = (uint64_t)addr; s.len = (uint8_t)len; s.val = val; return s;
}
std::vector<mfp_lct_net4> dev_nets4(const LTrie &T) {
    std::vector<mfp_lct_net4> o;
    for (auto &s : T.net) o.push_back(mfp_lct_net4{(uint32_t)s.a1, s.prefix, s.val, s.len});
    return o;
}
std::vector<mfp_lct_net6> dev_nets6(const LTrie &T) {
    std::vector<mfp_lct_net6> o;
    for (auto &s : T.net) o.push_back(mfp_lct_net6{s.a0, s.a1, s.prefix, s.val, s.len, 0});
    return o;
}

struct HostTables {
    std::vector<mfp_fp_slot> fp_slots;
    std::vector<mfp_entry> entry;
    std::vector<double> prior;
    std::vector<uint32_t> proc_id;
    std::vector<uint8_t> proc_mal;
    std::vector<uint32_t> proc_attr;
    std::vector<mfp_feat_slot> feat_slots;
    std::vector<mfp_update> upd;
    std::vector<char> pool;
    std::vector<mfp_fp_slot> prev_slots;   // known prevalence set
    LTrie asn4, asn6;                    // pyasn.db (subnet_data's ipv4/ipv6_subnet_trie)
    // additional attributes
    std::vector<mfp_fp_slot> doh_names, dom_slots;
    std::vector<uint32_t> doh_v4;
    std::vector<uint64_t> doh_v6;
    LTrie dom4, dom6;                    // domain-mappings.db (ipv4/ipv6_domain_trie)
    std::vector<uint32_t> dom_info;
    std::vector<uint8_t> dom_bytes;
};

uint32_t pool_add(HostTables &t, const std::string &s) {
    uint32_t off = (uint32_t)t.pool.size();
    t.pool.insert(t.pool.end(), s.begin(), s.end());
    while (t.pool.size() % 8) t.pool.push_back(0);
    return off;
}

void insert_string_slot(std::vector<mfp_fp_slot> &slots, uint64_t h, uint32_t id, uint32_t off, uint32_t len) {
    uint64_t mask = slots.size() - 1;
    for (uint64_t k = h & mask;; k = (k + 1) & mask) {
        if (slots[k].id == 0xffffffffu) {
            slots[k].hash = h; slots[k].id = id; slots[k].str_off = off; slots[k].str_len = len;
            return;
        }
    }
}

}  // namespace


namespace {

// the four LC-tries of subnet_data (addr.cc:460-705): pyasn.db IPv4 / IPv6
// (subnet_data::get_asn_info addr.cc:172-208) and the domain mappings
// (is_domain_faking addr.cc:707-792; a subnet's value = 1 + its dom_info index)
void build_tries(const mfp_classifier_s &cs, HostTables &t) {
    const mfp_classifier_s *c = &cs;
    {
        std::vector<LNet> v;
        for (auto &p : c->asn4) v.push_back(lnet4((uint32_t)(p.first >> 8), (int)(p.first & 0xff), p.second));
        t.asn4 = l_build<32>(std::move(v));
        v.clear();
        for (auto &p : c->asn6) {
            u128 a = 0;
            for (int k = 0; k < 16; k++) a = a << 8 | (uint8_t)p.first[k];
            v.push_back(lnet6(a, (uint8_t)p.first[16], p.second));
        }
        t.asn6 = l_build<128>(std::move(v));
    }
    for (int fam = 0; fam < 2; fam++) {
        const std::vector<DomPrefix> &src = fam == 0 ? c->dom4 : c->dom6;
        std::vector<LNet> v;
        for (size_t k = 0; k < src.size(); k++)
            v.push_back(fam == 0 ? lnet4((uint32_t)src[k].addr, src[k].len, (uint32_t)k) : lnet6(src[k].addr, src[k].len, (uint32_t)k));
        LTrie T = fam == 0 ? l_build<32>(std::move(v)) : l_build<128>(std::move(v));
        for (auto &s : T.net) {   // value: 1 + the subnet's dom_info index
            const DomPrefix &dp = src[s.val];
            s.val = (uint32_t)t.dom_info.size() / 2 + 1;
            t.dom_info.push_back(dp.type | (uint32_t)dp.idx.size() << 8);
            t.dom_info.push_back((uint32_t)t.dom_bytes.size());
            t.dom_bytes.insert(t.dom_bytes.end(), dp.idx.begin(), dp.idx.end());
        }
        (fam == 0 ? t.dom4 : t.dom6) = std::move(T);
    }
}
}  // namespace

int mfp_classifier_upload(mfp_classifier *c, int device) {
    HostTables t;
    // fingerprint table
    t.fp_slots.assign(pow2_at_least(2 * c->fpdb.size() + 2), mfp_fp_slot{0, 0xffffffffu, 0, 0});
    for (auto &fs : c->fp_order) {
        uint32_t off = pool_add(t, fs);
        insert_string_slot(t.fp_slots, mfpc::str_hash((const uint8_t *)fs.data(), (uint32_t)fs.size()), c->fpdb[fs], off,
                           (uint32_t)fs.size());
    }
    // known prevalence set
    t.prev_slots.assign(pow2_at_least(2 * c->known_prevalence.size() + 2), mfp_fp_slot{0, 0xffffffffu, 0, 0});
    for (auto &fs : c->known_prevalence) {
        uint32_t off = pool_add(t, fs);
        insert_string_slot(t.prev_slots, mfpc::str_hash((const uint8_t *)fs.data(), (uint32_t)fs.size()), 0, off,
                           (uint32_t)fs.size());
    }
    // entries, processes, features
    // the feature table: one open-addressing region per entry (a power of two,
    // at most half full), so a packet's six probes -- and those of every other
    // packet with the same fingerprint -- stay within the entry's few lines
    std::vector<uint64_t> reg_base(c->entries.size()), reg_mask(c->entries.size());
    uint64_t nslots = 0;
    for (uint32_t eid = 0; eid < c->entries.size(); eid++) {
        uint64_t nf = 0;
        for (auto &f : c->entries[eid]->f) nf += f.by_str.size() + f.by_int.size() + f.by_v6.size();
        const uint64_t r = pow2_at_least(2 * nf + 2);
        reg_base[eid] = nslots; reg_mask[eid] = r - 1;
        nslots += r;
    }
    if (nslots >> 32) { mfp_set_error("feature table too large"); return -1; }
    t.feat_slots.assign(nslots ? nslots : 1, mfp_feat_slot{0, 0xffffffffu, 0, 0, 0, 0, 0});
    auto put_feat = [&](uint32_t eid, uint32_t kind, uint64_t key, const std::vector<Upd> &lst, const std::string *str) {
        mfp_feat_slot s;
        s.key = key; s.entry = eid; s.kind = kind;
        s.upd_off = (uint32_t)t.upd.size(); s.upd_cnt = (uint32_t)lst.size();
        // a list whose process indices are distinct can be applied as one
        // lane-parallel scatter; repeated indices (e.g. two private IPv4
        // addresses normalised to one key) keep the reference's serial order
        {
            std::vector<uint32_t> ix;
            for (auto &u : lst) ix.push_back(u.idx);
            std::sort(ix.begin(), ix.end());
            if (std::adjacent_find(ix.begin(), ix.end()) != ix.end()) s.upd_cnt |= MFP_UPD_SERIAL;
        }
        s.str_off = str ? pool_add(t, *str) : 0; s.str_len = str ? (uint32_t)str->size() : 0;
        for (auto &u : lst) t.upd.push_back(mfp_update{u.idx, 0, u.val});
        const uint64_t base = reg_base[eid], mask = reg_mask[eid];
        for (uint64_t k = mfpc::feat_slot_hash(eid, kind, key) & mask;; k = (k + 1) & mask)
            if (t.feat_slots[base + k].entry == 0xffffffffu) { t.feat_slots[base + k] = s; break; }
    };
    for (uint32_t eid = 0; eid < c->entries.size(); eid++) {
        Entry &e = *c->entries[eid];
        mfp_entry me;
        me.proc_off = (uint32_t)t.prior.size();
        me.nproc = (uint32_t)e.prior.size();
        me.malware_db = e.malware_db;
        me.generic_dmz = 0xffffffffu;
        me.mal_bits = 0; me.pad = 0;
        me.feat_base = (uint32_t)reg_base[eid]; me.feat_mask = (uint32_t)reg_mask[eid];
        for (uint32_t i = 0; i < me.nproc; i++) {
            if (i < 32 && e.malware[i]) me.mal_bits |= 1u << i;
            t.prior.push_back(e.prior[i]);
            t.proc_id.push_back(c->proc_name_id[e.proc_name[i]]);
            t.proc_mal.push_back(e.malware[i]);
            t.proc_attr.push_back(e.attr[i]);
            if (e.proc_name[i] == "generic dmz process") me.generic_dmz = i;
        }
        t.entry.push_back(me);
        for (uint32_t k = 0; k < 7; k++) {
            for (auto &kv : e.f[k].by_int) put_feat(eid, k, kv.first, kv.second, nullptr);
            for (auto &kv : e.f[k].by_str)
                put_feat(eid, k, mfpc::str_hash((const uint8_t *)kv.first.data(), (uint32_t)kv.first.size()), kv.second,
                         &kv.first);
            for (auto &kv : e.f[k].by_v6)
                put_feat(eid, k, mfpc::str_hash((const uint8_t *)kv.first.data(), 16), kv.second, &kv.first);
        }
    }
    build_tries(*c, t);
    // encrypted_dns watchlist: names (hash table), addresses (sorted sets)
    t.doh_names.assign(pow2_at_least(2 * c->doh_names.size() + 2), mfp_fp_slot{0, 0xffffffffu, 0, 0});
    for (auto &nm : c->doh_names)
        insert_string_slot(t.doh_names, mfpc::str_hash((const uint8_t *)nm.data(), (uint32_t)nm.size()), 0,
                           pool_add(t, nm), (uint32_t)nm.size());
    t.doh_v4 = c->doh_v4;
    std::sort(t.doh_v4.begin(), t.doh_v4.end());
    t.doh_v4.erase(std::unique(t.doh_v4.begin(), t.doh_v4.end()), t.doh_v4.end());
    {
        auto v6 = c->doh_v6;
        std::sort(v6.begin(), v6.end());
        v6.erase(std::unique(v6.begin(), v6.end()), v6.end());
        for (auto &x : v6) { t.doh_v6.push_back(x.first); t.doh_v6.push_back(x.second); }
    }
    // domain_faking: mapped domains (hash table -> domain index) and the
    // mapping / exception prefixes (process_domain_mappings_final[_v6]
    // addr.cc:584-705: masked, sorted, deduplicated, longest match)
    t.dom_slots.assign(pow2_at_least(2 * c->dom_idx.size() + 2), mfp_fp_slot{0, 0xffffffffu, 0, 0});
    for (auto &kv : c->dom_idx)
        insert_string_slot(t.dom_slots, mfpc::str_hash((const uint8_t *)kv.first.data(), (uint32_t)kv.first.size()),
                           kv.second, pool_add(t, kv.first), (uint32_t)kv.first.size());
    if (t.pool.empty()) t.pool.push_back(0);
    if (t.upd.empty()) t.upd.push_back(mfp_update{0, 0, 0});
    if (t.prior.empty()) { t.prior.push_back(0); t.proc_id.push_back(0); t.proc_mal.push_back(0); t.proc_attr.push_back(0); }
    if (t.entry.empty()) t.entry.push_back(mfp_entry{0, 0, 0, 0, 0, 0, 0, 0});
    if (t.doh_v4.empty()) t.doh_v4.push_back(0);
    if (t.doh_v6.empty()) { t.doh_v6.push_back(0); t.doh_v6.push_back(0); }
    if (t.dom_info.empty()) { t.dom_info.push_back(0); t.dom_info.push_back(0); }
    if (t.dom_bytes.empty()) t.dom_bytes.push_back(0);

    // device copies of the tries (a table the reference leaves unbuilt gets
    // one placeholder node and no lookups: n_* = 0)
    auto nodes = [](const LTrie &T) { return T.node.empty() ? std::vector<mfp_lct_node>(1, mfp_lct_node{0, 0, 0, 0}) : T.node; };
    auto nets4 = [](const LTrie &T) { return T.net.empty() ? std::vector<mfp_lct_net4>(1, mfp_lct_net4{0, 0, 0, 0}) : dev_nets4(T); };
    auto nets6 = [](const LTrie &T) { return T.net.empty() ? std::vector<mfp_lct_net6>(1, mfp_lct_net6{0, 0, 0, 0, 0, 0}) : dev_nets6(T); };
    const auto asn4_node = nodes(t.asn4), asn6_node = nodes(t.asn6), dom4_node = nodes(t.dom4), dom6_node = nodes(t.dom6);
    const auto asn4_net = nets4(t.asn4), dom4_net = nets4(t.dom4);
    const auto asn6_net = nets6(t.asn6), dom6_net = nets6(t.dom6);
    mfp_classifier_dev &d = c->dev;
    mfp_classifier_free_device(d);
    if (hipSetDevice(device) != hipSuccess) return -1;
    c->device = device;
    auto up = [&](auto *&dst, const auto &vec) -> bool {
        size_t bytes = vec.size() * sizeof(vec[0]);
        if (hipMalloc((void **)&dst, bytes) != hipSuccess) return false;
        return hipMemcpy((void *)dst, vec.data(), bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    bool ok = up(d.fp_slots, t.fp_slots) && up(d.prev_slots, t.prev_slots) && up(d.entry, t.entry) &&
              up(d.prior, t.prior) && up(d.proc_id, t.proc_id) && up(d.proc_mal, t.proc_mal) &&
              up(d.proc_attr, t.proc_attr) && up(d.feat_slots, t.feat_slots) && up(d.upd, t.upd) && up(d.pool, t.pool) &&
              up(d.asn4_node, asn4_node) && up(d.asn4_net, asn4_net) && up(d.asn6_node, asn6_node) &&
              up(d.asn6_net, asn6_net) && up(d.doh_names, t.doh_names) &&
              up(d.doh_v4, t.doh_v4) && up(d.doh_v6, t.doh_v6) && up(d.dom_slots, t.dom_slots) &&
              up(d.dom4_node, dom4_node) && up(d.dom4_net, dom4_net) && up(d.dom6_node, dom6_node) &&
              up(d.dom6_net, dom6_net) && up(d.dom_info, t.dom_info) && up(d.dom_bytes, t.dom_bytes);
    if (!ok) { mfp_set_error("classifier device upload failed"); return -2; }
    {
        auto nb = [](const auto &v) { return (uint64_t)(v.size() * sizeof(v[0])); };
        c->device_bytes = nb(t.fp_slots) + nb(t.prev_slots) + nb(t.entry) + nb(t.prior) + nb(t.proc_id) +
                          nb(t.proc_mal) + nb(t.proc_attr) + nb(t.feat_slots) + nb(t.upd) + nb(t.pool) + nb(asn4_node) +
                          nb(asn4_net) + nb(asn6_node) + nb(asn6_net) + nb(t.doh_names) + nb(t.doh_v4) + nb(t.doh_v6) +
                          nb(t.dom_slots) + nb(dom4_node) + nb(dom4_net) + nb(dom6_node) + nb(dom6_net) +
                          nb(t.dom_info) + nb(t.dom_bytes);
    }
    d.fp_mask = t.fp_slots.size() - 1;
    d.prev_mask = t.prev_slots.size() - 1;
    d.n_asn4 = (uint32_t)t.asn4.node.size();
    d.n_asn6 = (uint32_t)t.asn6.node.size();
    const char *rnd[3] = {"tls/randomized", "tls/1/randomized", "tls/2/randomized"};
    for (int k = 0; k < 3; k++) {
        auto it = c->fpdb.find(rnd[k]);
        d.randomized_entry[k] = it == c->fpdb.end() ? 0xffffffffu : it->second;
    }
    d.types_mask = 0;
    for (uint32_t ty : c->fp_types) d.types_mask |= 1u << ty;
    d.max_nproc = 0;
    for (const auto &me : t.entry) d.max_nproc = std::max(d.max_nproc, me.nproc);
    d.enc_channel_idx = 7;
    d.faketls_idx = 9;
    d.doh_idx = 6;
    d.domain_faking_idx = 8;
    d.db_tags = 0;
    for (size_t k = MFP_ATTR_DB_FIRST; k < c->attr_names.size() && k < MFP_ATTR_MAX_TAGS; k++) d.db_tags |= 1u << k;
    d.doh_enabled = c->doh_enabled;
    d.doh_names_mask = t.doh_names.size() - 1;
    d.n_doh_v4 = (uint32_t)c->doh_v4.size() ? (uint32_t)t.doh_v4.size() : 0;
    d.n_doh_v6 = (uint32_t)(c->doh_v6.empty() ? 0 : t.doh_v6.size() / 2);
    d.faking_enabled = c->faking_enabled;
    d.dom_mask = t.dom_slots.size() - 1;
    d.n_dom4 = (uint32_t)t.dom4.node.size();
    d.n_dom6 = (uint32_t)t.dom6.node.size();
    return 0;
}

// Test hook (CPU): the four subnet tries built exactly as the device gets
// them and queried on the host with the device's lookup (mfp_lctrie.hpp),
// for subnet_data::get_asn_info and is_domain_faking (addr.cc:172-208,
// 707-792).  queries: "dst_ip<TAB>server_name" lines (no name: no faking
// check); returns the number of queries answered, -1 on a load error.
extern "C" MFP_EXPORT long long mfp_lpm_query(const char *resources, const char *queries, uint32_t *asn, int8_t *fake,
                                              size_t cap) {
    mfp_classifier *c = mfp_classifier_load(resources);
    if (!c) return -1;
    HostTables t;
    build_tries(*c, t);
    auto find4 = [](const LTrie &T, uint32_t k) -> const LNet * {
        if (T.node.empty()) return nullptr;
        const std::vector<mfp_lct_net4> nets = dev_nets4(T);
        const uint32_t s = lct_find4(T.node.data(), nets.data(), k);
        return s == MFP_LCT_NIL ? nullptr : &T.net[s];
    };
    auto find6 = [](const LTrie &T, uint64_t k0, uint64_t k1) -> const LNet * {
        if (T.node.empty()) return nullptr;
        const std::vector<mfp_lct_net6> nets = dev_nets6(T);
        const uint32_t s = lct_find6(T.node.data(), nets.data(), k0, k1);
        return s == MFP_LCT_NIL ? nullptr : &T.net[s];
    };
    auto dom_match = [&](const LNet *sub, uint32_t didx) -> bool {   // false: not faking
        if (!sub) return true;
        const uint32_t ty = t.dom_info[2 * (sub->val - 1)], off = t.dom_info[2 * (sub->val - 1) + 1];
        if ((ty & 0xff) == MFP_DOM_EXCEPTION) return false;
        for (uint32_t k = 0; k < (ty >> 8); k++)
            if ((uint32_t)t.dom_bytes[off + k] == didx) return false;
        return true;
    };
    long long n = 0;
    const char *q = queries;
    while (*q && (size_t)n < cap) {
        const char *e = strchr(q, '\n');
        std::string line = e ? std::string(q, e - q) : std::string(q);
        q = e ? e + 1 : q + line.size();
        const size_t tab = line.find('\t');
        const std::string ip = line.substr(0, tab), name = tab == std::string::npos ? "" : line.substr(tab + 1);
        uint8_t d[4];
        const bool v4 = sscanf(ip.c_str(), "%hhu.%hhu.%hhu.%hhu", d, d + 1, d + 2, d + 3) == 4;
        const uint32_t k4 = (uint32_t)d[0] << 24 | (uint32_t)d[1] << 16 | (uint32_t)d[2] << 8 | d[3];
        uint64_t k0 = 0, k1 = 0;
        bool v6 = false;
        if (!v4) {
            uint8_t b[16];
            int pos = 0;
            v6 = mfpc::parse_ipv6((const uint8_t *)ip.data(), (int)ip.size(), pos, b) && pos == (int)ip.size();
            for (int k = 0; k < 8; k++) { k0 = k0 << 8 | b[k]; k1 = k1 << 8 | b[8 + k]; }
        }
        const LNet *a = v4 ? find4(t.asn4, k4) : v6 ? find6(t.asn6, k0, k1) : nullptr;
        asn[n] = a ? a->val : 0;
        int8_t f = 0;
        if (!name.empty()) {
            const std::string nm = name.compare(0, 4, "www.") == 0 ? name.substr(4) : name;
            auto it = c->dom_idx.find(nm);
            if (it != c->dom_idx.end()) {
                if (v4) {
                    const bool priv = d[0] == 10 || (d[0] == 172 && (d[1] & 0xf0) == 16) || (d[0] == 192 && d[1] == 168);
                    f = !priv && dom_match(find4(t.dom4, k4), it->second);
                } else if (v6 && !t.dom6.node.empty()) {
                    const uint8_t b7 = (uint8_t)k0;   // is_private_address: the first byte in memory of a[0]
                    f = !(b7 == 0xfc || b7 == 0xfd) && dom_match(find6(t.dom6, k0, k1), it->second);
                }
            }
        }
        fake[n] = f;
        n++;
    }
    mfp_classifier_free(c);
    return n;
}

void mfp_classifier_free_device(mfp_classifier_dev &d) {
    void *ptrs[] = {d.fp_slots, d.prev_slots, d.entry, d.prior, d.proc_id, d.proc_mal, d.proc_attr,
                    d.feat_slots, d.upd, d.pool, d.asn4_node, d.asn4_net, d.asn6_node, d.asn6_net, d.doh_names,
                    d.doh_v4, d.doh_v6, d.dom_slots, d.dom4_node, d.dom4_net, d.dom6_node, d.dom6_net, d.dom_info,
                    d.dom_bytes};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    d = mfp_classifier_dev{};
}

const mfp_classifier_dev *mfp_classifier_device(const mfp_classifier *c) { return &c->dev; }
mfp_classifier_dev *mfp_classifier_device_mut(mfp_classifier *c) { return &c->dev; }

// host-only helper exported for tests: the normalisation the device uses
extern "C" MFP_EXPORT int mfp_normalize_server_name(const char *name, size_t len, char *out, size_t cap) {
    char buf[400];
    int n = mfpc::normalize_server_name((const uint8_t *)name, (int)len, buf);
    if ((size_t)n + 1 > cap) return -1;
    memcpy(out, buf, n);
    out[n] = 0;
    return n;
}
