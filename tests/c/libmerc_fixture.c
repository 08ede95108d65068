/*
 * libmerc_fixture.c -- the libmerc counters of the reference's unit tests
 * (unit_tests/libmerc_fixture.cc:107-314, cases from
 * unit_tests/libmerc_dbmultiprotocol_test.cc) as a plain C program over the
 * public libmerc API (include/mercury_amd_libmerc.h, the layout of
 * src/libmerc/libmerc.h).
 *
 *   libmerc_fixture <libmerc .so> <pcap dir> <resources-test.tgz>
 *
 * The library is dlopen()ed, so the same binary counts through
 * libmercury_amd.so (the MI355X path, on the GPU box) and through the
 * reference's own libmerc (oracle/_ref/libmerc_ref.so, on the dev host) --
 * the second run pins the expected numbers to the reference.  The pcaps are
 * the reference's test pcaps, written back from tests/golden/ref_packets.npz
 * by tests/test_libmerc_fixture.py.  Every configuration is the reference
 * test's, "all" included (its protocols outside the device path write no
 * record, tests/test_all.py).  Prints one line per case and exits
 * non-zero when a count differs from the reference test's expectation.
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/mercury_amd_libmerc.h"

/* the API, resolved from the library under test */
static mercury_context (*p_init)(const struct libmerc_config *, int);
static int (*p_finalize)(mercury_context);
static mercury_packet_processor (*p_construct)(mercury_context);
static void (*p_destruct)(mercury_packet_processor);
static size_t (*p_write_json_linktype)(mercury_packet_processor, void *, size_t, uint8_t *, size_t, struct timespec *,
                                       uint16_t);
static const struct analysis_context *(*p_get_ac_linktype)(mercury_packet_processor, uint8_t *, size_t,
                                                           struct timespec *, uint16_t);
static enum fingerprint_type (*p_fp_type)(const struct analysis_context *);
static const struct attribute_context *(*p_get_attributes)(mercury_packet_processor);
static void (*p_register_printf_err)(printf_err_ptr);

static int quiet(enum log_level l, const char *f, va_list a) { (void)l; (void)f; (void)a; return 0; }

static void *sym(void *h, const char *name) {
    void *s = dlsym(h, name);
    if (!s) { fprintf(stderr, "missing symbol %s\n", name); exit(2); }
    return s;
}

/* ---- classic pcap, whole file in memory ---- */
struct pcap { uint8_t *buf; size_t len, off; int swap; uint16_t linktype; };

static int pcap_open(struct pcap *p, const char *dir, const char *name) {
    char path[4096];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); return -1; }
    fseek(f, 0, SEEK_END);
    p->len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    p->buf = malloc(p->len + 64);
    if (fread(p->buf, 1, p->len, f) != p->len) { fclose(f); return -1; }
    fclose(f);
    uint32_t magic;
    memcpy(&magic, p->buf, 4);
    p->swap = magic == 0xd4c3b2a1u;
    uint32_t lt;
    memcpy(&lt, p->buf + 20, 4);
    if (p->swap) lt = __builtin_bswap32(lt);
    p->linktype = (uint16_t)lt;
    p->off = 24;
    return 0;
}

/* next packet: 1 and (data, len), 0 at the end */
static int pcap_next(struct pcap *p, uint8_t **data, size_t *len) {
    if (p->off + 16 > p->len) return 0;
    uint32_t incl;
    memcpy(&incl, p->buf + p->off + 8, 4);
    if (p->swap) incl = __builtin_bswap32(incl);
    p->off += 16;
    if (p->off + incl > p->len) return 0;
    *data = p->buf + p->off;
    *len = incl;
    p->off += incl;
    return 1;
}

/* ---- the fixture's counters ---- */
enum mode {
    JSON_COUNT,        /* counter(): write_json records (libmerc_fixture.cc:107-123) */
    JSON_TYPE,         /* counter(fp_type): records whose fingerprint is of that type (:125-146) */
    AC_TYPE,           /* counter(fp_type, callback): analysis contexts of that type (:148-170) */
    ATTR_COUNT,        /* counter(n, callback): attributes of the first attribute context (:172-201) */
    CHECK_ATTR,        /* check_attr(name) (:291-314) */
    FIRST_JSON_HAS,    /* get_first_json() contains a string */
};

struct tcase {
    const char *name, *pcap, *filter;
    int analysis;
    enum mode mode;
    int fp_type;        /* JSON_TYPE / AC_TYPE */
    const char *what;   /* JSON_TYPE: the JSON fingerprint key; CHECK_ATTR / FIRST_JSON_HAS: the string */
    int expected;
    int linktype;       /* 0: the pcap's */
};

static const struct tcase cases[] = {
    /* "test tls select strings producing different output line counts" */
    {"tls.client_hello lines", "capture2.pcap", "tls.client_hello", 0, JSON_COUNT, 0, NULL, 17, 0},
    {"tls.client_hello,tls.server_hello lines", "capture2.pcap", "tls.client_hello,tls.server_hello", 0, JSON_COUNT,
     0, NULL, 60, 0},
    /* "test http" / "test http with analysis" */
    {"http without analysis", "capture2.pcap", "http", 0, AC_TYPE, fingerprint_type_http, NULL, 0, 0},
    {"http with analysis", "capture2.pcap", "http", 1, AC_TYPE, fingerprint_type_http, NULL, 127, 0},
    {"multi-packet http request with analysis", "multi_packet_http_request.pcap", "http", 1, AC_TYPE,
     fingerprint_type_http, NULL, 1, 0},
    /* "test http with analysis and linktype raw" */
    {"http raw IP with analysis", "http_rawip.pcap", "http", 1, AC_TYPE, fingerprint_type_http, NULL, 9, 101},
    /* "test linux sll2" / "test linux sll[2] with analysis" */
    {"linux sll2 lines", "sll2_tls.pcap", "all", 0, JSON_COUNT, 0, NULL, 1, 276},
    {"linux sll2 with analysis", "sll2_tls.pcap", "all", 1, AC_TYPE, fingerprint_type_tls, NULL, 1, 276},
    {"linux sll with analysis", "sll_tls.pcap", "all", 1, AC_TYPE, fingerprint_type_tls, NULL, 1, 113},
    /* "test SGT encapsulated TLS with analysis" */
    {"SGT TLS with analysis", "tls_sgt.pcap", "tls.client_hello", 1, AC_TYPE, fingerprint_type_tls, NULL, 58, 0},
    {"SGT TLS lines", "tls_sgt.pcap", "tls.client_hello", 1, JSON_COUNT, 0, NULL, 58, 0},
    /* "test dtls ... without reassembly" */
    {"dtls fragmented, no reassembly", "dtls_fragmented_client_hello.pcap", "dtls", 0, JSON_TYPE,
     fingerprint_type_dtls, "\"dtls\"", 0, 0},
    {"dtls partial fragment, no reassembly", "dtls_fragmented_client_hello_partial.pcap", "dtls", 0, JSON_TYPE,
     fingerprint_type_dtls, "\"dtls\"", 1, 0},
    {"dtls partial fragment truncated", "dtls_fragmented_client_hello_partial.pcap", "dtls", 0, FIRST_JSON_HAS, 0,
     "\"reassembly_properties\":{\"truncated\":true", 1, 0},
    /* "test attribute detection with analysis" */
    {"malware_tls attributes", "malware_tls.pcap", "all", 1, ATTR_COUNT, 0, NULL, 2, 0},
    {"ipv6 domain_faking", "ipv6-domain-faking.pcap", "all", 1, CHECK_ATTR, 0, "domain_faking", 1, 0},
    {"faketls", "faketls_potatovpn.pcap", "all", 1, CHECK_ATTR, 0, "faketls", 1, 0},
    {"faketls domain_faking", "faketls_potatovpn.pcap", "all", 1, CHECK_ATTR, 0, "domain_faking", 1, 0},
};

static char out[1 << 16];

static int run_case(const struct tcase *c, const char *dir, const char *resources) {
    struct libmerc_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.packet_filter_cfg = (char *)c->filter;
    cfg.resources = (char *)resources;      /* the reference tests always name the archive */
    cfg.do_analysis = c->analysis;
    mercury_context mc = p_init(&cfg, 0);
    if (!mc) { printf("%-45s init failed\n", c->name); return -1; }
    mercury_packet_processor p = p_construct(mc);
    struct pcap pc;
    if (pcap_open(&pc, dir, c->pcap) != 0) { p_destruct(p); p_finalize(mc); return -1; }
    const uint16_t lt = c->linktype ? (uint16_t)c->linktype : pc.linktype;
    int count = 0, done = 0;
    uint8_t *d;
    size_t len;
    while (!done && pcap_next(&pc, &d, &len)) {
        struct timespec ts = {0, 0};
        switch (c->mode) {
        case JSON_COUNT:
            if (p_write_json_linktype(p, out, sizeof out, d, len, &ts, lt) > 0) count++;
            break;
        case JSON_TYPE: {
            size_t n = p_write_json_linktype(p, out, sizeof out, d, len, &ts, lt);
            if (n > 0) {
                out[n < sizeof out ? n : sizeof out - 1] = 0;
                const char *f = strstr(out, "\"fingerprints\":{");
                if (f && !strncmp(f + 16, c->what, strlen(c->what))) count++;
            }
            break;
        }
        case FIRST_JSON_HAS: {
            size_t n = p_write_json_linktype(p, out, sizeof out, d, len, &ts, lt);
            if (n > 0) {
                out[n < sizeof out ? n : sizeof out - 1] = 0;
                count = strstr(out, c->what) != NULL;
                done = 1;
            }
            break;
        }
        case AC_TYPE: {
            const struct analysis_context *ac = p_get_ac_linktype(p, d, len, &ts, lt);
            if (ac && (int)p_fp_type(ac) == c->fp_type) count++;
            break;
        }
        case ATTR_COUNT:
        case CHECK_ATTR: {
            const struct analysis_context *ac = p_get_ac_linktype(p, d, len, &ts, lt);
            if (c->mode == ATTR_COUNT && !ac) break;
            const struct attribute_context *at = p_get_attributes(p);
            if (!at) break;
            int n = 0, found = 0;
            for (size_t i = 0; i < at->attributes_len; i++) {
                if (at->prob_scores[i] > 0) {
                    n++;
                    if (c->what && !strcmp(at->tag_names[i], c->what)) found = 1;
                }
            }
            count = c->mode == ATTR_COUNT ? n : found;
            done = 1;
            break;
        }
        }
    }
    free(pc.buf);
    p_destruct(p);
    p_finalize(mc);
    return count;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <libmerc .so> <pcap dir> <resources-test.tgz> [case substring]\n", argv[0]);
        return 2;
    }
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "%s\n", dlerror()); return 2; }
    p_init = sym(h, "mercury_init");
    p_finalize = sym(h, "mercury_finalize");
    p_construct = sym(h, "mercury_packet_processor_construct");
    p_destruct = sym(h, "mercury_packet_processor_destruct");
    p_write_json_linktype = sym(h, "mercury_packet_processor_write_json_linktype");
    p_get_ac_linktype = sym(h, "mercury_packet_processor_get_analysis_context_linktype");
    p_fp_type = sym(h, "analysis_context_get_fingerprint_type");
    p_get_attributes = sym(h, "mercury_packet_processor_get_attributes");
    p_register_printf_err = sym(h, "register_printf_err_callback");
    p_register_printf_err(quiet);
    int failed = 0;
    for (size_t i = 0; i < sizeof cases / sizeof cases[0]; i++) {
        if (argc > 4 && !strstr(cases[i].name, argv[4])) continue;
        const int got = run_case(&cases[i], argv[2], argv[3]);
        const int ok = got == cases[i].expected;
        failed += !ok;
        printf("%-45s expected %4d got %4d %s\n", cases[i].name, cases[i].expected, got, ok ? "ok" : "FAIL");
    }
    printf("%d case(s) failed\n", failed);
    return failed ? 1 : 0;
}
