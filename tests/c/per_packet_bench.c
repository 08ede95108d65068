/*
 * per_packet_bench.c -- the libmerc per-packet API as an embedder drives it
 * (src/pkt_processing.h:155-163, the Cython binding, unit_tests/
 * libmerc_fixture.cc): T threads, one mercury_packet_processor each (one
 * processor per thread, libmerc.h:227-231), every thread calling
 * mercury_packet_processor_write_json_linktype or _get_analysis_context_linktype
 * once per packet over its share of a pcap for a fixed time.
 *
 *   per_packet_bench <libmerc .so> <pcap> <config> <resources|-> <threads> <seconds> json|an
 *
 * The library is dlopen()ed: the same binary times libmercury_amd.so (the
 * MI355X path) and the reference's libmerc (oracle/_ref/libmerc_ref.so).
 * Prints one JSON line: packets/s over all threads, per-call latency
 * percentiles (microseconds), records written / contexts returned.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/mercury_amd_libmerc.h"

static mercury_context (*p_init)(const struct libmerc_config *, int);
static int (*p_finalize)(mercury_context);
static mercury_packet_processor (*p_construct)(mercury_context);
static void (*p_destruct)(mercury_packet_processor);
static size_t (*p_write_json_linktype)(mercury_packet_processor, void *, size_t, uint8_t *, size_t, struct timespec *,
                                       uint16_t);
static const struct analysis_context *(*p_get_ac_linktype)(mercury_packet_processor, uint8_t *, size_t,
                                                           struct timespec *, uint16_t);
static void (*p_register_printf_err)(printf_err_ptr);

static int quiet(enum log_level l, const char *f, va_list a) { (void)l; (void)f; (void)a; return 0; }

static void *sym(void *h, const char *name) {
    void *s = dlsym(h, name);
    if (!s) { fprintf(stderr, "missing symbol %s\n", name); exit(2); }
    return s;
}

struct pkt { uint8_t *d; uint32_t len; };
static struct pkt *pkts;
static size_t npkts;
static uint16_t linktype = 1;
static mercury_context mc;
static int analysis_entry;
static double seconds;

static int load_pcap(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) { perror(path); return -1; }
    fseek(f, 0, SEEK_END);
    size_t n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *buf = malloc(n + 64);
    if (fread(buf, 1, n, f) != n) { fclose(f); return -1; }
    fclose(f);
    uint32_t magic, lt;
    memcpy(&magic, buf, 4);
    const int swap = magic == 0xd4c3b2a1u;
    memcpy(&lt, buf + 20, 4);
    linktype = (uint16_t)(swap ? __builtin_bswap32(lt) : lt);
    size_t cap = 1024, off = 24;
    pkts = malloc(cap * sizeof *pkts);
    while (off + 16 <= n) {
        uint32_t incl;
        memcpy(&incl, buf + off + 8, 4);
        if (swap) incl = __builtin_bswap32(incl);
        off += 16;
        if (off + incl > n) break;
        if (npkts == cap) { cap *= 2; pkts = realloc(pkts, cap * sizeof *pkts); }
        pkts[npkts].d = buf + off;
        pkts[npkts].len = incl;
        npkts++;
        off += incl;
    }
    return 0;
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

struct worker {
    pthread_t th;
    size_t lo, hi;
    unsigned long long calls, hits;
    double *lat;           /* per-call latency samples (us), every call up to lat_cap */
    size_t nlat, lat_cap;
};

static pthread_barrier_t start_barrier;

static void *run(void *arg) {
    struct worker *w = arg;
    mercury_packet_processor p = p_construct(mc);
    static __thread char out[1 << 16];
    pthread_barrier_wait(&start_barrier);
    const double t0 = now();
    size_t i = w->lo;
    while (now() - t0 < seconds) {
        for (int k = 0; k < 64; k++) {
            struct timespec ts = {1700000000, 0};
            const double a = now();
            if (analysis_entry) {
                if (p_get_ac_linktype(p, pkts[i].d, pkts[i].len, &ts, linktype)) w->hits++;
            } else {
                if (p_write_json_linktype(p, out, sizeof out, pkts[i].d, pkts[i].len, &ts, linktype) > 0) w->hits++;
            }
            const double b = now();
            if (w->nlat < w->lat_cap) w->lat[w->nlat++] = (b - a) * 1e6;
            w->calls++;
            if (++i >= w->hi) i = w->lo;
        }
    }
    p_destruct(p);
    return NULL;
}

static int cmp(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: %s <libmerc .so> <pcap> <config> <resources|-> <threads> <seconds> json|an\n", argv[0]);
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
    p_register_printf_err = sym(h, "register_printf_err_callback");
    p_register_printf_err(quiet);
    if (load_pcap(argv[2]) != 0 || npkts == 0) { fprintf(stderr, "no packets\n"); return 2; }
    const int threads = atoi(argv[5]);
    seconds = atof(argv[6]);
    analysis_entry = !strcmp(argv[7], "an");
    struct libmerc_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.packet_filter_cfg = argv[3];
    if (strcmp(argv[4], "-")) { cfg.resources = argv[4]; cfg.do_analysis = 1; }
    mc = p_init(&cfg, 0);
    if (!mc) { fprintf(stderr, "mercury_init failed\n"); return 1; }
    /* warm-up: one call initialises the device path lazily */
    {
        mercury_packet_processor p = p_construct(mc);
        char o[4096];
        struct timespec ts = {1700000000, 0};
        for (size_t i = 0; i < 16 && i < npkts; i++) {
            if (analysis_entry) p_get_ac_linktype(p, pkts[i].d, pkts[i].len, &ts, linktype);
            else p_write_json_linktype(p, o, sizeof o, pkts[i].d, pkts[i].len, &ts, linktype);
        }
        p_destruct(p);
    }
    struct worker *w = calloc((size_t)threads, sizeof *w);
    pthread_barrier_init(&start_barrier, NULL, (unsigned)threads + 1);
    for (int t = 0; t < threads; t++) {
        w[t].lo = npkts * (size_t)t / (size_t)threads;
        w[t].hi = npkts * (size_t)(t + 1) / (size_t)threads;
        if (w[t].hi <= w[t].lo) { w[t].lo = 0; w[t].hi = npkts; }
        w[t].lat_cap = 1 << 20;
        w[t].lat = malloc(w[t].lat_cap * sizeof(double));
        pthread_create(&w[t].th, NULL, run, &w[t]);
    }
    pthread_barrier_wait(&start_barrier);
    const double t0 = now();
    for (int t = 0; t < threads; t++) pthread_join(w[t].th, NULL);
    const double el = now() - t0;
    unsigned long long calls = 0, hits = 0;
    size_t nl = 0;
    for (int t = 0; t < threads; t++) { calls += w[t].calls; hits += w[t].hits; nl += w[t].nlat; }
    double *all = malloc((nl + 1) * sizeof(double));
    size_t k = 0;
    for (int t = 0; t < threads; t++) { memcpy(all + k, w[t].lat, w[t].nlat * sizeof(double)); k += w[t].nlat; }
    qsort(all, nl, sizeof(double), cmp);
    const double p50 = nl ? all[nl / 2] : 0, p99 = nl ? all[(size_t)(nl * 0.99)] : 0;
    printf("{\"threads\": %d, \"entry\": \"%s\", \"calls\": %llu, \"seconds\": %.3f, \"pps\": %.1f, "
           "\"lat_us_p50\": %.2f, \"lat_us_p99\": %.2f, \"hits\": %llu, \"packets_in_pcap\": %zu}\n",
           threads, analysis_entry ? "get_analysis_context" : "write_json", calls, el, calls / el, p50, p99, hits,
           npkts);
    p_finalize(mc);
    return 0;
}
