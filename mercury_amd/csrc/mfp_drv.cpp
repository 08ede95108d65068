// mfp_drv.cpp -- `mercury-amd`: the pcap-file paths of the `mercury` binary
// (src/pcap_reader.c, src/pcap_file_io.c:470-531) over the batch packet
// processors: every packet of the file goes through pkt_proc::apply() one at a
// time, exactly as pcap_file_dispatch_pkt_processor drives the reference's
// processors, into
//   -f FILE   JSON records (pkt_proc_json_writer_llq's output), or
//   -w FILE   the filtered packets in pcap format (`mercury -r in -w out`,
//             pkt_proc_filter_pcap_writer_llq; src/pkt_processing.cc:35-38).
// A summary line (packets, seconds, Mpkt/s, records, bytes) goes to stderr.
//
// usage: mercury-amd -r IN.pcap (-f OUT.json | -w OUT.pcap) [-c packet_filter_cfg]
//                    [-d device] [-b batch_pkts] [-t json_threads] [-l loop_count] [-B]
// -B: hand each block read from the file to mfp_pkt_proc_apply_batch instead
//     of one apply() per packet (the AF_PACKET block form)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "../../include/mercury_amd_pkt_proc.hpp"

static void usage(const char *a0) {
    fprintf(stderr,
            "usage: %s -r IN.pcap (-f OUT.json | -w OUT.pcap) [-c packet_filter_cfg] [-d device]\n"
            "          [-b batch_pkts] [-t json_threads] [-l loop_count] [-B]\n",
            a0);
    exit(2);
}

int main(int argc, char **argv) {
    const char *in = nullptr, *json_out = nullptr, *pcap_out = nullptr;
    std::string cfg;                      // "" = the reference's default selection ("all")
    int device = 0, loops = 1;
    bool bulk = false;
    mfp_pkt_proc_opts o{};
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        auto val = [&]() -> const char * { if (i + 1 >= argc) usage(argv[0]); return argv[++i]; };
        if (a == "-r") in = val();
        else if (a == "-f") json_out = val();
        else if (a == "-w") pcap_out = val();
        else if (a == "-c") cfg = val();
        else if (a == "-d") device = atoi(val());
        else if (a == "-b") o.batch_pkts = (size_t)strtoull(val(), nullptr, 10);
        else if (a == "-t") o.json_threads = atoi(val());
        else if (a == "-l") loops = atoi(val());
        else if (a == "-B") bulk = true;
        else usage(argv[0]);
    }
    if (!in || (!json_out == !pcap_out) || loops < 1) usage(argv[0]);
    const char *out_path = json_out ? json_out : pcap_out;
    FILE *out = strcmp(out_path, "-") == 0 ? stdout : fopen(out_path, "wb");
    if (!out) { perror(out_path); return 1; }
    static char obuf[1 << 22];
    setvbuf(out, obuf, _IOFBF, sizeof obuf);
    mfp_context ctx = mfp_init(cfg.c_str(), device, MFP_MODE_WRITE_JSON);
    if (!ctx) { fprintf(stderr, "mercury-amd: %s\n", mfp_last_error()); return 1; }
    if (pcap_out && !mercury_amd::write_pcap_header(out)) { perror(out_path); return 1; }

    int rc = 0;
    uint64_t pkts = 0, st[MFP_PKT_PROC_NSTATS] = {};
    double secs = 0, read_s = 0;
    try {
        mercury_amd::gpu_batch_proc *proc;   // (bulk: its handle, through mfp_pkt_proc_apply_batch)
        if (json_out) proc = new mercury_amd::pkt_proc_gpu_json_writer(ctx, out, &o);
        else proc = new mercury_amd::pkt_proc_gpu_filter_pcap_writer(ctx, out, &o);
        // the file is read in blocks (mfp_pcap_read_batch: the reference's
        // pcap_file_read_packet semantics, BUFLEN truncation included) and
        // each packet is handed to apply() on its own
        const size_t max_pkts = 65536, cap = (size_t)64 << 20;
        std::vector<uint8_t> arena(cap + 64);
        std::vector<mfp_pkt_desc> desc(max_pkts);
        std::vector<uint64_t> ts(max_pkts);
        const auto t0 = std::chrono::steady_clock::now();
        for (int l = 0; l < loops && rc == 0; l++) {
            mfp_pcap pc = mfp_pcap_open(in);
            if (!pc) { fprintf(stderr, "mercury-amd: %s\n", mfp_last_error()); rc = 1; break; }
            for (;;) {
                size_t used = 0;
                const auto tr = std::chrono::steady_clock::now();
                const long long n = mfp_pcap_read_batch(pc, arena.data(), cap, desc.data(), max_pkts, ts.data(), &used);
                read_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - tr).count();
                if (n < 0) { fprintf(stderr, "mercury-amd: %s\n", mfp_last_error()); rc = 1; break; }
                if (n == 0) break;
                if (bulk) {
                    proc->apply_batch(arena.data(), desc.data(), (size_t)n, ts.data());
                    pkts += (uint64_t)n;
                    continue;
                }
                for (long long i = 0; i < n; i++) {
                    packet_info pi;
                    pi.ts.tv_sec = (time_t)(ts[i] / 1000000000ull);
                    pi.ts.tv_nsec = (long)(ts[i] % 1000000000ull);
                    pi.caplen = pi.len = desc[i].caplen;
                    pi.linktype = desc[i].linktype;
                    proc->apply(&pi, arena.data() + desc[i].offset);
                }
                pkts += (uint64_t)n;
            }
            mfp_pcap_close(pc);
        }
        proc->finalize();
        secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        proc->stats(st);
        delete proc;
    } catch (const std::exception &e) {
        fprintf(stderr, "%s\n", e.what());
        rc = 1;
    }
    if (out != stdout) fclose(out);
    else fflush(out);
    mfp_finalize(ctx);
    fprintf(stderr,
            "{\"packets\": %llu, \"seconds\": %.6f, \"mpps\": %.3f, \"records\": %llu, \"bytes_out\": %llu, "
            "\"batches\": %llu, \"device_s\": %.6f, \"writer_s\": %.6f, \"read_s\": %.6f, \"skipped\": %llu}\n",
            (unsigned long long)pkts, secs, secs > 0 ? pkts / secs / 1e6 : 0.0, (unsigned long long)st[2],
            (unsigned long long)st[3], (unsigned long long)st[1], st[4] / 1e9, st[5] / 1e9, read_s, (unsigned long long)st[6]);
    return rc;
}
