// mfp_pcap.cpp -- host ingest into batch arenas: the
// classic-pcap reader and the TPACKET_V3 ring-block walk.  Host only.
//
// The pcap reader follows pcap_file_open / pcap_file_read_packet
// (src/pcap_file_io.c:106-254, 393-468) with batches as output:
//   * global header: magic a1b2c3d4 (native order) or d4c3b2a1 (swapped);
//     pcap-ng and every other magic are refused, as are link types other than
//     Ethernet, PPP, raw IP, Linux SLL/SLL2 and 0 (BSD loopback);
//   * a swapped file's link type is htons() applied to the 32-bit field
//     (pcap_file_io.c:236), so only its first two bytes count, swapped -- the
//     reference's behaviour, kept;
//   * a record longer than BUFLEN (65536) yields its first 65536 bytes and the
//     rest is skipped (pcap_file_io.c:432-456);
//   * a record whose data is cut short ends the file with an error; a partial
//     record header is the end of the file (fread returns 0 items).
// Timestamps are reported as tv_sec * 1e9 + tv_usec * 1000 ns
// (packet_info_init_from_pkthdr, pcap_file_io.c:462-468).
#include <linux/if_packet.h>
#include <sys/mman.h>
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/mfp.h"
#include "mfp_internal.h"

namespace {
constexpr uint32_t kMagic = 0xa1b2c3d4u, kCigam = 0xd4c3b2a1u, kPcapNg = 0x0a0d0d0au;
constexpr uint32_t kBufLen = 65536;   // BUFLEN, pcap_file_io.c:391
constexpr size_t kSlack = 16;         // readable zero bytes after the last packet (include/mfp.h)

uint32_t rd32(const uint8_t *p, bool swap) {
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}
}  // namespace

struct mfp_pcap_s {
    FILE *f = nullptr;
    bool swap = false;
    uint32_t linktype = 0;
    // the file is read in large blocks into buf (two small freads per packet,
    // each taking the stream's lock, cost more than the copy); [pos, end) unread
    std::vector<uint8_t> buf;
    const uint8_t *data = nullptr;       // the unread bytes: buf, or the mapped file
    size_t pos = 0, end = 0;
    bool eof = false;
    void *map = nullptr;                 // a regular file is mapped whole (no copy through a buffer)
    size_t map_len = 0;
    // at least `need` unread bytes, unless the file ends first
    bool avail(size_t need) {
        if (map) return end - pos >= need;
        while (end - pos < need && !eof) {
            if (pos) { memmove(buf.data(), buf.data() + pos, end - pos); end -= pos; pos = 0; }
            const size_t got = fread(buf.data() + end, 1, buf.size() - end, f);
            if (got == 0) eof = true;
            end += got;
        }
        return end - pos >= need;
    }
    bool try_map() {
        struct stat st;
        if (fstat(fileno(f), &st) != 0 || !S_ISREG(st.st_mode) || st.st_size <= 0) return false;
        void *m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fileno(f), 0);
        if (m == MAP_FAILED) return false;
        (void)madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
        map = m;
        map_len = (size_t)st.st_size;
        data = (const uint8_t *)m;
        end = map_len;
        return true;
    }
    // skip k bytes of the file: what is buffered, then the rest by seeking
    bool skip(size_t k) {
        if (map) { pos += std::min(k, end - pos); return true; }   // (fseek past the end succeeds too)
        const size_t b = std::min(k, end - pos);
        pos += b;
        k -= b;
        return k == 0 || fseek(f, (long)k, SEEK_CUR) == 0;
    }
    bool have_hdr = false;               // record header read, its data not yet taken
    uint32_t ts_sec = 0, ts_usec = 0, incl = 0;
    bool done = false, failed = false;
};

extern "C" MFP_EXPORT void mfp_pcap_close(mfp_pcap p) {
    if (!p) return;
    if (p->map) munmap(p->map, p->map_len);
    if (p->f) fclose(p->f);
    delete p;
}

extern "C" MFP_EXPORT mfp_pcap mfp_pcap_open(const char *path) {
    if (!path) { mfp_set_error("null path"); return nullptr; }
    FILE *f = fopen(path, "rb");
    if (!f) { mfp_set_error("%s: error opening read file %s", strerror(errno), path); return nullptr; }
    auto *p = new mfp_pcap_s;
    p->f = f;
    if (!p->try_map()) {
        p->buf.resize(8u << 20);   // > BUFLEN + a record header
        p->data = p->buf.data();
    }
    uint8_t h[24];
    if (!p->avail(sizeof h)) {
        mfp_set_error("could not read PCAP file header");
        mfp_pcap_close(p);
        return nullptr;
    }
    memcpy(h, p->data + p->pos, sizeof h);
    p->pos += sizeof h;
    uint32_t magic;
    memcpy(&magic, h, 4);
    if (magic == kMagic || magic == kCigam) {
        p->swap = magic == kCigam;
    } else {
        if (magic == kPcapNg) mfp_set_error("file %s: pcap-ng format is unsupported", path);
        else mfp_set_error("file %s not in pcap format (file header: %08x)", path, magic);
        mfp_pcap_close(p);
        return nullptr;
    }
    uint32_t network;
    memcpy(&network, h + 20, 4);
    if (p->swap) network = __builtin_bswap16((uint16_t)network);   // htons() of the 32-bit field
    switch (network) {
    case 0: case 1: case 9: case 101: case 113: case 276:
        break;
    default:
        mfp_set_error("pcap file linktype (%u) unsupported", network);
        mfp_pcap_close(p);
        return nullptr;
    }
    p->linktype = network;
    return p;
}

extern "C" MFP_EXPORT int mfp_pcap_linktype(mfp_pcap p) { return p ? (int)p->linktype : -1; }

extern "C" MFP_EXPORT long long mfp_pcap_read_batch(mfp_pcap p, uint8_t *arena, size_t arena_cap, mfp_pkt_desc *desc,
                                                    size_t max_pkts, uint64_t *ts_ns, size_t *arena_used) {
    if (!p || !arena || !desc) { mfp_set_error("null argument"); return -1; }
    if (arena_used) *arena_used = 0;
    if (arena_cap < kSlack) { mfp_set_error("arena too small"); return -1; }
    size_t used = 0, n = 0;
    while (n < max_pkts && !p->done) {
        if (!p->have_hdr) {
            if (!p->avail(16)) { p->done = true; break; }   // no (whole) record header: no more data
            const uint8_t *h = p->data + p->pos;
            p->pos += 16;
            p->ts_sec = rd32(h, p->swap);
            p->ts_usec = rd32(h + 4, p->swap);
            p->incl = rd32(h + 8, p->swap);
            p->have_hdr = true;
        }
        const uint32_t take = p->incl <= kBufLen ? p->incl : kBufLen;
        if (used + take + kSlack > arena_cap) {
            if (n == 0) {
                mfp_set_error("arena of %zu bytes cannot hold a %u-byte packet", arena_cap, take);
                return -1;
            }
            break;                       // next batch starts with this record
        }
        if (take && !p->avail(take)) {
            mfp_set_error("could not read packet with caplen %u", take);
            p->done = p->failed = true;
            break;
        }
        if (take) memcpy(arena + used, p->data + p->pos, take);
        p->pos += take;
        if (p->incl > take && !p->skip(p->incl - take)) {
            mfp_set_error("could not advance file pointer");
            p->done = p->failed = true;  // the truncated packet itself is still delivered
        }
        desc[n].offset = used;
        desc[n].caplen = take;
        desc[n].linktype = (uint16_t)p->linktype;
        desc[n].flags = 0;
        if (ts_ns) ts_ns[n] = (uint64_t)p->ts_sec * 1000000000ull + (uint64_t)p->ts_usec * 1000ull;
        used += take;
        n++;
        p->have_hdr = false;
    }
    memset(arena + used, 0, kSlack);
    if (arena_used) *arena_used = used;
    if (n == 0 && p->failed) return -1;
    return (long long)n;
}

// process_all_packets_in_block (src/af_packet_v3.c:174-210): the block's
// packets become descriptors over the ring memory itself -- no copy; the
// caller registers (or maps) the ring and passes it as the arena.  caplen is
// tp_snaplen and the link type Ethernet (packet_info's default, pkt_proc.hpp:18).
extern "C" MFP_EXPORT long long mfp_tpacket3_block(const uint8_t *arena_base, const uint8_t *block, size_t block_len,
                                                   mfp_pkt_desc *desc, size_t max_pkts, uint64_t *ts_ns) {
    if (!arena_base || !block || !desc || block < arena_base) { mfp_set_error("bad argument"); return -1; }
    if (block_len < sizeof(tpacket_block_desc)) { mfp_set_error("block shorter than its descriptor"); return -1; }
    tpacket_block_desc bd;
    memcpy(&bd, block, sizeof bd);
    const uint32_t num = bd.hdr.bh1.num_pkts;
    if (num > max_pkts) { mfp_set_error("block holds %u packets, room for %zu", num, max_pkts); return -1; }
    size_t off = bd.hdr.bh1.offset_to_first_pkt;
    for (uint32_t i = 0; i < num; i++) {
        tpacket3_hdr h;
        if (off + sizeof h > block_len) { mfp_set_error("packet %u header outside the block", i); return -1; }
        memcpy(&h, block + off, sizeof h);
        if (off + h.tp_mac + (size_t)h.tp_snaplen > block_len) {
            mfp_set_error("packet %u data outside the block", i);
            return -1;
        }
        desc[i].offset = (uint64_t)(block + off + h.tp_mac - arena_base);
        desc[i].caplen = h.tp_snaplen;
        desc[i].linktype = 1;
        desc[i].flags = 0;
        if (ts_ns) ts_ns[i] = (uint64_t)h.tp_sec * 1000000000ull + h.tp_nsec;
        off += h.tp_next_offset;
    }
    return (long long)num;
}
