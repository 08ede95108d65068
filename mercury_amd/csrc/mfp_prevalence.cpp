// mfp_prevalence.cpp -- the adaptive part of the classifier's
// fingerprint_prevalence (analysis.h:362-421): an LRU of at most `capacity`
// unknown TLS fingerprints (the reference: 100000, analysis.h:433), updated on
// every sighting, in stream order (perform_analysis_common analysis.h:1043-
// 1083):
//   in the set      -> status unlabeled, moved to the front;
//   not in the set  -> status randomized, inserted at the front, the least
//                      recently used one evicted when the set is full.
// Identity is the fingerprint string's 64-bit hash (mfpc::str_hash).
//
// The device finds a batch's sightings; this host object decides them, in
// order, for one context or for the shards of one stream (shard order), so the
// decision is the single-thread reference's.  Two ways in:
//   * distinct: the batch's distinct fingerprints with their first and last
//     sighting; exact whenever no eviction can happen inside the batch (the set
//     plus the batch's new fingerprints fit the capacity): the first sighting
//     of a fingerprint not in the set is randomized, everything else unlabeled,
//     and the recency order afterwards is the order of the last sightings;
//   * sequence: every sighting in stream order, simulated one by one (used
//     when the distinct form cannot be exact).  Long sequences are cut into
//     chunks decided in parallel: an LRU's content at any point is the
//     `capacity` most recent distinct keys, so each chunk's starting set is
//     rebuilt from the sightings before it (lru_at) and the decisions are the
//     single pass's.
#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <unordered_set>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/mfp.h"
#include "mfp_internal.h"

namespace {

// LRU over 64-bit keys: linear-probing index (keys stored in the slots,
// backward-shift deletion: no tombstones) + intrusive doubly linked list of
// nodes (node 0 is the list head sentinel; a node holds its key, its links
// and its slot, so relinking a node touches one cache line per node)
struct Lru {
    struct Slot { uint64_t key; uint32_t node; uint32_t pad; };   // node 0: empty
    struct Node { uint64_t key; uint32_t prev, next, where, pad; };
    uint32_t cap;
    std::vector<Node> nd;
    std::vector<Slot> slot;
    uint64_t mask;
    uint32_t size = 0;

    explicit Lru(uint32_t c) : cap(c ? c : 1) {
        nd.assign((size_t)cap + 1, Node{0, 0, 0, 0, 0});
        uint64_t s = 16;
        while (s < 2ull * cap + 16) s <<= 1;
        slot.assign(s, Slot{0, 0, 0});
        mask = s - 1;
    }
    static uint64_t mix(uint64_t x) {
        x ^= x >> 31; x *= 0x7fb5d329728ea185ull; x ^= x >> 27; x *= 0x81dadef4bc2dd44dull; x ^= x >> 33;
        return x;
    }
    uint64_t home(uint64_t k) const { return mix(k) & mask; }
    void prefetch(uint64_t k) const { __builtin_prefetch(&slot[home(k)]); }
    // the accesses of a sequence, prefetching slots 8 ahead (a second stage
    // prefetching the hit's node measured slower)
    void run(const uint64_t *hash, size_t s, size_t e, uint8_t *seen) {
        for (size_t j = s; j < e; j++) {
            if (j + 8 < e) prefetch(hash[j + 8]);
            seen[j] = access(hash[j]) ? 1 : 0;
        }
    }
    // slot of k (found), or the empty slot that ends its probe
    uint64_t find(uint64_t k, bool &found) const {
        uint64_t i = home(k);
        while (true) {
            const Slot &s = slot[i];
            if (s.node == 0) { found = false; return i; }
            if (s.key == k) { found = true; return i; }
            i = (i + 1) & mask;
        }
    }
    void erase_slot(uint64_t i) {   // backward-shift deletion
        uint64_t j = i;
        while (true) {
            j = (j + 1) & mask;
            if (slot[j].node == 0) break;
            const uint64_t h = home(slot[j].key);
            // slot j's entry may move to i unless its home lies cyclically in (i, j]
            const bool stay = (i <= j) ? (h > i && h <= j) : (h > i || h <= j);
            if (!stay) {
                slot[i] = slot[j];
                nd[slot[i].node].where = (uint32_t)i;
                i = j;
            }
        }
        slot[i].node = 0;
    }
    void unlink(uint32_t n) { nd[nd[n].prev].next = nd[n].next; nd[nd[n].next].prev = nd[n].prev; }
    void push_front(uint32_t n) {
        const uint32_t f = nd[0].next;
        nd[n].next = f; nd[n].prev = 0; nd[f].prev = n; nd[0].next = n;
    }
    void push_back(uint32_t n) {
        const uint32_t b = nd[0].prev;
        nd[n].prev = b; nd[n].next = 0; nd[b].next = n; nd[0].prev = n;
    }
    bool contains(uint64_t k) const { bool f; find(k, f); return f; }
    uint32_t insert_at(uint64_t i, uint64_t k) {   // i: the empty slot find() returned
        const uint32_t n = ++size;                 // nodes 1..size are live (evictions reuse theirs)
        nd[n].key = k;
        slot[i] = Slot{k, n, 0};
        nd[n].where = (uint32_t)i;
        return n;
    }
    // fingerprint_prevalence::update (analysis.h:386-408); returns whether k
    // was in the set (the caller's contains() before the update)
    bool access(uint64_t k) {
        bool found;
        uint64_t i = find(k, found);
        if (found) {
            const uint32_t n = slot[i].node;
            if (nd[0].next != n) { unlink(n); push_front(n); }
            return true;
        }
        if (size == cap) {                         // evict the least recently used, reuse its node
            const uint32_t t = nd[0].prev;
            unlink(t);
            erase_slot(nd[t].where);
            i = find(k, found);                    // the shift may have moved k's empty slot
            nd[t].key = k;
            slot[i] = Slot{k, t, 0};
            nd[t].where = (uint32_t)i;
            push_front(t);
            return false;
        }
        push_front(insert_at(i, k));
        return false;
    }
    // set-up from a recency list: k becomes the least recently used so far
    // (callers go from most to least recent); false if present or full
    bool append_lru(uint64_t k) {
        if (size == cap) return false;
        bool found;
        const uint64_t i = find(k, found);
        if (found) return false;
        push_back(insert_at(i, k));
        return true;
    }
    // the keys from least to most recently used
    void export_keys(std::vector<uint64_t> &out) const {
        out.clear();
        for (uint32_t n = nd[0].prev; n != 0; n = nd[n].prev) out.push_back(nd[n].key);
    }
};

// The set after the accesses hash[0..end) applied to a set whose keys are
// `init` (least to most recent): an LRU holds exactly the `cap` most recently
// accessed distinct keys, in recency order, so it is rebuilt by walking back
// from end-1 (then into init) until `cap` distinct keys are found.  The walk
// over the sequence stops after `budget` entries (a prefix of mostly repeated
// hot keys): false then, and the caller takes the set another way.
bool lru_at(Lru &L, const uint64_t *hash, size_t end, const std::vector<uint64_t> &init, size_t budget) {
    const size_t stop = end > budget ? end - budget : 0;
    size_t i = end;
    for (; i-- > stop && L.size < L.cap;) L.append_lru(hash[i]);
    if (L.size < L.cap && stop > 0) return false;
    for (size_t j = init.size(); j-- > 0 && L.size < L.cap;) L.append_lru(init[j]);
    return true;
}

}  // namespace

// One object may be shared by several contexts used from several threads (the
// libmerc shim's write_json and analysis contexts; shards): every entry point
// holds its lock, as the reference guards its LRU (analysis.h:372,390)
struct mfp_prevalence_s {
    Lru lru;
    std::mutex mu;
    explicit mfp_prevalence_s(uint32_t c) : lru(c) {}
};

static bool exact_locked(mfp_prevalence p, const mfp_sighting *d, size_t u) {
    std::unordered_set<uint64_t> fresh;
    for (size_t i = 0; i < u; i++)
        if (!p->lru.contains(d[i].hash)) fresh.insert(d[i].hash);
    return (uint64_t)p->lru.size + fresh.size() <= p->lru.cap;
}

extern "C" {

MFP_EXPORT mfp_prevalence mfp_prevalence_create(uint32_t capacity) {
    if (capacity == 0) { mfp_set_error("prevalence capacity must be > 0"); return nullptr; }
    return new mfp_prevalence_s(capacity);
}

MFP_EXPORT void mfp_prevalence_destroy(mfp_prevalence p) { delete p; }

MFP_EXPORT uint64_t mfp_prevalence_size(mfp_prevalence p) {
    if (!p) return 0;
    std::lock_guard<std::mutex> lk(p->mu);
    return p->lru.size;
}

MFP_EXPORT uint32_t mfp_prevalence_capacity(mfp_prevalence p) { return p ? p->lru.cap : 0; }

MFP_EXPORT int mfp_prevalence_contains(mfp_prevalence p, uint64_t hash) {
    if (!p) return 0;
    std::lock_guard<std::mutex> lk(p->mu);
    return p->lru.contains(hash) ? 1 : 0;
}

MFP_EXPORT long long mfp_prevalence_keys(mfp_prevalence p, uint64_t *out, size_t cap) {
    if (!p) return -1;
    std::lock_guard<std::mutex> lk(p->mu);
    std::vector<uint64_t> k;
    p->lru.export_keys(k);
    const size_t m = k.size() < cap ? k.size() : cap;
    if (out && m) memcpy(out, k.data(), m * sizeof(uint64_t));
    return (long long)k.size();
}

}  // extern "C"

// hash[0..m) decided against the set L, which becomes the set afterwards.
// Long sequences go in parallel chunks: chunk t decides hash[s_t..e_t) with
// its own LRU set up as the shared one would be at s_t (lru_at): the same
// decisions as one pass.  A chunk whose walk back runs past its budget (4
// chunk lengths) takes the previous chunk's finished set instead; the last
// chunk's set is the set after the whole sequence.
static void decide(Lru &L, const uint64_t *hash, size_t m, uint8_t *seen) {
    // chunks of at least 8 x capacity per thread (each chunk's starting set costs a walk back over about
    // `capacity` distinct keys); up to 16 threads, the per-GPU host share of the target machine
    // (MFP_LRU_THREADS: a lower cap, e.g. for several ranks on one host's cores)
    const unsigned hw = std::thread::hardware_concurrency();
    size_t tmax = std::min<size_t>(16, hw ? hw : 1);
    if (const char *e = getenv("MFP_LRU_THREADS")) tmax = std::max<size_t>(1, std::min<size_t>(tmax, strtoul(e, nullptr, 10)));
    size_t T = std::min<size_t>(m / (8 * (size_t)L.cap), tmax);
    if (T <= 1) {
        L.run(hash, 0, m, seen);
        return;
    }
    std::vector<uint64_t> init;
    L.export_keys(init);
    std::vector<Lru> sets(T, Lru(1));
    std::vector<uint8_t> done(T, 0);
    std::mutex dmu;
    std::condition_variable dcv;
    std::vector<std::thread> th;
    for (size_t t = 0; t < T; t++)
        th.emplace_back([&, t]() {
            const size_t s = m * t / T, e = m * (t + 1) / T;
            Lru C(L.cap);
            if (t > 0 && !lru_at(C, hash, s, init, 4 * (e - s))) {
                std::unique_lock<std::mutex> lk(dmu);
                dcv.wait(lk, [&] { return done[t - 1] != 0; });
                C = sets[t - 1];
            } else if (t == 0) {
                lru_at(C, hash, 0, init, 0);
            }
            C.run(hash, s, e, seen);
            std::lock_guard<std::mutex> lk(dmu);
            sets[t] = std::move(C);
            done[t] = 1;
            dcv.notify_all();
        });
    for (auto &x : th) x.join();
    std::swap(L, sets[T - 1]);
}

// the set whose most recent keys are recent[0..n) (most recent first), then
// the keys of `older` from its most recent down, up to the capacity
static void set_from(Lru &out, const uint64_t *recent, size_t n, const Lru &older) {
    for (size_t i = 0; i < n && out.size < out.cap; i++) out.append_lru(recent[i]);
    for (uint32_t k = older.nd[0].next; k != 0 && out.size < out.cap; k = older.nd[k].next) out.append_lru(older.nd[k].key);
}

extern "C" {

MFP_EXPORT int mfp_prevalence_resolve_sequence(mfp_prevalence p, const uint64_t *hash, size_t m, uint8_t *seen) {
    if (!p || (m && (!hash || !seen))) { mfp_set_error("mfp_prevalence_resolve_sequence: bad arguments"); return -1; }
    std::lock_guard<std::mutex> lk(p->mu);
    decide(p->lru, hash, m, seen);
    return 0;
}

// The distinct keys of hash[0..m) by their last sighting, most recent first,
// at most the capacity of p: what a walk back over this shard contributes to
// any later shard's starting set (lru_at)
MFP_EXPORT long long mfp_prevalence_summary(mfp_prevalence p, const uint64_t *hash, size_t m, uint64_t *out) {
    if (!p || (m && (!hash || !out))) { mfp_set_error("mfp_prevalence_summary: bad arguments"); return -1; }
    Lru S(p->lru.cap);
    for (size_t i = m; i-- > 0 && S.size < S.cap;) S.append_lru(hash[i]);
    long long k = 0;
    for (uint32_t n = S.nd[0].next; n != 0; n = S.nd[n].next) out[k++] = S.nd[n].key;
    return k;
}

// One shard of a stream whose earlier shards were decided elsewhere: the
// shard starts from the set that the earlier shards' summaries (prior,
// most recent shard first, each mfp_prevalence_summary) leave on top of p's
// set; hash[0..m) is decided from there.  p is not changed (see
// mfp_prevalence_advance).
MFP_EXPORT int mfp_prevalence_resolve_shard(mfp_prevalence p, const uint64_t *hash, size_t m, const uint64_t *prior,
                                            size_t nprior, uint8_t *seen) {
    if (!p || (m && (!hash || !seen)) || (nprior && !prior)) {
        mfp_set_error("mfp_prevalence_resolve_shard: bad arguments");
        return -1;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    Lru S(p->lru.cap);
    set_from(S, prior, nprior, p->lru);
    decide(S, hash, m, seen);
    return 0;
}

// The set after a whole step of shards: `recent` = every shard's summary,
// the last shard's first; p becomes that set (the same on every rank)
MFP_EXPORT int mfp_prevalence_advance(mfp_prevalence p, const uint64_t *recent, size_t n) {
    if (!p || (n && !recent)) { mfp_set_error("mfp_prevalence_advance: bad arguments"); return -1; }
    std::lock_guard<std::mutex> lk(p->mu);
    Lru S(p->lru.cap);
    set_from(S, recent, n, p->lru);
    std::swap(p->lru, S);
    return 0;
}

// Whether the distinct form is exact for these entries: no eviction can
// happen while they are applied (the set plus the fingerprints new to it fit).
// Entries may repeat a hash (the same fingerprint in several shards).
MFP_EXPORT int mfp_prevalence_distinct_exact(mfp_prevalence p, const mfp_sighting *d, size_t u) {
    if (!p || (u && !d)) return -1;
    std::lock_guard<std::mutex> lk(p->mu);
    return exact_locked(p, d, u) ? 1 : 0;
}

// Decide the first sighting of every entry and apply the entries to the set.
// `first`/`last` are positions in one stream order (for shards: the shard's
// base plus the batch index).  first_seen = 1: at that first sighting the
// fingerprint was in the set (status unlabeled); 0: randomized.  Every later
// sighting of an entry is unlabeled.  Fails with -2 (nothing applied) when
// the batch could evict: resolve the sighting sequence then.
MFP_EXPORT int mfp_prevalence_resolve_distinct(mfp_prevalence p, mfp_sighting *d, size_t u) {
    if (!p || (u && !d)) { mfp_set_error("mfp_prevalence_resolve_distinct: bad arguments"); return -1; }
    std::lock_guard<std::mutex> lk(p->mu);
    if (!exact_locked(p, d, u)) {
        mfp_set_error("mfp_prevalence_resolve_distinct: the batch can evict (set %u + new fingerprints > capacity %u); "
                      "resolve the sighting sequence instead", p->lru.size, p->lru.cap);
        return -2;
    }
    std::vector<size_t> ord(u);
    for (size_t i = 0; i < u; i++) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return d[a].first < d[b].first; });
    std::unordered_set<uint64_t> earlier;   // seen by an earlier entry of these (no eviction: stays in the set)
    for (size_t i : ord) {
        d[i].first_seen = (p->lru.contains(d[i].hash) || earlier.count(d[i].hash)) ? 1 : 0;
        earlier.insert(d[i].hash);
    }
    // recency afterwards: the order of the last sightings
    std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return d[a].last < d[b].last; });
    for (size_t i : ord) p->lru.access(d[i].hash);
    return 0;
}

}  // extern "C"
