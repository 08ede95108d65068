// mfp_analysis.h -- device-table layout of the --analysis classifier, shared
// by the host loader (mfp_classifier.cpp) and the classifier kernels
// (mfp_analysis.hip).  Internal to libmercury_amd.so.
#pragma once
#include <stdint.h>

#include "../../include/mfp.h"
#include "mfp_lctrie.hpp"

// open-addressing string table slot (fingerprint DB, known-prevalence set)
struct mfp_fp_slot {
    uint64_t hash;      // mfpc::str_hash of the string
    uint32_t id;        // entry id (0xffffffff = empty)
    uint32_t str_off;   // string in the pool, for exact verification
    uint32_t str_len;
    uint32_t pad;
};

// one fingerprint entry (fingerprint_data, analysis.h:123-218)
struct mfp_entry {
    uint32_t proc_off;      // first process in prior/proc_* arrays
    uint32_t nproc;         // P
    uint32_t malware_db;    // fingerprint_data::malware_db
    uint32_t generic_dmz;   // index of "generic dmz process" or 0xffffffff
    uint32_t mal_bits;      // bit p: process p is malware (p < 32)
    // the entry's own region of the feature table: slots [feat_base, feat_base +
    // feat_mask] (a power of two), probed by feat_slot_hash & feat_mask -- the
    // probes of packets with the same fingerprint touch the same few lines
    uint32_t feat_base, feat_mask;
    uint32_t pad;
};

// feature-table slot, keyed by (entry, kind, key) -- key is the value itself
// for ASN / port / IPv4, a str_hash for strings and IPv6 (verified)
struct mfp_feat_slot {
    uint64_t key;
    uint32_t entry;     // 0xffffffff = empty
    uint32_t kind;      // mfpc::FeatureKind
    uint32_t upd_off, upd_cnt;
    uint32_t str_off, str_len;
};

// mfp_feat_slot::upd_cnt flag: the list repeats a process index, apply it in order
#define MFP_UPD_SERIAL 0x80000000u

struct mfp_update {     // class update (naive_bayes.hpp:21-41)
    uint32_t idx, pad;
    double value;
};


// one batch's unknown-TLS sightings, per distinct fingerprint hash (the
// adaptive part of fingerprint_prevalence is decided on the host,
// mfp_prevalence.cpp, from this table)
struct mfp_seen_slot {          // the table is reset to all-ones bytes per batch
    unsigned long long hash;    // ~0 = empty
    unsigned int first;         // packet index of the first sighting (atomicMin)
    unsigned int nlast;         // ~(packet index of the last sighting) (atomicMin)
    unsigned int count_m1;      // sightings - 1 (atomicAdd from ~0)
    unsigned int pos;           // position in the distinct list (k_seen_export)
};
struct mfp_seen_tab {
    mfp_seen_slot *slots = nullptr;
    uint32_t mask = 0;          // slots - 1 (power of two)
    uint32_t *list = nullptr;   // distinct list: slot index per position
    uint32_t list_cap = 0;      // more distinct fingerprints than this: overflow
    unsigned int *counters = nullptr;   // [0] distinct, [1] overflow
};

struct mfp_classifier_dev {
    mfp_fp_slot *fp_slots = nullptr;   uint64_t fp_mask = 0;
    mfp_fp_slot *prev_slots = nullptr; uint64_t prev_mask = 0;
    mfp_entry *entry = nullptr;
    double *prior = nullptr;
    uint32_t *proc_id = nullptr;
    uint8_t *proc_mal = nullptr;
    uint32_t *proc_attr = nullptr;
    mfp_feat_slot *feat_slots = nullptr;   // per-entry regions (mfp_entry::feat_base / feat_mask)
    mfp_update *upd = nullptr;
    char *pool = nullptr;
    // pyasn.db as the reference's LC-tries (mfp_lctrie.hpp); n_* = node count, 0: no table
    mfp_lct_node *asn4_node = nullptr; mfp_lct_net4 *asn4_net = nullptr; uint32_t n_asn4 = 0;
    mfp_lct_node *asn6_node = nullptr; mfp_lct_net6 *asn6_net = nullptr; uint32_t n_asn6 = 0;
    uint32_t types_mask = 0;           // analyzable fingerprint types (fp_types)
    uint32_t max_nproc = 0;            // the largest process count of an entry (k_analyze_big when > 512)
    uint32_t enc_channel_idx = 7, faketls_idx = 9, doh_idx = 6, domain_faking_idx = 8;
    uint32_t randomized_entry[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu};   // "tls/", "tls/1/", "tls/2/" + "randomized"
    uint32_t db_tags = 0;              // bits of the archive's own attribute tags (>= MFP_ATTR_DB_FIRST)
    // classifier-agnostic attributes (check_additional_attributes_util,
    // analysis.h:555-570): encrypted_dns from doh-watchlist.txt, domain_faking
    // from domain-mappings.db (subnet_data::is_domain_faking addr.cc:707-792)
    uint32_t doh_enabled = 0, faking_enabled = 0;
    mfp_fp_slot *doh_names = nullptr; uint64_t doh_names_mask = 0;   // watchlist DNS names
    uint32_t *doh_v4 = nullptr; uint32_t n_doh_v4 = 0;               // sorted IPv4 (parse_ipv4 values)
    uint64_t *doh_v6 = nullptr; uint32_t n_doh_v6 = 0;               // sorted (hi, lo) pairs
    mfp_fp_slot *dom_slots = nullptr; uint64_t dom_mask = 0;         // mapped domain -> domain index (id)
    // domain-mapping LC-tries; a subnet's val = its dom_info index + 1; n_* = node count, 0: no table
    mfp_lct_node *dom4_node = nullptr; mfp_lct_net4 *dom4_net = nullptr; uint32_t n_dom4 = 0;
    mfp_lct_node *dom6_node = nullptr; mfp_lct_net6 *dom6_net = nullptr; uint32_t n_dom6 = 0;
    uint32_t *dom_info = nullptr;      // per prefix: [type (1 mapping, 2 exception) | count << 8, byte offset]
    uint8_t *dom_bytes = nullptr;      // mapped domain indices (uint8_t, as the reference stores them)
};
// the classifier's per-batch device words: the public counters
// (mfp_analysis_counters), then [MFP_AN_NCOUNTERS] the wave scorer's segment queue
// (+1..8: per-phase clock sums of k_analyze_wave in MFP_AN_PHASES probe builds)
#define MFP_AN_STATS_WORDS (MFP_AN_NCOUNTERS + 12)
#define MFP_DOM_MAPPING 1u
#define MFP_DOM_EXCEPTION 2u

typedef struct mfp_classifier_s mfp_classifier;

mfp_classifier *mfp_classifier_load(const char *path, const uint8_t *enc_key = nullptr);
int mfp_classifier_upload(mfp_classifier *c, int device);
void mfp_classifier_free(mfp_classifier *c);
void mfp_classifier_free_device(mfp_classifier_dev &d);
int mfp_classifier_tls_format(const mfp_classifier *c);
int mfp_classifier_quic_format(const mfp_classifier *c);
bool mfp_classifier_disabled(const mfp_classifier *c);
const char *mfp_classifier_process_name(const mfp_classifier *c, uint32_t id);
const char *mfp_classifier_attr_name(const mfp_classifier *c, uint32_t i);
int mfp_classifier_attr_count(const mfp_classifier *c);
const char *mfp_classifier_version(const mfp_classifier *c);
uint64_t mfp_classifier_device_bytes(const mfp_classifier *c);
// os_info entry k of process slot `slot` (proc_off + index); returns the count, -1 bad slot
int mfp_classifier_os_info(const mfp_classifier *c, uint32_t slot, uint32_t k, const char **name, uint64_t *prev);
void mfp_classifier_stats(const mfp_classifier *c, uint64_t out[8]);
const mfp_classifier_dev *mfp_classifier_device(const mfp_classifier *c);
mfp_classifier_dev *mfp_classifier_device_mut(mfp_classifier *c);
