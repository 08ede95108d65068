// mfp_lctrie.hpp -- the reference's level-compressed trie lookup (lct_find,
// src/libmerc/lctrie/lctrie.hpp:347-386) over the tables mfp_classifier.cpp
// builds with the reference's own construction (lct_build :262-319,
// build_inner :161-248, subnet_prefix lctrie_ip.hpp:440-585).  Shared by the
// host loader (tests, the host query helper) and the classifier kernels.
//
// The lookup is restated bit for bit, including what makes it differ from a
// clean longest-prefix match:
//   * only the bases' prefix chains are searched, and subnet_prefix caps the
//     size of a prefix of 64 or more host bits at UINT64_MAX, so an IPv6 /32
//     holding exactly one /48 counts as "full" and drops out of the chain
//     (an address in the /32 outside the /48 finds nothing);
//   * the IPv6 bit extraction (ipv6_lctrie.h:140-192) for more than 64 bits
//     keeps only the low 64 bits of the extracted field;
//   * shifts by the word width or more act as the x86-64 shift instructions
//     the reference compiles to (the count taken modulo 32 or 64).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#define MFP_LCT_NIL 0xffffffffu

// trie node (lct_node_t lctrie.hpp:54-58); a leaf (branch 0) holds the net index
// of its base directly (the reference's trie->bases[index])
struct mfp_lct_node { uint32_t index; uint8_t branch, skip; uint16_t pad; };
// subnets (lct_subnet lctrie_ip.hpp:88-106): address, length, the next
// enclosing non-full prefix (MFP_LCT_NIL: none), the value (ASN, or the domain
// info index + 1)
struct mfp_lct_net4 { uint32_t addr, prefix, val, len; };
struct mfp_lct_net6 { uint64_t a0, a1; uint32_t prefix, val, len, pad; };

// x86-64 shift semantics (count modulo the operand width)
__host__ __device__ inline uint32_t lct_shl32(uint32_t x, uint32_t s) { return x << (s & 31u); }
__host__ __device__ inline uint32_t lct_shr32(uint32_t x, uint32_t s) { return x >> (s & 31u); }
__host__ __device__ inline uint64_t lct_shl64(uint64_t x, uint32_t s) { return x << (s & 63u); }
__host__ __device__ inline uint64_t lct_shr64(uint64_t x, uint32_t s) { return x >> (s & 63u); }

// EXTRACT (common.hpp:86-90)
__host__ __device__ inline uint32_t lct_ext4(uint32_t pos, uint32_t num, uint32_t s) {
    return lct_shr32(lct_shl32(s, pos), 32u - num);
}
// EXTRACT / EXTRACT_IDX for IPv6 (ipv6_lctrie.h:140-192): the low word of the
// result (the high word is always zero); EXTRACT_IDX returns 0 for num > 64
__host__ __device__ inline uint64_t lct_ext6(uint32_t pos, uint32_t num, uint64_t a0, uint64_t a1) {
    if (pos < 64u && pos + num <= 64u) return lct_shr64(lct_shl64(a0, pos), 64u - num);
    if (pos < 64u) {
        const uint32_t num1 = pos + num - 64u, num2 = num - num1;
        const uint64_t b0 = lct_shr64(lct_shl64(a0, pos), 64u - num2);
        const uint64_t b1 = lct_shr64(a1, 64u - num1);
        return lct_shl64(b0, num1) | b1;
    }
    return lct_shr64(lct_shl64(a1, pos - 64u), 64u - num);
}
__host__ __device__ inline uint64_t lct_ext6_idx(uint32_t pos, uint32_t num, uint64_t a0, uint64_t a1) {
    return num > 64u ? 0 : lct_ext6(pos, num, a0, a1);
}

// lct_find (lctrie.hpp:347-386): the matching subnet's index, or MFP_LCT_NIL
__host__ __device__ inline uint32_t lct_find4(const mfp_lct_node *node, const mfp_lct_net4 *net, uint32_t key) {
    mfp_lct_node n = node[0];
    uint32_t pos = n.skip, branch = n.branch, idx = n.index;
    while (branch != 0) {
        n = node[idx + lct_ext4(pos, branch, key)];
        pos += branch + n.skip;
        branch = n.branch;
        idx = n.index;
    }
    const mfp_lct_net4 b = net[idx];
    const uint32_t m = b.addr ^ key;
    if (lct_ext4(0, b.len, m) == 0) return idx;
    for (uint32_t p = b.prefix; p != MFP_LCT_NIL;) {
        const mfp_lct_net4 q = net[p];
        if (lct_ext4(0, q.len, m) == 0) return p;
        p = q.prefix;
    }
    return MFP_LCT_NIL;
}

__host__ __device__ inline uint32_t lct_find6(const mfp_lct_node *node, const mfp_lct_net6 *net, uint64_t k0,
                                              uint64_t k1) {
    mfp_lct_node n = node[0];
    uint32_t pos = n.skip, branch = n.branch, idx = n.index;
    while (branch != 0) {
        n = node[idx + (uint32_t)lct_ext6_idx(pos, branch, k0, k1)];
        pos += branch + n.skip;
        branch = n.branch;
        idx = n.index;
    }
    const mfp_lct_net6 b = net[idx];
    const uint64_t m0 = b.a0 ^ k0, m1 = b.a1 ^ k1;
    if (lct_ext6(0, b.len, m0, m1) == 0) return idx;
    for (uint32_t p = b.prefix; p != MFP_LCT_NIL;) {
        const mfp_lct_net6 q = net[p];
        if (lct_ext6(0, q.len, m0, m1) == 0) return p;
        p = q.prefix;
    }
    return MFP_LCT_NIL;
}
