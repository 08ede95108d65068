"""Scratch (private segment) use of the kernels in libmercury_amd.so, read from
the AMDGPU metadata note of every gfx950 code object embedded in the library
(the clang offload bundles of its .hip_fatbin): the classifier, QUIC and
compaction kernels use none; the lane walkers stay within their recorded
bounds.  CPU only: reads the built library, runs nothing."""
import os
import struct

import pytest

msgpack = pytest.importorskip("msgpack")

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
LIB = os.path.join(ROOT, "mercury_amd", "libmercury_amd.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(blob):
    """The amdgcn entries of every offload bundle in `blob`."""
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if triple.startswith("hipv4-amdgcn") or triple.startswith("hip-amdgcn"):
                yield triple, blob[pos + off:pos + off + size]
        pos = blob.find(MAGIC, pos + 1)


def kernel_metadata(elf):
    """amdhsa.kernels of a code object's NT_AMDGPU_METADATA note."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for k in range(shnum):
        sh = shoff + k * shentsize
        sh_type, = struct.unpack_from("<I", elf, sh + 4)
        if sh_type != 7:      # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        p = off
        while p < off + size:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            name = elf[p + 12:p + 12 + namesz].rstrip(b"\0")
            d0 = p + 12 + ((namesz + 3) & ~3)
            if name == b"AMDGPU" and ntype == 32:
                return msgpack.unpackb(elf[d0:d0 + descsz], raw=False)["amdhsa.kernels"]
            p = d0 + ((descsz + 3) & ~3)
    return []


def kernel_scratch():
    if not os.path.exists(LIB):
        pytest.skip("libmercury_amd.so not built")
    blob = open(LIB, "rb").read()
    kernels = {}
    for triple, elf in code_objects(blob):
        assert "gfx950" in triple, triple
        for k in kernel_metadata(elf):
            kernels[k[".name"]] = k[".private_segment_fixed_size"]
    assert len(kernels) >= 15, sorted(kernels)
    return kernels


# The lane walkers of the HBM path (k_fingerprint<FAM>, k_fp_tls1) run at 3-4
# waves/SIMD with register caps below what the whole parser family wants, and
# spill; these are their current bounds (bytes per lane), so a growth shows up
# here.  FAM: 2 SSH, 4 HTTP, 16 DTLS, 63 all (the fallback lane).  k_an_features
# runs at 4 waves/SIMD with a 20-byte spill (faster than 3 waves without; round 5:
# the six feature probes' home slots loaded together, 8 -> 12 bytes, 8.55 -> 8.18 ms;
# the batch's items, records and descriptors prefetched into LDS, 12 -> 20 bytes, 8.22 -> 8.00 ms).
# The HTTP and fallback walkers carry the checks for selected protocols outside
# the path (tcp_other_matcher & co., round 4): +8 and +32 bytes.  k_fp_tls1
# (one instance per TLS format, round 4: plan length by arithmetic, uniform
# emitter) spills nothing for formats 0 and 1 and 8 bytes for format 2.
BOUNDED_SCRATCH = {"k_fp_tls1ILi0E": 0, "k_fp_tls1ILi1E": 0, "k_fp_tls1ILi2E": 8, "k_an_features": 20, "k_fingerprintILj2E": 176,
                  # the HTTP HBM lane walker (not a default bin kernel): 36 -> 64 with the 8-byte-word hex loads (round 6)
                  "k_fingerprintILj4E": 64,
                  "k_fingerprintILj16E": 496, "k_fingerprintILj63E": 944, "k_fp_ldsILb0ELj36864ELj63E": 176,
                  "k_fp_ldsILb0ELj36864ELj2E": 176,
                  # the one-parse transport parameter sort (round 4): the LDS TLS walker +12, the DTLS
                  # HBM lane walker (not a default bin kernel: DTLS runs from LDS) 444 -> 496, the fallback lane 896 -> 944
                  "k_fp_ldsILb0ELj36864ELj1E": 12,
                  # the HTTP segment walker with the header loop's windowed delimiter tests
                  # (MFP_HTTP_FAST 2, round 4): 8 bytes at its 128-VGPR cap; the HTTP HBM
                  # lane walker (not a default bin kernel) with both delimiter paths 28 -> 36;
                  # round 6: the ':' search's words kept for the value and delimiter (MFP_HTTP_WIN) 8 -> 16
                  "k_fp_segILj4E": 16}


def test_classifier_and_crypto_kernels_use_no_scratch():
    kernels = kernel_scratch()
    for name in ("k_an_features", "k_analyze_wave", "k_an_score", "k_quic", "k_classify", "k_analyze_huge"):
        assert any(name in k for k in kernels), name
    spills = {k: v for k, v in kernels.items() if v and not any(w in k for w in BOUNDED_SCRATCH)}
    assert not spills, spills


def test_walker_scratch_bounded():
    for k, v in kernel_scratch().items():
        for w, bound in BOUNDED_SCRATCH.items():
            if w in k:
                assert v <= bound, (k, v, bound)
