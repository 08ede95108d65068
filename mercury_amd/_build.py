"""In-tree build of libmercury_amd.so (hipcc, gfx950).  The built library is
git-ignored and travels to the GPU box with the working-tree snapshot."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmercury_amd.so")
OBJ = os.path.join(HERE, "_obj")

SOURCES = ["mfp_kernels.hip", "mfp_k_tls.hip", "mfp_k_http.hip", "mfp_k_small.hip", "mfp_k_all.hip", "mfp_analysis.hip", "mfp_compact.hip", "mfp_host.cpp", "mfp_classifier.cpp", "mfp_libmerc.cpp",
           "mfp_pcap.cpp", "mfp_json.cpp", "mfp_prevalence.cpp", "mfp_quic.hip", "mfp_reassembly.cpp",
           "mfp_pktproc.cpp"]
# the pcap -> JSON / filtered-pcap driver over the batch packet processors
# (mercury_amd/csrc/mfp_drv.cpp), linked against the library beside it
DRV_SRC = os.path.join(CSRC, "mfp_drv.cpp")
DRV = os.path.join(HERE, "mercury-amd")
ARCH = os.environ.get("MFP_OFFLOAD_ARCH", "gfx950")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _includes(path, seen=None):
    """`path` and the local headers it includes (#include "..."), transitively."""
    seen = set() if seen is None else seen
    path = os.path.normpath(path)
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path, encoding="utf-8", errors="replace") as f:
        for line in f:
            t = line.strip()
            if t.startswith("#include") and '"' in t:
                _includes(os.path.join(os.path.dirname(path), t.split('"')[1]), seen)
    return seen


def build(verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    objs, procs = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, s + ".o")
        objs.append(obj)
        if _newer(obj, sorted(_includes(src))):
            cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
                   "-Wall", "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd))
            procs.append((cmd, subprocess.Popen(cmd)))   # objects are independent: compile in parallel
    for cmd, p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    if _newer(LIB, objs):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs + ["-lz", "-lcrypto"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    if _newer(DRV, sorted(_includes(DRV_SRC)) + [LIB]):
        cmd = ["g++", "-O2", "-std=c++17", "-Wall", DRV_SRC, "-o", DRV, "-L" + HERE, "-lmercury_amd",
               "-Wl,-rpath,$ORIGIN", "-lpthread"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
