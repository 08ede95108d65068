import collections, sys
sys.path.insert(0, ".")
from tests import test_quic as t
arena, desc, sources = t.load()
rec, fps = t.run_gpu(arena, desc, t.MANIFEST["configs"]["q0"])
bad = t.compare(rec, fps, t.load_ref("q0"), sources)
c = collections.Counter(b[1].split(":")[0] if not b[1].startswith("synth:random") else "synth:random" for b in bad)
print(c)
for b in bad:
    if b[1].startswith("synth:") and not b[1].startswith("synth:random"): print(b)
print([b for b in bad if b[1].startswith("synth:random")][:10])
