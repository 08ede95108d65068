"""GPU box debugging aid: the first mismatches of the reference-pcap golden
(tests/test_gpu_parity.py) for one TLS format, expected against produced."""
import sys

sys.path.insert(0, ".")
from tests import test_gpu_parity as t  # noqa: E402

fmt = int(sys.argv[1]) if len(sys.argv) > 1 else 0
arena, desc, sources = t.load_golden()
ref = t.load_ref(fmt)
rec, fps = t.run_gpu(arena, desc, fmt)
n = 0
for i, (emit, ty, trunc, s) in enumerate(ref):
    if fps[i] != s or int(rec["fp_type"][i]) != ty:
        k = next((j for j in range(min(len(s), len(fps[i]))) if s[j] != fps[i][j]), min(len(s), len(fps[i])))
        print(i, sources[i], "type", ty, int(rec["fp_type"][i]), "len", len(s), len(fps[i]), "first diff at", k)
        print("  exp:", s[max(0, k - 40):k + 60])
        print("  got:", fps[i][max(0, k - 40):k + 60])
        n += 1
        if n >= 4:
            break
