# GPU debug: device-resident QUIC analysis for selected packets; dumps the sidecar and results
import os, sys
sys.path.insert(0, ".")
import numpy as np, torch
import mercury_amd
from mercury_amd import api
from tests import test_quic as t
arena, desc, sources = t.load()
sel = [192, 195, 4, 5]
cfg = f"select=quic;resources={os.path.join(t.GOLD, 'quic_resources.tgz')};analysis"
ctx = mercury_amd.Context(cfg, device=0, mode=api.MODE_ANALYSIS)
d_arena = torch.from_numpy(np.concatenate([arena, np.zeros(64, np.uint8)])).cuda()
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
n = len(desc)
d_rec = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
cap = 64 << 20
d_fp = torch.zeros(cap, dtype=torch.uint8, device="cuda")
d_used = torch.zeros(4, dtype=torch.int64, device="cuda")
d_out = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
ctx.process_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(), cap, d_used.data_ptr())
ctx.analyze_device(d_arena.data_ptr(), d_desc.data_ptr(), n, d_rec.data_ptr(), d_fp.data_ptr(), d_out.data_ptr())
torch.cuda.synchronize()
rec = d_rec.cpu().numpy().view(api.RECORD_DTYPE)
an = d_out.cpu().numpy().view(api.ANALYSIS_DTYPE)
fp = d_fp.cpu().numpy()
ref = {int(l.split("\t")[0]): l.split("\t") for l in __import__("gzip").open(os.path.join(t.GOLD, "quic_an.tsv.gz"), "rt")}
for i in sel:
    r = rec[i]
    o = int(r["fp_offset"]); L = int(r["fp_len"])
    sc = o + ((L + 7) & ~7) + 8
    side = bytes(fp[sc:sc + 400])
    def span(off, ln):
        return None if ln == 0xffff else side[off:off + ln]
    print(i, sources[i], "flags", int(r["flags"]), "sni", span(int(r["sni_off"]), int(r["sni_len"])), "ua", span(int(r["ua_off"]), int(r["ua_len"])),
          "alpn hdr", side[:4].hex())
    print("   dev:", int(an[i]["status"]), ctx.process_name(int(an[i]["process"])), float(an[i]["score"]), " ref:", ref[i][3:6])
ctx.close()
