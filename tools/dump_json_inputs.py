"""GPU box: the JSON writer's inputs for a CPU-side profile of
mfp_write_json_batch_analysis -- 60 000 packets of bench.py's mixed workload
(the config-4 templates), their records, fingerprints, analysis records and
attribute probabilities from one --analysis context (SURVEY archive) --
saved to gpurun_out/<tag>/json_inputs.npz (compressed, under gpurun's merge cap).
    python tools/dump_json_inputs.py <outdir>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import mercury_amd  # noqa: E402
from tests import synth, synth_db  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
a, d = synth.batch(60_000, seed=bench.TEMPLATE_SEED["mixed"], workload="mixed", n_templates=bench.N_TEMPLATES)
res = synth_db.build_survey()
ctx = mercury_amd.Context(f"select={bench.CONTRACT};resources={res};analysis", device=0)
rec, fp, an, ap = ctx.process_host_analysis(a, d, attr_prob=True)
np.savez_compressed(os.path.join(out, "json_inputs.npz"), arena=a, desc=d, rec=rec,
                    fp=np.frombuffer(fp, np.uint8), an=an, ap=ap)
print("saved", len(d), "packets")
