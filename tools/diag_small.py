"""Diagnostic: decode the many-small-pictures batch of tests/test_gpu_parity.py and list which
pictures differ from the oracle, and where (first differing sample of the first bad picture)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import recon_oracle as O  # noqa: E402
from p265_amd import records as R, recon, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1200
params = R.make_params(pic_width=64, pic_height=128, ctb_log2_size=5)
seeds = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [500, 501, 502, 503, 504]
uniq = [synth.make_picture(params, s, perf=False) for s in seeds]
pics = [uniq[i % len(uniq)] for i in range(n)]
with recon.ReconContext(params) as ctx:
    outs = ctx.decode(pics)
pd = R.params_dict(params)
refs = [O.decode_picture(pd, u.as_oracle_dict())[1] for u in uniq]
bad = []
for i in range(n):
    for c in range(3):
        if not np.array_equal(outs[i][c], refs[i % len(uniq)][c]):
            bad.append((i, c))
print("pictures:", n, "bad (pic, comp):", len(bad), bad[:20])
if bad:
    i, c = bad[0]
    d = np.argwhere(outs[i][c] != refs[i % len(uniq)][c])
    print("first bad picture", i, "comp", c, "uniq", i % len(uniq), "n diff", len(d), "first (y, x)", d[:5].tolist())
    print("bad pictures by uniq:", sorted(set(b[0] % 5 for b in bad)), "min/max pic", min(b[0] for b in bad), max(b[0] for b in bad))
