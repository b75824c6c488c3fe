import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import recon_oracle as O
from p265_amd import recon, synth, frontend
from p265_amd import records as R
log = open("gpurun_out/dbg.log", "a")
def say(*a):
    print(*a, file=log, flush=True); print(*a, flush=True)
cases = []
p2, pic2 = synth.c2_picture(); cases.append(("c2", p2, [pic2]))
params, pics = frontend.pictures_from_frontend_npz("tests/golden/sanity_frontend.npz"); cases.append(("sanity", params, pics))
for name, prm, pl in cases:
    say("case", name, "start")
    t = time.time()
    with recon.ReconContext(prm) as ctx:
        outs, recs = ctx.decode(pl, with_recon=True)
    say("case", name, "decoded in", time.time() - t)
    ok = True
    for i, p in enumerate(pl):
        rr, oo = O.decode_picture(R.params_dict(prm), p.as_oracle_dict())
        for c in range(3):
            if not np.array_equal(recs[i][c], rr[c]):
                bad = np.argwhere(recs[i][c] != rr[c]); ok = False
                say("  recon mismatch pic", i, "c", c, "n", len(bad), "first", bad[:3].tolist(), recs[i][c][tuple(bad[0])], rr[c][tuple(bad[0])])
            if not np.array_equal(outs[i][c], oo[c]):
                ok = False; say("  sao mismatch pic", i, "c", c)
    say("case", name, "ok" if ok else "MISMATCH")
