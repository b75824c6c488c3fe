"""GPU debugging aid: deblocking variants vs the C oracle, mismatch summary per variant."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import c_oracle
from p265_amd import recon, synth
from p265_amd import records as R


def run(label, params, pics):
    with recon.ReconContext(params) as ctx:
        outs, recs = ctx.decode(pics, with_recon=True)
    ref = c_oracle.decode(params, pics, threads=8)
    for i in range(len(pics)):
        for c in range(3):
            a, b = outs[i][c], ref[i][1][c]
            bad = np.argwhere(a != b)
            rb = int((recs[i][c] != ref[i][0][c]).sum())
            if len(bad) or rb:
                print(label, "pic", i, "c", c, "recon bad", rb, "out bad", len(bad), "first", bad[:6].tolist(),
                      [(int(a[tuple(p)]), int(b[tuple(p)])) for p in bad[:6]], flush=True)
                ys, xs = bad[:, 0], bad[:, 1]
                print("   x%8 hist", np.bincount(xs % 8, minlength=8).tolist(), "y%8 hist", np.bincount(ys % 8, minlength=8).tolist(), flush=True)
    print(label, "done", flush=True)


base = dict(pic_width=352, pic_height=288, ctb_log2_size=6)
for label, pk, mk in [
    ("dbk-only", dict(sample_adaptive_offset=0), dict(deblocking=True, sao=False)),
    ("dbk-cqp", dict(sample_adaptive_offset=0, pps_cb_qp_offset=-1, pps_cr_qp_offset=2), dict(deblocking=True, sao=False)),
    ("dbk-rand", dict(sample_adaptive_offset=0), dict(deblocking="random", sao=False)),
    ("dbk-pcm", dict(sample_adaptive_offset=0), dict(deblocking=True, sao=False, pcm_rate=0.05, bypass_rate=0.05)),
    ("dbk-sao", dict(), dict(deblocking=True)),
    ("full", dict(pps_cb_qp_offset=-1, pps_cr_qp_offset=2), dict(deblocking="random", bypass_rate=0.04, pcm_rate=0.03)),
]:
    params = R.make_params(**base, **pk)
    pics = [synth.make_picture(params, 1320, perf=False, **mk)]
    run(label, params, pics)
