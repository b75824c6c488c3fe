"""Break down the end-to-end decoder's host/GPU time per stage (run on the GPU box)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402
from p265_amd import bitstream, recon  # noqa: E402

one = open(os.path.join(ROOT, "tests", "golden", "synth_1080p_4pic.bin"), "rb").read()
data = one * 16
t = time.perf_counter(); pics = bitstream.decode_stream(data, threads=16); print("parse %.3f s" % (time.perf_counter() - t))
ctx = recon.ReconContext(pics[0].params)
ctx.decode([pics[0].picture])
recs = [p.picture for p in pics]
for bs in (16, 64):
    t0 = time.perf_counter()
    up = run = dl = 0.0
    for i in range(0, len(recs), bs):
        a = time.perf_counter(); b = ctx.upload(recs[i:i + bs]); up += time.perf_counter() - a
        a = time.perf_counter(); ctx.run(b); ctx.sync(); run += time.perf_counter() - a
        a = time.perf_counter(); outs = ctx.download(b); dl += time.perf_counter() - a
        b.free()
    tot = time.perf_counter() - t0
    print("batch %d: total %.3f s upload %.3f run %.3f download %.3f" % (bs, tot, up, run, dl))
a = time.perf_counter()
for o, p in zip(outs, pics):
    for c in range(3):
        bitstream.plane_hash(o[c], 0)
print("md5 of %d pictures %.3f s" % (len(outs), time.perf_counter() - a))
