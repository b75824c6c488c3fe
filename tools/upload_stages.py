"""Upload stage times of 512 synthetic 1080p pictures (the bench's PCIe-leg batch) on the GPU box.

Needs an experiments build for the per-stage lines on stderr:
  make variant V=exp FLAGS=-DP265R_EXPERIMENTS=1
  P265R_LIB=p265_amd/libp265r_exp.so python tools/upload_stages.py
"""
import os, sys, time
sys.path.insert(0, os.getcwd())
os.environ.setdefault("P265R_UPLOAD_TIMES", "1")
from p265_amd import recon, synth
from p265_amd import records as R
params = R.make_params(pic_width=1920, pic_height=1080)
t = time.perf_counter()
u = [synth.make_picture(params, 1000 + s, perf=True) for s in range(2)]
pics = [u[i % 2] for i in range(512)]
print("synth %.1f s" % (time.perf_counter() - t), flush=True)
with recon.ReconContext(params) as ctx:
    for rep in range(3):
        t = time.perf_counter(); b = ctx.upload(pics); ctx.sync(); dt = time.perf_counter() - t
        print("upload 512: %.1f ms" % (dt * 1e3), flush=True)
        b.free()
