import os, sys, time
sys.path.insert(0, os.getcwd())
from p265_amd import bitstream, recon
one = open("tests/golden/synth_1080p_4pic.bin", "rb").read()
pics = bitstream.decode_stream(one * 16, threads=16)
ctx = recon.ReconContext(pics[0].params)
for bs in (64, 16, 16, 64):
    t = time.perf_counter(); b = ctx.upload([p.picture for p in pics[:bs]]); dt = time.perf_counter() - t
    print("upload %d pictures: %.1f ms" % (bs, dt * 1e3), flush=True)
    ctx.run(b); ctx.sync()
    t = time.perf_counter(); o = ctx.download(b); print("download %d: %.1f ms" % (bs, (time.perf_counter() - t) * 1e3), flush=True)
    b.free()
