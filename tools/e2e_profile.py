"""Stage breakdown of the end-to-end decoder (run on the GPU box): bitstream -> native front-end
-> upload -> HIP decode -> download -> MD5 check, on tests/golden/synth_1080p_4pic.bin x REPS.

    python tools/e2e_profile.py [reps] > gpurun_out/e2e_profile.txt
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from p265_amd import bitstream, decoder  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 16
threads = min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
one = open(os.path.join(ROOT, "tests", "golden", "synth_1080p_4pic.bin"), "rb").read()
data = one * reps
bitstream.decode_stream(one, threads=threads)
t = time.perf_counter()
pics = bitstream.decode_stream(data, threads=threads)
parse_s = time.perf_counter() - t
n_ctu = sum(len(p.picture.ctus) for p in pics)
print("stream %d pictures, %d CTUs, %.1f MB, threads %d" % (len(pics), n_ctu, len(data) / 1e6, threads))
print("parse alone: %.3f s  %.0f CTU/s" % (parse_s, n_ctu / parse_s))
decoder.decode_bytes(one)                                    # warm: contexts, kernels
rows = []
MB = 1 << 20
configs = [(8, 2, 2 * MB), (8, 3, 2 * MB), (4, 3, 2 * MB), (8, 2, 1 * MB), (16, 2, 2 * MB), (8, 4, 2 * MB),
           (12, 3, 2 * MB)]
for batch, depth, chunk in configs:
    best = None
    for rep in range(2):
        st = decoder.StageTimes()
        t = time.perf_counter()
        frames = decoder.decode_bytes(data, batch=batch, threads=threads, depth=depth, stats=st, chunk=chunk)
        dt = time.perf_counter() - t
        assert len(frames) == len(pics) and all(f.hash_ok for f in frames)
        if best is None or dt < best[0]:
            best = (dt, st)
    dt, st = best
    row = {"batch": batch, "depth": depth, "chunk_mb": chunk // MB, "e2e_s": round(dt, 4), "e2e_ctu_s": round(n_ctu / dt),
           **{k: round(v, 4) for k, v in sorted(st.items())}}
    print(json.dumps(row), flush=True)
