"""Pure-Python CPU baseline: oracle/recon_oracle.py timed on whole synthetic 1080p pictures.

TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).  The reference's own
reconstruction cannot run (decoder/cu.py:487-488 returns before it; forced, it crashes
at tu.py:677) and cannot travel to the GPU box, so its stand-in is this restatement,
which follows the same per-TB structure (residual -> neighbours -> predict -> clip)
in Python + numpy.  One process per worker (multiprocessing, started here, in a process
that never touches the GPU); each decodes one picture.

    python -m oracle.py_baseline --procs 16      # prints one JSON line
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _one(seed):
    from oracle import recon_oracle as O
    from p265_amd import records as R
    from p265_amd import synth
    params = R.make_params(pic_width=1920, pic_height=1080)
    pic = synth.make_picture(params, seed, perf=True)
    t0 = time.perf_counter()
    O.decode_picture(R.params_dict(params), pic.as_oracle_dict())
    return time.perf_counter() - t0, len(pic.ctus)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--seed", type=int, default=268)
    a = ap.parse_args()
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(a.procs) as pool:
        res = pool.map(_one, [a.seed + i for i in range(a.procs)])
    wall = time.perf_counter() - t0
    ctus = sum(n for _, n in res)
    slowest = max(t for t, _ in res)
    print(json.dumps({"value": round(ctus / slowest, 2), "unit": "CTU/s", "cores": a.procs, "kind": "port",
                      "sample": "oracle/recon_oracle.py (pure Python + numpy restatement, per-TB loop) on %d synthetic "
                                "1080p pictures (%d CTUs), one process per core; slowest worker %.1f s, wall %.1f s"
                                % (a.procs, ctus, slowest, wall)}))


if __name__ == "__main__":
    main()
