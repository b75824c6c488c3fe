"""Child-process checks of the cross-group (XG) row kernel, started by tests/test_a_multirank.py so that
each runs with an environment of its own (GPU_MAX_HW_QUEUES, P265R_LIB, P265R_* knobs are read when HIP
or the library initialise).  Prints one JSON line; exit 0 = the check's expected outcome.

  python tests/xg_worker.py lanes      several small XG batches side by side on 16 lanes (16 hardware
                                       queues): more cross-group workgroups in flight than fit the GPU at
                                       once, so the dispatcher places parts of chains; every run must
                                       finish (row tickets: a row's predecessor is always held by a running
                                       wave) and equal the oracle (digest after every run)
  python tests/xg_worker.py broken     with P265R_LIB = a P265R_BR_BROKEN build and P265R_TR_CHECK=1: the
                                       half-CTU publish placed one job early must be caught on every run
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from oracle import recon_oracle as O  # noqa: E402
from p265_amd import _lib, digest, frontend, recon, synth  # noqa: E402
from p265_amd import records as R  # noqa: E402


def lanes():
    from oracle import c_oracle
    params = R.make_params(pic_width=256, pic_height=1088)   # 17 CTU rows per chain: 5 of its workgroups hold rows
    distinct = [synth.make_picture(params, 1500 + s, perf=bool(s % 2)) for s in range(4)]
    want = [digest.picture_digest(r[1]) for r in c_oracle.decode(params, distinct, with_recon=False)]
    n_lanes, reps = 16, 3
    with recon.ReconContext(params) as ctx:
        n_cus = int(ctx.describe()["num_cus"])
        xg = int(os.environ.get("P265R_XG", "4"))
        per = max(1, n_cus // (2 * xg))                  # the largest batch that still runs cross-group
        ctx.set_pipeline(n_lanes)
        idx = [[(k + i) % 4 for i in range(per)] for k in range(n_lanes)]
        sets = [[distinct[j] for j in ix] for ix in idx]
        bs = [ctx.upload(p) for p in sets]
        for rep in range(reps):
            for b in bs:
                ctx.run(b)
                ctx.digest_async(b, rep)
        bad = []
        for k, (b, ix) in enumerate(zip(bs, idx)):
            got = ctx.digest_slots(b, reps)
            for rep in range(reps):
                for i, j in enumerate(ix):
                    if not np.array_equal(got[rep, i], want[j]):
                        bad.append((k, rep, i))
            b.free()
        d = ctx.describe()
    res = {"ok": not bad, "bad": bad[:8], "lanes": n_lanes, "pictures_per_batch": per, "xg": xg,
           "xg_launches": d["row_launches"]["xg"], "workgroups_per_batch": 2 * per * xg}
    print(json.dumps(res), flush=True)
    return 0 if res["ok"] and res["xg_launches"] == n_lanes * reps else 1


def broken():
    from test_gpu_parity import _component_major
    params, sp = frontend.pictures_from_frontend_npz(os.path.join(HERE, "golden", "sanity_frontend.npz"))
    pics = [_component_major(sp[0])]
    pd = R.params_dict(params)
    ref = O.decode_picture(pd, pics[0].as_oracle_dict())[1]
    outcomes = []
    for _ in range(3):
        with recon.ReconContext(params) as ctx:
            b = ctx.upload(pics)
            ctx.run(b)
            try:
                out = ctx.download(b)[0]
                outcomes.append("parity ok" if all(np.array_equal(out[c], ref[c]) for c in range(3)) else "mismatch")
            except _lib.P265RError as e:
                outcomes.append("error: %s" % e)
            b.free()
            xg = ctx.describe()["row_launches"]["xg"]
    res = {"lib": os.path.basename(_lib.LIB_PATH), "outcomes": outcomes, "xg_launches": xg}
    print(json.dumps(res), flush=True)
    return 0 if xg and all(o != "parity ok" for o in outcomes) else 1


if __name__ == "__main__":
    sys.exit({"lanes": lanes, "broken": broken}[sys.argv[1]]())
