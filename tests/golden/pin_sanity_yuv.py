#!/usr/bin/env python3
"""Pin the decoded YUV of sanity.bin (config C1) in tests/golden/sanity_frontend.json.

For each definition of oracle/dump.py (conformant = recon -> deblocking -> SAO; recon_sao =
SURVEY.md §0.7's pre-deblocking recon + SAO; recon = the in-loop filter input) the SHA-256
of the 3-frame I420 output is computed four ways -- pure-Python and C oracle, on records
parsed from the bytes by the native front-end and on the committed capture of the
reference's own front-end -- which must all agree before the hash is written.  The GPU
tests then pin the HIP path to the same hashes, so the oracle and the kernels cannot drift
together unnoticed.

    python tests/golden/pin_sanity_yuv.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import dump  # noqa: E402


def main():
    meta_path = os.path.join(HERE, "sanity_frontend.json")
    meta = json.load(open(meta_path))
    pins = {}
    for d in dump.DEFINITIONS:
        got = {(impl, src): dump.dump(bitstream=os.path.join(HERE, "sanity.bin") if src == "bitstream" else None,
                                      records=os.path.join(HERE, "sanity_frontend.npz") if src == "records" else None,
                                      definition=d, impl=impl)["sha256"]
               for impl in ("py", "c") for src in ("bitstream", "records")}
        if len(set(got.values())) != 1:
            raise SystemExit("oracles disagree on %s: %s" % (d, got))
        pins[d] = next(iter(got.values()))
        print(d, pins[d])
    meta["decoded_yuv_sha256"] = pins
    meta["decoded_yuv"] = ("3 frames 352x288 I420 in output order; conformant = recon -> deblocking -> SAO, recon_sao = "
                           "recon -> SAO (deblocking off, SURVEY §0.7), recon = in-loop filter input; computed by "
                           "tests/golden/pin_sanity_yuv.py (oracle/dump.py, py and C oracles agree)")
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
