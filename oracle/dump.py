"""C1 ("sanity.bin on the pure-Python CPU path, dump YUV (golden, no GPU)"): decode a stream
on the CPU with the oracle and write the decoded pictures as I420 YUV.

TEST INFRASTRUCTURE ONLY -- the CPU restatement of what the reference's CLI
(``p265 -b sanity.bin -o out.yuv``, /root/reference/p265:7-20) was meant to do: its ``-o``
is declared (p265:9) and never written, and its reconstruction is dead (decoder/cu.py:487-488),
so the golden YUV is this oracle's.  Records come either from the native front-end parsing
the bitstream (``-b``) or from the committed capture of the reference's own Python
front-end (``--records tests/golden/sanity_frontend.npz``; pinned by its 95 golden traces).

Definitions (``--definition``):
  conformant  reconstruction -> deblocking (8.7.2) -> SAO (8.7.3): the decoded picture;
  recon_sao   reconstruction -> SAO with deblocking off: SURVEY.md §0.7's "pre-deblocking
              recon + SAO" parity definition for sanity.bin;
  recon       the reconstruction alone (the in-loop filter input, what
              Cu.get_reconstructed_sample serves, cu.py:617-632).
``--impl py`` is the pure-Python + numpy restatement (oracle/recon_oracle.py), ``c`` its
scalar C twin (oracle/recon_oracle.c); both must produce the same bytes.

    python -m oracle.dump -b tests/golden/sanity.bin -o /tmp/sanity.yuv
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

DEFINITIONS = ("conformant", "recon_sao", "recon")


def _without_deblocking(pic):
    from p265_amd import records as R
    ctus = pic.ctus.copy()
    ctus["flags"] &= np.uint8(0xff & ~R.CTU_DEBLOCK)
    ctus["deblock_offsets"] = 0
    return R.Picture(ctus=ctus, tbs=pic.tbs, coef=pic.coef, nofilter=pic.nofilter, meta=dict(pic.meta))


def load_pictures(bitstream=None, records=None):
    """-> [(params, Picture, crop)] in output order."""
    if records:
        from p265_amd import frontend
        params, pics = frontend.pictures_from_frontend_npz(records)
        return [(params, p, (0, 0, 0, 0)) for p in pics]          # sanity.bin: no conformance window
    from p265_amd import bitstream as B
    from p265_amd.decoder import OutputQueue
    q, out = OutputQueue(), []
    for d in B.decode_stream(open(bitstream, "rb").read()):
        out += q.push(d, d.cvs_id, d.poc, d.max_num_reorder, d.output_flag)
    out += q.flush()
    return [(d.params, d.picture, tuple(int(v) for v in d.crop)) for d in out]


def decode_planes(params, pic, definition, impl):
    from p265_amd import records as R
    if definition == "recon_sao":
        pic = _without_deblocking(pic)
    if impl == "c":
        from oracle import c_oracle
        rec, out = c_oracle.decode(params, [pic], threads=1, with_recon=True)[0]
    else:
        from oracle import recon_oracle as O
        rec, out = O.decode_picture(R.params_dict(params), pic.as_oracle_dict())
    planes = rec if definition == "recon" else out
    return [np.asarray(p, np.uint8) for p in planes]


def i420(planes, crop):
    l, r, t, b = crop
    h, w = planes[0].shape
    parts = [planes[0][t:h - b, l:w - r]] + [planes[c][t // 2:(h - b) // 2, l // 2:(w - r) // 2] for c in (1, 2)]
    return b"".join(np.ascontiguousarray(p).tobytes() for p in parts)


def dump(bitstream=None, records=None, output=None, definition="conformant", impl="py"):
    """Decode and (optionally) write the YUV; returns {"sha256", "frames", "bytes"}."""
    h = hashlib.sha256()
    n = size = 0
    f = open(output, "wb") if output else None
    try:
        for params, pic, crop in load_pictures(bitstream, records):
            data = i420(decode_planes(params, pic, definition, impl), crop)
            h.update(data)
            if f:
                f.write(data)
            n += 1
            size += len(data)
    finally:
        if f:
            f.close()
    return {"sha256": h.hexdigest(), "frames": n, "bytes": size, "definition": definition, "impl": impl}


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("-b", "--bitstream")
    ap.add_argument("--records", help="committed front-end capture (.npz) instead of parsing -b")
    ap.add_argument("-o", "--output")
    ap.add_argument("--definition", choices=DEFINITIONS, default="conformant")
    ap.add_argument("--impl", choices=("py", "c"), default="py")
    a = ap.parse_args()
    if not (a.bitstream or a.records):
        ap.error("-b or --records is required")
    print(json.dumps(dump(a.bitstream, a.records, a.output, a.definition, a.impl)))


if __name__ == "__main__":
    main()
