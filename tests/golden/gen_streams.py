"""Generate the committed synthetic bitstream fixtures (run once; outputs are data).

    python tests/golden/gen_streams.py

* synth_1080p_4pic.bin -- 4 all-intra IDR pictures, 1920x1080, CTB 64, QP 32, with the
  sanity.bin statistics of SURVEY.md §8(d) (luma TB area mix ~23/33/25/19 % for
  4/8/16/32 vs 26/31/26/17 % measured, ~300 B/CTU vs 316), SAO, deblocking on.  Used by
  bench.py's front-end / end-to-end legs (config C3 from real bytes).
* synth_4k_tiles.bin -- config C5 from a real bitstream: 3840x2160, 2x2 uniform tiles,
  2 pictures, loop filters not across tiles, SAO.
* synth_main10.bin -- Main 10: 416x240, BitDepth 10, 3 IDR pictures, CTB 64, cu_qp_delta (QpY
  down to -QpBdOffsetY), PCM at 9 / 8 bits, SAO offsets up to cMax 31, deblocking with per-slice
  overrides over two slices; MD5 over 16-bit little-endian samples.
Each picture is followed by a decoded-picture-hash SEI (MD5) of the C oracle's decode of
the generator's records, so any decode of these files is self-checking.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import streamgen  # noqa: E402
from oracle import c_oracle  # noqa: E402

STATS = dict(ctb_log2=6, min_cb_log2=3, max_tb_log2=5, max_th_depth=1, init_qp=26, slice_qp_delta=6,
             split_prob={6: 0.98, 5: 0.8, 4: 0.55, 3: 0.0}, tf_split_prob={5: 0.2, 4: 0.3, 3: 0.2},
             nxn_prob=0.41, cbf_prob=0.82, chroma_cbf_prob=0.14, density=0.33, big_prob=0.003,
             hash_sei="md5")

FIXTURES = {
    "synth_1080p_4pic.bin": dict(seed=1080, width=1920, height=1080, frames=4, idr_period=1, **STATS),
    "synth_4k_tiles.bin": dict(seed=2160, width=3840, height=2160, frames=2, idr_period=1, tiles=(2, 2),
                               lf_across_tiles=0, **STATS),
    "synth_main10.bin": dict(seed=1010, width=416, height=240, frames=3, idr_period=1, bit_depth=10,
                             qp_delta_depth=1, pcm=(3, 4, True), deblocking="override",
                             slices=[(0, False), (12, False)], **dict(STATS, init_qp=20, slice_qp_delta=4)),
}


def planes(params, pic):
    return c_oracle.decode(params, [pic], with_recon=False)[0][1]


def main():
    meta = {}
    for name, cfg in FIXTURES.items():
        cfg = dict(cfg)
        seed = cfg.pop("seed")
        g = streamgen.StreamGen(seed, **cfg)
        data, pics = g.stream(planes_fn=planes)
        open(os.path.join(HERE, name), "wb").write(data)
        n_ctus = sum(len(p.ctus) for _, p, _ in pics)
        meta[name] = dict(bytes=len(data), pictures=len(pics), ctus=n_ctus,
                          bytes_per_ctu=round(len(data) / n_ctus, 1),
                          config={k: (v if not isinstance(v, dict) else {str(a): b for a, b in v.items()})
                                  for k, v in cfg.items()}, seed=seed)
        print(name, meta[name]["bytes"], "bytes", n_ctus, "CTUs")
    json.dump(meta, open(os.path.join(HERE, "synth_streams.json"), "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
