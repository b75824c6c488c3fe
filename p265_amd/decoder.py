"""End-to-end all-intra decoder: Annex-B bytes -> native front-end -> MI355X back-end -> YUV.

This is the call stack the reference's ``p265 -b stream.bin -o out.yuv`` (p265:7-20,
dec.py:6-64) would have if its reconstruction worked: parsing runs in
the native front-end (libp265fe.so, host threads), reconstruction + deblocking + SAO
run in the HIP back-end (libp265r.so) in batches of pictures, and the decoded
pictures come back in output (POC) order, cropped to the conformance window
(sps.py:48-53; the reference parses it but never uses it), and checked against the
stream's decoded-picture-hash SEI when present (D.3.19).

No CPU reconstruction exists on this path: a missing library or GPU raises.
"""
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import bitstream
from . import recon


@dataclass
class DecodedFrame:
    poc: int
    output_rank: int
    decode_index: int
    planes: list                 # full decoded Y, Cb, Cr (uint8, pic_width x pic_height)
    crop: tuple                  # (left, right, top, bottom) luma samples
    hash_ok: Optional[bool]      # None: stream carries no picture hash for this picture

    def cropped(self):
        l, r, t, b = self.crop
        y = self.planes[0]
        h, w = y.shape
        out = [y[t:h - b, l:w - r]]
        for c in (1, 2):
            out.append(self.planes[c][t // 2:(h - b) // 2, l // 2:(w - r) // 2])
        return out


class HashMismatch(RuntimeError):
    pass


def _batches(items, key, size):
    cur, k0 = [], None
    for it in items:
        k = key(it)
        if cur and (k != k0 or len(cur) >= size):
            yield cur
            cur = []
        cur.append(it)
        k0 = k
    if cur:
        yield cur


def decode_bytes(data: bytes, device: int = 0, batch: int = 64, threads: int = 0,
                 verify_hash: bool = True) -> List[DecodedFrame]:
    """Decode a whole stream; returns the output pictures in output order.

    Picture hashes are computed on host threads (the C hash releases the GIL) while the
    next batch decodes on the GPU."""
    pics = bitstream.decode_stream(data, threads=threads)
    frames = []
    contexts = {}
    pool = ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1))
    checks = []
    try:
        for group in _batches(list(enumerate(pics)), lambda it: it[1].params.tobytes(), batch):
            key = group[0][1].params.tobytes()
            ctx = contexts.get(key)
            if ctx is None:
                ctx = contexts[key] = recon.ReconContext(group[0][1].params, device=device)
            outs = ctx.decode([d.picture for _, d in group])
            for (i, d), planes in zip(group, outs):
                fr = DecodedFrame(poc=d.poc, output_rank=d.output_rank, decode_index=i,
                                  planes=planes, crop=tuple(int(v) for v in d.crop), hash_ok=None)
                if d.hash is not None:
                    checks.append((fr, d, [pool.submit(bitstream.plane_hash, planes[c], d.hash_type) for c in range(3)]))
                if d.output_rank >= 0:
                    frames.append(fr)
        for fr, d, futs in checks:
            fr.hash_ok = all(f.result() == d.hash[c] for c, f in enumerate(futs))
            if verify_hash and not fr.hash_ok:
                raise HashMismatch("picture %d (POC %d): decoded picture hash SEI mismatch" % (fr.decode_index, d.poc))
    finally:
        pool.shutdown(wait=True)
        for ctx in contexts.values():
            ctx.close()
    frames.sort(key=lambda f: f.output_rank)
    return frames


def write_yuv(frames: List[DecodedFrame], path: str):
    """Planar 4:2:0 8-bit YUV (I420), cropped, in output order."""
    with open(path, "wb") as f:
        for fr in frames:
            for p in fr.cropped():
                f.write(np.ascontiguousarray(p).tobytes())
