"""Command line decoder, mirroring the reference's ``p265`` script (p265:7-20):

    python -m p265_amd.dec -b sanity.bin -o out.yuv

``-b/--bitstream`` and ``-o/--output`` keep the reference's meaning (its ``-o`` is
declared but never written, p265:9); ``--skip-syntax-dump`` is accepted for command
line compatibility (this decoder writes no syntax logs).  Parsing runs on host threads
(libp265fe.so), reconstruction on the MI355X (libp265r.so); the file is streamed
(bounded memory) and the YUV written in output order as pictures complete.
"""
import argparse
import sys
import time

from . import decoder


def parse_cmd(argv=None):
    ap = argparse.ArgumentParser(prog="p265_amd.dec")
    ap.add_argument("-b", "--bitstream", required=True, help="The h.265 bitstream to be decoded.")
    ap.add_argument("-o", "--output", help="The reconstructed YUV output (I420, cropped, output order).")
    ap.add_argument("--skip-syntax-dump", type=int, default=0, help="Accepted for compatibility; no effect.")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--threads", type=int, default=0, help="front-end parsing threads (0 = this process's CPU share, <= 16)")
    ap.add_argument("--batch", type=int, default=decoder.DEFAULT_BATCH, help="pictures per GPU batch")
    ap.add_argument("--depth", type=int, default=decoder.DEFAULT_DEPTH, help="GPU batches in flight (one warm context each)")
    ap.add_argument("--no-verify", action="store_true", help="do not fail on a decoded picture hash mismatch")
    return ap.parse_args(argv)


def main(argv=None):
    a = parse_cmd(argv)
    t0 = time.time()
    st = decoder.decode_file(a.bitstream, a.output, device=a.device, batch=a.batch, threads=a.threads,
                             depth=a.depth, verify_hash=not a.no_verify)
    dt = time.time() - t0
    print("decoded %d pictures in %.3f s; picture hash SEI checked %d, mismatched %d"
          % (st["pictures"], dt, st["hash_checked"], st["hash_mismatch"]))
    return 1 if st["hash_mismatch"] else 0


if __name__ == "__main__":
    sys.exit(main())
