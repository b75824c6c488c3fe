"""Config C1: the decoded YUV of sanity.bin, pinned (CPU only).

tests/golden/sanity_frontend.json holds the SHA-256 of the 3-frame I420 output for each
definition of oracle/dump.py (tests/golden/pin_sanity_yuv.py).  Both oracles, fed by the
native front-end's parse of the bytes and by the committed capture of the reference's own
front-end, must reproduce them; the C1 dump CLI must write a file with that hash.  The HIP
path is pinned to the same hashes in tests/test_gpu_parity.py::test_sanity_bin_yuv_pinned.
"""
import hashlib
import json
import os
import subprocess
import sys

import pytest

from oracle import dump

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PINS = json.load(open(os.path.join(GOLDEN, "sanity_frontend.json")))["decoded_yuv_sha256"]


@pytest.mark.parametrize("definition", dump.DEFINITIONS)
@pytest.mark.parametrize("impl", ["py", "c"])
@pytest.mark.parametrize("source", ["bitstream", "records"])
def test_oracles_reproduce_the_pinned_yuv(definition, impl, source):
    kw = {"bitstream": os.path.join(GOLDEN, "sanity.bin")} if source == "bitstream" else \
         {"records": os.path.join(GOLDEN, "sanity_frontend.npz")}
    got = dump.dump(definition=definition, impl=impl, **kw)
    assert got["frames"] == 3 and got["bytes"] == 3 * 352 * 288 * 3 // 2
    assert got["sha256"] == PINS[definition]


def test_pins_distinguish_the_definitions():
    assert len(set(PINS.values())) == 3


def test_c1_dump_cli_writes_the_pinned_file(tmp_path):
    out = tmp_path / "sanity.yuv"
    r = subprocess.run([sys.executable, "-m", "oracle.dump", "-b", os.path.join(GOLDEN, "sanity.bin"), "-o", str(out)],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["sha256"] == PINS["conformant"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == PINS["conformant"]
