"""HEVC all-intra bitstream generator (test infrastructure; never shipped or timed).

Writes conformant H.265 Annex-B streams from random syntax decisions with the
informative CABAC encoder of H.265 9.3.4.x (EncodeDecision / EncodeBypass /
EncodeTerminate / EncodeFlush) and, for the same decisions, the back-end records
through ``frontend.PictureBuilder`` -- i.e. what the reference's Cu.decode_leaf hook
would hand over.  The native front-end (libp265fe.so) must parse every generated
stream back into exactly those records: an encode -> decode round trip.

It covers what the reference's own parser raises on or never sees in sanity.bin
(pps.py:61-93 tiles, slice.py:177/181-189 deblocking override and entry points,
slice.py:295 end_of_subset_one_bit, nalu.py:130 SEI): tiles (uniform / explicit),
WPP, multiple and dependent slice segments, cu_qp_delta, PCM, cu_transquant_bypass,
transform skip, sign data hiding, deblocking override, slice chroma QP offsets,
conformance window, non-IDR pictures (POC) and decoded-picture-hash SEI.

Written independently of the C++ decoder (different structure: the encoder derives
contexts from its own neighbour maps), but both follow the same specification text;
the syntax that sanity.bin exercises is additionally pinned by the reference.
"""
import hashlib

import numpy as np

from p265_amd import frontend
from p265_amd import records as R

# ---------------------------------------------------------------------------------------------
# CABAC tables (H.265 Tables 9-46..9-47) and initType-0 init values (Tables 9-5..9-37)
# ---------------------------------------------------------------------------------------------
LPS = [[128, 176, 208, 240], [128, 167, 197, 227], [128, 158, 187, 216], [123, 150, 178, 205],
       [116, 142, 169, 195], [111, 135, 160, 185], [105, 128, 152, 175], [100, 122, 144, 166],
       [95, 116, 137, 158], [90, 110, 130, 150], [85, 104, 123, 142], [81, 99, 117, 135],
       [77, 94, 111, 128], [73, 89, 105, 122], [69, 85, 100, 116], [66, 80, 95, 110],
       [62, 76, 90, 104], [59, 72, 86, 99], [56, 69, 81, 94], [53, 65, 77, 89], [51, 62, 73, 85],
       [48, 59, 69, 80], [46, 56, 66, 76], [43, 53, 63, 72], [41, 50, 59, 69], [39, 48, 56, 65],
       [37, 45, 54, 62], [35, 43, 51, 59], [33, 41, 48, 56], [32, 39, 46, 53], [30, 37, 43, 50],
       [29, 35, 41, 48], [27, 33, 39, 45], [26, 31, 37, 43], [24, 30, 35, 41], [23, 28, 33, 39],
       [22, 27, 32, 37], [21, 26, 30, 35], [20, 24, 29, 33], [19, 23, 27, 31], [18, 22, 26, 30],
       [17, 21, 25, 28], [16, 20, 23, 27], [15, 19, 22, 25], [14, 18, 21, 24], [14, 17, 20, 23],
       [13, 16, 19, 22], [12, 15, 18, 21], [12, 14, 17, 20], [11, 14, 16, 19], [11, 13, 15, 18],
       [10, 12, 15, 17], [10, 12, 14, 16], [9, 11, 13, 15], [9, 11, 12, 14], [8, 10, 12, 14],
       [8, 9, 11, 13], [7, 9, 11, 12], [7, 9, 10, 12], [7, 8, 10, 11], [6, 8, 9, 11], [6, 7, 9, 10],
       [6, 7, 8, 9], [2, 2, 2, 2]]
TRANS_MPS = list(range(1, 63)) + [62, 63]
TRANS_LPS = [0, 0, 1, 2, 2, 4, 4, 5, 6, 7, 8, 9, 9, 11, 11, 12, 13, 13, 15, 15, 16, 16, 18, 18, 19, 19,
             21, 21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33, 33,
             33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63]

INIT = {
    "sao_merge": [153], "sao_type": [200], "split_cu": [139, 141, 157], "bypass": [154], "part_mode": [184],
    "prev_intra": [184], "chroma_mode": [63], "split_tf": [153, 138, 138], "cbf_luma": [111, 141],
    "cbf_chroma": [94, 138, 182, 154, 154], "qp_delta": [154, 154], "tskip": [139, 139],
    "last_x": [110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63],
    "last_y": [110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63],
    "csbf": [91, 171, 134, 141],
    "sig": [111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179,
            153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139,
            111, 136, 139, 111],
    "gt1": [140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166,
            182, 140, 227, 122, 197],
    "gt2": [138, 153, 136, 167, 152, 152],
}


def init_states(qp):
    st = {}
    q = min(max(qp, 0), 51)
    for k, vals in INIT.items():
        lst = []
        for v in vals:
            m, n = (v >> 4) * 5 - 45, ((v & 15) << 3) - 16
            pre = min(max(((m * q) >> 4) + n, 1), 126)
            mps = 0 if pre <= 63 else 1
            lst.append([pre - 64 if mps else 63 - pre, mps])
        st[k] = lst
    return st


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def bit(self, b):
        self.acc = (self.acc << 1) | (b & 1)
        self.n += 1
        if self.n == 8:
            self.out.append(self.acc)
            self.acc = 0
            self.n = 0

    def u(self, v, n):
        for i in range(n - 1, -1, -1):
            self.bit((v >> i) & 1)

    def ue(self, v):
        v += 1
        n = v.bit_length()
        self.u(0, n - 1)
        self.u(v, n)

    def se(self, v):
        self.ue(2 * v - 1 if v > 0 else -2 * v)

    def aligned(self):
        return self.n == 0

    def align_zero(self):
        while self.n:
            self.bit(0)

    def trailing(self):      # rbsp_trailing_bits / byte_alignment(): 1 then zeros
        self.bit(1)
        self.align_zero()

    def bytes(self):
        assert self.n == 0
        return bytes(self.out)


class CabacEncoder:
    """Informative arithmetic encoder of H.265 9.3.4.x writing into a BitWriter."""

    def __init__(self, bw):
        self.bw = bw
        self.start()

    def start(self):
        self.low, self.rng, self.first, self.outstanding = 0, 510, True, 0

    def _put(self, b):
        if self.first:
            self.first = False
        else:
            self.bw.bit(b)
        while self.outstanding:
            self.bw.bit(1 - b)
            self.outstanding -= 1

    def _renorm(self):
        while self.rng < 256:
            if self.low < 256:
                self._put(0)
            elif self.low >= 512:
                self.low -= 512
                self._put(1)
            else:
                self.low -= 256
                self.outstanding += 1
            self.rng <<= 1
            self.low <<= 1

    def decision(self, ctx, b):
        st, mps = ctx
        lps = LPS[st][(self.rng >> 6) & 3]
        self.rng -= lps
        if b != mps:
            self.low += self.rng
            self.rng = lps
            if st == 0:
                ctx[1] = 1 - mps
            ctx[0] = TRANS_LPS[st]
        else:
            ctx[0] = TRANS_MPS[st]
        self._renorm()

    def bypass(self, b):
        self.low <<= 1
        if b:
            self.low += self.rng
        if self.low >= 1024:
            self._put(1)
            self.low -= 1024
        elif self.low < 512:
            self._put(0)
        else:
            self.low -= 512
            self.outstanding += 1

    def bypass_bits(self, v, n):
        for i in range(n - 1, -1, -1):
            self.bypass((v >> i) & 1)

    def terminate(self, b):
        self.rng -= 2
        if b:
            self.low += self.rng
            self.rng = 2
            self._renorm()
            self._put((self.low >> 9) & 1)
            self.bw.bit((self.low >> 8) & 1)
            self.bw.bit(1)            # last bit of EncodeFlush: rbsp_stop_one_bit / alignment bit
        else:
            self._renorm()


# ---------------------------------------------------------------------------------------------
# scans (6.5.3-6.5.5)
# ---------------------------------------------------------------------------------------------
def _diag(n):
    out, x, y = [], 0, 0
    while len(out) < n * n:
        while y >= 0:
            if x < n and y < n:
                out.append((x, y))
            y -= 1
            x += 1
        y, x = x, 0
    return out


SCANS = {}
for _lg in range(4):
    _n = 1 << _lg
    SCANS[(_lg, 0)] = _diag(_n)
    SCANS[(_lg, 1)] = [(x, y) for y in range(_n) for x in range(_n)]
    SCANS[(_lg, 2)] = [(x, y) for x in range(_n) for y in range(_n)]
CTX_IDX_MAP = [0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8]


def qpc_of(qpi):
    if qpi < 30:
        return qpi
    if qpi >= 43:
        return qpi - 6
    return [29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37][qpi - 30]


def ceil_log2(v):
    r = 0
    while (1 << r) < v:
        r += 1
    return r


def nal(nal_type, rbsp, temporal_id=0):
    """Annex-B NAL unit: start code + header + payload with emulation prevention (7.4.2)."""
    out = bytearray(b"\x00\x00\x00\x01")
    out += bytes([(nal_type << 1) & 0x7E, temporal_id + 1])
    zeros = 0
    for b in rbsp:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


# ---------------------------------------------------------------------------------------------
# stream configuration
# ---------------------------------------------------------------------------------------------
DEFAULTS = dict(
    width=128, height=96, ctb_log2=4, min_cb_log2=3, min_tb_log2=2, max_tb_log2=4, max_th_depth=1,
    tiles=None,                 # None | (cols, rows) uniform | ([col widths], [row heights]) in CTBs
    wpp=False, slices=None,     # slices: list of (first CTB in tile-scan order, dependent?) ; None = one slice
    sign_hiding=True, tskip=True, qp_delta_depth=None, bypass=False, pcm=None,   # pcm: (log2min, log2max, lf_disabled)
    sao=True, strong=True, init_qp=26, slice_qp_delta=4, cb_qp_offset=0, cr_qp_offset=0,
    slice_chroma_offsets=None,  # (cb, cr) per independent slice, or None
    deblocking="on",            # "on" | "off" (pps disabled) | "override" (random per slice)
    lf_across_slices=1, lf_across_tiles=1, conf_window=None, hash_sei=None,   # hash_sei: None | "md5" | "crc" | "checksum"
    frames=1, idr_period=0, log2_max_poc_lsb=8, poc_order=None, max_reorder=0,   # poc_order: POC per frame (IDR first)
    split_prob=0.55, tf_split_prob=0.5, nxn_prob=0.4, cbf_prob=0.7, chroma_cbf_prob=0.35, pcm_prob=0.08,
    bypass_prob=0.1, tskip_prob=0.3, density=0.25, big_prob=0.03,
    bit_depth=8,                # BitDepthY = BitDepthC (8, or 9..12 -- QpBdOffset, SAO cMax, PCM depths)
    scaling_lists=None,         # None | "default" (enabled, no lists coded) | "sps" (random lists in the SPS) |
                                # "pps" (SPS lists overridden by random PPS lists)
)


class StreamGen:
    def __init__(self, seed=0, **cfg):
        self.cfg = dict(DEFAULTS)
        for k, v in cfg.items():
            if k not in DEFAULTS:
                raise KeyError(k)
            self.cfg[k] = v
        self.rng = np.random.default_rng(seed)
        c = self.cfg
        self.W, self.H = c["width"], c["height"]
        self.ctb = 1 << c["ctb_log2"]
        self.wc, self.hc = -(-self.W // self.ctb), -(-self.H // self.ctb)
        self._tiles()
        self.params = R.make_params(
            pic_width=self.W, pic_height=self.H, ctb_log2_size=c["ctb_log2"], min_tb_log2_size=c["min_tb_log2"],
            max_tb_log2_size=c["max_tb_log2"], strong_intra_smoothing=int(c["strong"]),
            sample_adaptive_offset=int(c["sao"]), loop_filter_across_tiles=int(c["lf_across_tiles"]) if c["tiles"] else 1,
            pps_cb_qp_offset=c["cb_qp_offset"], pps_cr_qp_offset=c["cr_qp_offset"],
            bit_depth_luma=c["bit_depth"], bit_depth_chroma=c["bit_depth"])
        self.bd = c["bit_depth"]
        self.qp_off = 6 * (self.bd - 8)                  # QpBdOffsetY = QpBdOffsetC
        self.pcm_bd = (8, 7) if self.bd == 8 else (self.bd - 1, self.bd - 2)
        self.params["scaling_list_enabled"] = int(c["scaling_lists"] is not None)
        self.scaling_factors = None
        if c["scaling_lists"] is not None:
            # the syntax of both lists is drawn now (a separate stream: the picture syntax stays as it was)
            srng = np.random.default_rng(seed + 7919)
            self.sps_sld = self._random_sld(srng) if c["scaling_lists"] in ("sps", "pps") else None
            self.pps_sld = self._random_sld(srng) if c["scaling_lists"] == "pps" else None
            from oracle import recon_oracle as O
            sld = self.pps_sld or self.sps_sld or {(s, m): ("pred", 0) for s in range(4) for m in range(0, 6, 3 if s == 3 else 1)}
            self.scaling_factors = O.scaling_factor_bytes(O.scaling_factors(*O.scaling_lists_from_syntax(sld)))

    # tile structure (6.5.1)
    def _tiles(self):
        t = self.cfg["tiles"]
        if t is None:
            cw, rh = [self.wc], [self.hc]
        elif isinstance(t[0], int):
            nc, nr = t
            cw = [((i + 1) * self.wc) // nc - (i * self.wc) // nc for i in range(nc)]
            rh = [((j + 1) * self.hc) // nr - (j * self.hc) // nr for j in range(nr)]
        else:
            cw, rh = list(t[0]), list(t[1])
            assert sum(cw) == self.wc and sum(rh) == self.hc
        self.cw, self.rh = cw, rh
        self.colbd = np.concatenate([[0], np.cumsum(cw)]).astype(int)
        self.rowbd = np.concatenate([[0], np.cumsum(rh)]).astype(int)
        ts_order, tile_of = [], np.zeros(self.wc * self.hc, int)
        tid = 0
        for j in range(len(rh)):
            for i in range(len(cw)):
                for y in range(self.rowbd[j], self.rowbd[j + 1]):
                    for x in range(self.colbd[i], self.colbd[i + 1]):
                        ts_order.append(y * self.wc + x)
                        tile_of[y * self.wc + x] = tid
                tid += 1
        self.ts_to_rs = ts_order
        self.rs_to_ts = {rs: ts for ts, rs in enumerate(ts_order)}
        self.tile_of = tile_of

    def tile_col0(self, cx):
        return max(b for b in self.colbd[:-1] if b <= cx)

    def tile_row0(self, cy):
        return max(b for b in self.rowbd[:-1] if b <= cy)

    # ----------------------------------------------------------------- scaling lists (7.3.4)
    @staticmethod
    def _random_sld(r):
        """Random scaling_list_data syntax: {(sizeId, matrixId): ("pred", delta) | ("coded", dc_minus8, deltas)},
        every resulting list value in 1..255 (oracle.recon_oracle.scaling_lists_from_syntax's form)."""
        sld = {}
        for size_id in range(4):
            step = 3 if size_id == 3 else 1
            for matrix_id in range(0, 6, step):
                if r.random() < 0.3:
                    sld[(size_id, matrix_id)] = ("pred", int(r.integers(0, matrix_id // step + 1)))
                    continue
                n = min(64, 1 << (4 + 2 * size_id))
                vals = r.integers(1, 256, n) if r.random() < 0.5 else np.clip(16 + np.cumsum(r.integers(-3, 6, n)), 1, 255)
                prev, dc = 8, None
                if size_id > 1:
                    dcv = int(r.integers(1, 256))
                    dc, prev = dcv - 8, dcv
                deltas = []
                for v in vals:
                    d = ((int(v) - prev + 128) % 256) - 128
                    deltas.append(d)
                    prev = int(v)
                sld[(size_id, matrix_id)] = ("coded", dc, deltas)
        return sld

    @staticmethod
    def _write_sld(bw, sld):
        for size_id in range(4):
            for matrix_id in range(0, 6, 3 if size_id == 3 else 1):
                kind = sld[(size_id, matrix_id)]
                if kind[0] == "pred":
                    bw.u(0, 1)
                    bw.ue(kind[1])
                else:
                    bw.u(1, 1)
                    if size_id > 1:
                        bw.se(kind[1])
                    for d in kind[2]:
                        bw.se(d)

    # ----------------------------------------------------------------- parameter sets
    def vps(self):
        bw = BitWriter()
        bw.u(0, 4); bw.u(1, 1); bw.u(1, 1); bw.u(0, 6); bw.u(0, 3); bw.u(1, 1); bw.u(0xFFFF, 16)
        self._ptl(bw)
        bw.u(1, 1); bw.ue(1); bw.ue(0); bw.ue(0)     # sub_layer_ordering_info + dpb
        bw.u(0, 6); bw.ue(0); bw.u(0, 1); bw.u(0, 1)  # max_layer_id, num_layer_sets_minus1, timing, ext
        bw.trailing()
        return nal(32, bw.bytes())

    def _ptl(self, bw):
        main10 = self.cfg["bit_depth"] > 8
        bw.u(0, 2); bw.u(0, 1); bw.u(2 if main10 else 1, 5)     # Main / Main 10 profile
        bw.u(0x20000000 if main10 else 0x60000000, 32)
        bw.u(0b1001, 4)
        bw.u(0, 43); bw.u(0, 1)
        bw.u(120, 8)

    def sps(self):
        c = self.cfg
        bw = BitWriter()
        bw.u(0, 4); bw.u(0, 3); bw.u(1, 1)
        self._ptl(bw)
        bw.ue(0); bw.ue(1)                               # sps id, chroma_format_idc
        bw.ue(self.W); bw.ue(self.H)
        if c["conf_window"]:
            bw.u(1, 1)
            for v in c["conf_window"]:
                bw.ue(v)
        else:
            bw.u(0, 1)
        bw.ue(self.bd - 8); bw.ue(self.bd - 8)           # bit_depth_luma / chroma_minus8
        bw.ue(c["log2_max_poc_lsb"] - 4)
        bw.u(1, 1); bw.ue(1 + c["max_reorder"]); bw.ue(c["max_reorder"]); bw.ue(0)
        bw.ue(c["min_cb_log2"] - 3); bw.ue(c["ctb_log2"] - c["min_cb_log2"])
        bw.ue(c["min_tb_log2"] - 2); bw.ue(c["max_tb_log2"] - c["min_tb_log2"])
        bw.ue(c["max_th_depth"]); bw.ue(c["max_th_depth"])
        if c["scaling_lists"] is None:
            bw.u(0, 1)                                   # scaling_list_enabled_flag 0
        else:
            bw.u(1, 1)
            bw.u(int(self.sps_sld is not None), 1)       # sps_scaling_list_data_present_flag
            if self.sps_sld is not None:
                self._write_sld(bw, self.sps_sld)
        bw.u(1, 1); bw.u(int(c["sao"]), 1)               # amp, sao
        if c["pcm"]:
            lo, hi, lfd = c["pcm"]
            bw.u(1, 1); bw.u(self.pcm_bd[0] - 1, 4); bw.u(self.pcm_bd[1] - 1, 4)   # PcmBitDepth Y / C
            bw.ue(lo - 3); bw.ue(hi - lo); bw.u(int(lfd), 1)
        else:
            bw.u(0, 1)
        bw.ue(1)                                         # one short-term RPS: one negative picture
        bw.ue(1); bw.ue(0); bw.ue(0); bw.u(1, 1)
        bw.u(0, 1); bw.u(0, 1); bw.u(int(c["strong"]), 1)   # long-term, temporal mvp, strong smoothing
        bw.u(1, 1)                                       # vui_parameters_present_flag
        bw.u(1, 1); bw.u(255, 8); bw.u(1, 16); bw.u(1, 16)  # aspect ratio (extended SAR)
        bw.u(0, 1); bw.u(1, 1); bw.u(5, 3); bw.u(0, 1); bw.u(1, 1); bw.u(1, 8); bw.u(1, 8); bw.u(1, 8)
        bw.u(0, 1); bw.u(0, 1); bw.u(0, 1); bw.u(0, 1); bw.u(0, 1)
        bw.u(1, 1); bw.u(1001, 32); bw.u(60000, 32); bw.u(0, 1)
        bw.u(1, 1)                                       # vui_hrd_parameters_present_flag
        bw.u(1, 1); bw.u(0, 1); bw.u(0, 1); bw.u(2, 4); bw.u(3, 4); bw.u(23, 5); bw.u(23, 5); bw.u(23, 5)
        bw.u(0, 1); bw.u(1, 1); bw.ue(0); bw.ue(0)       # fixed_pic_rate_general 0, within cvs 1, duration, cpb_cnt
        bw.ue(1000); bw.ue(2000); bw.u(0, 1)             # nal sub-layer hrd
        bw.u(0, 1)                                       # bitstream_restriction_flag
        bw.u(0, 1)                                       # sps_extension_present_flag
        bw.trailing()
        return nal(33, bw.bytes())

    def pps(self):
        c = self.cfg
        bw = BitWriter()
        bw.ue(0); bw.ue(0)
        dep = any(d for _, d in (c["slices"] or []))
        bw.u(int(dep), 1); bw.u(0, 1); bw.u(0, 3); bw.u(int(c["sign_hiding"]), 1); bw.u(1, 1)
        bw.ue(0); bw.ue(0); bw.se(c["init_qp"] - 26)
        bw.u(0, 1); bw.u(int(c["tskip"]), 1)
        if c["qp_delta_depth"] is not None:
            bw.u(1, 1); bw.ue(c["qp_delta_depth"])
        else:
            bw.u(0, 1)
        bw.se(c["cb_qp_offset"]); bw.se(c["cr_qp_offset"])
        bw.u(int(c["slice_chroma_offsets"] is not None), 1)
        bw.u(0, 1); bw.u(0, 1); bw.u(int(c["bypass"]), 1)
        bw.u(int(c["tiles"] is not None), 1); bw.u(int(c["wpp"]), 1)
        if c["tiles"] is not None:
            bw.ue(len(self.cw) - 1); bw.ue(len(self.rh) - 1)
            uniform = isinstance(c["tiles"][0], int)
            bw.u(int(uniform), 1)
            if not uniform:
                for v in self.cw[:-1]:
                    bw.ue(v - 1)
                for v in self.rh[:-1]:
                    bw.ue(v - 1)
            bw.u(int(c["lf_across_tiles"]), 1)
        bw.u(int(c["lf_across_slices"]), 1)
        dbk = c["deblocking"]
        if dbk == "on":
            bw.u(0, 1)
        else:
            bw.u(1, 1)
            bw.u(int(dbk == "override"), 1)
            bw.u(int(dbk == "off"), 1)
            if dbk != "off":
                bw.se(1); bw.se(-2)
        pps_sld = getattr(self, "pps_sld", None)
        bw.u(int(pps_sld is not None), 1)               # pps_scaling_list_data_present_flag
        if pps_sld is not None:
            self._write_sld(bw, pps_sld)
        bw.u(0, 1); bw.ue(0); bw.u(0, 1); bw.u(0, 1)
        bw.trailing()
        return nal(34, bw.bytes())

    # ----------------------------------------------------------------- stream
    def stream(self, planes_fn=None):
        """-> (bytes, [(params, records.Picture, poc)] in decode order).

        With ``hash_sei`` set, each picture is followed by a decoded-picture-hash SEI: of
        ``planes_fn(params, picture)`` (the decoded Y/Cb/Cr planes, e.g. from the oracle)
        when given, else random bytes (syntax test only)."""
        c = self.cfg
        out = [self.vps(), self.sps(), self.pps()]
        pics = []
        poc = 0
        max_lsb = 1 << c["log2_max_poc_lsb"]
        for f in range(c["frames"]):
            idr = f == 0 or (c["idr_period"] and f % c["idr_period"] == 0)
            if c["poc_order"] is not None:
                idr, poc = f == 0, c["poc_order"][f]
            elif idr:
                poc = 0
            nal_type = 19 if idr else 1
            nals, pic = self.picture(nal_type, poc % max_lsb)
            out += nals
            if c["hash_sei"] and planes_fn is not None:
                kind = {"md5": 0, "crc": 1, "checksum": 2}[c["hash_sei"]]
                extra = {} if self.scaling_factors is None else {"scaling": self.scaling_factors}
                hv = picture_hash(planes_fn(self.params, pic, **extra), c["hash_sei"])
                self.last_hash = (kind, hv)
                out.append(sei_nal(bytes([kind]) + b"".join(hv)))
            elif c["hash_sei"]:
                out.append(self.hash_sei_placeholder())
            pics.append((self.params, pic, poc))
            poc += 1
        return b"".join(out), pics

    def hash_sei_placeholder(self):
        """Suffix SEI with a decoded picture hash whose value is random (parse test only)."""
        kind = {"md5": 0, "crc": 1, "checksum": 2}[self.cfg["hash_sei"]]
        ln = {0: 16, 1: 2, 2: 4}[kind]
        payload = bytes([kind]) + bytes(self.rng.integers(0, 256, 3 * ln, dtype=np.uint8))
        self.last_hash = (kind, [payload[1 + i * ln: 1 + (i + 1) * ln] for i in range(3)])
        return sei_nal(payload)

    def picture(self, nal_type, poc_lsb):
        c = self.cfg
        self.builder = frontend.PictureBuilder(self.params, pcm_loop_filter_disabled=bool(c["pcm"] and c["pcm"][2]))
        n = self.wc * self.hc
        self.ctb_slice = np.full(n, -1, int)
        mcb = 1 << c["min_cb_log2"]
        self.depth = np.zeros((self.H // mcb, self.W // mcb), int)
        self.qpmap = np.zeros((self.H // mcb, self.W // mcb), int)
        self.ipm = np.ones(((self.H + 3) // 4, (self.W + 3) // 4), int)
        self.sao = {}
        segs = c["slices"] or [(0, False)]
        assert segs[0] == (0, False)
        bounds = [s for s, _ in segs] + [n]
        nals = []
        self.wpp_states = None
        indep_hdr = None
        for k, (start, dep) in enumerate(segs):
            end = bounds[k + 1]
            if not dep:
                indep_hdr = self._slice_params(start)
            nals.append(self._segment(nal_type, poc_lsb, start, end, dep, indep_hdr))
        return nals, self.builder.finish()

    def _slice_params(self, start):
        c = self.cfg
        r = self.rng
        h = dict(slice_addr=self.ts_to_rs[start], qp=c["init_qp"] + c["slice_qp_delta"],
                 sao_luma=int(c["sao"] and r.random() < 0.85), sao_chroma=int(c["sao"] and r.random() < 0.7),
                 cb=0, cr=0, dbk_disabled=0, beta=0, tc=0, override=0)
        if c["slice_chroma_offsets"] is not None:
            h["cb"], h["cr"] = c["slice_chroma_offsets"]
        if c["deblocking"] == "off":
            h["dbk_disabled"] = 1
        elif c["deblocking"] == "override":
            h["beta"], h["tc"] = 1, -2
            if r.random() < 0.6:
                h["override"] = 1
                h["dbk_disabled"] = int(r.random() < 0.3)
                if not h["dbk_disabled"]:
                    h["beta"], h["tc"] = int(r.integers(-6, 7)), int(r.integers(-6, 7))
        h["lf_across"] = c["lf_across_slices"]
        if c["lf_across_slices"] and (h["sao_luma"] or h["sao_chroma"] or not h["dbk_disabled"]):
            h["lf_across"] = int(r.random() < 0.5)
            h["code_lf_across"] = True
        return h

    def _header(self, bw, nal_type, poc_lsb, start, dep, h, entry_points):
        c = self.cfg
        n = self.wc * self.hc
        bw.u(int(start == 0), 1)
        if 16 <= nal_type <= 23:
            bw.u(0, 1)
        bw.ue(0)
        if start != 0:
            if any(d for _, d in (c["slices"] or [])):
                bw.u(int(dep), 1)
            bw.u(self.ts_to_rs[start], ceil_log2(n))
        if not dep:
            bw.ue(2)                                     # slice_type I
            if nal_type not in (19, 20):
                bw.u(poc_lsb, c["log2_max_poc_lsb"])
                bw.u(1, 1)                               # short_term_ref_pic_set_sps_flag (1 set: no idx)
            if c["sao"]:
                bw.u(h["sao_luma"], 1); bw.u(h["sao_chroma"], 1)
            bw.se(h["qp"] - c["init_qp"])
            if c["slice_chroma_offsets"] is not None:
                bw.se(h["cb"]); bw.se(h["cr"])
            if c["deblocking"] == "override":
                bw.u(h["override"], 1)
                if h["override"]:
                    bw.u(h["dbk_disabled"], 1)
                    if not h["dbk_disabled"]:
                        bw.se(h["beta"]); bw.se(h["tc"])
            if h.get("code_lf_across"):
                bw.u(h["lf_across"], 1)
        if c["tiles"] is not None or c["wpp"]:
            bw.ue(len(entry_points))
            if entry_points:
                ln = max(max(entry_points).bit_length(), 1)
                bw.ue(ln - 1)
                for e in entry_points:
                    bw.u(e - 1, ln)
        bw.trailing()

    def _segment(self, nal_type, poc_lsb, start, end, dep, h):
        """Encode slice segment data for CTBs [start, end) in tile-scan order; returns the NAL."""
        self.h = h
        data = BitWriter()
        enc = CabacEncoder(data)
        self.enc = enc
        substream_sizes = []
        sub_start = 0
        first = True
        for ts in range(start, end):
            rs = self.ts_to_rs[ts]
            cx, cy = rs % self.wc, rs // self.wc
            self.cur_tile = self.tile_of[rs]
            self.ctb_slice[rs] = h["slice_addr"]
            col0, row0 = self.tile_col0(cx), self.tile_row0(cy)
            first_in_tile = cx == col0 and cy == row0
            wpp_row = self.cfg["wpp"] and cx == col0
            if first or first_in_tile or wpp_row:
                if first_in_tile:
                    self.st = init_states(h["qp"])
                elif wpp_row:
                    tr = (cy - 1) * self.wc + cx + 1
                    if cx + 1 < self.wc and cy > 0 and self._ctb_avail(tr) and self.wpp_states is not None:
                        self.st = {k: [list(s) for s in v] for k, v in self.wpp_states.items()}
                    else:
                        self.st = init_states(h["qp"])
                elif dep:
                    self.st = {k: [list(s) for s in v] for k, v in self.ds_states.items()}
                else:
                    self.st = init_states(h["qp"])
                if (first and not dep) or first_in_tile or wpp_row:
                    self.first_qg = True
            first = False
            self._ctu(rs, ts)
            if self.cfg["wpp"] and cx == col0 + 1:
                self.wpp_states = {k: [list(s) for s in v] for k, v in self.st.items()}
            last = ts == end - 1
            enc.terminate(int(last))
            if last:
                break
            nrs = self.ts_to_rs[ts + 1]
            ncx = nrs % self.wc
            new_tile = self.cfg["tiles"] is not None and self.tile_of[nrs] != self.tile_of[rs]
            new_row = self.cfg["wpp"] and ncx == self.tile_col0(ncx)
            if new_tile or new_row:
                enc.terminate(1)                         # end_of_subset_one_bit + flush (its last bit = alignment 1)
                data.align_zero()
                enc.start()
                substream_sizes.append(len(data.out) - sub_start)
                sub_start = len(data.out)
        data.align_zero()                                # rbsp_slice_segment_trailing_bits after the flush's stop bit
        self.ds_states = {k: [list(s) for s in v] for k, v in self.st.items()}
        payload = data.bytes()
        # entry points count emulation prevention bytes of the slice data (7.4.7.1): iterate
        eps = self._ep_sizes(payload, substream_sizes, b"")
        for _ in range(4):
            hw = BitWriter()
            self._header(hw, nal_type, poc_lsb, start, dep, h, eps)
            head = hw.bytes()
            neweps = self._ep_sizes(payload, substream_sizes, head)
            if neweps == eps:
                break
            eps = neweps
        return nal(nal_type, head + payload)

    @staticmethod
    def _ep_sizes(payload, sizes, head):
        if not sizes:
            return []
        full = nal(0, head + payload)[6:]
        # map rbsp byte index -> escaped index
        idx, zeros, j = [], 0, 0
        src = head + payload
        esc = 0
        for b in src:
            if zeros >= 2 and b <= 3:
                esc += 1
                zeros = 0
            idx.append(j + esc)
            zeros = zeros + 1 if b == 0 else 0
            j += 1
        assert len(full) == len(src) + esc
        base = len(head)
        out, pos = [], 0
        for s in sizes:
            a, b_ = base + pos, base + pos + s
            out.append(idx[b_] - idx[a])
            pos += s
        return out

    # ----------------------------------------------------------------- CTU / SAO
    def _ctb_avail(self, rs):
        return self.ctb_slice[rs] == self.h["slice_addr"] and self.tile_of[rs] == self.cur_tile

    def _avail(self, x, y):
        if x < 0 or y < 0 or x >= self.W or y >= self.H:
            return False
        return self._ctb_avail((y // self.ctb) * self.wc + x // self.ctb)

    def _ctx(self, name, i=0):
        return self.st[name][i]

    def _ctu(self, rs, ts):
        h, r, enc = self.h, self.rng, self.enc
        cx, cy = rs % self.wc, rs // self.wc
        sao = dict(type=(0, 0, 0), abs=[[0] * 4 for _ in range(3)], sign=[[0] * 4 for _ in range(3)],
                   band=[0, 0, 0], eo=[0, 0, 0])
        if h["sao_luma"] or h["sao_chroma"]:
            merged = False
            if cx > 0 and rs > h["slice_addr"] and self.tile_of[rs] == self.tile_of[rs - 1]:
                ml = int(r.random() < 0.25)
                enc.decision(self._ctx("sao_merge"), ml)
                if ml:
                    sao, merged = self.sao[rs - 1], True
            if not merged and cy > 0 and rs - self.wc >= h["slice_addr"] and self.tile_of[rs] == self.tile_of[rs - self.wc]:
                mu = int(r.random() < 0.25)
                enc.decision(self._ctx("sao_merge"), mu)
                if mu:
                    sao, merged = self.sao[rs - self.wc], True
            if not merged:
                types = [0, 0, 0]
                for ci in range(3):
                    if not ((h["sao_luma"] and ci == 0) or (h["sao_chroma"] and ci > 0)):
                        continue
                    if ci < 2:
                        t = int(r.choice([0, 1, 2], p=[0.1, 0.3, 0.6]))
                        enc.decision(self._ctx("sao_type"), int(t != 0))
                        if t:
                            enc.bypass(int(t == 2))
                    else:
                        t = types[1]
                    types[ci] = t
                    if not t:
                        continue
                    cmax = (1 << (min(self.bd, 10) - 5)) - 1     # sao_offset_abs: TR, cMax by bit depth
                    for i in range(4):
                        a = int(r.integers(0, cmax + 1))
                        sao["abs"][ci][i] = a
                        for _ in range(a):
                            enc.bypass(1)
                        if a < cmax:
                            enc.bypass(0)
                    if t == 1:
                        for i in range(4):
                            if sao["abs"][ci][i]:
                                s = int(r.integers(0, 2))
                                sao["sign"][ci][i] = s
                                enc.bypass(s)
                        b = int(r.integers(0, 32))
                        sao["band"][ci] = b
                        enc.bypass_bits(b, 5)
                    else:
                        if ci < 2:
                            e = int(r.integers(0, 4))
                            enc.bypass_bits(e, 2)
                        else:
                            e = sao["eo"][1]
                        sao["eo"][ci] = e
                sao["type"] = tuple(types)
        self.sao[rs] = sao
        self.builder.add_ctu(rs, slice_addr=h["slice_addr"], tile_id=int(self.tile_of[rs]),
                             lf_across_slices=bool(h["lf_across"]), sao_type=sao["type"], sao_abs=sao["abs"],
                             sao_sign=sao["sign"], sao_band=sao["band"], sao_eo=sao["eo"],
                             deblocking=not h["dbk_disabled"], beta_offset_div2=h["beta"], tc_offset_div2=h["tc"])
        self._cqt(cx * self.ctb, cy * self.ctb, self.cfg["ctb_log2"], 0)

    # ----------------------------------------------------------------- coding quadtree / CU
    def _cqt(self, x0, y0, log2, depth):
        c, r, enc = self.cfg, self.rng, self.enc
        size = 1 << log2
        mcb = c["min_cb_log2"]
        if x0 + size <= self.W and y0 + size <= self.H and log2 > mcb:
            inc = 0
            if self._avail(x0 - 1, y0) and self.depth[y0 >> mcb, (x0 - 1) >> mcb] > depth:
                inc += 1
            if self._avail(x0, y0 - 1) and self.depth[(y0 - 1) >> mcb, x0 >> mcb] > depth:
                inc += 1
            sp = c["split_prob"]
            split = int(r.random() < (sp[log2] if isinstance(sp, dict) else sp))
            enc.decision(self._ctx("split_cu", inc), split)
        else:
            split = int(log2 > mcb)
        if split:
            hs = size >> 1
            for dx, dy in ((0, 0), (hs, 0), (0, hs), (hs, hs)):
                if x0 + dx < self.W and y0 + dy < self.H:
                    self._cqt(x0 + dx, y0 + dy, log2 - 1, depth + 1)
        else:
            self._cu(x0, y0, log2, depth)

    def _mpm(self, xp, yp):
        a = self.ipm[yp >> 2, (xp - 1) >> 2] if self._avail(xp - 1, yp) else 1
        ctb_top = (yp // self.ctb) * self.ctb
        b = self.ipm[(yp - 1) >> 2, xp >> 2] if (yp - 1 >= ctb_top and self._avail(xp, yp - 1)) else 1
        if a == b:
            return [0, 1, 26] if a < 2 else [a, 2 + ((a + 29) % 32), 2 + ((a - 2 + 1) % 32)]
        third = 0 if (a != 0 and b != 0) else (1 if (a != 1 and b != 1) else 26)
        return [a, b, third]

    def _cu(self, x0, y0, log2, depth):
        c, r, enc = self.cfg, self.rng, self.enc
        size = 1 << log2
        mcb = c["min_cb_log2"]
        self.depth[y0 >> mcb:(y0 + size) >> mcb, x0 >> mcb:(x0 + size) >> mcb] = depth
        qg_log2 = c["ctb_log2"] - (c["qp_delta_depth"] or 0)
        qmask = (1 << qg_log2) - 1
        if (x0 & qmask) == 0 and (y0 & qmask) == 0:
            self.qp_delta_coded = False
            self.qp_delta = 0
            prev = self.h["qp"] if self.first_qg else self.last_qp
            self.first_qg = False
            cm = self.ctb - 1
            qa = self.qpmap[y0 >> mcb, (x0 - 1) >> mcb] if (x0 & cm) else prev
            qb = self.qpmap[(y0 - 1) >> mcb, x0 >> mcb] if (y0 & cm) else prev
            self.qg_pred = (qa + qb + 1) >> 1
        bypass = 0
        if c["bypass"]:
            bypass = int(r.random() < c["bypass_prob"])
            enc.decision(self._ctx("bypass"), bypass)
        nxn = 0
        if log2 == mcb:
            nxn = int(r.random() < c["nxn_prob"])
            enc.decision(self._ctx("part_mode"), 1 - nxn)
        pcm = 0
        if c["pcm"] and not nxn and c["pcm"][0] <= log2 <= c["pcm"][1]:
            pcm = int(r.random() < c["pcm_prob"])
            enc.terminate(pcm)
        modes = [1, 1, 1, 1]
        mode_c = 0
        tus = []
        pcm_samples = None
        if pcm:
            self.ipm[y0 >> 2:(y0 + size) >> 2, x0 >> 2:(x0 + size) >> 2] = 1
            self.enc.bw.align_zero()                     # pcm_alignment_zero_bit(s) after the flush
            pcm_samples = []
            pby, pbc = self.pcm_bd
            for ci, (lg, bd) in enumerate(((log2, pby), (log2 - 1, pbc), (log2 - 1, pbc))):
                n = 1 << lg
                v = r.integers(0, 1 << bd, (n, n))
                for s in v.reshape(-1):
                    self.enc.bw.u(int(s), bd)
                pcm_samples.append((v << (self.bd - bd)).astype(np.int16))
            self.enc.start()
        else:
            nparts = 4 if nxn else 1
            pb = size >> 1 if nxn else size
            chosen, flags, code = [], [], []
            for i in range(nparts):
                xp, yp = x0 + pb * (i & 1), y0 + pb * (i >> 1)
                cand = self._mpm(xp, yp)
                if r.random() < 0.5:
                    m = cand[int(r.integers(0, 3))]
                else:
                    m = int(r.integers(0, 35))
                modes[i] = m
                self.ipm[yp >> 2:(yp + pb) >> 2, xp >> 2:(xp + pb) >> 2] = m
                if m in cand:
                    flags.append(1)
                    code.append(cand.index(m))
                else:
                    flags.append(0)
                    sc = sorted(cand)
                    rem = m - sum(1 for v in sc if v < m)
                    code.append(rem)
            for f in flags:
                enc.decision(self._ctx("prev_intra"), f)
            for f, v in zip(flags, code):
                if f:
                    enc.bypass(int(v > 0))
                    if v > 0:
                        enc.bypass(int(v > 1))
                else:
                    enc.bypass_bits(v, 5)
            icpm = int(r.integers(0, 5))
            if icpm == 4:
                enc.decision(self._ctx("chroma_mode"), 0)
                mode_c = modes[0]
            else:
                enc.decision(self._ctx("chroma_mode"), 1)
                enc.bypass_bits(icpm, 2)
                mode_c = [0, 26, 10, 1][icpm]
                if mode_c == modes[0]:
                    mode_c = 34
            self.cu = dict(x=x0, y=y0, log2=log2, nxn=nxn, bypass=bypass, modes=modes, mode_c=mode_c)
            self._tt(x0, y0, x0, y0, log2, 0, 0, 1, 1, tus)
        off = self.qp_off                                # QpY (8.6.1), then qP' = Qp + QpBdOffset for the records
        qpy = ((self.qg_pred + self.qp_delta + 52 + 2 * off) % (52 + off)) - off
        self.last_qp = qpy
        self.qpmap[y0 >> mcb:(y0 + size) >> mcb, x0 >> mcb:(x0 + size) >> mcb] = qpy
        h = self.h
        qcb = qpc_of(min(max(qpy + c["cb_qp_offset"] + h["cb"], -off), 57))
        qcr = qpc_of(min(max(qpy + c["cr_qp_offset"] + h["cr"], -off), 57))
        self.builder.add_cu(x0, y0, log2, 1 if nxn else 0, modes, mode_c, qpy + off, qcb + off, qcr + off, tus,
                            bypass=bool(bypass), pcm=bool(pcm), pcm_samples=pcm_samples)

    def _tt(self, x0, y0, xb, yb, log2, depth, blk, pcb, pcr, tus):
        c, r, enc, cu = self.cfg, self.rng, self.enc, self.cu
        maxd = c["max_th_depth"] + cu["nxn"]
        if log2 <= c["max_tb_log2"] and log2 > c["min_tb_log2"] and depth < maxd and not (cu["nxn"] and depth == 0):
            sp = c["tf_split_prob"]
            split = int(r.random() < (sp[log2] if isinstance(sp, dict) else sp))
            enc.decision(self._ctx("split_tf", 5 - log2), split)
        else:
            split = int(log2 > c["max_tb_log2"] or (cu["nxn"] and depth == 0))
        cb = cr = 0
        if log2 > 2:
            if depth == 0 or pcb:
                cb = int(r.random() < c["chroma_cbf_prob"])
                enc.decision(self._ctx("cbf_chroma", depth), cb)
            if depth == 0 or pcr:
                cr = int(r.random() < c["chroma_cbf_prob"])
                enc.decision(self._ctx("cbf_chroma", depth), cr)
        if split:
            hs = 1 << (log2 - 1)
            for i, (dx, dy) in enumerate(((0, 0), (hs, 0), (0, hs), (hs, hs))):
                self._tt(x0 + dx, y0 + dy, x0, y0, log2 - 1, depth + 1, i, cb, cr, tus)
            return
        cbl = int(r.random() < c["cbf_prob"])
        enc.decision(self._ctx("cbf_luma", 1 if depth == 0 else 0), cbl)
        ccb, ccr = (cb, cr) if log2 > 2 else (pcb, pcr)
        if (cbl or ccb or ccr) and c["qp_delta_depth"] is not None and not self.qp_delta_coded:
            lim = 26 + self.qp_off // 2                  # CuQpDeltaVal in -(26 + QpBdOffsetY / 2) .. 25 + QpBdOffsetY / 2
            v = int(r.integers(-lim, lim)) if r.random() < 0.7 else 0
            # bias towards the small values of real streams but keep large ones for the EG0 suffix
            if r.random() < 0.6:
                v = int(np.clip(v, -4, 4))
            a = abs(v)
            for i in range(min(a, 5)):
                enc.decision(self._ctx("qp_delta", 0 if i == 0 else 1), 1)
            if a < 5:
                enc.decision(self._ctx("qp_delta", 0 if a == 0 else 1), 0)
            else:
                s = a - 5                                # EG0 suffix
                k = 0
                while s >= (1 << k):
                    enc.bypass(1)
                    s -= 1 << k
                    k += 1
                enc.bypass(0)
                enc.bypass_bits(s, k)
            if a:
                enc.bypass(int(v < 0))
            self.qp_delta_coded = True
            self.qp_delta = v
        mode_y = cu["modes"][((y0 - cu["y"]) >= (1 << (cu["log2"] - 1))) * 2 + ((x0 - cu["x"]) >= (1 << (cu["log2"] - 1)))] \
            if cu["nxn"] else cu["modes"][0]
        t = dict(x=x0, y=y0, log2=log2, blk=blk, cbf=[cbl, 0, 0], tskip=[0, 0, 0], coef=[None, None, None])
        if cbl:
            t["coef"][0], t["tskip"][0] = self._residual(log2, 0, mode_y)
        if log2 > 2:
            t["cbf"][1], t["cbf"][2] = cb, cr
            for ci, f in ((1, cb), (2, cr)):
                if f:
                    t["coef"][ci], t["tskip"][ci] = self._residual(log2 - 1, ci, cu["mode_c"])
        elif blk == 3:
            t["cbf"][1], t["cbf"][2] = pcb, pcr
            for ci, f in ((1, pcb), (2, pcr)):
                if f:
                    t["coef"][ci], t["tskip"][ci] = self._residual(2, ci, cu["mode_c"])
        tus.append(t)

    # ----------------------------------------------------------------- residual_coding
    def _coefs(self, log2):
        r, c = self.rng, self.cfg
        n = 1 << log2
        blk = np.zeros((n, n), np.int64)
        dens = c["density"] * r.random()
        m = r.random((n, n)) < dens * np.exp(-(np.add.outer(np.arange(n), np.arange(n))) / max(1.0, n / 2.5)) * 2
        if not m.any():
            m[int(r.integers(0, n)), int(r.integers(0, n))] = True
        mag = r.geometric(0.5, (n, n))
        big = r.random((n, n)) < c["big_prob"]
        mag = np.where(big, r.integers(1, 32768, (n, n)), mag)
        sgn = r.choice(np.array([-1, 1]), (n, n))
        blk[m] = (mag * sgn)[m]
        return blk                                        # [y][x]

    def _residual(self, log2, ci, pred_mode):
        c, r, enc, cu = self.cfg, self.rng, self.enc, self.cu
        n = 1 << log2
        blk = self._coefs(log2)
        tskip = 0
        if c["tskip"] and not cu["bypass"] and log2 == 2:
            tskip = int(r.random() < c["tskip_prob"])
            enc.decision(self._ctx("tskip", 1 if ci else 0), tskip)
        scan = 0
        if log2 == 2 or (log2 == 3 and ci == 0):
            if 6 <= pred_mode <= 14:
                scan = 2
            elif 22 <= pred_mode <= 30:
                scan = 1
        lsb = log2 - 2
        sbs = SCANS[(lsb, scan)]
        cs = SCANS[(2, scan)]
        order = [((xs << 2) + xp, (ys << 2) + yp) for (xs, ys) in sbs for (xp, yp) in cs]
        nz = [i for i, (x, y) in enumerate(order) if blk[y, x] != 0]
        last = nz[-1]
        lx, ly = order[last]
        # sign data hiding: force the hidden sign to the parity rule (7.3.8.11)
        sdh = c["sign_hiding"] and not cu["bypass"]
        if sdh:
            for sb in range(len(sbs)):
                idx = [i for i in range(sb * 16, sb * 16 + 16) if blk[order[i][1], order[i][0]] != 0]
                if idx and idx[-1] - idx[0] > 3:
                    x, y = order[idx[0]]
                    s = int(sum(abs(blk[order[i][1], order[i][0]]) for i in idx))
                    blk[y, x] = -abs(blk[y, x]) if (s & 1) else abs(blk[y, x])
        # last_sig_coeff prefix / suffix (coded in the swapped frame when scanIdx == 2)
        cx, cy = (ly, lx) if scan == 2 else (lx, ly)
        if ci == 0:
            off, sh = 3 * (log2 - 2) + ((log2 - 1) >> 2), (log2 + 1) >> 2
        else:
            off, sh = 15, log2 - 2
        cmax = (log2 << 1) - 1

        def split_last(v):
            if v < 4:
                return v, None, 0
            p = 2 * (v.bit_length() - 1) + ((v >> (v.bit_length() - 2)) & 1)
            nb = (p >> 1) - 1
            return p, v - (1 << nb) * (2 + (p & 1)), nb

        px, sx, nbx = split_last(cx)
        py, sy, nby = split_last(cy)
        for name, p in (("last_x", px), ("last_y", py)):
            for i in range(p):
                enc.decision(self._ctx(name, off + (i >> sh)), 1)
            if p < cmax:
                enc.decision(self._ctx(name, off + (p >> sh)), 0)
        if sx is not None:
            enc.bypass_bits(sx, nbx)
        if sy is not None:
            enc.bypass_bits(sy, nby)
        last_sb = last // 16
        csbf = {}
        g1state, any_done = 1, False
        for i in range(last_sb, -1, -1):
            xs, ys = sbs[i]
            pos = [i * 16 + k for k in range(16)]
            vals = [int(blk[order[p][1], order[p][0]]) for p in pos]
            has = any(v != 0 for v in vals)
            infer_dc = False
            if 0 < i < last_sb:
                inc = min(csbf.get((xs + 1, ys), 0) + csbf.get((xs, ys + 1), 0), 1) + (2 if ci else 0)
                enc.decision(self._ctx("csbf", inc), int(has))
                csbf[(xs, ys)] = int(has)
                infer_dc = True
            else:
                csbf[(xs, ys)] = 1
            if not csbf[(xs, ys)]:
                continue
            start = (last - i * 16 - 1) if i == last_sb else 15
            sig = []
            if i == last_sb:
                sig.append(last - i * 16)
            prev = 0
            if log2 > 2:
                prev = csbf.get((xs + 1, ys), 0) | (csbf.get((xs, ys + 1), 0) << 1)
            for nn in range(start, -1, -1):
                xp, yp = cs[nn]
                v = vals[nn]
                if nn == 0 and infer_dc:
                    # an all-zero-except-DC coded sub-block infers its DC coefficient: must be non-zero
                    if v == 0:
                        blk[(ys << 2) + yp, (xs << 2) + xp] = 1
                        vals[nn] = v = 1
                    sig.append(nn)
                    continue
                if log2 == 2:
                    sc = CTX_IDX_MAP[(yp << 2) + xp]
                elif xs == 0 and ys == 0 and xp == 0 and yp == 0:
                    sc = 0
                else:
                    if prev == 0:
                        sc = 2 if xp + yp == 0 else (1 if xp + yp < 3 else 0)
                    elif prev == 1:
                        sc = 2 if yp == 0 else (1 if yp == 1 else 0)
                    elif prev == 2:
                        sc = 2 if xp == 0 else (1 if xp == 1 else 0)
                    else:
                        sc = 2
                    if ci == 0:
                        sc += (3 if (xs or ys) else 0) + ((9 if scan == 0 else 15) if log2 == 3 else 21)
                    else:
                        sc += 9 if log2 == 3 else 12
                enc.decision(self._ctx("sig", (27 + sc) if ci else sc), int(v != 0))
                if v != 0:
                    sig.append(nn)
                    infer_dc = False
            if not sig:
                continue
            # levels
            ctx_set = 0 if (i == 0 or ci > 0) else 2
            if any_done and g1state == 0:
                ctx_set += 1
            any_done = True
            g1state = 1
            absv = [abs(vals[nn]) for nn in sig]
            g1, g2 = [0] * len(sig), [0] * len(sig)
            first_g1 = -1
            for k in range(min(8, len(sig))):
                g1[k] = int(absv[k] > 1)
                enc.decision(self._ctx("gt1", ctx_set * 4 + g1state + (16 if ci else 0)), g1[k])
                if g1[k]:
                    g1state = 0
                    if first_g1 < 0:
                        first_g1 = k
                elif 0 < g1state < 3:
                    g1state += 1
            if first_g1 >= 0:
                g2[first_g1] = int(absv[first_g1] > 2)
                enc.decision(self._ctx("gt2", ctx_set + (4 if ci else 0)), g2[first_g1])
            hidden = sdh and (sig[0] - sig[-1] > 3)
            for k in range(len(sig) - (1 if hidden else 0)):
                enc.bypass(int(vals[sig[k]] < 0))
            rice = 0
            for k in range(len(sig)):
                base = 1 + g1[k] + g2[k]
                thr = (3 if k == first_g1 else 2) if k < 8 else 1
                if base == thr:
                    rem = absv[k] - base
                    if rem < (3 << rice):
                        pre = rem >> rice
                        for _ in range(pre):
                            enc.bypass(1)
                        enc.bypass(0)
                        enc.bypass_bits(rem & ((1 << rice) - 1), rice)
                    else:
                        # prefix P >= 3: value = (((1 << (P-3)) + 2) << rice) + suffix(P - 3 + rice bits)
                        pp = 3
                        while ((((1 << (pp + 1 - 3)) + 2) << rice)) <= rem:
                            pp += 1
                        for _ in range(pp):
                            enc.bypass(1)
                        enc.bypass(0)
                        enc.bypass_bits(rem - ((((1 << (pp - 3)) + 2) << rice)), pp - 3 + rice)
                    if absv[k] > 3 * (1 << rice):
                        rice = min(rice + 1, 4)
        return blk.astype(np.int16), tskip


def sei_nal(payload, nal_type=40, payload_type=132):
    bw = BitWriter()
    t, s = payload_type, len(payload)
    while t >= 255:
        bw.u(255, 8)
        t -= 255
    bw.u(t, 8)
    while s >= 255:
        bw.u(255, 8)
        s -= 255
    bw.u(s, 8)
    for b in payload:
        bw.u(b, 8)
    bw.trailing()
    return nal(nal_type, bw.bytes())


def picture_hash(planes, kind):
    """Decoded picture hash per component (D.3.19): md5 / crc / checksum of 8-bit planes, or of 16-bit
    planes (BitDepth > 8: pictureData holds every sample as two bytes, little-endian; the checksum adds
    (sample >> 8) ^ xorMask per sample too)."""
    out = []
    for c, p in enumerate(planes):
        p = np.ascontiguousarray(p)
        wide = p.dtype == np.uint16
        p = p.astype("<u2") if wide else p.astype(np.uint8)
        if kind == "md5":
            out.append(hashlib.md5(p.tobytes()).digest())
        elif kind == "crc":
            crc = 0xFFFF
            for b in np.frombuffer(p.tobytes(), np.uint8):
                for i in range(8):
                    msb = (crc >> 15) & 1
                    bit = (int(b) >> (7 - i)) & 1
                    crc = (((crc << 1) + bit) & 0xFFFF) ^ (msb * 0x1021)
            for _ in range(16):
                msb = (crc >> 15) & 1
                crc = ((crc << 1) & 0xFFFF) ^ (msb * 0x1021)
            out.append(crc.to_bytes(2, "big"))
        else:
            h, w = p.shape
            ys, xs = np.mgrid[0:h, 0:w]
            xm = (xs & 0xFF) ^ (ys & 0xFF) ^ (xs >> 8) ^ (ys >> 8)
            s = int(np.sum((p.astype(np.int64) & 0xFF) ^ xm))
            if wide:
                s += int(np.sum((p.astype(np.int64) >> 8) ^ xm))
            out.append((s & 0xFFFFFFFF).to_bytes(4, "big"))
    return out
