"""Host API of the MI355X reconstruction back-end (Python side of the C ABI).

Mirrors what the reference's reconstruction hook would do per picture
(decoder/cu.py:483-494 -> decode_intra, decoder/sao.py), but per batch:

    ctx = ReconContext(params, device=0)
    frames = ctx.decode([pic0, pic1, ...])          # -> [(Y, Cb, Cr), ...] planes (uint8; uint16 > 8 bits)

or, keeping inputs resident in HBM (the benchmark path):

    batch = ctx.upload(pics); ctx.run(batch); ctx.sync(); frames = ctx.download(batch)

Errors raise ``P265RError`` (negative C return codes); there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib
from . import records as R


def _params_c(p):
    c = _lib.Params()
    for name, _ in _lib.Params._fields_:
        if name == "reserved":
            continue
        setattr(c, name, int(p[name]))
    return c


def plane_shapes(params):
    w, h = int(params["pic_width"]), int(params["pic_height"])
    return [(h, w), (h // 2, w // 2), (h // 2, w // 2)]


class DecodedPicture:
    """One decoded picture, served back to the reference's read-back surface.

    ``get_reconstructed_sample(x, y, c_idx)`` has the semantics of Cu.get_reconstructed_sample
    (decoder/cu.py:617-632): (x, y) in LUMA coordinates for every component (chroma: the
    sample at (x >> 1, y >> 1) of its plane, cu.py:624-630), returning the reconstruction
    before the in-loop filters (pu.reconstructed_samples, reconstruction.py:25), which is what
    intra prediction of later blocks reads.  ``get_output_sample`` returns the decoded
    (deblocked + SAO) sample that is written out.  ``planes`` / ``recon`` are [Y, Cb, Cr]
    arrays indexed [y][x] (the reference's arrays are x-major [x][y]): uint8 at BitDepth 8, uint16
    above (Main 10)."""

    def __init__(self, planes, recon):
        self.planes, self.recon = planes, recon

    @staticmethod
    def _at(planes, x, y, c_idx):
        sub = 1 if c_idx else 0
        return int(planes[c_idx][y >> sub, x >> sub])

    def get_reconstructed_sample(self, x, y, c_idx):
        return self._at(self.recon, x, y, c_idx)

    def get_output_sample(self, x, y, c_idx):
        return self._at(self.planes, x, y, c_idx)


class Batch:
    def __init__(self, ctx, handle, pics, keep):
        self.ctx, self.handle, self.pics, self._keep = ctx, handle, pics, keep

    def free(self):
        if self.handle:
            _lib.check(self.ctx.lib.p265r_batch_free(self.ctx.handle, self.handle), "p265r_batch_free")
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class ReconContext:
    """One HIP device + stream + parameter set (p265r_ctx)."""

    def __init__(self, params, device=0, scaling=None):
        """``scaling``: the 2032-byte intra ScalingFactor table (p265r_set_scaling_factors) when
        params.scaling_list_enabled."""
        self.lib = _lib.load()
        self.params = params
        self._pc = _params_c(params)
        h = ctypes.c_void_p()
        _lib.check(self.lib.p265r_create(device, ctypes.byref(self._pc), ctypes.byref(h)), "p265r_create")
        self.handle = h
        self.device = device
        if scaling is not None:
            self.set_scaling_factors(scaling)

    def set_scaling_factors(self, factors):
        """The intra ScalingFactor table (2032 bytes, include/p265r.h) for every later run."""
        f = np.ascontiguousarray(factors, np.uint8).reshape(-1)
        _lib.check(self.lib.p265r_set_scaling_factors(self.handle, f.ctypes.data, int(f.size)),
                   "p265r_set_scaling_factors")

    def close(self):
        if getattr(self, "handle", None):
            self.lib.p265r_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- marshalling ------------------------------------------------------------
    def _pictures_c(self, pics, outs=None, recons=None):
        keep = []
        arr = (_lib.PictureC * len(pics))()
        for i, p in enumerate(pics):
            R.check_shapes(self.params, p)      # record contents: validated by p265r_batch_upload
            pp = R.pic_params(self.params, p)
            if pp is not self.params:           # a smaller picture of a ragged batch
                arr[i].pic_width, arr[i].pic_height = int(pp["pic_width"]), int(pp["pic_height"])
            ctus = np.ascontiguousarray(p.ctus, R.CTU_DTYPE)
            tbs = np.ascontiguousarray(p.tbs, R.TB_DTYPE)
            coef = np.ascontiguousarray(p.coef, np.int16)
            keep += [ctus, tbs, coef]
            c = arr[i]
            c.ctus = ctus.ctypes.data
            c.tbs = tbs.ctypes.data if len(tbs) else None
            c.n_tbs = len(tbs)
            c.coef = coef.ctypes.data if len(coef) else None
            c.n_coef = len(coef)
            if p.nofilter is not None:
                nf = np.ascontiguousarray(p.nofilter, np.uint8)
                keep.append(nf)
                c.nofilter = nf.ctypes.data
            for k in range(3):
                if outs is not None:
                    c.out[k] = outs[i][k].ctypes.data
                if recons is not None:
                    c.recon[k] = recons[i][k].ctypes.data
            if p.recon_input is not None:
                c.flags = R.PIC_RECON_INPUT
                dts = R.plane_dtypes(self.params)
                planes = [np.ascontiguousarray(p.recon_input[k], dts[k]) for k in range(3)]
                for k, (pl, shp) in enumerate(zip(planes, plane_shapes(pp))):
                    if pl.shape != shp:
                        raise R.RecordError("recon_input plane %d has shape %s, expected %s" % (k, pl.shape, shp))
                    c.recon[k] = pl.ctypes.data
                keep += planes
        return arr, keep

    def _alloc_planes(self, pics):
        dts = R.plane_dtypes(self.params)
        return [[np.empty(s, dt) for s, dt in zip(plane_shapes(R.pic_params(self.params, p)), dts)] for p in pics]

    # ---- batch API --------------------------------------------------------------
    def upload(self, pics):
        arr, keep = self._pictures_c(pics)
        h = ctypes.c_void_p()
        _lib.check(self.lib.p265r_batch_upload(self.handle, arr, len(pics), ctypes.byref(h)), "p265r_batch_upload")
        return Batch(self, h, pics, keep)

    def run(self, batch):
        _lib.check(self.lib.p265r_batch_run(self.handle, batch.handle), "p265r_batch_run")

    def download(self, batch, with_recon=False, only=None, into=None):
        """Planes of the batch's pictures (after its last run).  ``only``: indices of the pictures
        to copy back (the others are not transferred and come back as None).  ``into``: the output
        planes to fill instead of new arrays (a frame pool: per picture three C-contiguous arrays of the
        planes' shapes and dtype, e.g. a previous download's result) -- fresh host memory costs a page
        fault per 4 KB on its first write."""
        n = len(batch.pics)
        sel = set(range(n)) if only is None else {int(i) for i in only}
        shp = [plane_shapes(R.pic_params(self.params, p)) for p in batch.pics]
        dts = R.plane_dtypes(self.params)
        if into is not None:
            if len(into) != n:
                raise ValueError("into: one entry per picture")
            for i in sel:
                for k in range(3):
                    a = into[i][k]
                    if a.shape != tuple(shp[i][k]) or a.dtype != dts[k] or not a.flags.c_contiguous or not a.flags.writeable:
                        raise ValueError("into: picture %d plane %d does not match the plane layout" % (i, k))
            outs = [list(into[i]) if i in sel else None for i in range(n)]
        else:
            outs = [[np.empty(s, dt) for s, dt in zip(shp[i], dts)] if i in sel else None for i in range(n)]
        recs = ([[np.empty(s, dt) for s, dt in zip(shp[i], dts)] if i in sel else None for i in range(n)]
                if with_recon else None)
        arr = (_lib.PictureC * n)()
        for i in sel:
            for k in range(3):
                arr[i].out[k] = outs[i][k].ctypes.data
                if recs is not None:
                    arr[i].recon[k] = recs[i][k].ctypes.data
        _lib.check(self.lib.p265r_batch_download(self.handle, batch.handle, arr, n), "p265r_batch_download")
        return (outs, recs) if with_recon else outs

    def status(self, batch):
        """Wait for the batch and raise P265RError if any of its runs failed on the device
        (p265r_batch_status: the row kernel's sticky error word)."""
        _lib.check(self.lib.p265r_batch_status(self.handle, batch.handle), "p265r_batch_status")

    def digest(self, batch, recon=False):
        """Per-picture digests of the batch's planes after its last run, computed on the device
        (p265r_batch_digest; no plane download): uint64 array [n_pictures, 3] (Y, Cb, Cr), equal to
        digest.picture_digest() of the planes download() would return (recon: the reconstruction
        before the in-loop filters).  Raises P265RError like status()."""
        n = len(batch.pics)
        out = np.zeros(3 * n, np.uint64)
        _lib.check(self.lib.p265r_batch_digest(self.handle, batch.handle, 1 if recon else 0,
                                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), 3 * n),
                   "p265r_batch_digest")
        return out.reshape(n, 3)

    def digest_async(self, batch, slot, recon=False):
        """Enqueue the device digest of the batch's planes after every run enqueued so far into digest
        slot ``slot`` (0 .. _lib.DIGEST_SLOTS - 1) and return at once (p265r_batch_digest_async)."""
        _lib.check(self.lib.p265r_batch_digest_async(self.handle, batch.handle, 1 if recon else 0, int(slot)),
                   "p265r_batch_digest_async")

    def digest_slots(self, batch, n_slots):
        """Wait for the batch's lane; -> uint64 array [n_slots, n_pictures, 3] of the digest slots
        (p265r_batch_digest_slots).  Raises P265RError like status()."""
        n = len(batch.pics)
        out = np.zeros(3 * n * n_slots, np.uint64)
        _lib.check(self.lib.p265r_batch_digest_slots(self.handle, batch.handle,
                                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), int(n_slots)),
                   "p265r_batch_digest_slots")
        return out.reshape(n_slots, n, 3)

    def job_count(self, batch):
        """(luma, chroma) intra jobs of the batch's last run (p265r_batch_job_count)."""
        lu, ch = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _lib.check(self.lib.p265r_batch_job_count(self.handle, batch.handle, ctypes.byref(lu), ctypes.byref(ch)),
                   "p265r_batch_job_count")
        return int(lu.value), int(ch.value)

    def sync(self):
        _lib.check(self.lib.p265r_sync(self.handle), "p265r_sync")

    def set_pipeline(self, depth):
        """Bind batches uploaded from now on round-robin to `depth` streams (p265r_set_pipeline)."""
        _lib.check(self.lib.p265r_set_pipeline(self.handle, int(depth)), "p265r_set_pipeline")

    def set_row_waves(self, waves):
        """Force the row kernel's build (8 / 12 waves per workgroup) or 0 = by run (p265r_set_row_waves)."""
        _lib.check(self.lib.p265r_set_row_waves(self.handle, int(waves)), "p265r_set_row_waves")

    def set_timing(self, on=True):
        _lib.check(self.lib.p265r_set_timing(self.handle, int(bool(on))), "p265r_set_timing")

    def timings_total(self):
        """Sums of the per-phase times over every run since set_timing(True), and the run count."""
        t = _lib.Timings()
        n = ctypes.c_int(0)
        _lib.check(self.lib.p265r_timings_total(self.handle, ctypes.byref(t), ctypes.byref(n)), "p265r_timings_total")
        d = {f: getattr(t, f) for f, _ in _lib.Timings._fields_ if f != "reserved"}
        d["runs"] = n.value
        return d

    def describe(self):
        """Effective configuration of this context (p265r_describe) as a dict."""
        import json
        buf = ctypes.create_string_buffer(1024)
        n = _lib.check(self.lib.p265r_describe(self.handle, buf, len(buf)), "p265r_describe")
        if n >= len(buf):
            buf = ctypes.create_string_buffer(n + 1)
            _lib.check(self.lib.p265r_describe(self.handle, buf, len(buf)), "p265r_describe")
        return json.loads(buf.value.decode())

    def last_timings(self):
        t = _lib.Timings()
        _lib.check(self.lib.p265r_last_timings(self.handle, ctypes.byref(t)), "p265r_last_timings")
        return {f: getattr(t, f) for f, _ in _lib.Timings._fields_ if f != "reserved"}

    # ---- one-shot API (submit / wait) -------------------------------------------------
    def decode(self, pics, with_recon=False):
        outs = self._alloc_planes(pics)
        recs = self._alloc_planes(pics) if with_recon and pics[0].recon_input is None else None
        arr, keep = self._pictures_c(pics, outs, recs)
        _lib.check(self.lib.p265r_submit(self.handle, arr, len(pics)), "p265r_submit")
        _lib.check(self.lib.p265r_wait(self.handle), "p265r_wait")
        del keep
        return (outs, recs) if with_recon else outs


def decode_pictures(ctx, pics):
    """ReconContext.decode with the reconstruction too, as DecodedPicture objects (the
    read-back surface of decoder/cu.py:617-632)."""
    outs, recs = ctx.decode(pics, with_recon=True)
    return [DecodedPicture(o, r) for o, r in zip(outs, recs)]


def device_count():
    return _lib.check(_lib.load().p265r_device_count(), "p265r_device_count")
