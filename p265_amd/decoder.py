"""End-to-end all-intra decoder: Annex-B bytes -> native front-end -> MI355X back-end -> YUV.

This is the call stack the reference's ``p265 -b stream.bin -o out.yuv`` (p265:7-20,
dec.py:6-64) would have if its reconstruction worked: parsing runs in
the native front-end (libp265fe.so, host threads), reconstruction + deblocking + SAO
run in the HIP back-end (libp265r.so) in batches of pictures, and the decoded
pictures come back in output order, cropped to the conformance window (sps.py:48-53;
the reference parses it but never uses it), and checked against the stream's
decoded-picture-hash SEI when present (D.3.19).

Streaming: ``decode_chunks`` feeds the parser chunk by chunk on a background thread
(the ctypes calls release the GIL), so parsing overlaps the GPU batches and memory
stays bounded by a few chunks plus one batch; output order follows the bumping
process of C.5.2.2 (``OutputQueue``).  ``decode_file`` streams a file to YUV.

No CPU reconstruction exists on this path: a missing library or GPU raises.
"""
import os
import queue
import threading
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterable, Iterator, List, Optional

import numpy as np

from . import bitstream
from . import recon


@dataclass
class DecodedFrame:
    poc: int
    output_rank: int
    decode_index: int
    planes: list                 # full decoded Y, Cb, Cr (uint8; uint16 above 8 bits), pic_width x pic_height
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


class OutputQueue:
    """Output order: the "bumping" process of C.5.2.2 without the DPB-fullness trigger.

    Inside a coded video sequence a picture leaves, smallest POC first, as soon as more
    than sps_max_num_reorder_pics pictures wait; a new coded video sequence (IRAP with
    NoRaslOutputFlag) or the end of the stream outputs everything waiting."""

    def __init__(self):
        self.waiting = []
        self.cvs = None

    def push(self, item, cvs, poc, max_num_reorder, output_flag):
        out = []
        if self.cvs is not None and cvs != self.cvs:
            out += self.flush()
        self.cvs = cvs
        if output_flag:
            self.waiting.append((poc, item))
        while len(self.waiting) > max_num_reorder:
            k = min(range(len(self.waiting)), key=lambda i: self.waiting[i][0])
            out.append(self.waiting.pop(k)[1])
        return out

    def flush(self):
        out = [it for _, it in sorted(self.waiting, key=lambda e: e[0])]
        self.waiting = []
        return out


def _chunks(data, size):
    for i in range(0, len(data), size):
        yield data[i:i + size]


class StageTimes(dict):
    """Wall time per stage of decode_chunks' consumer thread (seconds), plus the parser thread's
    busy time: a stage breakdown of the end-to-end decoder (tools/e2e_profile.py)."""

    def add(self, k, dt):
        self[k] = self.get(k, 0.0) + dt


# Back-end contexts kept warm across decode calls (one per device and parameter set, like a
# decoder session): a context's first upload pins its staging memory and allocates the batch
# buffer, which a short stream would otherwise pay on every call.  release_contexts() frees them.
_CONTEXT_CACHE = {}                    # key -> [idle ReconContext]
_CONTEXT_LOCK = threading.Lock()


def _param_key(params, scaling):
    """A picture's back-end configuration: its params POD and, with scaling lists, its ScalingFactor table."""
    return params.tobytes() + (b"" if scaling is None else np.asarray(scaling, np.uint8).tobytes())


def _context(params, device, pipeline, scaling=None):
    key = (int(device), _param_key(params, scaling), int(pipeline))
    with _CONTEXT_LOCK:
        idle = _CONTEXT_CACHE.get(key)
        ctx = idle.pop() if idle else None         # checked out: one user at a time
    if ctx is None:
        ctx = recon.ReconContext(params, device=device, scaling=scaling)
        ctx.set_pipeline(max(1, min(16, pipeline)))
    return key, ctx


def _return_context(key, ctx, keep=8):
    with _CONTEXT_LOCK:
        idle = _CONTEXT_CACHE.setdefault(key, [])
        if len(idle) < keep:
            idle.append(ctx)
            return
    ctx.close()


def release_contexts():
    """Free the back-end contexts decode_chunks keeps between calls."""
    with _CONTEXT_LOCK:
        ctxs = [c for idle in _CONTEXT_CACHE.values() for c in idle]
        _CONTEXT_CACHE.clear()
    for c in ctxs:
        c.close()


def host_threads(cap=16):
    """This process's CPU share: affinity, cgroup quota, OMP_NUM_THREADS (the GPU pool announces
    its per-GPU share there), at most ``cap``."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(cap, n))


class _Lane:
    """One back-end context of the decoder and the lock that serialises its calls: the submit
    thread uploads into it while the consumer downloads from another one (contexts are not
    thread-safe, distinct contexts are independent)."""

    def __init__(self, key, ctx):
        self.key, self.ctx, self.lock = key, ctx, threading.Lock()
        self.failed = False             # a batch of it failed: the context is closed, not cached


# end-to-end defaults (tools/e2e_profile.py sweep on the GPU box, 128 x 1080p, 16 host threads; round 4,
# after small batches stopped forking their own streams: 8-picture batches over 4 lanes 504 k CTU/s,
# over 2 lanes 354 k)
DEFAULT_BATCH, DEFAULT_DEPTH, DEFAULT_CHUNK = 8, 4, 1 << 20


def decode_chunks(chunks: Iterable[bytes], device: int = 0, batch: int = DEFAULT_BATCH, threads: int = 0,
                  verify_hash: bool = True, min_batch: int = 8, prefetch: int = 4, depth: int = DEFAULT_DEPTH,
                  stats: Optional[StageTimes] = None, cache_contexts: bool = True) -> Iterator[DecodedFrame]:
    """Decode a stream given as an iterable of byte chunks; yields frames in output order.

    Three stages run concurrently: the parse thread (native front-end on its own host threads),
    the submit thread (groups pictures into GPU batches -- ``batch`` pictures, a parameter-set
    change, or ``min_batch`` when the parser has nothing else ready -- and uploads + enqueues
    them) and the caller's thread (downloads, checks the picture hashes on a host pool, emits in
    output order).  Batches alternate over ``depth`` back-end contexts, so batch k+1 uploads
    while batch k is downloaded; at most ``depth`` batches are in flight.  Contexts stay warm
    between calls (``cache_contexts``; ``release_contexts()`` frees them)."""
    import time
    clock = time.perf_counter
    if not threads:
        threads = host_threads()
    parser = bitstream.StreamParser(threads=threads, asynchronous=True)
    q = queue.Queue(maxsize=max(1, prefetch))
    done_q = queue.Queue()
    depth = max(1, min(16, depth))     # (clamped first: the semaphore and the cleanup use the same value)
    slots = threading.Semaphore(depth)
    stop = threading.Event()
    st = stats if stats is not None else StageTimes()

    def produce():
        # asynchronous parsing: feed() submits the complete access units to the parser's workers
        # and returns the parsed prefix; the number of pictures in the parser is bounded
        try:
            limit = max(8, 3 * (threads or 16))
            for ch in chunks:
                if stop.is_set():
                    q.put(None)         # the submitter ends on it (the consumer drains q)
                    return
                pics = parser.feed(ch)
                if pics:
                    q.put(pics)
                while parser.pending > limit and not stop.is_set():
                    t0 = clock()
                    pics = parser.wait()
                    st.add("parse_backpressure", clock() - t0)
                    if pics:
                        q.put(pics)
            pics = parser.feed(b"", flush=True)
            if pics:
                q.put(pics)
            while parser.pending and not stop.is_set():
                pics = parser.wait()
                if pics:
                    q.put(pics)
            q.put(None)
        except BaseException as e:  # noqa: BLE001 -- handed to the consumer
            q.put(e)

    lanes = {}                          # params bytes -> [_Lane] * depth
    k_submit = [0]

    def lanes_for(params, scaling):
        key = _param_key(params, scaling)
        ls = lanes.get(key)
        if ls is None:
            t0 = clock()
            ls = lanes[key] = [_Lane(*_context(params, device, 1, scaling)) for _ in range(depth)]
            st.add("context", clock() - t0)
        return ls

    def submit(group):
        lane = lanes_for(group[0].params, group[0].scaling)[k_submit[0] % depth]
        k_submit[0] += 1
        slots.acquire()                 # at most `depth` batches between upload and download
        if stop.is_set():
            slots.release()
            return
        with lane.lock:
            t0 = clock()
            b = lane.ctx.upload([d.picture for d in group])     # records -> HBM
            t1 = clock()
            lane.ctx.run(b)                                     # enqueued; decodes meanwhile
        st.add("upload", t1 - t0)
        st.add("run_enqueue", clock() - t1)
        done_q.put((lane, b, group))

    def submitter():
        try:
            pending = []
            while True:
                t0 = clock()
                item = q.get()
                st.add("wait_parser", clock() - t0)
                if isinstance(item, BaseException):
                    raise item
                end = item is None
                for d in item or []:
                    if pending and (len(pending) >= batch or
                                    _param_key(d.params, d.scaling) != _param_key(pending[0].params, pending[0].scaling)):
                        submit(pending)
                        pending = []
                    pending.append(d)
                # the parser has nothing ready right now: decode what is pending instead of waiting
                if pending and (end or (q.empty() and len(pending) >= min_batch)):
                    submit(pending)
                    pending = []
                if end or stop.is_set():
                    break
            done_q.put(None)
        except BaseException as e:  # noqa: BLE001 -- handed to the consumer
            done_q.put(e)

    th_p = threading.Thread(target=produce, name="p265fe-parse", daemon=True)
    th_s = threading.Thread(target=submitter, name="p265r-submit", daemon=True)
    th_p.start()
    th_s.start()
    pool = ThreadPoolExecutor(max_workers=threads)
    outq = OutputQueue()
    rank = 0

    def retire(lane, b, group):
        try:
            with lane.lock:
                t0 = clock()
                try:
                    outs = lane.ctx.download(b)                 # waits for the batch, planes -> host
                except BaseException:
                    lane.failed = True                          # closed at the end, never cached
                    raise
                finally:
                    st.add("download_wait", clock() - t0)
                    b.free()
        finally:
            slots.release()
        ready = []
        for d, planes in zip(group, outs):
            fr = DecodedFrame(poc=d.poc, output_rank=-1, decode_index=int(d.picture.meta["decode_index"]),
                              planes=planes, crop=tuple(int(v) for v in d.crop), hash_ok=None)
            futs = None
            if d.hash is not None:
                futs = [pool.submit(bitstream.plane_hash, planes[c], d.hash_type) for c in range(3)]
            ready += outq.push((fr, d, futs), d.cvs_id, d.poc, d.max_num_reorder, d.output_flag)
        return ready

    def emit(item):
        nonlocal rank
        fr, d, futs = item
        if futs is not None:
            t0 = clock()
            fr.hash_ok = all(f.result() == d.hash[c] for c, f in enumerate(futs))
            st.add("hash_wait", clock() - t0)
            if verify_hash and not fr.hash_ok:
                raise HashMismatch("picture %d (POC %d): decoded picture hash SEI mismatch" % (fr.decode_index, fr.poc))
        fr.output_rank = rank
        rank += 1
        return fr

    try:
        while True:
            t0 = clock()
            item = done_q.get()
            st.add("wait_submit", clock() - t0)
            if isinstance(item, BaseException):
                raise item
            if item is None:
                break
            for it in retire(*item):
                yield emit(it)
        for it in outq.flush():
            yield emit(it)
    finally:
        stop.set()
        for _ in range(depth):
            slots.release()             # a submitter blocked on a slot sees `stop`
        while th_p.is_alive() or th_s.is_alive():
            for qq in (q, done_q):
                try:
                    left = qq.get(timeout=0.02)
                except queue.Empty:
                    continue
                if isinstance(left, tuple) and len(left) == 3:
                    lane, b, _ = left
                    with lane.lock:
                        b.free()
        while True:                     # batches submitted but never retired
            try:
                left = done_q.get_nowait()
            except queue.Empty:
                break
            if isinstance(left, tuple) and len(left) == 3:
                lane, b, _ = left
                with lane.lock:
                    b.free()
        pool.shutdown(wait=True)
        t0 = clock()
        for ls in lanes.values():
            for lane in ls:
                if cache_contexts and not lane.failed:
                    _return_context(lane.key, lane.ctx)
                else:
                    lane.ctx.close()
        st.add("context", clock() - t0)


def decode_bytes(data: bytes, device: int = 0, batch: int = DEFAULT_BATCH, threads: int = 0,
                 verify_hash: bool = True, chunk: int = DEFAULT_CHUNK, **kw) -> List[DecodedFrame]:
    """Decode a whole stream held in memory; returns the output pictures in output order."""
    return list(decode_chunks(_chunks(data, chunk), device=device, batch=batch, threads=threads,
                              verify_hash=verify_hash, **kw))


def _file_chunks(path, chunk):
    with open(path, "rb") as f:
        while True:
            b = f.read(chunk)
            if not b:
                return
            yield b


def decode_file(path: str, output: Optional[str] = None, chunk: int = DEFAULT_CHUNK, **kw) -> dict:
    """Stream a bitstream file to a cropped I420 YUV file in output order; returns counts."""
    n = checked = bad = 0
    f = open(output, "wb") if output else None
    try:
        for fr in decode_chunks(_file_chunks(path, chunk), **kw):
            n += 1
            if fr.hash_ok is not None:
                checked += 1
                bad += int(not fr.hash_ok)
            if f:
                for p in fr.cropped():
                    f.write(np.ascontiguousarray(p).tobytes())
    finally:
        if f:
            f.close()
    return {"pictures": n, "hash_checked": checked, "hash_mismatch": bad}


def write_yuv(frames: List[DecodedFrame], path: str):
    """Planar 4:2:0 8-bit YUV (I420), cropped, in output order."""
    with open(path, "wb") as f:
        for fr in frames:
            for p in fr.cropped():
                f.write(np.ascontiguousarray(p).tobytes())
