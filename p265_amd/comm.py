"""Control-plane communicator over stdlib TCP sockets (no PyTorch).

One process per GPU; the data path needs no collective (pictures and tiles
are independent), so the ranks only need a control plane: the rendezvous that hands out
the RCCL unique id (p265_amd/rccl.py), barriers around the timed region, the MAX of the
elapsed times, gathering per-unit digests in tests, and (without RCCL, e.g. CPU tests)
the bytes of the SPS/PPS POD and of tile halos.

Star topology through rank 0: rank 0 listens on (addr, port), every other rank connects
once and announces its rank.  Every operation is collective (all ranks call it in the
same order); messages are length-prefixed.  Ranks launched by torch.distributed.run get
MASTER_ADDR / MASTER_PORT; the agent's own store holds MASTER_PORT, so the control plane
uses MASTER_PORT + 1 unless P265_CTRL_PORT says otherwise (``from_env``).
"""
import os
import socket
import struct
import time

_HDR = struct.Struct("<Q")


def _send(sock, data):
    sock.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(sock, n):
    out = bytearray()
    while len(out) < n:
        chunk = sock.recv(min(n - len(out), 1 << 20))
        if not chunk:
            raise ConnectionError("control-plane peer closed the connection")
        out += chunk
    return bytes(out)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


def pack_map(m):
    """{int: bytes} -> bytes"""
    parts = [struct.pack("<I", len(m))]
    for k in sorted(m):
        v = bytes(m[k])
        parts.append(struct.pack("<qQ", int(k), len(v)))
        parts.append(v)
    return b"".join(parts)


def unpack_map(b):
    (n,), off, out = struct.unpack_from("<I", b, 0), 4, {}
    for _ in range(n):
        k, ln = struct.unpack_from("<qQ", b, off)
        off += 16
        out[k] = b[off:off + ln]
        off += ln
    return out


class SocketComm:
    def __init__(self, rank, world, addr="127.0.0.1", port=29500, timeout=300.0):
        self.rank, self.world = int(rank), int(world)
        self.peers = {}                  # rank 0: {rank: socket}
        self.sock = None                 # other ranks: socket to rank 0
        self._listener = None
        if self.world == 1:
            return
        deadline = time.time() + timeout
        if self.rank == 0:
            ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            ls.bind((addr, int(port)))
            ls.listen(self.world)
            ls.settimeout(max(1.0, deadline - time.time()))
            self._listener = ls
            while len(self.peers) < self.world - 1:
                s, _ = ls.accept()
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                s.settimeout(timeout)
                (r,) = struct.unpack("<i", _recv(s))
                if r <= 0 or r >= self.world or r in self.peers:
                    raise ConnectionError("control plane: unexpected rank %d" % r)
                self.peers[r] = s
        else:
            while True:
                try:
                    s = socket.create_connection((addr, int(port)), timeout=5.0)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(timeout)
            _send(s, struct.pack("<i", self.rank))
            self.sock = s

    @classmethod
    def from_env(cls, timeout=300.0):
        rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("P265_CTRL_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        return cls(rank, world, addr, port, timeout)

    # ---- collectives (every rank calls them in the same order) ----------------------
    def gather(self, data: bytes):
        """-> [bytes of rank 0, 1, ...] on rank 0, None elsewhere."""
        if self.world == 1:
            return [bytes(data)]
        if self.rank == 0:
            return [bytes(data)] + [_recv(self.peers[r]) for r in range(1, self.world)]
        _send(self.sock, bytes(data))
        return None

    def bcast(self, data: bytes = b"", src=0) -> bytes:
        if self.world == 1:
            return bytes(data)
        if src != 0:                     # relay through rank 0
            if self.rank == src:
                _send(self.sock, bytes(data))
            if self.rank == 0:
                data = _recv(self.peers[src])
            src = 0
        if self.rank == 0:
            for r in range(1, self.world):
                _send(self.peers[r], bytes(data))
            return bytes(data)
        return _recv(self.sock)

    def allgather(self, data: bytes):
        parts = self.gather(data)
        packed = self.bcast(pack_map(dict(enumerate(parts))) if self.rank == 0 else b"")
        m = unpack_map(packed)
        return [m[r] for r in range(self.world)]

    def barrier(self):
        self.allgather(b"")

    def max(self, value: float) -> float:
        return max(struct.unpack("<d", b)[0] for b in self.allgather(struct.pack("<d", float(value))))

    def alltoall(self, sends):
        """sends: {dst_rank: bytes} -> {src_rank: bytes} (routed through rank 0)."""
        if self.world == 1:
            return {0: sends[0]} if 0 in sends else {}
        outgoing = self.gather(pack_map(sends))
        if self.rank == 0:
            inbox = {r: {} for r in range(self.world)}
            for src, packed in enumerate(outgoing):
                for dst, payload in unpack_map(packed).items():
                    inbox[int(dst)][src] = payload
            for r in range(1, self.world):
                _send(self.peers[r], pack_map(inbox[r]))
            return inbox[0]
        return unpack_map(_recv(self.sock))

    def close(self):
        for s in self.peers.values():
            s.close()
        self.peers = {}
        if self.sock:
            self.sock.close()
            self.sock = None
        if self._listener:
            self._listener.close()
            self._listener = None
