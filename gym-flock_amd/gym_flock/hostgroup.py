"""Torch-free host channel for the multi-rank path (one process per GPU).

The env batch shards over ranks with no exchange on the step path; the
only device collective is the RCCL reward all-gather inside libgymflock. What the ranks
still need on the host is small: the RCCL unique id from rank 0, barriers around the
timed region, the max of the ranks' times, and the local rewards that every rank uses
to check the whole gathered vector. HostGroup provides exactly that over plain TCP
sockets, so a GPU worker never imports torch (whose bundled HIP runtime and RCCL the
loader would otherwise bind libgymflock to, instead of the ROCm it was built against).

Topology: a star. Rank 0 listens on (MASTER_ADDR, port) and relays; every other rank
connects to it. Every operation is collective (all ranks call it in the same order).
Launchers: torchrun (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment;
torchrun's own store holds MASTER_PORT, so the default port is MASTER_PORT + 1, or
GYMFLOCK_HOST_PORT), bench.py's own launcher, or explicit arguments.

Messages are raw bytes or fixed-format struct values (float64, int64, bool); nothing
received is ever unpickled or evaluated. A shared token (GYMFLOCK_HOST_TOKEN, set by
bench.py's launcher) must accompany every rank's hello, so a stray local process that
reaches rank 0's port during the rendezvous is refused: its connection is dropped (as is
one that sends nothing within HELLO_TIMEOUT, a bad rank or a duplicate) and the
rendezvous goes on until every rank has joined or the timeout passes.
"""
import hmac
import os
import socket
import struct
import time

_HDR = struct.Struct("!Q")
_TOKEN_LEN = 32


def _send(sock, payload):
    sock.sendall(_HDR.pack(len(payload)) + payload)


def _recv_exact(sock, n):
    buf = bytearray(n)
    view, got = memoryview(buf), 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("hostgroup: peer closed the connection")
        got += k
    return bytes(buf)


def _recv(sock):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


class HostGroup:
    """rank, world: this process's rank and the number of ranks. addr, port: rank 0's
    listening address. timeout: seconds to wait for the rendezvous and for each op."""

    def __init__(self, rank, world, addr="127.0.0.1", port=29501, timeout=300.0, token=b""):
        self.rank, self.world = int(rank), int(world)
        token = (bytes(token) + bytes(_TOKEN_LEN))[:_TOKEN_LEN]
        if not (0 <= self.rank < self.world):
            raise ValueError("rank out of range")
        self.peers = {}  # rank 0: rank -> socket
        self.up = None   # other ranks: socket to rank 0
        self.refused = []  # rank 0: addresses of connections dropped in the rendezvous
        if self.world == 1:
            return
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, int(port)))
            srv.listen(self.world + 4)
            ok = False
            try:
                while len(self.peers) < self.world - 1:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        raise TimeoutError("hostgroup: %d of %d ranks joined before the rendezvous timeout"
                                           % (len(self.peers) + 1, self.world))
                    srv.settimeout(left)
                    try:
                        c, who = srv.accept()
                    except socket.timeout:
                        continue
                    r = self._hello(c, token, min(self.HELLO_TIMEOUT, max(0.1, deadline - time.monotonic())))
                    if r is None:
                        # a stray or broken client: dropped, the rendezvous goes on
                        c.close()
                        self.refused.append(who)
                        continue
                    c.settimeout(timeout)
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    self.peers[r] = c
                ok = True
            finally:
                srv.close()
                if not ok:
                    self.close()
        else:
            while True:
                try:
                    s = socket.create_connection((addr, int(port)), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise TimeoutError("hostgroup: rank 0 at %s:%s not reachable" % (addr, port))
                    time.sleep(0.1)
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("!I", self.rank) + token)
            self.up = s

    HELLO_TIMEOUT = 5.0  # seconds a connecting peer has to present its rank and token

    def _hello(self, c, token, limit):
        """The rank a new connection announces, or None (short read, timeout, wrong token,
        bad or duplicate rank): the caller drops such a connection."""
        try:
            c.settimeout(limit)
            hello = _recv_exact(c, 4 + _TOKEN_LEN)
        except (OSError, ConnectionError):
            return None
        (r,) = struct.unpack("!I", hello[:4])
        if not hmac.compare_digest(hello[4:], token):
            return None
        if not (0 < r < self.world) or r in self.peers:
            return None
        return r

    @classmethod
    def from_env(cls, timeout=300.0):
        """The group torchrun describes (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT)."""
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("GYMFLOCK_HOST_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        token = bytes.fromhex(os.environ.get("GYMFLOCK_HOST_TOKEN", ""))
        return cls(rank, world, addr, port, timeout, token)

    # ---------------------------------------------------------------- collectives
    def allgather_bytes(self, payload):
        """Every rank's bytes, in rank order, on every rank."""
        payload = bytes(payload)
        if self.world == 1:
            return [payload]
        if self.rank == 0:
            parts = [payload] + [_recv(self.peers[r]) for r in range(1, self.world)]
            blob = b"".join(_HDR.pack(len(p)) + p for p in parts)
            for r in range(1, self.world):
                _send(self.peers[r], blob)
            return parts
        _send(self.up, payload)
        blob, parts, off = _recv(self.up), [], 0
        for _ in range(self.world):
            (n,) = _HDR.unpack_from(blob, off)
            off += _HDR.size
            parts.append(blob[off:off + n])
            off += n
        return parts

    def _allgather_struct(self, fmt, value):
        st = struct.Struct(fmt)
        out = []
        for p in self.allgather_bytes(st.pack(value)):
            if len(p) != st.size:
                raise RuntimeError("hostgroup: malformed %r message (%d bytes)" % (fmt, len(p)))
            out.append(st.unpack(p)[0])
        return out

    def allgather_f64(self, value):
        return self._allgather_struct("!d", float(value))

    def allgather_i64(self, value):
        return self._allgather_struct("!q", int(value))

    def allgather_bool(self, value):
        return self._allgather_struct("!?", bool(value))

    def barrier(self):
        self.allgather_bytes(b"")

    def broadcast_bytes(self, payload, src=0):
        return self.allgather_bytes(payload if self.rank == src else b"")[src]

    def max(self, value):
        return max(self.allgather_f64(value))

    def close(self):
        for s in list(self.peers.values()) + ([self.up] if self.up else []):
            try:
                s.close()
            except OSError:
                pass
        self.peers, self.up = {}, None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
