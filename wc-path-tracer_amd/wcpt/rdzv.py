"""Host rendezvous of the processes of a one-process-per-device group (wcpt_group_create_rank), with no torch.

A group of N processes needs three small host exchanges and nothing else: the root's 128-byte RCCL id
(wcpt_group_unique_id) to every process before wcpt_group_create_rank, barriers around a timed region, and a gather of
per-rank numbers (times, work counters) to rank 0. The frames themselves travel over RCCL (xGMI). The reference host
is one process (src/main.jai:185-194), so it has no counterpart; this is what lets the product's own runtime (the
system HIP runtime libwcpt.so binds, as a Jai host would) run one process per GPU under torchrun without importing
torch -- torch brings its own HIP runtime into the process.

Transport: TCP on the host network. Rank 0 listens on (addr, port); ranks 1..N-1 connect (retrying until `timeout`)
and announce their rank; messages are length-prefixed byte strings. Under torchrun, `from_env` takes MASTER_ADDR and
MASTER_PORT + 1 (torchrun's own store holds MASTER_PORT), or WCPT_RDZV_PORT.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time


class RendezvousError(RuntimeError):
    pass


def _send(sock: socket.socket, data: bytes):
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise RendezvousError("peer closed the rendezvous connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket) -> bytes:
    (n,) = struct.unpack("<Q", _recv_exact(sock, 8))
    return _recv_exact(sock, n)


class Rendezvous:
    """Rank `rank` of `world` host processes. Rank 0 is the hub."""

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29600, timeout: float = 300.0):
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"rank {rank} of {world}")
        self.rank, self.world = rank, world
        self.peers: dict[int, socket.socket] = {}
        self.hub: socket.socket | None = None
        self._server: socket.socket | None = None
        if world == 1:
            return
        deadline = time.monotonic() + timeout
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(max(0.1, deadline - time.monotonic()))
            self._server = srv
            while len(self.peers) < world - 1:
                try:
                    c, _ = srv.accept()
                except socket.timeout:
                    raise RendezvousError(f"rank 0: {len(self.peers)} of {world - 1} peers connected before the "
                                          f"timeout") from None
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.settimeout(timeout)
                (r,) = struct.unpack("<I", _recv_exact(c, 4))
                if not 0 < r < world or r in self.peers:
                    c.close()
                    raise RendezvousError(f"rank 0: unexpected peer rank {r}")
                self.peers[r] = c
        else:
            while True:
                try:
                    c = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise RendezvousError(f"rank {rank}: no rendezvous at {addr}:{port}") from None
                    time.sleep(0.05)
            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c.settimeout(timeout)
            c.sendall(struct.pack("<I", rank))
            self.hub = c

    @classmethod
    def from_env(cls, timeout: float = 300.0) -> "Rendezvous":
        """RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as torchrun sets them; the port is MASTER_PORT + 1 (or
        WCPT_RDZV_PORT)."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("WCPT_RDZV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        return cls(rank, world, addr, port, timeout)

    # -- collectives over small host messages ---------------------------------------------------------------
    def broadcast(self, data: bytes | None = None) -> bytes:
        """Rank 0's `data` on every rank."""
        if self.world == 1:
            return data or b""
        if self.rank == 0:
            for r in sorted(self.peers):
                _send(self.peers[r], data or b"")
            return data or b""
        return _recv(self.hub)

    def gather(self, data: bytes) -> list[bytes] | None:
        """Every rank's `data`, in rank order, on rank 0 (None elsewhere)."""
        if self.world == 1:
            return [data]
        if self.rank == 0:
            return [data] + [_recv(self.peers[r]) for r in range(1, self.world)]
        _send(self.hub, data)
        return None

    def gather_obj(self, obj):
        got = self.gather(json.dumps(obj).encode())
        return None if got is None else [json.loads(g) for g in got]

    def allgather_obj(self, obj) -> list:
        got = self.gather_obj(obj)
        return json.loads(self.broadcast(json.dumps(got).encode() if self.rank == 0 else None))

    def barrier(self):
        self.gather(b"")
        self.broadcast(b"")

    def close(self):
        for s in list(self.peers.values()) + [self.hub, self._server]:
            if s is not None:
                try:
                    s.close()
                except OSError:
                    pass
        self.peers, self.hub, self._server = {}, None, None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
