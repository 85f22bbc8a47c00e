"""Host rendezvous of the processes of a one-process-per-device group (wcpt_group_create_rank), with no torch.

A group of N processes needs three small host exchanges and nothing else: the root's 128-byte RCCL id
(wcpt_group_unique_id) to every process before wcpt_group_create_rank, barriers around a timed region, and a gather of
per-rank numbers (times, work counters) to rank 0. The frames themselves travel over RCCL (xGMI). The reference host
is one process (src/main.jai:185-194), so it has no counterpart; this is what lets the product's own runtime (the
system HIP runtime libwcpt.so binds, as a Jai host would) run one process per GPU under torchrun without importing
torch -- torch brings its own HIP runtime into the process.

Transport: TCP on the host network. Rank 0 listens on the first free port of [port, port + span); ranks 1..N-1 try
those ports in turn (until `timeout`), and a connection counts only after a handshake: the client sends a magic word,
a job token and its rank, the hub answers with its magic word. So a port taken by an unrelated program, or by another
job's rendezvous, is skipped rather than hung on. Messages are length-prefixed byte strings. Under torchrun,
`from_env` starts at MASTER_PORT + 1 (torchrun's own store holds MASTER_PORT), or at WCPT_RDZV_PORT, and derives the
token from MASTER_PORT, WORLD_SIZE and TORCHELASTIC_RUN_ID.
"""
from __future__ import annotations

import hashlib
import json
import os
import socket
import struct
import time

MAGIC_CLIENT = b"WCPTRDZ1"
MAGIC_HUB = b"WCPTRDZA"
MAGIC_ACK = b"WCPTRDZK"
# The hub serves connections one at a time and gives each HELLO_S to send its hello; a client waits longer than that
# for the hub's answer, and the hub registers a client only once the client has acknowledged the answer, so a client
# that gave up (and closed) is never registered in place of its own retry.
HELLO_S = 5.0
CLIENT_WAIT_S = 2 * HELLO_S


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

    def __init__(self, rank: int, world: int, addr: str = "127.0.0.1", port: int = 29600, timeout: float = 300.0,
                 token: bytes = b"", span: int = 32):
        if world < 1 or not 0 <= rank < world:
            raise ValueError(f"rank {rank} of {world}")
        self.rank, self.world = rank, world
        self.peers: dict[int, socket.socket] = {}
        self.hub: socket.socket | None = None
        self._server: socket.socket | None = None
        self.port = None
        if world == 1:
            return
        tok = hashlib.sha256(token).digest()[:16]
        deadline = time.monotonic() + timeout
        if rank == 0:
            srv = None
            for p in range(port, port + span):
                s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                try:
                    s.bind((addr, p))
                except OSError:
                    s.close()
                    continue
                srv, self.port = s, p
                break
            if srv is None:
                raise RendezvousError(f"rank 0: no free port in [{port}, {port + span}) on {addr}")
            srv.listen(4 * world)
            self._server = srv
            while len(self.peers) < world - 1:
                srv.settimeout(max(0.1, deadline - time.monotonic()))
                try:
                    c, _ = srv.accept()
                except socket.timeout:
                    raise RendezvousError(f"rank 0: {len(self.peers)} of {world - 1} peers connected before the "
                                          f"timeout") from None
                try:
                    c.settimeout(HELLO_S)
                    hello = _recv_exact(c, len(MAGIC_CLIENT) + len(tok) + 4)
                except (OSError, RendezvousError):
                    c.close()
                    continue
                r = struct.unpack("<I", hello[-4:])[0]
                if hello[:len(MAGIC_CLIENT)] != MAGIC_CLIENT or hello[len(MAGIC_CLIENT):-4] != tok or \
                        not 0 < r < world or r in self.peers:
                    c.close()                          # another job, or not a rendezvous client at all
                    continue
                try:
                    c.sendall(MAGIC_HUB)
                    if _recv_exact(c, len(MAGIC_ACK)) != MAGIC_ACK:
                        raise RendezvousError("bad acknowledgement")
                except (OSError, RendezvousError):
                    c.close()                          # the client gave up before the answer: it will retry
                    continue
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.settimeout(timeout)
                self.peers[r] = c
        else:
            hello = MAGIC_CLIENT + tok + struct.pack("<I", rank)
            while self.hub is None:
                for p in range(port, port + span):
                    try:
                        c = socket.create_connection((addr, p), timeout=2.0)
                    except OSError:
                        continue
                    try:
                        c.settimeout(CLIENT_WAIT_S)
                        c.sendall(hello)
                        if _recv_exact(c, len(MAGIC_HUB)) == MAGIC_HUB:
                            c.sendall(MAGIC_ACK)
                            c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                            c.settimeout(timeout)
                            self.hub, self.port = c, p
                            break
                    except (OSError, RendezvousError):
                        pass
                    c.close()
                if self.hub is None:
                    if time.monotonic() > deadline:
                        raise RendezvousError(f"rank {rank}: no rendezvous hub on {addr}:[{port}, {port + span})")
                    time.sleep(0.05)

    @classmethod
    def from_env(cls, timeout: float = 300.0) -> "Rendezvous":
        """RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT as torchrun sets them; the port is MASTER_PORT + 1 (or
        WCPT_RDZV_PORT)."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        master = os.environ.get("MASTER_PORT", "29500")
        port = int(os.environ.get("WCPT_RDZV_PORT", int(master) + 1))
        token = f"{master}/{world}/{os.environ.get('TORCHELASTIC_RUN_ID', '')}".encode()
        return cls(rank, world, addr, port, timeout, token=token)

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
