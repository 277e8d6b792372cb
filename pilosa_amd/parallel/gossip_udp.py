"""UDP probe transport of the failure detector on ``[gossip] port``.

Reference: memberlist (gossip/gossip.go:525-597) listens on the gossip port
(default 14000) for its UDP ping / ack / indirect ping-req messages and, with
``gossip.key``, encrypts them with the 16/24/32-byte key (AES-GCM).  Here the
SWIM detector (parallel/swim.py) probes peers through this transport when the
port is configured:

* ``PING seq``            -> the peer answers ``ACK seq``;
* ``PINGREQ seq target``  -> the helper pings ``target`` (a member only) and
  relays its ``ACK seq`` to the requester (memberlist's indirect ping);
* with a key every packet carries an HMAC-SHA256 tag over its bytes and a
  packet without a valid tag is dropped.  The key authenticates the probes;
  they carry only node ids and sequence numbers, so nothing is encrypted
  (the Python standard library has no AES; cluster data travels over the
  HTTP port, encrypted with ``[tls]``).

Packet: ``b"PG" | version u8 | type u8 | seq u32 | len u16 + sender id |
len u16 + target id | [tag 32 bytes]``, big endian.
"""
from __future__ import annotations

import hashlib
import hmac
import socket
import struct
import threading
from typing import Callable, Dict, Iterable, Optional, Tuple

PING, ACK, PINGREQ = 1, 2, 3
_VERSION = 1
_HDR = struct.Struct(">2sBBI")
TAG_BYTES = 32
MAX_PACKET = 1400


def load_key(path: str) -> bytes:
    """The ``gossip.key`` file: 16, 24 or 32 raw bytes (memberlist's AES key
    sizes, server/config.go:183-191)."""
    with open(path, "rb") as fh:
        key = fh.read()
    if len(key) not in (16, 24, 32):
        raise ValueError(f"gossip key must be 16, 24 or 32 bytes, got {len(key)}")
    return key


class UdpProber:
    """One node's UDP endpoint on the gossip port.  ``members()`` lists the
    cluster's nodes (``id`` attributes); ``addr_of(node)`` is a node's
    (host, gossip port)."""

    def __init__(self, node_id: str, bind_host: str, port: int, members: Callable[[], Iterable],
                 addr_of: Callable[[object], Tuple[str, int]], key: Optional[bytes] = None, logger=None):
        self.node_id = node_id
        self.members = members
        self.addr_of = addr_of
        self.key = key
        self.logger = logger
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind((bind_host, int(port)))
        self.port = self.sock.getsockname()[1]
        self._seq = 0
        self._mu = threading.Lock()
        self._waiters: Dict[int, threading.Event] = {}
        self._relay: Dict[int, Tuple[Tuple[str, int], int]] = {}   # our seq -> (requester addr, its seq)
        self._closing = threading.Event()
        self.dropped = 0          # packets refused (bad tag, malformed, unknown target)
        self.received = 0
        self._thread = threading.Thread(target=self._loop, name=f"gossip-udp-{self.port}", daemon=True)
        self._thread.start()

    def close(self):
        self._closing.set()
        try:
            self.sock.close()
        except OSError:
            pass

    # ------------------------------------------------------------ wire
    def _pack(self, typ: int, seq: int, target: str = "") -> bytes:
        sid, tid = self.node_id.encode(), target.encode()
        body = _HDR.pack(b"PG", _VERSION, typ, seq & 0xFFFFFFFF) + struct.pack(">H", len(sid)) + sid + \
            struct.pack(">H", len(tid)) + tid
        if self.key is not None:
            body += hmac.new(self.key, body, hashlib.sha256).digest()
        return body

    def _unpack(self, data: bytes):
        try:
            if self.key is not None:
                body, tag = data[:-TAG_BYTES], data[-TAG_BYTES:]
                if len(data) <= TAG_BYTES or not hmac.compare_digest(
                        tag, hmac.new(self.key, body, hashlib.sha256).digest()):
                    return None
            else:
                body = data
            magic, ver, typ, seq = _HDR.unpack_from(body, 0)
            if magic != b"PG" or ver != _VERSION:
                return None
            o = _HDR.size
            (n,) = struct.unpack_from(">H", body, o)
            sender = body[o + 2:o + 2 + n].decode()
            o += 2 + n
            (m,) = struct.unpack_from(">H", body, o)
            target = body[o + 2:o + 2 + m].decode()
            return typ, seq, sender, target
        except (struct.error, UnicodeDecodeError, ValueError):
            return None

    def _next_seq(self) -> int:
        with self._mu:
            self._seq = (self._seq + 1) & 0xFFFFFFFF
            return self._seq

    def _send(self, addr, pkt: bytes):
        try:
            self.sock.sendto(pkt, addr)
        except OSError:
            pass

    # ------------------------------------------------------------ probes
    def _await(self, seq: int, send: Callable[[], None], timeout: float) -> bool:
        ev = threading.Event()
        with self._mu:
            self._waiters[seq] = ev
        try:
            send()
            return ev.wait(max(0.0, float(timeout)))
        finally:
            with self._mu:
                self._waiters.pop(seq, None)

    def ping(self, node, timeout: float) -> bool:
        """Direct probe: PING, then the node's ACK within ``timeout``."""
        seq = self._next_seq()
        return self._await(seq, lambda: self._send(self.addr_of(node), self._pack(PING, seq)), timeout)

    def ping_req(self, helper, target, timeout: float) -> bool:
        """Indirect probe: ask ``helper`` to ping ``target``; its relayed ACK
        within the helper's probe time plus ours."""
        seq = self._next_seq()
        return self._await(seq, lambda: self._send(self.addr_of(helper), self._pack(PINGREQ, seq, target.id)),
                           2 * timeout + 0.1)

    # ------------------------------------------------------------ receive
    def _loop(self):
        while not self._closing.is_set():
            try:
                data, addr = self.sock.recvfrom(MAX_PACKET)
            except OSError:
                return
            got = self._unpack(data)
            if got is None:
                self.dropped += 1
                continue
            self.received += 1
            typ, seq, sender, target = got
            if typ == PING:
                self._send(addr, self._pack(ACK, seq))
            elif typ == ACK:
                with self._mu:
                    ev = self._waiters.get(seq)
                    relay = self._relay.pop(seq, None)
                if ev is not None:
                    ev.set()
                if relay is not None:
                    raddr, rseq = relay
                    self._send(raddr, self._pack(ACK, rseq))
            elif typ == PINGREQ:
                node = next((n for n in self.members() if n.id == target and n.id != self.node_id), None)
                if node is None:     # only members are probed for a peer
                    self.dropped += 1
                    continue
                mine = self._next_seq()
                with self._mu:
                    self._relay[mine] = (addr, seq)
                self._send(self.addr_of(node), self._pack(PING, mine))
                # forget relays that never got an ACK
                if len(self._relay) > 4096:
                    with self._mu:
                        for k in list(self._relay)[:2048]:
                            self._relay.pop(k, None)
