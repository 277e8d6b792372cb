"""SWIM-style failure detection for the cluster's nodes.

Reference: the reference runs hashicorp/memberlist for membership
(gossip/gossip.go:269-272 maps the ``[gossip]`` config onto it): every
``ProbeInterval`` a node probes one peer (round robin over a shuffled list)
with a ``ProbeTimeout``; an unanswered probe is retried indirectly through
``IndirectChecks`` other peers; a peer nobody can reach becomes *suspect* and
is declared dead once it stays unreachable for the suspicion timeout,
``SuspicionMult * max(1, log10(N)) * ProbeInterval``; a suspect that answers
again refutes the suspicion.  Pilosa turns memberlist's leave event into the
node going DOWN (after confirmNodeDown, cluster.go:1699).

Here the probes travel over the nodes' HTTP API (``GET /version`` direct,
``POST /internal/probe`` for an indirect probe through a helper), driven by
the same ``[gossip]`` keys: ``probe-interval``, ``probe-timeout``,
``suspicion-mult`` and ``nodes`` (the indirect probers per failed probe).
The detector itself is transport-free (``probe`` / ``indirect`` callables)
so its timing is unit-testable; ``Server`` runs one per node.
"""
from __future__ import annotations

import concurrent.futures as cf
import math
import random
import threading
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

ALIVE, DOWN = "alive", "down"


def suspicion_timeout(mult: float, n_nodes: int, probe_interval: float) -> float:
    """memberlist's suspicion timeout: mult * max(1, log10(N)) * interval."""
    return float(mult) * max(1.0, math.log10(max(1, int(n_nodes)))) * float(probe_interval)


class FailureDetector:
    """One node's prober.  ``tick(nodes)`` runs one protocol period and
    returns the state transitions it concluded: ``(node_id, "down")`` for a
    suspect whose suspicion timed out, ``(node_id, "alive")`` for a node
    marked DOWN that answered again.  ``nodes`` are objects with ``id``,
    ``uri`` and ``state`` (cluster Nodes)."""

    def __init__(self, self_id: str, probe: Callable[[object, float], bool],
                 indirect: Optional[Callable[[object, object, float], bool]] = None,
                 probe_interval: float = 1.0, probe_timeout: float = 0.5, suspicion_mult: float = 4,
                 indirect_checks: int = 3, clock: Callable[[], float] = time.monotonic, seed: Optional[int] = None):
        self.self_id = self_id
        self.probe = probe
        self.indirect = indirect
        self.probe_interval = float(probe_interval)
        self.probe_timeout = float(probe_timeout)
        self.suspicion_mult = float(suspicion_mult)
        self.indirect_checks = max(0, int(indirect_checks))
        self.clock = clock
        self.rng = random.Random(seed)
        self.suspect_since: Dict[str, float] = {}
        self._order: List[str] = []
        self._pos = 0
        self._pool: Optional[cf.ThreadPoolExecutor] = None
        self._mu = threading.Lock()
        self.probes = 0
        self.indirect_probes = 0

    def close(self):
        if self._pool is not None:
            self._pool.shutdown(wait=False)
            self._pool = None

    # ------------------------------------------------------------ protocol period
    def _next_target(self, peers: Sequence) -> Optional[object]:
        """Round robin over a shuffled list, reshuffled after each pass
        (memberlist probeNode); nodes that joined are appended."""
        ids = {n.id: n for n in peers}
        self._order = [i for i in self._order if i in ids]
        for i in ids:
            if i not in self._order:
                self._order.insert(self.rng.randrange(len(self._order) + 1), i)
        if not self._order:
            return None
        if self._pos >= len(self._order):
            self.rng.shuffle(self._order)
            self._pos = 0
        t = ids[self._order[self._pos]]
        self._pos += 1
        return t

    def _reachable(self, target, peers: Sequence) -> bool:
        self.probes += 1
        try:
            if self.probe(target, self.probe_timeout):
                return True
        except Exception:  # noqa: BLE001 - any failure is a missed ack
            pass
        if self.indirect is None or not self.indirect_checks:
            return False
        helpers = [n for n in peers if n.id != target.id and getattr(n, "state", "") != "DOWN"]
        helpers = self.rng.sample(helpers, min(self.indirect_checks, len(helpers)))
        if not helpers:
            return False
        self.indirect_probes += len(helpers)
        if self._pool is None:
            self._pool = cf.ThreadPoolExecutor(max_workers=max(2, self.indirect_checks), thread_name_prefix="swim")
        futs = [self._pool.submit(self.indirect, h, target, self.probe_timeout) for h in helpers]
        ok = False
        for f in futs:
            try:
                ok |= bool(f.result(timeout=self.probe_timeout * 2 + 1.0))
            except Exception:  # noqa: BLE001 - a helper that fails says nothing
                pass
        return ok

    def tick(self, nodes: Sequence) -> List[Tuple[str, str]]:
        """One protocol period: probe the round-robin target and every
        current suspect (so a suspicion is confirmed or refuted within its
        timeout, whatever the cluster size)."""
        with self._mu:
            peers = [n for n in nodes if n.id != self.self_id]
            if not peers:
                self.suspect_since.clear()
                return []
            targets = []
            t = self._next_target(peers)
            if t is not None:
                targets.append(t)
            by_id = {n.id: n for n in peers}
            for sid in list(self.suspect_since):
                if sid not in by_id:
                    del self.suspect_since[sid]
                elif all(x.id != sid for x in targets):
                    targets.append(by_id[sid])
            timeout = suspicion_timeout(self.suspicion_mult, len(nodes), self.probe_interval)
            out: List[Tuple[str, str]] = []
            for n in targets:
                ok = self._reachable(n, peers)
                now = self.clock()
                if ok:
                    self.suspect_since.pop(n.id, None)
                    if getattr(n, "state", "") == "DOWN":
                        out.append((n.id, ALIVE))
                    continue
                since = self.suspect_since.setdefault(n.id, now)
                if now - since >= timeout and getattr(n, "state", "") != "DOWN":
                    out.append((n.id, DOWN))
            return out

    def detection_bound(self, n_nodes: int) -> float:
        """Worst-case time from a node stopping to this detector declaring it
        DOWN: up to N - 1 periods until the round robin reaches it, the
        suspicion timeout, and one period to conclude; a period takes up to
        an interval plus a direct and an indirect probe timeout."""
        period = self.probe_interval + 2 * self.probe_timeout
        return (max(1, n_nodes - 1) + 1) * period + suspicion_timeout(self.suspicion_mult, n_nodes,
                                                                       self.probe_interval)
