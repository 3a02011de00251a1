"""C5 — a cluster-style stream seen by node 1's collector.

N simulated nodes share one actor space (location = node).  Actors run the
RandomSpec op mix (spawn, link, release, ping; RandomSpec.scala:69-87), with
some spawns placed on another node and links/pings crossing nodes.  Each node
flushes its entries through the CRGC hooks (workload/mutator.py); node 1 merges
its own entries directly and every other node's entries as DeltaGraphs
(DeltaGraph.java:73-180, LocalGC.scala:159-177), in arrival order.  Then a node
is downed: node 1 builds its UndoLog from the deltas it merged from that node
(UndoLog.java:39-67) plus the survivors' ingress entries for messages from the
downed node they admitted (IngressEntry.java:91-100), and replays it
(ShadowGraph.mergeUndoLog) before tracing.

The collector-side merge order matches LocalGC: deltas merge on arrival
(LocalGC.scala:124-136), entries at the wakeup (:144-185), and deltas from a
removed node are dropped (:126).
"""
from __future__ import annotations

import random
from typing import Dict, List

from delta import DeltaGraph, IngressEntry, UndoLog, deltas_from_entries
from mutator import Mutator


class ClusterWorld:
    def __init__(self, seed: int, n_nodes: int = 8, max_actors: int = 2000,
                 p_remote_spawn: float = 0.25):
        self.rng = random.Random(seed)
        self.n = n_nodes
        self.nodes = [Mutator(location=k + 1) for k in range(n_nodes)]
        self.max_actors = max_actors
        self.p_remote = p_remote_spawn
        self.spawned = 0
        self.states = {}      # actor id -> State
        self.home = {}        # actor id -> node index
        self.acq = {}         # actor id -> {target: Refob}
        self.mail = {}        # actor id -> [(kind, refob, sender)]
        self.roots = []
        for k in range(n_nodes):
            st = self.nodes[k].spawn_root()
            a = st.self.target
            self.states[a], self.home[a], self.acq[a], self.mail[a] = st, k, {}, []
            self.roots.append(a)
        self.down = set()
        # admitted messages per (sender node -> receiver node), for ingress entries
        self.ingress: Dict[tuple, IngressEntry] = {}

    def _node(self, a):
        return self.nodes[self.home[a]]

    def _item(self, d):
        keys = list(d.keys())
        return d[keys[self.rng.randrange(len(keys))]]

    def _send(self, me, ref, kind, payload=None):
        self._node(me).send(self.states[me], ref)
        self.mail[ref.target].append((kind, payload, me))

    def _act(self, me):
        st, acq = self.states[me], self.acq[me]
        p = self.rng.random()
        if p < 0.2:
            self.spawned += 1
            if self.spawned <= self.max_actors:
                k = self.home[me]
                if self.rng.random() < self.p_remote:
                    k = self.rng.choice([j for j in range(self.n) if j not in self.down])
                # the child's init entry is flushed by its own node
                child = self.nodes[k].initState(st.self, actor_id=self.nodes[k].fresh_id())
                c = child.self.target
                from mutator import Refob
                ref = Refob(c)
                node = self._node(me)
                if not st.canRecordNewActor():
                    node.sendEntry(st, True)
                st.recordNewActor(ref)
                self.states[c], self.home[c], self.acq[c], self.mail[c] = child, k, {}, []
                self.nodes[k].onBlock(child)
                if c not in acq:
                    acq[c] = ref
        elif p < 0.4 and acq:
            owner, target = self._item(acq), self._item(acq)
            new = self._node(me).createRef(st, target, owner)
            self._send(me, owner, "link", new)
        elif p < 0.6 and acq:
            r = self._item(acq)
            del acq[r.target]
            self._node(me).release(st, [r])
        elif p < 0.8 and acq:
            self._send(me, self._item(acq), "ping")

    def _turn(self, me):
        msgs, self.mail[me] = self.mail[me], []
        node = self._node(me)
        for kind, payload, sender in msgs:
            node.receive(self.states[me])
            sk, rk = self.home[sender], self.home[me]
            if sk != rk:  # crossed an Artery link: the ingress stage counts it
                ie = self.ingress.setdefault((sk, rk), IngressEntry(sk + 1, rk + 1))
                ie.onMessage(me, [payload.target] if payload is not None else [])
            if kind == "link" and payload.target not in self.acq[me]:
                self.acq[me][payload.target] = payload
            if self.spawned < self.max_actors:
                self._act(me)
                self._act(me)
        node.onBlock(self.states[me])

    def run_turns(self, n_turns: int):
        for _ in range(n_turns):
            busy = [a for a, q in self.mail.items() if q and self.home[a] not in self.down]
            for r in self.roots:
                if self.home[r] not in self.down and self.rng.random() < 0.5:
                    self.mail[r].append(("ping", None, r))
                    busy.append(r)
            if not busy:
                return
            self._turn(self.rng.choice(busy))

    def flush(self, me_node: int = 0):
        """One wakeup's worth of input for node `me_node`'s collector:
        (own EntryBatch, [DeltaGraph per remote node, in arrival order])."""
        own = self.nodes[me_node].drain()
        deltas: List[DeltaGraph] = []
        per_node = {}
        for k, node in enumerate(self.nodes):
            if k == me_node:
                continue
            entries, node.queue = node.queue, []
            per_node[k] = deltas_from_entries(entries, address=k + 1)
        # interleave arrivals round-robin over nodes
        i = 0
        while any(per_node.values()):
            for k in list(per_node):
                if per_node[k]:
                    deltas.append((k, per_node[k].pop(0)))
            i += 1
        return own, deltas

    def undo_log(self, downed: int, merged_deltas, me_node: int = 0) -> UndoLog:
        log = UndoLog(downed + 1)
        for k, g in merged_deltas:
            if k == downed:
                log.mergeDeltaGraph(g)
        for (sk, rk), ie in self.ingress.items():
            if sk == downed:
                ie.isFinal = True
                log.mergeIngressEntry(ie)
        return log
