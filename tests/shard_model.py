"""A host-side model of the sharded trace protocol, run over torch.distributed.

The product (libcrgc_hip.so) hash-partitions the shadow graph over G shards
and traces it with per-round frontier exchanges.
This model restates that protocol with plain Python sets so it can run on CPU
ranks over the gloo backend; tests/test_dist_cpu.py checks, on world_size 2
and 3, that the protocol reproduces the unsharded oracle's garbage and kill
sets.  It is test infrastructure: the protocol's device implementation is
checked against the oracle on the GPU (tests/test_hip_sharded.py).

Each rank holds, from an exported graph state (GraphState: vertex id ->
(recv, flags, supervisor), (owner, target) -> count):
  * home shadows:   ids with crgc_shard_of(id, G) == rank, with their fields
                    and out-edges;
  * proxies:        every other id named by a home shadow's out-edge or
                    supervisor (no fields, no edges).
Mark (ShadowGraph.java:205-268): local fixpoint from the home pseudo-roots,
then rounds: marked proxies are sent to their home rank, which continues from
them; stop when no rank sends anything.  Sweep (:270-284): garbage = unmarked
home shadows; a local, non-halted garbage shadow is killed when its supervisor
is marked — asked of the supervisor's home rank when the supervisor is an
unmarked proxy.
"""
from __future__ import annotations

from collections import defaultdict, deque

from crgc_hip import abi, shard_of

F_INTERNED, F_LOCAL, F_BUSY, F_ROOT, F_HALTED = (abi.F_INTERNED, abi.F_LOCAL, abi.F_BUSY,
                                                  abi.F_ROOT, abi.F_HALTED)


class NullSupervisor(Exception):
    pass


class ShardModel:
    def __init__(self, state, rank: int, G: int):
        self.rank, self.G = rank, G
        self.home = {v: f for v, f in state.vertices.items() if shard_of(v, G) == rank}
        self.out = defaultdict(dict)
        for (o, t), c in state.edges.items():
            if o in self.home:
                self.out[o][t] = c

    def is_proxy(self, v):
        return v not in self.home

    def pseudo_root(self, v):
        recv, fl, _ = self.home[v]
        return bool(fl & (F_ROOT | F_BUSY) or recv != 0 or not fl & F_INTERNED) \
            and not fl & F_HALTED

    def trace(self, dist, should_kill=True):
        G, me = self.G, self.rank
        vis = set()
        work = deque()
        for v in self.home:
            if self.pseudo_root(v):
                vis.add(v)
                work.append(v)
        sent = set()
        rounds = 1
        while True:
            # local fixpoint (:224-268)
            while work:
                v = work.popleft()
                if self.is_proxy(v):
                    continue
                _, fl, sup = self.home[v]
                if fl & F_HALTED:
                    continue
                for t, c in self.out.get(v, {}).items():
                    if c > 0 and t not in vis:
                        vis.add(t)
                        work.append(t)
                if sup not in (abi.NO_ACTOR, abi.DEAD_ACTOR) and sup not in vis:
                    vis.add(sup)
                    work.append(sup)
            # export newly marked proxies to their homes
            out = defaultdict(list)
            for v in vis:
                if self.is_proxy(v) and v not in sent:
                    sent.add(v)
                    out[shard_of(v, G)].append(v)
            boxes = [None] * G
            dist.all_gather_object(boxes, dict(out))
            total = sum(len(x) for b in boxes for x in b.values())
            if total == 0:
                break
            rounds += 1
            for b in boxes:
                for v in b.get(me, []):
                    if v not in vis:
                        vis.add(v)
                        work.append(v)
        # sweep: kill requests for supervisors only their home can judge
        garbage = [v for v in self.home if v not in vis]
        kill, asks = [], defaultdict(list)
        npe = False
        for v in garbage:
            _, fl, sup = self.home[v]
            if not fl & F_LOCAL:
                continue
            if sup == abi.NO_ACTOR:
                npe = True
            elif should_kill and not fl & F_HALTED and sup != abi.DEAD_ACTOR:
                if sup in vis:
                    kill.append(v)
                elif self.is_proxy(sup):
                    asks[shard_of(sup, G)].append((v, sup))
        flags = [None] * G
        dist.all_gather_object(flags, npe)
        if any(flags):
            raise NullSupervisor()
        boxes = [None] * G
        dist.all_gather_object(boxes, {d: [s for _, s in q] for d, q in asks.items()})
        answers = {r: [s in vis for s in b.get(me, [])] for r, b in enumerate(boxes)}
        back = [None] * G
        dist.all_gather_object(back, answers)
        for d, q in asks.items():
            for (v, _), yes in zip(q, back[d][me]):
                if yes:
                    kill.append(v)
        live = sum(1 for v in self.home if v in vis)
        return set(garbage), set(kill), live, rounds
