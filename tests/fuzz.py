"""Seeded adversarial entry/delta/undo streams for parity tests.

Unlike kats.RandomWorld (a faithful RandomSpec mutator), these streams poke at
the merge semantics directly: several entries per actor per batch with
conflicting busy/root flags (last-write-wins), supervisor
reassignment by spawns and deltas (E3), negative edge and receive counts (E1),
references to collected actors (new incarnations, E9), interleaved delta
batches, and undo logs halting a remote location (E6).

They stay inside the reference's defined behaviour: an actor only emits
entries while it is live and either a root or spawned (so no local garbage
lacks a supervisor, E8), and undo logs only name existing actors (E11).
`sync(state)` feeds the oracle's exported state back after every trace.
"""
from __future__ import annotations

import random

import numpy as np

from crgc_hip import abi
from crgc_hip.batch import DeltaBatch, Entry, EntryBatch, UndoBatch

LOCAL = 1
REMOTES = (2, 3)


def mk(loc, n):
    return (loc << 48) | n


class Fuzz:
    def __init__(self, seed: int, n_roots: int = 4, F: int = 4):
        self.rng = random.Random(seed)
        self.F = F
        self.next = 1
        self.roots = [self.fresh(LOCAL) for _ in range(n_roots)]
        self.emitters = list(self.roots)      # local actors allowed to send entries
        self.known = list(self.roots)         # every id ever mentioned
        self.remote = [self.fresh(self.rng.choice(REMOTES)) for _ in range(8)]
        self.known += self.remote
        self.held = {}                        # actor -> list of targets it may release
        self.owed = {}                        # actor -> receives not yet reported
        self.halted_locs = set()
        self.live = set(self.known)

    def fresh(self, loc):
        i = mk(loc, self.next)
        self.next += 1
        return i

    def pick_known(self):
        r = self.rng.random()
        if r < 0.05 and self.known:
            return self.rng.choice(self.known)        # possibly collected: new incarnation
        pool = [x for x in self.live] if len(self.live) < 64 else None
        if pool is not None:
            return self.rng.choice(pool) if pool else self.rng.choice(self.known)
        return self.rng.choice(self.known)

    def entries(self, n: int) -> EntryBatch:
        rng, F = self.rng, self.F
        out = []
        for _ in range(n):
            me = rng.choice(self.emitters)
            e = Entry(self=me, isRoot=me in self.roots, isBusy=rng.random() < 0.25)
            owed = self.owed.get(me, 0)
            if owed and rng.random() < 0.8:
                k = min(owed, 32767)
                e.recvCount = k
                self.owed[me] = owed - k
            for _ in range(rng.randint(0, F)):
                owner = me if rng.random() < 0.3 else self.pick_known()
                target = self.pick_known()
                e.createdOwners.append(owner)
                e.createdTargets.append(target)
                self.held.setdefault(owner, []).append(target)
            for _ in range(rng.choice([0, 0, 0, 1, 2])):
                child = self.fresh(LOCAL)
                e.spawnedActors.append(child)
                self.known.append(child)
                self.live.add(child)
                self.emitters.append(child)
                self.held.setdefault(me, []).append(child)
            seen = set()
            for _ in range(rng.randint(0, F)):
                h = self.held.get(me)
                if h and rng.random() < 0.7:
                    t = h.pop(rng.randrange(len(h)))
                    deact = rng.random() < 0.8
                    if not deact:
                        h.append(t)
                else:
                    t = self.pick_known()
                    deact = rng.random() < 0.3
                if t in seen:
                    continue
                seen.add(t)
                cnt = rng.choice([0, 0, 1, 2, 5])
                self.owed[t] = self.owed.get(t, 0) + cnt
                e.updatedRefs.append(t)
                e.updatedInfos.append((cnt << 1) | (1 if deact else 0))
            out.append(e)
        return EntryBatch.from_entries(out)

    def deltas(self, n_graphs: int, per_graph: int = 6) -> DeltaBatch:
        rng = self.rng
        rows = []
        for _ in range(n_graphs):
            locs = [l for l in REMOTES if l not in self.halted_locs]
            if not locs:
                break
            loc = rng.choice(locs)
            members = []
            for _ in range(per_graph):
                if rng.random() < 0.5:
                    a = rng.choice([r for r in self.remote if (r >> 48) == loc] or [self.fresh(loc)])
                    if a not in self.remote:
                        self.remote.append(a); self.known.append(a); self.live.add(a)
                    interned = True
                else:
                    a = self.pick_known()
                    interned = False
                if a in members:
                    continue
                members.append(a)
            for a in members:
                fl = 0
                if interned and (a >> 48) == loc:
                    fl |= abi.DELTA_INTERNED
                    if rng.random() < 0.3: fl |= abi.DELTA_BUSY
                    if rng.random() < 0.1: fl |= abi.DELTA_ROOT
                sup = abi.NO_ACTOR
                if fl & abi.DELTA_INTERNED and rng.random() < 0.3:
                    sup = rng.choice(members)
                outs = []
                for _ in range(rng.randint(0, 3)):
                    t = rng.choice(members)
                    if t not in [x for x, _ in outs]:
                        outs.append((t, rng.choice([-1, 1, 1, 2])))
                rows.append((a, rng.choice([0, 0, -1, 1]), sup, fl, outs))
        return DeltaBatch.from_rows(rows)

    def undo(self, existing) -> UndoBatch:
        rng = self.rng
        loc = REMOTES[-1]
        self.halted_locs.add(loc)
        ex = sorted(existing)
        fields = []
        for a in rng.sample(ex, min(len(ex), 10)):
            outs = []
            for t in rng.sample(ex, min(len(ex), rng.randint(0, 3))):
                outs.append((t, rng.choice([-2, -1, 1])))
            fields.append((a, rng.choice([0, -1, 1, 3]), outs))
        return UndoBatch.from_fields(loc, fields)

    def sync(self, state):
        """Adopt the graph's live set after a trace (collected actors stop)."""
        self.live = set(state.vertices)
        keep = []
        for a in self.emitters:
            v = state.vertices.get(a)
            if v is None:
                continue  # collected: a stopped actor never sends another entry
            _, flags, sup = v
            if a in self.roots or sup != abi.NO_ACTOR:
                keep.append(a)
        self.emitters = keep or list(self.roots)
