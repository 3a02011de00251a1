"""Known-answer scenarios restated from the reference's own test specs.

Each scenario drives the CRGC mutator hooks (workload/mutator.py, a mirror of
State.java + CRGC.scala) through the message sequence of one reference spec and
states the outcome that spec asserts.  `run_scenario(graph, steps)` applies the
steps to any object with the ShadowGraph surface (the CPU oracle or the HIP
graph) and checks every expectation, so one scenario pins both.

Step kinds:
  ("merge", EntryBatch)                       one Wakeup's drained queue
  ("trace", garbage_ids, kill_ids)            trace(true) must return exactly these sets
  ("trace_any",)                              trace(true), outcome not asserted
"""
from __future__ import annotations

import random

from mutator import Mutator, Refob


def _wakeup(m: Mutator, steps, garbage=(), kill=()):
    steps.append(("merge", m.drain()))
    steps.append(("trace", set(garbage), set(kill)))


# ---------------------------------------------------------------------------
# SupervisionSpec.scala:32-57 — a parent is not collected before its children.
# ---------------------------------------------------------------------------
def supervision():
    m = Mutator()
    steps = []
    R = m.spawn_root()
    refP, P = m.spawn(R)                       # Init: spawn(Parent)
    refC1, C1 = m.spawn(P)                     # Parent constructor: two children
    refC2, C2 = m.spawn(P)
    m.onBlock(C1); m.onBlock(C2)
    toP = m.createRef(R, R.self, refP)         # actorA ! GetRef(createRef(self, actorA))
    m.send(R, refP)
    m.onBlock(R)
    m.receive(P)                               # Parent gets GetRef(root)
    r1 = m.createRef(P, refC1, toP); m.send(P, toP)
    r2 = m.createRef(P, refC2, toP); m.send(P, toP)
    m.release(P, [refC1, refC2])
    m.onBlock(P)
    m.receive(R); m.receive(R)                 # root gets both GetRefs
    m.onBlock(R)
    _wakeup(m, steps)
    m.release(R, [refP]); m.onBlock(R)         # ReleaseParent: nothing may stop
    _wakeup(m, steps)
    m.release(R, [r1]); m.onBlock(R)           # ReleaseChild1: child1 stops
    _wakeup(m, steps, {C1.self.target}, {C1.self.target})
    m.release(R, [r2]); m.onBlock(R)           # ReleaseChild2: child2 and parent stop;
    g = {C2.self.target, P.self.target}        # parent is told StopMsg, child2 dies with it
    _wakeup(m, steps, g, {P.self.target})
    return steps


# ---------------------------------------------------------------------------
# SimpleActorSpec.scala:26-60
# ---------------------------------------------------------------------------
def simple_actor():
    m = Mutator()
    steps = []
    A = m.spawn_root()
    refB, B = m.spawn(A)
    refC, C = m.spawn(A)
    m.onBlock(B); m.onBlock(C); m.onBlock(A)
    _wakeup(m, steps)
    m.send(A, refC); m.onBlock(A)              # SendC(Hello)
    m.receive(C); m.onBlock(C)
    _wakeup(m, steps)
    share = m.createRef(A, refC, refB)         # TellBAboutC
    m.send(A, refB); m.onBlock(A)
    m.receive(B); bC = share; m.onBlock(B)
    m.send(A, refB); m.onBlock(A)              # SendB(SendC(Hello))
    m.receive(B); m.send(B, bC); m.onBlock(B)
    m.receive(C); m.onBlock(C)
    _wakeup(m, steps)
    m.release(A, [refC]); m.onBlock(A)         # ReleaseC: C must survive (B holds it)
    _wakeup(m, steps)
    m.send(A, refB); m.onBlock(A)              # SendB(SendC(Hello)) still works
    m.receive(B); m.send(B, bC); m.onBlock(B)
    m.receive(C); m.onBlock(C)
    _wakeup(m, steps)
    m.send(A, refB); m.onBlock(A)              # SendB(ReleaseC): C terminates
    m.receive(B); m.release(B, [bC]); m.onBlock(B)
    _wakeup(m, steps, {C.self.target}, {C.self.target})
    m.release(A, [refB]); m.onBlock(A)         # ReleaseB: B terminates
    _wakeup(m, steps, {B.self.target}, {B.self.target})
    return steps


# ---------------------------------------------------------------------------
# SelfMessagingSpec.scala:27-34 — in-flight self messages keep B alive.
# ---------------------------------------------------------------------------
def self_messaging(n=40, wake_every=7):
    m = Mutator()
    steps = []
    A = m.spawn_root()
    refB, B = m.spawn(A)
    m.onBlock(B); m.onBlock(A)
    _wakeup(m, steps)
    m.send(A, refB)                            # actorB ! Countdown(n)
    m.release(A, [refB])                       # context.release(actorB)
    m.onBlock(A)
    _wakeup(m, steps)                          # B has an undelivered message: live
    for k in range(n, -1, -1):                 # B counts down through self-messages
        m.receive(B)
        if k > 0:
            m.send(B, B.self)
        m.onBlock(B)
        if k % wake_every == 0 and k > 0:
            _wakeup(m, steps)                  # still counting down: live
    b = B.self.target
    _wakeup(m, steps, {b}, {b})
    return steps


# ---------------------------------------------------------------------------
# ManyMessagesSpec.scala:33-42 — 4*Short.MaxValue messages bound-check the
# 16-bit counters and the forced busy flushes.
# ---------------------------------------------------------------------------
def many_messages(num=4 * 32767, batch=9000):
    m = Mutator()
    steps = []
    root = m.spawn_root()
    refA, A = m.spawn(root)
    refB, B = m.spawn(root)
    m.onBlock(A); m.onBlock(B)
    toB = m.createRef(root, refB, refA)        # NewAcquaintance(createRef(actorB, actorA))
    m.send(root, refA)
    m.release(root, [refA, refB])
    m.onBlock(root)
    m.receive(A)
    received = 0
    for i in range(num):                       # A sends NUM pings to B
        m.send(A, toB)
        if i % batch == batch - 1:             # B drains its mailbox concurrently
            while received < i + 1:
                m.receive(B); received += 1
            m.onBlock(B)
    m.onBlock(A)
    a, b = A.self.target, B.self.target
    # A is done sending and unreferenced: it stops (probeA gets Terminated);
    # B still has pings queued, so it must survive.
    _wakeup(m, steps, {a}, {a})
    while received < num:
        m.receive(B); received += 1
    m.onBlock(B)
    _wakeup(m, steps, {b}, {b})
    return steps


# ---------------------------------------------------------------------------
# RandomSpec.scala:18-125 — random spawn/link/release/ping (p = .2/.2/.2/.2);
# at the cap the root releases everything and every actor must be collected.
# The runner also checks soundness: a killed actor never has mail pending.
# ---------------------------------------------------------------------------
class RandomWorld:
    def __init__(self, seed: int, max_actors: int, wake_every: int = 25):
        self.rng = random.Random(seed)
        self.m = Mutator()
        self.max_actors = max_actors
        self.wake_every = wake_every
        self.spawned = 0
        self.root = self.m.spawn_root()
        self.states = {self.root.self.target: self.root}
        self.acq = {self.root.self.target: {}}   # holder -> {target: Refob}
        self.mail = {self.root.self.target: []}
        self.parent = {}
        self.stopped = set()
        self.released_all = False

    def _item(self, d):
        keys = list(d.keys())
        return d[keys[self.rng.randrange(len(keys))]]

    def _do_something(self, me):
        st = self.states[me]
        acq = self.acq[me]
        p = self.rng.random()
        if p < 0.2:
            self.spawned += 1
            if self.spawned <= self.max_actors:
                ref, child = self.m.spawn(st)
                c = child.self.target
                self.states[c], self.acq[c], self.mail[c] = child, {}, []
                self.parent[c] = me
                self.m.onBlock(child)            # child blocks after its setup
                if c not in acq:
                    acq[c] = ref
        elif p < 0.4 and acq:
            owner = self._item(acq)
            target = self._item(acq)
            new = self.m.createRef(st, target, owner)
            self.m.send(st, owner)
            self.mail[owner.target].append(("link", new))
        elif p < 0.6 and acq:
            r = self._item(acq)
            del acq[r.target]
            self.m.release(st, [r])
        elif p < 0.8 and acq:
            r = self._item(acq)
            self.m.send(st, r)
            self.mail[r.target].append(("ping", None))

    def _do_some_actions(self, me):
        if self.spawned >= self.max_actors:
            if me == self.root.self.target and not self.released_all:
                acq = self.acq[me]
                self.m.release(self.states[me], list(acq.values()))
                acq.clear()
                self.released_all = True
            return
        self._do_something(me)
        self._do_something(me)

    def turn(self, me):
        st = self.states[me]
        msgs, self.mail[me] = self.mail[me], []
        for kind, ref in msgs:
            self.m.receive(st)
            if kind == "link" and ref.target not in self.acq[me]:
                self.acq[me][ref.target] = ref
            self._do_some_actions(me)
        self.m.onBlock(st)

    def steps(self):
        """Yields (batch) for each wakeup; caller traces and reports kills."""
        root = self.root.self.target
        turns = 0
        idle_wakeups = 0
        while True:
            busy = [a for a, q in self.mail.items() if q and a not in self.stopped]
            if not self.released_all:
                self.mail[root].append(("ping", None))   # the root's timer
                if root not in busy:
                    busy.append(root)
            if busy:
                self.turn(self.rng.choice(busy))
                turns += 1
            if turns % self.wake_every == 0 or not busy:
                yield self.m.drain()
                if not busy:
                    idle_wakeups += 1
                    if idle_wakeups > 3:
                        return

    def kill(self, victims):
        """StopMsg to each victim: Akka stops it and all its descendants."""
        children = {}
        for c, p in self.parent.items():
            children.setdefault(p, []).append(c)
        stack = list(victims)
        out = set()
        while stack:
            a = stack.pop()
            if a in out:
                continue
            out.add(a)
            stack.extend(children.get(a, []))
        for a in out:
            assert not self.mail[a], f"unsound: killed actor {a:#x} has mail pending"
            self.stopped.add(a)
        return out


def run_random(graph, seed=1, max_actors=400, wake_every=25):
    """RandomSpec: returns (#collected, #spawned).  Completeness: all collected."""
    w = RandomWorld(seed, max_actors, wake_every)
    collected = set()
    for batch in w.steps():
        graph.merge_entries(batch)
        r = graph.trace(True)
        g = r.garbage_set()
        assert not (g & collected), "an actor was collected twice"
        collected |= g
        stopped = w.kill(r.kill_set())
        # Akka's cascade only stops garbage: every stopped actor is garbage.
        assert stopped <= collected, "unsound: a live descendant was stopped"
    everyone = set(w.states) - {w.root.self.target}
    return collected, everyone


def run_scenario(graph, steps):
    """Apply steps to `graph`; assert each expected garbage/kill set."""
    results = []
    for st in steps:
        if st[0] == "merge":
            graph.merge_entries(st[1])
        elif st[0] == "trace":
            r = graph.trace(True)
            assert r.garbage_set() == st[1], (r.garbage_set(), st[1])
            assert r.kill_set() == st[2], (r.kill_set(), st[2])
            results.append(r)
        elif st[0] == "trace_any":
            results.append(graph.trace(True))
    return results


SCENARIOS = {
    "supervision": supervision,
    "simple_actor": simple_actor,
    "self_messaging": self_messaging,
    "many_messages": many_messages,
}
