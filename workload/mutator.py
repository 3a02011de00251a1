"""Host-side mirror of CRGC's mutator hooks, for generating entry streams.

This restates how actors produce Entry records so that the known-answer tests
read like the reference's own integration specs:
  * State.java:45-124  (recordNewRefob / recordNewActor / recordUpdatedRefob /
    recordMessageReceived / flushToEntry, with the F-slot capacity checks)
  * CRGC.scala:69-221  (initState, spawnImpl, createRefImpl, releaseImpl,
    sendMessageImpl, onMessageImpl and the on-block flush hook)
  * Refob.scala:36-53 / RefobInfo.java (per-refob info word)
Ids carry the actor's location in their top 16 bits (include/crgc.h).
"""
from __future__ import annotations

import os
import sys
from typing import List, Optional

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "uigc-akka_amd"))
from crgc_hip.batch import Entry, EntryBatch, RefobInfo  # noqa: E402


def make_id(location: int, local: int) -> int:
    return ((location & 0xFFFF) << 48) | (local & 0xFFFFFFFFFFFF)


class Refob:
    """crgc.Refob (Refob.scala): one holder's reference object to `target`."""
    __slots__ = ("target", "info", "recorded")

    def __init__(self, target: int):
        self.target = target
        self.info = RefobInfo.activeRefob
        self.recorded = False

    def reset(self):                      # Refob.scala:51-54
        self.info = RefobInfo.resetCount(self.info)
        self.recorded = False


class State:
    """crgc.State (State.java): an actor's pending GC record."""

    def __init__(self, self_ref: Refob, F: int):
        self.self = self_ref
        self.F = F
        self.created: List[tuple] = []
        self.spawned: List[Refob] = []
        self.updated: List[Refob] = []
        self.recvCount = 0
        self.isRoot = False

    def canRecordNewRefob(self):
        return len(self.created) < self.F

    def recordNewRefob(self, owner: Refob, target: Refob):
        assert self.canRecordNewRefob()
        self.created.append((owner, target))

    def canRecordNewActor(self):
        return len(self.spawned) < self.F

    def recordNewActor(self, child: Refob):
        assert self.canRecordNewActor()
        self.spawned.append(child)

    def canRecordUpdatedRefob(self, r: Refob):
        return r.recorded or len(self.updated) < self.F

    def recordUpdatedRefob(self, r: Refob):
        assert self.canRecordUpdatedRefob(r)
        if r.recorded:
            return
        r.recorded = True
        self.updated.append(r)

    def canRecordMessageReceived(self):
        return self.recvCount < 32767

    def recordMessageReceived(self):
        assert self.canRecordMessageReceived()
        self.recvCount += 1

    def flushToEntry(self, isBusy: bool) -> Entry:  # State.java:90-124
        e = Entry(self=self.self.target, isBusy=isBusy, isRoot=self.isRoot)
        for owner, target in self.created:
            e.createdOwners.append(owner.target)
            e.createdTargets.append(target.target)
        self.created = []
        e.spawnedActors = [c.target for c in self.spawned]
        self.spawned = []
        e.recvCount = self.recvCount
        self.recvCount = 0
        for r in self.updated:
            e.updatedRefs.append(r.target)
            e.updatedInfos.append(r.info)
            r.reset()
        self.updated = []
        return e


class Mutator:
    """The CRGC engine's mutator side for one node: the entry queue plus hooks."""

    def __init__(self, location: int = 1, F: int = 4):
        self.location = location
        self.F = F
        self.queue: List[Entry] = []
        self._next = 1

    def fresh_id(self) -> int:
        i = make_id(self.location, self._next)
        self._next += 1
        return i

    # CRGC.scala:179-193
    def sendEntry(self, st: State, isBusy: bool):
        self.queue.append(st.flushToEntry(isBusy))

    # CRGC.scala:69-92 (spawnInfo.creator None => root)
    def initState(self, creator: Optional[Refob], actor_id: Optional[int] = None) -> State:
        self_ref = Refob(actor_id if actor_id is not None else self.fresh_id())
        st = State(self_ref, self.F)
        st.recordNewRefob(self_ref, self_ref)
        if creator is not None:
            st.recordNewRefob(creator, self_ref)
        else:
            st.isRoot = True
        return st

    def spawn_root(self) -> State:
        return self.initState(None)

    # CRGC.scala:100-112: returns (parent's refob to the child, child's state)
    def spawn(self, parent: State):
        child = self.initState(parent.self)
        ref = Refob(child.self.target)
        if not parent.canRecordNewActor():
            self.sendEntry(parent, True)
        parent.recordNewActor(ref)
        return ref, child

    # CRGC.scala:151-162: a new refob for `owner` pointing at target.target
    def createRef(self, st: State, target: Refob, owner: Refob) -> Refob:
        ref = Refob(target.target)
        if not st.canRecordNewRefob():
            self.sendEntry(st, True)
        st.recordNewRefob(owner, target)
        return ref

    # CRGC.scala:164-177
    def release(self, st: State, refs):
        for r in refs:
            if not st.canRecordUpdatedRefob(r):
                self.sendEntry(st, True)
            r.info = RefobInfo.deactivate(r.info)
            st.recordUpdatedRefob(r)

    # CRGC.scala:208-221
    def send(self, st: State, ref: Refob):
        if not RefobInfo.canIncrement(ref.info) or not st.canRecordUpdatedRefob(ref):
            self.sendEntry(st, True)
        ref.info = RefobInfo.incSendCount(ref.info)
        st.recordUpdatedRefob(ref)

    # CRGC.scala:114-127
    def receive(self, st: State):
        if not st.canRecordMessageReceived():
            self.sendEntry(st, True)
        st.recordMessageReceived()

    # CRGC.scala:84-88: the on-block hook at the end of a mailbox batch
    def onBlock(self, st: State):
        self.sendEntry(st, False)

    def drain(self) -> EntryBatch:
        b = EntryBatch.from_entries(self.queue)
        self.queue = []
        return b
