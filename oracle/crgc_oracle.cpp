// crgc_oracle.cpp — TEST INFRASTRUCTURE ONLY (see crgc_oracle.h).
//
// A line-by-line restatement of the reference's ShadowGraph semantics, keeping
// Java object identity: every Shadow is a heap object, `outgoing` is keyed by
// Shadow*, and a collected shadow is dropped from `shadowMap` and `from` but
// stays alive while some live shadow's `outgoing` still names it, exactly as
// the JVM keeps it reachable.  That is what makes incarnations
// come out right without any special casing.
//
// Deliberate, documented deviations (DESIGN.md "Oracle"):
//  * Lookups always go through the id map: the Refob.targetShadow
//    cache of ShadowGraph.java:23-33 is a JVM object-identity artefact.
//  * Where the reference throws (NPE at :277, CME at :162/:170) the oracle
//    returns the matching CRGC_E_* code and leaves the graph poisoned, as
//    LocalGC then restarts with an empty graph (LocalGC.scala:58).
//  * totalActorsSeen is kept in 64 bits (Java int, :12).
#include "crgc_oracle.h"

#include <cstdint>
#include <cstring>
#include <memory>
#include <unordered_map>
#include <vector>

namespace {

// Java int arithmetic: two's complement wraparound.
inline int32_t jadd(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a + (uint32_t)b);
}
inline int32_t jsub(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a - (uint32_t)b);
}

// RefobInfo.java:23-29
inline int16_t refob_count(int16_t info) { return (int16_t)(((int32_t)info) >> 1); }
inline bool refob_is_active(int16_t info) { return (info & 1) == 0; }

struct Shadow;
struct PtrHash {
  size_t operator()(const Shadow *p) const noexcept {
    uint64_t x = (uint64_t)(uintptr_t)p;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33;
    return (size_t)x;
  }
};

// Shadow.java:10-54
struct Shadow {
  uint64_t self = CRGC_NO_ACTOR;
  uint16_t location = 0;
  std::unordered_map<Shadow *, int32_t, PtrHash> outgoing;
  Shadow *supervisor = nullptr;
  int32_t recvCount = 0;
  bool mark = false;
  bool isRoot = false;
  bool interned = false;
  bool isLocal = false;
  bool isBusy = false;
  bool isHalted = false;
};

}  // namespace

struct oracle_graph {
  uint32_t F = 4;
  uint32_t deltaGraphSize = 64;
  bool MARKED = true;                                // ShadowGraph.java:11
  uint64_t totalActorsSeen = 0;                      // :12
  std::vector<Shadow *> from;                        // :13
  std::unordered_map<uint64_t, Shadow *> shadowMap;  // :14
  std::vector<std::unique_ptr<Shadow>> heap;         // keeps every object alive
  bool poisoned = false;

  // ShadowGraph.java:45-62
  Shadow *makeShadow(uint64_t ref) {
    totalActorsSeen++;
    heap.emplace_back(new Shadow());
    Shadow *s = heap.back().get();
    s->location = CRGC_LOCATION_OF(ref);
    s->self = ref;
    s->mark = !MARKED;
    s->interned = false;
    s->isLocal = false;
    shadowMap[ref] = s;
    from.push_back(s);
    return s;
  }
  // ShadowGraph.java:35-43
  Shadow *getShadow(uint64_t ref) {
    auto it = shadowMap.find(ref);
    if (it != shadowMap.end()) return it->second;
    return makeShadow(ref);
  }
  // ShadowGraph.java:64-73
  static void updateOutgoing(std::unordered_map<Shadow *, int32_t, PtrHash> &out,
                             Shadow *target, int32_t delta) {
    auto it = out.find(target);
    int32_t count = it == out.end() ? 0 : it->second;
    int32_t sum = jadd(count, delta);
    if (sum == 0) {
      if (it != out.end()) out.erase(it);
    } else if (it != out.end()) {
      it->second = sum;
    } else {
      out.emplace(target, sum);
    }
  }
};

namespace {

bool reserved_id(uint64_t id) {
  return id == CRGC_NO_ACTOR || id == CRGC_DEAD_ACTOR || CRGC_LOCATION_OF(id) == 0xFFFF;
}

// ShadowGraph.java:201-203
inline bool isPseudoRoot(const Shadow *s) {
  return (s->isRoot || s->isBusy || s->recvCount != 0 || !s->interned) && !s->isHalted;
}

int check_entries(const oracle_graph *g, const crgc_entry_batch *b) {
  if (!b || b->memory != CRGC_MEM_HOST) return CRGC_E_INVAL;
  if (b->n_entries == 0) return CRGC_OK;
  if (!b->self || !b->recv_count || !b->flags || !b->created_off || !b->spawned_off ||
      !b->updated_off)
    return CRGC_E_INVAL;
  for (uint64_t i = 0; i < b->n_entries; i++) {
    if (reserved_id(b->self[i])) return CRGC_E_INVAL;
    uint32_t nc = b->created_off[i + 1] - b->created_off[i];
    uint32_t ns = b->spawned_off[i + 1] - b->spawned_off[i];
    uint32_t nu = b->updated_off[i + 1] - b->updated_off[i];
    if (b->created_off[i + 1] < b->created_off[i] || b->spawned_off[i + 1] < b->spawned_off[i] ||
        b->updated_off[i + 1] < b->updated_off[i])
      return CRGC_E_INVAL;
    if (nc > g->F || ns > g->F || nu > g->F) return CRGC_E_INVAL;
    for (uint32_t k = b->created_off[i]; k < b->created_off[i + 1]; k++)
      if (reserved_id(b->created_owner[k]) || reserved_id(b->created_target[k]))
        return CRGC_E_INVAL;
    for (uint32_t k = b->spawned_off[i]; k < b->spawned_off[i + 1]; k++)
      if (reserved_id(b->spawned[k])) return CRGC_E_INVAL;
    for (uint32_t k = b->updated_off[i]; k < b->updated_off[i + 1]; k++)
      if (reserved_id(b->updated_ref[k])) return CRGC_E_INVAL;
  }
  return CRGC_OK;
}

}  // namespace

extern "C" {

oracle_graph *oracle_create(uint32_t entry_field_size, uint32_t delta_graph_size) {
  oracle_graph *g = new oracle_graph();
  g->F = entry_field_size ? entry_field_size : 4;
  g->deltaGraphSize = delta_graph_size ? delta_graph_size : 64;
  return g;
}

void oracle_destroy(oracle_graph *g) { delete g; }

// N x ShadowGraph.mergeEntry — ShadowGraph.java:75-125
int oracle_merge_entries(oracle_graph *g, const crgc_entry_batch *b) {
  if (!g) return CRGC_E_INVAL;
  if (g->poisoned) return CRGC_E_POISONED;
  int rc = check_entries(g, b);
  if (rc) return rc;
  for (uint64_t i = 0; i < b->n_entries; i++) {
    // Local information. (:77-82)
    Shadow *selfShadow = g->getShadow(b->self[i]);
    selfShadow->interned = true;
    selfShadow->isLocal = true;
    selfShadow->recvCount = jadd(selfShadow->recvCount, (int32_t)b->recv_count[i]);
    selfShadow->isBusy = (b->flags[i] & CRGC_ENTRY_BUSY) != 0;
    selfShadow->isRoot = (b->flags[i] & CRGC_ENTRY_ROOT) != 0;
    // Created refs: target resolved before owner. (:85-93)
    for (uint32_t k = b->created_off[i]; k < b->created_off[i + 1]; k++) {
      Shadow *targetShadow = g->getShadow(b->created_target[k]);
      Shadow *shadow = g->getShadow(b->created_owner[k]);
      oracle_graph::updateOutgoing(shadow->outgoing, targetShadow, 1);
    }
    // Spawned actors. (:96-104)
    for (uint32_t k = b->spawned_off[i]; k < b->spawned_off[i + 1]; k++) {
      Shadow *childShadow = g->getShadow(b->spawned[k]);
      childShadow->supervisor = selfShadow;
    }
    // Updated refs. (:107-123)
    for (uint32_t k = b->updated_off[i]; k < b->updated_off[i + 1]; k++) {
      Shadow *targetShadow = g->getShadow(b->updated_ref[k]);
      int16_t info = b->updated_info[k];
      int16_t sendCount = refob_count(info);
      bool isDeactivated = !refob_is_active(info);
      if (sendCount > 0) targetShadow->recvCount = jsub(targetShadow->recvCount, sendCount);
      if (isDeactivated) oracle_graph::updateOutgoing(selfShadow->outgoing, targetShadow, -1);
    }
  }
  return CRGC_OK;
}

// N x ShadowGraph.mergeDelta — ShadowGraph.java:127-156
int oracle_merge_deltas(oracle_graph *g, const crgc_delta_batch *b) {
  if (!g || !b || b->memory != CRGC_MEM_HOST) return CRGC_E_INVAL;
  if (g->poisoned) return CRGC_E_POISONED;
  for (uint64_t i = 0; i < b->n_shadows; i++) {
    if (reserved_id(b->id[i])) return CRGC_E_INVAL;
    if (b->supervisor[i] != CRGC_NO_ACTOR && reserved_id(b->supervisor[i])) return CRGC_E_INVAL;
    if (b->out_off[i + 1] < b->out_off[i]) return CRGC_E_INVAL;
    for (uint32_t k = b->out_off[i]; k < b->out_off[i + 1]; k++)
      if (reserved_id(b->out_target[k])) return CRGC_E_INVAL;
  }
  for (uint64_t i = 0; i < b->n_shadows; i++) {
    Shadow *shadow = g->getShadow(b->id[i]);
    bool dInterned = (b->flags[i] & CRGC_DELTA_INTERNED) != 0;
    shadow->interned = shadow->interned || dInterned;
    shadow->recvCount = jadd(shadow->recvCount, b->recv_count[i]);
    if (dInterned) {
      shadow->isBusy = (b->flags[i] & CRGC_DELTA_BUSY) != 0;
      shadow->isRoot = (b->flags[i] & CRGC_DELTA_ROOT) != 0;
    }
    if (b->supervisor[i] != CRGC_NO_ACTOR) shadow->supervisor = g->getShadow(b->supervisor[i]);
    for (uint32_t k = b->out_off[i]; k < b->out_off[i + 1]; k++)
      oracle_graph::updateOutgoing(shadow->outgoing, g->getShadow(b->out_target[k]),
                                   b->out_count[k]);
  }
  return CRGC_OK;
}

// ShadowGraph.mergeUndoLog — ShadowGraph.java:158-174
int oracle_merge_undo(oracle_graph *g, const crgc_undo_log *log) {
  if (!g || !log || log->memory != CRGC_MEM_HOST) return CRGC_E_INVAL;
  if (g->poisoned) return CRGC_E_POISONED;
  // UndoLog.admitted is a HashMap: one field per actor.
  std::unordered_map<uint64_t, uint64_t> admitted;
  for (uint64_t f = 0; f < log->n_fields; f++) {
    if (reserved_id(log->actor[f])) return CRGC_E_INVAL;
    if (!admitted.emplace(log->actor[f], f).second) return CRGC_E_INVAL;
  }
  // The reference iterates `from` while getShadow may append to it, which
  // throws ConcurrentModificationException: detect it up front.
  for (Shadow *s : g->from) {
    auto it = admitted.find(s->self);
    if (it == admitted.end()) continue;
    uint64_t f = it->second;
    for (uint32_t k = log->created_off[f]; k < log->created_off[f + 1]; k++)
      if (!g->shadowMap.count(log->created_target[k])) return CRGC_E_UNDO_NEW_SHADOW;
  }
  for (Shadow *shadow : g->from) {
    if (shadow->location == log->node_location) shadow->isHalted = true;
    auto it = admitted.find(shadow->self);
    if (it == admitted.end()) continue;
    uint64_t f = it->second;
    shadow->recvCount = jadd(shadow->recvCount, log->message_count[f]);
    for (uint32_t k = log->created_off[f]; k < log->created_off[f + 1]; k++)
      oracle_graph::updateOutgoing(shadow->outgoing, g->getShadow(log->created_target[k]),
                                   log->created_count[k]);
  }
  return CRGC_OK;
}

// ShadowGraph.trace — ShadowGraph.java:205-289
int oracle_trace(oracle_graph *g, int should_kill, crgc_trace_out *out) {
  if (!g || !out) return CRGC_E_INVAL;
  if (g->poisoned) return CRGC_E_POISONED;
  const bool MARKED = g->MARKED;
  crgc_trace_stats st{};
  std::vector<Shadow *> to;
  to.reserve(g->from.size());
  for (Shadow *shadow : g->from) {  // :217-223
    if (isPseudoRoot(shadow)) {
      to.push_back(shadow);
      shadow->mark = MARKED;
    }
  }
  st.pseudo_roots = to.size();
  for (size_t scanptr = 0; scanptr < to.size(); scanptr++) {  // :224-268
    Shadow *owner = to[scanptr];
    if (owner->isHalted) continue;
    st.edges_scanned += owner->outgoing.size();
    for (auto &kv : owner->outgoing) {
      Shadow *target = kv.first;
      if (kv.second > 0 && target->mark != MARKED) {
        to.push_back(target);
        target->mark = MARKED;
      }
    }
    Shadow *supervisor = owner->supervisor;
    if (supervisor != nullptr) {
      st.sup_edges++;
      if (supervisor->mark != MARKED) {
        to.push_back(supervisor);
        supervisor->mark = MARKED;
      }
    }
  }
  std::vector<uint64_t> garbage, kill;
  uint64_t nLive = 0;
  for (Shadow *shadow : g->from) {  // :273-284
    if (shadow->mark != MARKED) {
      garbage.push_back(shadow->self);
      g->shadowMap.erase(shadow->self);
      if (shadow->isLocal) {
        if (shadow->supervisor == nullptr) {  // NullPointerException in the reference
          g->poisoned = true;
          return CRGC_E_NULL_SUPERVISOR;
        }
        if (shadow->supervisor->mark == MARKED && should_kill && !shadow->isHalted)
          kill.push_back(shadow->self);
      }
    } else {
      nLive++;
    }
  }
  g->from.swap(to);  // :285
  g->MARKED = !g->MARKED;  // :286

  out->n_garbage = garbage.size();
  out->n_kill = kill.size();
  out->n_live = nLive;
  out->stats = st;
  bool big = false;
  if (out->garbage_ids) {
    if (out->garbage_cap < garbage.size()) big = true;
    else if (!garbage.empty()) memcpy(out->garbage_ids, garbage.data(), garbage.size() * 8);
  }
  if (out->kill_ids) {
    if (out->kill_cap < kill.size()) big = true;
    else if (!kill.empty()) memcpy(out->kill_ids, kill.data(), kill.size() * 8);
  }
  return big ? CRGC_E2BIG : CRGC_OK;
}

// ShadowGraph.startWave — ShadowGraph.java:291-299
int oracle_local_roots(oracle_graph *g, uint64_t *out, uint64_t cap, uint64_t *n) {
  if (!g || !n) return CRGC_E_INVAL;
  if (g->poisoned) return CRGC_E_POISONED;
  uint64_t k = 0;
  bool big = false;
  for (Shadow *s : g->from) {
    if (s->isRoot && s->isLocal) {
      if (out && k < cap) out[k] = s->self;
      else if (out) big = true;
      k++;
    }
  }
  *n = k;
  return big ? CRGC_E2BIG : CRGC_OK;
}

// ShadowGraph.investigateRemotelyHeldActors — ShadowGraph.java:302-330
int oracle_count_reachable_from(oracle_graph *g, uint16_t location, int64_t *out) {
  if (!g || !out) return CRGC_E_INVAL;
  if (g->poisoned) return CRGC_E_POISONED;
  const bool MARKED = g->MARKED;
  std::vector<Shadow *> to;
  for (Shadow *s : g->from) {
    if (s->location == location) {
      to.push_back(s);
      s->mark = MARKED;
    }
  }
  for (size_t scanptr = 0; scanptr < to.size(); scanptr++) {
    Shadow *owner = to[scanptr];
    if (owner->isHalted) continue;
    for (auto &kv : owner->outgoing) {
      Shadow *target = kv.first;
      if (kv.second > 0 && target->mark != MARKED) {
        to.push_back(target);
        target->mark = MARKED;
      }
    }
  }
  for (Shadow *s : to) s->mark = !MARKED;
  *out = (int64_t)to.size();
  return CRGC_OK;
}

int oracle_total_actors_seen(oracle_graph *g, uint64_t *out) {
  if (!g || !out) return CRGC_E_INVAL;
  *out = g->totalActorsSeen;
  return CRGC_OK;
}

int oracle_live_count(oracle_graph *g, uint64_t *out) {
  if (!g || !out) return CRGC_E_INVAL;
  *out = g->shadowMap.size();
  return CRGC_OK;
}

// Shadow/ShadowGraph.assertEquals made into a dump (ShadowGraph.java:176-199).
int oracle_export(oracle_graph *g, crgc_graph_export *out) {
  if (!g || !out) return CRGC_E_INVAL;
  if (g->poisoned) return CRGC_E_POISONED;
  auto current = [&](const Shadow *s) {
    auto it = g->shadowMap.find(s->self);
    return it != g->shadowMap.end() && it->second == s;
  };
  uint64_t nv = 0, ne = 0;
  bool big = false;
  for (auto &kv : g->shadowMap) {
    const Shadow *s = kv.second;
    if (out->id) {
      if (nv < out->vertex_cap) {
        out->id[nv] = s->self;
        out->recv_count[nv] = s->recvCount;
        out->flags[nv] = (s->interned ? CRGC_F_INTERNED : 0) | (s->isLocal ? CRGC_F_LOCAL : 0) |
                         (s->isBusy ? CRGC_F_BUSY : 0) | (s->isRoot ? CRGC_F_ROOT : 0) |
                         (s->isHalted ? CRGC_F_HALTED : 0);
        out->supervisor[nv] = s->supervisor == nullptr ? CRGC_NO_ACTOR
                              : current(s->supervisor) ? s->supervisor->self
                                                       : CRGC_DEAD_ACTOR;
      } else {
        big = true;
      }
    }
    nv++;
    for (auto &e : s->outgoing) {
      if (e.second == 0 || !current(e.first)) continue;
      if (out->edge_owner) {
        if (ne < out->edge_cap) {
          out->edge_owner[ne] = s->self;
          out->edge_target[ne] = e.first->self;
          out->edge_count[ne] = e.second;
        } else {
          big = true;
        }
      }
      ne++;
    }
  }
  out->n_vertices = nv;
  out->n_edges = ne;
  return big ? CRGC_E2BIG : CRGC_OK;
}

}  // extern "C"
