// omp_graph.cpp — BENCH INFRASTRUCTURE ONLY: the strong CPU baseline of SURVEY
// §8d / BASELINE.md §2 ("cpu_omp"): the whole wakeup — ShadowGraph.mergeEntry
// over a batch (ShadowGraph.java:75-125) and trace (:201-289) — as a parallel
// OpenMP implementation on the host cores given, on the same packed entry
// batches the GPU merges (include/crgc.h crgc_entry_batch, host memory).
//
//   merge: ids -> slots through a lock-free open-addressing table; receive
//          counts by atomic adds; isBusy / isRoot / supervisor by atomic
//          max-of-(call, record) tags, then the winners write; created and
//          deactivated refs as (owner, target, +-1) atoms, parallel-sorted by
//          key and segment-reduced, then merged per owner into its
//          target-sorted out-edge vector (zero counts dropped: absent == 0).
//   trace: pseudo-roots by a parallel scan; level-synchronous top-down BFS
//          with per-thread frontiers over out-edges with count > 0 and
//          supervisor edges, halted shadows marked but not expanded; sweep.
// Since round 6 it also merges DeltaGraph batches (ShadowGraph.mergeDelta,
// :127-156: the same atomics and last-write-wins tags, flags only when
// interned) and UndoLogs (mergeUndoLog, :158-174: the CME decided first, the
// node's shadows halted, admitted fields applied), so the full-size C5 GPU test
// has a checker.
// Collected slots are never reused (the incarnation rule E9 holds as in the
// HIP graph: edges to them have count <= 0 or come from halted owners).
// Not the product.  tests/test_omp_graph_cpu.py pins its garbage / kill sets to
// the oracle's; bench.py times it; the full-size GPU parity tests
// (tests/test_hip_full_size.py) use it as the checker where the single-thread
// oracle would take too long.
#include <omp.h>
#include <parallel/algorithm>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "../include/crgc.h"

namespace {

constexpr uint64_t K_EMPTY = ~0ull, K_TOMB = ~0ull - 1;
constexpr uint32_t V_PEND = ~0u, NONE = ~0u;
constexpr uint8_t ALIVE = 1, INTERNED = 2, LOCAL = 4, BUSY = 8, ROOT = 16, HALTED = 32;

inline uint64_t mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

struct Edge {
  uint32_t t;
  int32_t c;
};

struct Graph {
  uint32_t F = 4;
  uint64_t hcap = 0, scap = 0;
  std::vector<uint64_t> hkey;
  std::vector<uint32_t> hval;
  std::vector<uint64_t> vid, vseq, sseq;
  std::vector<int32_t> recv;
  std::vector<uint8_t> flags, mark;
  std::vector<uint32_t> sup;
  std::vector<std::vector<Edge>> out;
  uint64_t slot_top = 0, inserted = 0, epoch = 0;
  uint64_t n_live = 0;
};

uint32_t resolve(Graph &g, uint64_t id) {
  uint64_t h = mix(id) & (g.hcap - 1);
  for (;;) {
    uint64_t k = __atomic_load_n(&g.hkey[h], __ATOMIC_ACQUIRE);
    if (k == K_EMPTY) {
      uint64_t exp = K_EMPTY;
      if (__atomic_compare_exchange_n(&g.hkey[h], &exp, id, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        const uint64_t s = __atomic_fetch_add(&g.slot_top, 1, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g.inserted, 1, __ATOMIC_RELAXED);
        g.vid[s] = id;
        g.recv[s] = 0;
        g.flags[s] = ALIVE;
        g.sup[s] = NONE;
        g.vseq[s] = g.sseq[s] = 0;
        __atomic_store_n(&g.hval[h], (uint32_t)s, __ATOMIC_RELEASE);
        return (uint32_t)s;
      }
      k = exp;
    }
    if (k == id) {
      uint32_t v;
      while ((v = __atomic_load_n(&g.hval[h], __ATOMIC_ACQUIRE)) == V_PEND) {
      }
      return v;
    }
    h = (h + 1) & (g.hcap - 1);
  }
}

void reserve(Graph &g, uint64_t more) {
  const uint64_t need = g.slot_top + more;
  if (need <= g.scap && need * 2 <= g.hcap) return;
  uint64_t cap = std::max<uint64_t>(g.scap * 2, need + need / 2 + 1024);
  g.vid.resize(cap);
  g.vseq.resize(cap);
  g.sseq.resize(cap);
  g.recv.resize(cap);
  g.flags.resize(cap);
  g.mark.resize(cap);
  g.sup.resize(cap);
  g.out.resize(cap);
  g.scap = cap;
  if (need * 2 > g.hcap) {
    uint64_t hc = 1;
    while (hc < 4 * need) hc <<= 1;
    std::vector<uint64_t> nk(hc, K_EMPTY);
    std::vector<uint32_t> nv(hc, V_PEND);
    for (uint64_t i = 0; i < g.hcap; ++i) {
      const uint64_t k = g.hkey[i];
      if (k == K_EMPTY || k == K_TOMB) continue;
      uint64_t h = mix(k) & (hc - 1);
      while (nk[h] != K_EMPTY) h = (h + 1) & (hc - 1);
      nk[h] = k;
      nv[h] = g.hval[i];
    }
    g.hkey.swap(nk);
    g.hval.swap(nv);
    g.hcap = hc;
  }
}

inline void atomic_add(int32_t *p, int32_t d) {  // Java int wraparound
  __atomic_fetch_add(reinterpret_cast<uint32_t *>(p), (uint32_t)d, __ATOMIC_RELAXED);
}
inline void atomic_max(uint64_t *p, uint64_t v) {
  uint64_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (cur < v && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
}

// The slot of a live id, or NONE (no insert: mergeUndoLog's existence checks).
uint32_t lookup(const Graph &g, uint64_t id) {
  uint64_t h = mix(id) & (g.hcap - 1);
  for (uint64_t p = 0; p < g.hcap; ++p) {
    const uint64_t k = g.hkey[h];
    if (k == id) return g.hval[h];
    if (k == K_EMPTY) return NONE;
    h = (h + 1) & (g.hcap - 1);
  }
  return NONE;
}

// outgoing[o][t] += c for every atom (owner << 32 | target, c): sorted,
// reduced, merged per owner into its target-sorted vector; a zero count is
// removed (updateOutgoing, ShadowGraph.java:64-73).
void apply_atoms(Graph &g, std::vector<std::pair<uint64_t, int32_t>> &atoms) {
  __gnu_parallel::sort(atoms.begin(), atoms.end(),
                       [](const auto &x, const auto &y) { return x.first < y.first; });
  std::vector<std::pair<uint64_t, int32_t>> red;
  red.reserve(atoms.size());
  for (auto &a : atoms) {
    if (!red.empty() && red.back().first == a.first) red.back().second = (int32_t)((uint32_t)red.back().second + (uint32_t)a.second);
    else red.push_back(a);
  }
  std::vector<uint64_t> runs;  // first atom of each owner's run
  for (uint64_t k = 0; k < red.size(); ++k)
    if (k == 0 || (red[k].first >> 32) != (red[k - 1].first >> 32)) runs.push_back(k);
  runs.push_back(red.size());
  const uint64_t n_runs = runs.size() - 1;
#pragma omp parallel for schedule(dynamic, 64)
  for (uint64_t r = 0; r < n_runs; ++r) {
    const uint32_t o = (uint32_t)(red[runs[r]].first >> 32);
    std::vector<Edge> &cur = g.out[o];
    std::vector<Edge> nxt;
    nxt.reserve(cur.size() + (runs[r + 1] - runs[r]));
    uint64_t a = runs[r], e = 0;
    while (a < runs[r + 1] || e < cur.size()) {
      const uint32_t ta = a < runs[r + 1] ? (uint32_t)red[a].first : ~0u;
      const uint32_t te = e < cur.size() ? cur[e].t : ~0u;
      if (te < ta) {
        nxt.push_back(cur[e++]);
      } else {
        int32_t c = red[a].second;
        if (te == ta) c = (int32_t)((uint32_t)c + (uint32_t)cur[e++].c);
        if (c) nxt.push_back({ta, c});
        ++a;
      }
    }
    cur.swap(nxt);
  }
}

inline bool reserved(uint64_t id) { return id >= K_TOMB || (id >> 48) == 0xFFFFull; }

}  // namespace

extern "C" {

void *omp_graph_create(uint32_t F, uint64_t vertex_hint) {
  Graph *g = new (std::nothrow) Graph();
  if (!g) return nullptr;
  g->F = F ? F : 4;
  reserve(*g, std::max<uint64_t>(vertex_hint, 1024));
  return g;
}

void omp_graph_destroy(void *h) { delete (Graph *)h; }

// N x ShadowGraph.mergeEntry in batch order.  Returns 0 or CRGC_E_INVAL.
int omp_graph_merge(void *h, const crgc_entry_batch *b, int threads) {
  Graph &g = *(Graph *)h;
  if (!b || b->memory != CRGC_MEM_HOST) return CRGC_E_INVAL;
  if (threads > 0) omp_set_num_threads(threads);
  const uint64_t n = b->n_entries;
  if (!n) return 0;
  const uint64_t C = b->created_off[n], S = b->spawned_off[n], U = b->updated_off[n];
  reserve(g, n + 2 * C + S + U);
  const uint64_t ep = ++g.epoch;
  std::vector<uint32_t> me(n), co(C), ct(C), sp(S), ut(U);
  // ids -> slots: target before owner (:88, :91) only orders `from`, unobservable here
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) me[i] = resolve(g, b->self[i]);
#pragma omp parallel for schedule(static)
  for (uint64_t k = 0; k < C; ++k) {
    ct[k] = resolve(g, b->created_target[k]);
    co[k] = resolve(g, b->created_owner[k]);
  }
#pragma omp parallel for schedule(static)
  for (uint64_t k = 0; k < S; ++k) sp[k] = resolve(g, b->spawned[k]);
#pragma omp parallel for schedule(static)
  for (uint64_t k = 0; k < U; ++k) ut[k] = resolve(g, b->updated_ref[k]);
  // receive counts and the last-write-wins tags
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t tag = (ep << 32) | (i + 1);
    if (b->recv_count[i]) atomic_add(&g.recv[me[i]], b->recv_count[i]);
    atomic_max(&g.vseq[me[i]], tag);
    for (uint32_t k = b->spawned_off[i]; k < b->spawned_off[i + 1]; ++k) atomic_max(&g.sseq[sp[k]], tag);
    for (uint32_t k = b->updated_off[i]; k < b->updated_off[i + 1]; ++k) {
      const int32_t cnt = (int16_t)(((int32_t)b->updated_info[k]) >> 1);
      if (cnt > 0) atomic_add(&g.recv[ut[k]], -cnt);
    }
  }
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t tag = (ep << 32) | (i + 1);
    const uint32_t s = me[i];
    if (g.vseq[s] == tag) {
      uint8_t f = (uint8_t)((g.flags[s] & ~(BUSY | ROOT)) | INTERNED | LOCAL);
      if (b->flags[i] & CRGC_ENTRY_BUSY) f |= BUSY;
      if (b->flags[i] & CRGC_ENTRY_ROOT) f |= ROOT;
      g.flags[s] = f;
    }
    for (uint32_t k = b->spawned_off[i]; k < b->spawned_off[i + 1]; ++k)
      if (g.sseq[sp[k]] == tag) g.sup[sp[k]] = s;
  }
  // edge atoms: sort by (owner, target), reduce, merge per owner
  std::vector<std::pair<uint64_t, int32_t>> atoms;
  atoms.reserve(C + U);
  for (uint64_t k = 0; k < C; ++k) atoms.push_back({((uint64_t)co[k] << 32) | ct[k], 1});
  for (uint64_t i = 0; i < n; ++i)
    for (uint32_t k = b->updated_off[i]; k < b->updated_off[i + 1]; ++k)
      if (b->updated_info[k] & 1) atoms.push_back({((uint64_t)me[i] << 32) | ut[k], -1});
  apply_atoms(g, atoms);
  return 0;
}

// N x ShadowGraph.mergeDelta in batch order (ShadowGraph.java:127-156).
// Returns 0 or CRGC_E_INVAL.
int omp_graph_merge_deltas(void *h, const crgc_delta_batch *b, int threads) {
  Graph &g = *(Graph *)h;
  if (!b || b->memory != CRGC_MEM_HOST) return CRGC_E_INVAL;
  if (threads > 0) omp_set_num_threads(threads);
  const uint64_t n = b->n_shadows;
  if (!n) return 0;
  const uint64_t O = b->out_off[n];
  for (uint64_t i = 0; i < n; ++i) {
    if (reserved(b->id[i]) || (b->supervisor[i] != CRGC_NO_ACTOR && reserved(b->supervisor[i])) ||
        b->out_off[i + 1] < b->out_off[i])
      return CRGC_E_INVAL;
  }
  for (uint64_t k = 0; k < O; ++k)
    if (reserved(b->out_target[k])) return CRGC_E_INVAL;
  reserve(g, 2 * n + O);
  const uint64_t ep = ++g.epoch;
  std::vector<uint32_t> me(n), su(n), ot(O);
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    me[i] = resolve(g, b->id[i]);
    su[i] = b->supervisor[i] != CRGC_NO_ACTOR ? resolve(g, b->supervisor[i]) : NONE;
  }
#pragma omp parallel for schedule(static)
  for (uint64_t k = 0; k < O; ++k) ot[k] = resolve(g, b->out_target[k]);
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t tag = (ep << 32) | (i + 1);
    const uint32_t s = me[i];
    if (b->recv_count[i]) atomic_add(&g.recv[s], b->recv_count[i]);
    if (b->flags[i] & CRGC_DELTA_INTERNED) {  // interned |= ; busy / root only when interned (:139-146)
      __atomic_fetch_or(&g.flags[s], INTERNED, __ATOMIC_RELAXED);
      atomic_max(&g.vseq[s], tag);
    }
    if (su[i] != NONE) atomic_max(&g.sseq[s], tag);
  }
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t tag = (ep << 32) | (i + 1);
    const uint32_t s = me[i];
    if ((b->flags[i] & CRGC_DELTA_INTERNED) && g.vseq[s] == tag) {
      uint8_t f = (uint8_t)(g.flags[s] & ~(BUSY | ROOT));
      if (b->flags[i] & CRGC_DELTA_BUSY) f |= BUSY;
      if (b->flags[i] & CRGC_DELTA_ROOT) f |= ROOT;
      g.flags[s] = f;
    }
    if (su[i] != NONE && g.sseq[s] == tag) g.sup[s] = su[i];
  }
  std::vector<std::pair<uint64_t, int32_t>> atoms;
  atoms.reserve(O);
  for (uint64_t i = 0; i < n; ++i)
    for (uint32_t k = b->out_off[i]; k < b->out_off[i + 1]; ++k)
      atoms.push_back({((uint64_t)me[i] << 32) | ot[k], b->out_count[k]});
  apply_atoms(g, atoms);
  return 0;
}

// ShadowGraph.mergeUndoLog (ShadowGraph.java:158-174).  Returns 0,
// CRGC_E_INVAL (a reserved or repeated actor), or CRGC_E_UNDO_NEW_SHADOW (the
// reference's ConcurrentModificationException: an admitted actor's created ref
// names an unknown actor) with the graph unchanged.
int omp_graph_merge_undo(void *h, const crgc_undo_log *log, int threads) {
  Graph &g = *(Graph *)h;
  if (!log || log->memory != CRGC_MEM_HOST) return CRGC_E_INVAL;
  if (threads > 0) omp_set_num_threads(threads);
  const uint64_t n = log->n_fields;
  std::vector<uint64_t> ids(log->actor, log->actor + n);
  for (uint64_t f = 0; f < n; ++f)
    if (reserved(ids[f])) return CRGC_E_INVAL;
  std::sort(ids.begin(), ids.end());
  for (uint64_t f = 1; f < n; ++f)
    if (ids[f] == ids[f - 1]) return CRGC_E_INVAL;  // UndoLog.admitted: one field per actor
  std::vector<uint32_t> me(n);
  int cme = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(| : cme)
  for (uint64_t f = 0; f < n; ++f) {
    me[f] = lookup(g, log->actor[f]);
    if (me[f] == NONE) continue;  // not a shadow here: the log's field is not applied
    for (uint32_t k = log->created_off[f]; k < log->created_off[f + 1]; ++k)
      if (lookup(g, log->created_target[k]) == NONE) cme = 1;
  }
  if (cme) return CRGC_E_UNDO_NEW_SHADOW;
  const uint64_t top = g.slot_top;
#pragma omp parallel for schedule(static)
  for (uint64_t v = 0; v < top; ++v)
    if ((g.flags[v] & ALIVE) && (uint16_t)(g.vid[v] >> 48) == log->node_location) g.flags[v] |= HALTED;
  std::vector<std::pair<uint64_t, int32_t>> atoms;
  for (uint64_t f = 0; f < n; ++f) {
    if (me[f] == NONE) continue;
    if (log->message_count[f]) atomic_add(&g.recv[me[f]], log->message_count[f]);
    for (uint32_t k = log->created_off[f]; k < log->created_off[f + 1]; ++k)
      atoms.push_back({((uint64_t)me[f] << 32) | lookup(g, log->created_target[k]), log->created_count[k]});
  }
  apply_atoms(g, atoms);
  return 0;
}

// ShadowGraph.trace(shouldKill).  Returns 0 or CRGC_E_NULL_SUPERVISOR (graph
// unchanged).  *edges = traced (nonzero) out-edges.  With id buffers the
// garbage / kill ids are written too (order unspecified; CRGC_E2BIG, after the
// trace, when a capacity is short — the counts are exact either way).
int omp_graph_trace(void *h, int should_kill, int threads, uint64_t *n_garbage, uint64_t *n_kill, uint64_t *n_live,
                    uint64_t *edges, uint64_t *pseudo_roots, uint64_t *garbage_ids, uint64_t garbage_cap,
                    uint64_t *kill_ids, uint64_t kill_cap) {
  Graph &g = *(Graph *)h;
  if (threads > 0) omp_set_num_threads(threads);
  const uint64_t top = g.slot_top;
  std::fill(g.mark.begin(), g.mark.begin() + top, 0);
  std::vector<uint32_t> front;
  uint64_t pr = 0;
#pragma omp parallel
  {
    std::vector<uint32_t> mine;
#pragma omp for schedule(static) reduction(+ : pr)
    for (uint64_t v = 0; v < top; ++v) {
      const uint8_t f = g.flags[v];
      if ((f & ALIVE) && !(f & HALTED) && ((f & (ROOT | BUSY)) || g.recv[v] != 0 || !(f & INTERNED))) {
        g.mark[v] = 1;
        mine.push_back((uint32_t)v);
        ++pr;
      }
    }
#pragma omp critical
    front.insert(front.end(), mine.begin(), mine.end());
  }
  uint64_t ed = 0;
  while (!front.empty()) {
    std::vector<uint32_t> next;
#pragma omp parallel
    {
      std::vector<uint32_t> mine;
      auto claim = [&](uint32_t t) {
        uint8_t z = 0;
        if (!g.mark[t] && __atomic_compare_exchange_n(&g.mark[t], &z, 1, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED))
          mine.push_back(t);
      };
#pragma omp for schedule(dynamic, 256) reduction(+ : ed)
      for (uint64_t i = 0; i < front.size(); ++i) {
        const uint32_t v = front[i];
        if (g.flags[v] & HALTED) continue;  // (:226-229)
        const std::vector<Edge> &es = g.out[v];
        ed += es.size();
        for (const Edge &e : es)
          if (e.c > 0) claim(e.t);
        if (g.sup[v] != NONE) claim(g.sup[v]);
      }
#pragma omp critical
      next.insert(next.end(), mine.begin(), mine.end());
    }
    front.swap(next);
  }
  uint64_t ng = 0, nk = 0, nl = 0, npe = 0;
  const bool want_ids = garbage_ids || kill_ids;
  std::vector<uint64_t> gl, kl;
#pragma omp parallel
  {
    std::vector<uint64_t> mg, mk;
#pragma omp for schedule(static) reduction(+ : ng, nk, nl, npe)
    for (uint64_t v = 0; v < top; ++v) {
      const uint8_t f = g.flags[v];
      if (!(f & ALIVE)) continue;
      if (g.mark[v]) {
        ++nl;
        continue;
      }
      ++ng;
      if (want_ids) mg.push_back(g.vid[v]);
      if (f & LOCAL) {
        const uint32_t s = g.sup[v];
        if (s == NONE) ++npe;
        else if (should_kill && !(f & HALTED) && g.mark[s] && (g.flags[s] & ALIVE)) {
          ++nk;
          if (want_ids) mk.push_back(g.vid[v]);
        }
      }
    }
    if (want_ids) {
#pragma omp critical
      {
        gl.insert(gl.end(), mg.begin(), mg.end());
        kl.insert(kl.end(), mk.begin(), mk.end());
      }
    }
  }
  if (npe) return CRGC_E_NULL_SUPERVISOR;
#pragma omp parallel for schedule(static)
  for (uint64_t v = 0; v < top; ++v) {
    if (!(g.flags[v] & ALIVE) || g.mark[v]) continue;
    uint64_t hh = mix(g.vid[v]) & (g.hcap - 1);
    while (g.hkey[hh] != g.vid[v]) hh = (hh + 1) & (g.hcap - 1);
    g.hkey[hh] = K_TOMB;  // removed from shadowMap (:276); the next getShadow makes a new shadow
    g.flags[v] = 0;
    std::vector<Edge>().swap(g.out[v]);
  }
  bool big = false;
  if (garbage_ids) {
    if (gl.size() <= garbage_cap) std::copy(gl.begin(), gl.end(), garbage_ids);
    else big = true;
  }
  if (kill_ids) {
    if (kl.size() <= kill_cap) std::copy(kl.begin(), kl.end(), kill_ids);
    else big = true;
  }
  g.n_live = nl;
  *n_garbage = ng;
  *n_kill = nk;
  *n_live = nl;
  *edges = ed;
  *pseudo_roots = pr;
  return big ? CRGC_E2BIG : 0;
}

}  // extern "C"
