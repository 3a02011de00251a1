// world.cpp — seeded synthetic entry streams for the bench and parity tests.
//
// A native mirror of the CRGC mutator (CRGC.scala:69-221, State.java:45-124,
// RefobInfo.java) that can drive 1e7 actors: it emits Entry records in queue
// order exactly as the JVM engine would flush them, including the forced
// busy flushes when an entry's F slots fill up.  Not part of the product: it
// produces the inputs (SURVEY §8d "Synthetic inputs") that bench.py uploads to
// HBM before its timed region.
//
//  * wl_bulk_graph  C2 shape: a spawn tree plus a power-law acquaintance graph
//                   (Pareto out-degree, preferential-attachment targets), as
//                   the entries that would have built it.
//  * wl_chain_graph C3 shape: long live chains hanging off roots, deep
//                   supervisor chains, dead rings and dead chains.
//  * wl_simulate    steady state: actors with mail take turns (receive, then
//                   send / share / release / spawn), RandomSpec-style.
//  * wl_uniform_graph  C1 shape: uniform acquaintances, counts
//                   1 / 2 / -1, planted dead components.
//  * wl_wakeup      one wakeup's batch with turns in flight at its cut: a
//                   target share of the actors busy (mid-turn, last flush
//                   isBusy = true) and a target share with undelivered mail
//                   (receive count not yet flushed), as LocalGC sees a running
//                   system when its timer drains the queue.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Rng {  // splitmix64
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

struct Refob {
  uint32_t target;
  int16_t info;
  uint8_t recorded;
  uint8_t _pad;
};

struct Actor {
  uint64_t id;
  uint32_t self_refob;
  uint32_t mailbox = 0;
  bool root = false;
  bool ready = false;
  bool busy = false;       // mid-turn across a wakeup boundary (wl_wakeup)
  uint32_t busy_at = 0;    // index in wl_world::busy
  float budget_left = 0;   // actions of the turn still to do
  std::vector<uint32_t> held;   // refob indices this actor holds
  std::vector<uint32_t> inbox;  // refobs carried by pending messages
};

struct State {  // State.java
  uint32_t F;
  std::vector<std::pair<uint32_t, uint32_t>> created;  // (owner actor, target actor)
  std::vector<uint32_t> spawned;                       // child actors
  std::vector<uint32_t> updated;                       // refob indices
  int32_t recv = 0;
  void clear() {
    created.clear();
    spawned.clear();
    updated.clear();
    recv = 0;
  }
};

}  // namespace

extern "C" {

typedef struct wl_batch {
  uint64_t n, C, S, U;
  const uint64_t *self;
  const int16_t *recv;
  const uint8_t *flags;
  const uint32_t *c_off;
  const uint64_t *c_owner;
  const uint64_t *c_target;
  const uint32_t *s_off;
  const uint64_t *spawned;
  const uint32_t *u_off;
  const uint64_t *u_ref;
  const int16_t *u_info;
} wl_batch;

struct wl_world {
  Rng rng{1};
  uint32_t F = 4;
  uint16_t location = 1;
  std::vector<Actor> actors;
  std::vector<Refob> refobs;
  std::vector<uint32_t> free_refobs;
  std::vector<uint32_t> roots;
  std::vector<uint32_t> ready;  // actors with mail
  std::vector<uint32_t> busy;   // actors mid-turn (wl_wakeup)
  State st;
  // queued entries (struct of arrays, appended in flush order)
  std::vector<uint64_t> q_self;
  std::vector<int16_t> q_recv;
  std::vector<uint8_t> q_flags;
  std::vector<uint32_t> q_coff{0}, q_soff{0}, q_uoff{0};
  std::vector<uint64_t> q_cown, q_ctgt, q_sp, q_uref;
  std::vector<int16_t> q_uinf;
  uint64_t head = 0;  // first entry not yet taken
  // last taken batch (rebased copies)
  std::vector<uint32_t> t_coff, t_soff, t_uoff;
  // op mix: send / share / release / spawn
  double p_send = 0.40, p_share = 0.20, p_release = 0.20, p_spawn = 0.10;
  double actions_per_msg = 1.5;
  uint64_t n_entries_emitted = 0;
  uint32_t id_space = 0;  // 0: the historical id map (C1-C3, C5 streams); k: mix48(k << 32 | index)
};

// A bijection of the 48-bit integers (xor-shifts and odd multipliers mod 2^48).
static uint64_t mix48(uint64_t x) {
  const uint64_t M = 0xFFFFFFFFFFFFull;
  x &= M;
  x ^= x >> 23;
  x = (x * 0x9E3779B97F4A7C15ull) & M;
  x ^= x >> 25;
  x = (x * 0xBF58476D1CE4E5B9ull) & M;
  x ^= x >> 21;
  return x;
}

static uint64_t make_id(wl_world *w, uint64_t idx) {
  // Id space k > 0 (C4's components, wl_set_id_space): a bijection of
  // (k, actor index), so several simulated producers of one node never share an id.
  if (w->id_space) return ((uint64_t)w->location << 48) | mix48(((uint64_t)w->id_space << 32) | idx);
  // random-looking 48-bit local part so hash placement is uniform
  uint64_t x = (idx + 1) * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29;
  return ((uint64_t)w->location << 48) | ((x ^ (idx << 20)) & 0xFFFFFFFFFFFFull);
}

static uint32_t new_refob(wl_world *w, uint32_t target) {
  uint32_t r;
  if (!w->free_refobs.empty()) {
    r = w->free_refobs.back();
    w->free_refobs.pop_back();
  } else {
    r = (uint32_t)w->refobs.size();
    w->refobs.push_back({});
  }
  w->refobs[r] = Refob{target, 0, 0, 0};
  return r;
}

static uint32_t new_actor(wl_world *w) {
  uint32_t a = (uint32_t)w->actors.size();
  w->actors.emplace_back();
  Actor &x = w->actors.back();
  x.id = make_id(w, a);
  x.self_refob = new_refob(w, a);
  return a;
}

// Entry flush: State.flushToEntry (State.java:90-124) + Queue.add.
static void flush(wl_world *w, uint32_t actor, State &s, bool busy) {
  Actor &x = w->actors[actor];
  w->q_self.push_back(x.id);
  w->q_recv.push_back((int16_t)s.recv);
  w->q_flags.push_back((busy ? 1 : 0) | (x.root ? 2 : 0));
  for (auto &p : s.created) {
    w->q_cown.push_back(w->actors[p.first].id);
    w->q_ctgt.push_back(w->actors[p.second].id);
  }
  for (uint32_t c : s.spawned) w->q_sp.push_back(w->actors[c].id);
  for (uint32_t r : s.updated) {
    Refob &ro = w->refobs[r];
    w->q_uref.push_back(w->actors[ro.target].id);
    w->q_uinf.push_back(ro.info);
    ro.recorded = 0;
    const bool released = ro.info & 1;
    ro.info = 0;  // Refob.reset
    if (released) w->free_refobs.push_back(r);
  }
  w->q_coff.push_back((uint32_t)w->q_cown.size());
  w->q_soff.push_back((uint32_t)w->q_sp.size());
  w->q_uoff.push_back((uint32_t)w->q_uref.size());
  w->n_entries_emitted++;
  s.clear();
}

static bool can_record_updated(const State &s, const Refob &r) {
  return r.recorded || s.updated.size() < s.F;
}
static void record_updated(State &s, Refob &r, uint32_t idx) {
  if (r.recorded) return;
  r.recorded = 1;
  s.updated.push_back(idx);
}

static void deliver(wl_world *w, uint32_t target, int carried) {
  Actor &t = w->actors[target];
  t.mailbox++;
  if (carried >= 0) t.inbox.push_back((uint32_t)carried);
  if (!t.ready && !t.busy) {  // a busy actor reads it when its turn goes on
    t.ready = true;
    w->ready.push_back(target);
  }
}

// CRGC.sendMessageImpl (CRGC.scala:208-221)
static void do_send(wl_world *w, uint32_t me, uint32_t r, int carried) {
  Refob &ro = w->refobs[r];
  if (!(ro.info <= 32767 - 2) || !can_record_updated(w->st, ro)) flush(w, me, w->st, true);
  ro.info = (int16_t)(ro.info + 2);
  record_updated(w->st, w->refobs[r], r);
  deliver(w, w->refobs[r].target, carried);
}

static uint32_t random_held(wl_world *w, Actor &x) {
  return x.held[w->rng.below(x.held.size())];
}

// One action of a turn (RandomSpec's doSomething mix, CRGC hooks).
static void act(wl_world *w, uint32_t me) {
  const double p = w->rng.uni();
  Actor &x = w->actors[me];
  if (p < w->p_send) {
    if (x.held.empty()) return;
    do_send(w, me, random_held(w, x), -1);
  } else if (p < w->p_send + w->p_share) {
    if (x.held.empty()) return;
    const uint32_t r1 = random_held(w, x), r2 = random_held(w, x);
    const uint32_t owner = w->refobs[r1].target, target = w->refobs[r2].target;
    const uint32_t fresh = new_refob(w, target);  // createRefImpl (CRGC.scala:151-162)
    if (w->st.created.size() >= w->F) flush(w, me, w->st, true);
    w->st.created.push_back({owner, target});
    do_send(w, me, r1, (int)fresh);
  } else if (p < w->p_send + w->p_share + w->p_release) {
    if (x.held.empty()) return;
    const uint64_t k = w->rng.below(x.held.size());
    const uint32_t r = x.held[k];
    x.held[k] = x.held.back();
    x.held.pop_back();
    Refob &ro = w->refobs[r];
    if (!can_record_updated(w->st, ro)) flush(w, me, w->st, true);  // releaseImpl
    w->refobs[r].info = (int16_t)(w->refobs[r].info | 1);
    record_updated(w->st, w->refobs[r], r);
  } else if (p < w->p_send + w->p_share + w->p_release + w->p_spawn) {
    // spawnImpl (CRGC.scala:100-112); the child runs initState and blocks.
    const uint32_t c = new_actor(w);
    Actor &child = w->actors[c];
    State cs;
    cs.F = w->F;
    cs.created.push_back({c, c});
    cs.created.push_back({me, c});
    flush(w, c, cs, false);
    (void)child;
    if (w->st.spawned.size() >= w->F) flush(w, me, w->st, true);
    w->st.spawned.push_back(c);
    w->actors[me].held.push_back(new_refob(w, c));
  }
}

// A mailbox batch: receive everything, act, then block (on-block flush).
static void turn(wl_world *w, uint32_t me) {
  Actor &x = w->actors[me];
  const uint32_t msgs = x.mailbox;
  x.mailbox = 0;
  x.ready = false;
  std::vector<uint32_t> inbox;
  inbox.swap(x.inbox);
  for (uint32_t m = 0; m < msgs; ++m) {
    if (w->st.recv >= 32767) flush(w, me, w->st, true);  // onMessageImpl
    w->st.recv++;
  }
  for (uint32_t r : inbox) w->actors[me].held.push_back(r);
  double budget = msgs * w->actions_per_msg;
  while (budget > 0) {
    if (budget >= 1 || w->rng.uni() < budget) act(w, me);
    budget -= 1;
  }
  flush(w, me, w->st, false);
}

wl_world *wl_create(uint64_t seed, uint32_t F, uint16_t location) {
  wl_world *w = new wl_world();
  w->rng = Rng(seed * 0x2545F4914F6CDD1Dull + 0x5EED);
  w->F = F ? F : 4;
  w->st.F = w->F;
  w->location = location;
  return w;
}

void wl_destroy(wl_world *w) { delete w; }

// Before any actor exists: ids from the injective map of space k (1..65535).
int wl_set_id_space(wl_world *w, uint32_t k) {
  if (!w->actors.empty() || k > 0xFFFF) return -1;
  w->id_space = k;
  return 0;
}

void wl_set_mix(wl_world *w, double p_send, double p_share, double p_release, double p_spawn,
                double actions_per_msg) {
  w->p_send = p_send;
  w->p_share = p_share;
  w->p_release = p_release;
  w->p_spawn = p_spawn;
  w->actions_per_msg = actions_per_msg;
}

// C2 / C1 / C4 shape.  Roots are the first n_roots actors; every other actor's
// parent is uniform among earlier actors; acquaintance out-degrees are Pareto
// (alpha, min 1, cap) scaled to n_edges in total, targets by preferential
// attachment (endpoint of a uniformly chosen existing edge).
void wl_bulk_graph(wl_world *w, uint64_t n_actors, uint64_t n_edges, double alpha,
                   uint32_t n_roots, uint64_t cap) {
  Rng &g = w->rng;
  const uint64_t base = w->actors.size();
  w->actors.reserve(base + n_actors);
  for (uint64_t i = 0; i < n_actors; ++i) new_actor(w);
  for (uint32_t r = 0; r < n_roots && r < n_actors; ++r) {
    w->actors[base + r].root = true;
    w->roots.push_back((uint32_t)(base + r));
  }
  // Roots' initial entries: self-edge, isRoot.
  State s;
  s.F = w->F;
  for (uint32_t r = 0; r < n_roots && r < n_actors; ++r) {
    const uint32_t a = (uint32_t)(base + r);
    s.created.push_back({a, a});
    flush(w, a, s, false);
  }
  // Spawn tree: parent records `spawned`, child's init entry records
  // (child,child) and (parent,child); the parent holds a refob to the child.
  std::vector<uint32_t> pend_parent;
  for (uint64_t i = n_roots; i < n_actors; ++i) {
    const uint32_t c = (uint32_t)(base + i);
    const uint32_t p = (uint32_t)(base + (i < 4 * (uint64_t)n_roots ? g.below(n_roots)
                                                                      : g.below(i)));
    State ps;
    ps.F = w->F;
    ps.spawned.push_back(c);
    flush(w, p, ps, false);
    s.created.push_back({c, c});
    s.created.push_back({p, c});
    flush(w, c, s, false);
    w->actors[p].held.push_back(new_refob(w, c));
  }
  // Acquaintance edges: Pareto out-degree, preferential-attachment targets.
  const double mean_par = alpha > 1 ? alpha / (alpha - 1) : 2.0;
  const double scale = (double)n_edges / (double)std::max<uint64_t>(n_actors, 1) / mean_par;
  std::vector<uint32_t> endpoints;
  endpoints.reserve(n_edges + n_actors);
  for (uint64_t i = 0; i < n_actors; ++i) endpoints.push_back((uint32_t)(base + i));
  uint64_t made = 0;
  for (uint64_t i = 0; i < n_actors && made < n_edges; ++i) {
    const uint32_t a = (uint32_t)(base + i);
    double d = scale * std::pow(1.0 - g.uni(), -1.0 / alpha);
    uint64_t deg = (uint64_t)d + (g.uni() < (d - std::floor(d)) ? 1 : 0);
    deg = std::min<uint64_t>(std::min<uint64_t>(deg, cap), n_edges - made);
    for (uint64_t k = 0; k < deg; ++k) {
      const uint32_t t = endpoints[g.below(endpoints.size())];
      if (s.created.size() >= w->F) flush(w, a, s, false);
      s.created.push_back({a, t});
      w->actors[a].held.push_back(new_refob(w, t));
      endpoints.push_back(t);
    }
    made += deg;
    if (!s.created.empty()) flush(w, a, s, false);
  }
}

// C3 shape: chains a_0 -> a_1 -> ... hanging off roots (each link spawned by
// its predecessor, so supervisor chains run the other way), supervisor-only
// chains of depth sup_depth, and dead rings / dead chains: shadows whose only
// incoming references come from each other (collected together).
void wl_chain_graph(wl_world *w, uint32_t n_chains, uint32_t chain_len, uint32_t n_sup_chains,
                    uint32_t sup_depth, uint32_t n_rings, uint32_t ring_len) {
  State s;
  s.F = w->F;
  auto link = [&](uint32_t parent, uint32_t child, bool parent_keeps) {
    State ps;
    ps.F = w->F;
    ps.spawned.push_back(child);
    flush(w, parent, ps, false);
    s.created.push_back({child, child});
    s.created.push_back({parent, child});
    flush(w, child, s, false);
    if (parent_keeps) w->actors[parent].held.push_back(new_refob(w, child));
  };
  for (uint32_t c = 0; c < n_chains; ++c) {
    const uint32_t r = new_actor(w);
    w->actors[r].root = true;
    w->roots.push_back(r);
    s.created.push_back({r, r});
    flush(w, r, s, false);
    uint32_t prev = r;
    for (uint32_t k = 0; k < chain_len; ++k) {
      const uint32_t a = new_actor(w);
      link(prev, a, true);
      prev = a;
    }
  }
  // supervisor chains: each child spawned by the previous one, which then
  // releases it; only the deepest is referenced (by a root), so the chain is
  // live only through supervisor edges.
  for (uint32_t c = 0; c < n_sup_chains; ++c) {
    const uint32_t r = w->roots.empty() ? new_actor(w) : w->roots[c % w->roots.size()];
    if (w->roots.empty()) {
      w->actors[r].root = true;
      w->roots.push_back(r);
    }
    uint32_t prev = r;
    uint32_t last = r;
    for (uint32_t k = 0; k < sup_depth; ++k) {
      const uint32_t a = new_actor(w);
      State ps;
      ps.F = w->F;
      ps.spawned.push_back(a);
      flush(w, prev, ps, false);
      s.created.push_back({a, a});
      s.created.push_back({prev, a});
      flush(w, a, s, false);
      if (prev != r) {  // the spawner drops its reference to the child
        ps.updated.clear();
        const uint32_t ro = new_refob(w, a);
        w->refobs[ro].info = 1;
        w->refobs[ro].recorded = 1;
        ps.updated.push_back(ro);
        flush(w, prev, ps, false);
      }
      prev = a;
      last = a;
    }
    // the root references the deepest descendant
    s.created.push_back({r, last});
    flush(w, r, s, false);
  }
  // dead rings: members spawned by a root that immediately releases them,
  // linked in a cycle: unreachable, so collected (and killed, supervisor live)
  for (uint32_t c = 0; c < n_rings; ++c) {
    const uint32_t r = w->roots[c % w->roots.size()];
    std::vector<uint32_t> ring;
    for (uint32_t k = 0; k < ring_len; ++k) {
      const uint32_t a = new_actor(w);
      ring.push_back(a);
      State ps;
      ps.F = w->F;
      ps.spawned.push_back(a);
      flush(w, r, ps, false);
      s.created.push_back({a, a});
      s.created.push_back({r, a});
      flush(w, a, s, false);
    }
    for (uint32_t k = 0; k < ring_len; ++k) {
      const uint32_t a = ring[k], b = ring[(k + 1) % ring_len];
      s.created.push_back({a, b});
      flush(w, a, s, false);
    }
    // the root releases every member
    State ps;
    ps.F = w->F;
    for (uint32_t k = 0; k < ring_len; ++k) {
      const uint32_t ro = new_refob(w, ring[k]);
      w->refobs[ro].info = 1;
      w->refobs[ro].recorded = 1;
      if (ps.updated.size() >= w->F) flush(w, r, ps, false);
      ps.updated.push_back(ro);
    }
    flush(w, r, ps, false);
  }
}

// Steady state: run turns until `n_entries` more entries are queued.
void wl_simulate(wl_world *w, uint64_t n_entries) {
  const uint64_t goal = w->n_entries_emitted + n_entries;
  while (w->n_entries_emitted < goal) {
    if (w->ready.empty() || w->rng.uni() < 0.02) {
      if (w->roots.empty()) return;
      deliver(w, w->roots[w->rng.below(w->roots.size())], -1);  // a root's timer tick
    }
    const uint64_t k = w->rng.below(w->ready.size());
    const uint32_t a = w->ready[k];
    w->ready[k] = w->ready.back();
    w->ready.pop_back();
    turn(w, a);
  }
}

// C1 shape (BASELINE.json config 1): n_roots roots, a spawn tree
// (parent uniform among earlier actors), Poisson(mean_acq) acquaintances per
// live actor with uniform targets whose counts are 1 (90 %), 2 (8 %: two
// created refs) or -1 (2 %: a release whose creation is still unflushed by a
// busy creator), and dead components holding dead_frac of the actors: members
// spawned by a live actor that released them at once, linked in a cycle plus
// Poisson(2) extra internal refs each — unreachable, not pseudo-roots, killed
// (their supervisor is live).
static uint64_t poisson(Rng &g, double mean) {
  // Knuth, in chunks of 16 so exp() never underflows
  uint64_t k = 0;
  while (mean > 0) {
    const double m = mean > 16 ? 16 : mean;
    mean -= m;
    const double L = std::exp(-m);
    double p = 1.0;
    for (;;) {
      p *= g.uni();
      if (p <= L) break;
      ++k;
    }
  }
  return k;
}

void wl_uniform_graph(wl_world *w, uint64_t n_actors, double mean_acq, uint32_t n_roots, double dead_frac) {
  Rng &g = w->rng;
  const uint64_t base = w->actors.size();
  const uint64_t n_dead = (uint64_t)(dead_frac * (double)n_actors);
  const uint64_t n_live = n_actors - n_dead;
  w->actors.reserve(base + n_actors);
  for (uint64_t i = 0; i < n_actors; ++i) new_actor(w);
  State s;
  s.F = w->F;
  for (uint32_t r = 0; r < n_roots && r < n_live; ++r) {
    const uint32_t a = (uint32_t)(base + r);
    w->actors[a].root = true;
    w->roots.push_back(a);
    s.created.push_back({a, a});
    flush(w, a, s, false);
  }
  auto spawn = [&](uint32_t p, uint32_t c) {
    State ps;
    ps.F = w->F;
    ps.spawned.push_back(c);
    flush(w, p, ps, false);
    s.created.push_back({c, c});
    s.created.push_back({p, c});
    flush(w, c, s, false);
  };
  for (uint64_t i = n_roots; i < n_live; ++i) {
    const uint32_t c = (uint32_t)(base + i);
    const uint32_t p = (uint32_t)(base + (i < 4 * (uint64_t)n_roots ? g.below(n_roots) : g.below(i)));
    spawn(p, c);
    w->actors[p].held.push_back(new_refob(w, c));
  }
  for (uint64_t i = 0; i < n_live; ++i) {
    const uint32_t a = (uint32_t)(base + i);
    const uint64_t k = poisson(g, mean_acq);
    for (uint64_t j = 0; j < k; ++j) {
      const uint32_t t = (uint32_t)(base + g.below(n_live));
      const double u = g.uni();
      if (u < 0.98) {  // count 1, or 2 (two created refs)
        const int copies = u < 0.90 ? 1 : 2;
        for (int c = 0; c < copies; ++c) {
          if (s.created.size() >= w->F) flush(w, a, s, false);
          s.created.push_back({a, t});
          w->actors[a].held.push_back(new_refob(w, t));
        }
      } else {  // count -1: the owner's release of a ref whose creation is unflushed
        if (!s.created.empty() || !s.updated.empty()) flush(w, a, s, false);
        const uint32_t ro = new_refob(w, t);
        w->refobs[ro].info = 1;
        w->refobs[ro].recorded = 1;
        s.updated.push_back(ro);
        flush(w, a, s, false);
      }
    }
    if (!s.created.empty()) flush(w, a, s, false);
  }
  // dead components
  uint64_t next = n_live;
  while (next < n_actors) {
    const uint64_t size = std::min<uint64_t>(n_actors - next, 2 + g.below(19));
    const uint32_t p = (uint32_t)(base + g.below(n_live));
    std::vector<uint32_t> comp;
    for (uint64_t k = 0; k < size; ++k) comp.push_back((uint32_t)(base + next + k));
    next += size;
    State ps;
    ps.F = w->F;
    for (uint32_t c : comp) {
      spawn(p, c);
      const uint32_t ro = new_refob(w, c);  // ... and released at once
      w->refobs[ro].info = 1;
      w->refobs[ro].recorded = 1;
      if (ps.updated.size() >= w->F) flush(w, p, ps, false);
      ps.updated.push_back(ro);
    }
    flush(w, p, ps, false);
    for (uint64_t k = 0; k < size; ++k) {
      const uint32_t a = comp[k];
      const uint64_t extra = poisson(g, 2.0);
      std::vector<uint32_t> tg{comp[(k + 1) % size]};
      for (uint64_t e = 0; e < extra; ++e) tg.push_back(comp[g.below(size)]);
      for (uint32_t t : tg) {
        if (s.created.size() >= w->F) flush(w, a, s, false);
        s.created.push_back({a, t});
        w->actors[a].held.push_back(new_refob(w, t));
      }
      flush(w, a, s, false);
    }
  }
}

// ---- a wakeup with turns in flight at its cut (wl_wakeup) --------------------
// A busy turn starts like a turn (receive the mailbox, act on part of the
// budget), flushes with isBusy = true (CRGC.scala:215-216 forced flush / a turn
// running when LocalGC drains the queue) and stays open across the cut; it
// finishes in a later wakeup (mail that arrived meanwhile, the rest of the
// budget, the on-block flush with isBusy = false).
static void busy_remove(wl_world *w, uint32_t a) {
  Actor &x = w->actors[a];
  const uint32_t i = x.busy_at, last = w->busy.back();
  w->busy[i] = last;
  w->actors[last].busy_at = i;
  w->busy.pop_back();
  x.busy = false;
}

static void run_actions(wl_world *w, uint32_t me, double budget) {
  while (budget > 0) {
    if (budget >= 1 || w->rng.uni() < budget) act(w, me);
    budget -= 1;
  }
}

static uint32_t take_mail(wl_world *w, uint32_t me) {
  Actor &x = w->actors[me];
  const uint32_t msgs = x.mailbox;
  x.mailbox = 0;
  std::vector<uint32_t> inbox;
  inbox.swap(x.inbox);
  for (uint32_t m = 0; m < msgs; ++m) {
    if (w->st.recv >= 32767) flush(w, me, w->st, true);  // onMessageImpl
    w->st.recv++;
  }
  for (uint32_t r : inbox) w->actors[me].held.push_back(r);
  return msgs;
}

static void busy_start(wl_world *w, uint32_t me, double apm) {
  Actor &x = w->actors[me];
  x.ready = false;
  x.busy = true;  // before acting: a self-message must not queue it as ready
  x.busy_at = (uint32_t)w->busy.size();
  w->busy.push_back(me);
  const double budget = take_mail(w, me) * apm;
  const double now = std::ceil(budget * 0.75);
  run_actions(w, me, now);
  flush(w, me, w->st, true);
  w->actors[me].budget_left = (float)(budget - now);  // act() may grow `actors`
}

static void busy_finish(wl_world *w, uint32_t me, double apm) {
  busy_remove(w, me);
  const double budget = w->actors[me].budget_left + take_mail(w, me) * apm;
  w->actors[me].budget_left = 0;
  run_actions(w, me, budget);
  flush(w, me, w->st, false);
}

// Queue >= n_entries more entries so that, at the cut, about busy_target
// actors are mid-turn and about pending_target have undelivered mail.  The
// actions per received message adapt (hi while fewer than pending_target
// actors have mail, lo above it), which holds the number of actors with mail
// near the target without external messages (the reference's RandomSpec
// drives its actors from one root timer at 1 ms; at 1e5-1e7 actors a fixed
// rate would not keep a tenth of them busy).
void wl_wakeup(wl_world *w, uint64_t n_entries, uint64_t busy_target, uint64_t pending_target, double apm_lo,
               double apm_hi) {
  const uint64_t goal = w->n_entries_emitted + n_entries;
  // a quarter of the open turns end first (a busy turn spans ~4 wakeups),
  // at most 40 % of the batch
  uint64_t nf = std::min<uint64_t>(w->busy.size() / 4, n_entries * 2 / 5);
  while (w->n_entries_emitted < goal) {
    const double apm = w->ready.size() < pending_target ? apm_hi : apm_lo;
    if (nf && !w->busy.empty()) {
      --nf;
      busy_finish(w, w->busy[w->rng.below(w->busy.size())], apm);
      continue;
    }
    if (w->ready.empty()) {
      if (w->roots.empty()) return;
      const uint32_t r = w->roots[w->rng.below(w->roots.size())];
      if (!w->actors[r].busy) deliver(w, r, -1);  // a root's timer tick
      else busy_finish(w, r, apm);               // (a busy root reads it when it goes on)
      continue;
    }
    const uint64_t k = w->rng.below(w->ready.size());
    const uint32_t a = w->ready[k];
    w->ready[k] = w->ready.back();
    w->ready.pop_back();
    if (w->busy.size() < busy_target) {
      busy_start(w, a, apm);
    } else {
      const double save = w->actions_per_msg;
      w->actions_per_msg = apm;
      turn(w, a);
      w->actions_per_msg = save;
    }
  }
}

uint64_t wl_n_busy(wl_world *w) { return w->busy.size(); }
uint64_t wl_n_ready(wl_world *w) { return w->ready.size(); }

uint64_t wl_queued(wl_world *w) { return w->q_self.size() - w->head; }
uint64_t wl_n_actors(wl_world *w) { return w->actors.size(); }
uint64_t wl_n_refobs_held(wl_world *w) {
  uint64_t k = 0;
  for (auto &a : w->actors) k += a.held.size();
  return k;
}

// Take up to `max_entries` queued entries (queue order).  The views stay
// valid until the next wl_take / wl_simulate / wl_*_graph call.
int wl_take(wl_world *w, uint64_t max_entries, wl_batch *out) {
  const uint64_t h = w->head;
  const uint64_t n = std::min<uint64_t>(max_entries, w->q_self.size() - h);
  out->n = n;
  const uint32_t c0 = w->q_coff[h], s0 = w->q_soff[h], u0 = w->q_uoff[h];
  w->t_coff.resize(n + 1);
  w->t_soff.resize(n + 1);
  w->t_uoff.resize(n + 1);
  for (uint64_t i = 0; i <= n; ++i) {
    w->t_coff[i] = w->q_coff[h + i] - c0;
    w->t_soff[i] = w->q_soff[h + i] - s0;
    w->t_uoff[i] = w->q_uoff[h + i] - u0;
  }
  out->C = w->t_coff[n];
  out->S = w->t_soff[n];
  out->U = w->t_uoff[n];
  out->self = w->q_self.data() + h;
  out->recv = w->q_recv.data() + h;
  out->flags = w->q_flags.data() + h;
  out->c_off = w->t_coff.data();
  out->c_owner = w->q_cown.data() + c0;
  out->c_target = w->q_ctgt.data() + c0;
  out->s_off = w->t_soff.data();
  out->spawned = w->q_sp.data() + s0;
  out->u_off = w->t_uoff.data();
  out->u_ref = w->q_uref.data() + u0;
  out->u_info = w->q_uinf.data() + u0;
  w->head = h + n;
  return 0;
}

// Drop entries already taken (call between batches to bound memory).
void wl_compact(wl_world *w) {
  const uint64_t h = w->head;
  if (h == 0) return;
  const uint32_t c0 = w->q_coff[h], s0 = w->q_soff[h], u0 = w->q_uoff[h];
  w->q_self.erase(w->q_self.begin(), w->q_self.begin() + h);
  w->q_recv.erase(w->q_recv.begin(), w->q_recv.begin() + h);
  w->q_flags.erase(w->q_flags.begin(), w->q_flags.begin() + h);
  w->q_cown.erase(w->q_cown.begin(), w->q_cown.begin() + c0);
  w->q_ctgt.erase(w->q_ctgt.begin(), w->q_ctgt.begin() + c0);
  w->q_sp.erase(w->q_sp.begin(), w->q_sp.begin() + s0);
  w->q_uref.erase(w->q_uref.begin(), w->q_uref.begin() + u0);
  w->q_uinf.erase(w->q_uinf.begin(), w->q_uinf.begin() + u0);
  std::vector<uint32_t> co(w->q_coff.begin() + h, w->q_coff.end());
  std::vector<uint32_t> so(w->q_soff.begin() + h, w->q_soff.end());
  std::vector<uint32_t> uo(w->q_uoff.begin() + h, w->q_uoff.end());
  for (auto &x : co) x -= c0;
  for (auto &x : so) x -= s0;
  for (auto &x : uo) x -= u0;
  w->q_coff.swap(co);
  w->q_soff.swap(so);
  w->q_uoff.swap(uo);
  w->head = 0;
}

}  // extern "C"
