// deltas.cpp — host-side DeltaGraph production for the C5 cluster stream
// (bench / test input generation, not the product).
//
// A node with num-nodes > 1 folds every drained Entry into a DeltaGraph and
// broadcasts it once full (LocalGC.scala:159-177).  This restates
// DeltaGraph.mergeEntry / isFull (DeltaGraph.java:73-125, 174-180) in C++ so
// C5-sized streams can be generated quickly; workload/delta.py is the Python
// restatement the tests compare it with.  Output is the decoded batch the C
// ABI takes (crgc_delta_batch: ids through DeltaGraph.decoder, :162-169), with
// the DeltaGraph boundaries.
#include <cstddef>
#include <cstdint>
#include <unordered_map>
#include <vector>

namespace {

struct Shadow {
  int32_t recv = 0;
  int32_t sup = -1;  // compressed id, -1 = none
  bool interned = false, root = false, busy = false;
  std::vector<std::pair<int32_t, int32_t>> out;  // insertion order, zero deletes
};

void update(std::vector<std::pair<int32_t, int32_t>> &m, int32_t key, int32_t d) {
  for (size_t i = 0; i < m.size(); ++i) {
    if (m[i].first != key) continue;
    m[i].second += d;
    if (m[i].second == 0) m.erase(m.begin() + i);
    return;
  }
  if (d != 0) m.emplace_back(key, d);
}

struct Graph {
  std::unordered_map<uint64_t, int32_t> table;
  std::vector<uint64_t> decoder;
  std::vector<Shadow> shadows;
  int32_t encode(uint64_t ref) {
    auto it = table.find(ref);
    if (it != table.end()) return it->second;
    const int32_t i = (int32_t)shadows.size();
    table.emplace(ref, i);
    decoder.push_back(ref);
    shadows.emplace_back();
    return i;
  }
  void clear() {
    table.clear();
    decoder.clear();
    shadows.clear();
  }
};

inline int32_t refob_count(int16_t info) { return (int16_t)(((int32_t)info) >> 1); }
inline bool refob_active(int16_t info) { return (info & 1) == 0; }

}  // namespace

extern "C" {

typedef struct wl_entries {  // layout of world.cpp's wl_batch
  uint64_t n, C, S, U;
  const uint64_t *self;
  const int16_t *recv;
  const uint8_t *flags;  // bit 0 busy, bit 1 root
  const uint32_t *c_off;
  const uint64_t *c_owner;
  const uint64_t *c_target;
  const uint32_t *s_off;
  const uint64_t *spawned;
  const uint32_t *u_off;
  const uint64_t *u_ref;
  const int16_t *u_info;
} wl_entries;

typedef struct wl_deltas {
  uint64_t n_graphs, n_shadows, n_out;
  const uint32_t *graph_off;  // [n_graphs + 1]: shadows of DeltaGraph g
  const uint64_t *id;
  const int32_t *recv;
  const uint64_t *sup;
  const uint8_t *flags;       // 1 interned, 2 root, 4 busy (CRGC_DELTA_*)
  const uint32_t *out_off;    // [n_shadows + 1]
  const uint64_t *out_target;
  const int32_t *out_count;
} wl_deltas;

struct wl_delta_builder {
  std::vector<uint32_t> graph_off{0};
  std::vector<uint64_t> id, sup, out_target;
  std::vector<int32_t> recv, out_count;
  std::vector<uint8_t> flags;
  std::vector<uint32_t> out_off{0};
  Graph g;

  void emit() {
    for (size_t i = 0; i < g.shadows.size(); ++i) {
      const Shadow &s = g.shadows[i];
      id.push_back(g.decoder[i]);
      recv.push_back(s.recv);
      sup.push_back(s.sup >= 0 ? g.decoder[s.sup] : ~0ull);
      flags.push_back((s.interned ? 1 : 0) | (s.root ? 2 : 0) | (s.busy ? 4 : 0));
      for (auto &kv : s.out) {
        out_target.push_back(g.decoder[kv.first]);
        out_count.push_back(kv.second);
      }
      out_off.push_back((uint32_t)out_target.size());
    }
    graph_off.push_back((uint32_t)id.size());
    g.clear();
  }
};

wl_delta_builder *wl_deltas_create() { return new wl_delta_builder(); }
void wl_deltas_destroy(wl_delta_builder *b) { delete b; }

// Fold entries [0, e->n) into DeltaGraphs of `dgs` shadows (F-slot entries),
// emitting each full graph and the trailing one; results replace the last.
int wl_deltas_build(wl_delta_builder *b, const wl_entries *e, uint32_t F, uint32_t dgs, wl_deltas *out) {
  *b = wl_delta_builder();
  for (uint64_t i = 0; i < e->n; ++i) {
    Graph &g = b->g;
    const int32_t me = g.encode(e->self[i]);  // DeltaGraph.java:75-83
    {
      Shadow &s = g.shadows[me];
      s.interned = true;
      s.recv += e->recv[i];
      s.busy = e->flags[i] & 1;
      s.root = e->flags[i] & 2;
    }
    for (uint32_t k = e->c_off[i]; k < e->c_off[i + 1]; ++k) {  // :86-94
      const int32_t t = g.encode(e->c_target[k]);
      const int32_t o = g.encode(e->c_owner[k]);
      update(g.shadows[o].out, t, 1);
    }
    for (uint32_t k = e->s_off[i]; k < e->s_off[i + 1]; ++k)  // :97-103
      g.shadows[g.encode(e->spawned[k])].sup = me;
    for (uint32_t k = e->u_off[i]; k < e->u_off[i + 1]; ++k) {  // :106-123
      const int32_t t = g.encode(e->u_ref[k]);
      const int32_t cnt = refob_count(e->u_info[k]);
      if (cnt > 0) g.shadows[t].recv -= cnt;
      if (!refob_active(e->u_info[k])) update(g.shadows[me].out, t, -1);
    }
    if (g.shadows.size() + 4 * F + 1 >= dgs) b->emit();  // isFull, :174-180
  }
  if (!b->g.shadows.empty()) b->emit();
  out->n_graphs = b->graph_off.size() - 1;
  out->n_shadows = b->id.size();
  out->n_out = b->out_target.size();
  out->graph_off = b->graph_off.data();
  out->id = b->id.data();
  out->recv = b->recv.data();
  out->sup = b->sup.data();
  out->flags = b->flags.data();
  out->out_off = b->out_off.data();
  out->out_target = b->out_target.data();
  out->out_count = b->out_count.data();
  return 0;
}

}  // extern "C"
