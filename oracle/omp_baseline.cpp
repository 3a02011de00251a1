// omp_baseline.cpp — BENCH INFRASTRUCTURE ONLY: the strong CPU baseline of
// SURVEY §8d / BASELINE.md §2 ("cpu_omp"): ShadowGraph.trace's mark and
// sweep (ShadowGraph.java:201-289) as an OpenMP level-synchronous BFS over a
// CSR snapshot of a graph exported by the oracle, on the host cores given.
// It times the trace only (the snapshot is built untimed); bench.py reports
// it beside the single-threaded oracle.  Not a checker and not the product.
#include <omp.h>

#include <chrono>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "../include/crgc.h"

extern "C" {

// Vertices (ids, recv, CRGC_F_* flags, supervisor ids) and nonzero edges as
// oracle_export writes them.  Returns 0, or -1 on a malformed snapshot.
int omp_trace_bench(uint64_t nv, const uint64_t *ids, const int32_t *recv, const uint8_t *flags,
                    const uint64_t *sup_id, uint64_t ne, const uint64_t *eo, const uint64_t *et,
                    const int32_t *ec, int threads, int reps, double *best_s, uint64_t *edges_scanned,
                    uint64_t *n_marked, uint64_t *n_garbage, uint64_t *n_kill) {
  std::unordered_map<uint64_t, uint32_t> slot;
  slot.reserve(nv * 2);
  for (uint64_t i = 0; i < nv; ++i) slot.emplace(ids[i], (uint32_t)i);
  std::vector<uint32_t> sup(nv, ~0u);
  for (uint64_t i = 0; i < nv; ++i) {
    auto it = slot.find(sup_id[i]);
    if (it != slot.end()) sup[i] = it->second;
  }
  std::vector<uint64_t> row(nv + 1, 0);
  std::vector<uint32_t> src(ne), col(ne);
  for (uint64_t k = 0; k < ne; ++k) {
    auto a = slot.find(eo[k]), b = slot.find(et[k]);
    if (a == slot.end() || b == slot.end()) return -1;
    src[k] = a->second;
    col[k] = b->second;
    row[a->second + 1]++;
  }
  for (uint64_t i = 0; i < nv; ++i) row[i + 1] += row[i];
  std::vector<uint32_t> csr(ne);
  std::vector<int32_t> cnt(ne);
  {
    std::vector<uint64_t> pos(row.begin(), row.end() - 1);
    for (uint64_t k = 0; k < ne; ++k) {
      const uint64_t p = pos[src[k]]++;
      csr[p] = col[k];
      cnt[p] = ec[k];
    }
  }
  if (threads > 0) omp_set_num_threads(threads);
  std::vector<uint8_t> vis(nv);
  double best = 1e30;
  uint64_t scanned = 0, marked = 0, garbage = 0, kill = 0;
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint32_t> front;
    uint64_t sc = 0, mk = 0;
#pragma omp parallel
    {
      std::vector<uint32_t> mine;
#pragma omp for schedule(static)
      for (uint64_t v = 0; v < nv; ++v) {  // isPseudoRoot (:201-203)
        const uint8_t f = flags[v];
        const bool root = !(f & CRGC_F_HALTED) &&
                          ((f & (CRGC_F_ROOT | CRGC_F_BUSY)) || !(f & CRGC_F_INTERNED) || recv[v] != 0);
        vis[v] = root;
        if (root) mine.push_back((uint32_t)v);
      }
#pragma omp critical
      front.insert(front.end(), mine.begin(), mine.end());
    }
    mk = front.size();
    while (!front.empty()) {  // (:210-268)
      std::vector<uint32_t> next;
      uint64_t lsc = 0;
#pragma omp parallel reduction(+ : lsc)
      {
        std::vector<uint32_t> mine;
        auto visit = [&](uint32_t t) {
          if (!vis[t] && !__atomic_exchange_n(&vis[t], (uint8_t)1, __ATOMIC_RELAXED)) mine.push_back(t);
        };
#pragma omp for schedule(dynamic, 64)
        for (uint64_t i = 0; i < front.size(); ++i) {
          const uint32_t v = front[i];
          if (flags[v] & CRGC_F_HALTED) continue;  // marked, not expanded (:226-229)
          lsc += row[v + 1] - row[v];
          for (uint64_t k = row[v]; k < row[v + 1]; ++k)
            if (cnt[k] > 0) visit(csr[k]);
          if (sup[v] != ~0u) {
            ++lsc;
            visit(sup[v]);
          }
        }
#pragma omp critical
        next.insert(next.end(), mine.begin(), mine.end());
      }
      sc += lsc;
      mk += next.size();
      front.swap(next);
    }
    uint64_t g = 0, k = 0;
#pragma omp parallel for reduction(+ : g, k) schedule(static)
    for (uint64_t v = 0; v < nv; ++v) {  // sweep (:270-289)
      if (vis[v]) continue;
      ++g;
      const uint8_t f = flags[v];
      if ((f & CRGC_F_LOCAL) && !(f & CRGC_F_HALTED) && sup[v] != ~0u && vis[sup[v]]) ++k;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (s < best) best = s;
    scanned = sc;
    marked = mk;
    garbage = g;
    kill = k;
  }
  *best_s = best;
  *edges_scanned = scanned;
  *n_marked = marked;
  *n_garbage = garbage;
  *n_kill = kill;
  return 0;
}

}  // extern "C"
