/*
 * crgc_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's ShadowGraph (uigc-akka
 * src/main/java/edu/illinois/osl/uigc/engines/crgc/ShadowGraph.java), used as
 * the parity checker for the HIP path and as the bench's cpu_baseline ("port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  It is never linked into, or called by, the product library.
 *
 * It takes the same batch structs as include/crgc.h (host memory only) and
 * mirrors its entry points one for one.
 */
#ifndef CRGC_ORACLE_H
#define CRGC_ORACLE_H

#include "../include/crgc.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_graph oracle_graph;

oracle_graph *oracle_create(uint32_t entry_field_size, uint32_t delta_graph_size);
void oracle_destroy(oracle_graph *g);
int oracle_merge_entries(oracle_graph *g, const crgc_entry_batch *b);
int oracle_merge_deltas(oracle_graph *g, const crgc_delta_batch *b);
int oracle_merge_undo(oracle_graph *g, const crgc_undo_log *log);
int oracle_trace(oracle_graph *g, int should_kill, crgc_trace_out *out);
int oracle_local_roots(oracle_graph *g, uint64_t *out, uint64_t cap, uint64_t *n);
int oracle_count_reachable_from(oracle_graph *g, uint16_t location, int64_t *out);
int oracle_total_actors_seen(oracle_graph *g, uint64_t *out);
int oracle_live_count(oracle_graph *g, uint64_t *out);
int oracle_export(oracle_graph *g, crgc_graph_export *out);

#ifdef __cplusplus
}
#endif
#endif
