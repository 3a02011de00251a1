/*
 * crgc.h — C ABI of the MI355X-native CRGC garbage-detection hot path.
 *
 * This is the drop-in boundary for the reference's `ShadowGraph`
 * (uigc-akka, src/main/java/edu/illinois/osl/uigc/engines/crgc/ShadowGraph.java).
 * `LocalGC` (src/main/scala/.../crgc/LocalGC.scala:58) constructs a ShadowGraph
 * and calls exactly the methods listed below; each entry point names the
 * reference method it replaces.  A JVM binds these through a ~100-line JNI shim
 * (see INTEGRATION.md); tests and the bench bind them through Python ctypes.
 *
 * Conventions
 *  - Every function returns 0 (CRGC_OK) or a negative CRGC_E_* code.  Nothing
 *    throws or aborts across the ABI.
 *  - One caller thread per handle (LocalGC is a single actor on a
 *    PinnedDispatcher: CRGC.scala:54-58, reference.conf:11-14).
 *  - Actor identity: the JVM interns each ActorRef to a uint64 id.  The top 16
 *    bits of the id are the actor's location (the interned akka Address,
 *    `ref.path().address()`, ShadowGraph.java:49); the low 48 bits are free.
 *    Ids CRGC_NO_ACTOR and CRGC_DEAD_ACTOR (and location 0xFFFF) are reserved.
 *  - Input buffers are caller-owned.  Host buffers are only read during the
 *    call (a merge waits for its staging copies; the reference recycles an
 *    Entry right after merging it: LocalGC.scala:167-169).  Device (HBM)
 *    buffers are read by kernels queued on the graph's stream and must stay
 *    valid until the next synchronising call (a trace or a query).  `memory`
 *    says whether the pointers are host or device pointers.
 *  - Merges are stream-ordered and asynchronous with respect to the host; a
 *    trace (and every query) synchronises.  Merges between two traces commute
 *    except for the last-write-wins fields, which follow call order and then
 *    record order inside a call — exactly the order the reference would have
 *    applied them in.
 */
#ifndef CRGC_H
#define CRGC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRGC_ABI_VERSION 5u  /* 2: crgc_trace_stats.expand_launches / expand_bytes; 3: exchange_bytes;
                                 4: time_query_failures, direct_lists; 5: crgc_config.proxy_capacity */

/* ---- status codes ------------------------------------------------------- */
#define CRGC_OK 0
#define CRGC_E_INVAL (-1)          /* bad argument, reserved id, > F records   */
#define CRGC_E_NOMEM (-2)          /* device or host allocation failed         */
#define CRGC_E_DEVICE (-3)         /* a HIP call failed                        */
#define CRGC_E2BIG (-4)            /* output buffer too small; sizes written   */
#define CRGC_E_NULL_SUPERVISOR (-5)/* reference NPE, ShadowGraph.java:277      */
#define CRGC_E_UNDO_NEW_SHADOW (-6)/* reference CME, ShadowGraph.java:162,170  */
#define CRGC_E_POISONED (-7)       /* handle unusable after a device fault     */
#define CRGC_E_TIMEOUT (-8)        /* a bounded device spin gave up            */

/* ---- reserved ids ------------------------------------------------------- */
#define CRGC_NO_ACTOR ((uint64_t)0xFFFFFFFFFFFFFFFFull)   /* Java null        */
/* A supervisor that points at a removed (collected) shadow incarnation.  Only
 * appears in crgc_export output; it is non-null for the NPE test. */
#define CRGC_DEAD_ACTOR ((uint64_t)0xFFFFFFFFFFFFFFFEull)
#define CRGC_LOCATION_OF(id) ((uint16_t)((uint64_t)(id) >> 48))

/* ---- where a batch lives ----------------------------------------------- */
#define CRGC_MEM_HOST 0u   /* pageable or pinned host memory (copied H2D)   */
#define CRGC_MEM_DEVICE 1u /* device pointers on the handle's GPU            */

/* ---- vertex flag bits, as exported ------------------------------------ */
#define CRGC_F_INTERNED 0x02u
#define CRGC_F_LOCAL 0x04u
#define CRGC_F_BUSY 0x08u
#define CRGC_F_ROOT 0x10u
#define CRGC_F_HALTED 0x20u
#define CRGC_F_PROXY 0x40u   /* internal (sharded graphs); never exported   */

/* Entry.isBusy / Entry.isRoot bits in crgc_entry_batch.flags */
#define CRGC_ENTRY_BUSY 0x01u
#define CRGC_ENTRY_ROOT 0x02u
/* DeltaShadow.interned / isRoot / isBusy bits in crgc_delta_batch.flags */
#define CRGC_DELTA_INTERNED 0x01u
#define CRGC_DELTA_ROOT 0x02u
#define CRGC_DELTA_BUSY 0x04u

typedef struct crgc_graph crgc_graph; /* opaque; owns the HBM shadow graph */

/*
 * Hash-partitioned graphs (more shadows than one GPU should hold, or more
 * throughput): G shards, shard r holding the shadows whose actor id hashes to
 * r (crgc_shard_of).  Each shard is one crgc_graph on its own GPU; the shards
 * exchange marked frontier ids, kill requests and garbage ids through a
 * transport.  With G > 1 every entry point that changes or traces the graph is
 * COLLECTIVE: all G shards call it, in the same order (one thread or process
 * per shard).  Queries (live count, export, local roots, total actors seen)
 * are per shard; their union / sum is the whole graph's.
 */
typedef struct crgc_transport crgc_transport;
/* One process per GPU: RCCL over xGMI.  Shard 0 makes the id and shares it
 * out of band (e.g. torch.distributed); every shard then creates its
 * transport (collective, like ncclCommInitRank). */
int crgc_transport_rccl_id(uint8_t id[128]);
int crgc_transport_rccl(const uint8_t id[128], uint32_t n_shards, uint32_t shard, int32_t device,
                        crgc_transport **out);
/* One process, G shards (possibly on one GPU), one host thread per shard:
 * device-to-device copies.  Shared by the G handles. */
int crgc_transport_local(uint32_t n_shards, crgc_transport **out);
/* One process per shard, the bytes moved by the caller's own collectives over
 * host memory (e.g. torch.distributed gloo, MPI, the JVM's cluster messaging):
 * the transport stages each exchange in pinned host buffers and calls back on
 * the calling thread.  Every callback returns 0 on success; any other value
 * fails the exchange (CRGC_E_DEVICE, the handle poisoned).  For shards that
 * cannot share a GPU communicator (two ranks on one GPU) and for parity tests
 * of the multi-process protocol; RCCL is the transport for speed. */
typedef struct crgc_host_collectives {
  void *ctx;
  /* recv[r*bytes .. (r+1)*bytes) = shard r's send[0 .. bytes) */
  int (*allgather)(void *ctx, uint32_t shard, const void *send, void *recv, size_t bytes);
  /* send[soff[r] .. +sbytes[r]) goes to shard r; recv[roff[r] .. +rbytes[r])
   * gets shard r's block for this shard (rbytes[r] = r's sbytes[shard]) */
  int (*alltoallv)(void *ctx, uint32_t shard, const void *send, const size_t *soff, const size_t *sbytes,
                   void *recv, const size_t *roff, const size_t *rbytes);
} crgc_host_collectives;
int crgc_transport_host(const crgc_host_collectives *c, uint32_t n_shards, uint32_t shard, int32_t device,
                        crgc_transport **out);
/* Destroy after every handle using it. */
void crgc_transport_destroy(crgc_transport *t);
/* Home shard of an actor id. */
uint32_t crgc_shard_of(uint64_t id, uint32_t n_shards);

typedef struct crgc_config {
  uint32_t abi_version;        /* CRGC_ABI_VERSION                          */
  int32_t device;              /* HIP device ordinal                        */
  uint32_t entry_field_size;   /* F, uigc.crgc.entry-field-size (default 4)  */
  uint32_t delta_graph_size;   /* uigc.crgc.delta-graph-size (default 64)   */
  uint64_t vertex_capacity;    /* hint: expected live shadows (this shard)  */
  uint64_t edge_capacity;      /* hint: expected live (owner,target) pairs  */
  void *stream;                /* hipStream_t to run on; NULL = own stream  */
  uint32_t n_shards;           /* 0 or 1: unsharded                         */
  uint32_t shard;              /* this handle's shard, < n_shards           */
  crgc_transport *transport;   /* required when n_shards > 1                */
  uint64_t proxy_capacity;     /* n_shards > 1, hint: expected proxy slots   */
                               /* (far ends homed elsewhere); 0: like        */
                               /* vertex_capacity                            */
} crgc_config;

/*
 * A batch of Entry records in queue order (Entry.java:5-37, filled by
 * State.flushToEntry, State.java:90-124).  Record order is the order in which
 * LocalGC would have polled them (LocalGC.scala:152-172).
 * Per entry i the created/spawned/updated records are the half-open ranges
 * [x_off[i], x_off[i+1]) of the flat arrays — the reference's null-terminated
 * prefixes of F-slot arrays (ShadowGraph.java:86,97,108).
 */
typedef struct crgc_entry_batch {
  uint64_t n_entries;
  const uint64_t *self;           /* [n]   Entry.self                       */
  const int16_t *recv_count;      /* [n]   Entry.recvCount                  */
  const uint8_t *flags;           /* [n]   CRGC_ENTRY_BUSY | CRGC_ENTRY_ROOT */
  const uint32_t *created_off;    /* [n+1]                                  */
  const uint64_t *created_owner;  /* Entry.createdOwners                    */
  const uint64_t *created_target; /* Entry.createdTargets                   */
  const uint32_t *spawned_off;    /* [n+1]                                  */
  const uint64_t *spawned;        /* Entry.spawnedActors                    */
  const uint32_t *updated_off;    /* [n+1]                                  */
  const uint64_t *updated_ref;    /* Entry.updatedRefs                      */
  const int16_t *updated_info;    /* Entry.updatedInfos (RefobInfo word)    */
  uint32_t memory;                /* CRGC_MEM_HOST / CRGC_MEM_DEVICE        */
} crgc_entry_batch;

/*
 * A batch of DeltaGraph shadows, concatenated in arrival order and, inside one
 * DeltaGraph, in compressed-id order (ShadowGraph.java:131).  The host decodes
 * the compressed ids through DeltaGraph.decoder() (DeltaGraph.java:162-169).
 */
typedef struct crgc_delta_batch {
  uint64_t n_shadows;
  const uint64_t *id;          /* [n] decoder[i]                            */
  const int32_t *recv_count;   /* [n] DeltaShadow.recvCount                 */
  const uint64_t *supervisor;  /* [n] decoder[supervisor] or CRGC_NO_ACTOR  */
  const uint8_t *flags;        /* [n] CRGC_DELTA_*                          */
  const uint32_t *out_off;     /* [n+1] DeltaShadow.outgoing ranges         */
  const uint64_t *out_target;  /* decoder[key]                              */
  const int32_t *out_count;    /* value                                     */
  uint32_t memory;
} crgc_delta_batch;

/* An UndoLog (UndoLog.java:16-37) built on the host from delta graphs and
 * ingress entries (UndoLog.java:39-93). */
typedef struct crgc_undo_log {
  uint16_t node_location;        /* UndoLog.nodeAddress                     */
  uint16_t _pad[3];
  uint64_t n_fields;
  const uint64_t *actor;         /* [n] key of UndoLog.admitted             */
  const int32_t *message_count;  /* [n] Field.messageCount                  */
  const uint32_t *created_off;   /* [n+1] Field.createdRefs ranges          */
  const uint64_t *created_target;
  const int32_t *created_count;
  uint32_t memory;
} crgc_undo_log;

typedef struct crgc_trace_stats {
  uint64_t pseudo_roots;   /* shadows passing isPseudoRoot (:201-203)       */
  uint64_t edges_scanned;  /* nonzero out-edges of marked non-halted shadows */
  uint64_t sup_edges;      /* supervisor edges followed (:258-267)          */
  uint64_t levels;         /* non-empty BFS levels                          */
  uint64_t launches;       /* level-kernel launches (incl. trailing empty)  */
  double ms_mark;          /* device time of the pseudo-root + level kernels*/
  double ms_sweep;         /* device time: sweep + id compaction            */
  double ms_total;         /* host wall time of crgc_trace                  */
  /* per level kernel (device time summed over the trace's launches) */
  double ms_frontier;      /* k_frontier: pseudo-roots / frontier, sup edges */
  double ms_tail;          /* k_tail: level controller, narrow frontiers    */
  double ms_expand;        /* k_expand: out-edges of the frontier           */
  /* sharded graphs */
  uint64_t rounds;         /* exchange rounds (1 + frontier all-to-alls)    */
  uint64_t ids_sent;       /* marked proxies sent to other shards (any form)*/
  double ms_exchange;      /* host wall time spent in exchanges             */
  /* the k_expand roofline */
  uint64_t expand_launches;/* level expands of this trace that were timed: by
                              default (CRGC_KERNEL_TIMING=3) the wide levels
                              0 and 1; ms_expand and expand_bytes cover
                              exactly these launches                         */
  uint64_t expand_bytes;   /* bytes they read + wrote, by element width      */
  /* sharded graphs: bytes this shard sent in mark rounds (ids, home slots,
     frontier bitmaps) and in the home-slot resolution before them */
  uint64_t exchange_bytes;
  /* device-time queries (event pairs) the runtime could not answer; their ms
     count as 0, so a nonzero value means the ms_* fields above are short */
  uint64_t time_query_failures;
  /* 1: the garbage / kill ids were stored by the device straight into the
     caller's page-locked buffers (no copy-back round trip) */
  uint64_t direct_lists;
} crgc_trace_stats;

typedef struct crgc_trace_out {
  uint64_t *garbage_ids;   /* caller buffer or NULL (count only)            */
  uint64_t garbage_cap;
  uint64_t n_garbage;      /* TracingEvent.numGarbageActors (:275)          */
  uint64_t *kill_ids;      /* actors told StopMsg (:277-278)                */
  uint64_t kill_cap;
  uint64_t n_kill;
  uint64_t n_live;         /* TracingEvent.numLiveActors (:282)             */
  crgc_trace_stats stats;
} crgc_trace_out;

/*
 * DeltaGraphs of one wakeup's entries, built on the device:
 * what LocalGC does per entry when num-nodes > 1 (LocalGC.scala:159-177) —
 * fold the entries, in queue order, into DeltaGraph.mergeEntry
 * (DeltaGraph.java:73-125), finalize the graph whenever isFull() holds after
 * an entry (:174-180) and finalize the last non-empty one at the end.
 *
 * Outputs, per graph g, shadows in compressed-id order:
 *   - the decoded shadows as one crgc_delta_batch (graphs back to back,
 *     outgoing entries in Java iteration order), ready for crgc_merge_deltas
 *     on a remote node's graph;
 *   - the DataOutput bytes DeltaGraph.serialize writes between the address
 *     object and the compression table (DeltaGraph.java:196-200): big-endian
 *     writeShort(size), then DeltaShadow.serialize of every shadow
 *     (DeltaShadow.java:57-69) with the outgoing map in java.util.HashMap
 *     iteration order.  The JVM writes the address, these bytes
 *     (ObjectOutputStream.write: the same block-data stream as the field
 *     writes), then the compression table from decoder ids.
 * All arrays are caller buffers in `memory`; graph_off / wire_off /
 * out_off hold one more element than their counts.  Pass NULL arrays to learn
 * the sizes; CRGC_E2BIG when a capacity is short (the counts hold the sizes).
 * Requires delta_graph_size <= 64 and delta_graph_size > 4*F + 1.
 */
typedef struct crgc_delta_graphs {
  uint32_t memory;         /* CRGC_MEM_HOST / CRGC_MEM_DEVICE                  */
  uint32_t _pad;
  uint64_t graph_cap, n_graphs;
  uint32_t *graph_off;     /* [n_graphs+1] first shadow of each graph          */
  uint64_t *wire_off;      /* [n_graphs+1] first wire byte of each graph       */
  uint64_t shadow_cap, n_shadows;
  uint64_t *id;            /* [n_shadows] decoder[cid]                         */
  int32_t *recv_count;
  uint64_t *supervisor;    /* decoder[supervisor] or CRGC_NO_ACTOR             */
  uint8_t *flags;          /* CRGC_DELTA_*                                     */
  uint32_t *out_off;       /* [n_shadows+1]                                    */
  uint64_t out_cap, n_out;
  uint64_t *out_target;
  int32_t *out_count;
  uint64_t wire_cap, wire_bytes;
  uint8_t *wire;
} crgc_delta_graphs;

int crgc_build_delta_graphs(crgc_graph *g, const crgc_entry_batch *batch, crgc_delta_graphs *out);
/* With CRGC_MEM_DEVICE outputs the arrays are written by kernels queued on the
   graph's stream when crgc_build_delta_graphs returns (sizes are final): work
   queued after it on that stream sees them; crgc_sync waits for them. */
int crgc_sync(crgc_graph *g);

/*
 * UndoLog folding on the device.  A collector folds every
 * DeltaGraph it receives into the sender's UndoLog (LocalGC.scala:133,
 * UndoLog.mergeDeltaGraph, UndoLog.java:39-67) and every IngressEntry into
 * the log of its egress node (UndoLog.mergeIngressEntry, :69-93); when a node
 * leaves, its log is merged (ShadowGraph.mergeUndoLog, :158-174).  A
 * crgc_undo_acc is one such log, kept in HBM on its graph's device and
 * stream; destroy it before the graph.
 */
typedef struct crgc_undo_acc crgc_undo_acc;

typedef struct crgc_undo_log_out {
  uint64_t field_cap, n_fields;
  uint64_t *actor;             /* [n_fields] UndoLog.admitted keys             */
  int32_t *message_count;      /* [n_fields] Field.messageCount                */
  uint32_t *created_off;       /* [n_fields+1]                                 */
  uint64_t created_cap, n_created;
  uint64_t *created_target;    /* Field.createdRefs with nonzero counts        */
  int32_t *created_count;
} crgc_undo_log_out;

int crgc_undo_acc_create(crgc_graph *g, uint16_t node_location, crgc_undo_acc **out);
void crgc_undo_acc_destroy(crgc_undo_acc *u);
/* UndoLog.mergeDeltaGraph for every DeltaGraph of the batch (graphs back to
 * back, as crgc_merge_deltas takes them). */
int crgc_undo_acc_fold_deltas(crgc_undo_acc *u, const crgc_delta_batch *deltas);
/* UndoLog.mergeIngressEntry for the admitted fields of IngressEntries
 * (IngressEntry.admitted flattened like an UndoLog; node_location unused). */
int crgc_undo_acc_fold_ingress(crgc_undo_acc *u, const crgc_undo_log *fields);
/* The accumulated log, host arrays; two-phase: NULL arrays give the sizes,
 * CRGC_E2BIG when a capacity is short.  Field order unspecified. */
int crgc_undo_acc_export(crgc_undo_acc *u, crgc_undo_log_out *out);
/* ShadowGraph.mergeUndoLog with the accumulated log (crgc_merge_undo's rules). */
int crgc_merge_undo_acc(crgc_graph *g, crgc_undo_acc *u);

/* Full graph state, for parity tests and debugging (the reference's
 * ShadowGraph.assertEquals / Shadow.assertEquals, ShadowGraph.java:176-199).
 * Two-phase: call with NULL arrays to learn n_vertices / n_edges. */
typedef struct crgc_graph_export {
  uint64_t vertex_cap, n_vertices;
  uint64_t *id;
  int32_t *recv_count;
  uint8_t *flags;          /* CRGC_F_* bits                                 */
  uint64_t *supervisor;    /* id, CRGC_NO_ACTOR or CRGC_DEAD_ACTOR          */
  uint64_t edge_cap, n_edges; /* nonzero counts to live incarnations only   */
  uint64_t *edge_owner;
  uint64_t *edge_target;
  int32_t *edge_count;
} crgc_graph_export;

/* ShadowGraph(Context) — ShadowGraph.java:17-21 */
int crgc_create(const crgc_config *cfg, crgc_graph **out);
void crgc_destroy(crgc_graph *g);

/* N x ShadowGraph.mergeEntry(Entry) — ShadowGraph.java:75-125,
 * called from LocalGC Wakeup (LocalGC.scala:152-172). */
int crgc_merge_entries(crgc_graph *g, const crgc_entry_batch *batch);

/* The same merge for a drain loop that hands a wakeup's entries over in
 * chunks as it packs them (LocalGC.scala:152-172): a host batch wholly inside
 * memory registered with crgc_host_register is only enqueued — its PCIe read
 * and merge run while the caller packs the next chunk — and must stay
 * unchanged until the next crgc_trace or crgc_sync returns.  Any other batch
 * is merged exactly as by crgc_merge_entries.  Chunks merge in call order,
 * each its own merge (last write wins across chunks in that order). */
int crgc_merge_entries_async(crgc_graph *g, const crgc_entry_batch *batch);

/* N x ShadowGraph.mergeDelta(DeltaGraph) — ShadowGraph.java:127-156,
 * called on DeltaMsg (LocalGC.scala:124-136). */
int crgc_merge_deltas(crgc_graph *g, const crgc_delta_batch *batch);

/* ShadowGraph.mergeUndoLog(UndoLog) — ShadowGraph.java:158-174,
 * called when an undo log is ready (LocalGC.scala:254-263).
 * Returns CRGC_E_UNDO_NEW_SHADOW, without mutating the graph, where the
 * reference would throw ConcurrentModificationException. */
int crgc_merge_undo(crgc_graph *g, const crgc_undo_log *log);

/* ShadowGraph.trace(shouldKill) — ShadowGraph.java:205-289.
 * Writes garbage and kill ids (sets; order unspecified) and the counts.
 * Returns CRGC_E_NULL_SUPERVISOR, without mutating the graph, where the
 * reference would throw NullPointerException (:277).  On CRGC_E2BIG the trace
 * HAS happened; n_garbage / n_kill hold the sizes and crgc_last_trace copies
 * the retained lists into larger buffers. */
int crgc_trace(crgc_graph *g, int should_kill, crgc_trace_out *out);
int crgc_last_trace(crgc_graph *g, crgc_trace_out *out);

/* ShadowGraph.startWave() — ShadowGraph.java:291-299: ids to tell WaveMsg. */
int crgc_local_roots(crgc_graph *g, uint64_t *out, uint64_t cap, uint64_t *n);

/* ShadowGraph.investigateRemotelyHeldActors(Address) — ShadowGraph.java:302-330,
 * called from LocalGC.scala:234,276. */
int crgc_count_reachable_from(crgc_graph *g, uint16_t location, int64_t *out);

/* ShadowGraph.totalActorsSeen — ShadowGraph.java:12,46; LocalGC.scala:273. */
int crgc_total_actors_seen(crgc_graph *g, uint64_t *out);

/* Number of shadows in the graph (|from| == |shadowMap|). */
int crgc_live_count(crgc_graph *g, uint64_t *out);

/* Compact the graph now (no reference counterpart: the JVM's own GC does
   this for ShadowGraph's objects): live shadows renumbered densely, zero-count
   edges and edges to collected shadows dropped, edge and candidate segments
   repacked in slot order.  A trace does it by itself once dead slots
   outnumber live ones, and a merge when a capacity would be exceeded;
   results are unchanged either way. */
int crgc_compact(crgc_graph *g);

int crgc_export(crgc_graph *g, crgc_graph_export *out);

/* Pins a caller-owned host buffer for DMA, as a JVM would its direct
   ByteBuffers (packed by the Wakeup drain loop, LocalGC.scala:152-172, and
   reused every wakeup): host batches whose arrays lie in registered buffers
   are copied by the DMA engines, without the driver's pageable staging copy.
   No reference counterpart (the reference has no device boundary).  The
   buffer must stay valid until crgc_host_unregister or crgc_destroy;
   registering an overlapping range is CRGC_E_INVAL.  crgc_host_unregister
   is safe with crgc_merge_entries_async merges in flight: it waits for the
   copies and merges queued on the handle before unpinning the range. */
int crgc_host_register(crgc_graph *g, void *ptr, uint64_t bytes);

/* Slot and table usage (a diagnostic; no reference counterpart): the dense
   per-slot passes of a trace (pseudo-roots, frontier scans, sweep) scale with
   slot_top — live shadows plus the slots of collected ones not yet reused or
   compacted away — not with the live count.  Counters as of a host
   synchronisation this call makes. */
typedef struct crgc_usage {
  uint64_t slot_top, slot_cap;    /* home slots in use (dead ones included), capacity */
  uint64_t proxy_top, proxy_cap;  /* proxy region (sharded graphs)                    */
  uint64_t free_slots;            /* swept slots waiting for reuse by new shadows     */
  uint64_t pool_top, pool_cap;    /* edge pool entries                                */
  uint64_t etab_used, etab_cap;   /* edge-table keys                                  */
  uint64_t rebuilds, grows, repacks;
} crgc_usage;
int crgc_usage_of(crgc_graph *g, crgc_usage *out);
int crgc_host_unregister(crgc_graph *g, void *ptr);

/* Human-readable text for a status code. */
const char *crgc_strerror(int code);

/* Where the calling thread's last failed call went wrong ("file:line: what",
   e.g. the HIP status a runtime call returned, or the device error flags);
   empty when its last call through a graph handle succeeded.  Diagnostics
   only: the status code is the contract. */
const char *crgc_last_error_detail(void);

#ifdef __cplusplus
} /* extern "C" */
#endif
#endif /* CRGC_H */
