/* lakeside_gpu.h — C ABI of the MI355X sealed-segment DataExpr evaluator.
 *
 * Drop-in for the worker's per-segment evaluator seam:
 *   Commons.evaluatePushDownRequest(queryId, localParquet, pushDownRequest)
 *     core/src/main/scala/com/cardinal/utils/Commons.scala:343-397
 *   whose native seam is Commons.toGlobResultSet + resultSetToSource (Commons.scala:200-254, 280-341),
 *   i.e. DuckDB's read_parquet + filter + hash GROUP BY + ORDER BY behind JDBC/JNI.
 * The Scala side binds these symbols through JNA exactly as the reference already binds lib-trigram.so
 * (core/src/main/scala/com/cardinal/utils/ast/queries/NLPUtils.scala:43-52); see INTEGRATION.md.
 *
 * Conventions: 0 = success, negative = error (message in lk_last_error(), thread-local).  Never throws or
 * aborts across the ABI.  Inputs are borrowed for the duration of the call.  Results are owned by the
 * library until lk_result_free.  Calls on one engine are thread-safe and re-entrant: each evaluation leases its
 * own context (HIP stream, workspaces; up to "max_calls" in flight), so calls from several threads run
 * concurrently, as the worker's glob queries do (Commons.scala:371-372); only distributed calls
 * (lk_eval_pushdown_dist) are serialised, to keep every rank's collectives in one order, and a dictionary
 * compaction (see lk_engine_create) runs between loads / evaluations, never under one.
 *
 * Errors: a failure that belongs to one glob's DuckDB query in the reference -- a missing or unreadable segment,
 * corrupt Parquet, a column type the query cannot bind, a regex RE2 rejects -- empties that glob only
 * (Commons.toGlobResultSet, Commons.scala:249-253); the call still succeeds ("failed_globs" in lk_result_stats).
 */
#ifndef LAKESIDE_GPU_H
#define LAKESIDE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lk_engine lk_engine;   /* one per process per GPU: device, streams, HBM segment cache, RCCL comm */
typedef struct lk_result lk_result;   /* rows of one evaluation */

enum {
  LK_OK = 0,
  LK_ERR_ARG = -1,          /* bad argument / malformed JSON */
  LK_ERR_UNSUPPORTED = -2,  /* query or file shape outside the implemented path */
  LK_ERR_IO = -3,           /* file read / Parquet parse */
  LK_ERR_DEVICE = -4,       /* HIP / RCCL failure, or no GPU */
  LK_ERR_MEMORY = -5,
  LK_ERR_EVICTED = -6       /* a key registered with lk_segment_put was evicted from the HBM cache: re-put it */
};

/* Flags of lk_eval_pushdown. */
#define LK_PER_GLOB_ROWS 1u   /* rows of every glob separately (the worker's output, S17) */
#define LK_MERGED 2u          /* cells merged across globs as query-api does (TimeGroupedSketchAggregator, S19) */
#define LK_PLAN_BYTES 4u      /* optional, with either: the scan kernel counts the bytes its plan reads
                                 (lk_result_stats "plan_bytes"; measurement only, costs ~5% of scan time) */

/* options_json: {"device": 0, "hbm_budget_bytes": N, "max_calls": 4, "dict_compact_min_dead": 1024,
 *                "load_threads": 0}; NULL = defaults.
 * hbm_budget_bytes: weight bound of the HBM segment cache (the worker's Caffeine cache weight,
 * query-worker/.../WorkerApi.scala:53-64): inserting past it evicts least-recently-used segments; 0 (default) = no
 * bound, eviction only when HBM runs out.  max_calls: evaluations in flight (one stream each).
 * dict_compact_min_dead: engine dictionaries (one per column, value -> id) count the cached segments' references to
 * every id; once evictions leave at least max(live ids, this) ids unreferenced, the next load or evaluation renumbers
 * the live ids densely first, so group-dim spaces track the cached segments (results keep their strings).
 * load_threads: host threads of a segment load (page walk, decompression, staging copies); 0 (default) = the
 * process's OMP_NUM_THREADS share of the host's cores, at most 16.
 * Replaces DuckDbConnectionFactory (core/.../utils/DuckDbConnectionFactory.scala:76-114). */
int lk_engine_create(const char* options_json, lk_engine** out);
void lk_engine_destroy(lk_engine* e);

/* HBM segment cache (replaces the worker's Caffeine disk cache, worker/WorkerApi.scala:53-77).
 * lk_segment_put: register Parquet bytes under `key` (e.g. the path Commons.toParquetFilePath builds,
 * Commons.scala:256-278) and upload them; lk_segment_load: read a local Parquet file into the cache.
 * Re-putting an existing key replaces it. */
int lk_segment_put(lk_engine* e, const char* key, const uint8_t* data, size_t size);
int lk_segment_load(lk_engine* e, const char* path);
int lk_segment_evict(lk_engine* e, const char* key);
size_t lk_segment_count(const lk_engine* e);
/* HBM bytes held by the cache. */
size_t lk_segment_bytes(const lk_engine* e);
/* Engine counters as JSON: {"segments", "segment_bytes", "evictions", "dict_compactions",
 * "dictionaries": {column: {"size", "live", "generation"}}}; valid until the calling thread's next call. */
const char* lk_engine_stats(lk_engine* e);
/* Drops the engine's per-query caches -- parsed requests, per-(column, leaf) dictionary outcomes, value-key orders,
 * bulk-export pointer tables and distributed group-dim unions -- but keeps the cached segments and dictionaries: the
 * next evaluation of any request runs cold (the bench's cold_eval_ms).  Waits for in-flight evaluations. */
int lk_engine_drop_caches(lk_engine* e);

/* Mirrors one Commons.evaluatePushDownRequest call (Commons.scala:343-397).
 * push_down_json: PushDownRequest.toJson wire format (core/.../model/SegmentRequest.scala:30-60).
 * paths[i]: cache key (or local file, loaded on a miss) of segmentRequests[i].
 * glob_size: 10 for local Parquet, 5 for remote (Commons.scala:361); 0 = 10.
 * flags: LK_PER_GLOB_ROWS or LK_MERGED. */
int lk_eval_pushdown(lk_engine* e, const char* push_down_json, const char* const* paths, size_t n_paths,
                     int glob_size, unsigned flags, lk_result** out);

size_t lk_result_num_rows(const lk_result* r);
const int64_t* lk_result_timestamps(const lk_result* r);   /* ascending (ties: glob, then group order) */
const double* lk_result_values(const lk_result* r);
const uint32_t* lk_result_globs(const lk_result* r);       /* glob index per row (0 when merged) */
size_t lk_result_num_tag_columns(const lk_result* r);
const char* lk_result_tag_name(const lk_result* r, size_t col);             /* "name", groupBys, queryTags keys */
const char* lk_result_tag_value(const lk_result* r, size_t row, size_t col); /* NULL => tag absent (S15) */
/* Percentile aggregations (`p<NN>`, logs/traces): the row's serialized DDSketch (sketches-java DDSketch.serialize
 * wire format, the `Left(bytes)` of SketchTags, PushDownAggregatorStage.scala:163-167; relative accuracy 0.01); the
 * row's value is getValueAtQuantile(NN / 100) of that sketch (BaseExpr.scala:59-61).  *len = 0 / NULL for other
 * aggregations.  Valid until lk_result_free. */
const uint8_t* lk_result_sketch(const lk_result* r, size_t row, size_t* len);
/* Bulk tag export (replaces one lk_result_tag_value call per row and column; the reference materializes tags per
 * row in Commons.toDataPoint, Commons.scala:399-462).  The name / groupBy tag columns are the first
 * lk_result_num_group_columns columns.  Row r's value in such a column `col` is
 *     dict[(lk_result_group_ids(r)[row] / stride) % ndim]       (NULL: the tag is absent, S15)
 * with dict = lk_result_tag_dictionary(r, col, &stride, &ndim).  NULL dictionary (ndim 0): the column yields no
 * tag (a hidden tag).  A row whose group tags are all absent takes its glob's queryTags (Commons.scala:450-452):
 * lk_result_tag_value on the columns after the group columns.  Arrays are valid until lk_result_free; an
 * engine-dictionary column's table is shared with the engine and costs O(1) once built. */
const uint32_t* lk_result_group_ids(const lk_result* r);
size_t lk_result_num_group_columns(const lk_result* r);
const char* const* lk_result_tag_dictionary(const lk_result* r, size_t col, uint64_t* stride, uint64_t* ndim);
/* JSON: {"scan_ms":..,"total_ms":..,"rows_scanned":..,"algorithmic_bytes":..,"tiles":..,"cells":..,
 *        "failed_globs":..,"general_segments":..} */
const char* lk_result_stats(const lk_result* r);
void lk_result_free(lk_result* r);

const char* lk_last_error(void);

/* ---- multi-GPU (one process per GPU; segments sharded across ranks, partial tables merged over RCCL) ----
 * Replaces the pod fan-out + query-api merge: SegmentSequencer.allSources (query-api/.../engine/
 * SegmentSequencer.scala:53-160), QueryEngineV2.mergeSortedSource (QueryEngineV2.scala:76-97) and
 * TimeGroupedSketchAggregator (core/.../eval/TimeGroupedSketchAggregator.scala:57-177). */
#define LK_UNIQUE_ID_BYTES 128
/* Fill `id` (LK_UNIQUE_ID_BYTES) on rank 0; broadcast it out of band (e.g. torch.distributed). */
int lk_comm_unique_id(uint8_t* id);
int lk_comm_init(lk_engine* e, const uint8_t* id, int world, int rank);
/* Host transport instead of RCCL (e.g. torch.distributed/gloo or MPI supplied by the caller; also lets several
 * ranks share one GPU, which RCCL refuses).  fn(user, send, bytes, recv) must all-gather `bytes` from every rank
 * into recv (world * bytes, rank order) and return 0; it is called from inside lk_eval_pushdown_dist, on the
 * calling thread, the same number of times with the same sizes on every rank. */
typedef int (*lk_allgather_fn)(void* user, const void* send, size_t bytes, void* recv);
int lk_comm_init_host(lk_engine* e, int world, int rank, lk_allgather_fn fn, void* user);
/* Like lk_eval_pushdown with LK_MERGED, but this rank evaluates only the segments whose index i has
 * shard[i] == rank; partial tables are reduced to rank 0 over RCCL, which alone receives rows
 * (other ranks get an empty result). shard == NULL: i % world. */
int lk_eval_pushdown_dist(lk_engine* e, const char* push_down_json, const char* const* paths, size_t n_paths,
                          const int32_t* shard, int glob_size, lk_result** out);

#ifdef __cplusplus
}
#endif
#endif /* LAKESIDE_GPU_H */
