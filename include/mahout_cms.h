/*
 * mahout_cms.h -- C ABI of the MI355X-native count-min-sketch ingest and
 * sketch-cosine similarity path (libmahout_cms.so, gfx950).
 *
 * This is the drop-in boundary for Mahout Taste's CosineCM path.  Every entry
 * point below names the reference interface it replaces; "T/" abbreviates
 * mr/src/main/java/org/apache/mahout/cf/taste/ in jalhajj/mahout.
 *
 * Vocabulary (reference domain terms):
 *   owner  -- the entity a sketch belongs to.  CosineCM sketches a Taste
 *             "user" (T/impl/similarity/CosineCM.java:41-58); over a
 *             transposed DataModel (FileDataModel transpose=true,
 *             T/impl/model/file/FileDataModel.java:166,414-418) the owner is an
 *             item and this path is the sketch-cosine ItemSimilarity.
 *   key    -- the ID hashed into the sketch (the owner's preference IDs).
 *   row    -- dense index of an owner in the sorted owner-ID universe.
 *   depth d / width w -- sketch shape; counters are [d][w] row-major per
 *             owner (T/impl/common/DoubleCountMinSketch.java:62-64).
 *
 * Conventions:
 *   - every function is extern "C", noexcept, and returns int status
 *     (CMS_OK = 0) unless stated; the message of the last failure on the
 *     calling thread is cms_last_error().
 *   - pointers named h_* / plain are HOST memory, copied during the call and
 *     never retained; pointers named d_* are DEVICE memory on the handle's GPU.
 *   - similarity values are the reference's: in [-1, 1] or NaN ("unknown").
 *     NaN is a value, never an error.
 *   - the handle serialises ingest/finalize with an internal mutex; queries
 *     after cms_finalize are reentrant.
 */
#ifndef MAHOUT_CMS_H
#define MAHOUT_CMS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMS_ABI_VERSION 2 /* 2: cms_stats leads with struct_size */

/* ---- status codes (mapped to Java exceptions by the JNI shim) ---------- */
#define CMS_OK 0
#define CMS_E_PARAM 1      /* IllegalArgumentException / CMException (AbstractCountMinSketch.java:71-76) */
#define CMS_E_SHAPE 2      /* checkArgument w/d mismatch (DoubleCountMinSketch.java:117-118) */
#define CMS_E_NO_SUCH_ID 3 /* NoSuchUserException / NoSuchItemException (GenericDataModel.java:210-215) */
#define CMS_E_STATE 4      /* call-order violation (query before finalize, ...) */
#define CMS_E_VALUE 5      /* increment not a non-negative multiple of 2^-frac_bits below 2^(32-frac_bits) */
#define CMS_E_OVERFLOW 6   /* a counter could exceed the counter type */
#define CMS_E_HIP 7        /* HIP runtime error */
#define CMS_E_RCCL 8       /* RCCL error */
#define CMS_E_OOM 9        /* device or host allocation failed */
#define CMS_E_SKETCH 10    /* TasteException: CMException inside exportProfile (CosineCM.java:45-46) or no
                              configuration solution (CountMinSketchConfig.java:145-147) */

/* ---- parameters ----------------------------------------------------------- */
#define CMS_COUNTER_U32 0 /* exact integer counters (non-negative integer increments) */
#define CMS_COUNTER_F64 1 /* fp64 counters: DoubleCountMinSketch's own type, any float preference
                             (negative, non-dyadic); increments are applied per owner in ingest
                             order (the DataModel order CosineCM.exportProfile uses) and every sum
                             is the reference's sequential fp64 chain.  Single-GPU; fixed shapes
                             up to width 2^20, and per-owner shapes (cms_create_per_owner);
                             owners are built by CSR ingest or host COO ingest (stable by
                             owner), not by cms_ingest_device_rows. */

#define CMS_UNWEIGHTED 0 /* org.apache.mahout.cf.taste.common.Weighting */
#define CMS_WEIGHTED 1

typedef struct cms_params {
  uint32_t struct_size; /* = sizeof(cms_params); filled by cms_params_init */
  int32_t depth;        /* d, 1..32 (AbstractCountMinSketch.java:34-44 init; bound of this build) */
  int32_t width;        /* w: 1..32768 with CMS_COUNTER_U32, 1..2^20 with CMS_COUNTER_F64 */
  int32_t counter_type; /* CMS_COUNTER_* */
  int64_t seed;         /* HashFunctionBuilder(long seed) (HashFunctionBuilder.java:23) */
  int64_t num_owners;   /* n: rows of the sketch table */
  int32_t weighting;    /* CMS_UNWEIGHTED | CMS_WEIGHTED (CosineCM.java:33) */
  int32_t device;       /* HIP device ordinal; -1 = current device */
  int32_t frac_bits;    /* 0..31: preferences are multiples of 2^-frac_bits (1 for half-star
                           ratings); counters hold pref * 2^frac_bits.  Similarities are
                           scale-invariant bit for bit; point queries / counters read back
                           in preference units.  0 = integer preferences. */
  int32_t flags;        /* CMS_FLAG_* bits (0 = defaults) */
} cms_params;

/* cms_params.flags:
 * CMS_FLAG_COLLECTIVE_SINGLE_RANK -- a one-rank job still takes the multi-rank
 *   data path: cms_comm_init(h, uid, 0, 1) creates a real one-rank RCCL
 *   communicator (and cms_comm_init_transport(h, 0, 1, ...) attaches the
 *   caller's transport), so cms_finalize merges through the packed all-reduce,
 *   later COO batches go through the delta log and its all-gather, and
 *   cms_top_k_all through the collective merge -- each with one participant,
 *   so the results equal the plain single-GPU path bit for bit.  Without the
 *   flag a world of 1 detaches any communicator (the fast single-GPU path).
 *   Not with CMS_COUNTER_F64 (CMS_E_PARAM). */
#define CMS_FLAG_COLLECTIVE_SINGLE_RANK 0x1

typedef struct cms_handle cms_handle;

/* Defaults: d=5, w=4096, u32, seed=42, n=0, unweighted, device -1, frac_bits 0. */
int cms_params_init(cms_params* p);

/* AbstractCountMinSketch(double delta, double epsilon, ...) shape rule
 * (T/impl/common/AbstractCountMinSketch.java:69-83): w = ceil(e/eps),
 * d = ceil(ln(1/delta)); CMS_E_PARAM for the CMException ranges. */
int cms_shape_from_delta_epsilon(double delta, double epsilon, int32_t* width, int32_t* depth);

/* new DoubleCountMinSketch(width, depth, hfBuilder) for every owner at once
 * (T/impl/common/DoubleCountMinSketch.java:32-42) plus the CosineCM instance
 * state (CosineCM.java:26-39).  Counters start at zero.
 *
 * Tunables.  The library reads these environment variables once, here, and
 * never again (a handle's behaviour is fixed at creation); none changes any
 * result, only the storage or kernel a result comes from:
 *   CMS_NO_FORMS=1        narrow rows stay u16 (no 1/2/4/8-bit row forms)
 *   CMS_NO_COMPACT=1      every narrow row keeps a whole u16 slot (no compact row layout)
 *   CMS_EARLY_SLICES=1    the hot-routed split owners built beside pass 2 of the partition
 *   CMS_NO_VMM=1          the compact row arena as one hipMalloc grown by copying
 *                         (no reserved virtual range mapped in chunks)
 *   CMS_BIT_KEYS=<n>      byte-class owners of <= n keys try 1-bit rows first (64)
 *   CMS_CRUMB_KEYS=<n>    ... of <= n keys 2-bit rows (256)
 *   CMS_LIST_KEYS=<n>     ... of <= n keys, unit increments: sparse list rows (256; 0 = none)
 *   CMS_NO_HOT_ROUTING=1  the COO partition sends every owner through both passes
 *   CMS_NO_FP4=1          no e2m1 operand image: every single-limb pair on int8 MFMA
 *   CMS_NO_MLS=1          multi-limb slabs on the 128-row tile kernel instead of k_cosine_mls */
int cms_create(const cms_params* p, cms_handle** out);
void cms_destroy(cms_handle* h);
const char* cms_last_error(void);
int cms_abi_version(void);

/* Owner-ID universe: strictly ascending IDs, row i <-> ids[i] (the order of
 * DataModel.getUserIDs(), GenericDataModel.java:128-134).  Without this call
 * owner IDs are the row indices 0..n-1. */
int cms_set_owner_ids(cms_handle* h, const int64_t* ids, int64_t n);

/* The d hash parameters (a_i, b_i) of HashFunctionBuilder(seed)
 * (HashFunctionBuilder.java:40-61). */
int cms_hash_params(cms_handle* h, int64_t* a, int64_t* b);
/* Install a caller's HashFunctionBuilder parameters instead of the ones
 * drawn from p->seed: (a_i, b_i) = (randomParamA[i], randomParamB[i]) as the
 * builder drew them (HashFunctionBuilder.java:40-61) -- for a builder whose
 * seed is unknown (new HashFunctionBuilder() seeds from the clock).  count
 * must be the handle's depth (CMS_MAX_DEPTH = 32 for a per-owner handle: the
 * rows any owner's shape may use).  Before the first ingest only
 * (CMS_E_STATE otherwise; cms_reset allows it again). */
int cms_set_hash_params(cms_handle* h, const int64_t* a, const int64_t* b, int32_t count);

/* HashFunction.hash(key) for every row i < d, computed on the GPU
 * (HashFunction.java:31-34): out[k*d + i] = h_i(keys[k]). */
int cms_hash_keys(cms_handle* h, const int64_t* keys, int64_t n, int32_t* out);

/* ---- ingest: DoubleCountMinSketch.update(key, inc) for many owners --------
 * (DoubleCountMinSketch.java:72-80; CosineCM.exportProfile :41-58 feeds it the
 * owner's PreferenceArray).  val may be NULL (every increment 1.0, the
 * implicit-feedback stream).  With CMS_COUNTER_U32 every val must be a
 * non-negative integer (CMS_E_VALUE otherwise).  Duplicate (owner, key) pairs
 * ADD, as repeated update() calls do. */

/* COO pairs from host memory, owners by ID. */
int cms_ingest(cms_handle* h, const int64_t* owner, const int64_t* key, const float* val, int64_t n);
/* COO pairs already resident on the device, owners by row index. Asynchronous
 * on the handle's stream (use cms_synchronize).  The handle's stream is a
 * BLOCKING stream: it is ordered after work already queued on the device's
 * legacy default stream and before work queued there later.  Buffers written
 * on any other stream must be complete before the call, and every device
 * input must stay allocated until cms_synchronize (or a blocking call) returns. */
int cms_ingest_device_rows(cms_handle* h, const int64_t* d_row, const int64_t* d_key, const float* d_val,
                           int64_t n);
/* CSR from host memory: the owner at row r has keys[offsets[r] .. offsets[r+1])
 * -- the DataModel layout (one PreferenceArray per owner,
 * GenericUserPreferenceArray.java:52-54).  offsets has num_owners+1 entries. */
int cms_ingest_csr(cms_handle* h, const int64_t* offsets, const int64_t* keys, const float* vals);
/* CSR resident on the device.  The offsets are checked on the device before
 * any counter is touched (offsets[0] == 0, non-decreasing; CMS_E_PARAM
 * otherwise), so the build reads keys[0 .. offsets[num_owners]) only; d_keys
 * (and d_vals) must hold that many entries.  Asynchronous after that check.
 *
 * Device ingests are not all-or-nothing for the VALUES (unlike the host
 * ingests, which validate the whole batch first): a pair whose row is outside
 * [0, num_owners) (COO) or whose increment the counter type cannot take is
 * skipped, the others are applied, and the next synchronising call
 * (cms_synchronize / cms_finalize) reports CMS_E_PARAM / CMS_E_VALUE. */
int cms_ingest_csr_device(cms_handle* h, const int64_t* d_offsets, const int64_t* d_keys, const float* d_vals);

/* Forget all counters (next ingest rebuilds the table from zero). */
int cms_reset(cms_handle* h);

/* Return the handle's ingest/query scratch to the device allocator (the
 * table, norms and the all-pairs operands stay).  For 288 GB budgets: a
 * 1M-owner d=5 w=8192 table is 164 GB on its own. */
int cms_release_scratch(cms_handle* h);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ----------------------
 * The interaction stream is sharded by key (user) hash; each rank ingests its
 * shard into a full-shape partial table and cms_finalize sums the tables with
 * RCCL.  Counters are integers, so the merged table is bit-identical for any
 * rank count. */
int cms_comm_unique_id(void* out /* 128 bytes, ncclUniqueId */);
int cms_comm_init(cms_handle* h, const void* unique_id, int32_t rank, int32_t world);
/* The sharding function: rank that owns `key` among `world` ranks. */
int32_t cms_shard_of_key(int64_t key, int32_t world);

/* Merge (RCCL all-reduce when a communicator is attached), then derive the
 * per-(owner,row) norms the cosine needs.  Queries require it.
 * The merge is counter-width adaptive: one all-reduce of (row mass, largest
 * local counter) per owner bounds every merged counter of that owner, and the
 * counters then travel as bit fields of exactly that width packed into u64
 * words whose u64 sums cannot carry between fields -- the merged table is
 * bit-identical to a u32 all-reduce at a fraction of the xGMI bytes. */
int cms_finalize(cms_handle* h);
/* The same merge through a caller-supplied collective instead of RCCL (an MPI,
 * torch.distributed or Spark transport): fn(d_buf, count, user) must replace
 * the count u64 words at device pointer d_buf (on the handle's device; the
 * handle's stream is idle) by their sum over all ranks, and return 0.  It is
 * called a fixed number of times, with identical counts on every rank.  The
 * merged table takes no further ingest until cms_reset (CMS_E_STATE). */
typedef int (*cms_allreduce_fn)(void* d_buf, int64_t count, void* user);
int cms_finalize_with(cms_handle* h, cms_allreduce_fn fn, void* user);
/* A whole multi-rank communicator supplied by the caller instead of RCCL (an
 * MPI, torch.distributed or Spark transport).  After this call the handle
 * behaves exactly as after cms_comm_init: cms_finalize merges through
 * `allreduce` (as cms_finalize_with), later COO batches go into the delta log
 * and the next cms_finalize exchanges the logs through `allgather`, and
 * cms_top_k_all is collective (partial lists gathered through `allgather`,
 * merged exactly).  allgather(d_send, d_recv, bytes, user) must write the
 * `bytes` bytes of every rank's d_send, concatenated in rank order, to d_recv
 * (world * bytes, device memory on the handle's device; the handle's stream
 * is idle during the call) and return 0.  Every rank makes the same sequence
 * of calls with identical sizes.  world == 1 detaches any communicator. */
typedef int (*cms_allgather_fn)(const void* d_send, void* d_recv, int64_t bytes, void* user);
int cms_comm_init_transport(cms_handle* h, int32_t rank, int32_t world, cms_allreduce_fn allreduce,
                            cms_allgather_fn allgather, void* user);
int cms_synchronize(cms_handle* h);
/* Stream ordering without a host wait (stream: a hipStream_t of the handle's
 * device, e.g. the caller's current torch stream; NULL = legacy default).
 * cms_wait_stream: the handle's later work waits for everything queued on
 * `stream` so far (inputs written there are complete before they are read).
 * cms_release_to_stream: later work queued on `stream` waits for the handle's
 * work queued so far (device inputs may then be freed / reused on `stream`). */
int cms_wait_stream(cms_handle* h, void* stream);
int cms_release_to_stream(cms_handle* h, void* stream);

/* ---- queries (after cms_finalize) ---------------------------------------- */

/* CosineCM.userSimilarity(id1, id2) (CosineCM.java:83-96): min over the d rows
 * of the per-row cosine (DoubleCountMinSketch.cosine :114-149), then
 * normalizeWeightResult(r, 1, 0) (AbstractSimilarity.java:313-330).
 * CMS_E_NO_SUCH_ID for unknown owners. */
int cms_similarity(cms_handle* h, int64_t id1, int64_t id2, double* out);
/* ItemSimilarity.itemSimilarities(id1, ids2[]) (ItemSimilarity.java:58) as
 * one batched GPU call. */
int cms_similarities(cms_handle* h, int64_t id1, const int64_t* ids2, int64_t n, double* out);
/* DoubleCountMinSketch.get(key) of owner `id` (DoubleCountMinSketch.java:94-103),
 * the point query GenericUserBasedRecommender uses (:153-158). */
int cms_point_query(cms_handle* h, int64_t id, int64_t key, double* out);
/* GenericUserBasedRecommender.doEstimatePreference(user, neighbourhood, item)
 * with the CosineCM point query (GenericUserBasedRecommender.java:134-184) for
 * q items at once: out[i] is the float estimate for item_keys[i], NaN when
 * fewer than two neighbours carry data.  neighbor_ids is the neighbourhood in
 * the caller's order (NearestNUserNeighborhood order); use_capper applies
 * EstimatedPreferenceCapper(cap_min, cap_max) (:209-216).  The DataModel's own
 * preference short cut of estimatePreference (:108-116) stays with the caller. */
int cms_estimate_preferences(cms_handle* h, int64_t user_id, const int64_t* neighbor_ids, int64_t m,
                             const int64_t* item_keys, int64_t q, int32_t use_capper, float cap_min, float cap_max,
                             float* out);
/* cms_estimate_preferences for n users in one call -- the estimate phase of
 * GenericUserBasedRecommender.recommend (:84-105) for a whole user batch:
 * user u's neighbourhood is neighbor_ids[nb_offsets[u] .. nb_offsets[u+1])
 * (in NearestNUserNeighborhood order) and its candidate items
 * item_keys[item_offsets[u] .. item_offsets[u+1]); out is parallel to
 * item_keys.  Both offset arrays hold n + 1 non-decreasing entries from 0.
 * Every estimate equals the single-user call's (same order of fp64 sums). */
int cms_estimate_preferences_batch(cms_handle* h, int64_t n, const int64_t* user_ids, const int64_t* nb_offsets,
                                   const int64_t* neighbor_ids, const int64_t* item_offsets, const int64_t* item_keys,
                                   int32_t use_capper, float cap_min, float cap_max, float* out);
/* GenericUserBasedRecommender.recommend(userID, how_many) for n users at
 * once (GenericUserBasedRecommender.java:84-105), replacing one
 * Recommender.recommend call per user.  The caller supplies each user's
 * neighbourhood (nb_offsets / neighbor_ids: IDs in NearestNUserNeighborhood
 * order, e.g. from cms_top_k_all) and the DataModel's item IDs per user
 * (model_user_ids ascending; row r's items pref_items[pref_offsets[r] ..
 * pref_offsets[r + 1]) in getPreferencesFromUser order).  Per user: the
 * candidates are getAllOtherItems (:187-198) in FastIDSet iteration order,
 * their estimates come from one cms_estimate_preferences_batch over all
 * users, and the list is TopItems.getTopItems (TopItems.java:47-88) with the
 * JDK PriorityQueue's order for ties.  out_counts[n] (<= how_many, 0 for an
 * empty neighbourhood), out_items / out_values [n][how_many] (float values,
 * as RecommendedItem.getValue()).  A user or neighbour missing from the model
 * is CMS_E_NO_SUCH_ID (NoSuchUserException). */
int cms_recommend_batch(cms_handle* h, int64_t n, const int64_t* user_ids, const int64_t* nb_offsets,
                        const int64_t* neighbor_ids, int64_t n_model_users, const int64_t* model_user_ids,
                        const int64_t* pref_offsets, const int64_t* pref_items, int32_t how_many,
                        int32_t include_known, int32_t use_capper, float cap_min, float cap_max, int32_t* out_counts,
                        int64_t* out_items, float* out_values);
/* GenericUserBasedRecommender.mostSimilarUserIDs(id, k) with the CosineCM
 * estimator (:119-127, :231-247) and TopItems.getTopUsers (TopItems.java:91-136):
 * the first k other owners under (similarity desc, ID asc), NaN excluded.
 * Writes *count <= k entries; scores are the fp64 similarities. */
int cms_most_similar(cms_handle* h, int64_t id, int32_t k, int64_t* out_ids, double* out_scores, int32_t* count);
/* mostSimilar for every owner in rows [row_begin, row_begin+row_count): the
 * all-pairs top-k pass (config 4).  ids/scores are [row_count][k]; counts[row_count]. */
int cms_top_k_rows(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t k, int64_t* ids,
                   double* scores, int32_t* counts);
/* mostSimilar for EVERY owner (config 4, the suggested cms_topk_all of the
 * scope table): the same lists as cms_top_k_rows(h, 0, num_owners, ...), but
 * each unordered pair's similarity is computed once and streamed into both
 * owners' lists (no n x n slab).  ids/scores are [num_owners][k] by owner
 * row, counts[num_owners]; k <= 512.  Entries past counts[r] in row r are
 * padding with a defined value: ID -1 and a NaN score (every byte 0xFF), for
 * this call and for cms_top_k_refresh and the _device variants below. */
int cms_top_k_all(cms_handle* h, int32_t k, int64_t* ids, double* scores, int32_t* counts);
/* cms_top_k_all with the lists left on the device: d_ids / d_scores
 * [num_owners][k] and d_counts [num_owners] on the handle's GPU (no host copy
 * of the 1.6 GB answer at 1M owners, k = 100).  Returns when they are written. */
int cms_top_k_all_device(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts);
/* With a communicator (cms_comm_init, world G > 1) cms_top_k_all is collective:
 * rank r computes shard r of the pairs, the partial lists are all-gathered
 * over RCCL and merged exactly; every rank receives the full result
 * (G * k <= 1024).  The two pieces are also exported: */
/* The partial lists of shard `shard` of `nshards` ([num_owners][k] IDs and
 * scores, counts): every pair is computed by exactly one shard. */
int cms_top_k_all_partial(cms_handle* h, int32_t k, int32_t shard, int32_t nshards, int64_t* ids, double* scores,
                          int32_t* counts);
/* Exact merge of nparts partial lists laid out [nparts][num_owners][k] (counts
 * [nparts][num_owners]) into the final lists (nparts * k <= 1024). */
int cms_top_k_merge(cms_handle* h, int32_t k, int32_t nparts, const int64_t* ids, const double* scores,
                    const int32_t* counts, int64_t* out_ids, double* out_scores, int32_t* out_counts);
/* The periodic top-k refresh of a streaming table (config 5; the Refreshable
 * contract of the precomputed similarities, T/common/Refreshable.java:51,
 * feeding GenericItemSimilarity): returns exactly what cms_top_k_all returns
 * for the current table.  The first call (or one with another k, or after a
 * CSR ingest, cms_reset or the first multi-rank merge) runs the whole job and
 * keeps every owner's list 2k deep on the device; later calls recompute only
 * the pairs with an owner a COO ingest touched since, fold them into the kept
 * lists, and recompute whole any list that lost its exactness margin.
 * Collective like cms_top_k_all with a communicator. */
int cms_top_k_refresh(cms_handle* h, int32_t k, int64_t* ids, double* scores, int32_t* counts);
/* cms_top_k_refresh into device buffers (layout and padding as
 * cms_top_k_all_device). */
int cms_top_k_refresh_device(cms_handle* h, int32_t k, int64_t* d_ids, double* d_scores, int32_t* d_counts);
/* Statistics of the last cms_top_k_refresh: owners touched (num_owners for a
 * whole job), lists recomputed whole, whole jobs so far. */
int cms_refresh_stats(cms_handle* h, int64_t* touched, int64_t* redone, int64_t* full_jobs);
/* Operand classes of the last cms_top_k_refresh's all-pairs job: out6 =
 * {multi-limb owners, int8 owners, fp4 owners, touched multi-limb, touched
 * int8, touched fp4} (a whole job counts every owner as touched).  Each class
 * has its own pair cost (k_cosine_mls limb passes, int8 and fp4 symmetric
 * waves), so the work a refresh must redo follows from these six counts.
 * Zeros for per-owner and fp64 handles (no operand classes). */
int cms_refresh_classes(cms_handle* h, int64_t* out6);

/* cms_top_k_all written as FileSimilarItemsWriter does
 * (T/impl/similarity/precompute/FileSimilarItemsWriter.java:50-61): one line
 * "itemID,similarItemID,similarity" per similar item, owners in ascending ID
 * order, each list most similar first; similarity as Java's
 * String.valueOf(double), narrowed to float first when as_float (the
 * RecommendedItem values SimilarItems carries, SimilarItems.java:36-47). */
int cms_write_similar_items(cms_handle* h, const char* path, int32_t k, int32_t as_float);
/* The same all-pairs lists in the output formats of the other similarity
 * drivers a sketch cosine can stand in for:
 *   CMS_FORMAT_ITEM_SIMILARITY_JOB -- ItemSimilarityJob's text result
 *     (T/hadoop/similarity/item/ItemSimilarityJob.java:181-233): each pair of
 *     a list once as "aID\tbID\tsimilarity" with aID < bID, sorted by (aID, bID)
 *     (EntityEntityWritable.java:64-71); for a pair listed by both owners the
 *     lower ID's value is kept.
 *   CMS_FORMAT_SPARK_ITEMSIMILARITY -- spark-itemsimilarity's
 *     TextDelimitedIndexedDatasetWriter, default schema
 *     (spark/src/main/scala/org/apache/mahout/drivers/TextDelimitedReaderWriter.scala:244-303):
 *     "ID\tID1:s1 ID2:s2 ..." per owner, non-zero similarities by strength
 *     descending; a bare "ID" when the list is empty.
 * Values print as Java's Double.toString (fp64). */
#define CMS_FORMAT_ITEM_SIMILARITY_JOB 1
#define CMS_FORMAT_SPARK_ITEMSIMILARITY 2
int cms_write_similarities(cms_handle* h, const char* path, int32_t k, int32_t format);
/* cms_write_similarities with RowSimilarityJob's --threshold: pairs whose
 * similarity is below `threshold` are left out (of the lists before the top-k,
 * which for a top-k list is the same as dropping them afterwards;
 * RowSimilarityJob.java, ItemSimilarityJob.java:128-129).  In the
 * ItemSimilarityJob format a pair also needs similarity > Double.MIN_VALUE,
 * the TopSimilarItemsQueue sentinel (TopSimilarItemsQueue.java:50-58,
 * ItemSimilarityJob.java:203-209). */
int cms_write_similarities_threshold(cms_handle* h, const char* path, int32_t k, int32_t format, double threshold);
/* Java Double.toString(v) into buf (NUL-terminated); returns the length or -1. */
int cms_format_java_double(double v, char* buf, int32_t cap);

/* Counters of rows [row_begin, row_begin+row_count) as fp64 (the reference's
 * counter type), [row_count][d][w]. */
int cms_read_counters(cms_handle* h, int64_t row_begin, int64_t row_count, double* out);
/* The same counters without leaving the device: u32 in counter units (the
 * preference times 2^frac_bits), [row_count][d][w], written to d_out on the
 * handle's stream (asynchronous, like the device ingests) -- for a device-side
 * consumer of the sketches (getExportedCMProfile for many owners,
 * CosineCM.java:60-67) and for whole-table checks at sizes the host cannot hold. */
int cms_read_counters_device(cms_handle* h, int64_t row_begin, int64_t row_count, uint32_t* d_out);
/* How each owner's counters are stored (no reference counterpart: the
 * reference keeps every sketch as fp64): out_form[i] is one of CMS_FORM_*,
 * out_bound[i] the proven bound on the owner's counters the form was chosen
 * for (0 for u32 rows; either output may be NULL).  For capacity checks. */
#define CMS_FORM_U32 0  /* hot row: u32 slot */
#define CMS_FORM_U16 1
#define CMS_FORM_U8 2
#define CMS_FORM_U4 3
#define CMS_FORM_U2 4
#define CMS_FORM_U1 5
#define CMS_FORM_LIST 6 /* sparse key-bucket list */
int cms_owner_forms(cms_handle* h, int64_t row_begin, int64_t row_count, int32_t* out_form, uint32_t* out_bound);

/* ---- per-owner sketch shapes: CosineCM with its CountMinSketchConfig --------
 * The reference sizes every owner's sketch separately.  CountMinSketchConfig
 * (T/impl/common/CountMinSketchConfig.java:120-158) picks (d, w) per owner and
 * stores delta = exp(-d), epsilon = e/w; CosineCM.userSimilarity(u1, u2)
 * builds u1's sketch with u2's (delta, epsilon) and compares it with u2's own
 * cached sketch (T/impl/similarity/CosineCM.java:60-67,83-96), so the
 * similarity is asymmetric.  A per-owner handle keeps the DataModel (one
 * cms_ingest_csr / cms_ingest_csr_device call; a later call replaces it)
 * resident on the GPU; cms_finalize builds every owner's own sketch, and the
 * similarity kernels hash u1's preferences at u2's shape on the fly.
 * p->depth / p->width are ignored.  cms_similarity(ies), cms_point_query,
 * cms_estimate_preferences, cms_most_similar, cms_top_k_rows, cms_top_k_all
 * and cms_write_similar_items work as for fixed shapes; the COO ingests,
 * cms_read_counters, cms_hash_keys and cms_top_k_all_partial return
 * CMS_E_STATE.  Several GPUs: every rank ingests the whole DataModel (u1's
 * preferences are hashed at each candidate's shape) and, after
 * cms_comm_init / cms_comm_init_transport, cms_top_k_all splits the QUERY
 * rows over the ranks (256-row chunks round-robin) and all-gathers the lists,
 * so every rank returns the single-GPU answer. */
int cms_create_per_owner(const cms_params* p, cms_handle** out);
/* CountMinSketchConfig(q).configure(dataModel) -> computeConfig on the GPU:
 * per owner n = its CSR row length (PreferenceArray.length()), u = num_keys
 * (dataModel.getNumItems()); maximise Fmeasure(w, d, n, u, q) (:210-219) over
 * d in [1, 25), w in [d, n], ties to the last (>=, :137); delta = exp(-d),
 * epsilon = e/w.  Needs the DataModel first.  CMS_E_SKETCH for an owner with
 * no solution (the TasteException of :145-147). */
int cms_configure_owner_shapes(cms_handle* h, double q, int64_t num_keys);
/* Caller-supplied configuration: the getDelta(id) / getEpsilon(id) values of
 * a CountMinSketchConfig (:230-251), in owner-row order.  An owner whose pair
 * is outside the CMException ranges (AbstractCountMinSketch.java:71-76; e.g.
 * the 0.0 trove returns for a missing owner) fails, with CMS_E_SKETCH, exactly
 * the calls that need its shape with CMS_E_SKETCH (exportProfile, CosineCM.java:41-58).  Shapes
 * beyond this build (depth > 32, width > 2^24) are refused here. */
int cms_set_owner_delta_epsilon(cms_handle* h, const double* delta, const double* epsilon);
/* The configuration and the shape new DoubleCountMinSketch(delta, epsilon, ...)
 * derives from it (width = depth = 0: CMException).  Outputs may be NULL. */
int cms_get_owner_shapes(cms_handle* h, double* delta, double* epsilon, int32_t* width, int32_t* depth);
/* getExportedCMProfile(id) (CosineCM.java:60-67): the owner's own sketch as
 * fp64 [depth][width] (capacity in doubles; out NULL returns the shape only). */
int cms_read_owner_sketch(cms_handle* h, int64_t id, double* out, int64_t capacity, int32_t* width, int32_t* depth);

/* ---- instrumentation ------------------------------------------------------- */
typedef struct cms_stats {
  uint32_t struct_size;     /* sizeof(cms_stats) as the caller compiled it: only fields that fit are written */
  int64_t pairs_ingested;   /* update() calls applied on this rank */
  int64_t num_owners;
  int32_t depth, width;
  int32_t exact_norms;      /* 1 if every (owner,row) norm is < 2^53 (bit-exact fast path) */
  int32_t world, rank;
  int64_t table_bytes;       /* the narrow rows' arena as laid out (zero row + every row's place) + the hot owners' u32 rows */
  int64_t multi_limb_owners; /* owners with a counter >= 128 (all-pairs limb split; -1 before the first all-pairs call) */
  int64_t topk_redo;         /* top-k rows that needed the radix-select fallback */
  int64_t deep_limb_owners;  /* of those, owners with a counter >= 2^14 (3+ limbs); -1 before */
  int64_t fp4_owners;        /* single-limb owners with every counter <= 4 (fp4 MFMA operands); -1 before */
  int64_t merge_words;       /* u64 words the last multi-rank merge all-reduced (packed counters) */
  int64_t hot_rows;          /* owners whose counters are stored as u32 (the others narrow) */
  int64_t stored_bytes;      /* bytes of counters as stored: what one whole-table build writes */
  int64_t u8_rows;           /* narrow owners stored as u8 (every counter < 2^8) */
  int64_t nibble_rows;       /* narrow owners stored as 4-bit counters (every counter < 2^4) */
  int64_t crumb_rows;        /* narrow owners stored as 2-bit counters (every counter < 2^2) */
  int64_t bit_rows;          /* narrow owners stored as 1-bit counters (every counter 0 or 1) */
  int64_t collective_calls;  /* all-reduce / all-gather calls made through the communicator so far */
  int32_t comm_kind;         /* 0 none (single-GPU path), 1 RCCL (cms_comm_init), 2 caller transport */
  int32_t device;            /* HIP device ordinal of the handle */
  int64_t list_rows;         /* narrow owners stored as sparse key-bucket lists (2 + 2 d m bytes, m keys) */
  int64_t po_wide_pairs;     /* per-owner top-k: (query, wide owner) pairs given the row-0 bound so far */
  int64_t po_wide_exact;     /* of those, pairs the bound could not rule out (computed exactly) */
} cms_stats;
/* out->struct_size must be set (at least through pairs_ingested); an ABI-2
 * caller whose cms_stats is shorter (built before later fields were appended)
 * receives the fields it knows. ABI-1 structs had no struct_size: bindings
 * compare cms_abi_version() with CMS_ABI_VERSION at load time (mahout_amd/_lib.py,
 * the JNI shim's JNI_OnLoad) and refuse a mismatch. */
int cms_get_stats(cms_handle* h, cms_stats* out);

/* Per-kernel HIP-event timing on the handle's stream (off by default).
 * level 1: the roofline kernels' scopes only ("build_rows", "ingest_atomic",
 * "allreduce", the cosine / top-k families); level >= 2: every scope, the
 * ingest phases ("partition", "build_plan", "hot_norms", "norms", merge
 * phases) included -- each recorded event costs the stream a few us. */
int cms_set_timing(cms_handle* h, int32_t enabled);
/* Accumulated (total ms, launches) for a kernel family name, e.g.
 * "build_rows", "partition", "norms", "allreduce", "cosine".  Process-wide
 * host counters, whatever the timing switch (cleared by cms_reset_timing):
 * "host_alloc" = ms in the library's hipMalloc calls (launches = calls),
 * "host_free" = ms in the hipFree of a growing buffer (it waits for queued
 * device work), "host_alloc_bytes" = bytes allocated (in total_ms),
 * "host_alloc_max" = the slowest single hipMalloc (ms; its bytes in launches). */
int cms_get_timing(cms_handle* h, const char* name, double* total_ms, int64_t* launches);
int cms_reset_timing(cms_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* MAHOUT_CMS_H */
