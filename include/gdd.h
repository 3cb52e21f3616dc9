/*
 * gdd.h — C ABI of libgdd, the MI355X-native (gfx950) hot path of ClustGDD graph distillation.
 *
 * The reference (Tyler-Linchenwei/Graph-Distillation-for-Recommendation, ClustGDD/) has no FFI layer:
 * its hot path is inline Python inside ClustGDD.pretrained_clustering and distill_recsys.kmeans_cluster.
 * Each entry point below replaces one of those call sites; the cited file:line is the reference code
 * whose arithmetic the entry point restates (paths relative to the reference's ClustGDD/ directory,
 * or to scikit-learn 1.7.2 for the k-means internals the reference calls).
 *
 * Conventions (all entry points):
 *   - every array argument is a DEVICE pointer, caller-owned (PyTorch allocates), row-major, dense;
 *   - work is enqueued on `stream` (the caller's torch.cuda.current_stream()); no entry point
 *     synchronises the host except where its comment says so;
 *   - the library keeps no device memory and no global mutable state; scratch comes from a caller
 *     workspace sized by the matching *_ws_bytes() query;
 *   - return 0 on success, otherwise a GDD_E_* code or a hipError_t value; gdd_last_error() gives a
 *     thread-local message. Shapes are validated on the host before any launch.
 */
#ifndef GDD_H_
#define GDD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* gdd_stream_t; /* == hipStream_t */

#define GDD_OK 0
#define GDD_E_INVALID 0x10001   /* bad shape / null pointer / unsupported parameter */
#define GDD_E_WORKSPACE 0x10002 /* workspace too small */
#define GDD_E_NODEVICE 0x10003  /* no gfx950 device visible */

/* ---------------------------------------------------------------------------------------------- */
/* Library                                                                                          */
/* ---------------------------------------------------------------------------------------------- */
const char* gdd_last_error(void);
int gdd_abi_version(void); /* bumps on any signature change */
/* The bound of the library's LDS arrival-counter spins (1 << 16; 0 in the `make SPIN0=1` twin
   whose every bounded wait gives up, so that the redo paths run — tests/test_gpu_spin0.py). */
int gdd_spin_limit(void);
/* 1 if the current HIP device is gfx950 and the embedded code objects can run on it. */
int gdd_device_ok(void);
/* Streaming device copy (16-byte aligned, bytes % 16 == 0): the bench's measured HBM copy peak     */
/* (SURVEY §8(d) roofline: "measure the achievable peak on the box with a copy kernel").           */
int gdd_stream_copy(const void* src, void* dst, size_t bytes, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (a2) normalisation:  Â = D^-1/2 (A + I) D^-1/2                                                   */
/* Replaces deep_robust_utils.normalize_adj_tensor(adj, sparse=True)  (deep_robust_utils.py:245-256)  */
/*   -> to_scipy (:408-417) -> normalize_adj (:180-207) -> sparse_mx_to_torch_sparse_tensor (:389-396) */
/* Input: canonical CSR of A (rows ascending, columns strictly ascending per row, no duplicates);    */
/*   val == NULL means every stored value is 1.0f (binary adjacency).                               */
/* self_loops: -1 = reference rule (add I iff A[0,0] == 0, deep_robust_utils.py:199-200),            */
/*              0 = never, 1 = always.                                                              */
/* When I is added the row sums, r = rowsum^-1/2 (inf -> 0) and both scalings are done in fp64 and    */
/* the result is rounded to fp32 (sp.eye promotes the matrix to float64); otherwise in fp32.         */
/* Output: canonical CSR; entries whose scaled value is exactly 0 are dropped (scipy csr_matmat       */
/* drops them). col_out / val_out must hold nnz + n entries; rowptr_out[n] receives nnz_out.         */
/* ---------------------------------------------------------------------------------------------- */
size_t gdd_normalize_ws_bytes(int64_t n, int64_t nnz);
int gdd_normalize_csr(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                      const float* val, int self_loops, int32_t* rowptr_out, int32_t* col_out,
                      float* val_out, void* ws, size_t ws_bytes, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (a3) feature propagation                                                                         */
/* Replaces the loop clustgdd_agent_transduct.py:59-65 (and clustgdd_agent_induct.py:72-94):          */
/*   t = 0:      p = X,                 target = fp32(1-alpha) * X                                   */
/*   t = 1..T-1: p = (fp32(alpha) * Â) @ p,  target = target + fp32(1-alpha) * p                    */
/* Canonical summation order of one output row: its stored entries in CSR order are cut into         */
/* segments of GDD_PROP_SEG entries; each segment is an fp32 fma chain from +0 in entry order; the   */
/* segment partials are added left to right. `p_last` receives p after the last hop (X if T == 1).   */
/* X, target, p_last, p_tmp: n x d fp32; p_tmp is scratch (may alias nothing else).                  */
/* ---------------------------------------------------------------------------------------------- */
#define GDD_PROP_SEG 256
size_t gdd_propagate_ws_bytes(int64_t n, int64_t nnz, int d);
/* r06: from 1M rows a one-workgroup probe samples the CSR; where half the sampled entries point within */
/* 4,096 rows of their row (ids that carry locality) the hops walk the rows in order, else longest     */
/* rows first — a schedule only, the results are the same bits.                                       */
int gdd_propagate(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col, const float* val,
                  int d, const float* X, int T, float alpha, float* target, float* p_last,
                  float* p_tmp, void* ws, size_t ws_bytes, gdd_stream_t stream);
/* The same propagation with the intermediate hops in a relabelled node order (r05):  */
/* rho (device, a permutation of [0, n)) gives node r's row of the intermediate p at rho[r] and the   */
/* gathers after the first go through rho[col]; every row keeps its entries in CSR order, so target  */
/* and p_last (both by the original ids: the first hop reads X by them, the last hop stores by them)  */
/* are bit-identical to gdd_propagate's. A locality order (hubs first, RCM, communities) lets the    */
/* gathered rows of a hop share cache lines and pages; no separate permutation pass. r06: every hop's */
/* work list walks the rows in the new order (consecutive items gather neighbouring rows). rho is not */
/* checked on the device: a non-permutation writes out of bounds (gdd.propagate checks it on the host).*/
size_t gdd_propagate_relabeled_ws_bytes(int64_t n, int64_t nnz, int d);
int gdd_propagate_relabeled(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                            const float* val, const int32_t* rho, int d, const float* X, int T,
                            float alpha, float* target, float* p_last, float* p_tmp, void* ws,
                            size_t ws_bytes, gdd_stream_t stream);
/* one hop: y = (scale * Â) @ x with the canonical order above; if acc != NULL also                   */
/*   acc = acc + acc_scale * y  (two fp32 roundings, no contraction).                               */
int gdd_spmm(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col, const float* val,
             int d, float scale, const float* x, float* y, float* acc, float acc_scale, void* ws,
             size_t ws_bytes, gdd_stream_t stream);
/* The same hop split in two: gdd_spmm_plan builds the row-segment work list of a CSR structure in  */
/* ws (gdd_propagate_ws_bytes(n, nnz, d)); gdd_spmm_planned then runs hops against it without      */
/* rebuilding it (one k_hop + one fix-up launch per call) — the unit the bench times per launch.     */
int gdd_spmm_plan(int64_t n, int64_t nnz, const int32_t* rowptr, int d, void* ws, size_t ws_bytes,
                  gdd_stream_t stream);
int gdd_spmm_planned(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                     const float* val, int d, float scale, const float* x, float* y, float* acc,
                     float acc_scale, const void* ws, size_t ws_bytes, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (a5/a6/a8) k-means building blocks (scikit-learn 1.7.2 semantics, fp32 data)                      */
/* Replace MiniBatchKMeans/KMeans(...).fit at clustgdd_agent_transduct.py:102-105,                    */
/* clustgdd_agent_induct.py:131-134, distill_recsys.py:174-180. Loop control and the MT19937 draws    */
/* stay on the host (numpy RandomState is the reference's own RNG).                                 */
/* ---------------------------------------------------------------------------------------------- */

/* out[i] = sum_j X[i,j]^2 in numpy's einsum("ij,ij->i") float32 order (sklearn row_norms,           */
/* sklearn/utils/extmath.py:76): 4 lanes, 16-element blocks fed in reverse vector order, mul+add     */
/* (no fma), lanes reduced (l0+l1)+(l2+l3). Bit-exact with numpy on x86-64 SSE3 builds.              */
int gdd_row_norms(int64_t n, int dim, const float* X, float* out, gdd_stream_t stream);

/* Assignment (E-step) of sklearn _update_chunk_dense (sklearn/cluster/_k_means_lloyd.pyx:172-213):  */
/*   d[i,j] = fma(-2, sum_t X[i,t]*C[j,t] as a t-ordered fp32 fma chain, c_norm2[j])                */
/*   labels[i] = first j with minimal d  (strict <, lowest index wins)                              */
/* computed with v_mfma_f32_32x32x2_f32 (exact k-ordered fma chain = OpenBLAS sgemm, bit-exact).     */
/* rows == NULL: rows are 0..n-1; otherwise row i of the batch is X[rows[i]] (minibatch gather).     */
/* sq_dist (nullable): per-sample ||x - c_label||^2 in sklearn _euclidean_dense_dense order          */
/* (sklearn/cluster/_k_means_common.pyx:26-48: 4-term groups, mul+add, no fma).                      */
/* dim <= 512. Workspace: gdd_kmeans_assign_ws_bytes(n) (one 64-bit key per sample).              */
size_t gdd_kmeans_assign_ws_bytes(int64_t n);
int gdd_kmeans_assign(int64_t n, int dim, const float* X, const int64_t* rows, int k,
                      const float* C, const float* c_norm2, int32_t* labels, float* sq_dist,
                      void* ws, size_t ws_bytes, gdd_stream_t stream);
/* bf16 distance variant (configs 2, 3, 5 carry fp32 and bf16 distances). Same        */
/* arguments and outputs; the X and C operands are rounded to bf16 (nearest even) and the dot       */
/* products run as v_mfma_f32_32x32x16_bf16 chains with fp32 accumulation; distances use the fp32    */
/* c_norm2 (NULL: computed on the device, no separate launch on the common shapes). NOT bit-compatible with sklearn: a label may differ where two centres' distances lie     */
/* within the bf16 rounding of the dot products (|err| <= ~2^-7 ||x|| ||c||). sq_dist is the exact   */
/* fp32 distance to the chosen centre.                                                              */
int gdd_kmeans_assign_bf16(int64_t n, int dim, const float* X, const int64_t* rows, int k,
                           const float* C, const float* c_norm2, int32_t* labels, float* sq_dist,
                           void* ws, size_t ws_bytes, gdd_stream_t stream);

/* out[0] = sequential fp32 sum of sq_dist[i] * w[i] in sample order (w == NULL: ones); this is      */
/* sklearn _inertia_dense with one OpenMP thread (_k_means_common.pyx:92-121).                       */
/* Evaluated in parallel with the sequential result bit for bit (gdd_seqsum.hip: per-binade integer   */
/* advances with a round-to-even parity carry, scanned by one workgroup). Non-negative finite terms   */
/* take the parallel form; NaN, infinite or negative terms are added one at a time from there.       */
int gdd_inertia(int64_t n, const float* sq_dist, const float* w, float* out, gdd_stream_t stream);
/* The same sum for long arrays in three launches over ~2048-term segments (per-segment advances for  */
/* the two likeliest binades, then one resolving workgroup); ws: gdd_inertia_ws_bytes(n) bytes.       */
size_t gdd_inertia_ws_bytes(int64_t n);
int gdd_inertia_ws(int64_t n, const float* sq_dist, const float* w, float* out, void* ws,
                   size_t ws_bytes, gdd_stream_t stream);

/* MiniBatchKMeans center update, sklearn _minibatch_update_dense (_k_means_minibatch.pyx:11-108):    */
/* for each cluster c with batch weight ws > 0: C_new[c] = (C_old[c]*W[c] + sum_{i in c, batch order} */
/* X_i*w_i) * fp32(1/(W[c]+ws)), W[c] += ws; otherwise C_new[c] = C_old[c].                        */
size_t gdd_minibatch_update_ws_bytes(int64_t b, int k);
int gdd_minibatch_update(int64_t b, int dim, const float* X, const int64_t* rows, const float* w,
                         const int32_t* labels, int k, const float* C_old, float* C_new,
                         float* weight_sums, void* ws, size_t ws_bytes, gdd_stream_t stream);

/* One MiniBatchKMeans step on the device: sklearn _mini_batch_step without the reassignment        */
/* branch (_kmeans.py:1556-1638) — ||C_old||^2, MFMA assignment of the gathered batch X[rows],       */
/* sequential batch inertia, centre update into C_new — followed, with GDD_STEP_CONVERGE, by         */
/* _mini_batch_convergence (:1960-2027, EWA of inertia/b in unfused fp64, max_no_improvement; -1 =   */
/* None; the test reads only the batch inertia, so it may precede the host's reassignment).          */
/* `state` (gdd_minibatch_state_bytes(), zero-initialised) carries the EWA state and, as an int32 at */
/* offset 16, stop_at = 0 while running or s+1 once the test fired at step s: every kernel of a      */
/* later step is then a no-op, so the host may enqueue steps ahead of the decision. Each step leaves */
/* ||C_new||^2 in the workspace; pass GDD_STEP_NORMS_VALID when C_old is the previous step's C_new  */
/* (unmodified by the host) to reuse them. batch b <= 13312.                                         */
#define GDD_STEP_CONVERGE 1
#define GDD_STEP_NORMS_VALID 2
size_t gdd_minibatch_state_bytes(void);
size_t gdd_minibatch_step_ws_bytes(int64_t b, int k);
int gdd_minibatch_step(int64_t b, int dim, const float* X, const int64_t* rows, int k,
                       const float* C_old, float* C_new, float* weight_sums, int32_t* labels,
                       int step_i, int64_t n_samples, int max_no_improvement, int flags,
                       void* state, void* ws, size_t ws_bytes, gdd_stream_t stream);
int gdd_minibatch_converge(int64_t b, int k, int step_i, int64_t n_samples, int max_no_improvement,
                           void* state, void* ws, size_t ws_bytes, gdd_stream_t stream);

/* numpy legacy RandomState state: ('MT19937', key[624], pos, has_gauss, cached_gaussian).          */
typedef struct gdd_mt_state {
  uint32_t key[624];
  int32_t pos;
  int32_t has_gauss;
  double gauss;
} gdd_mt_state;

/* MiniBatchKMeans(n_clusters=k, batch_size, max_iter, max_no_improvement (-1 = None),              */
/* reassignment_ratio, init_size, n_init).fit(X) in one call (sklearn/cluster/_kmeans.py:2046-2200):  */
/* validation/init subsets, k-means++ seeding, the step loop with reassignment and early stopping,   */
/* and (compute_labels) the final labels pass + inertia. `rng` is the caller's RandomState, advanced */
/* exactly as scikit-learn advances it. argsort_cb must reproduce np.argsort(weight_sums); it is    */
/* only called when more than batch/2 centres are due for reassignment (possible only if k > b/2).   */
/* Host syncs: one per reassignment step and one at the end. centers_out k x dim, labels_out n,      */
/* inertia_out (device): compute_labels 1 -> 1 float, the inertia; compute_labels 2 -> n floats, the  */
/* per-sample squared distances (the caller folds them, e.g. on a side stream); n_steps_out, ewa_out  */
/* (nullable) host.                                                                                  */
size_t gdd_minibatch_kmeans_fit_ws_bytes(int64_t n, int dim, int k, int64_t batch_size,
                                         int64_t init_size);
int gdd_minibatch_kmeans_fit(int64_t n, int dim, const float* X, int k, int64_t batch_size,
                             int max_iter, int max_no_improvement, float reassignment_ratio,
                             int64_t init_size, int n_init, int compute_labels, void* rng,
                             void (*argsort_cb)(const float*, int64_t, int64_t*), float* centers_out,
                             int32_t* labels_out, float* inertia_out, int64_t* n_steps_out,
                             double* ewa_out, void* ws, size_t ws_bytes, void* host_ws,
                             size_t host_ws_bytes, gdd_stream_t stream);
/* pinned host staging the fit needs (host_ws: page-locked, caller-owned, e.g. a pinned torch tensor) */
size_t gdd_minibatch_kmeans_fit_host_ws_bytes(int64_t n, int k, int64_t batch_size, int64_t init_size);

/* Host-only numpy-legacy draws used by the native loops (exposed for parity tests):                */
/* randint(low, high, count) (int64), random_sample(count), permutation(n), and                      */
/* choice(n, p=w/w.sum()) for unit fp32 weights. `state` is a gdd_mt_state, advanced in place.       */
int gdd_rng_randint(void* state, int64_t low, int64_t high, int64_t count, int64_t* out);
int gdd_rng_random_sample(void* state, int64_t count, double* out);
int gdd_rng_permutation(void* state, int64_t n, int64_t* out);
int gdd_rng_choice_unit_weights(void* state, int64_t n, int64_t* out);

/* Stable grouping of samples by label: perm[offsets[c] .. offsets[c+1]) lists the samples of        */
/* cluster c in ascending sample order; counts[c] = offsets[c+1]-offsets[c]. Labels outside [0, k)    */
/* belong to no cluster (offsets[k] counts the others), as in the reference's `labels == i` loop.     */
size_t gdd_group_ws_bytes(int64_t n, int k);
int gdd_group_by_label(int64_t n, const int32_t* labels, int k, int32_t* perm, int32_t* offsets,
                       void* ws, size_t ws_bytes, gdd_stream_t stream);

/* Lloyd M-step accumulation, sklearn lloyd_iter_chunked_dense with one OpenMP thread                */
/* (_k_means_lloyd.pyx:111-160, 208-213): sums[c,:] = sequential fp32 sum over the samples of c in    */
/* sample order of X_i*w_i, wsum[c] = sequential fp32 sum of w_i.  Uses gdd_group_by_label output.    */
int gdd_segment_sum_f32(int64_t n, int dim, const float* X, const float* w, const int32_t* perm,
                        const int32_t* offsets, int k, float* sums, float* wsum, gdd_stream_t stream);

/* The same sums for clusters [c0, c1) only, written as a slice (row c - c0): the cluster-partitioned */
/* M-step of the multi-GPU Lloyd loop (gdd/sharded.py), bit-identical to the full call's rows.        */
int gdd_segment_sum_f32_part(int64_t n, int dim, const float* X, const float* w, const int32_t* perm,
                             const int32_t* offsets, int k, int c0, int c1, float* sums_part,
                             float* wsum_part, gdd_stream_t stream);

/* sklearn _average_centers (_k_means_common.pyx:215-236): w>0: C[c,:] *= fp32(1.0/(double)w);       */
/* w==0: C[c,:] = C[argmax(w),:] (first maximum; averaged already iff argmax < c, sklearn's loop     */
/* order). Then center_shift[c] = sqrt(||C_new[c]-C_old[c]||^2) in the          */
/* _euclidean_dense_dense order (_center_shift :239-251).                                           */
int gdd_average_centers(int k, int dim, float* C_new, const float* wsum, const float* C_old,
                        float* center_shift, gdd_stream_t stream);

/* Per-sample squared distance to a given center: out[i] = ||X[i] - C[labels[i]]||^2 in the          */
/* _euclidean_dense_dense order; with the final labels this is the per-sample term of sklearn        */
/* _inertia_dense (_k_means_common.pyx:92-121) used after the last Lloyd iteration.                  */
int gdd_point_center_sqdist(int64_t n, int dim, const float* X, const int32_t* labels,
                            const float* C, float* out, gdd_stream_t stream);

/* Relocation input of _relocate_empty_clusters_dense (_k_means_common.pyx:124-164):               */
/* out[i] = ((X[i] - C[labels[i]])**2).sum() in numpy's pairwise order over the row (fp32).           */
int gdd_relocate_distances(int64_t n, int dim, const float* X, const int32_t* labels,
                           const float* C, float* out, gdd_stream_t stream);

/* The device-resident Lloyd loop of sklearn _kmeans_single_lloyd (sklearn/cluster/_kmeans.py:       */
/* 690-735), replacing the per-iteration host loop of the reference's KMeans.fit call sites          */
/* (clustgdd_agent_transduct.py:104-105, clustgdd_agent_induct.py:133-134, distill_recsys.py:178).   */
/* Iteration i reads centres C[i%2] (C0/C1) and writes C[(i+1)%2]: labels (MFMA assignment), the     */
/* ordered M-step, _average_centers, _center_shift, strict convergence (labels == labels_old), then */
/* sum(shift^2) <= tol. Runs iterations it0.. until a stop or max_iter; chunks of iterations are    */
/* enqueued ahead of the decision (later kernels no-op through `state`). Returns *out_reason:       */
/* 0 max_iter, 1 strict, 2 tol, 3 an empty cluster needs _relocate_empty_clusters at iteration      */
/* *out_done (the caller relocates on C[(i+1)%2]/wsum, then calls again with it0=i, resume=1).      */
/* Otherwise *out_done = iterations completed. labels_old starts as -1 (the caller fills it).      */
/* state: gdd_lloyd_state_bytes() of device memory; host_ws: pinned, gdd_kmeans_lloyd_host_ws_bytes. */
/* For dim <= 48 with every centre in one LDS chunk, the E-step is bounded: a row whose Hamerly      */
/* bounds, widened by the fp32 rounding margin, prove sklearn's argmin keeps its label skips the     */
/* distance pass (labels identical; the workspace holds the bounds; GDD_LLOYD_PRUNE=0 disables).     */
size_t gdd_lloyd_state_bytes(void);
size_t gdd_kmeans_lloyd_ws_bytes(int64_t n, int dim, int k);
size_t gdd_kmeans_lloyd_host_ws_bytes(void);
int gdd_kmeans_lloyd_run(int64_t n, int dim, const float* X, int k, float* C0, float* C1,
                         int32_t* labels, int32_t* labels_old, float* wsum, float* shift, int it0,
                         int resume, int max_iter, double tol, void* state, int32_t* out_done,
                         int32_t* out_reason, void* ws, size_t ws_bytes, void* host_ws,
                         size_t host_ws_bytes, gdd_stream_t stream);

/* One iteration of the same loop in three phases, for a process group over the GPUs of a node      */
/* (gdd.sharded.ShardedKMeans): rank r runs the E-step (bounded as above) on its rows [r0, r1) and   */
/* the ordered M-step fold on its feature columns [f0, f1) of every cluster; between the phases the  */
/* caller all-gathers the labels and the column slices (RCCL, stream-ordered), and every rank runs  */
/* the same update. ws: gdd_kmeans_lloyd_ws_bytes(n, dim, k), kept across iterations (it holds the   */
/* rows' bounds); state as above, its stop word gating every kernel (iteration `it` = steps 2it and */
/* 2it+1), so chunks of iterations can be enqueued ahead of the host's read of the state.           */
/* gdd_lloyd_estep: labels[r0:r1) for centres C (shift: the previous update's, unless `first` — the */
/* first E-step of a fit or after a relocation, which sets the rows' bounds).                        */
/* gdd_lloyd_mstep: groups the full labels, sums_cols = k x (f1-f0) column sums, wsum = k weights,    */
/* then the empty-cluster check (reason 3).                                                          */
/* gdd_lloyd_update: C_new = the column slices in `parts` (slot r of k*fw floats: rank r's columns   */
/* [r*fw, min(dim, (r+1)*fw)) as a row-major k x w_r block; parts NULL: C_new already holds the      */
/* sums), _average_centers,                                                                          */
/* _center_shift, the labels-changed flag and the convergence test.                                  */
int gdd_lloyd_estep(int64_t n, int64_t r0, int64_t r1, int dim, const float* X, int k, const float* C,
                    const float* shift, int first, int32_t* labels, void* state, int it, void* ws,
                    size_t ws_bytes, gdd_stream_t stream);
int gdd_lloyd_mstep(int64_t n, int dim, const float* X, const int32_t* labels, int k, int f0, int f1,
                    float* sums_cols, float* wsum, void* state, int it, void* ws, size_t ws_bytes,
                    gdd_stream_t stream);
int gdd_lloyd_update(int64_t n, int dim, int k, const float* parts, int fw, float* C_new,
                     const float* wsum, const float* C_old, float* shift, const int32_t* labels,
                     int32_t* labels_old, double tol, void* state, int it, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* Greedy k-means++ seeding, sklearn _kmeans_plusplus (sklearn/cluster/_kmeans.py:174-272) on the    */
/* device. Host supplies the reference RNG draws: first_id (random_state.choice) and                 */
/* uniforms[(k-1) * n_trials] (random_state.uniform(size=n_trials) per center, concatenated).        */
/* Distances: fp64 upcast -2<x_c,x> + |x_c|^2 + |x|^2, stored fp32, clipped at 0 (pairwise.py:582-650), */
/* in OpenBLAS's per-shape summation orders (gdd_skl_sqdist). Potentials: the first as sdot, the     */
/* trials' as sgemv_t (_kmeans.py:239-251). Writes centers (k x dim) and indices. 1 <= n_trials <= 16. */
/* ---------------------------------------------------------------------------------------------- */
size_t gdd_kmeans_plusplus_ws_bytes(int64_t n, int dim, int n_trials);  /* bound for every k <= n */
/* the workspace for this k: the n x n distance tables only where they are built (the multi-block  */
/* table when (k - 1) 2.5e7 >= n^2 dim, i.e. when the rounds it saves cover its one-off build)      */
size_t gdd_kmeans_plusplus_ws_bytes_k(int64_t n, int dim, int n_trials, int k);
int gdd_kmeans_plusplus(int64_t n, int dim, const float* X, const float* w, int k, int n_trials,
                        int64_t first_id, const double* uniforms, float* centers, int64_t* indices,
                        void* ws, size_t ws_bytes, gdd_stream_t stream);

/* sklearn.metrics.pairwise._euclidean_distances(C, X, squared=True) for fp32 C (n_rows x dim) and X  */
/* (n x dim), as scikit-learn 1.7.2 computes it for k-means++ (_kmeans.py:229, 245): X in chunks of   */
/* batch_size rows upcast to fp64, numpy einsum norms, the OpenBLAS 0.3.29 SkylakeX summation order of */
/* each chunk's product, fp32, max(., 0). out: n_rows x n. Device pointers.                            */
int gdd_skl_sqdist(int n_rows, const float* C, int64_t n, int dim, const float* X, float* out,
                   gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (a8) StandardScaler(with_mean=True, with_std=True).fit_transform(X) on fp32 X                    */
/* Replaces the scaling step of distill_recsys.kmeans_cluster (distill_recsys.py:172), scikit-learn  */
/* 1.7.2 semantics (preprocessing/_data.py partial_fit/transform, utils/extmath.py                  */
/* _incremental_mean_and_var): fp64 column sums in row order, corrected two-pass variance,          */
/* near-constant columns scaled by 1, X_out = fp32(fp32(x - mean) / scale). mean/scale: dim doubles. */
/* ---------------------------------------------------------------------------------------------- */
int gdd_standard_scaler(int64_t n, int dim, const float* X, float* X_out, double* mean,
                        double* scale, gdd_stream_t stream);
/* KMeans.fit's centring (sklearn/cluster/_kmeans.py:1476-1487, _tolerance :279-288): mean = X.mean(0), */
/* var = X.var(0) (numpy: sequential fp32 column sums over the rows, quotient by n rounded to fp32), */
/* X_out = X - mean (fp32). mean/var: dim floats. X_out may not alias X.                           */
int gdd_center_columns(int64_t n, int dim, const float* X, float* X_out, float* mean, float* var,
                       gdd_stream_t stream);
/* The same with a workspace (r05): from 65,536 rows and 2 <= dim <= 256 the column chains run in the   */
/* exact parallel form (gdd_colsum.hip: per-segment transducers of the sequential fp32 sum, signed     */
/* terms); otherwise, or with GDD_CENTER_PAR=0, gdd_center_columns. Same bits either way.              */
size_t gdd_center_columns_ws_bytes(int64_t n, int dim);
int gdd_center_columns_ws(int64_t n, int dim, const float* X, float* X_out, float* mean, float* var,
                          void* ws, size_t ws_bytes, gdd_stream_t stream);
/* StandardScaler.transform with a fitted mean/scale (utils_graphsaint.py:41-44 fits on the train   */
/* rows and transforms every row): X_out = fp32(fp32(x - mean) / scale).                            */
int gdd_standard_scaler_transform(int64_t n, int dim, const float* X, const double* mean,
                                  const double* scale, float* X_out, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (a7) cluster-feature mean. Replaces clustgdd_agent_transduct.py:116-127 (induct :143-154) and the  */
/* teacher index_add_/bincount means of distill_recsys.py:623-636.                                   */
/* feat_syn[c,:] = fp32( (sequential fp64 sum over members of c in sample order) / count_c );         */
/* count_c == 0 -> NaN row (reference: mean of an empty selection) unless empty_as_zero != 0          */
/* (distill_recsys clamp_min(1) semantics -> zero row). counts: int64 per cluster.                   */
/* ---------------------------------------------------------------------------------------------- */
int gdd_cluster_mean(int64_t n, int d, const float* feat, const int32_t* perm, const int32_t* offsets,
                     int k, int empty_as_zero, float* feat_syn, long long* counts,
                     gdd_stream_t stream);
/* gdd_cluster_mean for clusters [c0, c1) only, written as a slice (row c - c0): the cluster-         */
/* partitioned cluster mean of the multi-GPU path, bit-identical to the full call's rows.             */
int gdd_cluster_mean_part(int64_t n, int d, const float* feat, const int32_t* perm,
                          const int32_t* offsets, int k, int c0, int c1, int empty_as_zero,
                          float* feat_part, long long* counts_part, gdd_stream_t stream);
/* labels_syn[c] = argmax_j centers[c,j] (first max wins, torch.argmax; transduct:126).              */
int gdd_argmax_rows(int k, int dim, const float* centers, int64_t* out, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (f1/f2) graph condensation: ClustGDD.graph_sparse + ClustGDD.graph_compress                      */
/* (clustgdd_agent_transduct.py:131-250, induct:156-274) and the effective-resistance estimators    */
/* of utils_clustgdd.py:149-182. Edges are the entries of a canonical CSR; rows[e] is each entry's */
/* row (gdd_coo_rows). Orders restated bit for bit by oracle/condense.py.                           */
/* ---------------------------------------------------------------------------------------------- */
int gdd_coo_rows(int64_t n, const int32_t* rowptr, int32_t* rows, gdd_stream_t stream);
size_t gdd_er_ws_bytes(int64_t n, int C);
/* attaw_ER_estimator (utils_clustgdd.py:162-182): rew[e] = val[e] * cos(ebd[src], ebd[dst])         */
/* (ebd: n x C logits), deg = row sums of rew (CSR order), er[e] = rew/deg[src] + rew/deg[dst].     */
int gdd_attaw_er(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* rows,
                 const int32_t* col, const float* val, int C, const float* ebd, float* rew, float* er,
                 void* ws, size_t ws_bytes, gdd_stream_t stream);
/* ER_estimator (utils_clustgdd.py:149-159): the same bound on val (NULL = binary).                 */
int gdd_vanilla_er(int64_t n, int64_t nnz, const int32_t* rowptr, const int32_t* rows,
                   const int32_t* col, const float* val, float* er, void* ws, size_t ws_bytes,
                   gdd_stream_t stream);
/* F.softmax(x, dim=-1) on n x C rows (e = fp32(exp(double(x - max))), sequential sum, e / sum).     */
int gdd_softmax_rows(int64_t n, int C, const float* x, float* p, gdd_stream_t stream);
size_t gdd_topk_ws_bytes(int64_t nnz, int nsets);
/* torch.topk(weight, m) per set, as the ascending edge ids of the m largest (NaN largest, ties to   */
/* the lower id): probs (n x nsets) given -> set i weighs edge e by (probs[src,i]*probs[dst,i])*er  */
/* (graph_sparse 'attaw', :154-182); probs NULL -> one set weighed by er ('vanilla'/'single').      */
/* sel: nsets x m int32.                                                                             */
int gdd_class_topk(int64_t nnz, const int32_t* rows, const int32_t* col, const float* er, int nsets,
                   const float* probs, int64_t m, int32_t* sel, void* ws, size_t ws_bytes,
                   gdd_stream_t stream);
size_t gdd_compress_ws_bytes(int kk);
/* graph_compress (:234-250) for one edge set (all m edges, or the m edge ids in sel):               */
/* out (kk x kk) = P^T A P with P = onehot(labels)/cluster sizes, diagonal removed; an empty        */
/* cluster gives a NaN row and column (the reference's 0/0 column of P). kk = max label + 1.        */
int gdd_graph_compress(int64_t n, const int32_t* labels, int kk, int64_t m, const int32_t* rows,
                       const int32_t* col, const float* val, const int32_t* sel, float* out, void* ws,
                       size_t ws_bytes, gdd_stream_t stream);
size_t gdd_select_csr_ws_bytes(int64_t n);
/* the selected edges (ascending ids, so already in CSR order) as a CSR: rowptr_out n+1, col/val m. */
int gdd_select_csr(int64_t n, const int32_t* rows, const int32_t* col, const float* val, int64_t m,
                   const int32_t* sel, int32_t* rowptr_out, int32_t* col_out, float* val_out, void* ws,
                   size_t ws_bytes, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* induced sub-graph adj_full[np.ix_(idx, idx)] as canonical CSR (utils_graphsaint.py:34-36; the   */
/* inductive agent's train/val/test graphs, clustgdd_agent_induct.py:38-94). idx: m strictly        */
/* increasing node ids. Two calls: _count writes rowptr_out (m+1; nnz_out = rowptr_out[m], read by  */
/* the caller to size col/val), _fill writes col_out / val_out (val_out NULL: binary) and copies a  */
/* flag (nonzero if idx was not strictly increasing or out of range) to bad_out (device, nullable). */
/* Both calls share one workspace (gdd_subgraph_ws_bytes), which _count fills and _fill reads.      */
/* ---------------------------------------------------------------------------------------------- */
size_t gdd_subgraph_ws_bytes(int64_t n, int64_t m);
int gdd_subgraph_count(int64_t n, const int32_t* rowptr, const int32_t* col, int64_t m,
                       const int32_t* idx, int32_t* rowptr_out, void* ws, size_t ws_bytes,
                       gdd_stream_t stream);
int gdd_subgraph_fill(int64_t n, const int32_t* rowptr, const int32_t* col, const float* val, int64_t m,
                      const int32_t* idx, const int32_t* rowptr_out, int32_t* col_out, float* val_out,
                      int32_t* bad_out, void* ws, size_t ws_bytes, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* CSR transpose Aᵀ of an n x n_cols matrix (output n_cols x n, canonical: each row's entries by    */
/* ascending column). The backward of the GCN evaluator's SpMM (models/gcn.py:36-51, d(A @ S)/dS =  */
/* Aᵀ @ grad) and the item side of the recommender's bipartite propagation (distill_recsys.py        */
/* :336-346). val may be NULL (binary: val_t gets 1.0f); val_t may be NULL (structure only);         */
/* perm_out (nullable, nnz) receives the source entry of every transposed entry, so callers whose    */
/* values change (learned edge weights) re-gather val_t = val[perm] without re-sorting.              */
/* ---------------------------------------------------------------------------------------------- */
size_t gdd_csr_transpose_ws_bytes(int64_t n, int64_t n_cols, int64_t nnz);
int gdd_csr_transpose(int64_t n, int64_t n_cols, int64_t nnz, const int32_t* rowptr, const int32_t* col,
                      const float* val, int32_t* rowptr_t, int32_t* col_t, float* val_t, int32_t* perm_out,
                      void* ws, size_t ws_bytes, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (f4) recommender condensation. build_condensed_bipartite (distill_recsys.py:184-201): the       */
/* interactions (train_u[e], train_i[e]) become super-node pairs (u2cu[u], i2ci[i]); the output is   */
/* the num_cu x num_ci matrix of pair counts as canonical CSR (what scipy's coo -> sum_duplicates -> */
/* tocsr gives): rowptr_out (num_cu+1), col_out / val_out with capacity E, the stored count written */
/* to nnz_out (device int). bad_out (device, nullable): nonzero if an id was out of range.          */
/* gdd_edge_dots: out[e] = sum_f a[ra[e],f] * b[rb[e],f] (fp32 fma chain, f ascending) - the edge   */
/* gradient of the LightGCN message passing (RecsysModel.propagate, :336-346). a has na rows, b nb:   */
/* an out-of-range row id is not read (out[e] = NaN) and sets *bad (device int, nullable).           */
/* ---------------------------------------------------------------------------------------------- */
size_t gdd_bipartite_condense_ws_bytes(int64_t E, int num_cu);
int gdd_bipartite_condense(int64_t E, const int32_t* train_u, const int32_t* train_i, int64_t num_users,
                           int64_t num_items, const int32_t* u2cu, const int32_t* i2ci, int num_cu,
                           int num_ci, int32_t* rowptr_out, int32_t* col_out, float* val_out,
                           int32_t* nnz_out, int32_t* bad_out, void* ws, size_t ws_bytes,
                           gdd_stream_t stream);
int gdd_edge_dots(int64_t E, int d, const int32_t* ra, const float* a, int64_t na, const int32_t* rb,
                  const float* b, int64_t nb, float* out, int32_t* bad, gdd_stream_t stream);

/* ---------------------------------------------------------------------------------------------- */
/* (f4) the recommender's refinement loop (distill_recsys.py:641-733).                              */
/* gdd_bpr_sample replaces sample_bpr_triplets_from_condensed (:217-272): host-only, draws from the  */
/* caller's numpy RandomState (`state`, a gdd_mt_state, advanced in place) in the reference's order; */
/* positive lists are CSR rows (indptr int64 [num_users+1], int32 indices in list order; `sorted`,   */
/* nullable, the rows sorted for the membership test when `indices` is not). u/pos/neg: batch.      */
/* gdd_recall_at_k replaces recall_at_k's masking, torch.topk and hit count (:475-497) for B users:   */
/* scores (device, B x I, overwritten), tr_ptr/tr_col their training positives, te_ptr/te_col their   */
/* sorted de-duplicated test items (device CSR, B rows); hits (device u64) += |top-k ∩ test|. Equal  */
/* scores rank in ascending item order; k <= 256.                                                    */
/* ---------------------------------------------------------------------------------------------- */
int gdd_bpr_sample(const int64_t* indptr, const int32_t* indices, const int32_t* sorted,
                   int64_t num_users, int64_t num_items, int64_t batch, void* state, int64_t* u_out,
                   int64_t* pos_out, int64_t* neg_out);
int gdd_recall_at_k(int B, int64_t I, int k, float* scores, const int32_t* tr_ptr, const int32_t* tr_col,
                    const int32_t* te_ptr, const int32_t* te_col, unsigned long long* hits,
                    gdd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GDD_H_ */
