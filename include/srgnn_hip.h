/*
 * srgnn_hip.h -- C-ABI of libsrgnn_hip.so, the MI355X (gfx950) implementation of the spectral
 * feature-propagation hot path of yyysyyy/Scalable-Roubust-GNN.
 *
 * Paths below are relative to "/root/reference/Scalable Spectral Robust GNN/" (SSRG/).
 *
 * Two groups of entry points:
 *
 *  (A) Drop-in replacements with the reference's exact signatures (host pointers, synchronous).
 *      The reference binds them through numpy.ctypeslib in operators/utils.py:17-47 and :49-79;
 *      pointing that load_library call at this library moves the product onto the GPU unchanged.
 *
 *  (B) Device entry points (device pointers, asynchronous on the caller's HIP stream) used by the
 *      device-resident K-hop driver and by the row-partitioned multi-GPU path.
 *
 * Conventions for (B):
 *   - Status: 0 on success, a negative SRG_ERR_* code on failure; srg_last_error() (thread-local)
 *     then holds a message.  Nothing is launched when an argument check fails.
 *   - Ownership: the caller owns every buffer.  The library allocates nothing on these paths.
 *   - CSR: int64 row pointers (nnz may exceed 2^31), int32 column ids, row-major dense panels with
 *     explicit leading dimensions (64-bit element offsets: N*d may exceed 2^31).
 *   - Column ids are trusted on (B): validate a matrix once with srg_csr_validate() before use.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream).  Every launch of an entry
 *     goes to the device `stream` belongs to (the current device for the null stream); the entry
 *     makes that device current for its duration and restores the caller's afterwards.
 *   - Threads: entries may be called concurrently from several host threads.  Hub rows fork onto a
 *     library-owned side stream per (device, caller stream) with its own fork / join events; the
 *     fork sequence is serialised by a library mutex.
 */
#ifndef SRGNN_HIP_H_
#define SRGNN_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------------------------------- */
#define SRG_OK 0
#define SRG_ERR_INVALID (-1)   /* bad argument (shape, null pointer, alignment, out-of-range id) */
#define SRG_ERR_HIP (-2)       /* a HIP runtime call failed */
#define SRG_ERR_ALLOC (-3)     /* device allocation failed (host-compat entries only) */

/* ---- SpMM flags ------------------------------------------------------------------------------ */
/* Default (0): every output element Y[i,c] is ONE sequential fp32 fma chain over row i's nonzeros
 * in stored CSR order, starting from +0.0f -- bit-identical to FloatCSRMulDenseOMP
 * (SSRG/operators/csrc/matmul.c:23-40) given a zeroed answer (SSRG/operators/utils.py:38). */
#define SRG_SPMM_ACCUMULATE 0x1u   /* chains start from Y's current content (matmul.c contract) */
#define SRG_SPMM_NT_STORE 0x2u     /* non-temporal stores of Y */
/* Diagnostic: one light row per wave.  By default d <= 32 runs 64 / S rows per wave (S = the power
 * of two >= d lanes per row), and d = 64 / 128 / 256 runs 512 / d light rows per wave (two 16-byte
 * column chunks per lane).  Results are identical either way. */
#define SRG_SPMM_WIDE_ROWS 0x4
/* Diagnostic: hub workgroups always use 256-nonzero windows (72 KB of LDS, two per CU).  By default
 * they do only when a launch has more hub workgroups than CUs.  Results are identical either way. */
#define SRG_SPMM_HUB_W256 0x8
/* The hub rows' workgroups are forked onto the library's hub side stream of (device, `stream`) and
 * NOT joined back into `stream` before the call returns: later launches on `stream` run beside
 * them (srgnn/dist.py issues the halo row chunks there).  The caller must srg_hub_join(stream)
 * before anything reads the hub rows, and before the next NOJOIN fork from the same stream (one
 * outstanding fork per caller stream). */
#define SRG_SPMM_HUB_NOJOIN 0x10u
/* Packed light rows keep 2 gathers per row in flight instead of 4: better for the short rows of a
 * column block (srgnn.spmm.hop passes it for column-blocked hops; products 7.15 -> 7.01 ms per hop),
 * worse for whole rows.  Results are identical either way. */
#define SRG_SPMM_PACKED_U2 0x20u
/* With SRG_SPMM_HUB_NOJOIN, after an unjoined NOJOIN fork from the same stream: the hub rows'
 * workgroups are appended to the hub side stream without a new fork from `stream` (and without
 * the dispatch delay).  For the column blocks of one hop: X is unchanged during the hop and only
 * the side stream touches the hub rows, so block b's hub span needs no order against block b-1's
 * main launch -- only against block b-1's hub span, which the side stream gives.  One join at the
 * end of the hop.  Without a pending fork it is an ordinary fork.  Results are identical.
 * The pending state belongs to the (device, stream handle) pair: join (srg_hub_join) a stream with
 * an unjoined NOJOIN fork before destroying it, or a new stream that reuses the handle value would
 * inherit the pending fork and its first CONTINUE launch would skip its own fork. */
#define SRG_SPMM_HUB_CONTINUE 0x80u
/* Tolerance mode (EXACT, FAST, ACCUMULATE).  The hub rows (the first n_hub of
 * row_order) are not one chain each: a hub row's entries are cut into 64 consecutive segments,
 * each an exact fp32 fma chain in CSR order (slice waves of the span kernel, into a scratch panel
 * taken from the stream-ordered pool with hipMallocAsync / hipFreeAsync on the hub side stream),
 * and the 64 partial sums are added in segment order (from Y's content with ACCUMULATE).  Results
 * are deterministic and within fp32 re-association error of the reference chain (the tests hold
 * them to the forward-error bound and 1e-5 relative); every other row is bit-exact.  The longest
 * row's latency drops ~64-fold: the straggler of a row-partitioned hop.  Plain and span entries
 * only (the aggregation / send / Chebyshev epilogues run exact).
 * DIAGNOSTIC / tolerance studies only: no configuration measured so far gains from it (one GPU:
 * the top row's exact chain runs beside the hop; 8 ranks: the hub group is bound by its share of
 * HBM beside the chunks, not by the top row's chain -- 1.09-1.11 ms per hop against 1.05-1.08
 * exact), so no default path sets it. */
#define SRG_SPMM_FAST 0x40u
/* The row kernel's launch reserves LDS so that at most 5 of its 4-wave blocks share a CU (gfx950's
 * 160 KiB of LDS per CU): fewer rows gather at once and the L2 re-serves more of
 * the lines they re-read.  For panels far beyond the caches (srgnn.spmm passes it for hops over
 * panels of >= 512 MiB): products 5.84 -> 5.81 ms per hop; arxiv's 87 MB panel is 3 % faster without.
 * Results are identical either way. */
#define SRG_SPMM_CAP_WAVES 0x200u

/* =============================================================================================
 * (A) drop-in entry points
 * ============================================================================================= */

/* Replaces FloatCSRMulDenseOMP, declared at SSRG/operators/csrc/matmul.h:5, defined at
 * SSRG/operators/csrc/matmul.c:23-40, bound at SSRG/operators/utils.py:34-45.
 * answer[mat_row*mat_col] += A * mat, A = CSR(data, indices, indptr) with mat_row rows; the
 * reference's caller passes a zeroed answer.  Host pointers; the product runs on the current HIP
 * device; returns after the result is back in `answer`.  The reference returns nothing and checks
 * nothing; here a failed check or HIP error leaves `answer` untouched and is reported through
 * srg_last_error_code()/srg_last_error(). */
void FloatCSRMulDenseOMP(float answer[], float data[], int indices[], int indptr[], float mat[],
                         int mat_row, int mat_col);

/* Replaces FloatCSRMulDense, SSRG/operators/csrc/cudamatmul.c:28-146 (declared void at
 * cudamatmul.h:4, defined int), bound at SSRG/operators/utils.py:65-77 (cuSPARSE CSR_ALG2 SpMM,
 * alpha = 1, beta = 0).  Overwrites answer with A * mat.  Returns 0 (EXIT_SUCCESS) or 1. */
int FloatCSRMulDense(float answer[], int data_nnz, float data[], int indices[], int indptr[],
                     float mat[], int mat_row, int mat_col);

/* =============================================================================================
 * (B) device entry points
 * ============================================================================================= */

/* One hop: Y[r,:] = A[r,:] * X for the local rows r in [0, n_rows).
 *   indptr[n_rows+1] int64, indices[nnz] int32 (ids into X's rows), values[nnz] fp32;
 *   row_order: optional (NULL) int32 permutation of [0, n_rows) giving the order in which rows are
 *              scheduled (srgnn plans pass rows by decreasing length so hubs start first);
 *   n_hub:     the first n_hub rows of row_order are hub rows: one workgroup per 32-column slice
 *              with producer waves keeping 64 KiB of gathers in flight (launched on a library-owned
 *              side stream, forked from and joined back into `stream` with events);
 *   n_heavy:   the next n_heavy rows are worked on in 32-column slices, one wave per slice (long
 *              power-law rows); both 0 without a row_order.
 *   Neither scheduling argument changes any result: every output element is one fma chain.
 *   X: ldx >= d; Y: ldy >= d.  Device pointers.  Replaces one call of csr_sparse_dense_matmul
 *   (SSRG/operators/utils.py:17-47) inside GraphOp.propagate (SSRG/operators/base_operator.py:33-35). */
int srg_spmm_csr_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                     int64_t n_rows, const int32_t* row_order, int64_t n_hub, int64_t n_heavy,
                     const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d, uint32_t flags,
                     void* stream);

/* K hops: panels[k] = A * panels[k-1] for k = 1..K, panels[0] = X (read only).  `panels` is a
 * HOST array of K+1 device pointers, all with leading dimension ld.  Replaces the hop loop of
 * GraphOp.propagate, SSRG/operators/base_operator.py:32-35 (with the per-hop host round trips of
 * utils.py:38-47 removed).  A square (n_rows == rows of X).  Given no schedule (row_order NULL,
 * n_hub = n_heavy = 0) and flags within NT_STORE | FAST, the hops run through a plan built for them
 * (srg_plan_build with automatic choices -- no hub rows under FAST, so FAST changes no bit there, as
 * before the planner -- released after the hops; the call then synchronises `stream` while it plans
 * and releases, and allocates the plan's memory for its duration, so it cannot be captured into a HIP
 * graph); with a schedule, or other flags, every hop is one launch over the caller's CSR (capturable). */
int srg_propagate_khop_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                           int64_t n_rows, const int32_t* row_order, int64_t n_hub,
                           int64_t n_heavy, float* const* panels,
                           int64_t ld, int32_t d, int32_t K, uint32_t flags, void* stream);

/* One launch of a column-blocked hop, as srgnn.csr.DeviceCSR holds a column block (or block 0's two
 * parts): a CSR over the row space (row_end == NULL: row_beg has row_space + 1 entries) or row spans of
 * a shared CSR (row_end != NULL: row r's entries are [row_beg[r], row_end[r])), the schedule
 * (row_order: n_rows row ids, the first n_hub hub rows, then n_heavy slice-wave rows) and the launch's
 * SRG_SPMM_* flags (ACCUMULATE for blocks 1.., PACKED_U2, HUB_NOJOIN / HUB_CONTINUE for chained hub
 * spans, NT_STORE, FAST). */
typedef struct srg_hop_launch {
    const int64_t* row_beg;
    const int64_t* row_end;
    const int32_t* indices;
    const float* values;
    const int32_t* row_order;
    int64_t n_rows;
    int64_t n_hub;
    int64_t n_heavy;
    uint32_t flags;
    /* optional (row_end != NULL only): the spans by schedule slot, slot_beg[i] / slot_end[i] = the span
     * of row row_order[i] (n_rows entries each, or both NULL): the packed light rows read these,
     * so consecutive slots read consecutive addresses */
    const int64_t* slot_beg;
    const int64_t* slot_end;
} srg_hop_launch;

/* K column-blocked hops: for k = 1..K, the n_launch launches of `launches` (a HOST array) run in
 * order with X = panels[k-1], Y = panels[k]; with join_hub, the hub side stream (forked by the
 * first HUB_NOJOIN launch of the hop) is joined back into `stream` at the end of every hop.  The
 * device-resident form of srgnn.spmm.propagate's blocked hop loop: bitwise the one-launch hops
 * (the same fma chains, continued across the blocks).  panels: HOST array of K+1 device pointers
 * of leading dimension ld.  A plan with HUB_NOJOIN launches over K > 1 hops needs join_hub (else
 * SRG_ERR_INVALID: hop k+1 would read hub rows still being written); with join_hub = 0 (K = 1) the
 * caller must srg_hub_join(stream) after the call, before anything reads the hub rows. */
int srg_propagate_plan_f32(const srg_hop_launch* launches, int32_t n_launch, int32_t join_hub,
                           float* const* panels, int64_t ld, int32_t d, int32_t K, void* stream);

/* ---- the one-GPU planner (csrc/srg_plan.hip) ------------------------------------------------------
 * The layout of a square operator for a run of `hops` hops over d-column panels, built on the device:
 * column blocks as row spans (col_blocks: 0 = automatic -- 12..16 blocks, one per ~100 MiB, for panels
 * of 512 MiB .. 16 GiB at d >= 64 and runs of >= 4 hops, 4 for larger panels, else 1), block 0 as its cut rows' spans and its whole rows (rows of
 * <= 48 entries), per-launch schedules by decreasing span length with their hub / slice-wave counts,
 * the hub spans chained on the side stream, spans by schedule slot and, for runs of at least
 * SRG_PLAN_MIN_HOPS_TO_COMPACT hops when it fits in a quarter of the free memory, compact copies of
 * the ids and values in launch order.  The same layout srgnn.spmm.prepare gives a DeviceCSR (the
 * srgnn package builds its K-hop runs with this planner).  Replaces the reference's per-hop
 * csr_sparse_dense_matmul setup inside GraphOp.propagate (SSRG/operators/base_operator.py:32-35,
 * utils.py:17-47), which re-reads the scipy CSR every hop.
 * Unlike the other (B) entries the plan allocates device memory (hipMalloc: the schedules, the spans
 * by slot, the copies -- srg_plan_describe's device_bytes -- and a scratch arena freed before it
 * returns) and synchronises `stream` while it builds.  The plan BORROWS indptr / indices / values (span
 * layouts read them every hop): they must outlive it.  values may be NULL with SRG_PLAN_SPANS: such a
 * plan serves srg_plan_cheby_step_f64 only (which brings its fp64 values per call).  indptr[n_rows + 1], indices / values
 * [indptr[n_rows] - indptr[0]], column ids in [0, n_rows) (not validated here: srg_csr_validate).
 * hub_threshold / heavy_threshold: SRG_PLAN_AUTO (per launch, from its nnz: hub rows > max(2048,
 * nnz / 1024) entries, slice-wave rows > max(96, nnz / 100000) for the one-launch hop, nnz / 30000 for
 * a column block's), SRG_PLAN_NONE (no such rows) or a row length that holds for every launch, as a
 * DeviceCSR built with explicit thresholds schedules its blocks (srgnn.csr.make_schedule). */
typedef struct srg_plan srg_plan;
#define SRG_PLAN_MIN_HOPS_TO_CUT 4       /* automatic column blocks for runs of at least this many hops */
#define SRG_PLAN_MIN_HOPS_TO_COMPACT 6   /* automatic compact copies (when they fit) from this many */
#define SRG_PLAN_COMPACT 0x1u        /* copy the entries in launch order whatever the run length */
#define SRG_PLAN_SPANS 0x2u          /* never copy: spans of the caller's arrays */
#define SRG_PLAN_SPLIT_BLOCK0 0x4u   /* block 0 as two launches (default: panels < 16 GiB) */
#define SRG_PLAN_WHOLE_BLOCK0 0x8u   /* block 0 as one launch */
#define SRG_PLAN_WHOLE_HUBS 0x10u    /* with an explicit hub_threshold (column-blocked plans): rows longer than it
                                        are whole hub rows -- cut nowhere, one launch of their own first in the
                                        hop -- as SRG_PLAN_AUTO does for rows > max(2048, nnz / 1024) */
#define SRG_PLAN_WHOLE_MAX_SHIFT 16
#define SRG_PLAN_WHOLE_MAX(n) ((uint32_t)(n) << SRG_PLAN_WHOLE_MAX_SHIFT)   /* block 0's whole rows: at most n
                                        entries (1..65535; 0 = the default 48) -- the fp64 steps' partial sums are
                                        1 KB per row per block, so their break-even row length differs */
#define SRG_PLAN_AUTO (-1)
#define SRG_PLAN_NONE (-2)
typedef struct {
    int64_t n_rows, nnz;
    int64_t device_bytes;            /* device memory the plan holds */
    int32_t d;                       /* the panel width it was built for (any width runs it) */
    int32_t col_blocks;              /* column blocks per hop (1: the one-launch hop) */
    int32_t n_launch;                /* k_spmm launches per hop */
    int32_t compact, split_block0, hub_chain;
    int32_t device;
    int32_t hub_rows_whole;          /* rows of the whole hub rows' launch (first in the hop; 0: none) */
} srg_plan_desc;
int srg_plan_build(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows,
                   int32_t d, int32_t hops, int32_t col_blocks, int64_t hub_threshold, int64_t heavy_threshold,
                   uint32_t opts, void* stream, srg_plan** plan);
/* The device memory srg_plan_build would take for these arguments (the ids and values are not read) --
 * keep_bytes for the plan's life,
 * scratch_bytes during the build -- and the choices it would make (resolved_opts: SRG_PLAN_COMPACT or
 * SPANS | SPLIT_BLOCK0 or WHOLE_BLOCK0; resolved_col_blocks).  One pass over indptr (synchronises
 * `stream`); nothing is allocated.  With srg_plan_build_in, a host puts the plan in memory of its own
 * allocator (srgnn: torch's caching allocator, so a plan competes for the same cached blocks as the
 * panels instead of beside them). */
int srg_plan_query(const int64_t* indptr, int64_t n_rows, int32_t d, int32_t hops, int32_t col_blocks,
                   int64_t hub_threshold, int64_t heavy_threshold, uint32_t opts, void* stream, size_t* keep_bytes,
                   size_t* scratch_bytes, uint32_t* resolved_opts, int32_t* resolved_col_blocks);
/* srg_plan_build into the caller's memory: `keep` (>= keep_bytes of srg_plan_query for the same
 * arguments and the resolved opts / col_blocks, 256-byte aligned) holds the plan until srg_plan_destroy
 * returns; `scratch` (>= scratch_bytes) only until this call returns.  The plan never frees either. */
int srg_plan_build_in(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows, int32_t d,
                      int32_t hops, int32_t col_blocks, int64_t hub_threshold, int64_t heavy_threshold, uint32_t opts,
                      void* keep, size_t keep_bytes, void* scratch, size_t scratch_bytes, void* stream,
                      srg_plan** plan);
/* Releases the plan after every reader of its memory.  The plan records, per stream its work was
 * enqueued on (its build, propagates, hops, graph replays, the row-span completion), an event after
 * that work with the hub side stream already joined; destroy makes `stream` wait for all of them,
 * joins the hub side stream of `stream`, drains `stream` (a host synchronisation), destroys the
 * executable graphs and only then frees the memory (srg_plan_build's; srg_plan_build_in's memory may
 * be reused by its owner once destroy returns).  Launches a caller ran itself from srg_plan_launch's
 * descriptors must be ordered before `stream` by the caller.  A plan is used by one host thread at a
 * time (a propagate over a width other than 64 / 128 / 256 completes its row-indexed spans in place;
 * srg_plan_launch does so up front). */
int srg_plan_destroy(srg_plan* plan, void* stream);
int srg_plan_describe(const srg_plan* plan, srg_plan_desc* desc);
/* Launch i of one hop over a d-column panel, as srg_plan_propagate_f32 runs it (flags included), and
 * whether the hops join the hub side stream at their ends: for callers that drive
 * srg_propagate_plan_f32 themselves, and for layout tests.  A compact plan built for a 64 / 128 / 256
 * column panel keeps row-indexed spans for its hub and slice-wave rows only (its light rows read the
 * spans by slot); the first srg_plan_launch call (or a propagate over another width) completes them,
 * enqueued on `stream`. */
int srg_plan_launch(const srg_plan* plan, int32_t i, int32_t d, srg_hop_launch* launch, int32_t* join_hub,
                    void* stream);
/* K hops through the plan: panels[k] = A * panels[k-1], k = 1..K (HOST array of K+1 device pointers
 * of leading dimension ld, d columns; any d, the layout was chosen for the build's d).  flags:
 * SRG_SPMM_NT_STORE, SRG_SPMM_FAST.  Bitwise srg_propagate_khop_f32's hops (FAST: its tolerance).
 * Repeated with the same panels, d, K, flags and a non-null stream, the call replays the K hops as a
 * HIP graph captured on its second occurrence (the same launches and arguments: the same bits). */
int srg_plan_propagate_f32(const srg_plan* plan, float* const* panels, int64_t ld, int32_t d, int32_t K,
                           uint32_t flags, void* stream);
/* One hop through the plan between panels of their own leading dimensions: Y = A * X (X: ldx, Y: ldy,
 * d columns; Y must not alias X) and, when agg is not NULL, the aggregation step fused into the
 * epilogue of the launch where each row's chain ends: agg = (agg_init ? 0 : agg) + w * Y (lda),
 * srg_hop_accumulate_f32's arithmetic, so bitwise the hop followed by that step.  A plan whose block 0
 * is one launch (panels >= 16 GiB) runs the hop, then that step.  flags: SRG_SPMM_NT_STORE,
 * SRG_SPMM_FAST (not with agg).  The aggregating hop of srgnn.aggregate's hop loop: the reference's
 * MessageOp.aggregate -> combine over the hop list (SSRG/operators/base_operator.py:49-59) folded
 * into the hops as they are produced. */
int srg_plan_hop_f32(const srg_plan* plan, const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d,
                     uint32_t flags, float* agg, int64_t lda, float w, int32_t agg_init, void* stream);
/* One fp64 Chebyshev order through the plan: srg_cheby_step_f64's recurrence and epilogue (below), bitwise,
 * with the plan's column blocks -- each block's launch gathers from one column block of Tc and continues
 * every row's chain from the fp64 partial sum the block before stored in Tn; the epilogue runs where the
 * chain ends (block 0's whole rows, the last block) -- and its whole hub rows as hub workgroups on the
 * hub side stream (joined before the call returns to `stream`'s order).  `values`: the operator's fp64
 * values (L for INIT, F for STEP: one plan serves both, the layout depends on indptr / indices only).  The
 * plan must read spans of the caller's arrays (SRG_PLAN_SPANS; its fp32 values may be NULL, the fp32
 * entry points then refuse it) with block 0 as two launches (SRG_PLAN_SPLIT_BLOCK0) when blocked; build it
 * for twice the panel width (the layout is sized by panel bytes).  Replaces pygsp cheby_op's per-order
 * L.dot (SSRG/models/base_scalable/base_model.py:236-265) for graphs whose fp64 panels outgrow the
 * Infinity Cache. */
int srg_plan_cheby_step_f64(const srg_plan* plan, const double* values, const double* Tc, const double* To, double* Tn,
                            int64_t ld, int32_t d, int mode, double a1, double a2, const double* coef_prev,
                            const double* coef, int32_t n_scales, double* R, int64_t r_stride, void* stream);

/* Chebyshev heat-kernel filter bank (wavelet basis), SSRG/models/base_scalable/base_model.py:
 * 184-191, 236-265 via pygsp cheby_op.  One fused launch per Chebyshev order:
 *   mode SRG_CHEBY_INIT (order 1):  Tn = (A*Tc - a2*Tc) / a1;   R_s  = (c0_s/2)*Tc + c1_s*Tn
 *   mode SRG_CHEBY_STEP (order k>=2): Tn = A*Tc - To;           R_s += ck_s*Tn
 * with A = L (combinatorial Laplacian) for INIT and A = F = (2/a1)(L - a2 I) for STEP (the caller
 * builds F's values).  R holds n_scales stacked panels: R + s*r_stride.  coef_prev (c0 per scale,
 * INIT only) and coef (c1 or ck per scale) are HOST arrays of n_scales <= 8 values.  fp64 follows
 * scipy's operation order (separate multiply and add, no fma); fp32 uses fma chains.  The fused steps
 * (srg_cheby_step_*, srg_cheby_step_hub_f64, srg_plan_cheby_step_f64) also take the epilogue's lean modes
 * below (SRG_CHEBY_INIT_T, SRG_CHEBY_STEP_FIRST with coef_prev = c0 then c1 per scale, | SRG_CHEBY_NO_T):
 * the same bits, four panel passes less per order-3 filter. */
#define SRG_CHEBY_INIT 0
#define SRG_CHEBY_STEP 1
int srg_cheby_step_f64(const int64_t* indptr, const int32_t* indices, const double* values,
                       int64_t n_rows, const int32_t* row_order, const double* Tc,
                       const double* To, double* Tn, int64_t ld, int32_t d, int mode, double a1,
                       double a2, const double* coef_prev, const double* coef, int32_t n_scales,
                       double* R, int64_t r_stride, void* stream);
/* srg_cheby_step_f64 with the first n_hub rows of row_order (its longest rows) as hub rows: each runs
 * as workgroups of 16-column slices, 8 waves gathering the row's X pieces into LDS for one wave's
 * chains, on the hub side stream beside the row waves of the other rows (srg_spmm_csr_f32's hub
 * fork; joined into `stream` before the call returns).  Bitwise srg_cheby_step_f64: the same chains
 * in the same order, the same epilogue.  Hub rows need an even d and ld and a 16-byte aligned Tc
 * (otherwise every row is a row wave).  mode | SRG_CHEBY_HUB_NOJOIN leaves the hub rows running (as
 * SRG_SPMM_HUB_NOJOIN): later launches on `stream` run beside them until the caller's srg_hub_join
 * (srgnn/dist.py forks a halo rank's hub group this way, then runs its row chunks).  Only this entry
 * takes the flag. */
#define SRG_CHEBY_HUB_NOJOIN 0x20
int srg_cheby_step_hub_f64(const int64_t* indptr, const int32_t* indices, const double* values,
                           int64_t n_rows, const int32_t* row_order, int64_t n_hub, const double* Tc,
                           const double* To, double* Tn, int64_t ld, int32_t d, int mode, double a1,
                           double a2, const double* coef_prev, const double* coef, int32_t n_scales,
                           double* R, int64_t r_stride, void* stream);
int srg_cheby_step_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                       int64_t n_rows, const int32_t* row_order, const float* Tc, const float* To,
                       float* Tn, int64_t ld, int32_t d, int mode, float a1, float a2,
                       const float* coef_prev, const float* coef, int32_t n_scales, float* R,
                       int64_t r_stride, void* stream);

/* The same Chebyshev order split in two for large graphs: a load-balanced srg_spmm_csr_f32 of
 * Tc into Tn (slice waves and hub workgroups for the high-degree rows), then this element-wise
 * epilogue turning Tn = A*Tc into the next T and updating R -- bit-identical to
 * srg_cheby_step_f32 (same fma chain, same epilogue arithmetic).  Every panel has its own leading
 * dimension (column blocks of S and R without copies); R_s = R + s*r_stride, rows ldr apart. */
/* Two-pass-saving modes of the epilogue (the split path of an order >= 2 filter):
 *   SRG_CHEBY_INIT_T (order 1):     Tn = (A*Tc - a2*Tc) / a1; R untouched (coef unused)
 *   SRG_CHEBY_STEP_FIRST (order 2): Tn = A*Tc - To with To = T0, Tc = T1;
 *                                   R_s = ((c0_s/2)*T0 + c1_s*T1) + c2_s*Tn
 *                                   coef_prev = [c0_0..c0_{ns-1}, c1_0..c1_{ns-1}], coef = c2
 *   | SRG_CHEBY_NO_T (any step):    Tn is not stored (the last order: no later step reads it)
 * INIT_T then STEP_FIRST gives the same bits as INIT then STEP (same operations, same order). */
#define SRG_CHEBY_INIT_T 2
#define SRG_CHEBY_STEP_FIRST 3
#define SRG_CHEBY_NO_T 0x10
int srg_cheby_epilogue_f32(float* Tn, int64_t ldn, const float* Tc, int64_t ldc, const float* To,
                           int64_t ldo, int64_t n_rows, int32_t d, int mode, float a1, float a2,
                           const float* coef_prev, const float* coef, int32_t n_scales, float* R,
                           int64_t ldr, int64_t r_stride, void* stream);

/* The split path's two launches in one: srg_spmm_csr_f32 of Tc into Tn (load-balanced: slice waves,
 * packed light rows, hub workgroups) with srg_cheby_epilogue_f32's arithmetic fused into the
 * store, so Tn receives the next T directly -- bit-identical to the split path.  Tn may be To
 * itself (same leading dimension): every element of T_{k-1} is read by its one owner before it is
 * overwritten, so an order of any depth needs two work panels.  Tn must not alias Tc, R no panel;
 * flags as srg_spmm_csr_f32 without SRG_SPMM_ACCUMULATE.  coef_prev / coef are host arrays. */
int srg_spmm_cheby_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                       int64_t n_rows, const int32_t* row_order, int64_t n_hub, int64_t n_heavy,
                       const float* Tc, int64_t ldc, float* Tn, int64_t ldn, int32_t d, uint32_t flags,
                       int mode, float a1, float a2, const float* To, int64_t ldo, const float* coef_prev,
                       const float* coef, int32_t n_scales, float* R, int64_t ldr, int64_t r_stride,
                       void* stream);

/* Hop aggregation without the K+1 panels (fused precompute of SGC / SSGC / GBP).  The reference
 * combines the hop list on the host (SSRG/operators/message_operator/{sum,mean,simple_weighted}_
 * message_op.py; operators/utils.py:426-437 one_dim_weighted_add); the host side plans the same
 * order of element-wise steps (Python sum(): left to right from +0; torch's CPU dim-0 sum: 16-term
 * blocks folded in levels).  Per element, separate multiply / add / correctly rounded divide:
 *   SRG_ACC_INIT: agg = 0 + w*y     SRG_ACC_ADD: agg = agg + w*y     SRG_ACC_DIV: agg = agg / w
 * agg and y are device panels [n_rows, d] with leading dimensions lda / ldy (y unused for DIV). */
#define SRG_ACC_INIT 0
#define SRG_ACC_ADD 1
#define SRG_ACC_DIV 2
int srg_hop_accumulate_f32(float* agg, int64_t lda, const float* y, int64_t ldy, int64_t n_rows,
                           int32_t d, float w, int mode, void* stream);

/* srg_spmm_csr_f32 with the aggregation step fused into its epilogue: Y = A*X as above and, for
 * every element y stored, agg = (agg_init ? 0 : agg) + w*y (separate multiply / add) -- the same
 * result as srg_spmm_csr_f32 followed by srg_hop_accumulate_f32(INIT or ADD), one panel pass less.
 * agg: device panel [n_rows, d], leading dimension lda, must not alias Y. */
int srg_spmm_agg_f32(const int64_t* indptr, const int32_t* indices, const float* values,
                     int64_t n_rows, const int32_t* row_order, int64_t n_hub, int64_t n_heavy,
                     const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d, uint32_t flags,
                     float* agg, int64_t lda, float w, int agg_init, void* stream);

/* One column block of a hop over ROW SPANS: row r's entries are [row_beg[r], row_end[r]) of the
 * shared indices / values arrays (both int64 [n_rows]), otherwise srg_spmm_csr_f32 (agg == NULL)
 * or srg_spmm_agg_f32 (agg != NULL).  When every row of Â holds sorted column ids (utils.py:81-93
 * builds them so), the entries of row r whose ids fall in a column block are one span of the row,
 * so block b of a hop is this call with row_beg = split_b, row_end = split_{b+1} (split_0 =
 * indptr[0:n], split_B = indptr[1:n+1]): no copy of the ids or values.  Block 0 runs from +0.0f,
 * blocks 1.. with SRG_SPMM_ACCUMULATE continue every chain from the fp32 value the previous block
 * stored -- the same fmas in the same order as the one-launch hop, so the same bits.  row_order /
 * n_hub / n_heavy schedule the spans' lengths.  Replaces one call of csr_sparse_dense_matmul
 * (SSRG/operators/utils.py:17-47) inside GraphOp.propagate's hop loop (base_operator.py:33-35). */
int srg_spmm_span_f32(const int64_t* row_beg, const int64_t* row_end, const int32_t* indices,
                      const float* values, int64_t n_rows, const int32_t* row_order, int64_t n_hub,
                      int64_t n_heavy, const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d,
                      uint32_t flags, float* agg, int64_t lda, float w, int agg_init, void* stream);

/* The last flat elements (< SRG_TAIL_MAX of them) of a torch dim-0 sum take its scalar row_sum
 * order (4 interleaved partials).  srg_tail_record_f32 stores w * y[flat_start + e] (flat index of
 * the row-major [n_rows, d] panel) into hist[e], one call per term with hist advanced by
 * SRG_TAIL_MAX floats; srg_tail_rowsum_f32 then writes 0 + row_sum(hist[0..n_terms)) into agg. */
#define SRG_TAIL_MAX 32
int srg_tail_record_f32(float* hist, const float* y, int64_t ldy, int32_t d, int64_t flat_start,
                        int32_t len, float w, void* stream);
int srg_tail_rowsum_f32(float* agg, int64_t lda, int32_t d, int64_t flat_start, int32_t len,
                        const float* hist, int32_t n_terms, void* stream);

/* construct_adj on the device (SSRG/operators/utils.py:81-93, adj_to_symmetric_norm): out[s] =
 * ((0 + v[p[s]]) + v[p[s]+1]) + ... over vals[seg_ptr[s] .. seg_ptr[s+1]) in fp64, left to right
 * -- the order in which scipy merges duplicate entries of adj + I and sums the rows for the
 * degrees.  seg_ptr has n_seg + 1 entries; all pointers are device pointers. */
int srg_segment_sum_f64(const int64_t* seg_ptr, const double* vals, int64_t n_seg, double* out, void* stream);
/* The same in fp32: the directed families' fp32 normalisations (SSRG/operators/utils.py:195-424:
 * torch_scatter.scatter_add over fp32 edge weights, a sequential sum in element order). */
int srg_segment_sum_f32(const int64_t* seg_ptr, const float* vals, int64_t n_seg, float* out, void* stream);

/* fp64 Y = A * X (X [rows of A's columns, d], ldx; Y [n_rows, d], ldy) in scipy's csr_matvec(s)
 * order (each element from 0, adding the separately rounded product of every stored entry in
 * storage order): the W @ x step of the fast PPR power iteration in
 * adj_to_fast_ppr_approx_symmetric_norm (SSRG/operators/utils.py:284-291) and the stationary
 * distribution of the two-order operator (:338-356).  Not a hop kernel. */
int srg_spmm_csr_f64(const int64_t* indptr, const int32_t* indices, const double* values, int64_t n_rows,
                     const double* X, int64_t ldx, double* Y, int64_t ldy, int32_t d, void* stream);

/* Row gather, the send-side pack of the multi-GPU halo exchange (srgnn/dist.py; no reference
 * counterpart -- the reference is single process): dst[i, :] = src[idx[i], :] for i < n_idx, a C
 * host's pack step before its RCCL sends.  src [n_src, d] / dst [n_idx, d] are device panels with
 * leading dimensions lds / ldd; idx is int64 on the device.  An index outside [0, n_src) leaves its
 * dst row unwritten (no fault).  Asynchronous on `stream`. */
int srg_gather_rows_f32(const float* src, int64_t lds, int64_t n_src, const int64_t* idx, int64_t n_idx,
                        float* dst, int64_t ldd, int32_t d, void* stream);

/* `stream` waits (on the device, not the host) for the hub workgroups of the last hub launch
 * forked from `stream` (an SRG_SPMM_HUB_NOJOIN one); no-op if none was forked. */
int srg_hub_join(void* stream);
/* Diagnostic: the number of live hub side streams over all devices (at most 8 per device; a caller
 * stream's entry is evicted, least recently used first, unless it has an unjoined NOJOIN fork). */
int srg_hub_side_streams(void);

/* Column-block split points of a device CSR for srg_spmm_span_f32 (asynchronous on `stream`):
 * splits[(b-1) * n_rows + r] = the first entry of row r with column id >= ceil(b * n_cols / n_blocks)
 * (binary search over the row's sorted ids), b = 1 .. n_blocks-1; splits: int64 [(n_blocks-1) * n_rows].
 * For any row the split points lie in [indptr[r], indptr[r+1]] and never decrease with b, so the
 * spans partition every row in CSR order and the blocked hop stays exact even for unsorted rows
 * (which only lose the blocks' locality).  n_blocks in [2, 64]. */
int srg_csr_col_splits(const int64_t* indptr, const int32_t* indices, int64_t n_rows, int64_t n_cols,
                       int32_t n_blocks, int64_t* splits, void* stream);

/* Span copy (the compact column blocks of srgnn.csr.DeviceCSR: a launch's entries laid out in the
 * order it takes its rows): for i < n_order, row r = order[i] has its span [beg[r], end[r]) of
 * indices / values copied to [pos[i], pos[i] + end[r] - beg[r]) of out_indices / out_values, and
 * out_beg[r] / out_end[r] set to that range (pos: the exclusive prefix sum of the spans' lengths in
 * `order`; rows not in `order` keep their out_beg / out_end).  Asynchronous on `stream`. */
int srg_csr_copy_spans(const int32_t* order, int64_t n_order, const int64_t* beg, const int64_t* end,
                       const int32_t* indices, const float* values, const int64_t* pos, int32_t* out_indices,
                       float* out_values, int64_t* out_beg, int64_t* out_end, void* stream);

/* Mirror positions (device construct_adj, srgnn/construct.py; SSRG/operators/utils.py:91 transposes
 * A+I): for a CSR whose rows hold strictly increasing column ids, mirror[e] = the position of entry
 * (c, r) in row c for entry e = (r, c) (rows[e] = r, int64 [nnz]), or -1 when row c has no column r.
 * Every entry found <=> the structure is symmetric, and the transpose is then the same structure
 * with values[mirror].  Asynchronous on `stream`. */
int srg_csr_mirror(const int64_t* indptr, const int32_t* indices, const int64_t* rows, int64_t n_rows,
                   int64_t nnz, int64_t* mirror, void* stream);

/* Checks a device CSR: indptr[0] == 0, indptr non-decreasing, indptr[n_rows] == nnz, and every
 * column id in [0, n_cols).  Synchronous on `stream`.  Returns SRG_OK or SRG_ERR_INVALID. */
int srg_csr_validate(const int64_t* indptr, const int32_t* indices, int64_t n_rows,
                     int64_t nnz, int64_t n_cols, void* stream);

/* ---- sparse x sparse: the wavelet model's phi * phi^-1 (torch_sparse.spspmm / spmm) ------------------
 * SpectralModel.preprocess (SSRG/models/base_scalable/base_model.py:208-219) multiplies the two sparse
 * wavelet bases with torch_sparse.spspmm and the product into the features with torch_sparse.spmm
 * (torch_sparse is absent here; its published CPU algorithms, which are scipy csr_matmat's arithmetic,
 * are restated): C[i,j] = ((0 + A[i,k1]*B[k1,j]) + A[i,k2]*B[k2,j]) + ... over row i of A in stored
 * order, each product rounded before it is added; sums equal to 0 dropped; columns ascending.
 * Two passes over the same arguments: phase 0 writes c_cnt[m] (entries per row of C); the caller
 * forms c_ptr (m + 1, exclusive prefix sum) and allocates C; phase 1 fills c_idx / c_val.
 * B with more than 16384 columns needs `scratch` (device, srg_spgemm_scratch_bytes() bytes, or any
 * smaller multiple of one row accumulator: fewer workgroups); B's row pointers index b_idx / b_val,
 * its column ids must be < n_cols.  SRG_SPGEMM_SERIAL_B: B's rows may repeat a column id (then each
 * B row is walked by one lane).  Asynchronous on `stream`. */
#define SRG_SPGEMM_SERIAL_B 0x1u
int srg_spgemm_scratch_bytes(int64_t m, int64_t n_cols, int64_t* bytes);
int srg_spgemm_f32(int phase, const int64_t* a_ptr, const int32_t* a_idx, const float* a_val, int64_t m,
                   const int64_t* b_ptr, const int32_t* b_idx, const float* b_val, int64_t n_cols,
                   int64_t* c_cnt, const int64_t* c_ptr, int32_t* c_idx, float* c_val, void* scratch,
                   int64_t scratch_bytes, uint32_t flags, void* stream);
/* torch_sparse.spmm(index, value, m, n, matrix) (index_select, mul, scatter_add): Y[r, :] = sum over
 * row r's entries in stored order of (v * X[c, :]), each product rounded, then added, from +0.  A CSR
 * whose rows hold the COO entries in index order (a stable sort by row). */
int srg_spmm_muladd_f32(const int64_t* indptr, const int32_t* indices, const float* values, int64_t n_rows,
                        const float* X, int64_t ldx, float* Y, int64_t ldy, int32_t d, void* stream);

/* ---- multi-GPU: communicators and the row-partitioned K-hop propagation ---------------------------
 * SURVEY.md §8(b) item 5, for C / C++ hosts (the Python package drives the same kernels through
 * torch.distributed: srgnn/dist.py).  RCCL is loaded at run time.  Rank r owns rows
 * [row_starts[r], row_starts[r+1]) of Â and of every hop panel.  srg_dist_propagate_khop_f32 is
 * SURVEY §8(e)'s all-gather, chunked by owner and overlapped with the SpMM: per hop every pair of
 * ranks swaps its blocks of the previous panel (grouped ncclSend / ncclRecv on a stream of that
 * pair: all links at once, lower ranks first), and each rank multiplies its rows in P column blocks
 * (block q = the entries whose columns rank q owns: a span of every row, since Â's rows hold sorted
 * ids), in ascending q, block q as soon as rank q's rows have arrived, blocks 1.. continuing the
 * chains (SRG_SPMM_ACCUMULATE).  Every hop is bitwise the one-GPU hop (each row's fma chain is
 * unchanged).  Rows with unsorted column ids are rejected (SRG_ERR_INVALID).  The halo exchange
 * below (srg_halo_*) moves only the referenced rows and is the faster path.  Replaces the
 * reference's single-process hop loop, SSRG/operators/base_operator.py:32-35. */
typedef struct srg_comm srg_comm;
#define SRG_COMM_ID_BYTES 128
/* RCCL unique id (SRG_COMM_ID_BYTES bytes) to share out of band before srg_comm_init_rank. */
int srg_comm_unique_id(void* id_out);
/* One rank per process: `device` is this process's HIP device. */
int srg_comm_init_rank(int nranks, const void* id, int rank, int device, srg_comm** comm);
/* One process driving ndev devices (devices == NULL: 0 .. ndev-1); rank i = devices[i]. */
int srg_comm_init_all(int ndev, const int* devices, srg_comm** comm);
int srg_comm_destroy(srg_comm* comm);
int srg_comm_size(const srg_comm* comm);

/* One local rank's share (device pointers on `device`). */
typedef struct {
    int device;
    const int64_t* indptr;        /* [n_rows + 1], rebased to 0 */
    const int32_t* indices;       /* global column ids (rows of the gathered panel) */
    const float* values;
    int64_t row0, n_rows;         /* must equal the rank's row_starts block */
    const int32_t* row_order;     /* optional schedule, as srg_spmm_csr_f32 */
    int64_t n_hub, n_heavy;
    float* x_full;                /* [row_starts[P], ld] gather buffer */
    float* const* panels;         /* HOST array of K + 1 pointers, each [n_rows, ld]; panels[0] = own X rows */
    void* stream;                 /* hipStream_t of `device` (NULL: its null stream) */
} srg_shard_f32;

/* panels[k] = (rank's rows of Â) * (panel k-1 gathered from every rank), k = 1..K, for every local
 * shard (shards[i] belongs to the communicator's i-th local rank).  Asynchronous on each shard's
 * stream, apart from one host sync per call (the owner split points and the sortedness check);
 * library-owned pair streams carry the exchange, and scratch for the split points comes from the
 * stream-ordered pool ((P - 1) * n_rows int64 per shard, freed at the end of the call). */
int srg_dist_propagate_khop_f32(srg_comm* comm, const srg_shard_f32* shards, int n_shards,
                                const int64_t* row_starts, int64_t ld, int32_t d, int32_t K);

/* ---- multi-GPU: the halo-exchange partition (the default multi-GPU path) -----------------------
 * The row-partitioned K-hop of srg_dist_propagate_khop_f32 moves every rank's whole block each hop
 * (an all-gather, 2.6x the bytes on the products graph at 8 ranks) and computes after the exchange.
 * The halo path moves only the remote rows each rank's rows reference, and overlaps that exchange
 * with the hop: a rank's rows are cut into C nnz-balanced row chunks plus one group of hub rows;
 * per hop the hub group is forked beside the chunks, and after each chunk's launch its rows that
 * peers need are packed and sent (grouped ncclSend / ncclRecv on a comm stream that waits only for
 * that pack), while the next chunks compute; the hub group's rows go last.  Low-degree halo rows
 * whose own columns are all local ("ghost rows") are computed locally instead of received.  Every
 * row keeps its entries in CSR order, so the hops are bitwise the one-GPU hops.  The same plan as
 * the Python package's srgnn/dist.py HaloPartitionedOperator runs on (it builds its shares with this
 * planner).  Replaces the reference's single-process hop loop, SSRG/operators/base_operator.py:32-35;
 * SURVEY.md §8(b) item 5, §8(e). */
#define SRG_HALO_AUTO (-1)     /* threshold chosen as the Python plan does (csr.auto_*_threshold) */
#define SRG_HALO_NONE (-2)     /* hub_threshold: no hub rows */
typedef struct srg_halo_plan srg_halo_plan;
typedef struct srg_halo_share srg_halo_share;
typedef struct {
    int64_t row0, n_rows;          /* own rows [row0, row0 + n_rows) of the global operator */
    int64_t n_recv, n_ghost, halo; /* panel rows after the own ones: received, then ghosts */
    int64_t nnz_local;             /* entries of the local CSR (own rows + ghost rows) */
    int64_t n_groups, hub_rows, send_rows;
    int32_t ghost_max_degree, chunks, nranks, rank;
} srg_halo_info;
/* Rank `rank`'s share, from the GLOBAL CSR on the host (int64 indptr[n+1] from 0, int32 column ids;
 * the same arrays on every rank).  chunks in [1, 250]; hub_threshold / heavy_threshold a row length,
 * SRG_HALO_AUTO, or (hub) SRG_HALO_NONE; ghost_max_degree >= 0 (0: no ghost rows) or SRG_HALO_AUTO:
 * the cap among 0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64 that minimises the modelled hop, max over
 * ranks of max(local SpMM bytes incl. ghost rows at 8.4e12 B/s, busiest peer link at link_bps per
 * direction; a row is 4d bytes on both sides, so d cancels) -- deterministic from the global graph
 * and link_bps, so every rank picks the same cap (pass every rank the same link_bps, e.g. the minimum
 * over ranks of a measured rate; <= 0: 64e9).  srg_halo_plan_info reports the cap taken.  Host-only:
 * needs no device; up to 16 host threads.  Validates the CSR (SRG_ERR_INVALID). */
int srg_halo_plan_build(const int64_t* indptr, const int32_t* indices, int64_t n, int32_t nranks, int32_t rank,
                        int32_t chunks, int64_t hub_threshold, int64_t heavy_threshold, int32_t ghost_max_degree,
                        double link_bps, srg_halo_plan** plan);
int srg_halo_plan_destroy(srg_halo_plan* plan);
int srg_halo_plan_info(const srg_halo_plan* plan, srg_halo_info* info);
/* Read-only view of one of the plan's host arrays (diagnostics and tests): *data points into the plan
 * (valid until it is destroyed), *count elements of the type given beside each selector. */
#define SRG_HALO_STARTS 0             /* int64 [nranks + 1] row blocks */
#define SRG_HALO_LOCAL_INDPTR 1       /* int64 [n_rows + halo + 1] */
#define SRG_HALO_LOCAL_INDICES 2      /* int32 [nnz_local] panel row ids */
#define SRG_HALO_GHOST_POSITIONS 3    /* int64: global entry positions of the ghost rows' entries */
#define SRG_HALO_HALO_IDS 4           /* int64 [halo] global ids of the halo rows, panel order */
#define SRG_HALO_GROUP_OFFSETS 5      /* int64 [n_groups] */
#define SRG_HALO_GHOST_SEND 6         /* int64 own local rows sent as peers' ghosts (X only) */
#define SRG_HALO_GHOST_SEND_COUNTS 7  /* int64 [nranks] */
#define SRG_HALO_GHOST_RECV_COUNTS 8  /* int64 [nranks] */
#define SRG_HALO_CHUNK_RANGES 9       /* int64 [chunks + 1] local row bounds of the chunks */
#define SRG_HALO_HUB_THRESHOLDS 10    /* int64 [nranks] */
#define SRG_HALO_VIEW_ORDER 11        /* int32 schedule of view `index` (chunks, hub group, ghosts) */
#define SRG_HALO_VIEW_META 12         /* int64 [4]: rows, hub rows, slice rows (d > 32), slice rows (d <= 32) */
#define SRG_HALO_SEND_ROWS 13         /* int64 own local rows sent in group `index`, peers ascending */
#define SRG_HALO_SEND_COUNTS 14       /* int64 [nranks] of group `index` */
#define SRG_HALO_RECV_COUNTS 15       /* int64 [nranks] of group `index` */
int srg_halo_plan_array(const srg_halo_plan* plan, int32_t what, int32_t index, const void** data, int64_t* count);
/* The share on `device`: local CSR (values gathered from the GLOBAL fp32 host array `values`),
 * schedules, send lists, a send buffer for panels up to d_max columns, a comm stream and events.
 * The plan must outlive the share.  The row chunks run in column blocks when d_max's panel asks for
 * them (srg_halo_share_col_blocks' automatic rule). */
int srg_halo_share_create(const srg_halo_plan* plan, const float* values, int device, int32_t d_max,
                          srg_halo_share** share);
int srg_halo_share_destroy(srg_halo_share* share);
/* Column blocks of the row chunks' launches (srgnn/dist.py HaloPartitionedOperator.chunk_blocks):
 * each chunk runs as n_blocks span launches over the own rows' spans whose GLOBAL column ids lie in
 * [ceil(b n / B), ceil((b+1) n / B)), rows of <= 48 entries whole in block 0, later blocks continuing
 * the chains (ACCUMULATE): bitwise the unblocked hop, with column locality for wide panels.
 * n_blocks in [1, 64] (1: unblocked) applies to every d; SRG_HALO_AUTO (the share's default) picks 8
 * for local panels ([own | halo] rows x d x 4 B) of >= 8 GiB at d >= 256, else 1, per call's d
 * Builds the split points and schedules on the host and uploads them (synchronous). */
int srg_halo_share_col_blocks(srg_halo_share* share, int32_t n_blocks);
/* Panel 0 from the WHOLE feature matrix X [n, ldx] on the share's device (as GraphOp.propagate is
 * handed the whole feature): own rows, then the halo rows gathered by global id.  Then pass
 * SRG_HALO_X_HALO_FILLED to srg_halo_propagate_f32 (no exchange of X). */
int srg_halo_fill_x_halo(const srg_halo_share* share, const float* X, int64_t ldx, float* panel0, int64_t ld,
                         int32_t d, void* stream);
/* K hops for the local shares of `comm` (shares[i] is the communicator's i-th local rank; for a
 * loopback communicator, ranks 0 .. nranks-1 in order).  panels: per share, a HOST array of K + 1
 * device pointers, each a [n_rows + halo, d] panel (ld == d: the halo rows are RCCL buffers) on the
 * share's device; panel 0's own rows hold X's rows of the rank, its halo is exchanged first unless
 * flags has SRG_HALO_X_HALO_FILLED.  streams: per share (NULL array or entries: the null stream).
 * Asynchronous on those streams; every panel k's own rows (and halo, k < K) are bitwise the one-GPU
 * hop k.  d <= the shares' d_max. */
#define SRG_HALO_X_HALO_FILLED 0x1u
int srg_halo_propagate_f32(srg_comm* comm, srg_halo_share* const* shares, int n_shards, float* const* const* panels,
                           int64_t ld, int32_t d, int32_t K, uint32_t flags, void* const* streams);
/* A communicator of nranks virtual ranks in ONE process on one device whose exchange is device-to-
 * device copies on a library stream: srg_halo_propagate_f32 then runs every rank's share (its
 * kernels, packs, groups and offsets) on one GPU -- the tests' and a single-GPU host's rehearsal of
 * the RCCL path.  Serves srg_halo_propagate_f32 only. */
int srg_comm_init_loopback(int nranks, int device, srg_comm** comm);

/* ---- diagnostics ----------------------------------------------------------------------------- */
const char* srg_last_error(void);   /* thread-local message of the last failure ("" if none) */
int srg_last_error_code(void);      /* thread-local status of the last call (SRG_OK if fine)  */
void srg_clear_error(void);
const char* srg_version(void);      /* build identification, incl. the offload arch          */

#ifdef __cplusplus
}
#endif
#endif /* SRGNN_HIP_H_ */
