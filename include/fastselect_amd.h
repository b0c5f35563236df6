/*
 * fastselect_amd.h -- C ABI of the MI355X Relief-family scoring engine.
 *
 * The reference (GavinLynch04/FastSelect v0.2.0) has no native FFI: its
 * hot-path boundary is the private Python "host callers" that each estimator's
 * fit() invokes once per fit.  The one-shot entry points below replace those
 * callers one-for-one (same arguments and meaning, plus a backend selector),
 * so the Python estimators call exactly one C function per fit:
 *
 *   fs_multisurf_score  replaces _multisurf_cpu_host_caller  (MultiSURF.py:256-270)
 *                       and      _multisurf_gpu_host_caller  (MultiSURF.py:147-162)
 *   fs_relieff_score    replaces _relieff_cpu_host_caller    (ReliefF.py:222-236)
 *                       and      _relieff_gpu_host_caller    (ReliefF.py:127-134)
 *   fs_surf_score       replaces _surf_cpu_host_caller       (SURF.py:198-218)
 *                       and      _surf_gpu_host_caller       (SURF.py:117-128)
 *
 * Every one-shot call is synchronous, takes caller-owned host arrays that must
 * stay valid for the duration of the call, and writes scores ALREADY DIVIDED
 * BY n (as the host callers return them).  Device memory is allocated and
 * freed inside the call; no pointer to caller memory is retained.
 *
 * The fs_plan_* entry points expose the same MultiSURF path split at its
 * three exchange points (per-row distance moments, per-row neighbour counts,
 * per-feature score sums) so that one process per GPU can shard the pair
 * tiles across ranks and sum those three small vectors with a collective
 * (RCCL all-reduce over xGMI, driven by torch.distributed in
 * fastselect_amd/parallel.py).  With world == 1 the stages compose to exactly
 * fs_multisurf_score.
 *
 * Errors: every function returns FS_OK (0) or a negative FS_E* code; a
 * thread-local human-readable message is available from fs_last_error().
 * The Python layer maps FS_EINVAL -> ValueError, FS_ENODEV / FS_EHIP /
 * FS_ENOTSUP -> RuntimeError, FS_EOOM -> MemoryError.
 *
 * Backends: FS_BACKEND_GPU runs the hand-written HIP kernels for gfx950
 * (MI355X) and fails with FS_ENODEV when no HIP device is visible -- it never
 * falls back to the CPU.  FS_BACKEND_CPU runs the native multithreaded CPU
 * implementation of the same pipeline (the reference's backend='cpu').
 */
#ifndef FASTSELECT_AMD_H
#define FASTSELECT_AMD_H

#include <stdint.h>

#if defined(__GNUC__)
#define FS_API __attribute__((visibility("default")))
#else
#define FS_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define FS_OK 0
#define FS_EINVAL (-1)   /* bad argument (shape, pointer, parameter) */
#define FS_ENODEV (-2)   /* GPU backend requested but no HIP device visible */
#define FS_EOOM (-3)     /* host or device allocation failed */
#define FS_EHIP (-4)     /* HIP runtime / kernel launch error */
#define FS_ENOTSUP (-5)  /* combination not supported by this build */

#define FS_BACKEND_CPU 0
#define FS_BACKEND_GPU 1

#define FS_ACCUM_FAST 0       /* default: symmetric pair weights, float64 partial sums */
#define FS_ACCUM_REFERENCE 1  /* the reference's float32 per-sample chains and column sums */

/*
 * Accumulation mode of the calling thread's subsequent scoring calls and
 * plan creations (a plan keeps the mode it was created with).  No reference
 * counterpart: the reference has one arithmetic, its kernels' float32 sums
 * (MultiSURF.py:198-253, ReliefF.py:181-220).
 *   FS_ACCUM_FAST       the default pass 2: each pair's two directed weights
 *                       folded into one, float32 streams summed in float64.
 *                       10-60x closer to the exact (float64) sums than the
 *                       reference's own float32 sums (DESIGN.md §The oracle).
 *   FS_ACCUM_REFERENCE  MultiSURF / MultiSURF*: every focal sample's hit and
 *                       miss diffs summed in float32 in ascending j, divided,
 *                       temp = miss - hit in float32, then each feature's
 *                       float32 sequential column sum; ReliefF: float32 temp of
 *                       the float64 update over argsort-ordered neighbours and
 *                       the same column sums.  MultiSURF then runs pass 1 on
 *                       32-bit operands with exact thresholds for every
 *                       flagged row.  SURF / SURF*: the reference's order at
 *                       n_jobs = 1 (its one fixed order; with more numba
 *                       threads it adds per-thread rows in schedule order,
 *                       SURF.py:195, 216): four float32 chains per sample in
 *                       ascending j, score_update in float32, one sequential
 *                       float32 sum over the samples (SURF.py:139-218).  The
 *                       scores are then bit-identical to the oracle's
 *                       sequential restatement of the reference's float32
 *                       order (oracle/relief_oracle.c; tests/test_refacc*.py).
 *                       The reference kernels are @njit(fastmath=True), which
 *                       lets LLVM reassociate its float64 distance sums; no
 *                       reference-produced fixture pins that level, so parity
 *                       with numba's own bits is unpinned.  The
 *                       one-shot calls and fs_*_score_devices with more than
 *                       one device run on one device (FS_ENOTSUP otherwise);
 *                       GPU MultiSURF plans with world > 1 run pass 2 as
 *                       fs_plan_ref_masks / fs_plan_ref_pass2 /
 *                       fs_plan_ref_sums, row plans (ReliefF, SURF) as
 *                       fs_plan_ref_temp / fs_plan_ref_sums (CPU backend:
 *                       FS_ENOTSUP).
 * previous (nullable) receives the mode in force before the call.  The mode
 * is per thread: a caller that scores from several threads passes it per
 * call instead (fs_*_score_ex below).
 */
FS_API int fs_set_accumulation(int mode, int* previous);
FS_API int fs_get_accumulation(void);

/*
 * TEST-ONLY: override one internal choice of the library for the calls that
 * follow, process-wide (tests/ uses it to reach routes the automatic choices
 * take only at other sizes; no product code calls it).  name = "reset"
 * restores every default; the others are listed in INTEGRATION.md §4
 * ("ksplit", "q16", "sparse", "shards", "q16_guard_off", "thr_exact_all",
 * "exact_gather", "row_panel",
 * "rf_xlds", "rf_fcap", "ties_1w", "ties_coop", "rf_ref_replay", "ref_q16", "surf_f64",
 * "colsort_bins12", "colsort_global", "star_split", "colsort_star").  FS_EINVAL for an unknown name.  Not thread-safe
 * against concurrent scoring calls.
 */
FS_API int fs_test_hook(const char* name, int64_t value);

/* Library identity and device discovery. */
FS_API const char* fs_version(void);
FS_API const char* fs_last_error(void);
/* Number of visible HIP devices (0 when none, never negative). */
FS_API int fs_device_count(void);
/* Free the device blocks the library keeps between calls.  Plans and the
 * column statistics return their device buffers to a per-device cache (up to
 * an eighth of the device's memory, FS_DEVICE_CACHE_MB overrides, 0
 * disables), so that the next fit skips hipMalloc's page mapping (190-310 ms
 * for a cfg4 plan).  Returns FS_OK. */
FS_API int fs_device_cache_release(void);
/* Pinned host memory for the float32 copy of X a fit makes (GPU backend):
 * the host threads cast into pinned, already-mapped pages and the upload of
 * X is a DMA from them.  Blocks are cached between calls (two at most;
 * fs_device_cache_release frees them).  FS_ENODEV without a GPU. */
FS_API int fs_host_alloc(uint64_t bytes, void** out);
FS_API int fs_host_free(void* p);
/* Stage X for one fit: upload the n x p row-major matrix (float32, or
 * float64 when x_is_f64) to `device` once.  Until fs_unstage_x, the GPU
 * backend's fs_column_stats and scoring calls given the same host pointer,
 * shape and dtype, made from the thread that staged it, read the staged copy
 * instead of uploading X again; the caller must not modify x in between.
 * *staged receives the handle. */
FS_API int fs_stage_x(int device, const void* x, int x_is_f64, int64_t n, int64_t p,
                      uint64_t* staged);
/* As fs_stage_x, but X is already on `device` (x_device: n x p row-major,
 * caller-owned, valid until fs_unstage_x, which does not free it): the
 * multi-GPU path uploads each rank's rows and all-gathers the rest over RCCL
 * (fastselect_amd/parallel.py), then registers the gathered copy under the
 * host array's key so that the column statistics and the plan read it. */
FS_API int fs_stage_x_device(int device, const void* x, const void* x_device, int x_is_f64,
                             int64_t n, int64_t p, uint64_t* staged);
/* The float64 -> float32 cast of X (round to nearest, as numpy's astype;
 * x_is_f64 = 0: a float32 X is copied as is) into the caller's `out`
 * (n x p, row-major; pinned memory from
 * fs_host_alloc makes the upload a DMA), fused with the finiteness check of
 * the result (*finite as fs_all_finite) and with fs_stage_x of `out`: row
 * blocks are uploaded while later ones are cast.  *staged = 0 when the device
 * had no room for the copy or a value is not finite (the cast is done either
 * way).  Replaces the cast in scikit-learn's validate_data(dtype=np.float32)
 * that MultiSURF.fit starts with (MultiSURF.py:384-386) plus the upload of
 * the cast array. */
FS_API int fs_stage_x_cast(int device, const void* x, int x_is_f64, int64_t n, int64_t p,
                           int n_jobs, float* out, int* finite, uint64_t* staged);
FS_API int fs_unstage_x(uint64_t staged);
/* *finite = 1 if every element of the n x p float32 / float64 matrix is
 * finite, else 0 (host threads; n_jobs as the scoring calls).  The
 * estimators call it in place of scikit-learn's single-threaded scan and fall
 * back to scikit-learn's own validation, and its error, when it reports 0. */
FS_API int fs_all_finite(const void* x, int x_is_f64, int64_t n, int64_t p, int n_jobs,
                         int* finite);

/*
 * MultiSURF / MultiSURF* feature scores.
 *   x            [n][p] float32, row-major (validated X, MultiSURF.py:384-386)
 *   y            [n] labels as float64; samples are hits when y[i] == y[j]
 *   recip        [p] float32 reciprocal feature ranges (MultiSURF.py:409-412)
 *   feat_idx     [n_kept] feature indices to score, or NULL for all p
 *                (the reference's feat_idx argument, MultiSURF.py:147,256)
 *   use_star     nonzero: MultiSURF* (far misses subtract, MultiSURF.py:236-243)
 *   is_discrete  [p] 0/1 (MultiSURF.py:416-420)
 *   n_jobs       CPU threads (-1 = all); ignored by the GPU backend
 *   device       HIP device ordinal for the GPU backend
 *   scores_out   [n_kept] float32, scores / n
 */
FS_API int fs_multisurf_score(int backend, int device, const float* x, int64_t n, int64_t p,
                       const double* y, const float* recip, const int64_t* feat_idx,
                       int64_t n_kept, int use_star, const uint8_t* is_discrete, int n_jobs,
                       float* scores_out);

/*
 * The decision check of this thread's last GPU fs_multisurf_score call
 * (new; the reference has no quantised pass).  MultiSURF (not MultiSURF*)
 * scored on 16-bit pass-1 operands estimates how far the near/far decisions
 * its quantised thresholds could change move the scores, relative to their
 * largest magnitude (risk_out; -1 when not evaluated: 32-bit operands,
 * MultiSURF*, the q16 test hook set, CPU backend); above 5e-6 the call scores again on
 * 32-bit operands and rerun_out is 1.  Signal-free inputs (scores at the
 * noise floor of the decisions) are what trips it.
 */
FS_API int fs_multisurf_last_guard(double* risk_out, int* rerun_out);

/*
 * MultiSURF / MultiSURF* score SUMS (not divided by n) of the focal samples
 * [row_begin, row_end) only, written to sums_out[n_kept] (host memory).
 * The reference's kernel is a prange over focal samples whose rows are
 * independent once each sample's threshold is known (MultiSURF.py:174-251):
 * thresholds and neighbour counts stay those of the whole fit, and each pair
 * contributes only the side of its focal sample inside the range.  Summing
 * the vectors of a partition of [0, n) and dividing by n gives the one-shot
 * scores up to float64 summation order; [0, 384) of the reference's
 * per-sample rows is the same as oracle i_range=(0, 384).  Other arguments as
 * fs_multisurf_score.
 */
FS_API int fs_multisurf_score_rows(int backend, int device, const float* x, int64_t n,
                                   int64_t p, const double* y, const float* recip,
                                   const int64_t* feat_idx, int64_t n_kept, int use_star,
                                   const uint8_t* is_discrete, int n_jobs, int64_t row_begin,
                                   int64_t row_end, double* sums_out);

/*
 * ReliefF feature scores (ReliefF.py:137-236).
 *   x            [n][p] float32 (the float32 cast of the float64-validated X, ReliefF.py:400)
 *   y_enc        [n] int32 class codes in [0, n_classes) (ReliefF.py:375)
 *   recip        [p] float32 (discrete and zero ranges forced to 1, ReliefF.py:377-380)
 *   is_discrete  [p] 0/1
 *   k            n_neighbors (>= 1)
 *   class_probs  [n_classes] float32 class priors (ReliefF.py:373-374)
 *   scores_out   [p] float32, scores / n
 * Neighbours are chosen as the reference chooses them: by its float32
 * distance key, ties at the k-th key in numba's quicksort order.
 */
FS_API int fs_relieff_score(int backend, int device, const float* x, int64_t n, int64_t p,
                     const int32_t* y_enc, const float* recip, const uint8_t* is_discrete,
                     int64_t k, const float* class_probs, int64_t n_classes, int n_jobs,
                     float* scores_out);

/*
 * SURF / SURF* feature scores (SURF.py:131-218).
 *   x            [n][p] float64, row-major (SURF.py:330-332)
 *   y            [n] int32 labels (y.astype(int32), SURF.py:371)
 *   recip        [p] float32 (SURF.py:352-355)
 *   use_star     nonzero: SURF* (far hits add, far misses subtract)
 *   scores_out   [p] float32, scores / n
 */
FS_API int fs_surf_score(int backend, int device, const double* x, int64_t n, int64_t p,
                  const int32_t* y, const float* recip, int use_star,
                  const uint8_t* is_discrete, int n_jobs, float* scores_out);

/*
 * The three one-shot calls with the accumulation mode as an argument
 * (FS_ACCUM_FAST / FS_ACCUM_REFERENCE, as fs_set_accumulation documents),
 * for that call only: the calling thread's fs_set_accumulation mode is
 * neither read nor changed.  Other arguments as fs_multisurf_score /
 * fs_relieff_score / fs_surf_score, which they replace for callers that do
 * not own the thread they score on (the reference's host callers take no
 * such mode: MultiSURF.py:256, ReliefF.py:222, SURF.py:198).
 */
FS_API int fs_multisurf_score_ex(int backend, int device, const float* x, int64_t n, int64_t p,
                                 const double* y, const float* recip, const int64_t* feat_idx,
                                 int64_t n_kept, int use_star, const uint8_t* is_discrete,
                                 int n_jobs, int accumulation, float* scores_out);
FS_API int fs_relieff_score_ex(int backend, int device, const float* x, int64_t n, int64_t p,
                               const int32_t* y_enc, const float* recip,
                               const uint8_t* is_discrete, int64_t k, const float* class_probs,
                               int64_t n_classes, int n_jobs, int accumulation,
                               float* scores_out);
FS_API int fs_surf_score_ex(int backend, int device, const double* x, int64_t n, int64_t p,
                            const int32_t* y, const float* recip, int use_star,
                            const uint8_t* is_discrete, int n_jobs, int accumulation,
                            float* scores_out);

/*
 * Row-sharded ReliefF / SURF: the float64 score SUMS (not
 * divided by n) of the focal samples [row_begin, row_end) only, written to
 * sums_out[p] (host memory).  Other arguments as fs_relieff_score /
 * fs_surf_score.  Neighbour selection is row-local in both algorithms
 * (ReliefF's k nearest per class, ReliefF.py:144-175; SURF's per-sample mean
 * threshold, SURF.py:146-163), so one process per GPU scores a slice of the
 * samples and a single SUM all-reduce of p doubles combines the slices:
 * summing the vectors of a partition of [0, n) and dividing by n gives the
 * one-shot scores up to float64 summation order.  The GPU computes every
 * distance tile that touches the slice's 128-sample blocks, so slices on
 * 128-sample boundaries (fastselect_amd.parallel.shard_rows) balance best.
 */
FS_API int fs_relieff_score_rows(int backend, int device, const float* x, int64_t n, int64_t p,
                                 const int32_t* y_enc, const float* recip,
                                 const uint8_t* is_discrete, int64_t k, const float* class_probs,
                                 int64_t n_classes, int n_jobs, int64_t row_begin,
                                 int64_t row_end, double* sums_out);
FS_API int fs_surf_score_rows(int backend, int device, const double* x, int64_t n, int64_t p,
                              const int32_t* y, const float* recip, int use_star,
                              const uint8_t* is_discrete, int n_jobs, int64_t row_begin,
                              int64_t row_end, double* sums_out);

/*
 * Single-process multi-GPU scoring (the estimators' `devices=`; SURVEY.md
 * §5 "Config / flags", §8(b) "Threading: one host thread per device").  One
 * host thread per entry of devices[0 .. n_devices) -- ordinals may repeat
 * (several plans share one device) -- with the partitions of the
 * one-process-per-GPU path (fastselect_amd/parallel.py): MultiSURF deals the
 * upper-triangle pair tiles round-robin (tile t -> thread t % N) and sums its
 * three exchange vectors (row moments, neighbour counts, score sums) on the
 * host in thread order after each stage, where the multi-process path
 * all-reduces them over RCCL; ReliefF / SURF give each thread whole 128-sample
 * blocks of the focal range and sum the score vectors once.  Write the
 * float64 score SUMS of the focal samples [row_begin, row_end) (not divided
 * by n; [0, n) for a whole fit) to sums_out.  Other arguments as the
 * one-shot calls; the reference's fit is one call on one device
 * (MultiSURF.py:393-440, ReliefF.py:382-403, SURF.py:339-372).
 */
FS_API int fs_multisurf_score_devices(const int* devices, int n_devices, const float* x, int64_t n,
                                      int64_t p, const double* y, const float* recip,
                                      const int64_t* feat_idx, int64_t n_kept, int use_star,
                                      const uint8_t* is_discrete, int n_jobs, int64_t row_begin,
                                      int64_t row_end, double* sums_out);
FS_API int fs_relieff_score_devices(const int* devices, int n_devices, const float* x, int64_t n,
                                    int64_t p, const int32_t* y_enc, const float* recip,
                                    const uint8_t* is_discrete, int64_t k, const float* class_probs,
                                    int64_t n_classes, int n_jobs, int64_t row_begin,
                                    int64_t row_end, double* sums_out);
FS_API int fs_surf_score_devices(const int* devices, int n_devices, const double* x, int64_t n,
                                 int64_t p, const int32_t* y, const float* recip, int use_star,
                                 const uint8_t* is_discrete, int n_jobs, int64_t row_begin,
                                 int64_t row_end, double* sums_out);

/*
 * Per-column statistics of X: the preprocessing each reference fit() runs on
 * the host before scoring -- x.min(axis=0), x.max(axis=0) and, per column,
 * np.unique(x[:, f]).size compared with discrete_limit (MultiSURF.py:141-144,
 * 409-420; ReliefF.py:366-380; SURF.py:347-355).
 *   x            [n][p] row-major, float32 (x_is_f64 = 0) or float64 (1)
 *   count_cap    distinct values are counted exactly up to count_cap (pass
 *                discrete_limit); a column with more reports count_cap + 1.
 *                The GPU backend supports count_cap <= 8191 (FS_ENOTSUP above)
 *   colmin_out, colmax_out  [p] in x's dtype
 *   ndistinct_out           [p] min(distinct values, count_cap + 1)
 * Equality is numpy's: -0.0 and +0.0 are one value; X must be finite (the
 * estimators validate it first, as the reference does).
 */
FS_API int fs_column_stats(int backend, int device, const void* x, int x_is_f64, int64_t n,
                           int64_t p, int64_t count_cap, void* colmin_out, void* colmax_out,
                           int64_t* ndistinct_out);

/* ---- Sharded MultiSURF plan (one plan per rank) ------------------------ */

typedef struct fs_plan fs_plan;

/*
 * Create a plan and upload its inputs (host arrays, same meaning as
 * fs_multisurf_score).  rank/world select which upper-triangle pair tiles
 * this plan computes (tile t belongs to rank t % world).  `stream` is a
 * hipStream_t (0 = the plan's own stream) on which every GPU stage is
 * enqueued; stages do not synchronise the host unless `stream` is 0.
 */
FS_API int fs_plan_create(fs_plan** plan_out, int backend, int device, const float* x, int64_t n,
                   int64_t p, const double* y, const float* recip, const int64_t* feat_idx,
                   int64_t n_kept, int use_star, const uint8_t* is_discrete, int rank, int world,
                   int n_jobs, uint64_t stream);

/*
 * Re-target the plan to another feature subset of the same samples
 * (feat_idx[n_kept] into the original columns, NULL = all), keeping X and
 * its column ranges resident: the next pass1/select/pass2 score the subset
 * exactly as a fresh plan on X[:, feat_idx] would (the reference scores such
 * subsets through feat_idx, MultiSURF.py:147,256; TuRF refits on them,
 * TuRF.py:93-115).  The scores vector of pass2 then has n_kept entries.
 */
FS_API int fs_plan_set_features(fs_plan* plan, const int64_t* feat_idx, int64_t n_kept);

/*
 * Stage 1: quantise the resident X, compute this rank's distance tiles and
 * write this rank's partials to rowstats[3n]: per row sum D, sum D^2 (D in the
 * plan's integer distance unit) and this rank's share of the mean correction
 * (its slice of the continuous features).  Pointers live in the plan's memory
 * space: device memory for the GPU backend, host memory for the CPU backend.
 */
FS_API int fs_plan_pass1(fs_plan* plan, double* rowstats);
/* Stage 2: thresholds from the all-reduced rowstats[3n], exact recomputation of this rank's ambiguous pairs (pairs whose
 * quantised distance lies so close to a threshold that the near/far decision
 * is not certain), then partial per-row (near hits, near misses) -> counts[2n]. */
FS_API int fs_plan_select(fs_plan* plan, const double* rowstats, double* counts);
/* Stage 3: pair weights from the all-reduced counts[2n]; partial per-feature
 * score sums (NOT divided by n) -> scores[n_kept], in feat_idx order. */
FS_API int fs_plan_pass2(fs_plan* plan, const double* counts, double* scores);
/* After the three stages of a MultiSURF step, with rowstats[3n], counts[2n]
 * and scores[n_kept] all-reduced (identical on every rank): the 16-bit
 * decision check of fs_multisurf_score (see fs_multisurf_last_guard) for
 * plans whose pass 1 runs on 16-bit operands.  risk_out = the estimated score
 * error of threshold-moved decisions over max |score| (-1: nothing to check:
 * 32-bit operands, MultiSURF*, the CPU backend).  Above the bound the plan
 * switches to 32-bit operands for good and *switched_out = 1: every rank
 * computed the same risk and switched alike, and the caller runs the step
 * again (the reference's single threshold rule, MultiSURF.py:193-217, and
 * TuRF's refits, TuRF.py:87,111, through the same plan). */
FS_API int fs_plan_decision_guard(fs_plan* plan, const double* rowstats, const double* counts,
                                  const double* scores, double* risk_out, int* switched_out);
/* Reference-order accumulation (fs_set_accumulation(FS_ACCUM_REFERENCE))
 * over world > 1 ranks, GPU backend.  The reference's float32 sums run over
 * every focal sample in order (MultiSURF.py:231-253, then
 * np.sum(temp, axis=0)), so pass 2 is not a sum of rank partials; after
 * pass1 / all-reduce / select / all-reduce, instead of fs_plan_pass2:
 *   1. fs_plan_ref_masks: this rank's pair-tile decisions as bit masks in
 *      masks[words] (device memory, words >= fs_plan_ref_mask_words; zeroed
 *      first, so every word outside this rank's tiles is 0);
 *   2. a SUM all-reduce of the masks as int64 (each word is nonzero on at
 *      most one rank, so the sum is the whole triangle's masks);
 *   3. fs_plan_ref_pass2 on every rank at once: the per-sample hit / miss
 *      chains of the focal rows [row_begin, row_end) of the rank's contiguous
 *      block (counts = the all-reduced counts[2n]) into the plan's float32
 *      temp rows;
 *   4. fs_plan_ref_sums on the ranks in order: rank r continues the float32
 *      column sums init[n_kept] it received from rank r - 1 (NULL on the
 *      first rank) over its temp rows and hands sums[n_kept] to rank r + 1;
 *      the last rank's sums, divided by n, are the reference's scores bit
 *      for bit (fastselect_amd/parallel.py ShardedMultiSURF). */
FS_API int fs_plan_ref_mask_words(fs_plan* plan, int64_t* words);
FS_API int fs_plan_ref_masks(fs_plan* plan, uint64_t* masks, int64_t words);
FS_API int fs_plan_ref_pass2(fs_plan* plan, const uint64_t* masks, const double* counts,
                             int64_t row_begin, int64_t row_end);
FS_API int fs_plan_ref_sums(fs_plan* plan, const double* init, double* sums);
/* The same rank chain for row-sharded ReliefF and SURF (fs_plan_create_relieff
 * / fs_plan_create_surf over the rank's focal rows, reference order, GPU
 * backend): fs_plan_ref_temp runs fs_plan_score up to the plan's float32 temp
 * rows (ReliefF.py:208-218, SURF.py:191-193) on every rank at once, then
 * fs_plan_ref_sums continues the previous rank's column sums over them
 * (ReliefF.py:219-220, SURF.py:195: one sequential float32 sum). */
FS_API int fs_plan_ref_temp(fs_plan* plan);
/* Restrict the next pass2 of a MultiSURF plan to the focal samples
 * [row_begin, row_end) (as fs_multisurf_score_rows; a new plan scores
 * [0, n)).  pass1 / select are unchanged: thresholds and counts are global. */
FS_API int fs_plan_set_rows(fs_plan* plan, int64_t row_begin, int64_t row_end);
/* Re-target a MultiSURF plan to the pair tiles of shard (rank, world) --
 * tile t belongs to rank t % world -- keeping X and its quantised operands
 * resident (the GPU plan frees the previous shard's distance tiles).  With
 * it one device scores a job whose distance tiles exceed its memory in
 * shards; the stages then run in three rounds, each over all shards (row
 * moments -> all-reduce; select -> counts -> all-reduce; select, pass2 ->
 * scores), every round recomputing the shard's distances
 * (fastselect_amd/parallel.py ShardedMultiSURF).  An N-GPU job with V
 * shards per GPU uses rank + N * v of N * V.  No reference counterpart (the
 * reference streams each focal sample's distance row, MultiSURF.py:174-214). */
FS_API int fs_plan_set_shard(fs_plan* plan, int rank, int world);
/* Shards per device that keep a MultiSURF job of n samples, p features and
 * `world` ranks within the device's free memory (1 when it fits, or without
 * a GPU; the shards test hook overrides).  The one-shot fs_multisurf_score[_rows]
 * shards by itself. */
FS_API int fs_multisurf_shards(int device, int64_t n, int64_t p, int world, int* shards);
/*
 * ReliefF / SURF plans (resident scoring): X uploaded once (GPU) or copied
 * (CPU), arguments as fs_relieff_score / fs_surf_score, focal samples
 * [row_begin, row_end) as fs_*_score_rows.  fs_plan_score writes the float64
 * score sums of those samples for the plan's current feature subset to
 * sums[n_kept] (device memory for the GPU backend, host memory for the CPU
 * backend); fs_plan_set_features re-targets the plan to another column subset
 * without re-uploading X, which is how TuRF re-scores its shrinking feature
 * sets (TuRF.py:93-115).  pass1 / select / pass2 are MultiSURF-only, and
 * fs_plan_score is ReliefF / SURF-only (FS_EINVAL otherwise).
 */
FS_API int fs_plan_create_relieff(fs_plan** plan_out, int backend, int device, const float* x,
                                  int64_t n, int64_t p, const int32_t* y_enc, const float* recip,
                                  const uint8_t* is_discrete, int64_t k, const float* class_probs,
                                  int64_t n_classes, int64_t row_begin, int64_t row_end,
                                  int n_jobs, uint64_t stream);
FS_API int fs_plan_create_surf(fs_plan** plan_out, int backend, int device, const double* x,
                               int64_t n, int64_t p, const int32_t* y, const float* recip,
                               int use_star, const uint8_t* is_discrete, int64_t row_begin,
                               int64_t row_end, int n_jobs, uint64_t stream);
FS_API int fs_plan_score(fs_plan* plan, double* sums);
/* Number of pair tiles this plan owns, the pair-feature evaluations one full
 * pass1+pass2 performs on this rank (throughput accounting) and the number of
 * ambiguous pairs the last stage 2 recomputed exactly.  NULL outputs are
 * skipped. */
FS_API int fs_plan_info(const fs_plan* plan, int64_t* owned_tiles, double* pair_feature_evals,
                        int64_t* refined_pairs);
/* Refinement-band calibration of the plan's current feature layout (GPU
 * MultiSURF / ReliefF plans; no reference counterpart -- it guards the
 * integer pass 1 that replaces the reference's float distance loop,
 * MultiSURF.py:176-188).  fs_plan_calibration writes out[6] (its size since
 * the first release): [0] 1 if pass 1 runs on 16-bit operands, [1] / [2] rms
 * / max |quantised - reference| distance error over 4096 sampled pairs
 * (integer units), [3] the independent-rounding model's standard deviation
 * sqrt(pc/6 + 1), [4] band / model band, [5] 1 if the coherence guard turned
 * 16-bit operands off, 2 if the per-row guard did (a row whose mean pass-1
 * error, measured by the mean correction, exceeds 12 standard deviations of
 * independent rounding); SURF plans (32-bit operands against its float64
 * terms, fs_surfint.hip): [5] 0 on integer distances, 3 on float64 ones (the
 * band above one float32 ulp of the shorter sampled distances, a small
 * problem, or the surf_f64 test hook).  fs_plan_calibration_ex writes min(n_out, 8)
 * values -- the six above, then [6] that row guard's largest row bias over
 * its limit (0 when it did not run) and [7] SC, the integer units per
 * scaled-diff unit of pass 1 (the row statistics of fs_plan_pass1 are in
 * these units: mu_i = (rowstats[3i] - rowstats[3i+2]) / (n - 1) / SC) -- and
 * returns how many it wrote (or a negative FS_E* code).  CPU plans:
 * {0, 0, 0, model sigma, 1, 0, 0, SC}. */
FS_API int fs_plan_calibration(const fs_plan* plan, double* out);
FS_API int fs_plan_calibration_ex(const fs_plan* plan, double* out, int n_out);
/* Owned pairs that carried a non-zero pass-2 weight in the last pass 2 (the
 * pairs the sparse GPU pass 2 evaluates; -1 when the plan does not count
 * them: CPU backend, dense pass 2, or before the first pass 2). */
FS_API int fs_plan_weighted_pairs(const fs_plan* plan, int64_t* pairs);
/* Average duration in milliseconds of the last pass1 / pass2 distance and
 * score kernels, measured with HIP events on the plan's stream (GPU only;
 * -1 when unavailable).  which: 0 = distance kernel, 1 = score kernel (for
 * ReliefF plans: neighbour selection, exact refinement and update), 2 =
 * ReliefF's first k_rf_select launch. */
FS_API double fs_plan_kernel_ms(const fs_plan* plan, int which);
FS_API int fs_plan_destroy(fs_plan* plan);

#ifdef __cplusplus
}
#endif

#endif /* FASTSELECT_AMD_H */
