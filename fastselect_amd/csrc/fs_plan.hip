// fs_plan.hip -- plan lifetime, layout, shards and the scoring entry points.
// Shared state and helpers: fs_gpu_internal.h.
#include "fs_gpu_internal.h"

namespace fs {
namespace gpu {

void plan_destroy(Plan* g) {
  if (!g) return;
  if (g->stream) (void)hipStreamSynchronize(g->stream);
  trace_mark("kernels (to sync)");
  if (g->side) (void)hipStreamSynchronize(g->side);
  if (g->side2) (void)hipStreamSynchronize(g->side2);
  for (void* q : g->owned) dev_free(q);
  for (void* q : g->owned_layout) dev_free(q);
  for (void* q : g->scratch) dev_free(q);
  for (void* q : g->owned_shard) dev_free(q);
  if (g->spart) dev_free(g->spart);
  if (g->temp) dev_free(g->temp);
  if (g->rkeys) dev_free(g->rkeys);
  if (g->sched) dev_free(g->sched);
  if (g->units8) dev_free(g->units8);
  if (g->x_staged) staged_release(g->x_staged);
  for (auto& e : g->ev) event_put(g->device, e, true);
  event_put(g->device, g->ev_fork, false);
  event_put(g->device, g->ev_join, false);
  event_put(g->device, g->ev_star, false);
  stream_put(g->device, g->side);
  if (g->side2) stream_put(g->device, g->side2);
  if (g->own_stream) stream_put(g->device, g->stream);
  delete g;
  trace_mark("plan: free");
}

// 16-bit pass-1 operands (Prepared::q16) halve k_dist.  ReliefF stays exact
// with them (every candidate near a k-th key gets its reference key), so it
// uses them from kQ16MinRowsRF samples on.  MultiSURF's threshold mu - sigma/2
// comes from the quantised row moments: the sigma error grows as 1/SC and the
// score error it causes (pairs decided on the wrong side of a threshold, each
// worth ~1/n^2) falls as ~n^-1.25 -- measured against the 32-bit path: 8.8e-6
// scale-relative at n=5000, 3.9e-6 at 8192, 1.9e-6 at 20000 --
// so MultiSURF takes them only from kQ16MinRowsMS samples on.  MultiSURF*
// is less sensitive (its far misses weigh the pairs between the two
// thresholds both ways): 5.5e-7 at cfg4, 1.5e-6 at cfg5 (n = 10000,
// p = 50000), so it takes them from kQ16MinRowsMSStar on.  The q16 test
// hook forces the choice.  SURF has its own float64 pass.
constexpr int64_t kQ16MinRowsRF = 4096, kQ16MinRowsMS = 16384, kQ16MinRowsMSStar = 10000;
static int choose_q16(const Prepared& P) {
  if (P.algo == ALGO_SURF || P.no_q16) return 0;
  // reference-order MultiSURF replays the reference's decisions: 32-bit
  // operands, whose thresholds need exact recomputation on a handful of rows
  if (P.algo == ALGO_MULTISURF && P.ref_accum && !test_hooks().ref_q16) return 0;
  if (test_hooks().q16 >= 0) return test_hooks().q16 != 0 ? 1 : 0;
  const int64_t min_rows = P.algo == ALGO_RELIEFF ? kQ16MinRowsRF
                           : P.use_star           ? kQ16MinRowsMSStar
                                                  : kQ16MinRowsMS;
  return (P.n >= min_rows && P.pc >= kFeatPad) ? 1 : 0;
}

// MultiSURF* / SURF* in fast accumulation: near pairs in pass 2, the far
// pairs' all-pairs part per column from its sorted values (fs_starterm.hip),
// for n <= 24576 and up to 8 classes (one workgroup sorts a column in LDS);
// the star_split test hook forces either form where it fits.  Its
// feature-major copy of the pass-2 values (xsT, n_pad x PW floats) is taken
// only while it stays under a quarter of the device's free memory; a plan
// that large keeps the dense star weights.
static bool choose_star_split(const Prepared& P, int device) {
  if (!P.use_star || P.ref_accum || P.algo == ALGO_RELIEFF) return false;
  if (!star_split_fits(P.n, P.n_classes)) return false;
  if (test_hooks().star_split >= 0) return test_hooks().star_split != 0;
  size_t free_b = 0, total_b = 0;
  if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return (double)P.n_pad * (double)P.PW * sizeof(float) <= 0.25 * (double)free_b;
}

// Pass 2 on the non-zero pair weights only (k_weights_sparse2 +
// k_score_sparse2) or on every pair (k_weights + k_score).  Round 1's sparse
// loop cost ~1.7x the dense one per evaluated pair; the v2 loop (round 4)
// ~1.3x, so it pays below ~75% density.  MultiSURF weighs the ~42% of pairs
// near one of their samples, SURF the ~62% (cfg5: the whole step 179.4 ->
// 156.6 ms sparse, profiles/r06/starsplit/surf_sparse_ab.txt); the star
// variants weigh every miss / every pair and go sparse through the star
// split (profiles/r06/near_density.txt).  SURF below kSparseMinRowsSurf
// samples keeps the dense loop: its pass 2 costs little there, and on the
// heavy-tailed tail sweep (tests/test_random_parity.py, seed 2: n = 300-3000)
// the sparse loop's float32 partials ended 4.8x closer to the float64 sums
// than the reference's own, against the 5x the attributed bar asks.  The
// sparse test hook forces either.
constexpr int64_t kSparseMinRowsSurf = 4096;
static int choose_sparse(const Plan* g, const Prepared& P) {
  if (P.algo == ALGO_RELIEFF) return 0;
  if (test_hooks().sparse >= 0) return test_hooks().sparse != 0 ? 1 : 0;
  if (g->star_split) return 1;
  if (!P.use_star) return (P.algo == ALGO_MULTISURF || P.n >= kSparseMinRowsSurf ||
                           g->r_hi - g->r_lo < P.n) ? 1 : 0;
  // the star weights without the split (n > 24576, > 8 classes): dense,
  // unless a row-sharded SURF* plan zeroes the sides it does not own
  return (P.algo == ALGO_SURF && g->r_hi - g->r_lo < P.n) ? 1 : 0;
}

// Feature-layout part of a plan: everything sized by the kept features
// (permutation tables, quantised operands, pass-2 partials), rebuilt when
// the plan is re-targeted to another feature subset (fs_plan_set_features).
// Reference-order accumulation (P.ref_accum): the kept columns of X in kept
// order, 256-padded (xk), with each kept feature's float32 recip and
// discreteness as the reference's kernels read them (MultiSURF.py:184-187,
// ReliefF.py:151-154), and a flag per 256-feature block that holds a
// discrete one.  Layout buffers: rebuilt with the feature subset.
// SURF (float64 X, SURF.py:330-332): the same in float64, 128-padded, one
// flag per 128-feature block (k_surf_chains' width).
static int ref_layout(Plan* g) {
  const Prepared& Q = g->P;
  const bool surf = Q.algo == ALGO_SURF;
  if (g->x_is_f64 != (surf ? 1 : 0)) {
    set_error("reference-order accumulation: float32 X for MultiSURF / ReliefF, float64 for SURF");
    return FS_ENOTSUP;
  }
  const int64_t blk_w = surf ? 128 : 256;
  g->Kp = (Q.n_kept + blk_w - 1) / blk_w * blk_w;
  std::vector<float> rec((size_t)g->Kp, 0.0f);
  std::vector<uint8_t> dsc((size_t)g->Kp, 0), blk((size_t)(g->Kp / blk_w), 0);
  for (int64_t k = 0; k < Q.n_kept; k++) {
    const int64_t col = Q.kept_col[k];
    rec[k] = Q.recip_in[col];
    dsc[k] = Q.disc_in[col] ? 1 : 0;
    if (dsc[k]) blk[k / blk_w] = 1;
  }
  g->alloc_target = 1;
  g->xk = nullptr;
  g->xk64 = nullptr;
  int rc;
  if ((rc = surf ? dalloc(g, &g->xk64, (size_t)Q.n_pad * g->Kp)
                 : dalloc(g, &g->xk, (size_t)Q.n_pad * g->Kp)) ||
      (rc = dalloc(g, &g->kcol, Q.n_kept)) || (rc = dalloc(g, &g->krecip, g->Kp)) ||
      (rc = dalloc(g, &g->kdisc, g->Kp)) || (rc = dalloc(g, &g->kblk, g->Kp / blk_w))) {
    g->alloc_target = 0;
    return rc;
  }
  g->alloc_target = 0;
  if ((rc = h2d(g, g->kcol, Q.kept_col.data(), Q.n_kept)) ||
      (rc = h2d(g, g->krecip, rec.data(), rec.size())) ||
      (rc = h2d(g, g->kdisc, dsc.data(), dsc.size())) ||
      (rc = h2d(g, g->kblk, blk.data(), blk.size())))
    return rc;
  rc = surf ? refacc::gather_kept64((const double*)g->x, Q.n, Q.n_pad, Q.p_in, g->kcol, Q.n_kept,
                                    g->Kp, g->xk64, g->stream)
            : refacc::gather_kept((const float*)g->x, Q.n, Q.n_pad, Q.p_in, g->kcol, Q.n_kept,
                                  g->Kp, g->xk, g->stream);
  if (rc == FS_OK) FS_HIP(hipStreamSynchronize(g->stream));  // host vectors above
  return rc;
}

// Rows exact_thresholds fixes per select, from the current layout's feature
// count (both backends use exact_thr_rows(n, pc + pd) of the layout in use,
// a TuRF refit with fewer features may fix more rows); the
// partials buffer grows with it.
static int size_exact_rows(Plan* g) {
  const Prepared& Q = g->P;
  if (Q.algo != ALGO_MULTISURF) return FS_OK;
  g->thr_rows = (int)(g->thr_all ? Q.n : exact_thr_rows(Q.n, Q.pc + Q.pd));
  const int64_t nchunk = (Q.n + kExChunk - 1) / kExChunk;
  const size_t need = (size_t)g->thr_rows * nchunk;
  if (need <= g->uparts_cap) return FS_OK;
  if (g->uparts) {
    g->owned.erase(std::remove(g->owned.begin(), g->owned.end(), (void*)g->uparts),
                   g->owned.end());
    dev_free(g->uparts);
    g->uparts = nullptr;
  }
  FS_TRY(dalloc(g, &g->uparts, need));
  g->uparts_cap = need;
  return FS_OK;
}

int plan_layout(Plan* g) {
  Prepared& Q = g->P;
  g->corr_ready = false;
  FS_HIP(hipStreamSynchronize(g->stream));
  if (g->side) FS_HIP(hipStreamSynchronize(g->side));
  if (g->side2) FS_HIP(hipStreamSynchronize(g->side2));
  for (void* q : g->owned_layout) dev_free(q);
  g->owned_layout.clear();
  int rc;
  Q.q16 = g->use_q16;
  if (!Q.ranges_ready) {
    // continuous column ranges, measured on the device once per plan
    const size_t esz = g->x_is_f64 ? 8 : 4;
    if (g->colmin.empty()) {
      g->colmin.resize((size_t)Q.p_in * esz);
      g->colmax.resize((size_t)Q.p_in * esz);
      // a staged copy's extrema were taken while it was cast (stage_x_cast)
      if (!(g->x_staged && staged_extrema(g->x_staged, g->colmin.data(), g->colmax.data()))) {
        if ((rc = column_minmax(g->x, g->x_is_f64, Q.n, Q.p_in, g->colmin.data(),
                                g->colmax.data(), g->stream))) {
          g->colmin.clear();
          return rc;
        }
        trace_mark("plan: device ranges");
      }
    }
    std::vector<double> cmin((size_t)Q.pc), cmax((size_t)Q.pc);
    for (int64_t c = 0; c < Q.pc; c++) {
      const int64_t col = Q.src_col[c];
      cmin[c] = g->x_is_f64 ? ((const double*)g->colmin.data())[col]
                            : (double)((const float*)g->colmin.data())[col];
      cmax[c] = g->x_is_f64 ? ((const double*)g->colmax.data())[col]
                            : (double)((const float*)g->colmax.data())[col];
    }
    if (finalize_scale(Q, cmin.data(), cmax.data())) return FS_EINVAL;
  } else if (set_integer_scale(Q, Q.q16)) {
    // the integer scale of the operand width in use (a plan switched to
    // 32-bit operands by plan_decision_guard keeps its ranges)
    return FS_EINVAL;
  }
  g->key_shift = colsort_key_shift(Q.qmax);
  g->alloc_target = 1;
  rc = FS_OK;
  if ((rc = dalloc(g, &g->src_col, Q.PW)) || (rc = dalloc(g, &g->out_pos, Q.PW)) ||
      (rc = dalloc(g, &g->off, Q.PW)) || (rc = dalloc(g, &g->qs, Q.PW)) ||
      (rc = dalloc(g, &g->scl, Q.PW)) || (rc = dalloc(g, &g->scl32, Q.PW)) ||
      (rc = dalloc(g, &g->dtab_off, Q.PW + 1)) ||
      (rc = dalloc(g, &g->dtab, Q.dtab.size())) ||
      // xs: two spare rows (the pass-2 B prefetch runs up to two rows past a
      // tile) plus kXsSlack floats: the asm loop of a last, partial feature
      // block reads a whole block width of each B row, past the end of the
      // last row when PW is narrower than the block
      (rc = dalloc(g, &g->xs, (size_t)(Q.n_pad + 2) * Q.PW + kXsSlack)) ||
      (g->star_split && ((rc = dalloc(g, &g->xsT, (size_t)Q.PW * Q.n_pad)) ||
                         (rc = dalloc(g, &g->tcol, Q.PW))))) {
  } else if (Q.algo == ALGO_SURF) {
    // its operands follow the route the calibration picks (below)
  } else if ((rc = dalloc(g, &g->xqT, (size_t)Q.PW * Q.n_pad)) == FS_OK) {
    rc = dalloc(g, &g->epsT, (size_t)Q.PW * Q.n_pad);
  }
  g->alloc_target = 0;
  if (rc) return rc;
  if ((rc = shard_segments(g))) return rc;
  std::vector<double> qs(Q.PW, 0.0);
  for (int64_t c = 0; c < Q.PW; c++) qs[c] = Q.scale[c] * Q.SC;
  std::vector<float> scl32(Q.PW, 0.0f);
  for (int64_t c = 0; c < Q.PW; c++) scl32[c] = (float)Q.scale[c];
  g->rows_direct = !g->x_is_f64 && Q.pd == 0 && Q.pc == Q.p_in && Q.p_in % 4 == 0;
  for (int64_t c = 0; g->rows_direct && c < Q.pc; c++) g->rows_direct = Q.src_col[c] == c;
  if ((rc = h2d(g, g->src_col, Q.src_col.data(), Q.PW)) ||
      (rc = h2d(g, g->out_pos, Q.out_pos.data(), Q.PW)) ||
      (rc = h2d(g, g->off, Q.offset.data(), Q.PW)) || (rc = h2d(g, g->qs, qs.data(), Q.PW)) ||
      (rc = h2d(g, g->scl, Q.scale.data(), Q.PW)) ||
      (rc = h2d(g, g->scl32, scl32.data(), Q.PW)) ||
      (rc = h2d(g, g->dtab_off, Q.dtab_off.data(), Q.PW + 1)) ||
      (rc = h2d(g, g->dtab, Q.dtab.data(), Q.dtab.size())))
    return rc;
  if ((rc = size_exact_rows(g))) return rc;
  if (Q.ref_accum && (rc = ref_layout(g))) return rc;
  if ((rc = calibrate_band(g))) return rc;
  if (Q.algo == ALGO_SURF) {  // integer (u32) or float64 feature-major operands
    g->alloc_target = 1;
    rc = g->surf_int ? dalloc(g, &g->xqT, (size_t)Q.PW * Q.n_pad)
                     : dalloc(g, &g->xT64, (size_t)Q.PW * Q.n_pad);
    g->alloc_target = 0;
    if (rc) return rc;
  }
  if ((rc = row_guard(g))) return rc;
  if (g->calib[5] != 0.0 && (rc = apply_operand_width(g))) return rc;
  FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

int apply_operand_width(Plan* g) {
  // the coherence guard switched to 32-bit operands: new scale and sort key
  const Prepared& Q = g->P;
  std::vector<double> qs(Q.PW, 0.0);
  for (int64_t c = 0; c < Q.PW; c++) qs[c] = Q.scale[c] * Q.SC;
  g->key_shift = colsort_key_shift(Q.qmax);
  FS_TRY(h2d(g, g->qs, qs.data(), Q.PW));
  FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

// Everything sized by the plan's owned tiles: the tile list, the distance
// planes (tiled for MultiSURF: one 128 x 128 block per tile), the K-split,
// row-moment partials and the pass-2 weights.  Called by plan_create and
// again by plan_set_shard, which frees the previous shard's buffers first.
static int setup_shard(Plan* g, const std::vector<int32_t>& bi, const std::vector<int32_t>& bj) {
  const Prepared& Q = g->P;
  g->n_tiles = (int64_t)bi.size();
  std::vector<int2> tl(g->n_tiles);
  for (int64_t t = 0; t < g->n_tiles; t++) tl[t] = make_int2(bi[t], bj[t]);
  g->h_tiles = tl;
  // MultiSURF reads distances only inside owned tiles: tiled layout, one
  // 128 x 128 block per owned tile (half the full matrix at world 1, 1/N of
  // the tiles per rank).  ReliefF / SURF select neighbours over whole rows.
  g->tiled = (Q.algo == ALGO_MULTISURF && !g->row_mode) ? 1 : 0;
  // ReliefF / SURF: the rows of the plan's focal 128-sample blocks only
  // (d_row_in): a whole fit holds n_pad^2, one rank of an N-way row split or
  // one row panel (rows_run_panels) its share
  if (g->tiled) {
    g->win = make_int2(0, 0);
  } else {
    const int64_t w0 = g->row_mode ? g->r_lo / kTile * kTile : 0;
    const int64_t w1 = g->row_mode ? std::min<int64_t>(Q.n_pad, (g->r_hi + kTile - 1) / kTile * kTile)
                                   : Q.n_pad;
    g->win = make_int2((int)w0, (int)std::max(w0, w1));
  }
  g->dplane = g->tiled ? std::max<int64_t>(g->n_tiles, 1) * kTile * kTile
                       : std::max<int64_t>((int64_t)(g->win.y - g->win.x), 1) * Q.n_pad;
  g->tw = g->tiled ? make_int2((int)g->nb, g->world) : make_int2(0, 0);
  // pass-1 chunk count and the per-tile work in feature units of 32-bit SAD
  const int64_t rows_q = (g->use_q16 ? Q.PC / 2 : Q.PC) + Q.PD;
  g->ksplit = choose_ksplit(g->n_tiles, g->device, (int)(rows_q / kBKQ),
                            (g->use_q16 ? Q.pc / 2 : Q.pc) + Q.pd,
                            Q.algo == ALGO_MULTISURF && Q.pc > 0);
  if (test_hooks().ksplit >= 1) g->ksplit = (int)std::min<int64_t>(16, test_hooks().ksplit);
  // SURF: its integer route splits k_dist's tiles like MultiSURF's (the
  // float64 route, k_dist_f64, has no K-split and ignores it)
  // ReliefF stores float32 keys (Dk), formed in k_dist's epilogue from whole
  // tiles: no K-split (partial sums cannot be keyed before they are added)
  const bool dkeys = Q.algo == ALGO_RELIEFF;
  if (dkeys) g->ksplit = 1;
  g->kfull = g->ksplit > 1 ? 0 : g->n_tiles;  // k_dist can split only a tail; all or none here
  g->alloc_target = 3;
  int rc = FS_OK;
  g->Dk = nullptr;
  if ((rc = dkeys ? dalloc(g, (float**)&g->D_alloc, (size_t)g->dplane)
                  : dalloc(g, (double**)&g->D_alloc, (size_t)g->dplane)) ||
      (dkeys ? (g->Dk = (float*)g->D_alloc - (int64_t)g->win.x * Q.n_pad, g->D = nullptr)
             : (g->D = (double*)g->D_alloc - (g->tiled ? 0 : (int64_t)g->win.x * Q.n_pad)),
       false) ||
      (rc = dalloc(g, &g->tiles, g->n_tiles)) ||
      (rc = dalloc(g, &g->rspart, (size_t)std::max<int64_t>(g->n_tiles, 1) * 256))) {
  } else if (Q.algo != ALGO_RELIEFF && !g->sparse) {
    rc = dalloc(g, &g->Wt, (size_t)(g->n_tiles + 1) * kTile * kTile);
  } else if (g->sparse) {
    // One spare tile: k_score_sparse prefetches two groups past the end of a
    // stream.  Zeroed once, so such reads (and stream tails never written)
    // hold in-range row offsets.
    const size_t count = (size_t)(g->n_tiles + 1) * kSWaves * kStreamEntries;
    if (!(rc = dalloc(g, &g->ent, count)) && !(rc = dalloc(g, &g->nnz, 1)) &&
        hipMemsetAsync(g->ent, 0, sizeof(uint2) * count, g->stream) != hipSuccess)
      rc = FS_EHIP;
  }
  if (!rc && g->ksplit > 1)
    rc = dalloc(g, &g->Dpart,
                (size_t)(g->n_tiles - g->kfull) * (g->ksplit - 1) * kTile * kTile);
  g->alloc_target = 0;
  if (rc) return rc;
  g->nnz_valid = false;
  return h2d(g, g->tiles, tl.data(), g->n_tiles);
}

int plan_set_shard(Plan* g, int rank, int world) {
  if (g->P.algo != ALGO_MULTISURF || g->row_mode) {
    set_error("tile shards of a plan are MultiSURF-only");
    return FS_EINVAL;
  }
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("invalid shard rank/world");
    return FS_EINVAL;
  }
  FS_HIP(hipSetDevice(g->device));
  FS_HIP(hipStreamSynchronize(g->stream));
  if (g->side) FS_HIP(hipStreamSynchronize(g->side));
  if (g->side2) FS_HIP(hipStreamSynchronize(g->side2));
  for (void* q : g->owned_shard) dev_free(q);
  g->owned_shard.clear();
  g->D = g->Dpart = nullptr;
  g->D_alloc = nullptr;
  g->Wt = nullptr;
  g->ent = nullptr;
  g->tiles = nullptr;
  g->rspart = nullptr;
  g->nnz = nullptr;
  g->rank = rank;
  g->world = world;
  std::vector<int32_t> bi, bj;
  owned_tiles(g->nb, rank, world, bi, bj);
  FS_TRY(setup_shard(g, bi, bj));
  return shard_segments(g);  // pass-2 segments and this shard's mean-correction columns
}

int plan_create(Plan** out, const Prepared& P, const void* x, int x_is_f64, int device,
                int rank, int world, uint64_t stream, int64_t r_lo, int64_t r_hi) {
  *out = nullptr;
  const int ndev = device_count();
  if (ndev <= 0) {
    set_error("backend='gpu' requested but no HIP device is visible");
    return FS_ENODEV;
  }
  if (device < 0 || device >= ndev) {
    set_error("device ordinal out of range");
    return FS_EINVAL;
  }
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("invalid rank/world");
    return FS_EINVAL;
  }
  if (P.n >= (1 << 20)) {  // k_colrank's packed histogram; D alone would be 8 TB
    set_error("the GPU backend supports fewer than 2^20 samples");
    return FS_ENOTSUP;
  }
  const bool row_mode = r_hi >= 0;
  if (row_mode && !(0 <= r_lo && r_lo <= r_hi && r_hi <= P.n)) {
    set_error("row range outside [0, n)");
    return FS_EINVAL;
  }
  FS_HIP(hipSetDevice(device));
  Plan* g = new Plan();
  g->P = P;
  g->device = device;
  g->rank = rank;
  g->world = world;
  g->x_is_f64 = x_is_f64;
  if (stream) {
    g->stream = (hipStream_t)(uintptr_t)stream;
  } else {
    if (!(g->stream = stream_get(device))) {
      delete g;
      return FS_EHIP;
    }
    g->own_stream = true;
  }
  auto fail = [&](int rc) {
    plan_destroy(g);
    return rc;
  };
  for (auto& e : g->ev)
    if (!(e = event_get(device, true))) return fail(FS_EHIP);
  if (!(g->side = stream_get(device)) || !(g->ev_fork = event_get(device, false)) ||
      !(g->ev_join = event_get(device, false)) || !(g->ev_star = event_get(device, false)))
    return fail(FS_EHIP);
  const Prepared& Q = g->P;
  g->nb = Q.n_pad / kTile;
  std::vector<int32_t> bi, bj;
  if (row_mode) {
    g->r_lo = r_lo;
    g->r_hi = r_hi;
    if (r_hi > r_lo) row_tiles(g->nb, r_lo / kTile, (r_hi + kTile - 1) / kTile, bi, bj);
  } else {
    g->r_lo = 0;
    g->r_hi = Q.n;
    owned_tiles(g->nb, rank, world, bi, bj);
  }
  g->row_mode = row_mode;
  // (ReliefF refines in k_rf_select and uses only the counter)
  g->list_cap = Q.algo == ALGO_RELIEFF ? 1 : std::max<int64_t>(1 << 16, Q.n * 64);
  g->use_q16 = choose_q16(Q);
  const size_t xbytes = (size_t)Q.n * Q.p_in * (x_is_f64 ? 8 : 4);
  int rc;
  trace_mark("plan: host setup");
  // the library's staged copy of X (fs_stage_x, fs_stage_x_cast) is read in
  // place, else X is copied from a caller's staged copy or uploaded
  g->x_staged = staged_acquire(x, Q.n, Q.p_in, x_is_f64, g->device);
  if (g->x_staged) g->x = const_cast<void*>(g->x_staged);
  if ((!g->x_staged && (rc = dalloc(g, (char**)&g->x, xbytes))) ||
      (rc = dalloc(g, &g->lab, Q.n_pad)) ||
      (rc = dalloc(g, &g->corr, Q.n_pad)) ||
      (rc = dalloc(g, &g->corr_part, (int64_t)kRowcorrMaxSlices * Q.n_pad)) ||
      (rc = dalloc(g, &g->thr, Q.n_pad)) ||
      (rc = dalloc(g, &g->list, g->list_cap)) || (rc = dalloc(g, &g->list_count, 1)))
    return fail(rc);
  if (Q.algo == ALGO_MULTISURF) {
    // test hook: every row's threshold from exact distances (the machinery
    // of exact_thresholds checked on all rows against the oracle's)
    g->thr_all = test_hooks().thr_exact_all != 0;
    // thr_rows and uparts: size_exact_rows (plan_layout, per feature layout)
    g->thr_rows = (int)(g->thr_all ? Q.n : exact_thr_rows(Q.n, Q.pc + Q.pd));
    if ((rc = dalloc(g, &g->unc, Q.n_pad)) || (rc = dalloc(g, &g->urows, Q.n_pad + 1)))
      return fail(rc);
    // reference-order accumulation: exact_thresholds' batch counts (every
    // flagged row is fixed, in batches of thr_rows).  thr_rows changes with
    // the feature layout (size_exact_rows) but never falls below
    // kExactThrRows, so n / kExactThrRows + 2 batches cover every layout a
    // later fs_plan_set_features may choose.  The decision masks
    // (n_pad^2 / 2 bytes) are allocated on first use by the one-device pass 2
    // (ref_masks): a multi-rank job writes into its own all-reduced buffer.
    if (Q.ref_accum &&
        (rc = dalloc(g, &g->bcnt, (size_t)(Q.n / kExactThrRows + 2))))
      return fail(rc);
  }
  g->star_split = choose_star_split(Q, device);
  g->sparse = choose_sparse(g, Q);
  if (g->star_split && (rc = dalloc(g, &g->alpha, Q.n_pad))) return fail(rc);
  if (g->star_split && Q.algo == ALGO_MULTISURF && !(g->side2 = stream_get(device)))
    return fail(FS_EHIP);
  if ((rc = setup_shard(g, bi, bj))) return fail(rc);
  trace_mark("plan: hipMalloc");
  std::vector<int32_t> lab(Q.n_pad, -1);
  std::copy(Q.labels.begin(), Q.labels.end(), lab.begin());
  // a caller-owned staged copy (fs_stage_x_device) is copied: its owner may
  // free it while the plan lives
  const void* sx = g->x_staged ? nullptr : staged_lookup(x, Q.n, Q.p_in, x_is_f64, g->device);
  if (sx && hipMemcpyAsync(g->x, sx, xbytes, hipMemcpyDeviceToDevice, g->stream) != hipSuccess) {
    (void)hipGetLastError();
    set_error("plan: device-to-device copy of the staged X failed");
    return fail(FS_EHIP);
  }
  if ((!g->x_staged && !sx && (rc = h2d(g, (char*)g->x, (const char*)x, xbytes))) ||
      (rc = h2d(g, g->lab, lab.data(), Q.n_pad)))
    return fail(rc);
  if (Q.algo == ALGO_RELIEFF) {
    std::vector<uint8_t> lab8((size_t)Q.n_pad + 16, 0);
    for (int64_t j = 0; j < Q.n; j++) lab8[j] = (uint8_t)Q.labels[j];
    if ((rc = dalloc(g, &g->lab8, lab8.size())) || (rc = h2d(g, g->lab8, lab8.data(), lab8.size())))
      return fail(rc);
  }
  if ((rc = plan_layout(g))) return fail(rc);
  trace_mark("plan: H2D + layout");
  *out = g;
  return FS_OK;
}

int plan_set_features(Plan* g, const Prepared& P) {
  FS_HIP(hipSetDevice(g->device));
  g->P = P;
  g->ref_rows = -1;  // temp rows of the old feature layout
  return plan_layout(g);
}

int plan_set_rows(Plan* g, int64_t r_lo, int64_t r_hi) {
  if (g->P.algo != ALGO_MULTISURF) {
    set_error("focal-row slices of a plan are MultiSURF-only (ReliefF / SURF: row plans)");
    return FS_EINVAL;
  }
  g->r_lo = r_lo;
  g->r_hi = r_hi;
  return FS_OK;
}

int plan_info(const Plan* g, int64_t* tiles, double* pfe, int64_t* refined) {
  if (tiles) *tiles = g->n_tiles;
  if (pfe) {
    // pairs visited by both passes (diagonal tiles count their full 128x128
    // pass-1 work) x real features
    *pfe = 2.0 * (double)g->n_tiles * kTile * kTile * (double)(g->P.pc + g->P.pd);
  }
  if (refined) *refined = g->n_refined;
  return FS_OK;
}

int plan_calibration(const Plan* g, double* out) {
  for (int k = 0; k < 7; k++) out[k] = g->calib[k];
  out[7] = g->P.SC;
  return FS_OK;
}

int plan_weighted_pairs(Plan* g, int64_t* pairs) {
  *pairs = -1;
  if (!g->sparse || !g->nnz_valid) return FS_OK;
  FS_HIP(hipSetDevice(g->device));
  unsigned long long v = 0;
  FS_HIP(hipMemcpyAsync(&v, g->nnz, sizeof(v), hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  *pairs = (int64_t)v;
  return FS_OK;
}

double plan_kernel_ms(const Plan* g, int which) {
  float ms = -1.0f;
  if (which < 0 || which > 2) return -1.0;
  hipEvent_t a = g->ev[2 * which], b = g->ev[2 * which + 1];
  if (hipEventSynchronize(b) != hipSuccess || hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();
    return -1.0;
  }
  return (double)ms;
}

// ---- one-shot runs --------------------------------------------------------

static int finish_scores(Plan* g, double* scores_dev, float* scores_out) {
  const Prepared& Q = g->P;
  std::vector<double> h(Q.n_kept);
  FS_HIP(hipMemcpyAsync(h.data(), scores_dev, sizeof(double) * Q.n_kept, hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  for (int64_t k = 0; k < Q.n_kept; k++) scores_out[k] = (float)(h[k] / (double)Q.n);
  return FS_OK;
}

// Tile shards a device needs for a MultiSURF job of `world` ranks: the
// tile-sized buffers (~260 KB per tile: the tiled distance block, the
// pass-2 weight streams, partials) of a rank's 1/world of the n_pad^2/2/128^2
// tiles, against the free device memory left after the per-sample buffers
// (X, quantised operands, pass-2 operands, correction terms: ~16 n PW
// bytes) and a 15% reserve.  1 when everything fits; the shards test hook
// forces it.
int multisurf_shards(const Prepared& P, int device, int world, int share) {
  if (test_hooks().shards >= 1) return (int)std::min<int64_t>(test_hooks().shards, 4096);
  size_t free_b = 0, total_b = 0;
  if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return 1;
  }
  const int64_t nb = P.n_pad / kTile;
  const double tiles = (double)nb * (nb + 1) / 2.0 / (double)std::max(world, 1);
  const double per_tile = 2.0 * kTile * kTile * 8.0 + 8.0 * kTile * 256.0 / 2.0;
  const double fixed = 16.0 * (double)P.n_pad * (double)P.PW + 8.0 * (double)P.n * 64.0;
  const double avail = 0.85 * (double)free_b / (double)std::max(share, 1) - fixed;
  if (avail <= 0.0) return 1;  // not even the samples fit: let the allocation report it
  const double v = std::ceil(tiles * per_tile / avail);
  return (int)std::max(1.0, std::min(v, 4096.0));
}

// One MultiSURF scoring pass on a single device in V tile shards (V > 1 when
// the tile buffers of the whole triangle exceed the device: n beyond HBM).
// The distances of a shard are recomputed in each of the three rounds (row
// moments; thresholds -> refinement -> neighbour counts; weights -> pass 2),
// because no shard's distances are kept while another shard runs: 3x the
// pass-1 work for O(n p + n^2 / V) device memory.  The reference streams
// each focal sample's distance row the same way (MultiSURF.py:174-214).
// V == 1 is the plain pass1 / select / pass2 sequence.
static int run_multisurf_shards(Plan* g, int shards, int rank, int world, double* rs, double* cnt,
                                double* sc) {
  const Prepared& Q = g->P;
  if (shards <= 1) {
    FS_TRY(plan_pass1(g, rs));
    FS_TRY(plan_select(g, rs, cnt));
    return plan_pass2(g, cnt, sc);
  }
  double *rs_v = nullptr, *cnt_v = nullptr, *sc_v = nullptr;
  FS_TRY(dalloc(g, &rs_v, 3 * Q.n));
  FS_TRY(dalloc(g, &cnt_v, 2 * Q.n));
  FS_TRY(dalloc(g, &sc_v, Q.n_kept));
  const int W = world * shards;
  auto add = [&](double* dst, const double* src, int64_t count, bool first) -> int {
    if (first)
      return hipMemcpyAsync(dst, src, sizeof(double) * count, hipMemcpyDeviceToDevice,
                            g->stream) == hipSuccess
                 ? FS_OK
                 : FS_EHIP;
    return accumulate(dst, src, count, g->stream);
  };
  for (int v = 0; v < shards; v++) {  // round 1: row moments
    FS_TRY(plan_set_shard(g, rank + world * v, W));
    FS_TRY(plan_pass1(g, rs_v));
    FS_TRY(add(rs, rs_v, 3 * Q.n, v == 0));
  }
  for (int v = 0; v < shards; v++) {  // round 2: thresholds, refinement, counts
    FS_TRY(plan_set_shard(g, rank + world * v, W));
    FS_TRY(plan_pass1(g, rs_v));
    FS_TRY(plan_select(g, rs, cnt_v));
    FS_TRY(add(cnt, cnt_v, 2 * Q.n, v == 0));
  }
  if (Q.ref_accum) {
    // reference order: every shard's decisions into the masks, then the
    // chains of all focal rows once (one device holds the whole job here)
    if (world != 1) {
      set_error("reference-order accumulation: one device per job in the one-shot calls");
      return FS_ENOTSUP;
    }
    for (int v = 0; v < shards; v++) {
      FS_TRY(plan_set_shard(g, rank + world * v, W));
      FS_TRY(plan_pass1(g, rs_v));
      FS_TRY(plan_select(g, rs, cnt_v));
      FS_TRY(ref_masks(g));
    }
    return ref_chains(g, cnt, sc);
  }
  for (int v = 0; v < shards; v++) {  // round 3: weights, pass 2
    FS_TRY(plan_set_shard(g, rank + world * v, W));
    FS_TRY(plan_pass1(g, rs_v));
    FS_TRY(plan_select(g, rs, cnt_v));
    FS_TRY(plan_pass2(g, cnt, sc_v));
    FS_TRY(add(sc, sc_v, Q.n_kept, v == 0));
  }
  return FS_OK;
}

// Decision risk of a MultiSURF score vector computed with 16-bit pass-1
// operands.  Their thresholds mu - sigma/2 take mu exactly (the quantised row
// sums minus the exact mean correction, fs_colsort.hip) but sigma from the
// quantised second moment: with pair errors e_ij of std sqrt(pc/6) quanta,
// independent of D_ij, sigma_q - sigma = cov_j(D_ij - mu_i, e_ij) / sigma_i
// has std ~ sqrt(pc/6) / sqrt(n) quanta, so T_i errs by about half that
// (kQ16ThrErr keeps a factor 2 of margin: sqrt(pc/6 + 1) / sqrt(n)).  Every
// pair whose exact distance lies between the two thresholds is decided
// differently from MultiSURF.py:193-217.  Row i holds ~ n * phi(1/2) / sigma_i
// such pairs per quantum of T error (Gaussian row distances, phi(1/2) =
// 0.352); each moves one sample across its near boundary, changing the row's
// hit or miss average by ~ dbar / m_i (m_i = the smaller of its near hit /
// miss counts, dbar the mean per-feature diff from the rows' mean distances,
// x2 for the features above the mean), i.e. the final score (divided by n)
// by dbar / (n m_i).  With random signs the expected score error is
// sqrt(sum_i flips_i * effect_i^2); the risk is that over max |score|.
// Measured against the oracle (tests/test_gpu_families.py): uniform noise
// with unrelated labels, n = 16384, is signal-free and trips it; cfg4
// (make_classification) does not.  Above kQ16MaxRisk a MultiSURF plan
// re-scores on 32-bit operands (plan_decision_guard).
constexpr double kQ16MaxRisk = 5e-6;
thread_local double g_last_risk = -1.0;
thread_local int g_last_rerun = 0;

// The risk above, on the device (q16_decision_risk): the step's exchange
// vectors stay in HBM and one double comes back (until round 5 three
// pageable copies of 5n + p doubles went to a host loop, ~0.15 ms of every
// cfg4 step).  One 256-thread workgroup; every sum is a fixed-order block
// reduction (block_sum_256), so every rank, holding the same all-reduced
// vectors, computes the same risk.
__global__ __launch_bounds__(256) void q16_decision_risk(const double* __restrict__ rs,
                                                       const double* __restrict__ cnt,
                                                       const double* __restrict__ sums, int64_t n64,
                                                       int64_t n_kept, double pc, double nfeat,
                                                       double SC, double* __restrict__ out) {
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const double n = (double)n64, nm1 = n - 1.0;
  double m = 0.0;
  for (int64_t k = tid; k < n_kept; k += 256) m = fmax(m, (double)fabsf((float)(sums[k] / n)));
  red[tid] = m;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) red[tid] = fmax(red[tid], red[tid + st]);
    __syncthreads();
  }
  const double smax = red[0];
  __syncthreads();
  if (n < 3.0 || nfeat <= 0.0 || SC <= 0.0) {
    if (tid == 0) out[0] = 0.0;
    return;
  }
  if (smax <= 0.0) {
    if (tid == 0) out[0] = HUGE_VAL;
    return;
  }
  double mu = 0.0;
  for (int64_t i = tid; i < n64; i += 256) mu += (rs[3 * i] - rs[3 * i + 2]) / nm1;
  const double mu_sum = block_sum_256(mu, red);
  const double thr_err = sqrt(pc / 6.0 + 1.0) / sqrt(n);
  const double dbar = 2.0 * mu_sum / n / (SC * nfeat);
  double acc = 0.0;
  for (int64_t i = tid; i < n64; i += 256) {
    const double mi = rs[3 * i] / nm1, var = rs[3 * i + 1] / nm1 - mi * mi;
    if (!(var > 0.0)) continue;
    const double flips = n * 0.352 * thr_err / sqrt(var);
    const double mm = fmax(1.0, fmin(cnt[2 * i], cnt[2 * i + 1]));
    const double eff = dbar / (n * mm);
    acc += flips * eff * eff;
  }
  acc = block_sum_256(acc, red);
  if (tid == 0) out[0] = sqrt(acc) / smax;
}

// After a MultiSURF step with 16-bit operands: the decision risk from the
// step's exchange vectors (rowstats[3n], counts[2n], score sums[n_kept],
// device memory, summed over every rank and shard -- so every rank computes
// the same risk and decides alike).  Above kQ16MaxRisk the plan is switched
// to 32-bit operands for good (its layout and shard rebuilt; X stays on the
// device) and *switched = 1: the caller runs the step again.  risk = -1 when
// there is nothing to check (32-bit operands, MultiSURF*, the q16 test hook).
int plan_decision_guard(Plan* g, const double* rowstats, const double* counts,
                        const double* sums, double* risk, int* switched) {
  *risk = -1.0;
  *switched = 0;
  const Prepared& Q = g->P;
  // reference order: every flagged row's threshold is exact, nothing to model
  if (Q.algo != ALGO_MULTISURF || !g->use_q16 || Q.use_star || Q.ref_accum ||
      test_hooks().q16 >= 0)
    return FS_OK;
  // a focal-row slice holds only its rows' partial sums: as the one-shot
  // slice calls (multisurf_rows, a partial multisurf_run_devices), no check
  // (max |score| of a partial sum would inflate the risk)
  if (g->r_lo != 0 || g->r_hi != Q.n) return FS_OK;
  FS_HIP(hipSetDevice(g->device));
  if (!g->risk_dev) FS_TRY(dalloc(g, &g->risk_dev, 1));  // owned: lives as long as the plan
  q16_decision_risk<<<1, 256, 0, g->stream>>>(rowstats, counts, sums, Q.n, Q.n_kept,
                                              (double)Q.pc, (double)(Q.pc + Q.pd), Q.SC,
                                              g->risk_dev);
  FS_TRY(launch_check("q16_decision_risk"));
  double r = 0.0;
  FS_HIP(hipMemcpyAsync(&r, g->risk_dev, sizeof(double), hipMemcpyDeviceToHost, g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  *risk = r;
  if (!(*risk > kQ16MaxRisk)) return FS_OK;
  trace_mark("multisurf: 16-bit decision risk above bound, 32-bit operands");
  g->use_q16 = 0;
  g->P.no_q16 = 1;
  FS_TRY(plan_layout(g));
  FS_TRY(plan_set_shard(g, g->rank, g->world));
  *switched = 1;
  return FS_OK;
}

int multisurf_last_guard(double* risk, int* rerun) {
  if (risk) *risk = g_last_risk;
  if (rerun) *rerun = g_last_rerun;
  return FS_OK;
}

int multisurf_run(const Prepared& P, const void* x, int device, float* scores_out) {
  Plan* g = nullptr;
  g_last_risk = -1.0;
  g_last_rerun = 0;
  const int shards = multisurf_shards(P, device, 1);
  Prepared Q = P;
  Q.defer_guard = 1;  // decided beside the first pass 1 (row_guard)
  FS_TRY(plan_create(&g, Q, x, 0, device, 0, shards, 0));
  double *rs = nullptr, *cnt = nullptr, *sc = nullptr;
  int rc, switched = 0;
  double risk = -1.0;
  if ((rc = dalloc(g, &rs, 3 * P.n)) || (rc = dalloc(g, &cnt, 2 * P.n)) ||
      (rc = dalloc(g, &sc, P.n_kept)) || (rc = run_multisurf_shards(g, shards, 0, 1, rs, cnt, sc)) ||
      (rc = plan_decision_guard(g, rs, cnt, sc, &risk, &switched)) ||
      (switched && (rc = run_multisurf_shards(g, shards, 0, 1, rs, cnt, sc))) ||
      (rc = finish_scores(g, sc, scores_out))) {
    plan_destroy(g);
    return rc;
  }
  g_last_risk = risk;
  g_last_rerun = switched;
  plan_destroy(g);
  return FS_OK;
}

int copy_sums(Plan* g, const double* sums_dev, double* sums_out) {
  FS_HIP(hipMemcpyAsync(sums_out, sums_dev, sizeof(double) * g->P.n_kept, hipMemcpyDeviceToHost,
                        g->stream));
  FS_HIP(hipStreamSynchronize(g->stream));
  return FS_OK;
}

int multisurf_rows(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                   double* sums_out) {
  Plan* g = nullptr;
  const int shards = multisurf_shards(P, device, 1);
  FS_TRY(plan_create(&g, P, x, 0, device, 0, shards, 0));
  double *rs = nullptr, *cnt = nullptr, *sc = nullptr;
  int rc;
  if ((rc = plan_set_rows(g, r_lo, r_hi)) || (rc = dalloc(g, &rs, 3 * P.n)) ||
      (rc = dalloc(g, &cnt, 2 * P.n)) || (rc = dalloc(g, &sc, P.n_kept)) ||
      (rc = run_multisurf_shards(g, shards, 0, 1, rs, cnt, sc)) ||
      (rc = copy_sums(g, sc, sums_out))) {
    plan_destroy(g);
    return rc;
  }
  plan_destroy(g);
  return FS_OK;
}

// Rows per panel of a ReliefF / SURF one-shot call: a plan stores the
// distance rows of its focal blocks (d_row_in), ~n_pad * 8 bytes per row plus
// its share of the pass-2 weights and selection scratch (~n_pad * 16 more),
// beside the per-sample buffers (X, the quantised and pass-2 operands:
// ~20 n_pad PW bytes).  Focal ranges whose rows exceed 80% of the free
// device memory are scored in panels of whole 128-sample blocks, one plan
// each, and their sums added -- the reference streams each focal sample's
// distance row the same way (ReliefF.py:143-157, SURF.py:139-163).
// The row_panel test hook forces the panel height.
static int64_t row_panel_rows(const Prepared& P, int device, int64_t rows) {
  if (const int64_t e = test_hooks().row_panel; e >= 1)
    return std::max<int64_t>(kTile, e / kTile * kTile);
  size_t free_b = 0, total_b = 0;
  if (hipSetDevice(device) != hipSuccess || hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
    (void)hipGetLastError();
    return rows;
  }
  const double fixed = 20.0 * (double)P.n_pad * (double)P.PW + 8.0 * (double)P.n * (double)P.p_in;
  // a stored row of D (8 bytes per sample; ReliefF's float32 keys 4) plus
  // the per-row scratch
  const double per_row = (P.algo == ALGO_RELIEFF ? 20.0 : 24.0) * (double)P.n_pad;
  const double avail = 0.8 * (double)free_b - fixed;
  if (avail <= per_row * kTile) return kTile;  // let the allocation report it
  const int64_t fit = (int64_t)(avail / per_row) / kTile * kTile;
  return std::max<int64_t>(kTile, std::min<int64_t>(fit, (rows + kTile - 1) / kTile * kTile));
}

// Score [r_lo, r_hi) in panels of `panel` rows (block-aligned), summing the
// panels' float64 sums in panel order.
template <typename Fn>
static int run_panels(const Prepared& P, int64_t r_lo, int64_t r_hi, int64_t panel,
                      double* sums_out, Fn&& one) {
  std::fill(sums_out, sums_out + P.n_kept, 0.0);
  std::vector<double> part((size_t)P.n_kept);
  for (int64_t lo = r_lo; lo < r_hi;) {
    const int64_t hi = std::min(r_hi, (lo / kTile * kTile) + panel);
    FS_TRY(one(lo, hi, part.data()));
    for (int64_t k = 0; k < P.n_kept; k++) sums_out[k] += part[k];
    lo = hi;
  }
  return FS_OK;
}

// Reference order (ReliefF / SURF): one float32 column sum over all panels,
// each panel's plan continuing the previous panel's sums (ReliefF.py:219-220,
// SURF.py:195: one sequential sum over the focal samples).
template <typename Fn>
static int run_panels_chained(const Prepared& P, const void* x, int device, int64_t r_lo,
                              int64_t r_hi, int64_t panel, double* sums_out, Fn&& one_seeded) {
  std::vector<double> prev((size_t)P.n_kept, 0.0);
  for (int64_t lo = r_lo; lo < r_hi;) {
    const int64_t hi = std::min(r_hi, (lo / kTile * kTile) + panel);
    FS_TRY(one_seeded(P, x, device, lo, hi, sums_out, lo == r_lo ? nullptr : prev.data()));
    std::copy(sums_out, sums_out + P.n_kept, prev.begin());
    lo = hi;
  }
  return FS_OK;
}

int surf_run(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
             double* sums_out) {
  const int64_t panel = row_panel_rows(P, device, r_hi - r_lo);
  if (r_hi - r_lo <= panel) return surf_run_one(P, x, device, r_lo, r_hi, sums_out);
  if (P.ref_accum) return run_panels_chained(P, x, device, r_lo, r_hi, panel, sums_out, surf_run_one);
  return run_panels(P, r_lo, r_hi, panel, sums_out, [&](int64_t lo, int64_t hi, double* o) {
    return surf_run_one(P, x, device, lo, hi, o);
  });
}

int relieff_run(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                double* sums_out) {
  const int64_t panel = row_panel_rows(P, device, r_hi - r_lo);
  if (r_hi - r_lo <= panel) return relieff_run_one(P, x, device, r_lo, r_hi, sums_out);
  if (P.ref_accum) return run_panels_chained(P, x, device, r_lo, r_hi, panel, sums_out, relieff_run_one);
  return run_panels(P, r_lo, r_hi, panel, sums_out, [&](int64_t lo, int64_t hi, double* o) {
    return relieff_run_one(P, x, device, lo, hi, o);
  });
}

int surf_run_one(const Prepared& P, const void* x, int device, int64_t r_lo, int64_t r_hi,
                 double* sums_out, const double* seed) {
  Plan* g = nullptr;
  FS_TRY(plan_create(&g, P, x, 1, device, 0, 1, 0, r_lo, r_hi));
  double* sc = nullptr;
  int rc = dalloc(g, &sc, g->P.n_kept);
  if (rc == FS_OK && seed) {
    // reference order, a later row panel: the float32 column sums go on from
    // the previous panels' (SURF.py:195 is one sequential sum)
    g->ref_seeded = true;
    rc = h2d(g, sc, seed, (size_t)g->P.n_kept);
  }
  if (rc == FS_OK) rc = plan_score_surf(g, sc);
  if (rc == FS_OK) rc = copy_sums(g, sc, sums_out);
  plan_destroy(g);
  return rc;
}

// ReliefF / SURF plans (resident scoring, fs_plan_score): float64 score sums
// of the plan's focal rows into device memory; per-call buffers are freed
// before returning.
// Reference order, row-sharded ReliefF over ranks (fs_plan_ref_temp): the
// plan's score up to its float32 temp rows; plan_ref_sums continues the
// previous rank's column sums over them.
int plan_ref_temp(Plan* g) {
  g->ref_defer = true;
  const int rc = plan_score(g, nullptr);
  g->ref_defer = false;
  return rc;
}

int plan_score(Plan* g, double* sums_dev) {
  FS_HIP(hipSetDevice(g->device));
  int rc;
  if (g->P.algo == ALGO_RELIEFF) {
    if (g->P.n_classes > 64) {
      set_error("GPU ReliefF supports at most 64 classes");
      return FS_ENOTSUP;
    }
    rc = plan_score_relieff(g, sums_dev);
  } else if (g->P.algo == ALGO_SURF) {
    rc = plan_score_surf(g, sums_dev);
  } else {
    set_error("fs_plan_score: MultiSURF plans score through pass1 / select / pass2");
    return FS_EINVAL;
  }
  if (hipStreamSynchronize(g->stream) != hipSuccess && rc == FS_OK) rc = FS_EHIP;
  for (void* q : g->scratch) dev_free(q);
  g->scratch.clear();
  return rc;
}

}  // namespace gpu
}  // namespace fs
