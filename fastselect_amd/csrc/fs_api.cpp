// fs_api.cpp -- the C ABI (include/fastselect_amd.h): argument validation,
// backend dispatch, error reporting.  See the header for the reference
// interface each entry point replaces.
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fastselect_amd.h"
#include "fs_internal.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>

namespace fs {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

static thread_local int g_accum = FS_ACCUM_FAST;
int accumulation_mode() { return g_accum; }

TestHooks& test_hooks() {
  static TestHooks h;
  return h;
}

bool trace_on() {
  static const bool on = std::getenv("FS_TRACE") != nullptr;
  return on;
}

void trace_mark(const char* phase) {
  if (!trace_on()) return;
  using clk = std::chrono::steady_clock;
  static thread_local clk::time_point last = clk::now();
  const clk::time_point now = clk::now();
  std::fprintf(stderr, "[fs_trace] %-22s %9.3f ms\n", phase,
               std::chrono::duration<double, std::milli>(now - last).count());
  last = now;
}
}  // namespace fs

using namespace fs;

static int map_prep_rc(int rc) { return rc == 0 ? FS_OK : FS_EINVAL; }

// The calling thread's accumulation mode into a prepared problem
// (fs_set_accumulation).  Reference order: MultiSURF's and ReliefF's
// per-sample sums and column sums (MultiSURF.py:198-253, ReliefF.py:181-220),
// SURF's in its n_jobs = 1 order (SURF.py:139-218: with more threads the
// reference adds its per-thread rows in schedule order); MultiSURF then
// takes 32-bit pass-1 operands.
static int apply_accumulation(Prepared& P) {
  P.ref_accum = g_accum == FS_ACCUM_REFERENCE ? 1 : 0;
  if (P.ref_accum && P.algo == ALGO_MULTISURF && !test_hooks().ref_q16) P.no_q16 = 1;
  return FS_OK;
}

static int no_reference_devices() {
  if (g_accum != FS_ACCUM_REFERENCE) return FS_OK;
  set_error("reference-order accumulation runs on one device (its column sums are one "
            "sequential float32 sum per feature)");
  return FS_ENOTSUP;
}

static int check_backend(int backend, int device) {
  if (backend != FS_BACKEND_CPU && backend != FS_BACKEND_GPU) {
    set_error("backend must be FS_BACKEND_CPU or FS_BACKEND_GPU");
    return FS_EINVAL;
  }
  if (backend == FS_BACKEND_GPU) {
    const int nd = gpu::device_count();
    if (nd <= 0) {
      set_error("backend='gpu' was selected, but no HIP device (MI355X) is visible");
      return FS_ENODEV;
    }
    if (device < 0 || device >= nd) {
      set_error("device ordinal out of range");
      return FS_EINVAL;
    }
  }
  return FS_OK;
}

// devices[0..n) for the multi-device entry points: at least one, each a
// visible HIP ordinal (repeats allowed: several plans share a device).
static int check_devices(const int* devices, int n) {
  if (!devices || n < 1) {
    set_error("devices: need at least one device ordinal");
    return FS_EINVAL;
  }
  const int nd = gpu::device_count();
  if (nd <= 0) {
    set_error("backend='gpu' was selected, but no HIP device (MI355X) is visible");
    return FS_ENODEV;
  }
  for (int i = 0; i < n; i++)
    if (devices[i] < 0 || devices[i] >= nd) {
      set_error("devices: ordinal " + std::to_string(devices[i]) + " out of range (" +
                std::to_string(nd) + " visible)");
      return FS_EINVAL;
    }
  return FS_OK;
}

extern "C" {

const char* fs_version(void) { return "fastselect_amd 0.1.0 (gfx950)"; }

const char* fs_last_error(void) { return g_last_error.c_str(); }

int fs_device_count(void) { return gpu::device_count(); }

int fs_set_accumulation(int mode, int* previous) {
  if (mode != FS_ACCUM_FAST && mode != FS_ACCUM_REFERENCE) {
    set_error("accumulation mode must be FS_ACCUM_FAST or FS_ACCUM_REFERENCE");
    return FS_EINVAL;
  }
  if (previous) *previous = g_accum;
  g_accum = mode;
  return FS_OK;
}

int fs_get_accumulation(void) { return g_accum; }

int fs_test_hook(const char* name, int64_t value) {
  if (!name) {
    set_error("fs_test_hook: name is NULL");
    return FS_EINVAL;
  }
  TestHooks& h = test_hooks();
  const std::string k(name);
  if (k == "reset") h = TestHooks();
  else if (k == "ksplit") h.ksplit = value;
  else if (k == "q16") h.q16 = value;
  else if (k == "sparse") h.sparse = value;
  else if (k == "shards") h.shards = value;
  else if (k == "q16_guard_off") h.q16_guard_off = value;
  else if (k == "thr_exact_all") h.thr_exact_all = value;
  else if (k == "exact_gather") h.exact_gather = value;
  else if (k == "row_panel") h.row_panel = value;
  else if (k == "rf_xlds") h.rf_xlds = value;
  else if (k == "rf_fcap") h.rf_fcap = value;
  else if (k == "ties_1w") h.ties_1w = value;
  else if (k == "ties_coop") h.ties_coop = value;
  else if (k == "rf_ref_replay") h.rf_ref_replay = value;
  else if (k == "ref_q16") h.ref_q16 = value;
  else if (k == "surf_f64") h.surf_f64 = value;
  else if (k == "star_split") h.star_split = value;
  else if (k == "colsort_star") h.colsort_star = value;
  else if (k == "colsort_bins12") h.colsort_bins12 = value;
  else if (k == "colsort_global") h.colsort_global = value;
  else {
    set_error("fs_test_hook: unknown hook '" + k + "'");
    return FS_EINVAL;
  }
  return FS_OK;
}

int fs_multisurf_last_guard(double* risk_out, int* rerun_out) {
  return gpu::multisurf_last_guard(risk_out, rerun_out);
}

int fs_device_cache_release(void) {
  gpu::dev_cache_release();
  return FS_OK;
}

int fs_host_alloc(uint64_t bytes, void** out) {
  if (!out) {
    set_error("fs_host_alloc: out is NULL");
    return FS_EINVAL;
  }
  *out = nullptr;
  if (gpu::device_count() <= 0) {
    set_error("backend='gpu' requested but no HIP device is visible");
    return FS_ENODEV;
  }
  return gpu::host_alloc(out, (size_t)bytes);
}

int fs_host_free(void* p) {
  gpu::host_free(p);
  return FS_OK;
}

int fs_stage_x(int device, const void* x, int x_is_f64, int64_t n, int64_t p, uint64_t* staged) {
  if (!x || !staged || n < 1 || p < 1) {
    set_error("fs_stage_x: need x, staged, n >= 1 and p >= 1");
    return FS_EINVAL;
  }
  if (gpu::device_count() <= 0) {
    set_error("backend='gpu' requested but no HIP device is visible");
    return FS_ENODEV;
  }
  return gpu::stage_x(device, x, x_is_f64, n, p, staged);
}

int fs_stage_x_device(int device, const void* x, const void* x_device, int x_is_f64, int64_t n,
                      int64_t p, uint64_t* staged) {
  if (!x || !x_device || !staged || n < 1 || p < 1) {
    set_error("fs_stage_x_device: need x, x_device, staged, n >= 1 and p >= 1");
    return FS_EINVAL;
  }
  if (gpu::device_count() <= 0) {
    set_error("backend='gpu' requested but no HIP device is visible");
    return FS_ENODEV;
  }
  return gpu::stage_x_device(device, x, x_device, x_is_f64, n, p, staged);
}

int fs_stage_x_cast(int device, const void* x, int x_is_f64, int64_t n, int64_t p, int n_jobs,
                    float* out, int* finite, uint64_t* staged) {
  if (!x || !out || !finite || !staged || n < 1 || p < 1) {
    set_error("fs_stage_x_cast: need x, out, finite, staged, n >= 1 and p >= 1");
    return FS_EINVAL;
  }
  if (gpu::device_count() <= 0) {
    set_error("backend='gpu' requested but no HIP device is visible");
    return FS_ENODEV;
  }
  return gpu::stage_x_cast(device, x, x_is_f64, n, p, n_jobs, out, finite, staged);
}

int fs_unstage_x(uint64_t staged) { return gpu::unstage_x(staged); }

int fs_all_finite(const void* x, int x_is_f64, int64_t n, int64_t p, int n_jobs, int* finite) {
  if (!x || !finite || n < 0 || p < 0) {
    set_error("fs_all_finite: need x, finite, n >= 0 and p >= 0");
    return FS_EINVAL;
  }
  *finite = cpu::all_finite(x, x_is_f64, n * p, n_jobs);
  return FS_OK;
}

int fs_column_stats(int backend, int device, const void* x, int x_is_f64, int64_t n, int64_t p,
                    int64_t count_cap, void* colmin_out, void* colmax_out,
                    int64_t* ndistinct_out) {
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  if (!x || !colmin_out || !colmax_out || !ndistinct_out || n < 1 || p < 1 || count_cap < 0) {
    set_error("fs_column_stats: need x, outputs, n >= 1, p >= 1 and count_cap >= 0");
    return FS_EINVAL;
  }
  const int f64 = x_is_f64 ? 1 : 0;
  trace_mark("column_stats: enter");
  if (backend == FS_BACKEND_GPU)
    rc = gpu::column_stats(x, f64, n, p, count_cap, device, colmin_out, colmax_out, ndistinct_out);
  else
    rc = cpu::column_stats(x, f64, n, p, count_cap, -1, colmin_out, colmax_out, ndistinct_out);
  trace_mark("column_stats");
  return rc;
}

int fs_multisurf_score(int backend, int device, const float* x, int64_t n, int64_t p,
                       const double* y, const float* recip, const int64_t* feat_idx,
                       int64_t n_kept, int use_star, const uint8_t* is_discrete, int n_jobs,
                       float* scores_out) {
  if (!scores_out) {
    set_error("scores_out is NULL");
    return FS_EINVAL;
  }
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  Prepared P;
  trace_mark("multisurf: enter");
  rc = prepare(P, ALGO_MULTISURF, x, 0, n, p, feat_idx, n_kept, recip, is_discrete, n_jobs,
               backend == FS_BACKEND_GPU);
  trace_mark("prepare (host)");
  if (rc) return map_prep_rc(rc);
  if (encode_labels_f64(P, y)) return FS_EINVAL;
  P.use_star = use_star ? 1 : 0;
  if ((rc = apply_accumulation(P)) != FS_OK) return rc;
  if (backend == FS_BACKEND_GPU) return gpu::multisurf_run(P, x, device, scores_out);
  cpu::CpuState st;
  std::vector<double> rs(3 * n), cnt(2 * n), S(P.n_kept);
  cpu::multisurf_pass1(P, x, 0, 1, n_jobs, st, rs.data());
  cpu::multisurf_select(P, x, 0, 1, rs.data(), n_jobs, st, cnt.data());
  cpu::multisurf_pass2(P, x, st, cnt.data(), 0, 1, n_jobs, 0, n, S.data());
  for (int64_t k = 0; k < P.n_kept; k++) scores_out[k] = (float)(S[k] / (double)n);
  return FS_OK;
}

int fs_multisurf_score_rows(int backend, int device, const float* x, int64_t n, int64_t p,
                            const double* y, const float* recip, const int64_t* feat_idx,
                            int64_t n_kept, int use_star, const uint8_t* is_discrete, int n_jobs,
                            int64_t row_begin, int64_t row_end, double* sums_out) {
  if (!sums_out) {
    set_error("sums_out is NULL");
    return FS_EINVAL;
  }
  if (!(0 <= row_begin && row_begin <= row_end && row_end <= n)) {
    set_error("row range must satisfy 0 <= row_begin <= row_end <= n");
    return FS_EINVAL;
  }
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  Prepared P;
  rc = prepare(P, ALGO_MULTISURF, x, 0, n, p, feat_idx, n_kept, recip, is_discrete, n_jobs,
               backend == FS_BACKEND_GPU);
  if (rc) return map_prep_rc(rc);
  if (encode_labels_f64(P, y)) return FS_EINVAL;
  P.use_star = use_star ? 1 : 0;
  if ((rc = apply_accumulation(P)) != FS_OK) return rc;
  if (backend == FS_BACKEND_GPU) return gpu::multisurf_rows(P, x, device, row_begin, row_end, sums_out);
  cpu::CpuState st;
  std::vector<double> rs(3 * n), cnt(2 * n);
  cpu::multisurf_pass1(P, x, 0, 1, n_jobs, st, rs.data());
  cpu::multisurf_select(P, x, 0, 1, rs.data(), n_jobs, st, cnt.data());
  return cpu::multisurf_pass2(P, x, st, cnt.data(), 0, 1, n_jobs, row_begin, row_end, sums_out);
}

// Shared by the one-shot and the row-range entry points: validate, prepare,
// score the focal samples [r_lo, r_hi) -> float64 sums (not divided by n).
static int relieff_sums(int backend, int device, const float* x, int64_t n, int64_t p,
                        const int32_t* y_enc, const float* recip, const uint8_t* is_discrete,
                        int64_t k, const float* class_probs, int64_t n_classes, int n_jobs,
                        int64_t r_lo, int64_t r_hi, double* sums, const int* devices = nullptr,
                        int n_devices = 0) {
  if (!y_enc || !class_probs || n_classes < 1 || k < 0) {
    set_error("invalid ReliefF arguments (y_enc, class_probs, n_classes, k)");
    return FS_EINVAL;
  }
  if (!(0 <= r_lo && r_lo <= r_hi && r_hi <= n)) {
    set_error("row range must satisfy 0 <= row_begin <= row_end <= n");
    return FS_EINVAL;
  }
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  Prepared P;
  trace_mark("relieff: enter");
  rc = prepare(P, ALGO_RELIEFF, x, 0, n, p, nullptr, p, recip, is_discrete, n_jobs,
               backend == FS_BACKEND_GPU);
  trace_mark("prepare (host)");
  if (rc) return map_prep_rc(rc);
  P.labels.assign(y_enc, y_enc + n);
  for (int64_t i = 0; i < n; i++)
    if (P.labels[i] < 0 || P.labels[i] >= n_classes) {
      set_error("y_enc entry outside [0, n_classes)");
      return FS_EINVAL;
    }
  P.n_classes = (int32_t)n_classes;
  P.class_prior.assign(n_classes, 0.0);
  for (int64_t c = 0; c < n_classes; c++) P.class_prior[c] = (double)class_probs[c];
  P.k_neighbors = k;
  if ((rc = apply_accumulation(P)) != FS_OK) return rc;
  if (devices) {
    if ((rc = no_reference_devices()) != FS_OK) return rc;
    if (n_classes > 64) {
      set_error("GPU ReliefF supports at most 64 classes");
      return FS_ENOTSUP;
    }
    return gpu::rows_run_devices(P, x, devices, n_devices, r_lo, r_hi, sums);
  }
  if (backend == FS_BACKEND_GPU) return gpu::relieff_run(P, x, device, r_lo, r_hi, sums);
  return cpu::relieff_run(P, x, n_jobs, r_lo, r_hi, sums);
}

static int surf_sums(int backend, int device, const double* x, int64_t n, int64_t p,
                     const int32_t* y, const float* recip, int use_star,
                     const uint8_t* is_discrete, int n_jobs, int64_t r_lo, int64_t r_hi,
                     double* sums, const int* devices = nullptr, int n_devices = 0) {
  if (!(0 <= r_lo && r_lo <= r_hi && r_hi <= n)) {
    set_error("row range must satisfy 0 <= row_begin <= row_end <= n");
    return FS_EINVAL;
  }
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  Prepared P;
  trace_mark("surf: enter");
  rc = prepare(P, ALGO_SURF, x, 1, n, p, nullptr, p, recip, is_discrete, n_jobs,
               backend == FS_BACKEND_GPU);
  trace_mark("prepare (host)");
  if (rc) return map_prep_rc(rc);
  if (encode_labels_i32(P, y)) return FS_EINVAL;
  P.use_star = use_star ? 1 : 0;
  if ((rc = apply_accumulation(P)) != FS_OK) return rc;
  if (devices) {
    if ((rc = no_reference_devices()) != FS_OK) return rc;
    return gpu::rows_run_devices(P, x, devices, n_devices, r_lo, r_hi, sums);
  }
  if (backend == FS_BACKEND_GPU) return gpu::surf_run(P, x, device, r_lo, r_hi, sums);
  return cpu::surf_run(P, x, n_jobs, r_lo, r_hi, sums);
}

int fs_relieff_score(int backend, int device, const float* x, int64_t n, int64_t p,
                     const int32_t* y_enc, const float* recip, const uint8_t* is_discrete,
                     int64_t k, const float* class_probs, int64_t n_classes, int n_jobs,
                     float* scores_out) {
  if (!scores_out) {
    set_error("scores_out is NULL");
    return FS_EINVAL;
  }
  std::vector<double> S(p > 0 ? p : 1);
  const int rc = relieff_sums(backend, device, x, n, p, y_enc, recip, is_discrete, k,
                              class_probs, n_classes, n_jobs, 0, n, S.data());
  if (rc != FS_OK) return rc;
  for (int64_t f = 0; f < p; f++) scores_out[f] = (float)(S[f] / (double)n);
  return FS_OK;
}

int fs_relieff_score_rows(int backend, int device, const float* x, int64_t n, int64_t p,
                          const int32_t* y_enc, const float* recip, const uint8_t* is_discrete,
                          int64_t k, const float* class_probs, int64_t n_classes, int n_jobs,
                          int64_t row_begin, int64_t row_end, double* sums_out) {
  if (!sums_out) {
    set_error("sums_out is NULL");
    return FS_EINVAL;
  }
  return relieff_sums(backend, device, x, n, p, y_enc, recip, is_discrete, k, class_probs,
                      n_classes, n_jobs, row_begin, row_end, sums_out);
}

int fs_surf_score(int backend, int device, const double* x, int64_t n, int64_t p,
                  const int32_t* y, const float* recip, int use_star,
                  const uint8_t* is_discrete, int n_jobs, float* scores_out) {
  if (!scores_out) {
    set_error("scores_out is NULL");
    return FS_EINVAL;
  }
  std::vector<double> S(p > 0 ? p : 1);
  const int rc = surf_sums(backend, device, x, n, p, y, recip, use_star, is_discrete, n_jobs, 0,
                           n, S.data());
  if (rc != FS_OK) return rc;
  for (int64_t f = 0; f < p; f++) scores_out[f] = (float)(S[f] / (double)n);
  return FS_OK;
}

int fs_surf_score_rows(int backend, int device, const double* x, int64_t n, int64_t p,
                       const int32_t* y, const float* recip, int use_star,
                       const uint8_t* is_discrete, int n_jobs, int64_t row_begin,
                       int64_t row_end, double* sums_out) {
  if (!sums_out) {
    set_error("sums_out is NULL");
    return FS_EINVAL;
  }
  return surf_sums(backend, device, x, n, p, y, recip, use_star, is_discrete, n_jobs, row_begin,
                   row_end, sums_out);
}

int fs_multisurf_score_devices(const int* devices, int n_devices, const float* x, int64_t n,
                               int64_t p, const double* y, const float* recip,
                               const int64_t* feat_idx, int64_t n_kept, int use_star,
                               const uint8_t* is_discrete, int n_jobs, int64_t row_begin,
                               int64_t row_end, double* sums_out) {
  if (!sums_out) {
    set_error("sums_out is NULL");
    return FS_EINVAL;
  }
  if (!(0 <= row_begin && row_begin <= row_end && row_end <= n)) {
    set_error("row range must satisfy 0 <= row_begin <= row_end <= n");
    return FS_EINVAL;
  }
  int rc = check_devices(devices, n_devices);
  if (rc != FS_OK) return rc;
  Prepared P;
  rc = prepare(P, ALGO_MULTISURF, x, 0, n, p, feat_idx, n_kept, recip, is_discrete, n_jobs, true);
  if (rc) return map_prep_rc(rc);
  if (encode_labels_f64(P, y)) return FS_EINVAL;
  P.use_star = use_star ? 1 : 0;
  if ((rc = no_reference_devices()) != FS_OK) return rc;
  return gpu::multisurf_run_devices(P, x, devices, n_devices, row_begin, row_end, sums_out);
}

int fs_relieff_score_devices(const int* devices, int n_devices, const float* x, int64_t n,
                             int64_t p, const int32_t* y_enc, const float* recip,
                             const uint8_t* is_discrete, int64_t k, const float* class_probs,
                             int64_t n_classes, int n_jobs, int64_t row_begin, int64_t row_end,
                             double* sums_out) {
  if (!sums_out) {
    set_error("sums_out is NULL");
    return FS_EINVAL;
  }
  const int rc = check_devices(devices, n_devices);
  if (rc != FS_OK) return rc;
  return relieff_sums(FS_BACKEND_GPU, devices[0], x, n, p, y_enc, recip, is_discrete, k,
                      class_probs, n_classes, n_jobs, row_begin, row_end, sums_out, devices,
                      n_devices);
}

int fs_surf_score_devices(const int* devices, int n_devices, const double* x, int64_t n,
                          int64_t p, const int32_t* y, const float* recip, int use_star,
                          const uint8_t* is_discrete, int n_jobs, int64_t row_begin,
                          int64_t row_end, double* sums_out) {
  if (!sums_out) {
    set_error("sums_out is NULL");
    return FS_EINVAL;
  }
  const int rc = check_devices(devices, n_devices);
  if (rc != FS_OK) return rc;
  return surf_sums(FS_BACKEND_GPU, devices[0], x, n, p, y, recip, use_star, is_discrete, n_jobs,
                   row_begin, row_end, sums_out, devices, n_devices);
}

}  // extern "C"

// The _ex one-shot calls: the accumulation mode is an argument, in force for
// that call only (the calling thread's fs_set_accumulation mode is restored
// on return, whatever it was).
namespace {
struct ScopedAccumulation {
  int prev;
  explicit ScopedAccumulation(int mode) : prev(g_accum) { g_accum = mode; }
  ~ScopedAccumulation() { g_accum = prev; }
};
int check_mode(int mode) {
  if (mode == FS_ACCUM_FAST || mode == FS_ACCUM_REFERENCE) return FS_OK;
  set_error("accumulation must be FS_ACCUM_FAST or FS_ACCUM_REFERENCE");
  return FS_EINVAL;
}
}  // namespace

extern "C" {

int fs_multisurf_score_ex(int backend, int device, const float* x, int64_t n, int64_t p,
                          const double* y, const float* recip, const int64_t* feat_idx,
                          int64_t n_kept, int use_star, const uint8_t* is_discrete, int n_jobs,
                          int accumulation, float* scores_out) {
  if (const int rc = check_mode(accumulation)) return rc;
  ScopedAccumulation mode(accumulation);
  return fs_multisurf_score(backend, device, x, n, p, y, recip, feat_idx, n_kept, use_star,
                            is_discrete, n_jobs, scores_out);
}

int fs_relieff_score_ex(int backend, int device, const float* x, int64_t n, int64_t p,
                        const int32_t* y_enc, const float* recip, const uint8_t* is_discrete,
                        int64_t k, const float* class_probs, int64_t n_classes, int n_jobs,
                        int accumulation, float* scores_out) {
  if (const int rc = check_mode(accumulation)) return rc;
  ScopedAccumulation mode(accumulation);
  return fs_relieff_score(backend, device, x, n, p, y_enc, recip, is_discrete, k, class_probs,
                          n_classes, n_jobs, scores_out);
}

int fs_surf_score_ex(int backend, int device, const double* x, int64_t n, int64_t p,
                     const int32_t* y, const float* recip, int use_star,
                     const uint8_t* is_discrete, int n_jobs, int accumulation,
                     float* scores_out) {
  if (const int rc = check_mode(accumulation)) return rc;
  ScopedAccumulation mode(accumulation);
  return fs_surf_score(backend, device, x, n, p, y, recip, use_star, is_discrete, n_jobs,
                       scores_out);
}

}  // extern "C"

// ---- sharded MultiSURF plan ------------------------------------------------

struct fs_plan {
  int backend = FS_BACKEND_CPU;
  int rank = 0, world = 1, n_jobs = -1;
  int x_is_f64 = 0;
  int64_t r_lo = 0, r_hi = 0;   // focal rows (MultiSURF: fs_plan_set_rows, else [0, n))
  Prepared P;
  Prepared P0;                  // as created (all columns): discrete tables for re-targeting
  gpu::Plan* g = nullptr;
  // CPU state
  std::vector<char> x;          // the CPU plan's copy of X (x_is_f64 ? double : float)
  cpu::CpuState st;
  const void* xp() const { return (const void*)x.data(); }
};

static bool is_multisurf_plan(const fs_plan* pl) {
  if (pl->P.algo == ALGO_MULTISURF) return true;
  set_error("pass1 / select / pass2 are the MultiSURF plan stages (use fs_plan_score)");
  return false;
}

extern "C" {

int fs_plan_create(fs_plan** plan_out, int backend, int device, const float* x, int64_t n,
                   int64_t p, const double* y, const float* recip, const int64_t* feat_idx,
                   int64_t n_kept, int use_star, const uint8_t* is_discrete, int rank, int world,
                   int n_jobs, uint64_t stream) {
  if (!plan_out) {
    set_error("plan_out is NULL");
    return FS_EINVAL;
  }
  *plan_out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("invalid rank/world");
    return FS_EINVAL;
  }
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  fs_plan* pl = new fs_plan();
  pl->backend = backend;
  pl->rank = rank;
  pl->world = world;
  pl->n_jobs = n_jobs;
  rc = prepare(pl->P, ALGO_MULTISURF, x, 0, n, p, feat_idx, n_kept, recip, is_discrete, n_jobs,
               backend == FS_BACKEND_GPU);
  if (rc || encode_labels_f64(pl->P, y)) {
    delete pl;
    return FS_EINVAL;
  }
  pl->P.use_star = use_star ? 1 : 0;
  if ((rc = apply_accumulation(pl->P)) != FS_OK) {
    delete pl;
    return rc;
  }
  if (pl->P.ref_accum && world > 1 && backend != FS_BACKEND_GPU) {
    delete pl;
    set_error("reference-order accumulation with world > 1 (fs_plan_ref_masks / "
              "fs_plan_ref_pass2) runs on the GPU backend only");
    return FS_ENOTSUP;
  }
  pl->r_lo = 0;
  pl->r_hi = n;
  if (backend == FS_BACKEND_GPU) {
    rc = gpu::plan_create(&pl->g, pl->P, x, 0, device, rank, world, stream);
    if (rc != FS_OK) {
      delete pl;
      return rc;
    }
  } else {
    const char* xb = (const char*)x;
    pl->x.assign(xb, xb + (size_t)n * p * sizeof(float));
  }
  *plan_out = pl;
  return FS_OK;
}

// ReliefF / SURF plans: prepared problem in pl->P, X uploaded (GPU) or copied
// (CPU), focal rows [r_lo, r_hi).
static int finish_rows_plan(fs_plan* pl, int device, const void* x, int64_t r_lo, int64_t r_hi,
                            uint64_t stream) {
  const Prepared& P = pl->P;
  if (pl->backend == FS_BACKEND_GPU && pl->x_is_f64) pl->P0 = P;  // value tables
  pl->r_lo = r_lo;
  pl->r_hi = r_hi;
  if (pl->backend == FS_BACKEND_GPU)
    return gpu::plan_create(&pl->g, P, x, pl->x_is_f64, device, 0, 1, stream, r_lo, r_hi);
  const char* xb = (const char*)x;
  pl->x.assign(xb, xb + (size_t)P.n * P.p_in * (pl->x_is_f64 ? 8 : 4));
  return FS_OK;
}

int fs_plan_create_relieff(fs_plan** plan_out, int backend, int device, const float* x,
                           int64_t n, int64_t p, const int32_t* y_enc, const float* recip,
                           const uint8_t* is_discrete, int64_t k, const float* class_probs,
                           int64_t n_classes, int64_t row_begin, int64_t row_end, int n_jobs,
                           uint64_t stream) {
  if (!plan_out || !y_enc || !class_probs || n_classes < 1 || k < 0) {
    set_error("invalid ReliefF plan arguments");
    return FS_EINVAL;
  }
  *plan_out = nullptr;
  if (!(0 <= row_begin && row_begin <= row_end && row_end <= n)) {
    set_error("row range must satisfy 0 <= row_begin <= row_end <= n");
    return FS_EINVAL;
  }
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  if (backend == FS_BACKEND_GPU && n_classes > 64) {
    set_error("GPU ReliefF supports at most 64 classes");
    return FS_ENOTSUP;
  }
  fs_plan* pl = new fs_plan();
  pl->backend = backend;
  pl->n_jobs = n_jobs;
  rc = prepare(pl->P, ALGO_RELIEFF, x, 0, n, p, nullptr, p, recip, is_discrete, n_jobs,
               backend == FS_BACKEND_GPU);
  if (rc) {
    delete pl;
    return map_prep_rc(rc);
  }
  pl->P.labels.assign(y_enc, y_enc + n);
  for (int64_t i = 0; i < n; i++)
    if (pl->P.labels[i] < 0 || pl->P.labels[i] >= n_classes) {
      delete pl;
      set_error("y_enc entry outside [0, n_classes)");
      return FS_EINVAL;
    }
  pl->P.n_classes = (int32_t)n_classes;
  pl->P.class_prior.assign(n_classes, 0.0);
  for (int64_t c = 0; c < n_classes; c++) pl->P.class_prior[c] = (double)class_probs[c];
  pl->P.k_neighbors = k;
  if ((rc = apply_accumulation(pl->P)) != FS_OK ||
      (rc = finish_rows_plan(pl, device, x, row_begin, row_end, stream)) != FS_OK) {
    delete pl;
    return rc;
  }
  *plan_out = pl;
  return FS_OK;
}

int fs_plan_create_surf(fs_plan** plan_out, int backend, int device, const double* x, int64_t n,
                        int64_t p, const int32_t* y, const float* recip, int use_star,
                        const uint8_t* is_discrete, int64_t row_begin, int64_t row_end,
                        int n_jobs, uint64_t stream) {
  if (!plan_out) {
    set_error("plan_out is NULL");
    return FS_EINVAL;
  }
  *plan_out = nullptr;
  if (!(0 <= row_begin && row_begin <= row_end && row_end <= n)) {
    set_error("row range must satisfy 0 <= row_begin <= row_end <= n");
    return FS_EINVAL;
  }
  int rc = check_backend(backend, device);
  if (rc != FS_OK) return rc;
  fs_plan* pl = new fs_plan();
  pl->backend = backend;
  pl->n_jobs = n_jobs;
  pl->x_is_f64 = 1;
  rc = prepare(pl->P, ALGO_SURF, x, 1, n, p, nullptr, p, recip, is_discrete, n_jobs,
               backend == FS_BACKEND_GPU);
  if (rc || encode_labels_i32(pl->P, y)) {
    delete pl;
    return FS_EINVAL;
  }
  pl->P.use_star = use_star ? 1 : 0;
  if ((rc = apply_accumulation(pl->P)) != FS_OK ||
      (rc = finish_rows_plan(pl, device, x, row_begin, row_end, stream)) != FS_OK) {
    delete pl;
    return rc;
  }
  *plan_out = pl;
  return FS_OK;
}

int fs_plan_score(fs_plan* pl, double* sums) {
  if (!pl || !sums) {
    set_error("NULL plan or buffer");
    return FS_EINVAL;
  }
  if (pl->P.algo == ALGO_MULTISURF) {
    set_error("fs_plan_score is for ReliefF / SURF plans (MultiSURF: pass1 / select / pass2)");
    return FS_EINVAL;
  }
  if (pl->g) return gpu::plan_score(pl->g, sums);
  if (pl->P.algo == ALGO_RELIEFF)
    return cpu::relieff_run(pl->P, pl->xp(), pl->n_jobs, pl->r_lo, pl->r_hi, sums);
  return cpu::surf_run(pl->P, pl->xp(), pl->n_jobs, pl->r_lo, pl->r_hi, sums);
}

int fs_plan_set_features(fs_plan* pl, const int64_t* feat_idx, int64_t n_kept) {
  if (!pl) {
    set_error("plan is NULL");
    return FS_EINVAL;
  }
  const Prepared& O = pl->P;
  const bool gpu = pl->backend == FS_BACKEND_GPU;
  // the GPU plan keeps X and its column ranges on the device; the CPU plan
  // keeps its own copy of X
  const void* x = gpu ? nullptr : pl->xp();
  Prepared P;
  int rc = prepare(P, O.algo, x, pl->x_is_f64, O.n, O.p_in, feat_idx, n_kept, O.recip_in.data(),
                   O.disc_in.data(), pl->n_jobs, gpu, gpu ? &pl->P0 : nullptr);
  if (rc) return map_prep_rc(rc);
  P.labels = O.labels;
  P.n_classes = O.n_classes;
  P.class_prior = O.class_prior;
  P.use_star = O.use_star;
  P.k_neighbors = O.k_neighbors;
  P.ref_accum = O.ref_accum;  // the plan's mode, fixed at creation
  P.no_q16 = O.ref_accum && O.algo == ALGO_MULTISURF && !test_hooks().ref_q16 ? 1 : 0;
  if (gpu) {
    rc = gpu::plan_set_features(pl->g, P);
    if (rc != FS_OK) return rc;
  }
  pl->P = P;
  return FS_OK;
}

int fs_plan_pass1(fs_plan* pl, double* rowstats) {
  if (!pl || !rowstats) {
    set_error("NULL plan or buffer");
    return FS_EINVAL;
  }
  if (!is_multisurf_plan(pl)) return FS_EINVAL;
  if (pl->g) return gpu::plan_pass1(pl->g, rowstats);
  return cpu::multisurf_pass1(pl->P, pl->xp(), pl->rank, pl->world, pl->n_jobs, pl->st,
                              rowstats);
}

int fs_plan_select(fs_plan* pl, const double* rowstats, double* counts) {
  if (!pl || !rowstats || !counts) {
    set_error("NULL plan or buffer");
    return FS_EINVAL;
  }
  if (!is_multisurf_plan(pl)) return FS_EINVAL;
  if (pl->g) return gpu::plan_select(pl->g, rowstats, counts);
  return cpu::multisurf_select(pl->P, pl->xp(), pl->rank, pl->world, rowstats, pl->n_jobs,
                               pl->st, counts);
}

int fs_plan_pass2(fs_plan* pl, const double* counts, double* scores) {
  if (!pl || !counts || !scores) {
    set_error("NULL plan or buffer");
    return FS_EINVAL;
  }
  if (!is_multisurf_plan(pl)) return FS_EINVAL;
  if (pl->g) return gpu::plan_pass2(pl->g, counts, scores);
  return cpu::multisurf_pass2(pl->P, pl->xp(), pl->st, counts, pl->rank, pl->world, pl->n_jobs,
                              pl->r_lo, pl->r_hi, scores);
}

int fs_plan_ref_mask_words(fs_plan* pl, int64_t* words) {
  if (!pl || !words) {
    set_error("NULL plan or buffer");
    return FS_EINVAL;
  }
  if (!is_multisurf_plan(pl)) return FS_EINVAL;
  if (!pl->g || !pl->P.ref_accum) {
    set_error("fs_plan_ref_mask_words: a GPU plan created in reference-order accumulation");
    return FS_ENOTSUP;
  }
  *words = gpu::ref_mask_words(pl->g);
  return FS_OK;
}

int fs_plan_ref_masks(fs_plan* pl, uint64_t* masks, int64_t words) {
  int64_t need = 0;
  int rc = fs_plan_ref_mask_words(pl, &need);
  if (rc) return rc;
  if (!masks || words < need) {
    set_error("fs_plan_ref_masks: mask buffer NULL or smaller than fs_plan_ref_mask_words");
    return FS_EINVAL;
  }
  return gpu::plan_ref_masks(pl->g, masks);
}

int fs_plan_ref_pass2(fs_plan* pl, const uint64_t* masks, const double* counts, int64_t row_begin,
                      int64_t row_end) {
  int64_t need = 0;
  int rc = fs_plan_ref_mask_words(pl, &need);
  if (rc) return rc;
  if (!masks || !counts) {
    set_error("NULL plan or buffer");
    return FS_EINVAL;
  }
  if (!(0 <= row_begin && row_begin <= row_end && row_end <= pl->P.n)) {
    set_error("fs_plan_ref_pass2: row range outside [0, n)");
    return FS_EINVAL;
  }
  return gpu::plan_ref_pass2(pl->g, masks, counts, row_begin, row_end);
}

// GPU plans in reference order: fs_plan_ref_temp takes the row plans
// (ReliefF, SURF), fs_plan_ref_sums every kind
static int ref_rows_plan(fs_plan* pl, bool rows_only, const char* what) {
  if (!pl) {
    set_error("plan is NULL");
    return FS_EINVAL;
  }
  if (rows_only && pl->P.algo == ALGO_MULTISURF) {
    set_error(std::string(what) + ": a ReliefF or SURF plan");
    return FS_EINVAL;
  }
  if (!pl->g || !pl->P.ref_accum) {
    set_error(std::string(what) + ": a GPU plan created in reference-order accumulation");
    return FS_ENOTSUP;
  }
  return FS_OK;
}

int fs_plan_ref_temp(fs_plan* pl) {
  const int rc = ref_rows_plan(pl, true, "fs_plan_ref_temp");
  return rc ? rc : gpu::plan_ref_temp(pl->g);
}

int fs_plan_ref_sums(fs_plan* pl, const double* init, double* sums) {
  const int rc = ref_rows_plan(pl, false, "fs_plan_ref_sums");
  if (rc) return rc;
  if (!sums) {
    set_error("NULL sums buffer");
    return FS_EINVAL;
  }
  return gpu::plan_ref_sums(pl->g, init, sums);
}

int fs_plan_decision_guard(fs_plan* pl, const double* rowstats, const double* counts,
                           const double* scores, double* risk_out, int* switched_out) {
  if (!pl || !rowstats || !counts || !scores || !risk_out || !switched_out) {
    set_error("NULL plan or buffer");
    return FS_EINVAL;
  }
  if (!is_multisurf_plan(pl)) return FS_EINVAL;
  *risk_out = -1.0;
  *switched_out = 0;
  // the CPU backend always runs pass 1 on 32-bit operands
  if (!pl->g) return FS_OK;
  return gpu::plan_decision_guard(pl->g, rowstats, counts, scores, risk_out, switched_out);
}

int fs_plan_set_rows(fs_plan* pl, int64_t row_begin, int64_t row_end) {
  if (!pl) {
    set_error("plan is NULL");
    return FS_EINVAL;
  }
  if (!is_multisurf_plan(pl)) return FS_EINVAL;
  if (!(0 <= row_begin && row_begin <= row_end && row_end <= pl->P.n)) {
    set_error("row range must satisfy 0 <= row_begin <= row_end <= n");
    return FS_EINVAL;
  }
  if (pl->g) {
    const int rc = gpu::plan_set_rows(pl->g, row_begin, row_end);
    if (rc != FS_OK) return rc;
  }
  pl->r_lo = row_begin;
  pl->r_hi = row_end;
  return FS_OK;
}

int fs_plan_set_shard(fs_plan* pl, int rank, int world) {
  if (!pl) {
    set_error("plan is NULL");
    return FS_EINVAL;
  }
  if (!is_multisurf_plan(pl)) return FS_EINVAL;
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("shard rank/world must satisfy 0 <= rank < world");
    return FS_EINVAL;
  }
  if (pl->P.ref_accum && world > 1 && !pl->g) {
    set_error("reference-order accumulation with world > 1 (fs_plan_ref_masks / "
              "fs_plan_ref_pass2) runs on the GPU backend only");
    return FS_ENOTSUP;
  }
  if (pl->g) {
    const int rc = gpu::plan_set_shard(pl->g, rank, world);
    if (rc != FS_OK) return rc;
  }
  pl->rank = rank;
  pl->world = world;
  return FS_OK;
}

int fs_multisurf_shards(int device, int64_t n, int64_t p, int world, int* shards) {
  if (!shards || n < 2 || p < 1 || world < 1) {
    set_error("fs_multisurf_shards: need shards, n >= 2, p >= 1, world >= 1");
    return FS_EINVAL;
  }
  *shards = 1;
  if (test_hooks().shards >= 1) {
    *shards = (int)std::min<int64_t>(test_hooks().shards, 4096);
    return FS_OK;
  }
  if (gpu::device_count() <= 0) return FS_OK;
  Prepared P;
  P.n = n;
  P.n_pad = (n + kTile - 1) / kTile * kTile;
  P.PW = (p + kFeatPad - 1) / kFeatPad * kFeatPad;
  *shards = gpu::multisurf_shards(P, device, world);
  return FS_OK;
}

int fs_plan_info(const fs_plan* pl, int64_t* owned_tiles_out, double* pfe,
                 int64_t* refined_rows) {
  if (!pl) {
    set_error("NULL plan");
    return FS_EINVAL;
  }
  if (pl->g) return gpu::plan_info(pl->g, owned_tiles_out, pfe, refined_rows);
  if (refined_rows) *refined_rows = pl->st.refined;
  std::vector<int32_t> bi, bj;
  owned_tiles(pl->P.n_pad / kTile, pl->rank, pl->world, bi, bj);
  if (owned_tiles_out) *owned_tiles_out = (int64_t)bi.size();
  if (pfe) *pfe = 2.0 * (double)bi.size() * kTile * kTile * (double)(pl->P.pc + pl->P.pd);
  return FS_OK;
}

int fs_plan_calibration_ex(const fs_plan* pl, double* out, int n_out) {
  if (!pl || !out || n_out < 0) {
    set_error("NULL plan or output, or n_out < 0");
    return FS_EINVAL;
  }
  double v[8] = {0.0, 0.0, 0.0, std::sqrt((double)pl->P.pc / 6.0 + 1.0), 1.0, 0.0, 0.0, pl->P.SC};
  if (pl->g) {
    const int rc = gpu::plan_calibration(pl->g, v);
    if (rc != FS_OK) return rc;
  }
  const int m = n_out < 8 ? n_out : 8;
  for (int k = 0; k < m; k++) out[k] = v[k];
  return m;
}

// The six values documented since the first release (writing
// out[6] / out[7] through the old signature overran double[6] callers).
int fs_plan_calibration(const fs_plan* pl, double* out) {
  const int rc = fs_plan_calibration_ex(pl, out, 6);
  return rc < 0 ? rc : FS_OK;
}

int fs_plan_weighted_pairs(const fs_plan* pl, int64_t* pairs) {
  if (!pl || !pairs) {
    set_error("NULL plan or output");
    return FS_EINVAL;
  }
  *pairs = -1;
  if (pl->g) return gpu::plan_weighted_pairs(pl->g, pairs);
  return FS_OK;
}

double fs_plan_kernel_ms(const fs_plan* pl, int which) {
  if (!pl || !pl->g) return -1.0;
  return gpu::plan_kernel_ms(pl->g, which);
}

int fs_plan_destroy(fs_plan* pl) {
  if (!pl) return FS_OK;
  if (pl->g) gpu::plan_destroy(pl->g);
  delete pl;
  return FS_OK;
}

}  // extern "C"
