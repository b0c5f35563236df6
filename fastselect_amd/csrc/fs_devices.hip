// fs_devices.hip -- single-process multi-GPU (the estimators' devices=).
// Shared state and helpers: fs_gpu_internal.h.
#include "fs_gpu_internal.h"
// ---------------------------------------------------------------------------
// Single-process multi-GPU (the estimators' `devices=`)
// ---------------------------------------------------------------------------
namespace fs {
namespace gpu {

namespace {
// dst[k] = sum over r = 0..N-1, in that order, of parts[r][k]: every device
// sums the gathered vectors in the same order, so all get bit-identical sums
__global__ void k_rank_sum(double* __restrict__ dst, const double* __restrict__ parts, int N,
                           int64_t len) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= len) return;
  double s = 0.0;
  for (int r = 0; r < N; r++) s += parts[(int64_t)r * len + k];
  dst[k] = s;
}

// Peer access between every pair of distinct devices of a devices= call
// (xGMI copies instead of staging through host memory); once per pair.
void enable_peers(const int* devices, int N) {
  static std::mutex mu;
  static std::vector<std::pair<int, int>> done;
  std::lock_guard<std::mutex> lk(mu);
  for (int a = 0; a < N; a++)
    for (int b = 0; b < N; b++) {
      const int da = devices[a], db = devices[b];
      if (da == db) continue;
      if (std::find(done.begin(), done.end(), std::make_pair(da, db)) != done.end()) continue;
      done.emplace_back(da, db);
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, da, db) == hipSuccess && can && hipSetDevice(da) == hipSuccess)
        (void)hipDeviceEnablePeerAccess(db, 0);
      (void)hipGetLastError();  // already enabled, or no peer path: copies still work
    }
}

// One device thread of a devices= call: its plan's stream, an event per
// exchange, and the thread's view of the group (barrier, every thread's
// send buffer and event).
struct DevGroup {
  int N;
  const int* devices;
  StageBarrier bar;
  std::vector<const void*> send;  // per thread: the buffer its peers copy from
  std::vector<hipEvent_t> ready;  // per thread: recorded once `send` holds the data
  explicit DevGroup(int n, const int* d) : N(n), devices(d), bar(n), send(n), ready(n) {}
};

// Thread r's part of an exchange: thread r's `part` (len doubles, on its
// device, complete once its stream reaches this point) is summed over all
// threads into `out` on every device.  Each stream waits for the peers'
// events and copies their parts into `gather` [N][len] (device to device
// over xGMI; a repeated ordinal copies within the device), then k_rank_sum
// adds them in thread order.  Nothing passes through host memory, and no
// thread waits for another's device work on the host: one barrier makes the
// events and buffers visible.  A part must not be rewritten until every peer
// has copied it: the callers give each exchange its own part buffer, and
// every later write to it is ordered behind the next exchange's waits.
bool exchange_parts(DevGroup& G, int r, hipStream_t st, hipEvent_t ev, const double* part,
                    double* gather, double* out, int64_t len, int& rc) {
  int e = rc;
  if (!e && hipEventRecord(ev, st) != hipSuccess) {
    set_error("multi-device exchange: event record failed");
    e = FS_EHIP;
  }
  G.send[r] = part;
  G.ready[r] = ev;
  if (!G.bar.arrive(e, e ? std::string(fs_last_error()) : std::string())) return false;
  for (int k = 0; k < G.N && !rc; k++) {
    if (hipStreamWaitEvent(st, G.ready[k], 0) != hipSuccess ||
        hipMemcpyPeerAsync(gather + (int64_t)k * len, G.devices[r], G.send[k], G.devices[k],
                           sizeof(double) * len, st) != hipSuccess) {
      (void)hipGetLastError();
      set_error("multi-device exchange: peer copy failed");
      rc = FS_EHIP;
    }
  }
  if (!rc) {
    k_rank_sum<<<(unsigned)((len + 255) / 256), 256, 0, st>>>(out, gather, G.N, len);
    rc = launch_check("k_rank_sum");
  }
  // the peers read G.ready / G.send of this exchange before the next
  // exchange's barrier rewrites them: keep them apart with a second barrier
  return G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
}

// X on every device of a devices= call, moved over the host link once: thread
// r uploads its 1/N of the rows into a full-size buffer on its device, then
// copies the other threads' row ranges from their devices (xGMI peer copies;
// a repeated ordinal copies within the device).  *buf receives the buffer
// (caller frees it after a barrier that follows the last peer copy).
bool distribute_x(DevGroup& G, int r, const void* x, size_t row_bytes, int64_t n, void** buf,
                  hipStream_t st, hipEvent_t ev, int& rc) {
  const int dev = G.devices[r];
  *buf = nullptr;
  if (!rc) rc = dev_alloc(buf, row_bytes * (size_t)n, dev);
  auto lo = [&](int k) { return n * k / G.N; };
  if (!rc && hipMemcpyAsync((char*)*buf + row_bytes * lo(r), (const char*)x + row_bytes * lo(r),
                            row_bytes * (size_t)(lo(r + 1) - lo(r)), hipMemcpyHostToDevice,
                            st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("multi-device X: host-to-device copy of the row share failed");
    rc = FS_EHIP;
  }
  int e = rc;
  if (!e && hipEventRecord(ev, st) != hipSuccess) e = FS_EHIP;
  G.send[r] = *buf;
  G.ready[r] = ev;
  if (!G.bar.arrive(e, e ? std::string(fs_last_error()) : std::string())) return false;
  for (int k = 0; k < G.N && !rc; k++) {
    if (k == r || lo(k + 1) == lo(k)) continue;
    if (hipStreamWaitEvent(st, G.ready[k], 0) != hipSuccess ||
        hipMemcpyPeerAsync((char*)*buf + row_bytes * lo(k), dev,
                           (const char*)G.send[k] + row_bytes * lo(k), G.devices[k],
                           row_bytes * (size_t)(lo(k + 1) - lo(k)), st) != hipSuccess) {
      (void)hipGetLastError();
      set_error("multi-device X: peer copy failed");
      rc = FS_EHIP;
    }
  }
  if (!rc && hipStreamSynchronize(st) != hipSuccess) {
    (void)hipGetLastError();
    rc = FS_EHIP;
  }
  if (r == 0 && trace_on()) {
    char msg[160];
    snprintf(msg, sizeof msg, "devices: X on %d devices (%.1f MB per device over the host link, "
             "the rest peer-copied)", G.N, (double)row_bytes * (double)(lo(1) - lo(0)) / 1e6);
    trace_mark(msg);
  }
  return G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
}

// how many of devices[0..N) are `d` (plans sharing a device share its memory)
int ordinal_share(const int* devices, int N, int d) {
  int m = 0;
  for (int k = 0; k < N; k++) m += devices[k] == d;
  return std::max(m, 1);
}
}  // namespace

// MultiSURF over several devices from one process: thread r (devices[r],
// repeats allowed) owns the tiles t with t % (N V) == r + N v of the
// upper triangle -- the partition of parallel.py's one-process-per-GPU path.
// X crosses the host link once (distribute_x: 1/N of the rows per device,
// the rest by peer copies), and the three exchange vectors (row moments,
// neighbour counts, score sums) are summed device-side (exchange_parts: peer
// copies of every thread's part, a fixed-order sum on each device) where the
// multi-process path all-reduces them over RCCL.  V > 1 tile shards per
// device when the largest share exceeds a device's memory (sized with the
// device's memory split between the plans that share it).  Focal samples
// [r_lo, r_hi) as fs_multisurf_score_rows; sums (not / n).
int multisurf_run_devices(const Prepared& P, const void* x, const int* devices, int ndev,
                          int64_t r_lo, int64_t r_hi, double* sums_out) {
  const int N = ndev;
  int V = 1;
  for (int r = 0; r < N; r++)
    V = std::max(V, multisurf_shards(P, devices[r], N, ordinal_share(devices, N, devices[r])));
  const int W = N * V;
  const int64_t n = P.n, nk = P.n_kept;
  enable_peers(devices, N);
  DevGroup G(N, devices);
  std::vector<double> result((size_t)nk);
  const bool whole = r_lo == 0 && r_hi == n;
  if (whole) {
    g_last_risk = -1.0;
    g_last_rerun = 0;
  }
  auto worker = [&](int r) {
    Plan* g = nullptr;
    // per exchange: this thread's part, the gathered parts, the sum
    double *rs_p = nullptr, *cnt_p = nullptr, *sc_p = nullptr, *gath = nullptr;
    double *rs = nullptr, *cnt = nullptr, *sc = nullptr, *tmp = nullptr;
    void* xbuf = nullptr;
    uint64_t staged = 0;
    hipStream_t xs_st = nullptr;
    hipEvent_t evs[4] = {nullptr, nullptr, nullptr, nullptr};
    int rc = hipSetDevice(devices[r]) == hipSuccess ? FS_OK : FS_EHIP;
    for (auto& e : evs)
      if (!rc && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) rc = FS_EHIP;
    if (!rc && hipStreamCreateWithFlags(&xs_st, hipStreamNonBlocking) != hipSuccess) rc = FS_EHIP;
    bool ok = distribute_x(G, r, x, sizeof(float) * (size_t)P.p_in, n, &xbuf, xs_st, evs[0], rc);
    if (ok && !rc) rc = stage_x_device(devices[r], x, xbuf, 0, n, P.p_in, &staged);
    if (ok && !rc) rc = plan_create(&g, P, x, 0, devices[r], r, W, 0);
    if (staged) unstage_x(staged);
    if (ok && !rc) rc = plan_set_rows(g, r_lo, r_hi);
    const int64_t glen = (int64_t)N * std::max<int64_t>(3 * n, nk);
    if (ok && !rc && ((rc = dalloc(g, &rs_p, 3 * n)) || (rc = dalloc(g, &cnt_p, 2 * n)) ||
                      (rc = dalloc(g, &sc_p, nk)) || (rc = dalloc(g, &rs, 3 * n)) ||
                      (rc = dalloc(g, &cnt, 2 * n)) || (rc = dalloc(g, &sc, nk)) ||
                      (rc = dalloc(g, &gath, glen)) ||
                      (rc = dalloc(g, &tmp, std::max<int64_t>(3 * n, nk)))))
      ;
    // every peer has copied its rows of xbuf (the barrier after the copies)
    // and the plan holds its own copy: free it
    if (xbuf) dev_free(xbuf);
    hipStream_t st = g ? g->stream : nullptr;
    auto exch = [&](int which) {
      double* part = which == 0 ? rs_p : which == 1 ? cnt_p : sc_p;
      double* out = which == 0 ? rs : which == 1 ? cnt : sc;
      const int64_t len = which == 0 ? 3 * n : which == 1 ? 2 * n : nk;
      return exchange_parts(G, r, st, evs[1 + which], part, gath, out, len, rc);
    };
    auto acc = [&](double* dst, const double* src, int64_t len, bool first) -> int {
      if (first)
        return hipMemcpyAsync(dst, src, sizeof(double) * len, hipMemcpyDeviceToDevice, st) ==
                       hipSuccess
                   ? FS_OK
                   : FS_EHIP;
      return accumulate(dst, src, len, st);
    };
    auto stages = [&]() {
      if (V == 1) {
        if (!rc) rc = plan_pass1(g, rs_p);
        ok = exch(0);
        if (ok && !rc) rc = plan_select(g, rs, cnt_p);
        ok = ok && exch(1);
        if (ok && !rc) rc = plan_pass2(g, cnt, sc_p);
        ok = ok && exch(2);
        return;
      }
      for (int round = 0; round < 3 && ok; round++) {
        for (int v = 0; v < V && !rc; v++) {
          if ((rc = plan_set_shard(g, r + N * v, W))) break;
          if ((rc = plan_pass1(g, tmp))) break;
          if (round == 0) { rc = acc(rs_p, tmp, 3 * n, v == 0); continue; }
          if ((rc = plan_select(g, rs, tmp))) break;
          if (round == 1) { rc = acc(cnt_p, tmp, 2 * n, v == 0); continue; }
          if ((rc = plan_pass2(g, cnt, tmp))) break;
          rc = acc(sc_p, tmp, nk, v == 0);
        }
        ok = exch(round);
      }
    };
    if (ok) stages();
    // the decision check on a whole-range call: every thread holds the same
    // summed vectors, so every thread reaches the same decision
    if (ok && whole) {
      double risk = -1.0;
      int sw = 0;
      if (!rc) rc = plan_decision_guard(g, rs, cnt, sc, &risk, &sw);
      if (r == 0) {
        g_last_risk = risk;
        g_last_rerun = sw;
      }
      ok = G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
      if (ok && sw) stages();
    }
    if (ok && !rc && r == 0) {
      if (hipMemcpyAsync(result.data(), sc, sizeof(double) * nk, hipMemcpyDeviceToHost, st) !=
              hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("multi-device MultiSURF: device-to-host copy of the sums failed");
        rc = FS_EHIP;
      }
    }
    if (g) plan_destroy(g);
    if (ok) G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
    // after the final barrier nobody waits on this thread's events any more
    if (xs_st) (void)hipStreamDestroy(xs_st);
    for (auto& e : evs)
      if (e) (void)hipEventDestroy(e);
    return rc;
  };
  std::vector<std::thread> th;
  for (int r = 1; r < N; r++) th.emplace_back(worker, r);
  worker(0);
  for (auto& t : th) t.join();
  if (G.bar.rc() != FS_OK) {
    set_error(G.bar.err().empty() ? std::string("multi-device MultiSURF failed") : G.bar.err());
    return G.bar.rc();
  }
  std::copy(result.begin(), result.end(), sums_out);
  return FS_OK;
}

// ReliefF / SURF over several devices: thread r scores the focal samples of
// its whole 128-sample blocks of [r_lo, r_hi) (parallel.shard_rows) on
// devices[r]; the float64 sums are added on the host in rank order.  Their
// neighbour selection is row-local (ReliefF.py:144-175, SURF.py:146-163),
// so there is no other exchange.
int rows_run_devices(const Prepared& P, const void* x, const int* devices, int ndev,
                     int64_t r_lo, int64_t r_hi, double* sums_out) {
  const int N = ndev;
  const int64_t b0 = r_lo / kTile, b1 = (r_hi + kTile - 1) / kTile, nb = b1 - b0;
  const int x_f64 = P.algo == ALGO_SURF ? 1 : 0;  // SURF's kernel dtype (SURF.py:330-333)
  std::vector<std::vector<double>> parts(N, std::vector<double>(P.n_kept, 0.0));
  enable_peers(devices, N);
  DevGroup G(N, devices);
  auto worker = [&](int r) {
    const int64_t lo = std::max(r_lo, (b0 + nb * r / N) * kTile);
    const int64_t hi = std::min(r_hi, (b0 + nb * (r + 1) / N) * kTile);
    void* xbuf = nullptr;
    uint64_t staged = 0;
    hipStream_t st = nullptr;
    hipEvent_t ev = nullptr;
    int rc = hipSetDevice(devices[r]) == hipSuccess ? FS_OK : FS_EHIP;
    if (!rc && (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess))
      rc = FS_EHIP;
    // X once over the host link: 1/N of the rows per device, the rest by
    // peer copies, registered as this thread's staged X for the plans
    const bool ok = distribute_x(G, r, x, (x_f64 ? 8 : 4) * (size_t)P.p_in, P.n, &xbuf, st, ev, rc);
    if (ok && !rc) rc = stage_x_device(devices[r], x, xbuf, x_f64, P.n, P.p_in, &staged);
    if (ok && !rc && hi > lo)
      rc = P.algo == ALGO_RELIEFF ? relieff_run(P, x, devices[r], lo, hi, parts[r].data())
                                  : surf_run(P, x, devices[r], lo, hi, parts[r].data());
    if (staged) unstage_x(staged);
    if (xbuf) dev_free(xbuf);
    if (ok) G.bar.arrive(rc, rc ? std::string(fs_last_error()) : std::string());
    if (st) (void)hipStreamDestroy(st);
    if (ev) (void)hipEventDestroy(ev);
  };
  std::vector<std::thread> th;
  for (int r = 1; r < N; r++) th.emplace_back(worker, r);
  worker(0);
  for (auto& t : th) t.join();
  if (G.bar.rc() != FS_OK) {
    set_error(G.bar.err().empty() ? std::string("multi-device scoring failed") : G.bar.err());
    return G.bar.rc();
  }
  // the row partition's float64 sums, added in thread order (one small
  // vector per device; there is no other exchange)
  std::fill(sums_out, sums_out + P.n_kept, 0.0);
  for (int r = 0; r < N; r++)
    for (int64_t k = 0; k < P.n_kept; k++) sums_out[k] += parts[r][k];
  return FS_OK;
}

}  // namespace gpu
}  // namespace fs
