// fs_gpu_mem.hip -- devices, the device block cache and pinned host staging.
// Shared state and helpers: fs_gpu_internal.h.
#include "fs_gpu_internal.h"

namespace fs {
namespace gpu {

int device_count() {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return c < 0 ? 0 : c;
}

// ---------------------------------------------------------------------------
// Device block cache
// ---------------------------------------------------------------------------
// hipMalloc of the ~11 GB a cfg4 plan holds took 190-310 ms per fit on the
// MI355X (fresh pages are mapped on allocation; tools/fit_breakdown.py) --
// more than the scoring.  Blocks that plans and the column statistics free
// are kept per device up to a cap (an eighth of the device's memory;
// FS_DEVICE_CACHE_MB overrides, 0 disables) and handed to the next request
// they cover within 2x, so repeated fits (TuRF refits, CV folds, benchmarks)
// skip the mapping.  A failed hipMalloc releases the device's cache and
// retries; fs_device_cache_release() returns everything.  Callers free a
// block only after the streams that use it are synchronised, and every
// consumer writes or clears what it reads (blocks come back with stale data).
namespace {
struct Block {
  size_t bytes;
  int device;
  bool cached;
};
std::mutex cache_mu;
std::unordered_map<void*, Block> blocks;             // every block handed out or cached
std::multimap<std::pair<int, size_t>, void*> cache;  // (device, bytes) -> cached block
std::map<int, size_t> cache_bytes;

size_t cache_cap(int device) {  // with cache_mu held
  static long long env_mb = -2;
  if (env_mb == -2) {
    const char* e = std::getenv("FS_DEVICE_CACHE_MB");
    env_mb = (e && *e) ? std::max(0LL, std::atoll(e)) : -1;
  }
  if (env_mb >= 0) return (size_t)env_mb << 20;
  static std::map<int, size_t> total;
  auto it = total.find(device);
  if (it == total.end()) {
    size_t t = 0;
    if (hipDeviceTotalMem(&t, device) != hipSuccess) {
      (void)hipGetLastError();
      t = 0;
    }
    it = total.emplace(device, t).first;
  }
  return it->second / 8;
}

void release_device(int device) {  // with cache_mu held; device < 0: all
  for (auto it = cache.begin(); it != cache.end();) {
    if (device >= 0 && it->first.first != device) {
      ++it;
      continue;
    }
    (void)hipFree(it->second);
    blocks.erase(it->second);
    cache_bytes[it->first.first] -= it->first.second;
    it = cache.erase(it);
  }
}
}  // namespace

int dev_alloc(void** out, size_t bytes, int device) {
  if (bytes == 0) bytes = 1;
  std::lock_guard<std::mutex> lk(cache_mu);
  auto it = cache.lower_bound({device, bytes});
  if (it != cache.end() && it->first.first == device && it->first.second <= 2 * bytes) {
    *out = it->second;
    cache_bytes[device] -= it->first.second;
    blocks[it->second].cached = false;
    cache.erase(it);
    return FS_OK;
  }
  hipError_t e = hipMalloc(out, bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    release_device(device);
    e = hipMalloc(out, bytes);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error(std::string("hipMalloc of ") + std::to_string(bytes) +
              " bytes failed: " + hipGetErrorString(e));
    return FS_EOOM;
  }
  blocks[*out] = Block{bytes, device, false};
  return FS_OK;
}

void dev_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(cache_mu);
  auto it = blocks.find(p);
  if (it == blocks.end()) {
    (void)hipFree(p);
    return;
  }
  Block& b = it->second;
  if (!b.cached && cache_bytes[b.device] + b.bytes <= cache_cap(b.device)) {
    b.cached = true;
    cache.emplace(std::make_pair(b.device, b.bytes), p);
    cache_bytes[b.device] += b.bytes;
    return;
  }
  if (!b.cached) {
    blocks.erase(it);
    (void)hipFree(p);
  }
}

// Pinned host blocks (hipHostMalloc) for the float32 copy of X an estimator
// makes: the host threads cast into already-pinned, already-faulted pages and
// the upload of X is a DMA from them (cfg4 fit: the cast of 3.2 GB of
// float64 into fresh pageable pages and the copy through the runtime's
// staging buffers took ~140 ms of a 330 ms fit).  Freed blocks are kept
// (up to kHostCacheBlocks) for the next fit of a similar size (within 2x).
namespace {
constexpr size_t kHostCacheBlocks = 2;
std::mutex host_mu;
std::unordered_map<void*, size_t> host_live;
std::multimap<size_t, void*> host_cache;
}  // namespace

int host_alloc(void** out, size_t bytes) {
  *out = nullptr;
  if (bytes == 0) bytes = 1;
  {
    std::lock_guard<std::mutex> lk(host_mu);
    auto it = host_cache.lower_bound(bytes);
    if (it != host_cache.end() && it->first <= 2 * bytes) {
      *out = it->second;
      host_live[it->second] = it->first;
      host_cache.erase(it);
      return FS_OK;
    }
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    set_error("hipHostMalloc failed");
    return FS_EOOM;
  }
  std::lock_guard<std::mutex> lk(host_mu);
  host_live[p] = bytes;
  *out = p;
  return FS_OK;
}

void host_free(void* p) {
  if (!p) return;
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> lk(host_mu);
    auto it = host_live.find(p);
    if (it == host_live.end()) return;
    host_cache.emplace(it->second, p);
    host_live.erase(it);
    while (host_cache.size() > kHostCacheBlocks) {  // keep the largest blocks
      drop.push_back(host_cache.begin()->second);
      host_cache.erase(host_cache.begin());
    }
  }
  for (void* q : drop) (void)hipHostFree(q);
}

void dev_cache_release() {
  {
    std::lock_guard<std::mutex> lk(cache_mu);
    release_device(-1);
  }
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> lk(host_mu);
    for (auto& kv : host_cache) drop.push_back(kv.second);
    host_cache.clear();
  }
  for (void* q : drop) (void)hipHostFree(q);
}

// ---------------------------------------------------------------------------
// Stream and event pool: a plan takes two streams and eight events, and
// creating and destroying them cost ~1 ms per fit; released ones are kept
// per device (idle: every plan synchronises its streams before returning
// them) and handed to the next plan.
// ---------------------------------------------------------------------------
namespace {
std::mutex pool_mu;
std::map<int, std::vector<hipStream_t>> stream_pool;
std::map<std::pair<int, bool>, std::vector<hipEvent_t>> event_pool;
constexpr size_t kPoolCap = 16;
}  // namespace

hipStream_t stream_get(int device) {
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    auto& v = stream_pool[device];
    if (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      return s;
    }
  }
  hipStream_t s = nullptr;
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    set_error("hipStreamCreate failed");
    return nullptr;
  }
  return s;
}

void stream_put(int device, hipStream_t s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    auto& v = stream_pool[device];
    if (v.size() < kPoolCap) {
      v.push_back(s);
      return;
    }
  }
  (void)hipStreamDestroy(s);
}

hipEvent_t event_get(int device, bool timing) {
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    auto& v = event_pool[{device, timing}];
    if (!v.empty()) {
      hipEvent_t e = v.back();
      v.pop_back();
      return e;
    }
  }
  hipEvent_t e = nullptr;
  if (hipSetDevice(device) != hipSuccess ||
      (timing ? hipEventCreate(&e) : hipEventCreateWithFlags(&e, hipEventDisableTiming)) !=
          hipSuccess) {
    (void)hipGetLastError();
    set_error("hipEventCreate failed");
    return nullptr;
  }
  return e;
}

void event_put(int device, hipEvent_t e, bool timing) {
  if (!e) return;
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    auto& v = event_pool[{device, timing}];
    if (v.size() < 4 * kPoolCap) {
      v.push_back(e);
      return;
    }
  }
  (void)hipEventDestroy(e);
}

// ---------------------------------------------------------------------------
// Staged X: an estimator's fit uploads X once (fs_stage_x) and both the
// column statistics and the scoring plans read that copy in place (a plan
// holds a reference: staged_acquire / staged_release, so fs_unstage_x while a
// plan lives defers the free to the last release).  The caller keeps the
// host array unchanged until fs_unstage_x.  Saves one host-to-device copy of
// X per fit (1.6 GB at cfg4, 4 GB of float64 at cfg5) and the plan's own
// device copy.  A copy made by fs_stage_x_cast also carries its column
// extrema, taken by the casting threads, so that neither the column
// statistics nor the plan measure them again.
// ---------------------------------------------------------------------------
namespace {
struct Staged {
  const void* host;
  int64_t n, p;
  int f64, device;
  void* dev;
  std::thread::id owner;  // only the staging thread's calls read it (concurrent
                          // fits of one array stage and free their own copies)
  bool borrowed;          // caller-owned device copy (stage_x_device): not freed
  int refs = 0;           // plans reading it (staged_acquire)
  bool released = false;  // fs_unstage_x came while refs > 0: freed by the last release
  std::vector<char> cmin, cmax;  // column extrema in X's dtype (empty: not known)
};
std::mutex staged_mu;
std::vector<Staged> staged;
}  // namespace

int stage_x(int device, const void* x, int x_is_f64, int64_t n, int64_t p, uint64_t* handle) {
  *handle = 0;
  if (device < 0 || device >= device_count()) {
    set_error("fs_stage_x: device ordinal out of range");
    return FS_ENODEV;
  }
  FS_HIP(hipSetDevice(device));
  const size_t bytes = (size_t)n * p * (x_is_f64 ? 8 : 4);
  void* d = nullptr;
  if (int rc = dev_alloc(&d, bytes, device)) return rc;
  if (hipMemcpy(d, x, bytes, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipGetLastError();
    dev_free(d);
    set_error("fs_stage_x: host-to-device copy failed");
    return FS_EHIP;
  }
  std::lock_guard<std::mutex> lk(staged_mu);
  staged.push_back(
      Staged{x, n, p, x_is_f64 ? 1 : 0, device, d, std::this_thread::get_id(), false, 0, false, {}, {}});
  *handle = (uint64_t)(uintptr_t)d;
  return FS_OK;
}

// A device copy the caller already holds (e.g. X assembled on the GPU by an
// all-gather of each rank's rows) registered under the host array's key.
int stage_x_device(int device, const void* x, const void* x_dev, int x_is_f64, int64_t n,
                   int64_t p, uint64_t* handle) {
  *handle = 0;
  if (device < 0 || device >= device_count()) {
    set_error("fs_stage_x_device: device ordinal out of range");
    return FS_ENODEV;
  }
  std::lock_guard<std::mutex> lk(staged_mu);
  for (const Staged& e : staged)
    if (e.dev == x_dev) {
      set_error("fs_stage_x_device: this device buffer is already staged");
      return FS_EINVAL;
    }
  staged.push_back(Staged{x, n, p, x_is_f64 ? 1 : 0, device, const_cast<void*>(x_dev),
                          std::this_thread::get_id(), true, 0, false, {}, {}});
  *handle = (uint64_t)(uintptr_t)x_dev;
  return FS_OK;
}

// The float64 -> float32 cast of X that validation makes (or, for float32
// X, a copy into pinned memory), fused with its finiteness scan and its
// upload: host threads cast row blocks (32 MB of float32 each) into `out`
// while this thread copies every finished block to the device (pinned
// `out`: a DMA beside the casting of later blocks).  The
// device copy is registered under `out` as fs_stage_x would; without device
// room for it (or with a non-finite value, which validation will reject) the
// cast alone is done and *handle stays 0.  cfg4 (3.2 GB of float64): the cast
// and the 1.6 GB upload overlap instead of following each other.
int stage_x_cast(int device, const void* x, int x_is_f64, int64_t n, int64_t p, int n_jobs,
                 float* out, int* finite, uint64_t* handle) {
  *handle = 0;
  *finite = 1;
  if (device < 0 || device >= device_count()) {
    set_error("fs_stage_x_cast: device ordinal out of range");
    return FS_ENODEV;
  }
  FS_HIP(hipSetDevice(device));
  const int64_t total = n * p;
  void* d = nullptr;
  hipStream_t st = nullptr;
  if (dev_alloc(&d, (size_t)total * sizeof(float), device) != FS_OK ||
      hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    if (d) dev_free(d);
    d = nullptr;
    st = nullptr;
  }
  const int64_t blk_rows = std::max<int64_t>(1, (int64_t(8) << 20) / p);
  const int64_t nblk = (n + blk_rows - 1) / blk_rows;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(hardware_threads(n_jobs), nblk));
  // per-thread column extrema of the float32 values (merged below): what
  // x32.min(0) / x32.max(0) give, for the column statistics and the plans
  std::vector<std::vector<float>> tmin((size_t)nt), tmax((size_t)nt);
  std::vector<char> done((size_t)nblk, 0);
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<int64_t> next{0};
  std::atomic<int> bad{0};
  auto work = [&](int w) {
    std::vector<float>& mn = tmin[(size_t)w];
    std::vector<float>& mx = tmax[(size_t)w];
    for (int64_t b = next++; b < nblk; b = next++) {
      const int64_t r0 = b * blk_rows, r1 = std::min(n, (b + 1) * blk_rows);
      if (mn.empty()) {  // this thread's first row block seeds its extrema
        mn.resize((size_t)p);
        mx.resize((size_t)p);
        for (int64_t c = 0; c < p; c++)
          mn[c] = mx[c] = x_is_f64 ? (float)((const double*)x)[r0 * p + c]
                                   : ((const float*)x)[r0 * p + c];
      }
      float* __restrict__ lo_ = mn.data();
      float* __restrict__ hi_ = mx.data();
      uint32_t any = 0;
      for (int64_t r = r0; r < r1; r++) {
        float* __restrict__ o = out + r * p;
        if (x_is_f64) {
          const double* __restrict__ xd = (const double*)x + r * p;
          for (int64_t c = 0; c < p; c++) {
            const float v = (float)xd[c];  // round to nearest, as numpy's astype
            o[c] = v;
            lo_[c] = v < lo_[c] ? v : lo_[c];
            hi_[c] = v > hi_[c] ? v : hi_[c];
          }
        } else {
          const float* __restrict__ xf = (const float*)x + r * p;
          for (int64_t c = 0; c < p; c++) {
            const float v = xf[c];
            o[c] = v;
            lo_[c] = v < lo_[c] ? v : lo_[c];
            hi_[c] = v > hi_[c] ? v : hi_[c];
          }
        }
        // non-finite values: the row's exponent bits (one pass over what was written)
        const uint32_t* ou = (const uint32_t*)o;
        for (int64_t c = 0; c < p; c++) any |= (uint32_t)((ou[c] & 0x7f800000u) == 0x7f800000u);
      }
      if (any) bad.store(1, std::memory_order_relaxed);
      {
        std::lock_guard<std::mutex> lk(mu);
        done[(size_t)b] = 1;
      }
      cv.notify_all();
    }
  };
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int w = 0; w < nt; w++) th.emplace_back(work, w);
  bool copy_ok = d != nullptr;
  for (int64_t b = 0; b < nblk; b++) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return done[(size_t)b] != 0; });
    }
    if (!copy_ok) continue;
    const int64_t lo = b * blk_rows * p, hi = std::min(n, (b + 1) * blk_rows) * p;
    if (hipMemcpyAsync((float*)d + lo, out + lo, (size_t)(hi - lo) * sizeof(float),
                       hipMemcpyHostToDevice, st) != hipSuccess) {
      (void)hipGetLastError();
      copy_ok = false;
    }
  }
  for (auto& t : th) t.join();
  if (st) {
    if (hipStreamSynchronize(st) != hipSuccess) {
      (void)hipGetLastError();
      copy_ok = false;
    }
    (void)hipStreamDestroy(st);
  }
  *finite = bad.load() ? 0 : 1;
  if (d && (!copy_ok || !*finite)) {
    dev_free(d);
    d = nullptr;
  }
  if (d) {
    Staged e{out, n, p, 0, device, d, std::this_thread::get_id(), false, 0, false, {}, {}};
    if (*finite) {
      std::vector<float> mn, mx;
      for (int w = 0; w < nt; w++) {
        if (tmin[(size_t)w].empty()) continue;
        if (mn.empty()) {
          mn = tmin[(size_t)w];
          mx = tmax[(size_t)w];
          continue;
        }
        for (int64_t c = 0; c < p; c++) {
          mn[c] = tmin[(size_t)w][c] < mn[c] ? tmin[(size_t)w][c] : mn[c];
          mx[c] = tmax[(size_t)w][c] > mx[c] ? tmax[(size_t)w][c] : mx[c];
        }
      }
      e.cmin.assign((const char*)mn.data(), (const char*)(mn.data() + mn.size()));
      e.cmax.assign((const char*)mx.data(), (const char*)(mx.data() + mx.size()));
    }
    std::lock_guard<std::mutex> lk(staged_mu);
    staged.push_back(std::move(e));
    *handle = (uint64_t)(uintptr_t)d;
  }
  trace_mark("stage: cast + upload of X");
  return FS_OK;
}

int unstage_x(uint64_t handle) {
  void* d = (void*)(uintptr_t)handle;
  bool borrowed = false;
  {
    std::lock_guard<std::mutex> lk(staged_mu);
    auto it = std::find_if(staged.begin(), staged.end(),
                           [&](const Staged& e) { return e.dev == d && !e.released; });
    if (it == staged.end()) {
      set_error("fs_unstage_x: unknown handle");
      return FS_EINVAL;
    }
    if (it->refs > 0) {  // plans still read it: the last staged_release frees it
      it->released = true;
      return FS_OK;
    }
    borrowed = it->borrowed;
    staged.erase(it);
  }
  if (!borrowed) dev_free(d);  // every reader synchronised its stream before returning
  return FS_OK;
}

const void* staged_acquire(const void* host, int64_t n, int64_t p, int x_is_f64, int device) {
  std::lock_guard<std::mutex> lk(staged_mu);
  // only the library's own copies: a caller-owned one (stage_x_device) may
  // be freed by its owner while a plan still lives, so plans copy those
  for (Staged& e : staged)
    if (!e.released && !e.borrowed && e.host == host && e.n == n && e.p == p &&
        e.f64 == (x_is_f64 ? 1 : 0) && e.device == device &&
        e.owner == std::this_thread::get_id()) {
      e.refs++;
      return e.dev;
    }
  return nullptr;
}

void staged_release(const void* dev) {
  void* q = nullptr;
  {
    std::lock_guard<std::mutex> lk(staged_mu);
    auto it = std::find_if(staged.begin(), staged.end(), [&](const Staged& e) {
      return e.dev == dev && e.refs > 0;
    });
    if (it == staged.end()) return;
    if (--it->refs == 0 && it->released) {
      if (!it->borrowed) q = it->dev;
      staged.erase(it);
    }
  }
  if (q) dev_free(q);  // the releasing plan synchronised its streams
}

bool staged_extrema(const void* dev, void* cmin, void* cmax) {
  std::lock_guard<std::mutex> lk(staged_mu);
  for (const Staged& e : staged)
    if (e.dev == dev && !e.cmin.empty()) {
      std::memcpy(cmin, e.cmin.data(), e.cmin.size());
      std::memcpy(cmax, e.cmax.data(), e.cmax.size());
      return true;
    }
  return false;
}

const void* staged_lookup(const void* host, int64_t n, int64_t p, int x_is_f64, int device) {
  std::lock_guard<std::mutex> lk(staged_mu);
  for (const Staged& e : staged)
    if (!e.released && e.host == host && e.n == n && e.p == p && e.f64 == (x_is_f64 ? 1 : 0) &&
        e.device == device && e.owner == std::this_thread::get_id())
      return e.dev;
  return nullptr;
}

}  // namespace gpu
}  // namespace fs
