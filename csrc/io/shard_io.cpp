// Native Module-1 data path: mmap shard reader, pinned-slab ring with a producer thread, copy-stream
// H2D with hipEvent-fenced slab reuse, and a chunked bulk uploader for GPU-resident shards.
//
// Reference (Python, experimental): Module_1/labl_loader(EXPERIMENTAL).py
//   LABLShardedReader.open_shard (:7-28)  -> ecg_shard_open / ecg_shard_close (mmap + madvise)
//   PinnedRing (:30-36)                    -> slots allocated with hipHostMalloc (page-locked, device-mapped)
//   LABLPrefetcher (:38-136)               -> Prefetcher: std::thread producer, free/full queues,
//                                             per-window z-score (float64 accumulate) , EOF sentinel n=0
// and the one-shot upload of Module_3/shard_dataset.py:103-115 -> ecg_upload_shards (pinned double
// buffer + hipMemcpyAsync on the caller's stream, sized for multi-GB per-GPU shards on 288 GB HBM).
//
// Race safety (the reference recycles a slab while its non_blocking copy may still be in flight,
// train_ecg_labl(EXPERIMENTAL).py:59-62,82): a slot handed to ecg_prefetch_h2d / recycle_after is
// only refilled after hipEventSynchronize on the event recorded behind the copy that consumed it.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <mutex>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#define ECG_API extern "C" __attribute__((visibility("default")))

namespace {

enum Status : int { kOk = 0, kBadArg = 1, kIoError = 4, kHipError = 3, kTimeout = 5, kEof = 6 };

struct ShardMap {
  int fd = -1;
  void* base = nullptr;
  size_t size = 0;
  int64_t N = 0, L = 0;
  const float* data() const { return reinterpret_cast<const float*>(static_cast<const char*>(base) + 16); }
};

int open_map(const char* path, ShardMap* m) {
  m->fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (m->fd < 0) return kIoError;
  struct stat st;
  if (fstat(m->fd, &st) != 0 || st.st_size < 16) {
    ::close(m->fd);
    m->fd = -1;
    return kIoError;
  }
  m->size = (size_t)st.st_size;
  m->base = mmap(nullptr, m->size, PROT_READ, MAP_PRIVATE, m->fd, 0);
  if (m->base == MAP_FAILED) {
    m->base = nullptr;
    ::close(m->fd);
    m->fd = -1;
    return kIoError;
  }
  madvise(m->base, m->size, MADV_SEQUENTIAL);
  const int64_t* hdr = static_cast<const int64_t*>(m->base);
  m->N = hdr[0];
  m->L = hdr[1];
  if (m->N < 0 || m->L <= 0 || (size_t)(16 + 4 * m->N * m->L) != m->size) {
    munmap(m->base, m->size);
    ::close(m->fd);
    m->base = nullptr;
    m->fd = -1;
    return kIoError;
  }
  return kOk;
}

void close_map(ShardMap* m) {
  if (m->base) munmap(m->base, m->size);
  if (m->fd >= 0) ::close(m->fd);
  m->base = nullptr;
  m->fd = -1;
}

void zscore_copy(const float* src, float* dst, int64_t L) {
  double s = 0.0;
  for (int64_t i = 0; i < L; ++i) s += src[i];
  const double mean = s / (double)L;
  double v = 0.0;
  for (int64_t i = 0; i < L; ++i) {
    double d = src[i] - mean;
    v += d * d;
  }
  const double sd = std::sqrt(v / (double)L) + 1e-8;
  for (int64_t i = 0; i < L; ++i) dst[i] = (float)((src[i] - mean) / sd);
}

struct Filled {
  int slot;
  int n;
  double fill_ms;
};

struct Prefetcher {
  std::vector<std::string> paths;
  int B = 0, nslots = 0;
  int64_t L = 0;
  bool normalize = true, pinned = true, loop = false;
  std::vector<float*> slots;
  std::vector<hipEvent_t> events;     // fence recorded behind the consumer's copy (pinned mode)
  std::vector<char> event_pending;
  std::mutex mu;
  std::condition_variable cv_free, cv_full;
  std::deque<int> q_free;
  std::deque<Filled> q_full;
  std::thread producer;
  std::atomic<bool> stop{false};
  bool started = false;
  int shard_idx = 0;
  int64_t offset = 0;
  std::string error;

  ~Prefetcher() { shutdown(); release(); }

  void release() {
    for (size_t i = 0; i < slots.size(); ++i) {
      if (!slots[i]) continue;
      if (pinned) (void)hipHostFree(slots[i]);
      else std::free(slots[i]);
      slots[i] = nullptr;
    }
    for (auto& e : events)
      if (e) (void)hipEventDestroy(e);
    events.clear();
  }

  void shutdown() {
    stop.store(true);
    cv_free.notify_all();
    cv_full.notify_all();
    if (producer.joinable()) producer.join();
  }

  void push_full(Filled f) {
    {
      std::lock_guard<std::mutex> g(mu);
      q_full.push_back(f);
    }
    cv_full.notify_one();
  }

  void run() {
    ShardMap cur;
    int cur_idx = -1;
    try {
      while (!stop.load()) {
        int slot;
        {
          std::unique_lock<std::mutex> g(mu);
          cv_free.wait_for(g, std::chrono::milliseconds(100), [&] { return !q_free.empty() || stop.load(); });
          if (stop.load()) break;
          if (q_free.empty()) continue;
          slot = q_free.front();
          q_free.pop_front();
        }
        if (pinned && event_pending[slot]) {  // the previous H2D out of this slab must be finished
          (void)hipEventSynchronize(events[slot]);
          event_pending[slot] = 0;
        }
        if (shard_idx >= (int)paths.size()) {
          if (loop && !paths.empty()) {
            shard_idx = 0;
            offset = 0;
          } else {
            push_full({slot, 0, 0.0});  // EOF sentinel
            break;
          }
        }
        const auto t0 = std::chrono::steady_clock::now();
        int n = 0;
        float* dst = slots[slot];
        while (n < B && !stop.load()) {
          if (shard_idx >= (int)paths.size()) break;
          if (cur_idx != shard_idx) {
            close_map(&cur);
            if (open_map(paths[shard_idx].c_str(), &cur) != kOk || cur.L != L) {
              error = "bad shard: " + paths[shard_idx];
              throw 1;
            }
            cur_idx = shard_idx;
          }
          if (offset >= cur.N) {
            ++shard_idx;
            offset = 0;
            break;  // like the reference, a batch never spans two shards
          }
          const int64_t take = std::min<int64_t>(B - n, cur.N - offset);
          const float* src = cur.data() + offset * L;
          if (normalize) {
            for (int64_t r = 0; r < take; ++r) zscore_copy(src + r * L, dst + (n + r) * L, L);
          } else {
            std::memcpy(dst + (int64_t)n * L, src, (size_t)take * L * sizeof(float));
          }
          n += (int)take;
          offset += take;
        }
        const double ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (n == 0) {
          std::lock_guard<std::mutex> g(mu);
          q_free.push_front(slot);
          continue;
        }
        push_full({slot, n, ms});
      }
    } catch (...) {
      push_full({-1, 0, 0.0});  // wake the consumer; error string is queryable
    }
    close_map(&cur);
  }
};

}  // namespace

// ------------------------------------------------------------------ mmap reader
ECG_API int ecg_shard_open(const char* path, void** handle, int64_t* N, int64_t* L) {
  if (!path || !handle) return kBadArg;
  ShardMap* m = new ShardMap();
  int st = open_map(path, m);
  if (st != kOk) {
    delete m;
    return st;
  }
  *handle = m;
  if (N) *N = m->N;
  if (L) *L = m->L;
  return kOk;
}

ECG_API const float* ecg_shard_data(void* handle) { return handle ? static_cast<ShardMap*>(handle)->data() : nullptr; }

ECG_API int ecg_shard_close(void* handle) {
  if (!handle) return kOk;
  ShardMap* m = static_cast<ShardMap*>(handle);
  close_map(m);
  delete m;
  return kOk;
}

// ------------------------------------------------------------------ prefetcher (LABL)
ECG_API int ecg_prefetch_create(const char** paths, int npaths, int batch, int nslots, int normalize, int pinned,
                                int loop, void** handle, int64_t* L_out) {
  if (!paths || npaths <= 0 || batch <= 0 || nslots <= 0 || !handle) return kBadArg;
  Prefetcher* p = new Prefetcher();
  for (int i = 0; i < npaths; ++i) p->paths.emplace_back(paths[i]);
  ShardMap m;
  if (open_map(p->paths[0].c_str(), &m) != kOk) {
    delete p;
    return kIoError;
  }
  p->L = m.L;
  close_map(&m);
  p->B = batch;
  p->nslots = nslots;
  p->normalize = normalize != 0;
  p->pinned = pinned != 0;
  p->loop = loop != 0;
  const size_t bytes = (size_t)batch * p->L * sizeof(float);
  p->slots.assign(nslots, nullptr);
  p->event_pending.assign(nslots, 0);
  for (int i = 0; i < nslots; ++i) {
    void* ptr = nullptr;
    if (p->pinned) {
      if (hipHostMalloc(&ptr, bytes, hipHostMallocDefault) != hipSuccess) {
        delete p;
        return kHipError;
      }
    } else {
      ptr = std::aligned_alloc(64, (bytes + 63) / 64 * 64);
      if (!ptr) {
        delete p;
        return kBadArg;
      }
    }
    p->slots[i] = static_cast<float*>(ptr);
    p->q_free.push_back(i);
  }
  if (p->pinned) {
    p->events.assign(nslots, nullptr);
    for (int i = 0; i < nslots; ++i)
      if (hipEventCreateWithFlags(&p->events[i], hipEventDisableTiming) != hipSuccess) {
        delete p;
        return kHipError;
      }
  }
  *handle = p;
  if (L_out) *L_out = p->L;
  return kOk;
}

ECG_API int ecg_prefetch_start(void* handle) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  if (!p || p->started) return kBadArg;
  p->started = true;
  p->producer = std::thread([p] { p->run(); });
  return kOk;
}

ECG_API float* ecg_prefetch_slot_ptr(void* handle, int slot) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  if (!p || slot < 0 || slot >= p->nslots) return nullptr;
  return p->slots[slot];
}

// Blocks up to timeout_ms for a filled slab. n == 0 signals end of data (or a producer error).
ECG_API int ecg_prefetch_next(void* handle, int timeout_ms, int* slot, int* n, double* fill_ms) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  if (!p || !slot || !n) return kBadArg;
  std::unique_lock<std::mutex> g(p->mu);
  const bool ok = p->cv_full.wait_for(g, std::chrono::milliseconds(timeout_ms),
                                      [&] { return !p->q_full.empty() || p->stop.load(); });
  if (!ok || p->q_full.empty()) return kTimeout;
  Filled f = p->q_full.front();
  p->q_full.pop_front();
  *slot = f.slot;
  *n = f.n;
  if (fill_ms) *fill_ms = f.fill_ms;
  if (f.n == 0) {
    if (f.slot >= 0) p->q_free.push_back(f.slot);
    return p->error.empty() ? kEof : kIoError;
  }
  return kOk;
}

ECG_API int ecg_prefetch_recycle(void* handle, int slot) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  if (!p || slot < 0 || slot >= p->nslots) return kBadArg;
  {
    std::lock_guard<std::mutex> g(p->mu);
    p->q_free.push_back(slot);
  }
  p->cv_free.notify_one();
  return kOk;
}

// Recycle once all work currently enqueued on ``stream`` (e.g. the H2D reading the slab) is done.
ECG_API int ecg_prefetch_recycle_after(void* handle, int slot, hipStream_t stream) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  if (!p || slot < 0 || slot >= p->nslots || !p->pinned) return kBadArg;
  if (hipEventRecord(p->events[slot], stream) != hipSuccess) return kHipError;
  p->event_pending[slot] = 1;
  return ecg_prefetch_recycle(handle, slot);
}

// One coalesced async H2D of the slab into ``dst`` on ``stream``, then fence-and-recycle the slab.
ECG_API int ecg_prefetch_h2d(void* handle, int slot, int n, float* dst, hipStream_t stream) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  if (!p || !dst || slot < 0 || slot >= p->nslots || n <= 0 || n > p->B || !p->pinned) return kBadArg;
  const size_t bytes = (size_t)n * p->L * sizeof(float);
  if (hipMemcpyAsync(dst, p->slots[slot], bytes, hipMemcpyHostToDevice, stream) != hipSuccess) return kHipError;
  return ecg_prefetch_recycle_after(handle, slot, stream);
}

ECG_API int ecg_prefetch_shutdown(void* handle) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  if (!p) return kBadArg;
  p->shutdown();
  return kOk;
}

ECG_API int ecg_prefetch_destroy(void* handle) {
  delete static_cast<Prefetcher*>(handle);
  return kOk;
}

ECG_API const char* ecg_prefetch_error(void* handle) {
  Prefetcher* p = static_cast<Prefetcher*>(handle);
  return p ? p->error.c_str() : "";
}

// ------------------------------------------------------------------ bulk upload (GPU-resident shards)
// Streams up to max_rows windows of the given shards into dst [max_rows, L] through kStages pinned staging
// buffers of chunk_rows windows.  Per chunk, ``threads`` host threads copy disjoint slices of the mmap'd shard
// into the free staging buffer (one thread cannot move page-cache bytes at the PCIe/DMA rate), then one
// hipMemcpyAsync moves it to HBM while the next chunk is being copied: host copy and DMA overlap, and a
// staging buffer is reused only after the event behind its DMA completed.  Returns rows uploaded in *rows_out.
// Synchronises ``stream`` before returning (the staging buffers are freed).  Sized for multi-GB per-GPU shards
// on 288 GB of HBM (Module_3/shard_dataset.py:103-115 does one pageable, effectively synchronous copy).
constexpr int kStages = 3;

void parallel_copy(float* dst, const float* src, size_t bytes, int threads) {
  if (threads <= 1 || bytes < ((size_t)4 << 20)) {
    std::memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> pool;
  const size_t per = (bytes / threads + 4095) & ~(size_t)4095;
  for (int t = 0; t < threads; ++t) {
    const size_t lo = std::min(bytes, (size_t)t * per), hi = std::min(bytes, lo + per);
    if (lo >= hi) break;
    pool.emplace_back([=] {
      std::memcpy(reinterpret_cast<char*>(dst) + lo, reinterpret_cast<const char*>(src) + lo, hi - lo);
    });
  }
  for (auto& th : pool) th.join();
}

ECG_API int ecg_upload_shards_mt(const char** paths, int npaths, int64_t max_rows, int64_t L, float* dst,
                                 int64_t chunk_rows, int threads, hipStream_t stream, int64_t* rows_out) {
  if (!paths || npaths <= 0 || !dst || L <= 0 || chunk_rows <= 0) return kBadArg;
  if (threads <= 0) threads = 1;
  const size_t chunk_bytes = (size_t)chunk_rows * L * sizeof(float);
  float* stage[kStages] = {};
  hipEvent_t ev[kStages] = {};
  bool pending[kStages] = {};
  int st = kOk;
  int64_t row = 0;
  for (int i = 0; i < kStages; ++i) {
    if (hipHostMalloc((void**)&stage[i], chunk_bytes, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) {
      st = kHipError;
      break;
    }
  }
  int s = 0;
  for (int f = 0; f < npaths && st == kOk && row < max_rows; ++f) {
    ShardMap m;
    if (open_map(paths[f], &m) != kOk || m.L != L) {
      close_map(&m);
      st = kIoError;
      break;
    }
    madvise(m.base, m.size, MADV_WILLNEED);
    int64_t off = 0;
    while (off < m.N && row < max_rows) {
      const int64_t take = std::min<int64_t>(std::min<int64_t>(chunk_rows, m.N - off), max_rows - row);
      if (pending[s]) {
        (void)hipEventSynchronize(ev[s]);
        pending[s] = false;
      }
      const size_t bytes = (size_t)take * L * sizeof(float);
      parallel_copy(stage[s], m.data() + off * L, bytes, threads);
      if (hipMemcpyAsync(dst + row * L, stage[s], bytes, hipMemcpyHostToDevice, stream) != hipSuccess ||
          hipEventRecord(ev[s], stream) != hipSuccess) {
        st = kHipError;
        break;
      }
      pending[s] = true;
      s = (s + 1) % kStages;
      row += take;
      off += take;
    }
    close_map(&m);
  }
  (void)hipStreamSynchronize(stream);
  for (int i = 0; i < kStages; ++i) {
    if (ev[i]) (void)hipEventDestroy(ev[i]);
    if (stage[i]) (void)hipHostFree(stage[i]);
  }
  if (rows_out) *rows_out = row;
  return st;
}

ECG_API int ecg_upload_shards(const char** paths, int npaths, int64_t max_rows, int64_t L, float* dst,
                              int64_t chunk_rows, hipStream_t stream, int64_t* rows_out) {
  return ecg_upload_shards_mt(paths, npaths, max_rows, L, dst, chunk_rows, 1, stream, rows_out);
}
