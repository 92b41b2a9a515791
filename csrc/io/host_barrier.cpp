// Single-node host barrier for the ranks of one job: a sense-reversing counter in a POSIX shared-memory page.
//
// Used by bench.py to bracket the timed region (barrier + synchronize on both sides).  torch.distributed's
// barrier on the RCCL backend is an all-reduce of one element plus a stream synchronisation (tens of us per call
// at 8 ranks); the ranks of a single-node job can meet in host memory instead, in about a microsecond of
// cache-line traffic, so the barrier that closes the timed region measures the ranks' arrival times and not a
// collective's latency.  Semantics are those of any barrier: no rank returns before every rank has arrived.
//
// Protocol: {count, sense} 32-bit atomics on separate cache lines.  A rank flips its local sense, increments
// count; the last arriver resets count and publishes the new sense; everyone else spins (pause, then
// sched_yield) until sense equals its local sense.  Spins are bounded by a timeout (the call returns an error
// instead of hanging when a peer died).  The creator (rank 0) makes the segment with O_EXCL under a name that
// is unique to the job; peers open it only after a torch.distributed barrier, and rank 0 unlinks it at close.
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#define ECG_API extern "C" __attribute__((visibility("default")))

namespace {

struct alignas(64) Line {
  std::atomic<int32_t> v;
  char pad[60];
};

struct Shared {
  Line count;
  Line sense;
  Line world;
};

struct Barrier {
  Shared* sh = nullptr;
  int world = 0;
  int local_sense = 0;
  bool creator = false;
  char name[128];
};

constexpr int kErrArg = -1, kErrSys = -2, kErrTimeout = -3, kErrWorld = -4;

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

}  // namespace

// Create (create != 0: rank 0, O_EXCL) or open the segment ``name`` (e.g. "/ecg_bar_<token>") for ``world``
// ranks.  Returns an opaque handle in *out, 0 on success, < 0 on error.
ECG_API int ecg_host_barrier_open(const char* name, int world, int create, void** out) {
  if (!name || !out || world < 1 || strlen(name) >= sizeof(Barrier::name) || name[0] != '/') return kErrArg;
  const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return kErrSys;
  if (create && ftruncate(fd, sizeof(Shared)) != 0) {
    close(fd);
    shm_unlink(name);
    return kErrSys;
  }
  void* p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (create) shm_unlink(name);
    return kErrSys;
  }
  Barrier* b = new Barrier();
  b->sh = static_cast<Shared*>(p);
  b->world = world;
  b->creator = create != 0;
  strncpy(b->name, name, sizeof(b->name) - 1);
  if (create) {  // a fresh segment is zero-filled; record the world size for the peers' check
    b->sh->count.v.store(0, std::memory_order_relaxed);
    b->sh->sense.v.store(0, std::memory_order_relaxed);
    b->sh->world.v.store(world, std::memory_order_release);
  } else if (b->sh->world.v.load(std::memory_order_acquire) != world) {
    munmap(p, sizeof(Shared));
    delete b;
    return kErrWorld;
  }
  *out = b;
  return 0;
}

// Wait until all ``world`` ranks have called this (the n-th call of every rank meets the n-th call of the
// others).  0 on success, kErrTimeout after ``timeout_ms`` (the barrier is then unusable).
ECG_API int ecg_host_barrier_wait(void* handle, int timeout_ms) {
  Barrier* b = static_cast<Barrier*>(handle);
  if (!b) return kErrArg;
  const int s = b->local_sense = 1 - b->local_sense;
  if (b->sh->count.v.fetch_add(1, std::memory_order_acq_rel) == b->world - 1) {
    b->sh->count.v.store(0, std::memory_order_relaxed);
    b->sh->sense.v.store(s, std::memory_order_release);
    return 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (long it = 0;; ++it) {
    if (b->sh->sense.v.load(std::memory_order_acquire) == s) return 0;
    if (it < 20000) {
      cpu_relax();
    } else {
      sched_yield();  // a long wait (a straggling rank): stop burning the core
      if ((it & 255) == 0 && std::chrono::duration_cast<std::chrono::milliseconds>(
                                 std::chrono::steady_clock::now() - t0).count() > timeout_ms)
        return kErrTimeout;
    }
  }
}

// Remove the segment's name once every rank holds its mapping (the creator calls this right after the ranks
// agreed they all opened it): the page then lives exactly as long as the mappings, so a rank that crashes or
// times out never leaves /dev/shm/ecg_bar_* behind.  Idempotent; a no-op for non-creators.
ECG_API int ecg_host_barrier_unlink(void* handle) {
  Barrier* b = static_cast<Barrier*>(handle);
  if (!b || !b->creator) return 0;
  b->creator = false;
  return shm_unlink(b->name) == 0 ? 0 : kErrSys;
}

// Unmap; a creator that has not unlinked yet also unlinks the name (peers keep their mapping until they close).
ECG_API int ecg_host_barrier_close(void* handle) {
  Barrier* b = static_cast<Barrier*>(handle);
  if (!b) return 0;
  munmap(b->sh, sizeof(Shared));
  if (b->creator) shm_unlink(b->name);
  delete b;
  return 0;
}
