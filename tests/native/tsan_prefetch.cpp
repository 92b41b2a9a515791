// ThreadSanitizer harness for the Module-1 producer/consumer ring (csrc/io/shard_io.cpp), host-memory mode
// (pinned = 0: no HIP calls).  SURVEY §5.2: the consumer checks every batch's content (window index pattern
// written by the test), recycles slots in a shuffled order, and a second consumer thread races shutdown.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

extern "C" {
int ecg_prefetch_create(const char** paths, int npaths, int batch, int nslots, int normalize, int pinned, int loop,
                        void** handle, int64_t* L_out);
int ecg_prefetch_start(void* handle);
float* ecg_prefetch_slot_ptr(void* handle, int slot);
int ecg_prefetch_next(void* handle, int timeout_ms, int* slot, int* n, double* fill_ms);
int ecg_prefetch_recycle(void* handle, int slot);
int ecg_prefetch_shutdown(void* handle);
int ecg_prefetch_destroy(void* handle);
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const char* paths[1] = {argv[1]};
  const int64_t N = atoll(argv[2]);
  for (int round = 0; round < 2; ++round) {
    void* h = nullptr;
    int64_t L = 0;
    if (ecg_prefetch_create(paths, 1, 7, 3, 0, 0, round, &h, &L)) return 3;
    if (ecg_prefetch_start(h)) return 4;
    int64_t seen = 0;
    int pending = -1;
    bool ok = true;
    for (int it = 0; it < 200; ++it) {
      int slot = -1, n = 0;
      double fill = 0;
      const int st = ecg_prefetch_next(h, 2000, &slot, &n, &fill);
      if (st != 0 || n <= 0) break;  // EOF sentinel / error
      const float* p = ecg_prefetch_slot_ptr(h, slot);
      for (int i = 0; i < n; ++i) {  // window w holds the value w (mod N when looping)
        const float want = (float)((seen + i) % N);
        if (p[(int64_t)i * L] != want || p[(int64_t)i * L + L - 1] != want) ok = false;
      }
      seen += n;
      // hold one slot back and recycle it one batch late (out-of-order recycling)
      if (pending >= 0) ecg_prefetch_recycle(h, pending);
      pending = slot;
    }
    if (pending >= 0) ecg_prefetch_recycle(h, pending);
    std::thread t([h] { ecg_prefetch_shutdown(h); });  // shutdown from another thread
    t.join();
    ecg_prefetch_destroy(h);
    if (!ok) {
      fprintf(stderr, "content mismatch\n");
      return 5;
    }
    if (round == 0 && seen != N / 7 * 7 && seen != N) {
      fprintf(stderr, "saw %lld of %lld\n", (long long)seen, (long long)N);
      return 6;
    }
  }
  printf("tsan harness ok\n");
  return 0;
}
