// Host-side stress test of the native FramePool (csrc/runtime/frame_pool.cpp) for the
// sanitizer builds: 8 threads acquire / write / release slots with random
// timeouts while a checker asserts no slot is ever held twice; a closer thread then wakes the
// blocked waiters.  Built by tests/test_native_sanitizers.py with -fsanitize=address,undefined
// and, separately, -fsanitize=thread (CPU storage: device_index = -1).
#include "../../aiko_services_amd/csrc/runtime/frame_pool.cpp"

#include <atomic>
#include <cstring>
#include <cstdio>
#include <random>
#include <thread>

int main() {
  constexpr int kSlots = 6, kThreads = 8, kIters = 4000;
  FramePool pool(kSlots, 1000, -1);
  std::atomic<int> held[kSlots];
  for (auto& h : held) h.store(0);
  std::atomic<long> ok{0}, timeouts{0};
  std::atomic<bool> bad{false};
  // raw slot memory: the worker threads call only the pool's own methods (no ATen ops, which
  // would run uninstrumented library code under TSan)
  uint8_t* base = pool.storage().data_ptr<uint8_t>();
  const int64_t sb = pool.slot_bytes();
  std::vector<std::thread> ts;
  for (int t = 0; t < kThreads; ++t) {
    ts.emplace_back([&, t] {
      std::mt19937 rng(t);
      for (int i = 0; i < kIters; ++i) {
        const int64_t s = pool.acquire(rng() % 3);
        if (s < 0) {
          ++timeouts;
          continue;
        }
        if (held[s].fetch_add(1) != 0) bad = true;           // two owners of one slot
        uint8_t* slot = base + s * sb;
        std::memset(slot, t + 1, sb);                        // owner writes its slot ...
        for (int64_t b = 0; b < sb; b += 97)
          if (slot[b] != t + 1) bad = true;                  // ... and nobody else does
        held[s].fetch_sub(1);
        pool.release(s);
        ++ok;
      }
    });
  }
  for (auto& th : ts) th.join();
  auto st = pool.stats();
  // blocked waiters are released by close()
  std::vector<int64_t> all;
  for (int i = 0; i < kSlots; ++i) all.push_back(pool.acquire(-1));
  std::thread waiter([&] { if (pool.acquire(-1) != -1) bad = true; });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  pool.close();
  waiter.join();
  // typed views still work after the stress (single-threaded)
  if (pool.view(0, {250}, static_cast<int64_t>(at::kInt)).numel() != 250) bad = true;
  std::printf("ok=%ld timeouts=%ld high_water=%lld acquired=%lld bad=%d\n", ok.load(), timeouts.load(),
              (long long)st[2], (long long)st[3], (int)bad.load());
  return (!bad && ok + timeouts == (long)kThreads * kIters && st[3] == ok && st[2] <= kSlots) ? 0 : 1;
}
