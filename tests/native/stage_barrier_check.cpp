// Test driver: StageBarrier (fastselect_amd/csrc/fs_internal.h), the barrier
// of the devices= threads.  ADVICE r3: a waiter used to read the shared
// status only after re-acquiring the lock, so when the last thread to arrive
// at a passed stage went on and failed the next stage first, the waiter saw
// the passed stage as failed, skipped its remaining barriers and left its
// peers waiting forever.  Here thread 0 always arrives last at stage 1 and
// fails stage 2 at once; thread 1 must see stage 1 passed and stage 2
// failed, every time.  Prints "ok <rounds>" or the first bad round.
#include <cstdio>
#include <thread>

#include "../../fastselect_amd/csrc/fs_internal.h"

void fs::set_error(const std::string&) {}

int main() {
  const int rounds = 2000;
  for (int r = 0; r < rounds; r++) {
    fs::StageBarrier bar(2);
    bool s1 = false, s2 = true;
    std::thread t1([&] {
      s1 = bar.arrive(0, "");  // arrives first and waits
      s2 = bar.arrive(0, "");
    });
    // let thread 1 block in stage 1 before thread 0 completes it
    while (true) {
      std::this_thread::yield();
      if (bar.waiting() == 1) break;
    }
    const bool a = bar.arrive(0, "");    // completes stage 1 (passed)
    const bool b = bar.arrive(-4, "x");  // fails stage 2 right away
    t1.join();
    if (!a || b || !s1 || s2) {
      std::printf("bad round %d: t0 %d %d, t1 %d %d\n", r, (int)a, (int)b, (int)s1, (int)s2);
      return 1;
    }
  }
  std::printf("ok %d\n", rounds);
  return 0;
}
