// ThreadSanitizer driver of the direct-RCCL completion tracking (csrc/include/tea_watchdog.h):
// the same template rccl_direct.cpp runs on HIP events + RCCL, here on a fake backend whose
// events complete after a random delay (or never, on one "held" stream) and one of whose
// communicators reports an async error.  Four enqueue threads track collectives and wait on
// them, one thread destroys communicators, one aborts a healthy one, while the watchdog thread
// retires probes, records follow-ups, marks deadlines and aborts.  Built with -fsanitize=thread
// by tests/test_sanitizers.py (ROCm's clang: gcc 11's TSan reports false "double lock"s for a
// lock_guard released by an exception unwind); any data race fails the run.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "tea_watchdog.h"

namespace {

using Clock = std::chrono::steady_clock;
constexpr int kHeldStream = 666;  // events recorded here never complete
constexpr int kCaptureStream = 7;  // "being captured": no follow-up probes
constexpr int kErrComm = 99;       // reports an async error

struct FakeBackend {
  using Event = int;  // 1-based id into done_at (0 = none)
  using Stream = int;
  using Comm = int;
  std::mutex m;
  std::vector<Clock::time_point> done_at;
  std::mt19937 rng{7};
  std::atomic<int> aborts{0}, teardowns{0}, created{0};

  Event create_event() {
    std::lock_guard<std::mutex> lock(m);
    done_at.push_back(Clock::time_point::max());
    ++created;
    return static_cast<int>(done_at.size());
  }
  bool record(Event e, Stream s) {
    std::lock_guard<std::mutex> lock(m);
    const auto delay = std::chrono::microseconds(std::uniform_int_distribution<int>(0, 400)(rng));
    done_at[e - 1] = s == kHeldStream ? Clock::time_point::max() : Clock::now() + delay;
    return true;
  }
  int query(Event e) {
    std::lock_guard<std::mutex> lock(m);
    return Clock::now() >= done_at[e - 1] ? 0 : 1;
  }
  void destroy_event(Event) {}
  bool capturing(Stream s) { return s == kCaptureStream; }
  void set_device(int) {}
  void comm_abort(Comm) { ++aborts; }
  bool async_error(Comm c, std::string* why) {
    if (c != kErrComm) return false;
    *why = "fake remote error";
    return true;
  }
  bool tracking_enabled() { return true; }
  bool teardown_on_failure() { return false; }
  void teardown(const std::string&) { ++teardowns; }
  void fail(const std::string& msg) { throw std::runtime_error(msg); }  // raises to the caller
};

}  // namespace

int main() {
  FakeBackend b;
  tea_wd::Watchdog<FakeBackend> wd(b);
  // handles 0-5 healthy (streams 1-3, one capture stream), 6 on the held stream, 7 async error,
  // 8-9 destroyed mid-run, 10 aborted by "a peer" mid-run
  std::vector<int64_t> h;
  for (int i = 0; i < 11; ++i) h.push_back(wd.add(i == 7 ? kErrComm : i, 0, i == 6 ? 30 : 2000));
  auto stream_of = [](int i) { return i == 6 ? kHeldStream : i == 4 ? kCaptureStream : 1 + i % 3; };
  std::atomic<int> unexpected{0}, waits_ok{0}, waits_failed{0}, unusable{0};
  std::atomic<bool> go{false};

  auto enqueuer = [&](int tid) {
    std::mt19937 r(100 + tid);
    while (!go.load()) std::this_thread::yield();
    for (int it = 0; it < 3000; ++it) {
      const int i = std::uniform_int_distribution<int>(0, 10)(r);
      try {
        wd.usable(h[i]);  // the real enqueue path checks first, then RCCL, then track
        wd.track(h[i], stream_of(i));
        if (it % 97 == 0) {
          const bool ok = wd.wait(h[i], i == 6 ? 20 : 2000);
          (ok ? waits_ok : waits_failed) += 1;
          if (!ok && i != 6) ++unexpected;
        }
      } catch (const std::runtime_error&) {
        ++unusable;  // failed / aborted / destroyed by another thread: the caller's error
      }
      if (it % 50 == 0) std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  };
  auto destroyer = [&]() {
    while (!go.load()) std::this_thread::yield();
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    for (int i : {8, 9}) {
      if (!wd.drain_for_destroy(h[i], std::chrono::seconds(5))) ++unexpected;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
    wd.mark_failed(h[10], "aborted: a peer failed", true);
    if (!wd.wait_aborted(h[10], 5000)) ++unexpected;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t) th.emplace_back(enqueuer, t);
  th.emplace_back(destroyer);
  go = true;
  for (auto& t : th) t.join();
  // the held communicator's deadline and the async error are found by the watchdog
  const auto until = Clock::now() + std::chrono::seconds(10);
  while ((wd.state(h[6]) < tea_wd::kAborted || wd.state(h[7]) < tea_wd::kAborted) && Clock::now() < until)
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  // the healthy ones drain: every probe retires
  for (int i = 0; i < 6; ++i)
    if (!wd.wait(h[i], 5000)) ++unexpected;
  const int s6 = wd.state(h[6]), s7 = wd.state(h[7]), s8 = wd.state(h[8]), s10 = wd.state(h[10]);
  wd.shutdown();
  bool ok = unexpected == 0 && s6 == tea_wd::kAborted && s7 == tea_wd::kAborted && s8 == tea_wd::kDestroyed &&
            s10 == tea_wd::kAborted && b.teardowns == 0 && b.aborts >= 3;
  for (int i = 0; i < 6; ++i) ok = ok && wd.state(h[i]) == tea_wd::kOk;
  std::printf("watchdog_tsan: waits ok %d failed %d unusable %d unexpected %d aborts %d events %d states %d %d %d %d\n",
              waits_ok.load(), waits_failed.load(), unusable.load(), unexpected.load(), b.aborts.load(),
              b.created.load(), s6, s7, s8, s10);
  if (!ok) return 1;
  std::printf("watchdog_tsan: ok\n");
  return 0;
}
