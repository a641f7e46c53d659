// Completion tracking + failure handling of the direct RCCL communicators,
// separated from HIP / RCCL so a fake backend can drive it under ThreadSanitizer
// (csrc/tests/watchdog_tsan.cpp, tests/test_sanitizers.py).  csrc/runtime/rccl_direct.cpp
// instantiates it with the HIP events + RCCL calls.
//
// Protocol (all shared state under one mutex; device calls outside it):
// * every collective enqueued on a communicator is tracked: a probe event is recorded behind
//   it when none is in flight, otherwise it is COUNTED and the watchdog thread records one
//   follow-up probe behind the counted ones when the in-flight probe retires (a record costs
//   ~5 us of host time: a burst of syncs pays it once);
// * the watchdog snapshots the oldest probes under the lock and queries them WITHOUT it (a
//   query takes the runtime's own locks), then re-finds each by sequence number (retired
//   events are pooled and reused);
// * a probe still pending at its deadline, a failed query or an async error marks the
//   communicator failed; the watchdog aborts it outside the lock and, unless a host waiter
//   observed the failure itself or teardown is off, tears the process down (c10d's default);
// * host waiters (wait / destroy) record their own probe behind everything they enqueued.
//
// Backend B provides: types Event, Stream, Comm; Event create_event(); bool record(Event, Stream);
// int query(Event) (0 done, 1 not ready, 2 error); const char* query_error(Event); void
// destroy_event(Event); bool capturing(Stream); void set_device(int); void comm_abort(Comm);
// bool async_error(Comm, std::string*); bool tracking_enabled(); bool teardown_on_failure();
// void teardown(const std::string& msg) (does not return for the real backend); [[noreturn]]
// void fail(const std::string& msg) (raises to the caller).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace tea_wd {

using Clock = std::chrono::steady_clock;

enum CommState : int { kOk = 0, kFailed = 1, kAborted = 2, kDestroyed = 3 };

template <class B>
class Watchdog {
 public:
  using Event = typename B::Event;
  using Stream = typename B::Stream;
  using Comm = typename B::Comm;

  explicit Watchdog(B& backend) : b_(backend) {}

  // ---- communicator table
  int64_t add(Comm comm, int device, int64_t timeout_ms) {
    auto e = std::make_unique<Entry>();
    e->comm = comm;
    e->device = device;
    e->timeout_ms = timeout_ms;
    std::lock_guard<std::mutex> lock(mu_);
    comms_.push_back(std::move(e));
    return static_cast<int64_t>(comms_.size()) - 1;
  }

  bool valid(int64_t h) {
    std::lock_guard<std::mutex> lock(mu_);
    return valid_locked(h);
  }

  // the communicator of a usable handle (fail() otherwise)
  Comm usable(int64_t h) {
    std::lock_guard<std::mutex> lock(mu_);
    Entry& c = ref_locked(h);
    const int s = c.state.load();
    if (s != kOk) b_.fail("rccl_direct: communicator " + std::to_string(h) + " is unusable (" +
                          (s == kDestroyed ? std::string("destroyed") : c.reason) + ")");
    return c.comm;
  }

  std::pair<Comm, int> comm_and_device(int64_t h) {
    std::lock_guard<std::mutex> lock(mu_);
    Entry& c = ref_locked(h);
    return {c.comm, c.device};
  }

  void set_timeout(int64_t h, int64_t ms) {
    std::lock_guard<std::mutex> lock(mu_);
    ref_locked(h).timeout_ms = ms;
  }

  // 0 ok, 1 failed (abort pending), 2 aborted, 3 destroyed; -1 unknown handle
  int state(int64_t h) {
    std::lock_guard<std::mutex> lock(mu_);
    return valid_locked(h) ? comms_[h]->state.load() : -1;
  }

  std::string reason(int64_t h) {
    std::lock_guard<std::mutex> lock(mu_);
    return ref_locked(h).reason;
  }

  // mark failed (once) and queue the abort for the watchdog thread (started if needed)
  void mark_failed(int64_t h, const std::string& why, bool observed) {
    std::lock_guard<std::mutex> lock(mu_);
    if (!valid_locked(h)) return;
    mark_failed_locked(h, why, observed);
    ensure_thread_locked();
  }

  bool wait_aborted(int64_t h, int64_t timeout_ms) {
    std::unique_lock<std::mutex> lk(mu_);
    Entry& c = ref_locked(h);
    return cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return c.state.load() >= kAborted; });
  }

  // ---- tracking: caller does NOT hold the lock.  A probe event when none is in flight, else
  // counted for the watchdog's follow-up probe.  force: always record (a host waiter needs a
  // probe behind everything it enqueued).  Returns the probe's sequence number (0 = none).
  uint64_t track(int64_t h, Stream s, bool force = false) {
    if (!b_.tracking_enabled() && !force) return 0;
    {
      std::lock_guard<std::mutex> lock(mu_);
      Entry& c = ref_locked(h);
      c.last_stream = s;
      c.has_last = true;
      if (c.probes > 0 && !force) {
        ++c.untracked;
        return 0;
      }
      ++c.probes;
      if (force) c.untracked = 0;  // the forced probe covers everything before it on the stream
    }
    const uint64_t seq = record_probe(h, s);
    if (seq == 0) b_.fail("rccl_direct: hipEventRecord failed");
    return seq;
  }

  // Block until the newest collective of h completes, at most timeout_ms.  false = deadline
  // passed: the communicator is marked failed (observed: no teardown) and aborted.
  bool wait(int64_t h, int64_t timeout_ms) {
    Stream s{};
    bool has_last = false;
    {
      std::lock_guard<std::mutex> lock(mu_);
      Entry& c = ref_locked(h);
      if (c.state.load() != kOk) b_.fail("rccl_direct: communicator " + std::to_string(h) + " is unusable (" + c.reason + ")");
      s = c.last_stream;
      has_last = c.has_last;
    }
    if (!has_last) return true;  // nothing was ever enqueued
    // our own probe behind the newest collective ("the newest pending entry" is not enough: a
    // counted collective's follow-up probe may still be on its way from the watchdog)
    const uint64_t seq = track(h, s, true);
    const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
    for (;;) {
      Event ev{};
      bool found = false;
      {
        std::lock_guard<std::mutex> lock(mu_);
        for (const auto& p : pending_)
          if (p.seq == seq) {
            ev = p.ev;
            found = true;
          }
        if (!found) return comms_[h]->state.load() == kOk;  // retired by the watchdog
      }
      // query outside the lock, then re-check by sequence number: the watchdog may have
      // retired the probe (and pooled its event) meanwhile
      const int q = b_.query(ev);
      {
        std::lock_guard<std::mutex> lock(mu_);
        bool still = false;
        for (const auto& p : pending_) still |= p.seq == seq;
        if (!still) return comms_[h]->state.load() == kOk;
        if (q == 0) return true;
        if (q == 2 || Clock::now() > deadline) {
          mark_failed_locked(h, q == 2 ? std::string("completion query failed") :
                                         "a collective did not complete within " + std::to_string(timeout_ms) + " ms",
                             true);
          ensure_thread_locked();
          return false;
        }
      }
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }

  // Destroy support: record a probe behind everything, wait (bounded) for this handle's probes
  // with the queries outside the lock; true = drained and the handle is now DESTROYED (the
  // caller frees the communicator), false = not ok / not drained (marked failed: aborted).
  bool drain_for_destroy(int64_t h, std::chrono::milliseconds budget) {
    Stream s{};
    bool has_last = false;
    {
      std::lock_guard<std::mutex> lock(mu_);
      if (!valid_locked(h) || comms_[h]->state.load() != kOk) return false;
      s = comms_[h]->last_stream;
      has_last = comms_[h]->has_last;
    }
    if (has_last) track(h, s, true);
    const auto deadline = Clock::now() + budget;
    for (;;) {
      std::vector<std::pair<uint64_t, Event>> mine;
      {
        std::lock_guard<std::mutex> lock(mu_);
        if (comms_[h]->state.load() != kOk) return false;
        for (const auto& p : pending_)
          if (p.handle == h) mine.emplace_back(p.seq, p.ev);
      }
      std::vector<uint64_t> busy_seqs;
      for (const auto& m : mine)
        if (b_.query(m.second) == 1) busy_seqs.push_back(m.first);
      bool busy = false;
      {
        std::lock_guard<std::mutex> lock(mu_);
        for (const auto& p : pending_)
          for (uint64_t q : busy_seqs) busy |= p.seq == q;  // still queued: the queried event was its own
        if (!busy) {
          if (comms_[h]->state.load() != kOk) return false;
          comms_[h]->state.store(kDestroyed);
          for (auto it = pending_.begin(); it != pending_.end();) {
            if (it->handle == h) {
              pool_.push_back(it->ev);
              it = pending_.erase(it);
            } else {
              ++it;
            }
          }
          return true;
        }
        if (Clock::now() > deadline) {
          mark_failed_locked(h, "work still pending at destroy", true);
          ensure_thread_locked();
          return false;
        }
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }

  // stop the watchdog thread (after draining the abort queue)
  void shutdown() {
    std::thread* t = nullptr;
    {
      std::lock_guard<std::mutex> lock(mu_);
      t = thread_;
      thread_ = nullptr;
      stop_ = true;
      cv_.notify_all();
    }
    if (t) {
      t->join();
      delete t;
    }
  }

  // test support: pending probes / pooled events (under the lock)
  size_t pending_count() {
    std::lock_guard<std::mutex> lock(mu_);
    return pending_.size();
  }

 private:
  struct Entry {
    Comm comm{};
    int device = 0;
    int64_t timeout_ms = 600000;
    std::atomic<int> state{kOk};
    bool observed = false;  // a blocking waiter reported the failure itself (no teardown)
    bool teardown = false;  // decided when the failure is detected
    std::string reason;
    int probes = 0;          // probe events in flight
    uint64_t untracked = 0;  // collectives enqueued behind the in-flight probe
    Stream last_stream{};
    bool has_last = false;
  };
  struct Pending {
    Event ev;
    int64_t handle;
    Clock::time_point deadline;
    uint64_t seq;
  };

  bool valid_locked(int64_t h) const {
    return h >= 0 && h < static_cast<int64_t>(comms_.size()) && comms_[h] != nullptr;
  }
  Entry& ref_locked(int64_t h) {
    if (!valid_locked(h)) b_.fail("rccl_direct: invalid communicator handle " + std::to_string(h));
    return *comms_[h];
  }

  void mark_failed_locked(int64_t h, const std::string& why, bool observed) {
    Entry& c = *comms_[h];
    int expect = kOk;
    if (!c.state.compare_exchange_strong(expect, kFailed)) return;
    c.reason = why;
    c.observed = observed;
    c.teardown = !observed && b_.teardown_on_failure();
    abort_q_.push_back(h);
    cv_.notify_all();
  }

  void ensure_thread_locked() {
    if (!thread_) {
      stop_ = false;
      thread_ = new std::thread([this] { loop(); });
    }
  }

  Event take_event() {
    Event ev{};
    bool have = false;
    {
      std::lock_guard<std::mutex> lock(mu_);
      if (!pool_.empty()) {
        ev = pool_.back();
        pool_.pop_back();
        have = true;
      }
    }
    if (!have) ev = b_.create_event();
    return ev;
  }

  // record a probe for h on s and queue it (caller does NOT hold the lock and has already counted
  // it in probes); its sequence number, or 0 when the record failed (count undone)
  uint64_t record_probe(int64_t h, Stream s) {
    Event ev = take_event();
    const bool ok = ev != Event{} && b_.record(ev, s);
    std::lock_guard<std::mutex> lock(mu_);
    Entry& c = *comms_[h];
    if (!ok) {
      --c.probes;
      if (ev != Event{}) pool_.push_back(ev);
      return 0;
    }
    const uint64_t seq = ++seq_;
    pending_.push_back({ev, h, Clock::now() + std::chrono::milliseconds(c.timeout_ms), seq});
    ensure_thread_locked();
    cv_.notify_all();
    return seq;
  }

  void abort_comm(int64_t h) {
    Comm comm;
    int device;
    {
      std::lock_guard<std::mutex> lock(mu_);
      comm = comms_[h]->comm;
      device = comms_[h]->device;
    }
    b_.set_device(device);
    b_.comm_abort(comm);  // unblocks the communicator's kernels, frees its resources
    bool teardown;
    std::string why;
    {
      std::lock_guard<std::mutex> lock(mu_);
      Entry& c = *comms_[h];
      c.state.store(kAborted);
      c.probes = 0;
      c.untracked = 0;
      teardown = c.teardown;
      why = c.reason;
      // the aborted collectives' events complete once the stream drains; drop them unqueried
      for (auto it = pending_.begin(); it != pending_.end();) {
        if (it->handle == h) {
          b_.destroy_event(it->ev);
          it = pending_.erase(it);
        } else {
          ++it;
        }
      }
      cv_.notify_all();
    }
    if (teardown)
      b_.teardown("[torcheval_amd] rccl_direct: communicator " + std::to_string(h) + " failed (" + why +
                  "); aborted it and tearing the process down (set TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING=0 to "
                  "raise on the next sync instead)");
  }

  void loop() {
    auto last_async_poll = Clock::now();
    struct Probe {
      uint64_t seq;
      Event ev;
      int64_t handle;
      Clock::time_point deadline;
      int q;
    };
    std::vector<Probe> batch;
    std::vector<std::pair<int64_t, Stream>> follow_ups;
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      if (!abort_q_.empty()) {
        const int64_t h = abort_q_.back();
        abort_q_.pop_back();
        lk.unlock();
        abort_comm(h);
        lk.lock();
        continue;
      }
      if (pending_.empty()) {
        cv_.wait_for(lk, std::chrono::milliseconds(200));
        continue;
      }
      // query a snapshot of the oldest probes WITHOUT the lock
      batch.clear();
      for (const auto& p : pending_) {
        batch.push_back({p.seq, p.ev, p.handle, p.deadline, 0});
        if (batch.size() >= 64) break;
      }
      lk.unlock();
      for (auto& pr : batch) pr.q = b_.query(pr.ev);
      const auto now = Clock::now();
      lk.lock();
      follow_ups.clear();
      for (const auto& pr : batch) {
        auto it = pending_.begin();
        while (it != pending_.end() && it->seq != pr.seq) ++it;
        if (it == pending_.end()) continue;  // retired meanwhile (destroy / abort / waiter)
        Entry& c = *comms_[pr.handle];
        if (pr.q == 0) {
          pool_.push_back(it->ev);
          pending_.erase(it);
          --c.probes;
          if (c.state.load() == kOk && c.probes == 0 && c.untracked > 0 && c.has_last) {
            // collectives enqueued behind the retired probe: probe them now
            c.untracked = 0;
            ++c.probes;
            follow_ups.emplace_back(pr.handle, c.last_stream);
          }
          continue;
        }
        if (c.state.load() == kOk) {
          if (pr.q == 2) mark_failed_locked(pr.handle, "completion query failed", false);
          else if (now > pr.deadline)
            mark_failed_locked(pr.handle, "a collective did not complete within " + std::to_string(c.timeout_ms) + " ms",
                               false);
        }
      }
      if (!follow_ups.empty()) {
        lk.unlock();
        for (const auto& fu : follow_ups) {
          int dev = 0;
          {
            std::lock_guard<std::mutex> lock(mu_);
            dev = comms_[fu.first]->device;
          }
          b_.set_device(dev);
          // never insert into a stream that is being captured into a graph
          const bool capturing = b_.capturing(fu.second);
          const bool ok = !capturing && record_probe(fu.first, fu.second) != 0;  // a failed record undoes its count
          if (!ok) {
            std::lock_guard<std::mutex> lock(mu_);
            Entry& c = *comms_[fu.first];
            if (capturing) --c.probes;
            ++c.untracked;  // probed at the next sync of this communicator
          }
        }
        lk.lock();
      }
      if (now - last_async_poll > std::chrono::milliseconds(10)) {
        last_async_poll = now;
        std::vector<std::pair<int64_t, Comm>> live;
        for (const auto& p : pending_) {
          Entry& c = *comms_[p.handle];
          if (c.state.load() == kOk) live.emplace_back(p.handle, c.comm);
        }
        lk.unlock();
        std::vector<std::pair<int64_t, std::string>> errors;
        for (const auto& l : live) {
          std::string why;
          if (b_.async_error(l.second, &why)) errors.emplace_back(l.first, why);
        }
        lk.lock();
        for (const auto& e : errors) mark_failed_locked(e.first, "async error: " + e.second, false);
      }
      cv_.wait_for(lk, std::chrono::microseconds(500));
    }
  }

  B& b_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<std::unique_ptr<Entry>> comms_;  // handle = index
  std::deque<Pending> pending_;
  std::vector<Event> pool_;
  std::vector<int64_t> abort_q_;
  uint64_t seq_ = 0;
  std::thread* thread_ = nullptr;  // joined by shutdown
  bool stop_ = false;
};

}  // namespace tea_wd
