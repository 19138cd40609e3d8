// Thread test of the pinned-slot pool (csrc/xfer_pool.h), host only: the
// library's claim/release code over a fake event backend, run by several
// threads at once under ThreadSanitizer (make check-xfer; tests/test_asan_host.py).
//
// Model: each thread is one stream.  A copy claims a slot, (if told to) waits
// on the slot's previous event, "copies" (writes a thread tag into the slot
// and reads it back), and releases; an H2D-style copy leaves its event
// pending, completed later by a device thread (out of order across streams,
// in order within one).  Checked: a slot is never held by two threads, a
// thread is only ever told to wait on an event of its own stream, a pending
// event never completes before its copy was released, no copy deadlocks
// (every thread finishes within a deadline), and the pool is used (claims
// succeed) without ever calling a blocking query under the lock.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "xfer_pool.h"

namespace {

struct FakeEvent {
    std::atomic<int> done{1};
    int stream = -1;
};

struct FakeBackend {
    using Event = FakeEvent *;
    using Stream = int;
    std::atomic<int> *allocs;
    template <typename S>
    bool alloc(S &s)
    {
        s.h = static_cast<char *>(std::malloc(64));
        s.ev = new FakeEvent;
        allocs->fetch_add(1);
        return s.h != nullptr;
    }
    bool done(FakeEvent *e) { return e->done.load(std::memory_order_acquire) != 0; }
};

using Pool = tspgpu::XferPool<FakeBackend, 4>;

std::atomic<int> g_fail{0};
void fail(const char *what)
{
    if (g_fail.fetch_add(1) < 10) std::fprintf(stderr, "check_xfer: FAIL %s\n", what);
}

// the "device": completes pending events, in order per stream
struct Device {
    std::mutex mu;
    std::vector<std::deque<FakeEvent *>> q;
    explicit Device(int streams) : q(streams) {}
    void enqueue(int st, FakeEvent *e)
    {
        std::lock_guard<std::mutex> g(mu);
        q[st].push_back(e);
    }
    bool step(std::mt19937 &rng)
    {
        std::lock_guard<std::mutex> g(mu);
        bool any = false;
        for (auto &d : q) any |= !d.empty();
        if (!any) return false;
        for (;;) {
            auto &d = q[rng() % q.size()];
            if (d.empty()) continue;
            d.front()->done.store(1, std::memory_order_release);
            d.pop_front();
            return true;
        }
    }
    void wait_for(FakeEvent *e)  // a stream's own event: its queue drains in order
    {
        while (!e->done.load(std::memory_order_acquire)) std::this_thread::yield();
    }
};

}  // namespace

int main()
{
    constexpr int kThreads = 8, kIters = 4000;
    std::atomic<int> allocs{0};
    Pool pool(FakeBackend{&allocs});
    Device dev(kThreads);
    std::atomic<int> holders[4] = {};
    std::atomic<long> claimed{0}, fallback{0}, waited{0};
    std::atomic<bool> stop{false};

    std::thread device([&] {
        std::mt19937 rng(7);
        while (!stop.load()) {
            if (!dev.step(rng)) std::this_thread::yield();
        }
        while (dev.step(rng)) {
        }
    });
    std::vector<std::thread> th;
    for (int t = 0; t < kThreads; ++t)
        th.emplace_back([&, t] {
            std::mt19937 rng(100 + t);
            for (int it = 0; it < kIters; ++it) {
                bool wait = false;
                Pool::Slot *s = pool.claim(t, &wait);
                if (!s) {
                    fallback.fetch_add(1);
                    continue;
                }
                claimed.fetch_add(1);
                // identify the slot by its event object
                int sid = -1;
                static FakeEvent *ids[4] = {};
                static std::mutex idmu;
                {
                    std::lock_guard<std::mutex> g(idmu);
                    for (int k = 0; k < 4 && sid < 0; ++k) {
                        if (ids[k] == s->ev) sid = k;
                        else if (!ids[k]) ids[sid = k] = s->ev;
                    }
                }
                if (sid < 0) fail("more slots than the pool holds");
                if (sid >= 0 && holders[sid].fetch_add(1) != 0) fail("a slot held by two threads");
                if (wait) {
                    waited.fetch_add(1);
                    if (s->ev->stream != t) fail("told to wait on another stream's event");
                    dev.wait_for(s->ev);
                } else if (!s->ev->done.load()) {
                    fail("a slot handed out with its last copy still running");
                }
                std::memset(s->h, t, 64);
                for (int b = 0; b < 64; ++b)
                    if (s->h[b] != (char)t) fail("slot bytes changed under the owner");
                const bool h2d = rng() & 1;
                if (sid >= 0) holders[sid].fetch_sub(1);
                if (h2d) {
                    s->ev->stream = t;
                    s->ev->done.store(0, std::memory_order_release);
                    pool.release(s, t, true);
                    dev.enqueue(t, s->ev);
                } else {
                    pool.release(s, t, false);
                }
            }
        });
    const auto t0 = std::chrono::steady_clock::now();
    for (auto &x : th) x.join();
    stop.store(true);
    device.join();
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (sec > 120) fail("too slow (a copy blocked?)");
    if (claimed.load() == 0) fail("no copy used the pool");
    if (allocs.load() > 4) fail("more allocations than slots");
    std::printf("check_xfer: %s (claims %ld, runtime-path fallbacks %ld, own-stream waits %ld, %d threads, %.2f s)\n",
                g_fail.load() ? "FAILED" : "ok", claimed.load(), fallback.load(), waited.load(), kThreads, sec);
    return g_fail.load() ? 1 : 0;
}
