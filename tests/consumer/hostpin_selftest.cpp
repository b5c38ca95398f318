// CPU self-test of the engine's pinned-memory registry
// (hadoofus_amd/csrc/crc32c_hostpin.h) with a fake runtime backend that
// models the HIP runtime's view of registrations: byte ranges registered,
// refused, failing to unregister.  Scenarios are the ones round 2's
// illegal-address fault pointed at: buffers freed and re-allocated at the
// same address (mmap reuse) between calls, buffers that share a page,
// nested and concurrent needs of one range, early returns, a failed
// unregistration, memory pinned by someone else.  Prints "N failures".
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <set>
#include <thread>
#include <vector>

#include "crc32c_hostpin.h"

using hdfs_crc32c::PinBackend;
using hdfs_crc32c::PinRegistry;

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      g_fail++;                                                    \
    }                                                              \
  } while (0)

// The runtime as the engine sees it: a set of registered byte ranges (a
// registration must not overlap another's bytes; ranges may share a page),
// plus ranges pinned by "another allocator" (hipHostMalloc'd by someone else).
struct FakeRuntime final : PinBackend {
  std::set<std::pair<uintptr_t, uintptr_t>> regs, foreign;
  int nreg = 0, nunreg = 0, fail_unreg = 0, fail_reg = 0;
  static bool overlaps(const std::set<std::pair<uintptr_t, uintptr_t>> &s, uintptr_t a, uintptr_t b) {
    for (auto &r : s)
      if (r.first < b && a < r.second) return true;
    return false;
  }
  int reg(uintptr_t p, size_t n) override {
    if (fail_reg) return kFail;
    if (overlaps(regs, p, p + n) || overlaps(foreign, p, p + n)) return pinned_elsewhere(p) ? kAlready : kFail;
    regs.insert({p, p + n});
    nreg++;
    return kOk;
  }
  int unreg(uintptr_t p) override {
    nunreg++;
    for (auto it = regs.begin(); it != regs.end(); ++it)
      if (it->first == p) {
        if (fail_unreg) return kFail;  // stays registered in the runtime
        regs.erase(it);
        return kOk;
      }
    return kFail;
  }
  bool pinned_elsewhere(uintptr_t p) override {
    for (auto &r : foreign)
      if (r.first <= p && p < r.second) return true;
    return false;
  }
  // the runtime DMAs a copy only from inside ONE registration
  bool dma_ok(uintptr_t p, size_t n) const {
    for (auto &r : regs)
      if (r.first <= p && p + n <= r.second) return true;
    for (auto &r : foreign)
      if (r.first <= p && p + n <= r.second) return true;
    return false;
  }
  bool in_reg(uintptr_t p) const {  // the runtime would treat byte p as registered
    for (auto &r : regs)
      if (r.first <= p && p < r.second) return true;
    return false;
  }
  bool pinned(uintptr_t p, size_t n) const {  // every byte in a registration
    for (uintptr_t a = p; a < p + n;) {
      bool hit = false;
      for (auto &r : regs)
        if (r.first <= a && a < r.second) {
          a = r.second;
          hit = true;
          break;
        }
      if (!hit) return false;
    }
    return true;
  }
};

int main() {
  const size_t page = size_t(sysconf(_SC_PAGESIZE));
  CHECK(page == 4096);
  FakeRuntime rt;
  PinRegistry reg(&rt, page);

  // 1. a call pins, the call ends, the range is unregistered; the buffer is
  //    freed and a NEW buffer mapped at the same address is pinned afresh
  //    (nothing from the old registration is trusted)
  {
    const size_t n = 46 << 20;
    void *a = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    CHECK(a != MAP_FAILED);
    {
      PinRegistry::Scope s(reg);
      CHECK(s.acquire(static_cast<uint8_t *>(a) + 32, n - 32) == 0);
      CHECK(rt.pinned(uintptr_t(a) + 32, n - 32));
      CHECK(s.release() == 0);
    }
    CHECK(rt.regs.empty() && reg.entries().empty());
    munmap(a, n);
    void *b = mmap(a, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);  // hint: same address
    CHECK(b != MAP_FAILED);
    const int before = rt.nreg;
    {
      PinRegistry::Scope s(reg);
      CHECK(s.acquire(static_cast<uint8_t *>(b) + 32, n - 32) == 0);
      CHECK(rt.nreg == before + 1);  // registered again, not found "already pinned"
      CHECK(rt.pinned(uintptr_t(b) + 32, n - 32));
    }  // early return: the destructor unpins
    CHECK(rt.regs.empty() && reg.entries().empty());
    munmap(b, n);
  }

  // 2. data, CRCs and bitmap of one call share pages (adjacent small
  //    arrays, the CRCs at an odd address): ONE registration over all three,
  //    so each buffer's DMA lies inside a single registration (round 3: the
  //    CRC array began in the data's registration and ran into a second
  //    one; the runtime refused the copy)
  {
    alignas(4096) static uint8_t buf[4 * 4096];
    PinRegistry::Scope s(reg);
    CHECK(s.acquire({{buf + 100, 6000}, {buf + 6103, 4000}, {buf + 10103, 375}}) == 0);
    CHECK(rt.regs.size() == 1);
    CHECK(rt.dma_ok(uintptr_t(buf) + 100, 6000) && rt.dma_ok(uintptr_t(buf) + 6103, 4000) &&
          rt.dma_ok(uintptr_t(buf) + 10103, 375));
    auto e = reg.entries();
    CHECK(e.size() == 1 && e[0].second.refs == 1);
    // the pages' other bytes (a heap neighbour: the engine's own pageable
    // staging vector) stay outside every registration -- a copy from there
    // must not be taken for a registered one that runs past its end
    CHECK(!rt.in_reg(uintptr_t(buf) + 99) && !rt.in_reg(uintptr_t(buf) + 10478) && !rt.in_reg(uintptr_t(buf)));
    // the gap between two merged buffers (bytes 6100..6102, not the
    // caller's) IS inside the registration: an object there is
    // used in place when it fits inside (one reference more, nothing
    // registered), and one that runs on past the registration's end is
    // refused with a message -- never DMA-ed across the end
    CHECK(rt.in_reg(uintptr_t(buf) + 6100) && rt.in_reg(uintptr_t(buf) + 6102));
    {
      PinRegistry::Scope g(reg);
      const int nreg0 = rt.nreg;
      CHECK(g.acquire(buf + 6100, 3) == 0);
      CHECK(rt.nreg == nreg0 && reg.entries()[0].second.refs == 2);
      PinRegistry::Scope h(reg);
      CHECK(h.acquire(buf + 6100, 5000) != 0);
      CHECK(std::strstr(reg.last_error(), "partly overlaps") != nullptr);
      CHECK(h.held() == 0 && rt.nreg == nreg0);
    }
    CHECK(reg.entries().size() == 1 && reg.entries()[0].second.refs == 1);
    CHECK(s.release() == 0);
    CHECK(rt.regs.empty() && reg.entries().empty());
    // buffers on separate pages of one call: separate registrations
    PinRegistry::Scope t(reg);
    CHECK(t.acquire({{buf, 4096}, {buf + 2 * 4096, 10}}) == 0);
    CHECK(rt.regs.size() == 2);
  }
  CHECK(rt.regs.empty() && reg.entries().empty());

  // 3. nested needs (verify_crcdata pins the region, host_pipeline its parts)
  //    and a second concurrent scope on an overlapping range
  {
    alignas(4096) static uint8_t buf[16 * 4096];
    PinRegistry::Scope outer(reg);
    CHECK(outer.acquire(buf, sizeof(buf)) == 0);
    const int nreg0 = rt.nreg, nun0 = rt.nunreg;
    {
      PinRegistry::Scope inner(reg);
      CHECK(inner.acquire(buf + 5000, 20000) == 0);
      CHECK(inner.acquire(buf + 100, 50) == 0);
      CHECK(rt.nreg == nreg0);  // covered: no new registration
    }
    CHECK(rt.regs.size() == 1 && rt.nunreg == nun0);  // the inner scope did not unregister the outer's pages
    PinRegistry::Scope other(reg);
    CHECK(other.acquire(buf + 15 * 4096 + 10, 3 * 4096) != 0);  // runs past the outer range: refused
    CHECK(std::strstr(reg.last_error(), "partly overlaps") != nullptr);
    CHECK(rt.regs.size() == 1 && reg.entries().size() == 1 && reg.entries()[0].second.refs == 1);
    CHECK(other.acquire(buf + 3 * 4096, 4096) == 0);  // inside it: shared
    CHECK(outer.release() == 0);
    // the other scope's reference keeps the registration (a range is
    // unregistered whole, by its last user)
    CHECK(rt.regs.size() == 1 && rt.dma_ok(uintptr_t(buf) + 3 * 4096, 4096));
    CHECK(other.release() == 0);
    CHECK(rt.regs.empty() && reg.entries().empty());
  }

  // 4. engine allocations (hdfs_crc32c_host_alloc) are used in place, never
  //    registered or unregistered by a call; after host_free a pageable buffer
  //    at that address is registered normally
  {
    alignas(4096) static uint8_t blk[8 * 4096];
    reg.add_owned(blk, sizeof(blk));
    const int nreg0 = rt.nreg, nun0 = rt.nunreg;
    {
      PinRegistry::Scope s(reg);
      CHECK(s.acquire(blk + 77, 5 * 4096) == 0);
      CHECK(s.held() == 0);
    }
    CHECK(rt.nreg == nreg0 && rt.nunreg == nun0);
    CHECK(reg.remove_owned(blk));
    CHECK(!reg.remove_owned(blk));
    PinRegistry::Scope s(reg);
    CHECK(s.acquire(blk + 77, 5 * 4096) == 0);
    CHECK(rt.nreg == nreg0 + 1);
  }
  CHECK(rt.regs.empty() && reg.entries().empty());

  // 5. memory another allocator pinned (a torch pinned tensor): the runtime
  //    refuses the registration, both ends are pinned elsewhere -> used in
  //    place, never unregistered; a range only PARTLY pinned elsewhere is an
  //    error and leaves nothing behind
  {
    alignas(4096) static uint8_t buf[10 * 4096];
    rt.foreign.insert({uintptr_t(buf), uintptr_t(buf) + 4 * 4096});
    {
      PinRegistry::Scope s(reg);
      CHECK(s.acquire(buf + 10, 3 * 4096) == 0);
      CHECK(s.held() == 0 && rt.regs.empty());
    }
    {
      PinRegistry::Scope s(reg);
      CHECK(s.acquire(buf + 10, 6 * 4096) != 0);  // pages 4..6 are not pinned by anyone
      CHECK(std::strstr(reg.last_error(), "another allocator") != nullptr);
      CHECK(rt.regs.empty() && reg.entries().empty());
    }
    rt.foreign.clear();
  }

  // 6. a failed unregistration is reported (not swallowed), and the registry
  //    forgets the range: a later call registers again instead of trusting it
  {
    alignas(4096) static uint8_t buf[4 * 4096];
    PinRegistry::Scope s(reg);
    CHECK(s.acquire(buf, sizeof(buf)) == 0);
    rt.fail_unreg = 1;
    CHECK(s.release() != 0);
    CHECK(std::strstr(reg.last_error(), "unregistration") != nullptr);
    CHECK(reg.entries().empty());
    rt.fail_unreg = 0;
    rt.regs.clear();  // (the runtime's leftover; the engine reported it)
  }

  // 7. a failed registration undoes the pins the same acquire took
  {
    alignas(4096) static uint8_t buf[8 * 4096];
    PinRegistry::Scope a(reg);
    CHECK(a.acquire(buf + 6 * 4096, 4096) == 0);  // page 6 pinned by another call
    PinRegistry::Scope s(reg);
    rt.fail_reg = 1;
    // page 6 shared (ref taken), pages 0-1 then fail: the ref is given back
    CHECK(s.acquire({{buf + 6 * 4096 + 8, 100}, {buf, 2 * 4096}}) != 0);
    rt.fail_reg = 0;
    auto e = reg.entries();
    CHECK(e.size() == 1 && e[0].second.refs == 1);
    CHECK(a.release() == 0);
    CHECK(rt.regs.empty() && reg.entries().empty());
  }

  // 8b. two calls whose buffers share a page but no byte: separate
  //     registrations, each DMA inside its own, released independently
  {
    alignas(4096) static uint8_t buf[4 * 4096];
    PinRegistry::Scope a(reg), b(reg);
    CHECK(a.acquire(buf + 16, 5000) == 0);
    CHECK(b.acquire(buf + 5016, 7000) == 0);
    CHECK(rt.regs.size() == 2 && rt.dma_ok(uintptr_t(buf) + 16, 5000) && rt.dma_ok(uintptr_t(buf) + 5016, 7000));
    CHECK(a.release() == 0);
    CHECK(rt.regs.size() == 1 && rt.dma_ok(uintptr_t(buf) + 5016, 7000));
    CHECK(b.release() == 0);
    CHECK(rt.regs.empty() && reg.entries().empty());
  }

  // 8. many threads pinning ranges of one buffer: the whole buffer, or a
  //    part of it inside whatever registration is live, or a disjoint slice
  {
    static uint8_t big[64 * 4096] __attribute__((aligned(4096)));
    std::vector<std::thread> th;
    std::atomic<int> refused{0};
    for (int t = 0; t < 8; t++)
      th.emplace_back([&, t] {
        for (int k = 0; k < 200; k++) {
          PinRegistry::Scope s(reg);
          const size_t off = size_t((t * 7919 + k * 104729) % (60 * 4096));
          const int rc = (k % 3 == 0) ? s.acquire(big, sizeof(big)) : s.acquire(big + off, 3 * 4096 + 5);
          if (rc) refused++;  // a partial overlap of another thread's live pin: refused, never corrupted
          for (auto &r : reg.entries())
            if (r.second.refs == 0 && !r.second.owned) g_fail++;
        }
      });
    for (auto &x : th) x.join();
    CHECK(rt.regs.empty() && reg.entries().empty());
    std::printf("concurrent: %d of 1600 acquires refused (partial overlaps)\n", refused.load());
  }

  std::printf("%d failures\n", g_fail);
  return g_fail ? 1 : 0;
}
