// Engine-owned registry of the pinned host memory the engine DMAs from or to.
//
// The host paths (hdfs_crc32c_{compute,verify}_host, verify_crcdata beyond
// the staging buffer, host packet streams) copy straight from the caller's
// buffers, which must be page-locked for the duration of the call.  Round 2
// decided "pinned already?" by asking the HIP runtime about the caller's
// address (hipPointerGetAttributes) and registered the rest, dropping the
// result of hipHostUnregister.  Two hazards follow from that: a stale or
// failed unregistration makes a later, unrelated buffer at a reused address
// look pinned (and be DMA-ed from dead pages), and two registrations of
// buffers that share a page overlap.  This registry replaces both:
//
//  * the engine's own hipHostMalloc blocks (hdfs_crc32c_host_alloc, session
//    slots) are recorded as OWNED ranges;
//  * every other range a call needs is pinned by the call itself, over the
//    caller's EXACT bytes: the buffers of one call that share a page (data
//    and CRCs side by side) are merged into ONE registration spanning them
//    -- the runtime DMAs a copy only from inside a single registration, so a
//    CRC array that began in the data's registration and ran on into a
//    second one was refused ("invalid argument") -- and a range that lies
//    inside a registration another call holds shares it (reference counted).
//    The merged registration also spans the gap bytes between the merged
//    buffers (less than a page, not the caller's): an object in
//    the gap is used in place when it fits inside the registration, and one
//    that runs on past its end is refused as a partial overlap -- an error
//    with a message, never a DMA across the end (self-test case 2);
//    Registrations are NOT widened to whole pages: the runtime looks a
//    pointer up by the registered byte range, so a page-rounded registration
//    would capture unrelated heap objects on the same pages (the engine's
//    own pageable staging vectors among them), whose copies then ran past
//    the registration's end and were refused;
//  * a scope releases its pins when the call ends -- after draining the
//    streams that may still read or write them -- and the LAST reference
//    unregisters, with the result checked and reported;
//  * a range that only partly overlaps the bytes of another call's
//    registration cannot be one registration: the call is refused (no DMA
//    straddles two); ranges of different calls that merely share a page are
//    registered separately;
//  * memory pinned by someone else (a torch pinned tensor) is detected by the
//    runtime refusing the registration (already registered) and confirmed at
//    both ends of the caller's bytes; it is used in place, never unregistered.
//
// Header-only and templated on nothing: the HIP calls go through a backend
// interface, so tests/consumer/hostpin_selftest.cpp runs the bookkeeping on
// the CPU with a fake backend (reused addresses, overlaps, failures).
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <initializer_list>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

namespace hdfs_crc32c {

struct PinBackend {
  enum { kOk = 0, kAlready = 1, kFail = -1 };
  virtual ~PinBackend() = default;
  // exact byte range; kOk, kAlready (the runtime has it pinned), kFail
  virtual int reg(uintptr_t p, size_t n) = 0;
  virtual int unreg(uintptr_t p) = 0;  // kOk / kFail
  // the runtime reports byte p as page-locked host memory (someone else's)
  virtual bool pinned_elsewhere(uintptr_t p) = 0;
};

class PinRegistry {
 public:
  struct Entry {
    uintptr_t end;
    uint32_t refs;
    bool owned;
  };

  explicit PinRegistry(PinBackend *b, size_t page = 4096) : be_(b), page_(page) {}
  void set_backend(PinBackend *b) { be_ = b; }

  // An engine allocation (hipHostMalloc'd).
  void add_owned(const void *p, size_t n) {
    if (!p || !n) return;
    std::lock_guard<std::mutex> lk(mu_);
    map_[uintptr_t(p)] = Entry{uintptr_t(p) + n, 0u, true};
  }
  bool remove_owned(const void *p) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = map_.find(uintptr_t(p));
    if (it == map_.end() || !it->second.owned) return false;
    map_.erase(it);
    return true;
  }

  // Pins held by one call.  acquire() every buffer the call DMAs, then
  // release(drain) once its GPU work is done; the destructor releases what an
  // early return left (its result is then only in last_error()).
  class Scope {
   public:
    explicit Scope(PinRegistry &r) : r_(r) {}
    Scope(const Scope &) = delete;
    Scope &operator=(const Scope &) = delete;
    ~Scope() { (void)release(); }
    // Every host buffer one call DMAs, at once: 0, or -1 with last_error()
    // set (registration refused / partly pinned elsewhere).
    int acquire(std::initializer_list<std::pair<const void *, size_t>> bufs) {
      std::vector<std::pair<uintptr_t, size_t>> v;
      for (auto &b : bufs)
        if (b.first && b.second) v.emplace_back(uintptr_t(b.first), b.second);
      return r_.acquire(v, held_);
    }
    int acquire(const void *p, size_t n) { return acquire({{p, n}}); }
    // Unpin: 0, or -1 if an unregistration failed (every pin is released
    // regardless).  The caller drains its streams first.
    int release() {
      const int rc = r_.release(held_);
      held_.clear();
      return rc;
    }
    size_t held() const { return held_.size(); }

   private:
    PinRegistry &r_;
    std::vector<uintptr_t> held_;  // starts of referenced registered entries
  };

  const char *last_error() const { return err_; }
  // Introspection for the self-test: (start, end, refs, owned) of every entry.
  std::vector<std::pair<uintptr_t, Entry>> entries() {
    std::lock_guard<std::mutex> lk(mu_);
    return std::vector<std::pair<uintptr_t, Entry>>(map_.begin(), map_.end());
  }

 private:
  uintptr_t down(uintptr_t x) const { return x & ~uintptr_t(page_ - 1); }
  uintptr_t up(uintptr_t x) const { return (x + page_ - 1) & ~uintptr_t(page_ - 1); }

  int acquire(std::vector<std::pair<uintptr_t, size_t>> bufs, std::vector<uintptr_t> &held) {
    if (bufs.empty()) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    // byte ranges of the buffers, merged where they share a page
    std::sort(bufs.begin(), bufs.end());
    struct Need {
      uintptr_t s, e;
      std::vector<std::pair<uintptr_t, size_t>> parts;  // the caller's bytes inside
    };
    std::vector<Need> need;
    for (auto &b : bufs) {
      const uintptr_t s = b.first, e = b.first + b.second;
      if (!need.empty() && down(s) < up(need.back().e)) {
        need.back().e = e > need.back().e ? e : need.back().e;
        need.back().parts.push_back(b);
      } else {
        need.push_back(Need{s, e, {b}});
      }
    }
    std::vector<uintptr_t> took;  // refs taken here (undone on failure)
    auto undo = [&]() {
      for (uintptr_t k : took) drop(k);
    };
    for (const Need &nd : need) {
      // entries whose bytes overlap [nd.s, nd.e)
      auto it = map_.upper_bound(nd.s);
      if (it != map_.begin() && std::prev(it)->second.end > nd.s) --it;
      const bool any = it != map_.end() && it->first < nd.e;
      if (any && it->first <= nd.s && it->second.end >= nd.e) {  // inside one entry: share it
        if (!it->second.owned) {
          it->second.refs++;
          took.push_back(it->first);
        }
        continue;
      }
      if (any) {
        undo();
        snprintf_err("host range %#lx+%lu partly overlaps pinned memory of another call or allocation", nd.s,
                     nd.e - nd.s);
        return -1;
      }
      const int r = be_->reg(nd.s, nd.e - nd.s);
      if (r == PinBackend::kOk) {
        map_.emplace(nd.s, Entry{nd.e, 1u, false});
        took.push_back(nd.s);
        continue;
      }
      bool elsewhere = r == PinBackend::kAlready;  // pinned by its owner: used in place
      for (auto &b : nd.parts)
        elsewhere = elsewhere && be_->pinned_elsewhere(b.first) && be_->pinned_elsewhere(b.first + b.second - 1);
      if (elsewhere) continue;
      undo();
      snprintf_err(r == PinBackend::kAlready ? "host range %#lx+%lu is partly pinned by another allocator"
                                             : "host registration of %#lx+%lu failed",
                   nd.s, nd.e - nd.s);
      return -1;
    }
    held.insert(held.end(), took.begin(), took.end());
    return 0;
  }

  // One reference less on the entry starting at k (caller holds mu_); the
  // last one unregisters.  Returns the backend's result.
  int drop(uintptr_t k) {
    auto it = map_.find(k);
    if (it == map_.end() || it->second.owned || it->second.refs == 0) return PinBackend::kFail;
    if (--it->second.refs) return PinBackend::kOk;
    const int r = be_->unreg(k);
    map_.erase(it);  // even on failure: the range is not ours to trust any more
    return r;
  }

  int release(const std::vector<uintptr_t> &held) {
    if (held.empty()) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    int rc = 0;
    for (uintptr_t k : held)
      if (drop(k) != PinBackend::kOk && rc == 0) {
        snprintf_err("host unregistration of %#lx failed", k, size_t(0));
        rc = -1;
      }
    return rc;
  }

  void snprintf_err(const char *fmt, uintptr_t a, size_t b) {
    std::snprintf(err_, sizeof(err_), fmt, static_cast<unsigned long>(a), static_cast<unsigned long>(b));
  }

  PinBackend *be_;
  size_t page_;
  std::mutex mu_;
  std::map<uintptr_t, Entry> map_;
  // per thread: a call reads the message its own acquire / release wrote
  // (a registry-wide buffer read after mu_ was dropped could carry another
  // thread's message, or a torn one -- ADVICE r3)
  static inline thread_local char err_[160] = "";
};

}  // namespace hdfs_crc32c
