// C ABI (include/kvgpu.h) + device runtime: HBM residency of compiled policy
// sets and ingested batches, launch-time folding of batch-constant user info,
// result decoding (failing paths) on the host.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <emmintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <stdexcept>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kvgpu.h"
#include "kvdev.h"
#include "kvinternal.hpp"
#include "kvjit.hpp"

using namespace kv;
using namespace kvh;

namespace {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) throw HipError(std::string(#x) + ": " + hipGetErrorString(e_));      \
  } while (0)

bool pinned_src(const void* src, size_t bytes);  // page-locked store array (PinnedStore)

// HIP streams cost milliseconds to create and to destroy on this runtime (hipStreamCreate* 2.3-3.8
// ms, hipStreamDestroy 1.8-2.6 ms per call in the rocprofv3 HIP API trace of a C2 kv_validate: 15 of
// its 44 ms), so sessions and staged uploads take idle streams from a per-(device, flags) pool and
// give them back instead. The pool also knows every stream it ever created per device (`all`): a
// released device buffer becomes reusable once an event recorded on each of them has completed
// (DevPool below).
struct StreamPool {
  std::mutex mu;
  std::map<std::tuple<int, unsigned, int>, std::vector<hipStream_t>> free;
  std::map<int, std::vector<hipStream_t>> all;
  static StreamPool& get() {
    static StreamPool* p = new StreamPool();  // never destroyed (streams die with the process)
    return *p;
  }
  std::vector<hipStream_t> streams_of(int dev) {
    std::lock_guard<std::mutex> g(mu);
    return all[dev];
  }
  // a stream of the current device `dev`; low: the lowest scheduling priority (its workgroups are
  // dispatched when the other queues' kernels leave slots free)
  hipStream_t take(int dev, unsigned flags, bool low = false) {
    const int prio = low ? lowest() : 0;
    {
      std::lock_guard<std::mutex> g(mu);
      auto& v = free[{dev, flags, prio}];
      if (!v.empty()) {
        hipStream_t s = v.back();
        v.pop_back();
        return s;
      }
    }
    hipStream_t s = nullptr;
    if (low) HIPCHK(hipStreamCreateWithPriority(&s, flags, prio));
    else HIPCHK(hipStreamCreateWithFlags(&s, flags));
    std::lock_guard<std::mutex> g(mu);
    all[dev].push_back(s);
    return s;
  }
  void give(int dev, unsigned flags, hipStream_t s, bool low = false) {
    if (!s) return;
    (void)hipStreamSynchronize(s);
    const int prio = low ? lowest() : 0;
    std::lock_guard<std::mutex> g(mu);
    free[{dev, flags, prio}].push_back(s);
  }
  static int lowest() {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return least;
  }
};

// Device allocations are expensive to create and to free (hipMalloc maps pages, hipFree also
// waits for the device), and a host that validates batch after batch allocates the same store,
// column and result buffers for every batch. Released buffers are therefore kept per device and
// handed to the next allocation of a similar size. A released block is reusable once the work
// queued before its release has finished (hipFree's own guarantee, without blocking the releasing
// thread or any other session on the device): give() records an event on every stream the library
// created on the device and on the null stream, and take() hands the block out only when all of
// them have completed. At most kv_device_pool_limit() bytes are kept (default 32 GiB of the 288 GiB
// HBM); when a hipMalloc fails the device's kept buffers are freed and the allocation retried, and
// kv_device_trim() returns them to the device for co-resident allocators (e.g. torch).
// KVGPU_DEVPOOL=0: plain hipMalloc / hipFree.
struct DevPool {
  struct Pending {
    void* p;
    size_t cap;
    std::vector<hipEvent_t> ev;
  };
  std::mutex mu;
  std::map<int, std::multimap<size_t, void*>> free;  // device -> capacity -> block
  std::map<int, std::vector<Pending>> pending;        // released, maybe still in use by queued work
  std::map<int, size_t> held;                         // free + pending bytes
  std::map<int, std::vector<hipEvent_t>> evs;         // idle events per device
  size_t hold = 32ull << 30;
  static DevPool& get() {
    static DevPool* p = new DevPool();  // never destroyed: buffers may be released during static teardown
    return *p;
  }
  static bool enabled() {
    static const bool on = !(getenv("KVGPU_DEVPOOL") && getenv("KVGPU_DEVPOOL")[0] == '0');
    return on;
  }
  // (mu held) pending blocks whose events have all completed move to the free list
  void settle(int dev) {
    auto& pv = pending[dev];
    for (size_t i = 0; i < pv.size();) {
      bool done = true;
      for (hipEvent_t e : pv[i].ev) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipErrorNotReady) {
          done = false;
          break;
        }
        if (q != hipSuccess) (void)hipGetLastError();
      }
      if (!done) {
        i++;
        continue;
      }
      for (hipEvent_t e : pv[i].ev) evs[dev].push_back(e);
      free[dev].emplace(pv[i].cap, pv[i].p);
      pv[i] = std::move(pv.back());
      pv.pop_back();
    }
  }
  // a block of at least `bytes` on the current device `dev` (its capacity in *cap)
  void* take(int dev, size_t bytes, size_t* cap) {
    if (enabled()) {
      std::lock_guard<std::mutex> g(mu);
      settle(dev);
      auto& f = free[dev];
      auto it = f.lower_bound(bytes);
      if (it != f.end() && it->first <= bytes + bytes / 4 + (2u << 20)) {
        void* p = it->second;
        *cap = it->first;
        held[dev] -= it->first;
        f.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      trim(dev);
      HIPCHK(hipMalloc(&p, bytes));
    }
    *cap = bytes;
    return p;
  }
  // `dev` is the current device
  void give(int dev, void* p, size_t cap) {
    if (enabled()) {
      std::vector<hipStream_t> st = StreamPool::get().streams_of(dev);
      st.push_back(nullptr);  // (the null stream: synchronous copies, RCCL setup)
      std::lock_guard<std::mutex> g(mu);
      if (held[dev] + cap <= hold) {
        Pending pe{p, cap, {}};
        bool ok = true;
        for (hipStream_t s : st) {
          hipEvent_t e = nullptr;
          auto& idle = evs[dev];
          if (!idle.empty()) {
            e = idle.back();
            idle.pop_back();
          } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            ok = false;
            break;
          }
          pe.ev.push_back(e);
          if (hipEventRecord(e, s) != hipSuccess) {
            (void)hipGetLastError();
            ok = false;
            break;
          }
        }
        if (ok) {
          pending[dev].push_back(std::move(pe));
          held[dev] += cap;
          return;
        }
        for (hipEvent_t e : pe.ev) evs[dev].push_back(e);
      }
    }
    (void)hipDeviceSynchronize();  // (hipFree waits for the device anyway)
    (void)hipFree(p);
  }
  size_t held_on(int dev) {
    std::lock_guard<std::mutex> g(mu);
    return held[dev];
  }
  // free every kept block of `dev` (the current device): waits for the device first
  void trim(int dev) {
    std::multimap<size_t, void*> f;
    std::vector<Pending> pv;
    {
      std::lock_guard<std::mutex> g(mu);
      f.swap(free[dev]);
      pv.swap(pending[dev]);
      held[dev] = 0;
    }
    if (f.empty() && pv.empty()) return;
    (void)hipDeviceSynchronize();
    for (auto& [c, p] : f) (void)hipFree(p);
    std::lock_guard<std::mutex> g(mu);
    for (Pending& pe : pv) {
      (void)hipFree(pe.p);
      for (hipEvent_t e : pe.ev) evs[dev].push_back(e);
    }
  }
};

struct DevBuf {
  void* p = nullptr;
  size_t n = 0, cap = 0;
  int dev = -1;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  template <class T, class A>
  void upload(const std::vector<T, A>& v, int device) {
    upload_raw(v.data(), v.size() * sizeof(T), device);
  }
  void upload_raw(const void* src, size_t bytes, int device) {
    alloc(bytes, device);
    if (bytes) upload_h2d(p, src, bytes);
  }
  // a page-locked source is copied asynchronously on `st` (the caller synchronizes `st` before
  // the source may change or the buffer is read elsewhere); a pageable one as upload_raw
  template <class T, class A>
  void upload_async(const std::vector<T, A>& v, int device, hipStream_t st) {
    const size_t bytes = v.size() * sizeof(T);
    alloc(bytes, device);
    if (!bytes) return;
    if (pinned_src(v.data(), bytes))
      HIPCHK(hipMemcpyAsync(p, v.data(), bytes, hipMemcpyHostToDevice, st));
    else
      upload_h2d(p, v.data(), bytes);
  }
  // Host-to-device copy of a (pageable) host range. Large ranges go through a pinned staging
  // ring: host threads copy chunk i into a page-locked buffer while the DMA engine moves chunk
  // i-1 (32 MB chunks, 4 buffers, up to 16 copy threads).
  static void upload_h2d(void* dst, const void* src, size_t bytes) {
    constexpr size_t kChunk = 32u << 20;
    constexpr size_t kMin = 16u << 20;
    constexpr int kRing = 4;
    if (bytes < kMin || pinned_src(src, bytes)) {
      HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
      return;
    }
    static std::mutex mu;  // one staged upload at a time per process (the ring is shared)
    static char* ring[kRing] = {};
    std::lock_guard<std::mutex> g(mu);
    if (!ring[0]) {
      for (int i = 0; i < kRing; i++) {
        if (hipHostMalloc((void**)&ring[i], kChunk, hipHostMallocPortable) != hipSuccess) {
          (void)hipGetLastError();
          for (int j = 0; j < i; j++) (void)hipHostFree(ring[j]);
          ring[0] = nullptr;
          HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
          return;
        }
      }
    }
    int sdev = 0;
    HIPCHK(hipGetDevice(&sdev));
    hipStream_t st = StreamPool::get().take(sdev, hipStreamNonBlocking);
    hipEvent_t ev[kRing];
    for (int i = 0; i < kRing; i++) HIPCHK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    bool used[kRing] = {};
    static const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    size_t k = 0;
    for (size_t off = 0; off < bytes; off += kChunk, k++) {
      const int i = (int)(k % kRing);
      const size_t len = std::min(kChunk, bytes - off);
      if (used[i]) HIPCHK(hipEventSynchronize(ev[i]));  // the DMA out of this buffer is done
      const char* s = (const char*)src + off;
      std::vector<std::thread> th;
      const size_t part = (len + T - 1) / T;
      for (unsigned t = 0; t < T; t++) {
        const size_t a = std::min(len, t * part), e = std::min(len, a + part);
        if (a < e) th.emplace_back([=]() { memcpy(ring[i] + a, s + a, e - a); });
      }
      for (auto& x : th) x.join();
      HIPCHK(hipMemcpyAsync((char*)dst + off, ring[i], len, hipMemcpyHostToDevice, st));
      HIPCHK(hipEventRecord(ev[i], st));
      used[i] = true;
    }
    HIPCHK(hipStreamSynchronize(st));
    for (int i = 0; i < kRing; i++) (void)hipEventDestroy(ev[i]);
    StreamPool::get().give(sdev, hipStreamNonBlocking, st);
  }
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
    std::swap(dev, o.dev);
  }
  void alloc(size_t bytes, int device) {  // (a buffer allocated before is released first)
    release();
    dev = device;
    n = bytes;
    p = DevPool::get().take(device, std::max<size_t>(bytes, 16), &cap);
  }
  void release() {
    if (!p) return;
    int cur;
    if (hipGetDevice(&cur) == hipSuccess) {
      (void)hipSetDevice(dev);
      DevPool::get().give(dev, p, cap);
      (void)hipSetDevice(cur);
    }
    p = nullptr;
    n = 0;
    cap = 0;
  }
};

struct DevPolicySet {
  DevBuf prog, preds, alts, conjs, atoms, rules, filters, kinds, strrefs, strpairs, sels, sellabels, selexprs, kgs,
      gsegs, gwords, pstr, fword, fbit, flist, frule, rcompact, gsdesc, gsmem;
  // site-record groups of the specialized kernels (kvdevtypes.h GSiteDesc)
  uint32_t gs_groups = 0, gs_members = 0;
  DevPS view{};
  // specialized kernels (KV_COMPILE_SPECIALIZE): one module per kernel program, one
  // function per rule chunk
  std::vector<hipModule_t> mods;
  std::vector<hipFunction_t> fns;
  // output-mode variants (JitImage::variants): DevOut::full value -> a function per rule kernel
  // (the variant where it compiled within the plan's registers, else the generic kernel)
  std::map<uint32_t, std::vector<hipFunction_t>> vfns;
  const std::vector<hipFunction_t>& fns_for(uint32_t full) const {
    auto it = vfns.find(full);
    return it == vfns.end() ? fns : it->second;
  }
  // the rule kernels longest first, as the first session to time them found (DevSession::
  // order_kernels); later sessions of the policy set on this device, kv_validate's single pass
  // included, start from it
  std::mutex order_mu;
  std::vector<uint32_t> korder;
  hipFunction_t ptab_fn = nullptr;  // value-predicate table builder (kvj_ptab)
  uint32_t mtup_words = 0;          // match words per tuple (kv_mfac + kv_mtup, factored match)
  uint32_t fac_slots = 0;
  uint32_t memo_words = 0, ptab_rows = 0;
  int dev = -1;
  bool specialized() const { return !mods.empty(); }
  ~DevPolicySet() {
    if (!mods.empty()) {
      int cur;
      if (hipGetDevice(&cur) == hipSuccess) {
        (void)hipSetDevice(dev);
        for (hipModule_t m : mods) (void)hipModuleUnload(m);
        (void)hipSetDevice(cur);
      }
    }
  }
};

struct DevBatchRes {
  DevBuf nodes, vals, res, kvs, bstr, nsbits, koff, klen, kstr, nsms, lsets, asets, tuprep, tupkent, kentrep, view_dev;
  // pattern variables (kvvars.cpp): the batch predicate table (a DevPS with its pred tables),
  // outcome ids per [dynamic leaf][res], statuses per [dynamic rule][res]
  DevBuf dpreds, dalts, dconjs, datoms, dgsegs, dgwords, dpstr, dps, dleaf, dynst;
  // path columns of the specialized kernels (kvcol.h): the pool, the column descriptors, the
  // families and their per-group element-row prefixes; build time and pool size
  DevBuf pcol, pcold, pfam, perow;
  double pcol_ms = 0;
  DevBatch view{};
};

}  // namespace

struct kv_policyset {
  PolicySet ps;
  std::unique_ptr<JitImage> jit;  // KV_COMPILE_SPECIALIZE
  std::mutex mu;
  std::map<int, std::unique_ptr<DevPolicySet>> dev;
};

struct kv_batch {
  Batch b;
  const kv_policyset* owner = nullptr;
  std::mutex mu;
  // device copies, shared with the sessions that use them (a session keeps its copy alive when
  // the batch drops it: kv_batch_free, a parts session's detach)
  std::map<int, std::shared_ptr<DevBatchRes>> dev;
  std::once_flag dyn_once;
  DynHost dyn;  // pattern-variable tables (build_dyn), on first use
  const DynHost& dyn_host(const PolicySet& ps) {
    std::call_once(dyn_once, [&]() { build_dyn(ps, b, &dyn); });
    return dyn;
  }
  // caller index -> store index (the inverse of Batch::order), on first use; null: identity
  std::once_flag inv_once;
  std::vector<uint32_t> inv;
  const uint32_t* inverse() {
    if (b.order.empty()) return nullptr;
    std::call_once(inv_once, [&]() {
      inv.assign(b.order.size(), 0);
      for (size_t i = 0; i < b.order.size(); i++) inv[b.order[i]] = (uint32_t)i;
    });
    return inv.data();
  }
};

namespace {

// Page-locked host blocks are expensive to create (pinning), so released result
// buffers are kept for the next result of the process (up to 8 GiB): a host that
// validates batch after batch pays the pinning once.
// A caller that knows its batches' size can page-lock an arena up front (kv_host_reserve, outside
// ingest): blocks are then carved from it (first fit, 2 MiB granules, freed ranges coalesce) before
// any new block is page-locked, so even a process's first batch ingests into page-locked memory
// that is already there.
struct PinnedPool {
  std::mutex mu;
  std::multimap<size_t, void*> free;  // capacity -> block
  size_t held = 0;
  char* arena = nullptr;
  size_t arena_bytes = 0;
  std::map<size_t, size_t> arena_free;  // offset -> bytes
  static constexpr size_t kGran = 2u << 20;
  static PinnedPool& get() {
    static PinnedPool* p = new PinnedPool();  // never destroyed: blocks may outlive static teardown
    return *p;
  }
  bool reserve(size_t bytes) {
    std::lock_guard<std::mutex> g(mu);
    if (arena) return arena_bytes >= bytes;
    bytes = (bytes + kGran - 1) / kGran * kGran;
    void* p = nullptr;
    if (!bytes || hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    arena = (char*)p;
    arena_bytes = bytes;
    arena_free[0] = bytes;
    return true;
  }
  bool in_arena(const void* p) const { return arena && (const char*)p >= arena && (const char*)p < arena + arena_bytes; }
  void* take(size_t bytes, size_t* cap) {
    {
      std::lock_guard<std::mutex> g(mu);
      auto it = free.lower_bound(bytes);
      if (it != free.end() && it->first <= 2 * bytes + (1u << 20)) {
        void* p = it->second;
        *cap = it->first;
        held -= it->first;
        free.erase(it);
        return p;
      }
      if (arena) {
        const size_t want = (bytes + kGran - 1) / kGran * kGran;
        for (auto a = arena_free.begin(); a != arena_free.end(); ++a)
          if (a->second >= want) {
            const size_t off = a->first, left = a->second - want;
            arena_free.erase(a);
            if (left) arena_free[off + want] = left;
            *cap = want;
            return arena + off;
          }
      }
    }
    // headroom (+1/8, 16 MiB granules) so the next batch's slightly larger result fits the block
    const size_t want = bytes < (16u << 20) ? bytes : ((bytes + bytes / 8 + (16u << 20) - 1) & ~(size_t)((16u << 20) - 1));
    void* p = nullptr;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    *cap = want;
    return p;
  }
  void give(void* p, size_t cap) {
    std::lock_guard<std::mutex> g(mu);
    if (in_arena(p)) {  // back into the arena, merged with its free neighbours
      size_t off = (size_t)((char*)p - arena), len = cap;
      auto nx = arena_free.lower_bound(off);
      if (nx != arena_free.end() && nx->first == off + len) {
        len += nx->second;
        nx = arena_free.erase(nx);
      }
      if (nx != arena_free.begin()) {
        auto pv = std::prev(nx);
        if (pv->first + pv->second == off) {
          off = pv->first;
          len += pv->second;
          arena_free.erase(pv);
        }
      }
      arena_free[off] = len;
      return;
    }
    if (held + cap > (8ull << 30)) {
      (void)hipHostFree(p);
      return;
    }
    free.emplace(cap, p);
    held += cap;
  }
};

// Page-locked store arrays of ingested batches (kvinternal.hpp HostMem): blocks from the
// pool, registered by address so the upload can tell a page-locked source (direct DMA)
// from a pageable one (staging ring), and so a block returns to the pool when freed.
struct PinnedStore {
  std::mutex mu;
  std::map<uintptr_t, size_t> live;  // block -> capacity
  static PinnedStore& get() {
    static PinnedStore* p = new PinnedStore();
    return *p;
  }
  static bool enabled() {
    static const bool on = []() {
      if (getenv("KVGPU_PINNED") && getenv("KVGPU_PINNED")[0] == '0') return false;
      int n = 0;  // no device (host-only use of the library): plain memory
      if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return false;
      }
      return true;
    }();
    return on;
  }
  static void* take(size_t bytes) {
    if (!enabled()) return nullptr;
    size_t cap = 0;
    void* p = PinnedPool::get().take(bytes, &cap);
    if (!p) return nullptr;
    std::lock_guard<std::mutex> g(get().mu);
    get().live[(uintptr_t)p] = cap;
    return p;
  }
  static bool give(void* p) {
    size_t cap = 0;
    {
      std::lock_guard<std::mutex> g(get().mu);
      auto it = get().live.find((uintptr_t)p);
      if (it == get().live.end()) return false;
      cap = it->second;
      get().live.erase(it);
    }
    PinnedPool::get().give(p, cap);
    return true;
  }
  // [src, src + bytes) inside one live page-locked block
  static bool contains(const void* src, size_t bytes) {
    std::lock_guard<std::mutex> g(get().mu);
    auto& m = get().live;
    auto it = m.upper_bound((uintptr_t)src);
    if (it == m.begin()) return false;
    --it;
    return (uintptr_t)src + bytes <= it->first + it->second;
  }
};
struct InstallHostMem {
  InstallHostMem() {
    g_hostmem.take = &PinnedStore::take;
    g_hostmem.give = &PinnedStore::give;
  }
} install_host_mem_;

bool pinned_src(const void* src, size_t bytes) { return PinnedStore::contains(src, bytes); }

// Host array without value-initialisation; page-locked (pooled hipHostMalloc) unless
// KVGPU_PINNED=0, so device-to-host copies of results are direct DMA.
template <class T>
struct HostArray {
  T* p = nullptr;
  size_t n = 0, cap = 0;
  bool pinned = false;
  HostArray() = default;
  HostArray(const HostArray&) = delete;
  HostArray& operator=(const HostArray&) = delete;
  HostArray(HostArray&& o) noexcept : p(o.p), n(o.n), cap(o.cap), pinned(o.pinned) { o.p = nullptr; o.n = 0; }
  ~HostArray() { release(); }
  void alloc(size_t count) {
    release();
    n = count;
    if (!count) return;
    static const bool use_pinned = !(getenv("KVGPU_PINNED") && getenv("KVGPU_PINNED")[0] == '0');
    if (use_pinned && (p = (T*)PinnedPool::get().take(count * sizeof(T), &cap)) != nullptr) {
      pinned = true;
      return;
    }
    p = (T*)malloc(count * sizeof(T));
    if (!p) throw std::bad_alloc();
  }
  void release() {
    if (p) {
      if (pinned) PinnedPool::get().give(p, cap);
      else free(p);
    }
    p = nullptr;
    n = 0;
    cap = 0;
    pinned = false;
  }
  T* data() const { return p; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  T& operator[](size_t i) const { return p[i]; }
};

}  // namespace

// Records of one device shard: FAIL / ERROR / SKIP pairs, rule-major and in
// resource order (kv_rec_* kernels). Record of (rule, local res): base[rule] +
// offs[rule][tile] + the record pairs before it in its tile (from the statuses).
struct ResultPart {
  std::shared_ptr<kv_batch> shard;  // the shard's batch (null: the result's own batch)
  uint64_t lo = 0, n = 0;           // resources [lo, lo + n) of the result
  uint32_t tiles = 0;
  HostArray<uint32_t> offs;         // [rule][tile] exclusive record offsets within the rule (page-locked:
                                    // C3's 38 MB crossed PCIe through a staging copy at ~1 GB/s)
  std::vector<uint64_t> base;       // [rule + 1] record offsets of the rules
  HostArray<ErrRec8> rec;           // compact records (with `uni`: only the rules that are not uniform)
  HostArray<ErrRec> recw;           // full records, parallel to rec (only when some record is wide)
  // Record codes (kv_rec_code_kernel): record i of a coded rule is its rule's table entry
  // tab[rule * KV_REC_CODES + code[i]] (the lane field left out); a raw rule's records are
  // rec[nbase[rule] ...). Empty `raw`: rec holds every record.
  std::vector<uint8_t> raw;
  std::vector<ErrRec8> tab;
  HostArray<uint8_t> code;
  std::vector<uint64_t> nbase;
  // Status transfer form (kv_status_pack_kernel): the flags of the (rule, KV_RWG-status segment)s
  // the pass wrote, their statuses at 4 bits (KV_RWG / 2 bytes a segment, rule-major), the first
  // packed segment of each rule; the other segments are NOMATCH. Empty sflag: the part's statuses
  // crossed as dense rows of kv_result::status.
  HostArray<uint8_t> sflag, spack;
  std::vector<uint64_t> sbase;
  uint64_t nwg = 0;
  // statuses [lo, lo + n) of rule `rule` from the transfer form into dst[0, n)
  void unpack_row(uint32_t rule, uint8_t* dst) const {
    if (!n || sbase.empty()) return;  // (a part without resources packs nothing)
    const uint8_t* f = sflag.data() + (size_t)rule * nwg;
    const uint8_t* src = spack.data() + sbase[rule] * (KV_RWG / 2);
    const __m128i lo4 = _mm_set1_epi8(0x0F);
    for (uint64_t g = 0; g < nwg; g++) {
      const uint64_t q0 = g * KV_RWG, m = std::min<uint64_t>(KV_RWG, n - q0);
      uint8_t* d = dst + q0;
      if (!f[g]) {
        memset(d, ST_NOMATCH, m);
        continue;
      }
      uint64_t i = 0;
      for (; i + 32 <= m; i += 32) {
        const __m128i b = _mm_loadu_si128((const __m128i*)(src + i / 2));
        const __m128i l = _mm_and_si128(b, lo4), h = _mm_and_si128(_mm_srli_epi16(b, 4), lo4);
        _mm_storeu_si128((__m128i*)(d + i), _mm_unpacklo_epi8(l, h));
        _mm_storeu_si128((__m128i*)(d + i + 16), _mm_unpackhi_epi8(l, h));
      }
      for (; i < m; i++) d[i] = (src[i / 2] >> (4 * (i & 1))) & 15u;
      src += KV_RWG / 2;
    }
  }
  uint64_t n_rec() const { return base.empty() ? 0 : base.back(); }
  // record i of rule `rule` (base[rule] <= i < base[rule + 1])
  ErrRec8 r8(uint32_t rule, uint64_t i) const {
    if (raw.empty()) return rec[i];
    return raw[rule] ? rec[nbase[rule] + (i - base[rule])] : tab[(size_t)rule * KV_REC_CODES + code[i]];
  }
};

struct kv_result {
  const kv_policyset* ps = nullptr;
  const kv_batch* b = nullptr;
  uint64_t n_rules = 0, n_res = 0;
  // [rule][res] in the batch's store order (Batch::order), or in the caller's order with
  // caller_order; `res` below is an index into it unless named a caller index.
  // kv_result_status returns the caller order (status_c, a host permutation, when they differ).
  HostArray<uint8_t> status;
  std::once_flag sc_once;
  HostArray<uint8_t> status_c;
  // the parts hold their statuses in the transfer form (ResultPart::sflag) until an accessor
  // materialises `status` (st_store) or the caller-order copy (status_caller)
  bool sparse = false;
  std::once_flag st_once;
  // statuses and records were fetched in the caller's order (a permuted batch fetched whole:
  // DevSession::fetch); `status` is then the caller order and `res` below a caller index
  bool caller_order = false;
  std::vector<ResultPart> parts;    // by resource range
  bool errors = false;              // KV_MODE_ERRORS: records fetched
  std::vector<int64_t> counts;
  std::vector<int64_t> scope_counts;  // [scope][rule][KV_HIST] (KV_MODE_SCOPES)
  double kernel_ms = 0;
  uint32_t mode = 0;
  // wall-clock phases of the kv_validate that made this result (kv_result_phase): upload, setup,
  // pass, then the fetch's device work and copies, each ended by a stream synchronize
  std::vector<std::pair<std::string, double>> phases;
  // bulk failure export (kv_result_failures), built on first use
  std::once_flag fail_once;
  std::vector<uint32_t> f_rule, f_path;
  std::vector<uint64_t> f_res;
  std::vector<std::string> f_paths;

  bool has_err() const { return errors; }
  // store index of caller index `res`
  uint64_t sidx(uint64_t res) const { return caller_order ? res : store_of(res); }
  // the batch's store slot of caller index `res` (indexes the batch-side tables: dynamic leaves)
  uint64_t store_of(uint64_t res) const {
    const uint32_t* iv = const_cast<kv_batch*>(b)->inverse();
    return iv ? iv[res] : res;
  }
  // caller index of status / record index `s`
  uint64_t cidx(uint64_t s) const { return caller_order || b->b.order.empty() ? s : b->b.order[s]; }
  bool has_status() const { return sparse || !status.empty(); }
  static unsigned host_threads() { return std::max(1u, std::min<unsigned>(16u, std::thread::hardware_concurrency())); }
  // out[c] = row[inv[c]] (a gather: sequential 8-byte stores, reads from a row that stays in the
  // core's cache; 2.5x the rate of the scatter out[ord[q]] = row[q] on this host's cores)
  static void gather_row(const uint8_t* row, const uint32_t* inv, uint64_t n, uint8_t* out) {
    uint64_t c = 0;
    for (; c + 8 <= n; c += 8) {
      uint64_t v = 0;
      for (int k = 0; k < 8; k++) v |= (uint64_t)row[inv[c + k]] << (8 * k);
      memcpy(out + c, &v, 8);
    }
    for (; c < n; c++) out[c] = row[inv[c]];
  }
  // rows [rule][0, n_res) of dst from the parts' transfer form, rules split over host threads;
  // with `inv` (caller index -> store index) each row is unpacked in store order and gathered
  void unpack_rows(uint8_t* dst, const uint32_t* inv) const {
    const unsigned T = host_threads();
    std::vector<std::thread> th;
    for (unsigned t = 0; t < T; t++)
      th.emplace_back([&, t]() {
        std::vector<uint8_t> tmp(inv ? n_res : 0);
        for (uint64_t rl = t; rl < n_rules; rl += T) {
          uint8_t* row = inv ? tmp.data() : dst + rl * n_res;
          for (const ResultPart& p : parts) p.unpack_row((uint32_t)rl, row + p.lo);
          if (inv) gather_row(row, inv, n_res, dst + rl * n_res);
        }
      });
    for (auto& x : th) x.join();
  }
  // the status matrix in the records' order (store order unless caller_order), materialised from
  // the transfer form on first use
  const uint8_t* st_store() {
    if (sparse)
      std::call_once(st_once, [this]() {
        status.alloc(n_rules * n_res);
        unpack_rows(status.data(), nullptr);
      });
    return status.empty() ? nullptr : status.data();
  }
  // the statuses in caller order: rows of the store-order matrix gathered through the batch's
  // inverse order, rules split over host threads (a permuted batch only); from the transfer form directly
  // when the store-order matrix was not materialised
  const uint8_t* status_caller() {
    if (b->b.order.empty() || !has_status() || caller_order) return st_store();
    std::call_once(sc_once, [this]() {
      status_c.alloc(n_rules * n_res);
      const uint32_t* inv = const_cast<kv_batch*>(b)->inverse();
      if (status.empty()) {
        unpack_rows(status_c.data(), inv);
        return;
      }
      const unsigned T = host_threads();
      std::vector<std::thread> th;
      for (unsigned t = 0; t < T; t++)
        th.emplace_back([&, t]() {
          for (uint64_t rl = t; rl < n_rules; rl += T)
            gather_row(status.data() + rl * n_res, inv, n_res, status_c.data() + rl * n_res);
        });
      for (auto& x : th) x.join();
    });
    return status_c.data();
  }
  const Batch& batch_of(const ResultPart& p) const { return p.shard ? p.shard->b : b->b; }
  const ResultPart* part_of(uint64_t res) const {
    for (const ResultPart& p : parts)
      if (res >= p.lo && res < p.lo + p.n) return &p;
    return nullptr;
  }
  static ErrRec decode(const ErrRec8& c) {
    ErrRec e{};
    e.kind_flags = (c.w0 & 15u) | (((c.w0 >> 4) & 3u) << 16);
    e.pnode = c.w0 >> 7;
    e.keynode = ABSENT;
    e.resnode = ABSENT;
    e.idx[0] = c.w1 & 1023u;
    e.idx[1] = (c.w1 >> 10) & 255u;
    e.idx[2] = (c.w1 >> 18) & 255u;
    e.idx[3] = 0;
    return e;
  }
  // record index of pair (rule, res) within its part
  uint64_t rec_index(const ResultPart& p, uint32_t rule, uint64_t res) const {
    const uint64_t local = res - p.lo;
    const uint64_t tile = local / KV_WG;
    uint64_t idx = p.base[rule] + p.offs[(size_t)rule * p.tiles + tile];
    const uint8_t* row = const_cast<kv_result*>(this)->st_store() + (size_t)rule * n_res;
    for (uint64_t q = p.lo + tile * KV_WG; q < res; q++) {
      const uint8_t s = row[q];
      idx += s == ST_FAIL || s == ST_ERROR || s == ST_SKIP;
    }
    return idx;
  }
  // error record of a FAIL / ERROR / SKIP pair, and the batch its node ids refer to
  bool err(uint32_t rule, uint64_t res, ErrRec* e, const Batch** bt) const {
    const ResultPart* p = part_of(res);
    if (!p || !errors) return false;
    const uint64_t i = rec_index(*p, rule, res);
    if (i >= p->n_rec() || i < p->base[rule] || i >= p->base[rule + 1]) return false;
    const ErrRec8 c = p->r8(rule, i);
    *e = (c.w0 & ERR8_WIDE) && !p->recw.empty() ? p->recw[i] : decode(c);
    *bt = &batch_of(*p);
    return true;
  }
};

namespace {

int fail(kv_error** err, int code, const std::string& msg) {
  if (err) {
    *err = (kv_error*)malloc(sizeof(kv_error));
    (*err)->code = code;
    (*err)->message = strdup(msg.c_str());
  }
  return code;
}

DevPolicySet& dev_ps(kv_policyset* s, int device) {
  std::lock_guard<std::mutex> g(s->mu);
  auto it = s->dev.find(device);
  if (it != s->dev.end()) return *it->second;
  auto d = std::make_unique<DevPolicySet>();
  const PolicySet& ps = s->ps;
  d->prog.upload(ps.prog, device);
  d->preds.upload(ps.preds, device);
  d->alts.upload(ps.alts, device);
  d->conjs.upload(ps.conjs, device);
  d->atoms.upload(ps.atoms, device);
  d->rules.upload(ps.rules, device);
  d->filters.upload(ps.filters, device);
  d->kinds.upload(ps.kinds, device);
  d->strrefs.upload(ps.strrefs, device);
  d->strpairs.upload(ps.strpairs, device);
  d->sels.upload(ps.selectors, device);
  d->sellabels.upload(ps.sellabels, device);
  d->selexprs.upload(ps.selexprs, device);
  d->kgs.upload(ps.kg_specs, device);
  d->gsegs.upload(ps.gsegs, device);
  d->gwords.upload(ps.gwords, device);
  d->pstr.upload_raw(ps.strs.data(), ps.strs.size(), device);
  DevPS& v = d->view;
  v.prog = (const Inst*)d->prog.p;
  v.preds = (const Pred*)d->preds.p;
  v.alts = (const Alt*)d->alts.p;
  v.conjs = (const Conj*)d->conjs.p;
  v.atoms = (const Atom*)d->atoms.p;
  v.rules = (const RuleRec*)d->rules.p;
  v.filters = (const MFilter*)d->filters.p;
  v.kinds = (const KindSpec*)d->kinds.p;
  v.strrefs = (const StrRef*)d->strrefs.p;
  v.strpairs = (const StrPair*)d->strpairs.p;
  v.sels = (const Selector*)d->sels.p;
  v.sellabels = (const SelLabel*)d->sellabels.p;
  v.selexprs = (const SelExpr*)d->selexprs.p;
  v.kg_specs = (const uint32_t*)d->kgs.p;
  v.gsegs = (const GSeg*)d->gsegs.p;
  v.gwords = (const GWord*)d->gwords.p;
  v.n_rules = (uint32_t)ps.rules.size();
  v.n_filters = (uint32_t)ps.filters.size();
  v.n_sels = (uint32_t)ps.selectors.size();
  v.pstr = (const uint8_t*)d->pstr.p;
  // resource version "*" (checkKind, pkg/engine/utils.go:49): when "*" is not in the key dictionary no
  // resource can carry it, and an unknown version (KEY_NONE) must not compare equal to it
  v.star_id = ps.lookup("*");
  if (v.star_id == KEY_NONE) v.star_id = KEY_NONE - 1;
  d->dev = device;
  if (s->jit) {
    const JitImage& J = *s->jit;
    std::map<std::string, hipFunction_t> byname;
    for (size_t i = 0; i < J.codes.size(); i++) {
      hipModule_t m;
      HIPCHK(hipModuleLoadData(&m, J.codes[i].data()));
      d->mods.push_back(m);
      hipFunction_t f;
      HIPCHK(hipModuleGetFunction(&f, m, J.kernel_name[i].c_str()));
      byname[J.kernel_name[i]] = f;
    }
    for (const JitImage::Variant& v : J.variants) {
      std::map<std::string, hipFunction_t> vname;
      for (size_t i = 0; i < v.codes.size() && i < J.kernel_name.size(); i++) {
        if (v.codes[i].empty()) continue;
        hipModule_t m;
        HIPCHK(hipModuleLoadData(&m, v.codes[i].data()));
        d->mods.push_back(m);
        hipFunction_t f;
        HIPCHK(hipModuleGetFunction(&f, m, J.kernel_name[i].c_str()));
        vname[J.kernel_name[i]] = f;
      }
      std::vector<hipFunction_t>& fv = d->vfns[v.full];
      for (auto& ch : J.chunks) {
        auto it = vname.find(ch.name);
        fv.push_back(it != vname.end() ? it->second : byname.at(ch.name));
      }
    }
    for (auto& ch : J.chunks) {
      auto it = byname.find(ch.name);
      if (it == byname.end()) throw std::runtime_error("specialized kernel " + ch.name + " missing");
      hipFunction_t f = it->second;
      d->fns.push_back(f);
      if (getenv("KVGPU_VERBOSE")) {  // register / scratch use of each specialized kernel
        int regs = 0, local = 0;
        (void)hipFuncGetAttribute(&regs, HIP_FUNC_ATTRIBUTE_NUM_REGS, f);
        (void)hipFuncGetAttribute(&local, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, f);
        fprintf(stderr, "[kvgpu] %s: %zu rules, %d VGPRs, %d B scratch/lane\n", ch.name.c_str(), ch.rules.size(), regs,
                local);
      }
    }
    d->rcompact.upload(J.rec_compact, device);  // record layout per rule (JitImage::rec_compact)
    if (!J.gs_desc.empty()) {
      d->gs_groups = (uint32_t)(J.gs_desc.size() / 4u);
      d->gs_members = J.gs_members;
      d->gsdesc.upload(J.gs_desc, device);
      d->gsmem.upload(J.gs_mem, device);
    }
    if (J.mtup_words) {  // factored-match descriptors of the kernels' match bits
      d->mtup_words = J.mtup_words;
      d->fac_slots = J.fac_slots;
      d->fword.upload(J.fac_word, device);
      d->fbit.upload(J.fac_bit, device);
      d->flist.upload(J.fac_flist, device);
      d->frule.upload(J.fac_rule, device);
      v.fac_word = (const uint32_t*)d->fword.p;
      v.fac_bit = (const uint32_t*)d->fbit.p;
      v.fac_flist = (const uint32_t*)d->flist.p;
      v.fac_rule = (const uint32_t*)d->frule.p;
      v.fac_slots = J.fac_slots;
      v.fac_words = J.mtup_words;
    }
    if (J.memo_words) {
      d->ptab_fn = byname.at("kvj_ptab");
      d->memo_words = J.memo_words;
      d->ptab_rows = (uint32_t)((J.memo_preds.size() + J.ptab_row - 1) / J.ptab_row);
    }
  }
  auto& ref = *d;
  s->dev[device] = std::move(d);
  return ref;
}

// Path columns of the batch for the policy set's specialized kernels (kvcol.h, kvdevtypes.h):
// family 0 at [wave group][column][lane] (wave groups padded to whole workgroups, so every lane
// of the rule kernels' grid has its cells), then each family's element rows; built once per
// batch and device from the node rows (d->view_dev must hold the batch view).
void build_pcol(const JitImage& J, const Batch& b, DevBatchRes* d, int device) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint32_t nf = (uint32_t)J.fam_ncols.size(), j0 = J.fam_ncols.at(0);
  const uint64_t groups64 = (b.res.size() + KV_WG - 1) / KV_WG * (KV_WG / KV_LANES);
  if (groups64 > 0x3FFFFFFull) throw std::runtime_error("path columns: too many resources");
  const uint32_t groups = (uint32_t)groups64;
  d->pcold.upload(J.cols, device);
  d->perow.alloc((size_t)std::max<uint32_t>(1u, nf - 1) * (groups + 1) * sizeof(uint32_t), device);
  HIPCHK(hipMemset(d->perow.p, 0, d->perow.n));
  std::vector<ColFam> fams(nf);
  for (uint32_t f = 0; f < nf; f++) {
    fams[f].arr_col = J.fam_arr[f];
    fams[f].ncols = J.fam_ncols[f];
    fams[f].erow = f ? (uint32_t*)d->perow.p + (size_t)(f - 1) * (groups + 1) : nullptr;
  }
  d->pfam.upload(fams, device);
  const DevBatch* Bd = (const DevBatch*)d->view_dev.p;
  const ColDesc* cd = (const ColDesc*)d->pcold.p;
  std::vector<uint32_t> erow;
  if (nf > 1) {
    HIPCHK(launch_pcol_rows(Bd, cd, (const ColFam*)d->pfam.p, nf, groups, nullptr));
    erow.resize((size_t)(nf - 1) * (groups + 1));
    HIPCHK(hipMemcpy(erow.data(), d->perow.p, erow.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  const uint64_t root_cells = (uint64_t)groups * j0 * KV_LANES;
  uint64_t cells = root_cells;
  for (uint32_t f = 1; f < nf; f++) {
    fams[f].off_lo = (uint32_t)cells;
    fams[f].off_hi = (uint32_t)(cells >> 32);
    cells += (uint64_t)erow[(size_t)(f - 1) * (groups + 1) + groups] * fams[f].ncols * KV_LANES;
  }
  // (the kernels index cells with 32 bits)
  if (cells >= (1ull << 32)) throw std::runtime_error("path columns: more than 2^32 cells");
  HIPCHK(hipMemcpy(d->pfam.p, fams.data(), fams.size() * sizeof(ColFam), hipMemcpyHostToDevice));
  // two planes (kvcol.h col_put): (kt, a, c) 12 B per cell, then b 4 B per cell
  d->pcol.alloc(cells * sizeof(Node), device);
  uint32_t* pool = (uint32_t*)d->pcol.p;
  if (cells > root_cells) {  // element rows past a lane's own elements stay zero (both planes)
    HIPCHK(hipMemset(pool + 3 * root_cells, 0, (cells - root_cells) * 12u));
    HIPCHK(hipMemset(pool + 3 * cells + root_cells, 0, (cells - root_cells) * 4u));
  }
  HIPCHK(launch_pcol_build(Bd, cd, (const ColFam*)d->pfam.p, j0, 0, j0, groups, false, pool, cells, nullptr));
  HIPCHK(launch_pcol_build(Bd, cd, (const ColFam*)d->pfam.p, j0, j0, (uint32_t)J.cols.size() - j0, groups, true,
                           pool, cells, nullptr));
  HIPCHK(hipStreamSynchronize(nullptr));
  d->view.pcol = pool;
  d->view.pcolb = pool + 3 * cells;
  d->pcol_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (getenv("KVGPU_VERBOSE"))
    fprintf(stderr, "[kvgpu] path columns: %zu columns in %u families, %.1f MB, built in %.2f ms\n", J.cols.size(), nf,
            cells * sizeof(Node) / 1e6, d->pcol_ms);
}

std::shared_ptr<DevBatchRes> dev_batch(kv_batch* bt, const PolicySet& ps, int device) {
  std::lock_guard<std::mutex> g(bt->mu);
  auto it = bt->dev.find(device);
  if (it != bt->dev.end()) return it->second;
  auto d = std::make_shared<DevBatchRes>();
  const Batch& b = bt->b;
  if (b.rmask.size() != b.n_rows || b.rwide.size() != b.n_rows || b.roff.size() != b.n_rows)
    throw std::runtime_error("batch: packed row arrays do not match the row count");
  // packed rows: upload the non-zero cells, masks and row offsets, then expand to the
  // wave-group layout on the device. The page-locked arrays (rows, values, resources) go as
  // asynchronous copies on one stream, the expansion behind them, while this thread uploads the
  // pageable ones (strings, key table, match inputs) through the staging path beside them.
  hipStream_t us = StreamPool::get().take(device, hipStreamNonBlocking);
  DevBuf pc, rm, rw, ro;
  pc.upload_async(b.tcells, device, us);
  rm.upload_async(b.rmask, device, us);
  rw.upload_async(b.rwide, device, us);
  ro.upload_async(b.roff, device, us);
  d->vals.upload_async(b.vals, device, us);
  d->nodes.alloc(b.n_cells() * sizeof(Node), device);
  HIPCHK(launch_expand_rows((const uint64_t*)pc.p, (const uint64_t*)rm.p, (const uint64_t*)rw.p, (const uint32_t*)ro.p,
                            (const Val*)d->vals.p, b.n_rows, (Node*)d->nodes.p, us));
  d->res.upload_async(b.res, device, us);
  d->kvs.upload(b.kvs, device);
  d->bstr.upload_raw(b.strs.data(), b.strs.size(), device);
  d->nsbits.upload(b.ns_bits, device);
  // key string table: static dictionary then batch-dynamic keys
  std::vector<uint32_t> off, len;
  std::string ks;
  key_table(ps, b, &off, &len, &ks);
  d->koff.upload(off, device);
  d->klen.upload(len, device);
  d->kstr.upload_raw(ks.data(), ks.size(), device);
  d->nsms.upload(b.nsms, device);
  d->lsets.upload(b.lsets, device);
  d->asets.upload(b.asets, device);
  d->tuprep.upload(b.tup_rep, device);
  d->tupkent.upload(b.tup_kent, device);
  d->kentrep.upload(b.kent_rep, device);
  DevBatch& v = d->view;
  v.nodes = (const Node*)d->nodes.p;
  v.vals = (const Val*)d->vals.p;
  v.res = (const Res*)d->res.p;
  v.kvs = (const KV*)d->kvs.p;
  v.bstr = (const uint8_t*)d->bstr.p;
  v.ns_bits = (const uint32_t*)d->nsbits.p;
  v.key_off = (const uint32_t*)d->koff.p;
  v.key_len = (const uint32_t*)d->klen.p;
  v.kstr = (const uint8_t*)d->kstr.p;
  v.nsms = (const StrRef*)d->nsms.p;
  v.lsets = (const KVSet*)d->lsets.p;
  v.asets = (const KVSet*)d->asets.p;
  v.n_nsm = (uint32_t)b.nsms.size();
  v.n_lsets = (uint32_t)b.lsets.size();
  v.n_asets = (uint32_t)b.asets.size();
  v.ns_words = b.ns_words;
  v.n_res = (uint32_t)b.res.size();
  v.tup_rep = (const uint32_t*)d->tuprep.p;
  v.n_tup = (uint32_t)b.tup_rep.size();
  v.tup_kent = (const uint32_t*)d->tupkent.p;
  v.kent_rep = (const uint32_t*)d->kentrep.p;
  v.n_kent = (uint32_t)b.kent_rep.size();
  v.n_ns = (uint32_t)b.namespaces.size();
  {  // pattern variables: every pointer valid (16-byte buffers when the policy set has none)
    const DynHost& h = bt->dyn_host(ps);
    d->dpreds.upload(h.tbl.preds, device);
    d->dalts.upload(h.tbl.alts, device);
    d->dconjs.upload(h.tbl.conjs, device);
    d->datoms.upload(h.tbl.atoms, device);
    d->dgsegs.upload(h.tbl.gsegs, device);
    d->dgwords.upload(h.tbl.gwords, device);
    d->dpstr.upload_raw(h.tbl.strs.data(), h.tbl.strs.size(), device);
    DevPS dv{};
    dv.preds = (const Pred*)d->dpreds.p;
    dv.alts = (const Alt*)d->dalts.p;
    dv.conjs = (const Conj*)d->dconjs.p;
    dv.atoms = (const Atom*)d->datoms.p;
    dv.gsegs = (const GSeg*)d->dgsegs.p;
    dv.gwords = (const GWord*)d->dgwords.p;
    dv.pstr = (const uint8_t*)d->dpstr.p;
    d->dps.upload_raw(&dv, sizeof(DevPS), device);
    d->dleaf.upload(h.dleaf, device);
    d->dynst.upload(h.dyn_st, device);
    v.dps = (const DevPS*)d->dps.p;
    v.dleaf = (const uint32_t*)d->dleaf.p;
    v.dyn_st = (const uint8_t*)d->dynst.p;
  }
  d->view_dev.upload_raw(&d->view, sizeof(DevBatch), device);
  HIPCHK(hipStreamSynchronize(us));
  StreamPool::get().give(device, hipStreamNonBlocking, us);
  pc.release();
  rm.release();
  rw.release();
  ro.release();
  if (bt->owner && bt->owner->jit && !bt->owner->jit->cols.empty() && !b.res.empty()) {
    build_pcol(*bt->owner->jit, b, d.get(), device);
    d->view_dev.upload_raw(&d->view, sizeof(DevBatch), device);
  }
  bt->dev[device] = d;
  return d;
}

// Path segments from the pattern root to pnode p: keys (resolved wildcard keys
// from the record's key node) and array indices (loop counters of the record).
struct PathSeg {
  bool index;
  std::string key;
};
std::vector<PathSeg> path_segs(const PolicySet& ps, const Batch& b, const ErrRec& e, uint32_t p) {
  std::vector<PathSeg> segs;
  while (p != 0xFFFFFFFFu && p < ps.pnodes.size()) {
    const PNodeInfo& n = ps.pnodes[p];
    switch (n.seg) {
      case SEG_ROOT: break;
      case SEG_KEY: segs.push_back({false, n.key}); break;
      case SEG_LOOP: segs.push_back({true, std::to_string(e.idx[n.level & 3])}); break;
      case SEG_CONST_INDEX: segs.push_back({true, std::to_string(n.level)}); break;
      case SEG_RESOLVED: {
        if (e.keynode != ABSENT && e.keynode < b.n_cells()) {
          uint32_t k = node_key(b.cell(e.keynode).kt);
          segs.push_back({false, k < ps.keys.size() ? ps.keys[k] : b.dyn_keys[k - ps.keys.size()]});
        } else {
          segs.push_back({false, n.key});
        }
        break;
      }
    }
    p = n.parent;
  }
  std::reverse(segs.begin(), segs.end());
  return segs;
}

std::string join_path(const std::vector<PathSeg>& segs) {
  std::string out = "/";
  for (const PathSeg& s : segs) out += s.key + "/";
  return out;
}

uint32_t err_kind(const ErrRec& e) { return e.kind_flags & 0xFFFF; }

// pnode whose path is the PatternError path: the "*" shortcut reports its parent
// map (anchor.go:139), every other form the node it was raised at
uint32_t path_pnode(const PolicySet& ps, const ErrRec& e) {
  if (err_kind(e) == E_STAR && e.pnode < ps.pnodes.size()) return ps.pnodes[e.pnode].parent;
  return e.pnode;
}

std::string render_path(const PolicySet& ps, const Batch& b, const ErrRec& e) {
  return join_path(path_segs(ps, b, e, path_pnode(ps, e)));
}

// ---- Go fmt of resource values (unstructured typing: int64 / float64 / string /
// bool / nil / map[string]interface{} / []interface{}), for '%v' and %T operands
std::string res_T(const JDoc& d, int64_t n) {
  if (n < 0) return "<nil>";
  switch (d.at((uint32_t)n).t) {
    case J_MAP: return "map[string]interface {}";
    case J_ARR: return "[]interface {}";
    case J_STR: return "string";
    case J_BOOL: return "bool";
    case J_INT: return "int64";
    case J_FLOAT: return "float64";
    default: return "<nil>";
  }
}

std::string res_v(const JDoc& d, int64_t n) {
  if (n < 0) return "<nil>";
  const JNode& x = d.at((uint32_t)n);
  switch (x.t) {
    case J_MAP: {  // fmt prints maps with sorted keys
      std::vector<uint32_t> ix;
      for (uint32_t c = x.first; c < x.first + x.count; c++) ix.push_back(c);
      std::sort(ix.begin(), ix.end(), [&](uint32_t a, uint32_t b) { return d.key(d.at(a)) < d.key(d.at(b)); });
      std::string o = "map[";
      for (size_t k = 0; k < ix.size(); k++) {
        if (k) o += ' ';
        o += d.key(d.at(ix[k]));
        o += ':';
        o += res_v(d, ix[k]);
      }
      return o + "]";
    }
    case J_ARR: {
      std::string o = "[";
      for (uint32_t c = x.first; c < x.first + x.count; c++) {
        if (c > x.first) o += ' ';
        o += res_v(d, c);
      }
      return o + "]";
    }
    case J_STR: return std::string(d.sval(x));
    case J_BOOL: return x.b ? "true" : "false";
    case J_INT: return std::to_string(x.i);
    case J_FLOAT: return go_format_g(x.f);
    default: return "<nil>";
  }
}

// resource element at a pattern path (-1 when absent)
int64_t res_at(const JDoc& d, const std::vector<PathSeg>& segs) {
  int64_t n = d.root;
  for (const PathSeg& s : segs) {
    if (n < 0) return -1;
    const JNode& x = d.at((uint32_t)n);
    if (x.t == J_MAP) {
      n = d.get((uint32_t)n, s.key);
    } else if (x.t == J_ARR && s.index) {
      uint64_t i = std::stoull(s.key);
      n = i < x.count ? (int64_t)(x.first + i) : -1;
    } else {
      return -1;
    }
  }
  return n;
}

// err.Error() of the PatternError behind a FAIL / ERROR / SKIP record
// (pkg/engine/validate/validate.go:62-172, pkg/engine/anchor/anchor.go:61-261;
// condition / global anchor handlers wrap what propagates through them,
// anchor.go:72-95 with common/anchorKey.go:21-40)
std::string error_message(const PolicySet& ps, const Batch& b, const ErrRec& e, const JDoc& doc,
                          const std::string* dyn_pat_v = nullptr) {
  const uint32_t kind = err_kind(e);
  if (e.pnode >= ps.pnodes.size()) return "";
  PNodeInfo P = ps.pnodes[e.pnode];
  if (P.dleaf >= 0 && dyn_pat_v) P.pat_v = *dyn_pat_v;  // the resource's substituted pattern value
  const std::vector<PathSeg> segs = path_segs(ps, b, e, e.pnode);
  const std::string path = join_path(segs);
  std::string m;
  switch (kind) {
    case E_TYPE_MAP:
      m = "pattern and resource have different structures. Path: " + path + ". Expected " + P.pat_t + ", found " +
          res_T(doc, res_at(doc, segs));
      break;
    case E_TYPE_ARR:
      m = "validation rule Failed at path " + path + ", resource does not satisfy the expected overlay pattern";
      break;
    case E_VALUE:
      m = "resource value '" + res_v(doc, res_at(doc, segs)) + "' does not match '" + P.pat_v + "' at path " + path;
      break;
    case E_EMPTY_PATARR: m = "pattern Array empty"; break;
    case E_LEN: {
      int64_t n = res_at(doc, segs);
      uint32_t rl = n >= 0 && doc.at((uint32_t)n).t == J_ARR ? doc.at((uint32_t)n).count : 0;
      m = "validate Array failed, array length mismatch, resource Array len is " + std::to_string(rl) +
          " and pattern Array len is " + std::to_string(P.pat_len);
      break;
    }
    case E_NEG: m = path + "/" + (segs.empty() ? std::string() : segs.back().key) + " is not allowed"; break;
    case E_STAR: {
      std::vector<PathSeg> ps_ = segs;
      std::string key = ps_.empty() ? std::string() : ps_.back().key;
      if (!ps_.empty()) ps_.pop_back();
      m = join_path(ps_) + "/" + key + " not found";
      break;
    }
    case E_EXIST_PATLIST:
      m = "invalid pattern type " + P.pat_t + ": Pattern has to be of list to compare against resource";
      break;
    case E_EXIST_PATMAP:
      m = "invalid pattern type " + P.pat_t + ": Pattern has to be of type map to compare against items in resource";
      break;
    case E_EXIST_RESTYPE:
      m = "invalid resource type " + res_T(doc, res_at(doc, segs)) +
          ": Existence ^ () anchor can be used only on list/array type resource";
      break;
    case E_EXIST_FAIL: m = "existence anchor validation failed at path " + path; break;
    default: return "";
  }
  for (uint32_t q = e.pnode; q != 0xFFFFFFFFu && q < ps.pnodes.size(); q = ps.pnodes[q].parent) {
    if (ps.pnodes[q].wrap == 1) m = "conditional anchor mismatch: " + m;
    else if (ps.pnodes[q].wrap == 2) m = "global anchor mismatch: " + m;
  }
  return m;
}

}  // namespace

namespace {

// A launch configuration on one device over one batch (a whole batch or a
// shard): device-resident inputs and output buffers.
struct DevSession {
  kv_policyset* ps = nullptr;
  kv_batch* bt = nullptr;
  int device = 0;
  uint32_t mode = 0;
  uint64_t nrules = 0, nres = 0;
  DevBuf fflags, pview, st, er8, er, cn, scope, scn, ptab, mtab, mtbf, mtup, ftab;
  // The per-pass tables of the specialized kernels (value-predicate table kvj_ptab, match tables
  // kv_mtab / kv_mfac / kv_mtup) are double-buffered between consecutive passes (ptab / ptab1,
  // mtab / mtab1, ... read through pview / pview1): pass i + 1's tables are built on `pside` while
  // pass i's rule kernels run, waiting only for pass i - 1's rule kernels (the last readers of
  // their buffers), so their waves fill the workgroup slots the rule kernels' last round leaves
  // idle. ev_pt[b]: tables b built; ev_rk[b]: the rule kernels that read tables b done.
  // KVGPU_PTAB_PIPE=0: one set, built ahead of each pass's rule kernels (ptab on the session
  // stream, the match tables on `side`).
  DevBuf ptab1, pview1, mtab1, mtup1, ftab1, cn1, scn1;  // (counts of set 1: zeroed with its tables)
  uint32_t *mt1_ns = nullptr, *mt1_ann = nullptr, *mt1_sel = nullptr;
  hipStream_t pside = nullptr;
  hipEvent_t ev_pt[2] = {nullptr, nullptr}, ev_rk[2] = {nullptr, nullptr};
  bool ptab_pipe = false;
  uint32_t fac_entities = 0, ntup = 0;
  bool rec_compact = false;  // the last pass wrote records per wave segment (specialized kernels)
  // the batch's device copy, shared with the batch's cache and other sessions on it; a part of a
  // parts session keeps it after dropping the batch (detach_batch): the caller's host batch may
  // be freed once the part is attached
  std::shared_ptr<DevBatchRes> batch_ref;
  DevBuf r_offs, r_tot, r_base, r_out8, r_outw, r_wide;  // record compaction (fetch)
  DevBuf r_tkey, r_raw, r_nbase, r_code, r_out8b;        // record codes (fetch)
  DevBuf s_ccnt, s_cbase, s_pack;                        // status transfer form (fetch)
  HostArray<uint8_t> hstage;                             // page-locked staging of the fetch's small copies
  DevBuf inv_d, stc;                                     // caller-order statuses (fetch)
  DevBuf ord_d, r_mask;                                  // caller-order records: batch order, record lanes
  DevBuf stamps;                                         // KVGPU_STAMPS diagnostics
  DevBuf gsite, gcnt;                                    // site records of rule groups (pass)
  DevBuf sflag;                                          // written status segments (specialized)
  uint32_t mt_words = 0, mt_entities = 0;
  uint32_t *mt_ns = nullptr, *mt_ann = nullptr, *mt_sel = nullptr;
  uint32_t nscopes = 0, nvals = 0;
  DevOut O{};
  const DevBatch* bview = nullptr;
  const DevBatch* bhost = nullptr;  // host copy of the batch view (device pointers)
  DevPolicySet* dps = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  // specialized passes: the match tables (kv_mtab, kv_mfac, kv_mtup) run on `side` while
  // `stream` builds the value-predicate table (kvj_ptab); the rule kernels wait for both
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_rkf = nullptr, ev_rkj[3] = {};  // rule kernels over several streams (launch_specialized)
  std::vector<hipStream_t> rkx;                  // (the streams beyond `stream` and `side`)
  std::vector<hipEvent_t> kev;                   // start / end of each rule kernel in the timed pass
  std::vector<uint32_t> korder;                  // rule kernels, longest first (after a timed pass)
  bool ktiming = false;

  double upload_ms = 0;  // policy set + batch upload of the constructor (path columns included)
  DevSession(kv_policyset* p, kv_batch* b, const char* ctx_json, int dev, uint32_t m)
      : ps(p), bt(b), device(dev), mode(m) {
    HIPCHK(hipSetDevice(device));
    const auto tc0 = std::chrono::steady_clock::now();
    DevPolicySet& dp = dev_ps(ps, device);
    batch_ref = dev_batch(bt, ps->ps, device);
    DevBatchRes& db = *batch_ref;
    upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count();
    if (getenv("KVGPU_VERBOSE")) fprintf(stderr, "[kvgpu] session: policy set + batch upload %.1f ms\n", upload_ms);
    bview = (const DevBatch*)db.view_dev.p;
    bhost = &db.view;
    dps = &dp;
    fflags.upload(fold_filters(ps->ps, ctx_json), device);
    DevPS P = dp.view;
    P.fflags = (const uint32_t*)fflags.p;
    if (dp.ptab_fn) {  // value-predicate table of the specialized kernels: memo_words per distinct value
      nvals = (uint32_t)bt->b.vals.size();
      ptab.alloc((size_t)dp.memo_words * (nvals + KV_PTAB_PSEUDO) * sizeof(uint32_t), device);
      P.ptab = (const uint32_t*)ptab.p;
      P.n_vals = nvals + KV_PTAB_PSEUDO;
    }
    {  // match tables: one allocation, three [word][entity] tables
      const PolicySet& pp = ps->ps;
      const Batch& bb = bt->b;
      P.mt_ns_words = (pp.n_nss_bits + 31) / 32;
      P.mt_ann_words = (pp.n_ann_bits + 31) / 32;
      P.mt_sel_words = (uint32_t)((pp.selectors.size() + 31) / 32);
      const size_t n_ns = (size_t)P.mt_ns_words * bb.nsms.size(), n_an = (size_t)P.mt_ann_words * bb.asets.size(),
                   n_sl = (size_t)P.mt_sel_words * bb.lsets.size();
      mtab.alloc(std::max<size_t>(n_ns + n_an + n_sl, 1) * sizeof(uint32_t), device);
      mt_ns = (uint32_t*)mtab.p;
      mt_ann = mt_ns + n_ns;
      mt_sel = mt_ann + n_an;
      P.mt_ns = mt_ns;
      P.mt_ann = mt_ann;
      mtbf.upload(mtab_bit_filters(pp), device);
      P.mt_bitf = (const uint32_t*)mtbf.p;
      P.mt_sel = mt_sel;
      mt_words = P.mt_ns_words + P.mt_ann_words + P.mt_sel_words;
      mt_entities = (uint32_t)std::max({bb.nsms.size(), bb.asets.size(), bb.lsets.size()});
    }
    if (dp.mtup_words) {  // match bits of every rule per match tuple: mtup_words per tuple
      mtup.alloc(std::max<size_t>((size_t)dp.mtup_words * bt->b.tup_rep.size(), 1) * sizeof(uint32_t), device);
      P.mtup = (const uint32_t*)mtup.p;
      P.mtup_words = dp.mtup_words;
      // factor tables [slot][entity] of the five entity types, one allocation
      const DevBatch& bv = *bhost;
      const uint32_t ne[KV_FAC_TYPES] = {bv.n_kent, bv.n_nsm, bv.n_asets, bv.n_lsets, bv.n_ns};
      uint64_t at = 0;
      for (uint32_t t = 0; t < KV_FAC_TYPES; t++) {
        P.fac_off[t] = at;
        at += (uint64_t)dp.fac_slots * ne[t];
        fac_entities = std::max(fac_entities, ne[t]);
      }
      ftab.alloc(std::max<uint64_t>(at, 1) * sizeof(uint32_t), device);
      P.fac_tab = (uint32_t*)ftab.p;
    }
    pview.upload_raw(&P, sizeof(DevPS), device);  // read through a uniform pointer (scalar loads)
    ptab_pipe = dp.specialized() && !(getenv("KVGPU_PTAB_PIPE") && getenv("KVGPU_PTAB_PIPE")[0] == '0');
    if (ptab_pipe) {  // the second set of per-pass tables
      if (dp.ptab_fn) {
        ptab1.alloc(ptab.n, device);
        P.ptab = (const uint32_t*)ptab1.p;
      }
      mtab1.alloc(mtab.n, device);
      mt1_ns = (uint32_t*)mtab1.p;
      mt1_ann = mt1_ns + (mt_ann - mt_ns);
      mt1_sel = mt1_ns + (mt_sel - mt_ns);
      P.mt_ns = mt1_ns;
      P.mt_ann = mt1_ann;
      P.mt_sel = mt1_sel;
      if (dp.mtup_words) {
        mtup1.alloc(mtup.n, device);
        P.mtup = (const uint32_t*)mtup1.p;
        ftab1.alloc(ftab.n, device);
        P.fac_tab = (uint32_t*)ftab1.p;
      }
      pview1.upload_raw(&P, sizeof(DevPS), device);
    }
    nrules = ps->ps.rules.size();
    nres = bt->b.res.size();
    ntup = (uint32_t)bt->b.tup_rep.size();
    O.full = 0;
    // the status matrix: asked for, or the bytecode engine's per-scope counts read it back
    // (the specialized kernels count scopes inside the pass, O.full bit 3)
    if ((mode & (KV_MODE_STATUS | KV_MODE_ERRORS)) || ((mode & KV_MODE_SCOPES) && !dp.specialized())) {
      st.alloc(nrules * nres, device);
      O.status = (uint8_t*)st.p;
      O.full |= 1;
      if (dp.specialized()) {  // (flags of every segment, set by each pass)
        sflag.alloc(std::max<uint64_t>(nrules * ((nres + KV_RWG - 1) / KV_RWG), 1), device);
        HIPCHK(hipMemset(sflag.p, 1, sflag.n));
        O.sflag = (uint8_t*)sflag.p;
      }
    }
    if (mode & KV_MODE_ERRORS) {
      er8.alloc(nrules * nres * sizeof(ErrRec8), device);
      O.err8 = (ErrRec8*)er8.p;
      O.err = nullptr;  // full records: allocated by fetch() for the re-run pass, if some record is wide
      O.full |= 2;
      if (dp.gs_groups) {  // 64 x members 16 B slots per wave and group, a count per (group, wave)
        const uint64_t nw = (nres + 63) / 64;
        gsite.alloc(std::max<uint64_t>((uint64_t)dp.gs_members * nw * 64u * 16u, 16), device);
        gcnt.alloc(std::max<uint64_t>((uint64_t)dp.gs_groups * nw * sizeof(uint32_t), 4), device);
        O.gsite = (uint32_t*)gsite.p;
        O.gcnt = (uint32_t*)gcnt.p;
      }
    }
    cn.alloc(std::max<uint64_t>(nrules, 1) * KV_HIST * sizeof(unsigned long long), device);
    O.counts = (unsigned long long*)cn.p;
    if (ptab_pipe) cn1.alloc(cn.n, device);
    if (mode & KV_MODE_SCOPES) {
      // scope of every resource = its namespace index in the batch namespace table
      std::vector<uint32_t> sc(nres);
      for (uint64_t i = 0; i < nres; i++) sc[i] = bt->b.res[i].ns_index;
      nscopes = (uint32_t)bt->b.namespaces.size();
      scope.upload(sc, device);
      scn.alloc(std::max<uint64_t>((uint64_t)nscopes * nrules, 1) * KV_HIST * sizeof(unsigned long long), device);
      if (ptab_pipe) scn1.alloc(scn.n, device);
      O.scope = (const uint32_t*)scope.p;
      O.scounts = (unsigned long long*)scn.p;
      if (dp.specialized()) O.full |= 8;
    }
    if (getenv("KVGPU_JIT_STAMPS") && dp.specialized()) {  // diagnostics: segment stamps of the rule kernels' waves
      const uint64_t n = (nres + KV_RWG - 1) / KV_RWG * KV_RWAVES * kJitStamps;
      stamps.alloc(std::max<uint64_t>(n, 1) * sizeof(unsigned long long), device);
      HIPCHK(hipMemset(stamps.p, 0, stamps.n));
      for (hipModule_t m : dp.mods) {  // the kernels' global kvj_stamps -> this buffer
        hipDeviceptr_t g = nullptr;
        size_t gs = 0;
        if (hipModuleGetGlobal(&g, &gs, m, "kvj_stamps") == hipSuccess && gs == sizeof(void*))
          HIPCHK(hipMemcpy(g, &stamps.p, sizeof(void*), hipMemcpyHostToDevice));
        else
          (void)hipGetLastError();
      }
    }
    stream = StreamPool::get().take(device, hipStreamDefault);
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    side = StreamPool::get().take(device, hipStreamNonBlocking);
    if (ptab_pipe) {
      pside = StreamPool::get().take(device, hipStreamNonBlocking, true);  // (the lowest priority)
      for (int b = 0; b < 2; b++) {
        HIPCHK(hipEventCreateWithFlags(&ev_pt[b], hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_rk[b], hipEventDisableTiming));
      }
    }
    HIPCHK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_rkf, hipEventDisableTiming));
    for (hipEvent_t& e : ev_rkj) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // drop the kv_batch (parts sessions: the host batch is the caller's, and may be freed after
  // kv_session_attach_part); the session keeps the device copy through batch_ref, and so does
  // every other session using it (the batch's cache keeps its entry for later sessions)
  void detach_batch() { bt = nullptr; }
  // renumber the scope of every resource through map (batch namespace -> session scope) and
  // size the per-scope counts for n_total scopes
  void remap_scopes(const std::vector<uint32_t>& map, uint32_t n_total) {
    if (!(mode & KV_MODE_SCOPES)) return;
    HIPCHK(hipSetDevice(device));
    DevBuf m;
    m.upload(map, device);
    HIPCHK(launch_remap_u32((uint32_t*)scope.p, nres, (const uint32_t*)m.p, stream));
    HIPCHK(hipStreamSynchronize(stream));
    nscopes = n_total;
    scn.alloc(std::max<uint64_t>((uint64_t)nscopes * nrules, 1) * KV_HIST * sizeof(unsigned long long), device);
    if (ptab_pipe) scn1.alloc(scn.n, device);
    O.scounts = (unsigned long long*)scn.p;
  }
  ~DevSession() {
    (void)hipSetDevice(device);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_join) (void)hipEventDestroy(ev_join);
    if (ev_rkf) (void)hipEventDestroy(ev_rkf);
    for (hipEvent_t e : ev_rkj)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : kev) (void)hipEventDestroy(e);
    for (hipStream_t x : rkx) StreamPool::get().give(device, hipStreamNonBlocking, x);
    for (int b = 0; b < 2; b++) {
      if (ev_pt[b]) (void)hipEventDestroy(ev_pt[b]);
      if (ev_rk[b]) (void)hipEventDestroy(ev_rk[b]);
    }
    StreamPool::get().give(device, hipStreamNonBlocking, pside, true);
    StreamPool::get().give(device, hipStreamNonBlocking, side);
    StreamPool::get().give(device, hipStreamDefault, stream);
  }
  // enqueue `iters` passes, wait, return HIP-event milliseconds of all passes
  // vm: run the passes on the bytecode engine even when the policy set has specialized kernels
  // (the full-record re-run of fetch: the specialized kernels write compact records only)
  double run(int iters, bool vm = false) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipEventRecord(e0, stream));
    const bool pipe = ptab_pipe && dps->specialized() && !vm && nres;
    if (pipe && iters > 0) {  // pass 0's tables, after the start event
      HIPCHK(hipStreamWaitEvent(pside, e0, 0));
      launch_tables(0);
    }
    for (int i = 0; i < iters; i++) {
      rec_compact = dps->specialized() && !vm;
      if (pipe) {  // tables and zeroed counts of set i & 1 from launch_tables
        const int b = i & 1;
        launch_specialized(b);
        if (O.full & 8u)
          HIPCHK(launch_scope_totals((const unsigned long long*)(b ? scn1.p : scn.p), nscopes, (uint32_t)nrules,
                                     (unsigned long long*)(b ? cn1.p : cn.p), stream));
        // set b's last readers (rule kernels) and writers (scope totals) are done after this event:
        // launch_tables(b) of pass i + 2 zeroes its counts behind it
        HIPCHK(hipEventRecord(ev_rk[b], stream));
        if (i + 1 < iters) {  // the next pass's tables, once pass i - 1's kernels are done with them
          const int nb = (i + 1) & 1;
          if (i >= 1) HIPCHK(hipStreamWaitEvent(pside, ev_rk[nb], 0));
          launch_tables(nb);
        }
        continue;
      }
      // the match tables on the side stream, forked from and joined back into `stream`
      // (specialized passes; the bytecode engine runs everything in order on `stream`)
      hipStream_t ms = rec_compact ? side : stream;
      if (rec_compact) {
        HIPCHK(hipEventRecord(ev_fork, stream));
        HIPCHK(hipStreamWaitEvent(side, ev_fork, 0));
      }
      HIPCHK(hipMemsetAsync(cn.p, 0, cn.n, ms));
      if (mode & KV_MODE_SCOPES) HIPCHK(hipMemsetAsync(scn.p, 0, scn.n, ms));
      HIPCHK(launch_mtab((const DevPS*)pview.p, bview, mt_words, mt_entities, mt_ns, mt_ann, mt_sel, ms));
      if (rec_compact) {
        launch_specialized();  // (per-scope counts inside the rule kernels)
        if (O.full & 8u)  // per-rule totals from the per-scope counts (the kernels add only those)
          HIPCHK(launch_scope_totals((const unsigned long long*)scn.p, nscopes, (uint32_t)nrules,
                                     (unsigned long long*)cn.p, stream));
      } else {
        DevOut Ov = O;
        Ov.full &= ~8u;
        HIPCHK(launch_validate((const DevPS*)pview.p, bview, (uint32_t)nres, Ov, 0, (uint32_t)nrules, stream));
        if (mode & KV_MODE_SCOPES)
          HIPCHK(launch_scope_counts(O.status, (const uint32_t*)scope.p, (uint32_t)nres, (uint32_t)nrules, nscopes,
                                     (unsigned long long*)scn.p, stream));
      }
    }
    HIPCHK(hipEventRecord(e1, stream));
    HIPCHK(hipEventSynchronize(e1));
    order_kernels();
    if (pipe && iters > 0 && ((iters - 1) & 1)) {  // the last pass counted into set 1: it becomes set 0
      cn.swap(cn1);
      scn.swap(scn1);
      O.counts = (unsigned long long*)cn.p;
      if (mode & KV_MODE_SCOPES) O.scounts = (unsigned long long*)scn.p;
    }
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, e0, e1));
    if (stamps.p) report_stamps();
    return t;
  }
  // mean shader cycles per wave between consecutive stamps of the last rule kernel (segment k: from
  // stamp k - 1 to stamp k), and the mean wave lifetime
  void report_stamps() {
    std::vector<unsigned long long> h(stamps.n / sizeof(unsigned long long));
    HIPCHK(hipMemcpy(h.data(), stamps.p, stamps.n, hipMemcpyDeviceToHost));
    double seg[kJitStamps] = {}, life = 0;
    uint64_t n[kJitStamps] = {}, nl = 0;
    for (size_t w = 0; w + kJitStamps <= h.size(); w += kJitStamps) {
      const unsigned long long* x = &h[w];
      uint32_t last = 0;
      for (uint32_t k = 1; k < kJitStamps; k++)
        if (x[k] && x[last]) {
          seg[k] += (double)(x[k] - x[last]);
          n[k]++;
          last = k;
        }
      if (x[0] && x[last] && last) {
        life += (double)(x[last] - x[0]);
        nl++;
      }
    }
    fprintf(stderr, "[kvgpu] stamps: wave lifetime %.0f cycles;", nl ? life / nl : 0.0);
    for (uint32_t k = 1; k < kJitStamps; k++)
      if (n[k]) fprintf(stderr, " seg%u %.0f", k, seg[k] / n[k]);
    fprintf(stderr, "\n");
  }
  // one launch per rule kernel of the specialized kernels, 256 resources per workgroup
  // the per-pass tables of set b (match tables, factored match, value-predicate table) of a
  // pipelined pass, on `pside`, then their event
  void launch_tables(int b) {
    const DevPS* P = (const DevPS*)(b ? pview1.p : pview.p);
    DevBuf& c = b ? cn1 : cn;
    HIPCHK(hipMemsetAsync(c.p, 0, c.n, pside));
    if (mode & KV_MODE_SCOPES) {
      DevBuf& sc = b ? scn1 : scn;
      HIPCHK(hipMemsetAsync(sc.p, 0, sc.n, pside));
    }
    HIPCHK(launch_mtab(P, bview, mt_words, mt_entities, b ? mt1_ns : mt_ns, b ? mt1_ann : mt_ann, b ? mt1_sel : mt_sel,
                       pside));
    if (dps->mtup_words && ntup)
      HIPCHK(launch_mfac(P, bview, dps->fac_slots, fac_entities, dps->mtup_words, ntup,
                         (uint32_t*)(b ? mtup1.p : mtup.p), pside));
    if (dps->ptab_fn) {
      const Val* V = bhost->vals;
      const uint8_t* S = bhost->bstr;
      uint32_t NV = nvals;
      uint32_t* PT = (uint32_t*)(b ? ptab1.p : ptab.p);
      void* targs[] = {(void*)&P, (void*)&V, (void*)&S, (void*)&NV, (void*)&PT};
      HIPCHK(hipModuleLaunchKernel(dps->ptab_fn, (NV + KV_PTAB_PSEUDO + KV_WG - 1) / KV_WG, dps->ptab_rows, 1, KV_WG, 1, 1,
                                   0, pside, targs, nullptr));
    }
    HIPCHK(hipEventRecord(ev_pt[b], pside));
  }
  // pb: the pipelined table this pass reads (launch_ptab), -1: build the table here
  void launch_specialized(int pb = -1) {
    if (nres == 0) {  // (join the side stream's table work all the same)
      HIPCHK(hipEventRecord(ev_join, side));
      HIPCHK(hipStreamWaitEvent(stream, ev_join, 0));
      return;
    }
    const uint32_t blocks = (uint32_t)((nres + KV_RWG - 1) / KV_RWG);
    const DevPS* P = (const DevPS*)(pb == 1 ? pview1.p : pview.p);
    const Node* N = bhost->nodes;
    const Val* V = bhost->vals;
    const uint8_t* S = bhost->bstr;
    if (pb >= 0) {
      HIPCHK(hipStreamWaitEvent(stream, ev_pt[pb], 0));
    } else {
    if (dps->ptab_fn) {  // every leaf predicate once per distinct value (+ pseudo columns), before the rule kernels
      uint32_t NV = nvals;
      uint32_t* PT = (uint32_t*)ptab.p;
      void* targs[] = {(void*)&P, (void*)&V, (void*)&S, (void*)&NV, (void*)&PT};
      HIPCHK(hipModuleLaunchKernel(dps->ptab_fn, (NV + KV_PTAB_PSEUDO + KV_WG - 1) / KV_WG, dps->ptab_rows, 1, KV_WG, 1, 1, 0,
                                   stream, targs, nullptr));
    }
    if (dps->mtup_words && ntup)  // every rule's match bit per tuple (after kv_mtab, on the side stream)
      HIPCHK(launch_mfac(P, bview, dps->fac_slots, fac_entities, dps->mtup_words, ntup, (uint32_t*)mtup.p, side));
    HIPCHK(hipEventRecord(ev_join, side));
    HIPCHK(hipStreamWaitEvent(stream, ev_join, 0));
    }
    DevOut Ov = O;
    if (pb == 1) {  // counts of set 1
      Ov.counts = (unsigned long long*)cn1.p;
      if (mode & KV_MODE_SCOPES) Ov.scounts = (unsigned long long*)scn1.p;
    }
    uint32_t r0 = 0;
    void* args[] = {(void*)&P, (void*)&bview, (void*)&N, (void*)&V, (void*)&S, (void*)&Ov, (void*)&r0};
    // Rule kernels of a pass (they write disjoint rule rows): three or more are dealt round-robin
    // over `stream`, `side` and a third stream, forked from and joined back into `stream`, so a
    // kernel's last workgroups share the chip with the next kernels' first instead of draining it;
    // once a pass has timed them, they go longest first (and two kernels then go over two
    // streams: the short one fills the long one's tail). C3 (17 kernels), ms per pass on one box:
    // one stream 3.56, two 2.96-3.01, three 2.66-2.69, four 2.73-2.75 (a process has 4 hardware
    // queues; the pipeline stream takes one). C4 (2 kernels, 150 and 515 us): one stream 0.690,
    // two in plan order 0.713-0.714, two longest first 0.613-0.617.
    constexpr uint32_t kRuleStreams = 3;
    const std::vector<hipFunction_t>& fs = dps->fns_for(Ov.full);
    const uint32_t nk = (uint32_t)fs.size();
    if (korder.empty() && nk > 1) {
      std::lock_guard<std::mutex> g(dps->order_mu);
      if (dps->korder.size() == nk) korder = dps->korder;
    }
    const bool ordered = korder.size() == nk && nk > 1;
    const uint32_t ns = nk >= 3 ? std::min<uint32_t>(kRuleStreams, nk) : (ordered ? nk : 1u);
    // the first pass of a session with 2+ kernels times them (events around each launch)
    const bool timing = !ordered && nk > 1 && !ktiming;
    if (timing) {
      while (kev.size() < 2 * nk) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        kev.push_back(e);
      }
      ktiming = true;
    }
    while (rkx.size() + 2 < ns) rkx.push_back(StreamPool::get().take(device, hipStreamNonBlocking));
    hipStream_t sts[4] = {stream, side, rkx.size() > 0 ? rkx[0] : nullptr, rkx.size() > 1 ? rkx[1] : nullptr};
    if (ns > 1) {
      HIPCHK(hipEventRecord(ev_rkf, stream));
      for (uint32_t q = 1; q < ns; q++) HIPCHK(hipStreamWaitEvent(sts[q], ev_rkf, 0));
    }
    for (uint32_t k = 0; k < nk; k++) {
      const uint32_t f = ordered ? korder[k] : k;
      hipStream_t st = sts[k % ns];
      if (timing) HIPCHK(hipEventRecord(kev[2 * f], st));
      HIPCHK(hipModuleLaunchKernel(fs[f], blocks, 1, 1, KV_RWG, 1, 1, 0, st, args, nullptr));
      if (timing) HIPCHK(hipEventRecord(kev[2 * f + 1], st));
    }
    for (uint32_t q = 1; q < ns; q++) {
      HIPCHK(hipEventRecord(ev_rkj[q - 1], sts[q]));
      HIPCHK(hipStreamWaitEvent(stream, ev_rkj[q - 1], 0));
    }
  }
  // after a timed pass has completed: the rule kernels' launch order, longest first
  void order_kernels() {
    if (!ktiming || !korder.empty()) return;
    const uint32_t nk = (uint32_t)(kev.size() / 2);
    std::vector<std::pair<float, uint32_t>> d(nk);
    for (uint32_t k = 0; k < nk; k++) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, kev[2 * k], kev[2 * k + 1]) != hipSuccess) {
        (void)hipGetLastError();
        return;  // (not timed in this run: keep the plan order)
      }
      d[k] = {ms, k};
    }
    std::stable_sort(d.begin(), d.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    for (const auto& x : d) korder.push_back(x.second);
    std::lock_guard<std::mutex> g(dps->order_mu);
    if (dps->korder.empty()) dps->korder = korder;
  }
  // status-matrix bytes the last pass wrote: the (rule, workgroup) segments whose flag it set (a
  // segment left unwritten is all NOMATCH and filled at fetch), or the whole matrix without flags
  uint64_t written_status_bytes() {
    if (!O.status) return 0;
    if (!O.sflag || !dps->specialized()) return nrules * nres;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamSynchronize(stream));
    std::vector<uint8_t> f(sflag.n);
    if (!f.empty()) HIPCHK(hipMemcpy(f.data(), sflag.p, f.size(), hipMemcpyDeviceToHost));
    const uint64_t nwg = (nres + KV_RWG - 1) / KV_RWG, last = nres - (nwg - 1) * KV_RWG;
    uint64_t bytes = 0;
    for (uint64_t i = 0; i < nrules * nwg && i < f.size(); i++)
      if (f[i]) bytes += (i % nwg == nwg - 1) ? last : KV_RWG;
    return bytes;
  }
  std::vector<int64_t> read_counts() {
    HIPCHK(hipSetDevice(device));
    std::vector<unsigned long long> c(nrules * KV_HIST);
    if (!c.empty()) HIPCHK(hipMemcpy(c.data(), cn.p, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return std::vector<int64_t>(c.begin(), c.end());
  }
  std::vector<int64_t> read_scope_counts() {
    HIPCHK(hipSetDevice(device));
    std::vector<unsigned long long> c((size_t)nscopes * nrules * KV_HIST);
    if (!c.empty()) HIPCHK(hipMemcpy(c.data(), scn.p, c.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return std::vector<int64_t>(c.begin(), c.end());
  }
  // statuses into rows [rule][lo, lo + nres) of the result's [rule][n_total] matrix, and
  // the compacted error records of this shard
  void fetch(kv_result* out, ResultPart* part, uint64_t lo, uint64_t n_total) {
    HIPCHK(hipSetDevice(device));
    const bool verbose = getenv("KVGPU_VERBOSE") != nullptr;
    auto tl = std::chrono::steady_clock::now();
    // phase boundary: the stream drained, the time since the last one into the result's phases
    // (the first part's, so parts on several devices do not add up)
    auto lap = [&](const char* what) {
      HIPCHK(hipStreamSynchronize(stream));
      const auto now = std::chrono::steady_clock::now();
      const double ms = std::chrono::duration<double, std::milli>(now - tl).count();
      tl = now;
      if (part == &out->parts[0]) out->phases.push_back({what, ms});
      if (verbose) fprintf(stderr, "[kvgpu] fetch: %s %.1f ms\n", what, ms);
    };
    const bool want_st = O.status && (mode & (KV_MODE_STATUS | KV_MODE_ERRORS)) && nres && nrules;
    bool side_copy = false;
    uint64_t spack_bytes = 0;
    // A permuted batch fetched whole comes back in the caller's order: the statuses are gathered on
    // the device (stc[rule][j] = st[rule][store index of j]) and the records scattered to the
    // caller's (rule, resource) order, so one status matrix crosses PCIe and the host permutes
    // nothing. Its copy runs on the side stream, beside the record kernels.
    // Specialized passes: the statuses cross in the transfer form (the segments the pass wrote, 4
    // bits a status; C3: 0.48 GB for a 2.47 GB matrix) and the host materialises the matrix when an
    // accessor reads it; records then stay in store order
    const bool packed = want_st && out->sparse;
    if (packed) {
      const uint64_t nwg = (nres + KV_RWG - 1) / KV_RWG, nch = (nwg + KV_WG - 1) / KV_WG;
      if (s_ccnt.n < nrules * nch * sizeof(uint32_t)) {
        s_ccnt.alloc(nrules * nch * sizeof(uint32_t), device);
        s_cbase.alloc(nrules * nch * sizeof(unsigned long long), device);
      }
      HIPCHK(launch_status_pack(O.status, O.sflag, (uint32_t)nres, (uint32_t)nrules, nullptr, (uint32_t*)s_ccnt.p,
                                nullptr, stream));
      std::vector<uint32_t> cc(nrules * nch);
      std::vector<unsigned long long> cb(nrules * nch);
      HIPCHK(hipMemcpyAsync(cc.data(), s_ccnt.p, cc.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
      part->nwg = nwg;
      part->sbase.resize(nrules);
      unsigned long long t = 0;
      for (size_t i = 0; i < cc.size(); i++) {
        if (i % nch == 0) part->sbase[i / nch] = t;
        cb[i] = t;
        t += cc[i];
      }
      const uint64_t bytes = t * (KV_RWG / 2);
      if (s_pack.n < std::max<uint64_t>(bytes, 1)) s_pack.alloc(std::max<uint64_t>(bytes, 1), device);
      HIPCHK(hipMemcpyAsync(s_cbase.p, cb.data(), cb.size() * sizeof(unsigned long long), hipMemcpyHostToDevice, stream));
      HIPCHK(launch_status_pack(O.status, O.sflag, (uint32_t)nres, (uint32_t)nrules,
                                (const unsigned long long*)s_cbase.p, nullptr, (uint8_t*)s_pack.p, stream));
      part->sflag.alloc(nrules * nwg);
      part->spack.alloc(bytes);
      // copied after the records: the record steps' small copies (offsets, flags, code tables)
      // would otherwise queue behind these bytes on the copy engines at every host round trip
      spack_bytes = bytes;
      lap("status_pack");
    }
    bool caller = !packed && want_st && bt && lo == 0 && nres == n_total && !bt->b.order.empty();
    if (caller && !stc.p) {  // the gathered copy is a second status matrix: only with room to spare
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) != hipSuccess) caller = false;
      fr += DevPool::get().held_on(device);  // (kept buffers are freed when an allocation needs them)
      if (fr < nrules * nres + nres * 8u + (512ull << 20)) caller = false;
    }
    if (caller) {
      if (!inv_d.p) inv_d.upload_raw(bt->inverse(), nres * sizeof(uint32_t), device);
      if (!stc.p) stc.alloc(nrules * nres, device);
      HIPCHK(launch_gather_rows((const uint8_t*)st.p, (const uint32_t*)inv_d.p, nrules, nres, (uint8_t*)stc.p, stream));
      HIPCHK(hipEventRecord(ev_fork, stream));
      HIPCHK(hipStreamWaitEvent(side, ev_fork, 0));
      HIPCHK(hipMemcpyAsync(out->status.data(), stc.p, nrules * nres, hipMemcpyDeviceToHost, side));
      side_copy = true;
      out->caller_order = true;
      lap("status_gather");
    } else if (want_st && !packed) {
      HIPCHK(hipMemcpy2DAsync(out->status.data() + lo, n_total, st.p, nres, nres, nrules, hipMemcpyDeviceToHost,
                              stream));
      lap("status_d2h");
    }
    if (O.err8 && nres && nrules) {
      const uint32_t tiles = (uint32_t)((nres + KV_WG - 1) / KV_WG);
      part->tiles = tiles;
      if (!r_offs.p) {
        r_offs.alloc((size_t)nrules * tiles * sizeof(uint32_t), device);
        r_tot.alloc(nrules * sizeof(unsigned long long), device);
        r_base.alloc((nrules + 1) * sizeof(unsigned long long), device);
        r_wide.alloc(sizeof(uint32_t), device);
      }
      const uint32_t* ord = nullptr;
      unsigned long long* masks = nullptr;
      if (caller) {  // record ranks over the caller-order statuses
        if (!ord_d.p) ord_d.upload_raw(bt->b.order.data(), nres * sizeof(uint32_t), device);
        if (!r_mask.p) r_mask.alloc((size_t)nrules * tiles * (KV_WG / 64) * sizeof(unsigned long long), device);
        ord = (const uint32_t*)ord_d.p;
        masks = (unsigned long long*)r_mask.p;
      }
      const uint8_t* rank_st = caller ? (const uint8_t*)stc.p : O.status;
      // a specialized pass's unwritten segments hold no records: the record kernels skip them
      // (their statuses are neither filled nor read)
      const uint8_t* seg_flags = rec_compact && !caller ? O.sflag : nullptr;
      HIPCHK(launch_rec_compact(rank_st, O.err8, nullptr, (uint32_t)nres, (uint32_t)nrules, (uint32_t*)r_offs.p,
                                (unsigned long long*)r_tot.p, (unsigned long long*)r_base.p, nullptr, nullptr, nullptr,
                                0, rec_compact ? (const uint8_t*)dps->rcompact.p : nullptr, nullptr, masks, seg_flags,
                                stream));
      // the fetch's small device-to-host copies go through one page-locked staging block (a copy
      // into pageable memory is staged by the runtime and waited for behind the DMA queue)
      const size_t tb = (size_t)nrules * KV_REC_CODES, sb = ((nrules + 1) * 8 + 63) & ~(size_t)63;
      if (hstage.size() < sb + nrules * 4 + 64 + tb * 8) hstage.alloc(sb + nrules * 4 + 64 + tb * 8);
      part->base.resize(nrules + 1);
      part->offs.alloc((size_t)nrules * tiles);
      HIPCHK(hipMemcpyAsync(hstage.data(), r_base.p, part->base.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(part->offs.data(), r_offs.p, part->offs.size() * sizeof(uint32_t), hipMemcpyDeviceToHost,
                            stream));
      lap("records_count");
      memcpy(part->base.data(), hstage.data(), part->base.size() * sizeof(uint64_t));
      const uint64_t total = part->base[nrules];
      if (r_out8.n < total * sizeof(ErrRec8)) {
        r_out8.alloc(std::max<uint64_t>(total, 1) * sizeof(ErrRec8), device);
        lap("records_alloc");
      }
      HIPCHK(hipMemsetAsync(r_wide.p, 0, sizeof(uint32_t), stream));
      if (rec_compact && O.gsite) {  // the groups' site records to their members' slots
        HIPCHK(launch_gsite_expand(O.gsite, O.gcnt, (const GSiteDesc*)dps->gsdesc.p, (const uint32_t*)dps->gsmem.p,
                                   dps->gs_groups, (uint32_t)nres, O.err8, stream));
        lap("records_expand");
      }
      HIPCHK(launch_rec_compact(O.status, O.err8, nullptr, (uint32_t)nres, (uint32_t)nrules, (uint32_t*)r_offs.p,
                                nullptr, (unsigned long long*)r_base.p, (ErrRec8*)r_out8.p, nullptr,
                                (uint32_t*)r_wide.p, 1, rec_compact ? (const uint8_t*)dps->rcompact.p : nullptr, ord,
                                masks, seg_flags, stream));
      HIPCHK(hipMemcpyAsync(hstage.data() + sb, r_wide.p, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      lap("records_scatter");
      uint32_t wide = 0;
      memcpy(&wide, hstage.data() + sb, sizeof(uint32_t));
      // Record codes: a rule's records cross PCIe as 1-byte codes into a table of its distinct
      // records (C2: 206 MB of 8-byte records -> 26 MB of codes, C3: 3.6 GB -> 0.45 GB); skipped
      // when some record is wide (the full records of the re-run below are kept parallel to every
      // compact record)
      const ErrRec8* src = (const ErrRec8*)r_out8.p;
      uint64_t keep = total;
      bool coded = false;
      part->raw.clear();
      if (!wide && total && nrules) {
        if (r_tkey.n < tb * sizeof(unsigned long long)) {
          r_tkey.alloc(tb * sizeof(unsigned long long), device);
          r_raw.alloc(nrules * sizeof(uint32_t), device);
          r_nbase.alloc(nrules * sizeof(unsigned long long), device);
        }
        if (r_code.n < total) r_code.alloc(total, device);
        HIPCHK(hipMemsetAsync(r_tkey.p, 0xFF, tb * sizeof(unsigned long long), stream));
        HIPCHK(hipMemsetAsync(r_raw.p, 0, nrules * sizeof(uint32_t), stream));
        HIPCHK(launch_rec_codes((const ErrRec8*)r_out8.p, (const unsigned long long*)r_base.p, (uint32_t)nrules,
                                (unsigned long long*)r_tkey.p, (uint8_t*)r_code.p, (uint32_t*)r_raw.p, nullptr, nullptr,
                                0, stream));
        const uint32_t* rawf = (const uint32_t*)hstage.data();
        const unsigned long long* keys = (const unsigned long long*)(hstage.data() + ((nrules * 4 + 63) & ~(size_t)63));
        HIPCHK(hipMemcpyAsync((void*)rawf, r_raw.p, nrules * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIPCHK(hipMemcpyAsync((void*)keys, r_tkey.p, tb * sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        part->raw.assign(nrules, 0);
        part->nbase.assign(nrules, 0);
        part->tab.assign(tb, ErrRec8{0u, 0u});
        keep = 0;
        for (uint64_t q = 0; q < nrules; q++) {
          part->raw[q] = rawf[q] ? 1 : 0;
          part->nbase[q] = keep;
          if (rawf[q]) keep += part->base[q + 1] - part->base[q];
        }
        for (size_t t = 0; t < tb; t++)
          if (keys[t] != ~0ull) part->tab[t] = ErrRec8{(uint32_t)(keys[t] >> 32), (uint32_t)keys[t]};
        if (keep) {
          if (r_out8b.n < keep * sizeof(ErrRec8)) r_out8b.alloc(keep * sizeof(ErrRec8), device);
          HIPCHK(hipMemcpyAsync(r_nbase.p, part->nbase.data(), nrules * sizeof(unsigned long long),
                                hipMemcpyHostToDevice, stream));
          HIPCHK(launch_rec_codes((const ErrRec8*)r_out8.p, (const unsigned long long*)r_base.p, (uint32_t)nrules,
                                  nullptr, nullptr, (uint32_t*)r_raw.p, (const unsigned long long*)r_nbase.p,
                                  (ErrRec8*)r_out8b.p, 1, stream));
          src = (const ErrRec8*)r_out8b.p;
        }
        coded = true;
        lap("records_code");
      }
      const auto th0 = std::chrono::steady_clock::now();
      part->rec.alloc(keep);
      if (part == &out->parts[0])
        out->phases.push_back(
            {"host_alloc", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count()});
      if (coded) part->code.alloc(total);
      tl = std::chrono::steady_clock::now();
      if (keep) HIPCHK(hipMemcpyAsync(part->rec.data(), src, keep * sizeof(ErrRec8), hipMemcpyDeviceToHost, stream));
      if (coded) HIPCHK(hipMemcpyAsync(part->code.data(), r_code.p, total, hipMemcpyDeviceToHost, stream));
      lap("records_d2h");
      if (wide) {  // re-run the pass once writing full records (same statuses), compact those too
        if (!er.p) er.alloc(nrules * nres * sizeof(ErrRec), device);
        O.err = (ErrRec*)er.p;
        O.full |= 4;
        run(1, true);
        O.full &= ~4u;
        if (r_outw.n < total * sizeof(ErrRec)) r_outw.alloc(std::max<uint64_t>(total, 1) * sizeof(ErrRec), device);
        HIPCHK(launch_rec_compact(O.status, O.err8, O.err, (uint32_t)nres, (uint32_t)nrules, (uint32_t*)r_offs.p,
                                  nullptr, (unsigned long long*)r_base.p, (ErrRec8*)r_out8.p, (ErrRec*)r_outw.p,
                                  (uint32_t*)r_wide.p, 1, nullptr, ord, masks, nullptr, stream));
        part->recw.alloc(total);
        HIPCHK(hipMemcpyAsync(part->recw.data(), r_outw.p, total * sizeof(ErrRec), hipMemcpyDeviceToHost, stream));
        lap("records_wide_rerun");
      }
    }
    if (packed) {  // the statuses' transfer form (kv_status_pack_kernel above; the re-run leaves it)
      HIPCHK(hipMemcpyAsync(part->sflag.data(), O.sflag, part->sflag.size(), hipMemcpyDeviceToHost, stream));
      if (spack_bytes) HIPCHK(hipMemcpyAsync(part->spack.data(), s_pack.p, spack_bytes, hipMemcpyDeviceToHost, stream));
      lap("status_d2h");
    }
    HIPCHK(hipStreamSynchronize(stream));
    if (side_copy) {
      HIPCHK(hipStreamSynchronize(side));
      lap("status_d2h_wait");
    }
  }
};

// Sessions on the devices of a mask: contiguous resource shards, one host thread
// + HIP stream per part, policy set replicated, per-rule (and per-scope) counts
// summed over the parts by one RCCL all-reduce (distinct devices) when read.
struct SessionSet {
  kv_policyset* ps = nullptr;
  kv_batch* bt = nullptr;
  uint32_t mode = 0;
  uint64_t nrules = 0, nres = 0;
  std::vector<std::shared_ptr<kv_batch>> shards;           // empty: one part over the whole batch
  std::vector<std::pair<uint64_t, uint64_t>> ranges;       // resource range of each part
  std::vector<std::unique_ptr<DevSession>> parts;
  std::vector<ncclComm_t> comms;                           // one per part (distinct devices only)
  bool reduced = false;
  std::vector<int64_t> counts_, scope_counts_;
  std::vector<double> part_ms;                             // HIP-event ms of each part's last run
  // parts session (kv_session_create_parts): one caller batch per part, attached one by one;
  // scopes = the sorted union of the parts' namespaces, set when the last part is attached
  bool parts_mode = false, finalized = true;
  std::string ctx;
  std::vector<int> devs;
  std::vector<std::vector<std::string>> part_ns;
  std::vector<std::string> scope_names;

  // parts session: n empty parts (kv_session_attach_part fills them)
  SessionSet(kv_policyset* p, const char* ctx_json, uint32_t m, uint32_t n)
      : ps(p), mode(m), parts_mode(true), finalized(false), ctx(ctx_json ? ctx_json : "") {
    nrules = ps->ps.rules.size();
    parts.resize(n);
    ranges.assign(n, {0, 0});
    devs.assign(n, -1);
    part_ns.resize(n);
  }
  // part k = batch b on device d: uploaded, its device copy detached from the caller's batch
  void attach(uint32_t k, kv_batch* b, int d) {
    if (!parts_mode || finalized) throw std::runtime_error("not an open parts session");
    if (k >= parts.size()) throw std::runtime_error("part index out of range");
    if (parts[k]) throw std::runtime_error("part already attached");
    auto ds = std::make_unique<DevSession>(ps, b, ctx.empty() ? nullptr : ctx.c_str(), d, mode);
    part_ns[k] = b->b.namespaces;
    ds->detach_batch();
    parts[k] = std::move(ds);
    devs[k] = d;
    for (auto& q : parts)
      if (!q) return;
    finalize();
  }
  void finalize() {
    uint64_t at = 0;
    for (size_t k = 0; k < parts.size(); k++) {
      ranges[k] = {at, at + parts[k]->nres};
      at += parts[k]->nres;
    }
    nres = at;
    std::vector<std::string> all;
    for (auto& v : part_ns) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    scope_names = all;
    for (size_t k = 0; k < parts.size(); k++) {
      std::vector<uint32_t> map(part_ns[k].size());
      for (size_t i = 0; i < map.size(); i++)
        map[i] = (uint32_t)(std::lower_bound(all.begin(), all.end(), part_ns[k][i]) - all.begin());
      parts[k]->remap_scopes(map, (uint32_t)all.size());
    }
    init_comms(devs);
    finalized = true;
  }
  void init_comms(const std::vector<int>& devices) {
    std::vector<int> uniq(devices);
    std::sort(uniq.begin(), uniq.end());
    if (devices.size() > 1 && std::unique(uniq.begin(), uniq.end()) == uniq.end()) {  // one rank per device
      comms.resize(devices.size());
      if (ncclCommInitAll(comms.data(), (int)devices.size(), devices.data()) != ncclSuccess) {
        comms.clear();
        throw HipError("ncclCommInitAll failed");
      }
    }
  }
  void check_ready() const {
    if (!finalized) throw std::runtime_error("parts session: not every part is attached");
  }
  int rccl_ranks() const {
    if (comms.empty()) return 0;
    int n = 0;
    if (ncclCommCount(comms[0], &n) != ncclSuccess) return -1;
    return n;
  }

  SessionSet(kv_policyset* p, kv_batch* b, const char* ctx_json, const std::vector<int>& devices, uint32_t m)
      : ps(p), bt(b), mode(m) {
    nrules = ps->ps.rules.size();
    nres = bt->b.res.size();
    if (devices.size() == 1) {
      ranges.push_back({0, nres});
      parts.push_back(std::make_unique<DevSession>(ps, bt, ctx_json, devices[0], mode));
      // KVGPU_RCCL_ALWAYS=1: reduce through a one-rank communicator too (exercises RCCL on one GPU)
      if (getenv("KVGPU_RCCL_ALWAYS") && getenv("KVGPU_RCCL_ALWAYS")[0] == '1') {
        comms.resize(1);
        if (ncclCommInitAll(comms.data(), 1, devices.data()) != ncclSuccess) {
          comms.clear();
          throw HipError("ncclCommInitAll failed");
        }
      }
      return;
    }
    ranges = shard_ranges(nres, (uint32_t)devices.size());
    shards.resize(devices.size());
    std::vector<std::thread> th;
    std::vector<std::string> errs(devices.size());
    for (size_t k = 0; k < devices.size(); k++)
      th.emplace_back([&, k]() {
        try {
          auto sb = std::make_shared<kv_batch>();
          sb->owner = ps;
          make_shard(bt->b, ranges[k].first, ranges[k].second, &sb->b);
          shards[k] = sb;
        } catch (const std::exception& e) {
          errs[k] = e.what();
        }
      });
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (!e.empty()) throw std::runtime_error(e);
    parts.resize(devices.size());
    th.clear();
    for (size_t k = 0; k < devices.size(); k++)
      th.emplace_back([&, k]() {
        try {
          parts[k] = std::make_unique<DevSession>(ps, shards[k].get(), ctx_json, devices[k], mode);
        } catch (const std::exception& e) {
          errs[k] = e.what();
        }
      });
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (!e.empty()) throw HipError(e);
    init_comms(devices);  // RCCL needs one rank per device
  }
  ~SessionSet() {
    for (ncclComm_t c : comms) (void)ncclCommDestroy(c);
  }
  template <class F>
  void each(F f) {
    if (parts.size() == 1) {
      f(0);
      return;
    }
    std::vector<std::thread> th;
    std::vector<std::string> errs(parts.size());
    for (size_t k = 0; k < parts.size(); k++)
      th.emplace_back([&, k]() {
        try {
          f(k);
        } catch (const std::exception& e) {
          errs[k] = e.what();
        }
      });
    for (auto& t : th) t.join();
    for (auto& e : errs)
      if (!e.empty()) throw HipError(e);
  }
  // `iters` passes on every part concurrently; the slowest part's HIP-event time
  double run(int iters) {
    check_ready();
    std::vector<double> ms(parts.size(), 0.0);
    each([&](size_t k) { ms[k] = parts[k]->run(iters); });
    reduced = false;
    part_ms = ms;
    return *std::max_element(ms.begin(), ms.end());
  }
  // a failed collective leaves ranks waiting: abort every communicator, never reuse them
  [[noreturn]] void abort_comms(const std::string& what) {
    for (ncclComm_t c : comms) (void)ncclCommAbort(c);
    comms.clear();
    comms_failed = true;
    throw HipError(what);
  }
  bool comms_failed = false;
  // counts of the last pass summed over the parts: RCCL all-reduce (ncclUint64, sum)
  // of the device count arrays across distinct devices, else a host sum
  void reduce() {
    check_ready();
    if (comms_failed) throw HipError("RCCL communicators were aborted after a failed all-reduce");
    if (reduced) return;
    counts_.assign(nrules * KV_HIST, 0);
    scope_counts_.clear();
    const bool scopes = (mode & KV_MODE_SCOPES) != 0;
    if (!comms.empty()) {
      if (ncclGroupStart() != ncclSuccess) abort_comms("ncclGroupStart failed");
      ncclResult_t enq = ncclSuccess;  // first failed enqueue; the group is still closed below
      for (size_t k = 0; k < parts.size() && enq == ncclSuccess; k++) {
        DevSession& d = *parts[k];
        HIPCHK(hipSetDevice(d.device));
        enq = ncclAllReduce(d.cn.p, d.cn.p, nrules * KV_HIST, ncclUint64, ncclSum, comms[k], d.stream);
        if (scopes && enq == ncclSuccess)
          enq = ncclAllReduce(d.scn.p, d.scn.p, (size_t)d.nscopes * nrules * KV_HIST, ncclUint64, ncclSum, comms[k],
                              d.stream);
      }
      const ncclResult_t end = ncclGroupEnd();
      if (enq != ncclSuccess) abort_comms(std::string("ncclAllReduce failed: ") + ncclGetErrorString(enq));
      if (end != ncclSuccess) abort_comms(std::string("RCCL all-reduce failed: ") + ncclGetErrorString(end));
      for (auto& d : parts) {
        HIPCHK(hipSetDevice(d->device));
        if (hipStreamSynchronize(d->stream) != hipSuccess) abort_comms("RCCL all-reduce: stream synchronize failed");
      }
      counts_ = parts[0]->read_counts();
      if (scopes) scope_counts_ = parts[0]->read_scope_counts();
    } else {
      for (auto& d : parts) {
        std::vector<int64_t> c = d->read_counts();
        for (size_t i = 0; i < c.size(); i++) counts_[i] += c[i];
        if (scopes) {
          std::vector<int64_t> sc = d->read_scope_counts();
          if (scope_counts_.empty()) scope_counts_.assign(sc.size(), 0);
          for (size_t i = 0; i < sc.size(); i++) scope_counts_[i] += sc[i];
        }
      }
    }
    reduced = true;
  }
  void fetch(kv_result* out, double ms) {
    if (parts_mode) throw std::runtime_error("kv_session_fetch: a parts session keeps no host batch");
    out->ps = ps;
    out->b = bt;
    out->n_rules = nrules;
    out->n_res = nres;
    out->mode = mode;
    out->kernel_ms = ms;
    reduce();
    out->counts = counts_;
    if (mode & KV_MODE_SCOPES) out->scope_counts = scope_counts_;
    out->sparse = parts[0]->O.status && parts[0]->O.sflag && (mode & (KV_MODE_STATUS | KV_MODE_ERRORS)) && nres &&
                  nrules && std::all_of(parts.begin(), parts.end(), [](const auto& p) { return p->rec_compact; });
    if (parts[0]->O.status && (mode & (KV_MODE_STATUS | KV_MODE_ERRORS)) && !out->sparse) {
      HIPCHK(hipSetDevice(parts[0]->device));
      const auto ta = std::chrono::steady_clock::now();
      out->status.alloc(nrules * nres);
      out->phases.push_back(
          {"host_alloc", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count()});
    }
    out->errors = (mode & KV_MODE_ERRORS) != 0;
    out->parts.resize(parts.size());
    for (size_t k = 0; k < parts.size(); k++) {
      out->parts[k].lo = ranges[k].first;
      out->parts[k].n = ranges[k].second - ranges[k].first;
      if (!shards.empty()) out->parts[k].shard = shards[k];
    }
    each([&](size_t k) { parts[k]->fetch(out, &out->parts[k], ranges[k].first, nres); });
  }
};

// devices of a mask, each repeated KVGPU_SHARDS_PER_DEVICE times (logical shards: the
// multi-device path on one GPU, for tests; counts are then summed on the host)
std::vector<int> mask_devices(uint32_t mask) {
  std::vector<int> d;
  int per = 1;
  if (const char* e = getenv("KVGPU_SHARDS_PER_DEVICE")) per = std::max(1, atoi(e));
  for (int i = 0; i < 32; i++)
    if (mask & (1u << i))
      for (int k = 0; k < per; k++) d.push_back(i);
  return d;
}

void run(kv_policyset* ps, kv_batch* bt, const char* ctx_json, const std::vector<int>& devices, uint32_t mode,
         kv_result* out, int warmup, int iters, double* ms) {
  if (devices.empty()) throw std::runtime_error("empty device mask");
  const auto t0 = std::chrono::steady_clock::now();
  SessionSet s(ps, bt, ctx_json, devices, mode);
  const auto t1 = std::chrono::steady_clock::now();
  if (warmup > 0) s.run(warmup);
  int n = std::max(iters, 1);
  double t = s.run(n) / n;
  const auto t2 = std::chrono::steady_clock::now();
  if (ms) *ms = t;
  if (out) {
    auto d = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const double up = s.parts.empty() ? 0.0 : s.parts[0]->upload_ms;
    out->phases = {{"upload", up}, {"setup", d(t0, t1) - up}, {"pass", d(t1, t2)}};
    s.fetch(out, t);
  }
  if (getenv("KVGPU_VERBOSE")) {  // host-boundary breakdown
    const auto t3 = std::chrono::steady_clock::now();
    auto d = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "[kvgpu] kv_validate: setup+upload %.1f ms, passes %.1f ms, fetch %.1f ms\n", d(t0, t1), d(t1, t2),
            d(t2, t3));
  }
}

}  // namespace

struct kv_session {
  SessionSet set;
  kv_session(kv_policyset* p, kv_batch* b, const char* ctx_json, const std::vector<int>& devices, uint32_t m)
      : set(p, b, ctx_json, devices, m) {}
  kv_session(kv_policyset* p, const char* ctx_json, uint32_t m, uint32_t n) : set(p, ctx_json, m, n) {}
};

extern "C" {

int kv_compile(const char* policies_json, size_t len, uint32_t flags, kv_policyset** out, kv_error** err) {
  if (!policies_json || !out) return fail(err, KV_E_INVALID, "null argument");
  try {
    auto* s = new kv_policyset();
    try {
      compile_policies(policies_json, len, &s->ps);
      if (flags & KV_COMPILE_SPECIALIZE) {
        s->jit = std::make_unique<JitImage>();
        const uint32_t chunk = jit_chunk_rules();
        jit_generate(s->ps, chunk, s->jit.get());
        if (const char* dump = getenv("KVGPU_JIT_DUMP")) {
          if (FILE* f = fopen(dump, "w")) {
            fwrite(s->jit->source.data(), 1, s->jit->source.size(), f);
            fclose(f);
          }
        }
        if (!getenv("KVGPU_JIT_SKIP_COMPILE")) {  // (dump-only analysis runs skip it)
          const std::string pkey = jit_plan_key(*s->jit);
          const bool cached_plan = jit_load_plan(pkey, s->jit.get());
          if (!cached_plan) jit_refine_blocks(s->ps, chunk, s->jit.get());  // block sizes from probe compiles
          double ms = s->jit->compile_ms;
          jit_generate(s->ps, chunk, s->jit.get());
          // register budget: re-plan kernels that spill until the compiled plan is the final one
          // (the codes must belong to the last generated image: a plan still changing when the
          // rounds run out is an error, never shipped nor cached)
          bool settled = false;
          for (int round = 0; round < 64 && !settled; round++) {
            jit_compile(s->jit.get());
            ms += s->jit->compile_ms;
            settled = !jit_plan_spills(s->jit.get());
            if (!settled) jit_generate(s->ps, chunk, s->jit.get());
          }
          if (!settled)
            throw std::runtime_error("kvjit: the register plan did not settle (kernels still spill after 64 re-plans)");
          const double c0 = s->jit->compile_ms;
          jit_compile_variants(s->jit.get());  // (output-mode variants of the final kernels)
          ms += s->jit->compile_ms - c0;
          s->jit->compile_ms = ms;
          jit_save_plan(pkey, *s->jit);
          if (const char* dump = getenv("KVGPU_JIT_DUMP")) {  // (the source of the final plan)
            if (FILE* f = fopen(dump, "w")) {
              fwrite(s->jit->source.data(), 1, s->jit->source.size(), f);
              fclose(f);
            }
          }
        }
        if (const char* dump = getenv("KVGPU_JIT_DUMP_CO")) {  // gfx950 code objects (llvm-objdump / readelf)
          for (size_t i = 0; i < s->jit->codes.size(); i++) {
            if (FILE* f = fopen((std::string(dump) + "." + s->jit->kernel_name[i] + ".co").c_str(), "wb")) {
              fwrite(s->jit->codes[i].data(), 1, s->jit->codes[i].size(), f);
              fclose(f);
            }
          }
          for (const JitImage::Variant& v : s->jit->variants)  // (output-mode variants: <name>.m<full>)
            for (size_t i = 0; i < v.codes.size(); i++) {
              if (v.codes[i].empty()) continue;
              const std::string fn = std::string(dump) + "." + s->jit->kernel_name[i] + ".m" + std::to_string(v.full) + ".co";
              if (FILE* f = fopen(fn.c_str(), "wb")) {
                fwrite(v.codes[i].data(), 1, v.codes[i].size(), f);
                fclose(f);
              }
            }
        }
      }
    } catch (...) {
      delete s;
      throw;
    }
    *out = s;
    return 0;
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_policyset_info(const kv_policyset* ps, uint32_t* n_policies, uint32_t* n_rules) {
  if (!ps) return KV_E_INVALID;
  if (n_policies) *n_policies = (uint32_t)ps->ps.policy_names.size();
  if (n_rules) *n_rules = (uint32_t)ps->ps.rules.size();
  return 0;
}

int kv_policyset_jit_info(const kv_policyset* ps, uint32_t* n_kernels, double* gen_ms, double* compile_ms,
                          uint64_t* code_bytes) {
  if (!ps) return KV_E_INVALID;
  const JitImage* j = ps->jit.get();
  if (n_kernels) *n_kernels = j ? (uint32_t)j->chunks.size() : 0;
  if (gen_ms) *gen_ms = j ? j->gen_ms : 0;
  if (compile_ms) *compile_ms = j ? j->compile_ms : 0;
  if (code_bytes) *code_bytes = j ? kvh::code_bytes(*j) : 0;
  return 0;
}

int kv_rule_info_get(const kv_policyset* ps, uint32_t rule, kv_rule_info* out) {
  if (!ps || !out) return KV_E_INVALID;
  if (rule >= ps->ps.rules.size()) return KV_E_RANGE;
  const RuleHost& rh = ps->ps.rhost[rule];
  const RuleRec& rr = ps->ps.rules[rule];
  out->policy = rh.policy;
  out->policy_name = ps->ps.policy_names[rh.policy].c_str();
  out->name = rh.name.c_str();
  out->route = rr.route;
  out->route_reason = rh.route_reason.c_str();
  out->message = rh.message.c_str();
  out->any_pattern = rh.anypattern ? 1 : 0;
  out->const_status = rr.const_status;
  out->const_message = rh.const_message.c_str();
  return 0;
}

int kv_ingest(const kv_policyset* ps, const char* resources_json, size_t len, const char* ns_labels_json, kv_batch** out,
              kv_error** err) {
  if (!ps || !resources_json || !out) return fail(err, KV_E_INVALID, "null argument");
  try {
    auto* b = new kv_batch();
    b->owner = ps;
    try {
      ingest_resources(ps->ps, resources_json, len, ns_labels_json, &b->b);
    } catch (...) {
      delete b;
      throw;
    }
    if (getenv("KVGPU_VERBOSE"))
      fprintf(stderr, "[kvgpu] ingest: %zu resources, %zu cells, %zu vals, %zu string bytes\n", b->b.res.size(),
              (size_t)b->b.cells_used, b->b.vals.size(), b->b.strs.size());
    *out = b;
    return 0;
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_batch_info(const kv_batch* b, uint64_t* n_res, uint64_t* store_bytes) {
  if (!b) return KV_E_INVALID;
  if (n_res) *n_res = b->b.res.size();
  if (store_bytes) *store_bytes = b->b.bytes_referenced;
  return 0;
}

int kv_batch_transfer_bytes(const kv_batch* b, uint64_t* bytes) {
  if (!b || !bytes) return KV_E_INVALID;
  *bytes = b->b.transfer_bytes();
  return 0;
}

int kv_validate(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, int device, uint32_t mode,
                kv_result** out, kv_error** err) {
  if (!ps || !b || !out) return fail(err, KV_E_INVALID, "null argument");
  if (b->owner != ps) return fail(err, KV_E_INVALID, "batch was ingested for a different policy set");
  try {
    auto* r = new kv_result();
    try {
      run(const_cast<kv_policyset*>(ps), const_cast<kv_batch*>(b), ctx_json, {device}, mode, r, 0, 1, nullptr);
    } catch (...) {
      delete r;
      throw;
    }
    *out = r;
    return 0;
  } catch (const HipError& e) {
    return fail(err, KV_E_DEVICE, e.what());
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_validate_devices(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, uint32_t device_mask,
                        uint32_t mode, kv_result** out, kv_error** err) {
  if (!ps || !b || !out) return fail(err, KV_E_INVALID, "null argument");
  if (b->owner != ps) return fail(err, KV_E_INVALID, "batch was ingested for a different policy set");
  try {
    auto* r = new kv_result();
    try {
      run(const_cast<kv_policyset*>(ps), const_cast<kv_batch*>(b), ctx_json, mask_devices(device_mask), mode, r, 0, 1,
          nullptr);
    } catch (...) {
      delete r;
      throw;
    }
    *out = r;
    return 0;
  } catch (const HipError& e) {
    return fail(err, KV_E_DEVICE, e.what());
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_bench(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, int device, uint32_t mode, int warmup,
             int iters, double* ms_per_iter, kv_error** err) {
  if (!ps || !b || !ms_per_iter) return fail(err, KV_E_INVALID, "null argument");
  try {
    run(const_cast<kv_policyset*>(ps), const_cast<kv_batch*>(b), ctx_json, {device}, mode, nullptr, warmup, iters,
        ms_per_iter);
    return 0;
  } catch (const HipError& e) {
    return fail(err, KV_E_DEVICE, e.what());
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_result_status(const kv_result* r, const uint8_t** status, uint64_t* n_rules, uint64_t* n_res) {
  if (!r) return KV_E_INVALID;
  if (status) {
    try {
      *status = const_cast<kv_result*>(r)->status_caller();
    } catch (const std::exception&) {
      return KV_E_NOMEM;
    }
  }
  if (n_rules) *n_rules = r->n_rules;
  if (n_res) *n_res = r->n_res;
  return 0;
}

int kv_host_reserve(uint64_t bytes) {
  try {
    return PinnedStore::enabled() && PinnedPool::get().reserve(bytes) ? 0 : KV_E_DEVICE;
  } catch (const std::exception&) {
    return KV_E_DEVICE;
  }
}

int kv_device_pool_limit(uint64_t bytes) {
  DevPool& p = DevPool::get();
  std::lock_guard<std::mutex> g(p.mu);
  p.hold = (size_t)bytes;
  return 0;
}

int kv_device_trim(int device) {
  int n = 0, cur = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n || hipGetDevice(&cur) != hipSuccess) {
    (void)hipGetLastError();
    return KV_E_DEVICE;
  }
  if (hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    return KV_E_DEVICE;
  }
  DevPool::get().trim(device);
  (void)hipSetDevice(cur);
  return 0;
}

int kv_result_phase(const kv_result* r, uint32_t i, const char** name, double* ms) {
  if (!r) return KV_E_INVALID;
  if (i >= r->phases.size()) return KV_E_RANGE;
  if (name) *name = r->phases[i].first.c_str();
  if (ms) *ms = r->phases[i].second;
  return 0;
}

int kv_result_counts(const kv_result* r, const int64_t** counts) {
  if (!r || !counts) return KV_E_INVALID;
  *counts = r->counts.data();
  return 0;
}

int kv_result_scope_counts(const kv_result* r, const int64_t** counts, uint32_t* n_scopes) {
  if (!r || !counts) return KV_E_INVALID;
  if (!(r->mode & KV_MODE_SCOPES)) return KV_E_INVALID;
  *counts = r->scope_counts.data();
  if (n_scopes) *n_scopes = (uint32_t)r->b->b.namespaces.size();
  return 0;
}

int kv_batch_namespaces(const kv_batch* b, uint32_t* n) {
  if (!b || !n) return KV_E_INVALID;
  *n = (uint32_t)b->b.namespaces.size();
  return 0;
}

const char* kv_batch_namespace(const kv_batch* b, uint32_t i) {
  if (!b || i >= b->b.namespaces.size()) return nullptr;
  return b->b.namespaces[i].c_str();
}

int kv_result_path(const kv_result* r, uint32_t rule, uint64_t res, char* buf, size_t cap) {
  if (!r || !r->has_err()) return KV_E_INVALID;
  if (rule >= r->n_rules || res >= r->n_res) return KV_E_RANGE;
  res = r->sidx(res);
  size_t o = (size_t)rule * r->n_res + res;
  if (const_cast<kv_result*>(r)->st_store()[o] != ST_FAIL) return KV_E_INVALID;
  ErrRec e;
  const Batch* bt = nullptr;
  if (!r->err(rule, res, &e, &bt)) return KV_E_INVALID;
  std::string p = render_path(r->ps->ps, *bt, e);
  if (buf && cap) {
    size_t n = std::min(cap - 1, p.size());
    memcpy(buf, p.data(), n);
    buf[n] = 0;
  }
  return (int)p.size();
}

int kv_result_error(const kv_result* r, uint32_t rule, uint64_t res, uint32_t* kind, uint32_t* flags) {
  if (!r || !r->has_err()) return KV_E_INVALID;
  if (rule >= r->n_rules || res >= r->n_res) return KV_E_RANGE;
  res = r->sidx(res);
  const uint8_t st = const_cast<kv_result*>(r)->st_store()[(size_t)rule * r->n_res + res];
  if (st != ST_FAIL && st != ST_ERROR && st != ST_SKIP) return KV_E_INVALID;
  ErrRec e;
  const Batch* bt = nullptr;
  if (!r->err(rule, res, &e, &bt)) return KV_E_INVALID;
  if (kind) *kind = e.kind_flags & 0xFFFF;
  if (flags) *flags = e.kind_flags >> 16;
  return 0;
}

int kv_result_error_message(const kv_result* r, uint32_t rule, uint64_t res, const char* resource_json, size_t len,
                            char* buf, size_t cap) {
  if (!r || !r->has_err() || !resource_json) return KV_E_INVALID;
  if (rule >= r->n_rules || res >= r->n_res) return KV_E_RANGE;
  const uint64_t s = r->store_of(res);  // the batch's tables are in store order
  res = r->sidx(res);  // the caller's document of its resource `res`, the record of its status slot
  size_t o = (size_t)rule * r->n_res + res;
  const uint8_t st = const_cast<kv_result*>(r)->st_store()[o];
  if (st != ST_FAIL && st != ST_ERROR && st != ST_SKIP) return KV_E_INVALID;
  std::string m;
  try {
    JDoc doc;
    parse_json(resource_json, len, NUM_UNSTRUCTURED, &doc);
    ErrRec e;
    const Batch* bt = nullptr;
    if (!r->err(rule, res, &e, &bt)) return KV_E_INVALID;
    std::string pv;
    const std::string* dyn_pv = nullptr;
    if (e.pnode < r->ps->ps.pnodes.size() && r->ps->ps.pnodes[e.pnode].dleaf >= 0) {
      const ResultPart* p = r->part_of(s);
      kv_batch* kb = p->shard ? p->shard.get() : const_cast<kv_batch*>(r->b);
      const DynHost& h = kb->dyn_host(r->ps->ps);
      const uint64_t nl = kb->b.res.size(), local = s - p->lo;
      const uint32_t o = h.dleaf[(size_t)r->ps->ps.pnodes[e.pnode].dleaf * nl + local];
      pv = pattern_go_v(outcome_value(kb->b.vout_tab[o]));
      dyn_pv = &pv;
    }
    m = error_message(r->ps->ps, *bt, e, doc, dyn_pv);
  } catch (const std::exception&) {
    return KV_E_PARSE;
  }
  if (m.empty()) return KV_E_INVALID;  // a compile-time constant status: no pattern error record
  if (buf && cap) {
    size_t n = std::min(cap - 1, m.size());
    memcpy(buf, m.data(), n);
    buf[n] = 0;
  }
  return (int)m.size();
}

int kv_result_subst_error(const kv_result* r, uint32_t rule, uint64_t res, char* buf, size_t cap) {
  if (!r) return KV_E_INVALID;
  if (rule >= r->n_rules || res >= r->n_res) return KV_E_RANGE;
  if (!r->has_status()) return KV_E_INVALID;  // counts-only result: no statuses were fetched
  const uint64_t s = r->store_of(res);          // (the batch's tables are in store order)
  res = r->sidx(res);
  try {
    const RuleRec& rr = r->ps->ps.rules[rule];
    if (!rr.dyn || const_cast<kv_result*>(r)->st_store()[(size_t)rule * r->n_res + res] != ST_ERROR) return 0;
    const ResultPart* p = r->part_of(s);
    if (!p) return 0;
    kv_batch* kb = p->shard ? p->shard.get() : const_cast<kv_batch*>(r->b);
    const DynHost& h = kb->dyn_host(r->ps->ps);
    const uint64_t nl = kb->b.res.size(), local = s - p->lo;
    const size_t q = (size_t)(rr.dyn - 1) * nl + local;
    if (h.dyn_st[q] != ST_ERROR) return 0;
    // ruleError(rule, Validation, "variable substitution failed", err) (validation.go:186-188)
    const std::string m = "variable substitution failed: " + kb->b.vout_tab[h.dyn_msg[q]].substr(1);
    if (buf && cap) {
      size_t n = std::min(cap - 1, m.size());
      memcpy(buf, m.data(), n);
      buf[n] = 0;
    }
    return (int)m.size();
  } catch (const std::exception&) {
    return KV_E_INVALID;
  }
}

double kv_result_kernel_ms(const kv_result* r) { return r ? r->kernel_ms : -1.0; }

int kv_result_failures(const kv_result* cr, uint64_t* n, const uint32_t** rule, const uint64_t** res,
                       const uint32_t** path_id) {
  if (!cr || !cr->has_err() || !n) return KV_E_INVALID;
  kv_result* r = const_cast<kv_result*>(cr);
  try {
    std::call_once(r->fail_once, [r]() {
      // one pass over the statuses: records come rule-major, in resource order per part
      std::unordered_map<uint64_t, uint32_t> compact;      // (path pnode, packed indices) -> path id
      std::unordered_map<std::string, uint32_t> rendered;  // wide records: by rendered path
      const PolicySet& ps = r->ps->ps;
      const uint8_t* stm = r->st_store();
      for (uint32_t rl = 0; rl < r->n_rules; rl++) {
        const uint8_t* row = stm + (size_t)rl * r->n_res;
        for (const ResultPart& p : r->parts) {
          uint64_t i = p.base[rl];
          for (uint64_t q = p.lo; q < p.lo + p.n; q++) {
            const uint8_t st = row[q];
            if (st != ST_FAIL && st != ST_ERROR && st != ST_SKIP) continue;
            uint32_t id = KV_PATH_NONE;
            if (st == ST_FAIL) {
              const ErrRec8 c = p.r8(rl, i);
              if ((c.w0 & ERR8_WIDE) && !p.recw.empty()) {
                const std::string path = render_path(ps, r->batch_of(p), p.recw[i]);
                auto it = rendered.find(path);
                if (it == rendered.end()) {
                  it = rendered.emplace(path, (uint32_t)r->f_paths.size()).first;
                  r->f_paths.push_back(path);
                }
                id = it->second;
              } else {
                const ErrRec e = kv_result::decode(c);
                const uint64_t key = (uint64_t)path_pnode(ps, e) << 32 | (c.w1 & ERR8_IDX_MASK);
                auto it = compact.find(key);
                if (it == compact.end()) {
                  const std::string path = render_path(ps, r->batch_of(p), e);
                  auto jt = rendered.find(path);
                  if (jt == rendered.end()) {
                    jt = rendered.emplace(path, (uint32_t)r->f_paths.size()).first;
                    r->f_paths.push_back(path);
                  }
                  it = compact.emplace(key, jt->second).first;
                }
                id = it->second;
              }
            }
            r->f_rule.push_back(rl);
            r->f_res.push_back(r->cidx(q));
            r->f_path.push_back(id);
            i++;
          }
        }
      }
      if (!r->b->b.order.empty() && !r->caller_order) {
        // caller order: by rule, then caller resource index. Each rule's pairs are a subset of
        // [0, n_res) with distinct caller indices: a rule with pairs on 1/16 of the resources or more
        // is scattered into a per-thread slot array and swept in order, a sparser one sorted
        // (rules split over host threads)
        std::vector<size_t> rb(r->n_rules + 1, 0);
        for (size_t i = 0; i < r->f_rule.size(); i++) rb[r->f_rule[i] + 1]++;
        for (uint32_t rl = 0; rl < r->n_rules; rl++) rb[rl + 1] += rb[rl];
        std::vector<uint64_t> fs(r->f_res.size());
        std::vector<uint32_t> fp(r->f_path.size());
        const unsigned T = std::max(1u, std::min<unsigned>(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned t = 0; t < T; t++)
          th.emplace_back([&, t]() {
            std::vector<uint32_t> slot;  // caller index -> path id + 1 (0: no pair)
            for (uint32_t rl = t; rl < r->n_rules; rl += T) {
              if (rb[rl] == rb[rl + 1]) continue;
              if ((rb[rl + 1] - rb[rl]) * 16u < r->n_res) {
                std::vector<std::pair<uint64_t, uint32_t>> v;
                v.reserve(rb[rl + 1] - rb[rl]);
                for (size_t i = rb[rl]; i < rb[rl + 1]; i++) v.push_back({r->f_res[i], r->f_path[i]});
                std::sort(v.begin(), v.end());
                for (size_t i = 0; i < v.size(); i++) {
                  fs[rb[rl] + i] = v[i].first;
                  fp[rb[rl] + i] = v[i].second;
                }
                continue;
              }
              if (slot.empty()) slot.assign(r->n_res, 0u);
              for (size_t i = rb[rl]; i < rb[rl + 1]; i++) slot[r->f_res[i]] = r->f_path[i] + 1u;
              size_t o = rb[rl];
              for (uint64_t j = 0; j < r->n_res && o < rb[rl + 1]; j++)
                if (slot[j]) {
                  fs[o] = j;
                  fp[o++] = slot[j] - 1u;
                  slot[j] = 0u;
                }
            }
          });
        for (auto& x : th) x.join();
        r->f_res.swap(fs);
        r->f_path.swap(fp);
        // path ids numbered by first appearance in the returned order
        std::vector<uint32_t> renum(r->f_paths.size(), KV_PATH_NONE);
        std::vector<std::string> paths;
        for (uint32_t& id : r->f_path) {
          if (id == KV_PATH_NONE) continue;
          if (renum[id] == KV_PATH_NONE) {
            renum[id] = (uint32_t)paths.size();
            paths.push_back(std::move(r->f_paths[id]));
          }
          id = renum[id];
        }
        r->f_paths.swap(paths);
      }
    });
  } catch (const std::exception&) {
    return KV_E_NOMEM;
  }
  *n = r->f_rule.size();
  if (rule) *rule = r->f_rule.data();
  if (res) *res = r->f_res.data();
  if (path_id) *path_id = r->f_path.data();
  return 0;
}

const char* kv_path_string(const kv_result* r, uint32_t path_id) {
  if (!r || path_id >= r->f_paths.size()) return nullptr;
  return r->f_paths[path_id].c_str();
}

int kv_session_create(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, int device, uint32_t mode,
                      kv_session** out, kv_error** err) {
  if (!ps || !b || !out) return fail(err, KV_E_INVALID, "null argument");
  if (b->owner != ps) return fail(err, KV_E_INVALID, "batch was ingested for a different policy set");
  try {
    *out = new kv_session(const_cast<kv_policyset*>(ps), const_cast<kv_batch*>(b), ctx_json, {device}, mode);
    return 0;
  } catch (const HipError& e) {
    return fail(err, KV_E_DEVICE, e.what());
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_session_create_devices(const kv_policyset* ps, const kv_batch* b, const char* ctx_json, uint32_t device_mask,
                              uint32_t mode, kv_session** out, kv_error** err) {
  if (!ps || !b || !out) return fail(err, KV_E_INVALID, "null argument");
  if (b->owner != ps) return fail(err, KV_E_INVALID, "batch was ingested for a different policy set");
  try {
    const std::vector<int> devs = mask_devices(device_mask);
    if (devs.empty()) return fail(err, KV_E_INVALID, "empty device mask");
    *out = new kv_session(const_cast<kv_policyset*>(ps), const_cast<kv_batch*>(b), ctx_json, devs, mode);
    return 0;
  } catch (const HipError& e) {
    return fail(err, KV_E_DEVICE, e.what());
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_session_create_parts(const kv_policyset* ps, const char* ctx_json, uint32_t mode, uint32_t n_parts,
                            kv_session** out, kv_error** err) {
  if (!ps || !out || n_parts == 0) return fail(err, KV_E_INVALID, "bad argument");
  try {
    *out = new kv_session(const_cast<kv_policyset*>(ps), ctx_json, mode, n_parts);
    return 0;
  } catch (const std::exception& e) {
    return fail(err, KV_E_PARSE, e.what());
  }
}

int kv_session_attach_part(kv_session* s, uint32_t part, const kv_batch* b, int device, kv_error** err) {
  if (!s || !b) return fail(err, KV_E_INVALID, "null argument");
  if (b->owner != s->set.ps) return fail(err, KV_E_INVALID, "batch was ingested for a different policy set");
  try {
    s->set.attach(part, const_cast<kv_batch*>(b), device);
    return 0;
  } catch (const HipError& e) {
    return fail(err, KV_E_DEVICE, e.what());
  } catch (const std::exception& e) {
    return fail(err, KV_E_INVALID, e.what());
  }
}

int kv_session_scopes(const kv_session* s, uint32_t* n_scopes) {
  if (!s || !n_scopes) return KV_E_INVALID;
  if (s->set.parts_mode) {
    if (!s->set.finalized) return KV_E_INVALID;
    *n_scopes = (uint32_t)s->set.scope_names.size();
  } else {
    *n_scopes = (uint32_t)s->set.bt->b.namespaces.size();
  }
  return 0;
}

const char* kv_session_scope_name(const kv_session* s, uint32_t i) {
  if (!s) return nullptr;
  const std::vector<std::string>& v = s->set.parts_mode ? s->set.scope_names : s->set.bt->b.namespaces;
  return i < v.size() ? v[i].c_str() : nullptr;
}

int kv_session_rccl_ranks(const kv_session* s, int* ranks) {
  if (!s || !ranks) return KV_E_INVALID;
  *ranks = s->set.rccl_ranks();
  return *ranks < 0 ? KV_E_DEVICE : 0;
}

int kv_session_status_bytes(kv_session* s, uint64_t* bytes) {
  if (!s || !bytes) return KV_E_INVALID;
  try {
    uint64_t t = 0;
    for (auto& p : s->set.parts)
      if (p) t += p->written_status_bytes();
    *bytes = t;
    return 0;
  } catch (const std::exception&) {
    return KV_E_DEVICE;
  }
}

int kv_session_part_ms(const kv_session* s, double* ms) {
  if (!s || !ms) return KV_E_INVALID;
  for (size_t k = 0; k < s->set.parts.size(); k++) ms[k] = k < s->set.part_ms.size() ? s->set.part_ms[k] : 0.0;
  return 0;
}

int kv_session_parts(const kv_session* s, uint32_t* n_parts) {
  if (!s || !n_parts) return KV_E_INVALID;
  *n_parts = (uint32_t)s->set.parts.size();
  return 0;
}

int kv_session_fetch(kv_session* s, kv_result** out, kv_error** err) {
  if (!s || !out) return fail(err, KV_E_INVALID, "null argument");
  try {
    auto* r = new kv_result();
    try {
      s->set.fetch(r, 0.0);
    } catch (...) {
      delete r;
      throw;
    }
    *out = r;
    return 0;
  } catch (const std::exception& e) {
    return fail(err, KV_E_DEVICE, e.what());
  }
}

int kv_session_run(kv_session* s, int iters, double* event_ms, kv_error** err) {
  if (!s || iters < 0) return fail(err, KV_E_INVALID, "bad argument");
  try {
    double t = s->set.run(iters);
    if (event_ms) *event_ms = t;
    return 0;
  } catch (const std::exception& e) {
    return fail(err, KV_E_DEVICE, e.what());
  }
}

int kv_session_counts(kv_session* s, int64_t* counts) {
  if (!s || !counts) return KV_E_INVALID;
  try {
    s->set.reduce();
    std::copy(s->set.counts_.begin(), s->set.counts_.end(), counts);
    return 0;
  } catch (const std::exception&) {
    return KV_E_DEVICE;
  }
}

int kv_session_scope_counts(kv_session* s, int64_t* counts) {
  if (!s || !counts || !(s->set.mode & KV_MODE_SCOPES)) return KV_E_INVALID;
  try {
    s->set.reduce();
    std::copy(s->set.scope_counts_.begin(), s->set.scope_counts_.end(), counts);
    return 0;
  } catch (const std::exception&) {
    return KV_E_DEVICE;
  }
}

void kv_free_session(kv_session* s) { delete s; }

void kv_free_policyset(kv_policyset* ps) { delete ps; }
void kv_free_batch(kv_batch* b) { delete b; }
void kv_free_result(kv_result* r) { delete r; }
void kv_free_error(kv_error* e) {
  if (e) {
    free(e->message);
    free(e);
  }
}
void kv_free_buffer(char* p) { free(p); }

}  // extern "C"
