// capi.cpp — extern "C" implementation of include/kwgpu.h: environment and batch lifetime, HBM
// residency, planning and launch of the hot path (kernels.hip) and the host epilogue (service.cpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kwgpu.h"
#include "automaton.hpp"
#include "batch.hpp"
#include "env.hpp"
#include "kernels.hpp"
#include "metrics.hpp"
#include "service.hpp"
#include "slotplan.hpp"
#include "yaml.hpp"

using namespace kw;


struct kw_env {
  Env e;
  // identity of this environment for plan caches (an address can be reused by a later one)
  uint64_t uid = next_uid();
  static uint64_t next_uid() {
    static std::atomic<uint64_t> n{1};
    return n++;
  }
};

namespace kw {

// Caching allocators for device memory and pinned host staging: a micro-batch front evaluates
// thousands of small batches per second, and hipMalloc / hipHostMalloc per batch would dominate.
// Blocks are kept per (device, size class) up to max_cached() bytes per pool.
struct BlockPool {
  bool host;
  std::mutex m;
  std::map<std::pair<int, size_t>, std::vector<void*>> free;
  size_t cached = 0;
  // cached bytes: device 32 GiB (of 288), pinned host 16 GiB — the bulk path's per-call blocks
  // (bounce, ring, descriptors) and a re-uploaded batch's image come back from the cache
  size_t max_cached() const { return host ? (size_t)16 << 30 : (size_t)32 << 30; }
  explicit BlockPool(bool h) : host(h) {}
  // size classes: 4 KiB, then eight steps per power of two (<= 12.5 % slack: C5's 3.6 GB image
  // took a 4 GiB block before)
  static size_t cls(size_t n) {
    if (n <= 4096) return 4096;
    size_t p = 4096;
    while (p * 2 < n) p <<= 1;  // p < n <= 2p
    const size_t step = p / 8;
    return (n + step - 1) / step * step;
  }
  hipError_t alloc(int dev, size_t n, void** p) {
    const size_t c = cls(n);
    {
      std::lock_guard<std::mutex> g(m);
      auto& v = free[{dev, c}];
      if (!v.empty()) {
        *p = v.back();
        v.pop_back();
        cached -= c;
        return hipSuccess;
      }
    }
    return host ? hipHostMalloc(p, c, hipHostMallocDefault) : hipMalloc(p, c);
  }
  void release(int dev, void* p, size_t n) {
    if (!p) return;
    const size_t c = cls(n);
    std::lock_guard<std::mutex> g(m);
    if (cached + c > max_cached()) {
      (void)(host ? hipHostFree(p) : hipFree(p));
      return;
    }
    free[{dev, c}].push_back(p);
    cached += c;
  }
};
BlockPool& dev_pool() {
  static BlockPool* p = new BlockPool(false);  // process lifetime (blocks outlive every batch)
  return *p;
}
BlockPool& host_pool() {
  static BlockPool* p = new BlockPool(true);
  return *p;
}

// Non-blocking streams and timing-free events handed back for reuse, per device: creating a
// stream costs host time on the order of a tenth of a millisecond, and a bulk pass used three.
// A stream returns here drained (its owner synchronized it). KW_STREAM_POOL=0: A/B knob.
struct StreamPool {
  std::mutex m;
  std::map<int, std::vector<hipStream_t>> streams;
  std::map<int, std::vector<hipEvent_t>> events;
  const bool on = !(getenv("KW_STREAM_POOL") && atoi(getenv("KW_STREAM_POOL")) == 0);
  hipError_t get(int dev, hipStream_t* s) {
    if (on) {
      std::lock_guard<std::mutex> g(m);
      auto& v = streams[dev];
      if (!v.empty()) {
        *s = v.back();
        v.pop_back();
        return hipSuccess;
      }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  }
  void put(int dev, hipStream_t s) {
    if (!s) return;
    if (!on) {
      (void)hipStreamDestroy(s);
      return;
    }
    std::lock_guard<std::mutex> g(m);
    streams[dev].push_back(s);
  }
  hipError_t get(int dev, hipEvent_t* e) {
    if (on) {
      std::lock_guard<std::mutex> g(m);
      auto& v = events[dev];
      if (!v.empty()) {
        *e = v.back();
        v.pop_back();
        return hipSuccess;
      }
    }
    return hipEventCreateWithFlags(e, hipEventDisableTiming);
  }
  void put(int dev, hipEvent_t e) {
    if (!e) return;
    if (!on) {
      (void)hipEventDestroy(e);
      return;
    }
    std::lock_guard<std::mutex> g(m);
    events[dev].push_back(e);
  }
};
StreamPool& stream_pool() {
  static StreamPool* p = new StreamPool;  // process lifetime, like the block pools
  return *p;
}

// Host copy spread over up to 16 threads for large buffers (staging fills and verdict read-back:
// one thread moves ≈ 10 GB/s, the host's memory system several times that).
void parallel_copy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kMin = (size_t)8 << 20;
  if (bytes < kMin) {
    memcpy(dst, src, bytes);
    return;
  }
  const size_t nt = std::min<size_t>(16, std::max<size_t>(1, std::min<size_t>(std::thread::hardware_concurrency(), bytes / (kMin / 2))));
  std::vector<std::thread> th;
  for (size_t t = 0; t < nt; ++t) {
    const size_t a = bytes * t / nt, e = bytes * (t + 1) / nt;
    th.emplace_back([=] { memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, e - a); });
  }
  for (auto& x : th) x.join();
}

// Persistent host workers for the bulk path (kw_validate_host): a parallel-for over many short
// tasks (copy segments, tile ranges) without starting threads per call. The caller runs tasks too.
// Each call is a Job on the caller's stack; a worker joins it under the lock (users + 1) and the
// caller returns only when every task is done and every worker that joined has left, so no worker
// ever sees another call's counters or a finished call's function.
class HostWorkers {
 public:
  static HostWorkers& get() {
    static HostWorkers* w = new HostWorkers();  // process lifetime (workers park on a condition)
    return *w;
  }
  // fn(i) for every i in [0, n), spread over the workers and the caller; returns when all are done
  // A single task runs inline on the caller: no lock, no wake-up (kwhost's small micro-batches plan
  // one tile range per pass, and its pipeline workers must not serialise on run_m_ for that).
  void run(size_t n, const std::function<void(size_t)>& fn) {
    if (n == 0) return;
    if (n == 1) {
      fn(0);
      return;
    }
    std::lock_guard<std::mutex> one(run_m_);  // one parallel-for at a time
    Job job;
    job.fn = &fn;
    job.n = n;
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &job;
      ++gen_;
    }
    cv_.notify_all();
    const size_t mine = job.work();
    std::unique_lock<std::mutex> g(m_);
    job_ = nullptr;  // no worker joins after this
    job.done += mine;
    done_cv_.wait(g, [&] { return job.done == job.n && job.users == 0; });
  }

 private:
  struct Job {
    const std::function<void(size_t)>* fn = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0};
    size_t done = 0;     // tasks finished (under m_)
    unsigned users = 0;  // workers inside work() (under m_)
    size_t work() {
      size_t k = 0;
      for (size_t i; (i = next.fetch_add(1)) < n; ++k) (*fn)(i);
      return k;
    }
  };
  HostWorkers() {
    const char* e = getenv("KW_HOST_THREADS");
    unsigned n = e ? (unsigned)std::max(1, atoi(e)) : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    for (unsigned i = 1; i < n; ++i) std::thread([this] { loop(); }).detach();
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      Job* j = nullptr;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return gen_ != seen && job_ != nullptr; });
        seen = gen_;
        j = job_;
        ++j->users;
      }
      const size_t mine = j->work();
      std::lock_guard<std::mutex> g(m_);
      j->done += mine;
      --j->users;
      if (j->done == j->n && j->users == 0) done_cv_.notify_all();
    }
  }
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_cv_;
  Job* job_ = nullptr;
  uint64_t gen_ = 0;
};

// Copies of several (dst, src, bytes) segments cut into ~1 MB tasks on the host workers.
struct CopySeg {
  void* dst;
  const void* src;
  size_t bytes;
};
void parallel_copy_segs(const std::vector<CopySeg>& segs) {
  constexpr size_t kTask = (size_t)1 << 20;
  std::vector<CopySeg> tasks;
  for (const CopySeg& c : segs)
    for (size_t a = 0; a < c.bytes; a += kTask)
      tasks.push_back({(uint8_t*)c.dst + a, (const uint8_t*)c.src + a, std::min(kTask, c.bytes - a)});
  HostWorkers::get().run(tasks.size(), [&](size_t i) { memcpy(tasks[i].dst, tasks[i].src, tasks[i].bytes); });
}

// Requests per tile of the tile kernel forced by KW_SLOT_ROWS (8..255, A/B knob), 0 = chosen per
// batch (plan_pass: kSlotRows, or taller tiles where they keep enough workgroups per CU).
// Tile schedule of a launch of `ntiles` tiles over `grid` workgroups: the dynamic one (per-XCD
// counters, kernels.hip) only where a workgroup runs more than 16 tiles, so that drift between
// workgroups has room to build up; below that the strided schedule is as balanced and skips the
// counter traffic: every fetch is an atomic on one L2 line per XCD, serialised — r05 same-box A/B
// (profiles/r05_sched_ab.txt): strided C4 -2.4 %, C2 -6 %, C1 -40 %, a 64k-request shard -47 %; the
// dynamic one C5 -7 % (its heavy region), C6 -2 %, C3 -2 %. KW_SCHED=static / dynamic forces one.
// Tables read from global memory (C6) make tile costs vary with the caches: there the dynamic
// schedule pays from 4 tiles a workgroup (C6 at 15: -2 %).
bool sched_dynamic(uint64_t ntiles, uint32_t grid, bool lds_tables) {
  const char* e = getenv("KW_SCHED");
  if (e && std::string(e) == "static") return false;
  if (e && std::string(e) == "dynamic") return true;
  return ntiles > (lds_tables ? 16ull : 4ull) * std::max<uint32_t>(grid, 1);
}

// Tile height of a split batch's heavy region (KW_HEAVY_ROWS, A/B knob; 0: planned like any batch).
uint32_t heavy_rows() {
  const char* e = getenv("KW_HEAVY_ROWS");
  const int v = e ? atoi(e) : 0;
  return (v >= 8 && v <= 255) ? (uint32_t)v : 0u;
}

uint32_t slot_rows_forced() {
  const char* e = getenv("KW_SLOT_ROWS");  // read per pass (tests switch it between passes)
  const int v = e ? atoi(e) : 0;
  return (v >= 8 && v <= 255) ? (uint32_t)v : 0u;  // tile-local owners are u8
}

// The next-tile L2 prefetch at run time (KW_L2_PREFETCH=1, A/B knob; the kernel carries its code when
// built with KW_PREFETCH). Off: running it costs C4 3.5 % and C6 3.8 % (r04 same-box A/B), while the
// kernel built with the code present and the plan leaving it off was 2 % faster on C2 / C3 / C4
// than the kernel built without it (profiles/r04_prefetch_ab.txt).
bool l2_prefetch() {
  static const bool on = KW_PREFETCH && getenv("KW_L2_PREFETCH") && atoi(getenv("KW_L2_PREFETCH")) != 0;
  return on;
}

// Per-tile entity counts and staged byte ranges of a batch, reduced to a high quantile (tile_quantile).
struct TileStats {
  uint32_t ctr = 0, lbl = 0, kadd = 0, kdrop = 0;
  uint32_t bytes[NSTR] = {};
};

// A split batch's entity maps (upload_batch, permute_batch): the source entity of each destination
// entity, per level — what the upload gathers the string bytes by (gather_column).
struct RowOrder {
  const std::vector<uint64_t>* perm = nullptr;  // rows (DeviceBatch::perm)
  std::vector<uint32_t> cmap, lmap, amap, dmap;  // containers, labels, added / dropped capabilities
  uint64_t src(int m, uint64_t e) const {
    switch (m) {
      case S_NS: return (*perm)[e];
      case S_CAPADD: return amap[e];
      case S_CAPDROP: return dmap[e];
      case S_LK: case S_LV: return lmap[e];
      default: return cmap[e];
    }
  }
};

// Device copy of a batch: one allocation for the input columns, lazily sized verdict / plan /
// side-data buffers, a private stream and timing events.
struct DeviceBatch {
  int device = -1;
  hipStream_t stream = nullptr;  // the batch's stream (passes without a caller stream)
  bool owns_stream = true;       // false: the caller's stream (kw_batch_to_device_async)
  void* staging = nullptr;       // pinned host staging of the last upload
  size_t staging_bytes = 0;
  hipStream_t cur = nullptr;     // stream of the last pass (kw_batch_verdicts synchronises on it)
  uint8_t* cols = nullptr;
  size_t cols_bytes = 0;
  // device views of the columns
  const uint8_t* req_flags = nullptr;
  const uint32_t *ctr_off = nullptr, *lbl_off = nullptr, *capadd_off = nullptr, *capdrop_off = nullptr;
  const uint8_t* ctr_flags = nullptr;
  struct DCol {
    const uint32_t* off = nullptr;
    const uint8_t* bytes = nullptr;
    uint64_t n = 0;
    uint64_t nbytes = 0;
  } str[NSTR];
  uint32_t* verdicts = nullptr;
  size_t verdict_cap = 0;
  size_t last_verdicts = 0;
  uint32_t last_row_words = 0;  // verdict words per row of the last pass (npol; rows mode 1)
  // light / heavy split (upload_batch, split_rows): the device copy holds the batch's rows in
  // another order — the light rows, then the heavy ones — and every device buffer indexed by row
  // (verdicts, side data, the rows-mode column map) follows that order; kw_batch_verdicts and
  // load_side_data scatter them back. perm[d]: the batch row at device row d; split: the light
  // region's rows (0: not split); dev_b: the reordered batch the planner reads (its offsets only:
  // the string bytes are dropped after the upload).
  std::vector<uint64_t> perm;
  uint64_t split = 0;
  std::unique_ptr<Batch> dev_b;
  // the last all-pairs pass's plan (capi.cpp validate_cached; a PassPlan): reused while the
  // environment, the policy list, the origin and every KW_* setting stay the same — planning a
  // 64-policy pass is ~60-300 us of host time, the whole GPU time of a small shard
  std::shared_ptr<void> plan_cache;
  uint64_t plan_env = 0, plan_knobs = 0;
  std::vector<int32_t> plan_pols;
  int plan_origin = -1;
  std::unique_ptr<RowOrder> order;  // (until the upload's staging is filled)
  uint32_t loaded = 0;        // string columns (bits of Str) whose bytes are resident (kw_validate_host uploads only its pass's)
  uint32_t* sched = nullptr;  // tile counters (zeroed once; each launch leaves them zero)
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  // the last pass's plan as the kernels read it (host copies detect a changed plan)
  TileArgs* d_tiles = nullptr;
  size_t d_tiles_cap = 0;
  std::vector<TileArgs> h_tiles;
  uint8_t* d_slots = nullptr;
  size_t d_slots_cap = 0;
  std::vector<uint8_t> h_slots;
  uint32_t* rowcol = nullptr;
  size_t rowcol_cap = 0;
  std::vector<uint32_t> h_rowcol;
  // host-built tile descriptors + overflow list, cached for one plan geometry (desc_key)
  TileDesc* desc = nullptr;
  size_t desc_cap = 0;
  uint32_t* overflow = nullptr;  // [count, request indices...]
  size_t overflow_cap = 0;
  std::vector<TileDesc> h_desc;
  std::vector<uint32_t> h_ovf;
  uint32_t n_overflow = 0;
  uint64_t ndesc = 0;
  uint64_t reg_desc[2] = {0, 0}, reg_ndesc[2] = {0, 0};  // each region's descriptors within desc
  uint64_t desc_key = 0;
  bool desc_valid = false;   // D.desc holds the whole batch's descriptors for desc_key
  uint32_t needs_stride = 1;  // tile needs sampled every needs_stride-th tile (set by kw_validate_host)
  // overflow path: per-string classes in HBM (one allocation) and the wide-argument side data
  uint16_t* g_cls = nullptr;
  size_t g_cls_cap = 0;
  // NFA elements: their classes ([label][nlv] | [container][nim]) and the Pike VMs' scratch
  uint16_t* nfa_cls = nullptr;
  size_t nfa_cls_cap = 0;
  uint32_t* nfa_scratch = nullptr;
  size_t nfa_scratch_cap = 0;
  uint32_t max_image_len = 0xffffffffu;  // longest image reference of the batch (computed on first use)
  uint32_t* wide_count = nullptr;
  bool wide_valid = false;  // the last pass zeroed wide_count and ran the overflow kernels
  WideRec* wide_rec = nullptr;
  size_t wide_rec_cap = 0;
  uint64_t* wide_groups = nullptr;
  size_t wide_groups_cap = 0;
  // wide policy groups (WideGroupPass): the members' pass output, the combine kernel's records,
  // value-stack scratch and the cause bitsets
  uint32_t* member_words = nullptr;
  size_t member_words_cap = 0;
  uint8_t* wg_data = nullptr;
  size_t wg_data_cap = 0;
  uint64_t* wg_stack = nullptr;
  size_t wg_stack_cap = 0;
  uint64_t* big_causes = nullptr;
  size_t big_causes_cap = 0;
  uint32_t last_big_stride = 0;
  std::vector<WideData::BigRef> last_big_ref;
  // what the last pass left in the side buffers
  uint32_t last_nwide = 0, last_wide_cap = 0;
  bool last_rows_mode = false;
  std::vector<int32_t> last_wide_policy;
  // tile capacities of this batch (plan_pass), per tile height tried
  struct RowsPlan {
    uint32_t rows = 0;
    uint64_t lo = 0, hi = 0;         // the region's rows
    uint32_t stride = 1;            // needs of every stride-th tile (kw_validate_host samples)
    std::vector<TileStats> need, q;  // per-tile needs and their quantiles
    uint64_t cap_key = 0;
    int cap_choice = -1;   // quantile index chosen for cap_key
    uint32_t cap_cu = 0;   // its workgroups per CU
    uint32_t cap_lds = 0;  // its LDS bytes
  };
  std::deque<RowsPlan> rows_plans;  // deque: plan_rows hands out references that must survive later insertions
  ~DeviceBatch() {
    if (device < 0) return;  // host-only view (kw_debug_plan)
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (cur && cur != stream) (void)hipStreamSynchronize(cur);
    BlockPool& P = dev_pool();
    P.release(device, d_tiles, d_tiles_cap * sizeof(TileArgs));
    P.release(device, d_slots, d_slots_cap);
    P.release(device, rowcol, rowcol_cap * 4);
    P.release(device, desc, desc_cap * sizeof(TileDesc));
    P.release(device, overflow, overflow_cap * 4);
    P.release(device, cols, cols_bytes);
    P.release(device, verdicts, verdict_cap * 4);
    P.release(device, g_cls, g_cls_cap * 2);
    P.release(device, nfa_cls, nfa_cls_cap * 2);
    P.release(device, nfa_scratch, nfa_scratch_cap * 4);
    P.release(device, wide_rec, wide_rec_cap * sizeof(WideRec));
    P.release(device, wide_groups, wide_groups_cap * 8);
    P.release(device, member_words, member_words_cap * 4);
    P.release(device, wg_data, wg_data_cap);
    P.release(device, wg_stack, wg_stack_cap * 8);
    P.release(device, big_causes, big_causes_cap * 8);
    P.release(device, sched, 512 * sizeof(uint32_t));  // every launch leaves the tile counters zero
    P.release(device, wide_count, sizeof(uint32_t));
    host_pool().release(device, staging, staging_bytes);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (stream && owns_stream) stream_pool().put(device, stream);
  }
};

}  // namespace kw

struct kw_batch {
  Batch b;
  std::unique_ptr<DeviceBatch> dev;
  std::vector<void*> host_pinned;  // kw_batch_pin_host: column arrays page-locked in place
  ~kw_batch() {
    dev.reset();  // synchronizes the batch's streams: no copy can still read a registered column
    for (void* p : host_pinned) (void)hipHostUnregister(p);
  }
};

namespace {

void put_err(char* buf, size_t cap, const std::string& s) {
  if (!buf || cap == 0) return;
  size_t n = std::min(cap - 1, s.size());
  memcpy(buf, s.data(), n);
  buf[n] = 0;
}

int put_out(const std::string& s, char* buf, size_t cap, size_t* need) {
  if (need) *need = s.size() + 1;
  if (!buf || cap < s.size() + 1) return KW_E_NOSPACE;
  memcpy(buf, s.data(), s.size());
  buf[s.size()] = 0;
  return KW_OK;
}

#define HIPCHK(x)                             \
  do {                                        \
    hipError_t _e = (x);                      \
    if (_e != hipSuccess) return KW_E_DEVICE; \
  } while (0)

// Device buffer of at least n elements from the pool (the current device's), replacing a smaller one.
template <typename T>
int ensure(T** p, size_t* cap, size_t n) {
  if (*cap >= n && *p) return KW_OK;
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  dev_pool().release(dev, *p, *cap * sizeof(T));
  *p = nullptr;
  const size_t want = BlockPool::cls(std::max<size_t>(n, 1) * sizeof(T)) / sizeof(T);
  void* q = nullptr;
  HIPCHK(dev_pool().alloc(dev, want * sizeof(T), &q));
  *p = (T*)q;
  *cap = want;
  return KW_OK;
}

int upload_env(kw_env* env, int device) {
  if (device < 0) return KW_OK;
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipMalloc(&env->e.d_blob, env->e.blob.size()));
  HIPCHK(hipMemcpy(env->e.d_blob, env->e.blob.data(), env->e.blob.size(), hipMemcpyHostToDevice));
  env->e.device = device;
  return KW_OK;
}

const StrCol& host_str(const Batch& B, int m) {
  switch (m) {
    case S_NS: return B.ns;
    case S_IMG: return B.ctr_image;
    case S_AA: return B.ctr_aa;
    case S_CAPADD: return B.cap_add;
    case S_CAPDROP: return B.cap_drop;
    case S_LK: return B.lbl_key;
    default: return B.lbl_val;
  }
}

// Entity range [g0, g1) of string column m for requests [r0, r1).
void str_range(const Batch& B, int m, uint64_t r0, uint64_t r1, uint64_t* g0, uint64_t* g1) {
  switch (m) {
    case S_NS: *g0 = r0; *g1 = r1; break;
    case S_CAPADD: *g0 = B.capadd_off[B.ctr_off[r0]]; *g1 = B.capadd_off[B.ctr_off[r1]]; break;
    case S_CAPDROP: *g0 = B.capdrop_off[B.ctr_off[r0]]; *g1 = B.capdrop_off[B.ctr_off[r1]]; break;
    case S_LK: case S_LV: *g0 = B.lbl_off[r0]; *g1 = B.lbl_off[r1]; break;
    default: *g0 = B.ctr_off[r0]; *g1 = B.ctr_off[r1]; break;
  }
}

constexpr uint32_t kTableBudget = 64 * 1024;   // classifiers + chunk records staged per workgroup
constexpr uint32_t kTileLdsBudget = 160 * 1024;  // tile-kernel LDS per workgroup (gfx950: 160 KB per CU)
constexpr uint32_t kMaxTileEntities = 60000;    // per-request indices in a tile stay below ARG's 65535
constexpr double kTileQuantiles[] = {1.0, 0.99995, 0.9999, 0.9995, 0.999, 0.998};  // capacity candidates

// What each tile of `rows` requests of rows [lo, hi) stages: entity counts and the 16-B aligned byte
// span of each string column.
std::vector<TileStats> tile_needs(const Batch& B, uint32_t rows, uint32_t stride, uint64_t lo, uint64_t hi) {
  const uint64_t ntiles_all = (hi - lo + rows - 1) / rows;
  const uint64_t ntiles = (ntiles_all + stride - 1) / stride;  // sampled tiles: every stride-th
  std::vector<TileStats> v(ntiles);
  // tiles in ranges of 256 on the host workers (each tile's reads are cache misses: 1M requests
  // take ~3 ms on one thread per tile height)
  constexpr uint64_t kRange = 256;
  HostWorkers::get().run((size_t)((ntiles + kRange - 1) / kRange), [&](size_t q) {
  for (uint64_t j = q * kRange, t1 = std::min<uint64_t>(ntiles, (q + 1) * kRange); j < t1; ++j) {
    const uint64_t t = j * stride;
    const uint64_t r0 = lo + t * rows, r1 = std::min<uint64_t>(hi, lo + (t + 1) * rows);
    TileStats& st = v[j];
    st.ctr = B.ctr_off[r1] - B.ctr_off[r0];
    st.lbl = B.lbl_off[r1] - B.lbl_off[r0];
    st.kadd = B.capadd_off[B.ctr_off[r1]] - B.capadd_off[B.ctr_off[r0]];
    st.kdrop = B.capdrop_off[B.ctr_off[r1]] - B.capdrop_off[B.ctr_off[r0]];
    for (int m = 0; m < (int)NSTR; ++m) {
      const StrCol& c = host_str(B, m);
      uint64_t g0, g1;
      str_range(B, m, r0, r1, &g0, &g1);
      st.bytes[m] = ((c.off[g1] + 15u) & ~15u) - (c.off[g0] & ~15u);
    }
  }
  });
  return v;
}

// Per-dimension quantile of the tile needs (quantile 1 = the batch maximum).
TileStats tile_quantile(const std::vector<TileStats>& need, double quantile) {
  TileStats st;
  if (need.empty()) return st;
  const uint64_t n = need.size();
  const uint64_t q = quantile >= 1.0 ? n - 1 : (uint64_t)(quantile * (double)(n - 1));
  std::vector<uint32_t> v(n);
  auto quant = [&](auto f) {
    for (uint64_t t = 0; t < n; ++t) v[t] = f(need[t]);
    std::nth_element(v.begin(), v.begin() + (long)q, v.end());
    return v[q];
  };
  st.ctr = quant([](const TileStats& x) { return x.ctr; });
  st.lbl = quant([](const TileStats& x) { return x.lbl; });
  st.kadd = quant([](const TileStats& x) { return x.kadd; });
  st.kdrop = quant([](const TileStats& x) { return x.kdrop; });
  for (int m = 0; m < (int)NSTR; ++m) st.bytes[m] = quant([m](const TileStats& x) { return x.bytes[m]; });
  return st;
}

// All the capacity-candidate quantiles at once (kTileQuantiles order): per dimension one selection
// at the lowest quantile and a sort of the tail above it (the candidates are all >= 0.998: a few
// dozen values of a 1M-request batch's 15k tiles), dimensions on the host workers.
std::vector<TileStats> tile_quantiles(const std::vector<TileStats>& need, const double* qs, size_t nq) {
  std::vector<TileStats> out(nq);
  if (need.empty() || nq == 0) return out;
  const uint64_t n = need.size();
  std::vector<uint64_t> qi(nq);
  uint64_t qmin = n - 1;
  for (size_t k = 0; k < nq; ++k) {
    qi[k] = qs[k] >= 1.0 ? n - 1 : (uint64_t)(qs[k] * (double)(n - 1));
    qmin = std::min(qmin, qi[k]);
  }
  constexpr int kDims = 4 + (int)NSTR;
  auto dim = [](const TileStats& x, int d) -> uint32_t {
    return d == 0 ? x.ctr : d == 1 ? x.lbl : d == 2 ? x.kadd : d == 3 ? x.kdrop : x.bytes[d - 4];
  };
  auto put = [](TileStats& x, int d, uint32_t v) {
    if (d == 0) x.ctr = v;
    else if (d == 1) x.lbl = v;
    else if (d == 2) x.kadd = v;
    else if (d == 3) x.kdrop = v;
    else x.bytes[d - 4] = v;
  };
  auto one_dim = [&](size_t di) {
    const int d = (int)di;
    std::vector<uint32_t> v(n);
    for (uint64_t t = 0; t < n; ++t) v[t] = dim(need[t], d);
    std::nth_element(v.begin(), v.begin() + (long)qmin, v.end());
    std::sort(v.begin() + (long)qmin, v.end());
    for (size_t k = 0; k < qi.size(); ++k) put(out[k], d, v[qi[k]]);
  };
  if (n < 8192) {  // a small batch (kwhost's micro-batches): inline, no worker wake-up
    for (int d = 0; d < kDims; ++d) one_dim((size_t)d);
  } else {
    HostWorkers::get().run(kDims, one_dim);
  }
  return out;
}

struct PassPlan {
  bool rows_mode = false;
  const uint8_t* env_blob = nullptr;  // host copy of the environment's blob (DevHeader first)
  NfaPass nfa{};                      // filled by ensure_nfa when the pass has NFA elements
  uint32_t nfa_threads = 0;
  std::vector<SlotChunk> chunks;
  std::vector<std::pair<uint32_t, uint32_t>> launches;  // chunk ranges [first, last)
  std::vector<TileArgs> tiles;                          // one per launch (record pointers filled at upload)
  std::vector<uint8_t> slot_blob;                       // the chunks' records, concatenated
  std::vector<uint32_t> slot_at;                        // offset of each chunk's record in slot_blob
  TileArgs geom;  // the first region's geometry (the fields every region shares)
  EvalArgs args;
  uint32_t grid = 0;
  // tile geometry per region of the device rows: one, or the light and heavy regions of a split
  // batch (DeviceBatch::split), each with its own capacities, LDS layout and grid; `tiles` holds
  // region k's launches at [k * launches.size(), (k + 1) * launches.size())
  struct Region {
    uint64_t lo = 0, hi = 0;
    TileArgs geom;
    uint32_t grid = 0;
    bool dyn = true;  // the dynamic tile schedule (sched_dynamic), else the strided one
  };
  std::vector<Region> regions;
  uint32_t nwide = 0;
  std::vector<int32_t> wide_policy;
  std::vector<uint32_t> rowcol;  // rows mode
  uint64_t wide_cap_per_row = 0;
  double evaluate_bytes = 0;
  // wide policy groups of the pass (> 64 members or deep stacks): their combine records, jump
  // code, member slot -> member-pass column maps, the member-pass policy list
  struct Wide {
    std::vector<WideGroupArgs> groups;
    std::vector<int32_t> policy;
    std::vector<uint8_t> progs;
    std::vector<uint32_t> midx;
    std::vector<int32_t> members;
    // split group members (env.cpp split_policy): records of kind 2 / 3 after the groups' own in
    // the upload; a member slot's midx entry is kSplitMember | record index
    std::vector<WideGroupArgs> aux;
    uint32_t cause_stride = 0, stack_words = 0;
  } wide;
};

// The wide groups among the pass's columns (plan->wide): column ids are the output column
// (all pairs) or the rows-mode column code ((chunk << 16) | column, as rowcol holds).
void plan_wide_groups(const Env& E, const std::vector<int32_t>& list, const std::vector<uint32_t>* rows_code,
                      int origin, PassPlan* plan) {
  PassPlan::Wide& W = plan->wide;
  W = PassPlan::Wide{};
  std::map<int32_t, uint32_t> mcol, aux_of;
  auto member_col = [&](int32_t m) {
    auto it = mcol.find(m);
    if (it == mcol.end()) {
      it = mcol.emplace(m, (uint32_t)W.members.size()).first;
      W.members.push_back(m);
    }
    return it->second;
  };
  // a group member that is split: its word is combined from its parts' words where the group
  // reads it (before, the member pass left a placeholder and the group rejected)
  auto split_member = [&](int32_t m) -> uint32_t {
    auto it = aux_of.find(m);
    if (it != aux_of.end()) return it->second;
    const PolicyRec& M = E.pol[(size_t)m];
    WideGroupArgs a;
    memset(&a, 0, sizeof(a));
    while (W.progs.size() % 4) W.progs.push_back(0);
    a.prog_off = (uint32_t)W.progs.size();
    a.prog_len = (uint32_t)(M.part_off.size() * 4);
    W.progs.insert(W.progs.end(), (const uint8_t*)M.part_off.data(), (const uint8_t*)(M.part_off.data() + M.part_off.size()));
    a.kind = M.family == FAM_CAPABILITIES ? 3u : 2u;
    a.nmem = (uint32_t)M.parts.size();
    a.okw = finish_word(M.mode, M.allowed_to_mutate, origin, 0, 0, false);
    a.mutw = finish_word(M.mode, M.allowed_to_mutate, origin, 0, 0, true);
    a.rejb = finish_word(M.mode, M.allowed_to_mutate, origin, 1, 0, false) & ~0xff00u;
    std::vector<uint32_t> cols;
    for (int32_t q : M.parts) cols.push_back(member_col(q));
    a.midx_off = (uint32_t)W.midx.size();
    W.midx.insert(W.midx.end(), cols.begin(), cols.end());
    const uint32_t k = (uint32_t)W.aux.size();
    W.aux.push_back(a);
    aux_of.emplace(m, k);
    return k;
  };
  for (uint32_t j = 0; j < (uint32_t)list.size(); ++j) {
    const PolicyRec& P = E.pol[(size_t)list[j]];
    const bool split = !P.parts.empty() && !P.init_error;
    if (!split && (!P.is_group || P.init_error || !P.prog.valid || P.prog.eval_error || !P.prog.wide)) continue;
    WideGroupArgs g;
    memset(&g, 0, sizeof(g));
    while (W.progs.size() % 4) W.progs.push_back(0);
    g.prog_off = (uint32_t)W.progs.size();
    if (split) {  // the parts' index offsets (u32 each)
      g.prog_len = (uint32_t)(P.part_off.size() * 4);
      W.progs.insert(W.progs.end(), (const uint8_t*)P.part_off.data(), (const uint8_t*)(P.part_off.data() + P.part_off.size()));
    } else {
      g.prog_len = (uint32_t)P.prog.code.size();
      W.progs.insert(W.progs.end(), P.prog.code.begin(), P.prog.code.end());
    }
    g.col = rows_code ? (*rows_code)[j] : j;
    const std::vector<int32_t>& mem = split ? P.parts : P.members;
    g.nmem = (uint32_t)mem.size();
    std::vector<uint32_t> cols;
    for (int32_t m : mem) {
      const PolicyRec& M = E.pol[(size_t)m];
      cols.push_back(!split && !M.parts.empty() && !M.init_error ? kSplitMember | split_member(m) : member_col(m));
    }
    g.midx_off = (uint32_t)W.midx.size();
    W.midx.insert(W.midx.end(), cols.begin(), cols.end());
    if (split) {  // a plain policy's words (slotplan.cpp CK_PLAIN), the reason and argument from its parts
      g.kind = P.family == FAM_CAPABILITIES ? 3u : 2u;
      g.okw = finish_word(P.mode, P.allowed_to_mutate, origin, 0, 0, false);
      g.mutw = finish_word(P.mode, P.allowed_to_mutate, origin, 0, 0, true);
      g.rejb = finish_word(P.mode, P.allowed_to_mutate, origin, 1, 0, false) & ~0xff00u;
      g.cause_words = 0;
    } else {
      g.okw = finish_word(P.mode, 0, origin, 0, 0, false);
      g.rejb = finish_word(P.mode, 0, origin, KW_R_GROUP, kArgWide, false);
      g.errw = finish_word(P.mode, 0, origin, KW_R_GROUP_EXPR, 0, false);
      g.kind = P.prog.script ? 1u : 0u;
      g.cause_words = (g.nmem + 63u) / 64u;
    }
    // all pairs: every wide column has its own words in a row; rows mode: a row has one column
    g.cause_off = rows_code ? 0u : W.cause_stride;
    W.cause_stride = rows_code ? std::max(W.cause_stride, g.cause_words) : W.cause_stride + g.cause_words;
    if (!split)
      W.stack_words = std::max<uint32_t>(W.stack_words, P.prog.script ? (uint32_t)run_script_words(P.prog.code.data())
                                                                       : (P.prog.depth + 63u) / 64u);
    W.groups.push_back(g);
    W.policy.push_back(list[j]);
  }
}

// The rows the device holds, in device order: the reordered copy of a split batch, else the batch.
const Batch& dev_rows(const kw_batch* kb) { return kb->dev && kb->dev->dev_b ? *kb->dev->dev_b : kb->b; }

// Plan one pass: slot-plan chunks of the policy list, the launches they take, the tile geometry
// and LDS layout, the kernel arguments.
int plan_pass(const kw_env* env, kw_batch* kb, const int32_t* pols, uint32_t npol, const int32_t* row_policy,
              int origin, PassPlan* plan) {
  const Env& E = env->e;
  DeviceBatch& D = *kb->dev;
  const Batch& B = dev_rows(kb);
  const DevHeader* H = (const DevHeader*)E.blob.data();
  plan->env_blob = E.blob.data();
  plan->rows_mode = row_policy != nullptr;
  static const bool pdbg = getenv("KW_BULK_DEBUG") && atoi(getenv("KW_BULK_DEBUG")) != 0;  // diagnostics
  const auto pt0 = std::chrono::steady_clock::now();
  auto pms = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - pt0).count(); };
  // ---- the columns of the pass and their slot-plan chunks
  std::vector<int32_t> list;
  std::map<int32_t, uint32_t> col_of;  // rows mode: policy -> column
  if (plan->rows_mode) {
    for (uint64_t r = 0; r < B.n; ++r)
      if (col_of.emplace(row_policy[r], (uint32_t)list.size()).second) list.push_back(row_policy[r]);
  } else {
    list.assign(pols, pols + npol);
  }
  Status st = build_slot_chunks(E, list.data(), (uint32_t)list.size(), origin, plan->rows_mode, &plan->chunks);
  if (!st.ok()) return st.code;
  if (!plan->rows_mode) plan_wide_groups(E, list, nullptr, origin, plan);
  if (plan->rows_mode) {
    std::vector<uint32_t> at(list.size());
    for (uint32_t c = 0; c < plan->chunks.size(); ++c)
      for (uint32_t j = 0; j < plan->chunks[c].ncols; ++j) at[plan->chunks[c].col0 + j] = (c << 16) | j;
    plan_wide_groups(E, list, &at, origin, plan);
    plan->rowcol.resize(B.n);  // (in device-row order)
    for (uint64_t r = 0; r < B.n; ++r) plan->rowcol[r] = at[col_of[row_policy[D.split ? D.perm[r] : r]]];
  }
  plan->nwide = 0;
  plan->wide_policy.clear();
  for (const SlotChunk& c : plan->chunks) {
    const ColInfo* ci = (const ColInfo*)(c.rec.data() + ((const SlotHdr*)c.rec.data())->o_cols);
    for (uint32_t j = 0; j < c.ncols; ++j)
      if (ci[j].wide != ~0u) plan->wide_policy.push_back((int32_t)ci[j].policy);
  }
  plan->nwide = plan->rows_mode ? (plan->wide_policy.empty() ? 0u : 1u) : (uint32_t)plan->wide_policy.size();

  const double t_slots = pdbg ? pms() : 0.0;
  // ---- what the chunks classify
  uint32_t need = 0;
  bool any_ctr = false, any_caps = false, any_trs = false, any_lbl = false, any_ctr_fam = false;
  uint32_t nslots = 1;
  for (const SlotChunk& c : plan->chunks) {
    const SlotHdr& h = *(const SlotHdr*)c.rec.data();
    if (h.ns) need |= 1u << S_NS;
    if (h.trs) need |= 1u << S_IMG, any_trs = true;
    if (h.aa) need |= 1u << S_AA;
    if (h.caps) need |= (1u << S_CAPADD) | (1u << S_CAPDROP), any_caps = true;
    if (h.lbl) {
      need |= 1u << S_LK;
      if (H->kv_off) need |= 1u << S_LV;
      any_lbl = true;
    }
    any_ctr = any_ctr || (h.priv[0] | h.priv[1] | h.priv[2] | h.priv[3] | h.caps | h.aa | h.trs) != 0;
    any_ctr_fam = any_ctr_fam || (h.priv[0] | h.priv[1] | h.priv[2] | h.priv[3] | h.caps | h.aa) != 0;
    nslots = std::max(nslots, c.nslots);
  }
  if (H->bypass_cls) need |= 1u << S_NS;
  ImgLayout il{0, 0, 0};
  if (any_trs) {
    il.nreg = (H->col[COL_REG].lit_off ? 1u : 0u) + H->col[COL_REG].ndfa;
    il.ntag = (H->col[COL_TAG].lit_off ? 1u : 0u) + H->col[COL_TAG].ndfa;
    il.nimg = H->col[COL_IMG].ndfa;
  }
  const uint32_t nlv = (need & (1u << S_LV)) ? H->col[COL_LV].ndfa : 0u;

  // ---- the classifiers the pass stages: literal tables, DFA chains, the per-key value region
  struct Stage {
    uint32_t blob, bytes;
  };
  std::vector<Stage> stages;
  uint32_t lit_of[NCOL] = {}, dfa_of[NCOL] = {};
  auto stage_col = [&](Col c, bool lit, bool dfa) {
    const DevCol& dc = H->col[c];
    if (lit && dc.lit_off) {
      lit_of[c] = (uint32_t)stages.size() + 1;
      stages.push_back({dc.lit_off, dc.lit_bytes});
    }
    if (dfa && dc.dfa_off) {
      dfa_of[c] = (uint32_t)stages.size() + 1;
      stages.push_back({dc.dfa_off, dc.dfa_bytes});
    }
  };
  if (need & (1u << S_NS)) stage_col(COL_NS, true, false);
  if (need & (1u << S_IMG)) {
    stage_col(COL_REG, true, true);
    stage_col(COL_TAG, true, true);
    stage_col(COL_IMG, false, true);
  }
  if (need & (1u << S_AA)) stage_col(COL_AA, true, false);
  if (need & (1u << S_CAPADD)) stage_col(COL_CAP, true, false);
  if (need & (1u << S_LK)) stage_col(COL_LK, true, false);
  uint32_t kv_stage = 0;
  static const bool kv_global = getenv("KW_KV_GLOBAL") && atoi(getenv("KW_KV_GLOBAL")) != 0;  // A/B knob
  if ((need & (1u << S_LV)) && !kv_global) {
    kv_stage = (uint32_t)stages.size() + 1;
    stages.push_back({H->kv_off, H->kv_bytes});
  }
  uint32_t table_bytes = 0;
  for (const Stage& s : stages) table_bytes += (s.bytes + 15u) & ~15u;

  // ---- launches: chunks grouped so tables + staged records fit the per-workgroup budget; a pass
  //      whose tables or a single chunk alone exceed it reads them from global memory (L2)
  bool ldst = table_bytes <= kTableBudget;
  for (const SlotChunk& c : plan->chunks) ldst = ldst && table_bytes + c.staged <= kTableBudget;
  if (const char* g = getenv("KW_GLOBAL_TABLES")) ldst = ldst && atoi(g) == 0;  // diagnostics / tests
  plan->launches.clear();
  uint32_t area = ldst ? table_bytes : 0;
  for (uint32_t c = 0; c < plan->chunks.size();) {
    uint32_t e = c, bytes = 0;
    while (e < plan->chunks.size() && e - c < kMaxChunks &&
           (!ldst || table_bytes + bytes + plan->chunks[e].staged <= kTableBudget))
      bytes += plan->chunks[e++].staged;
    plan->launches.push_back({c, e});
    if (ldst) area = std::max(area, table_bytes + bytes);
    c = e;
  }

  // ---- tile geometry and LDS layout
  TileArgs& T = plan->geom;
  auto align = [](uint32_t x) { return (x + 15u) & ~15u; };
  uint32_t rows = kSlotRows;  // the tile height the layout below is computed for
  const uint32_t vw_stride = nslots | 1u;  // odd stride: lanes (requests) spread over the banks
  const uint32_t nim = il.n();
  auto layout = [&](const TileStats& ts) -> uint32_t {
    memset(&T, 0, sizeof(T));
    double scale = 1.0;
    for (;;) {
      const uint32_t cmax = std::min<uint32_t>(kMaxTileEntities, (uint32_t)std::max(1.0, scale * ts.ctr));
      const uint32_t kmax = std::min<uint32_t>(kMaxTileEntities, (uint32_t)std::max(1.0, scale * std::max(ts.kadd, ts.kdrop)));
      const uint32_t lmax = std::min<uint32_t>(kMaxTileEntities, (uint32_t)std::max(1.0, scale * ts.lbl));
      uint32_t off = 16 + align(area);
      auto take = [&](uint32_t bytes) {
        const uint32_t o = off;
        off = align(off + bytes);
        return o;
      };
      T.o_rf = take(rows);
      T.o_coff = take((rows + 1) * 4);
      T.o_loff = take((rows + 1) * 4);
      T.o_cflags = take(cmax + 8);  // staged from the dword holding the first flag
      T.o_cadd = take((cmax + 1) * 4);
      T.o_cdrop = take((cmax + 1) * 4);
      T.o_ns = take(rows * 2);
      T.o_aa = take((need & (1u << S_AA)) ? cmax * 2 : 0);
      T.o_img = take((need & (1u << S_IMG)) ? cmax * nim * 2 : 0);
      T.o_capadd = take(any_caps ? kmax * 2 : 0);
      T.o_capdrop = take(any_caps ? kmax * 2 : 0);
      T.o_lk = take(any_lbl ? lmax * 2 : 0);
      T.o_lv = take(any_lbl ? lmax * nlv * 2 : 0);
      T.o_vadd = take(any_caps ? kmax * 8 : 0);
      T.o_vl = take(any_lbl ? lmax * 8 : 0);
      T.o_vc = take(cmax * 8);
      T.o_vtr = take(any_trs ? cmax * 8 : 0);
      T.o_own_c = take(cmax);
      T.o_own_l = take(lmax);
      T.o_rej = take(rows * 8);
      T.o_mut = take(rows * 8);
      T.o_byp = take(rows);
      T.o_sa = take(NSTR * 4);
      T.o_nx = take(16);  // (kernels.hpp TileArgs::o_nx)
      T.o_desc = take(2 * sizeof(TileDesc));
      T.o_pf = l2_prefetch() ? take(4 * kPfLanes) : 0u;
      // union: the staged strings (P0-P1) and the violation words (P2-P3)
      const uint32_t u0 = off;
      uint32_t su = u0;
      for (int m = 0; m < (int)NSTR; ++m) {
        T.o_so[m] = T.o_sb[m] = T.sb_cap[m] = 0;
        if (!(need & (1u << m))) continue;
        const uint32_t cnt = m == S_NS ? rows : (m == S_CAPADD || m == S_CAPDROP) ? kmax : (m == S_LK || m == S_LV) ? lmax : cmax;
        T.o_so[m] = su;
        su = align(su + (cnt + 1) * 4);
        T.sb_cap[m] = align((uint32_t)std::min(16384.0, std::max(16.0, scale * ts.bytes[m])));  // longer tiles split
        T.o_sb[m] = su;
        su = align(su + T.sb_cap[m] + 48);  // slack: batched dword reads may run <= 36 bytes past a string start
      }
      T.o_vw = u0;
      T.vw_stride = vw_stride;
      off = std::max(su, align(u0 + rows * vw_stride * 4));
      if (off > kTileLdsBudget && scale > 1e-5) {  // capacities shrink until the layout fits; bigger tiles split
        scale *= 0.8;
        continue;
      }
      T.rows = rows;
      T.cmax = cmax;
      T.kmax = kmax;
      T.lmax = lmax;
      T.lds_bytes = off;
      break;
    }
    return T.lds_bytes;
  };
  auto per_cu = [](uint32_t b) { return std::min<uint32_t>(2048 / kSlotThreads, lds_workgroups_per_cu(b)); };
  // Capacities at a tile height: the highest occupancy (workgroups per CU, LDS-bound) whose layout
  // splits at most 2 % of the tiles (a tile beyond the capacities runs as halves, upload_tile_descs),
  // over per-dimension quantiles of the tile needs; at a given occupancy the largest capacities
  // (fewest split tiles). Chosen once per batch, tile height and layout signature.
  const uint64_t key = ((uint64_t)area << 40) ^ ((uint64_t)nslots << 20) ^ ((uint64_t)nim << 12) ^ ((uint64_t)nlv << 8) ^ need;
  uint64_t rlo = 0, rhi = B.n;  // the region being planned
  auto plan_rows = [&](uint32_t r) -> DeviceBatch::RowsPlan& {
    DeviceBatch::RowsPlan* R = nullptr;
    for (auto& x : D.rows_plans)
      if (x.rows == r && x.lo == rlo && x.hi == rhi) R = &x;
    if (!R) {
      D.rows_plans.emplace_back();
      R = &D.rows_plans.back();
      R->rows = r;
      R->lo = rlo;
      R->hi = rhi;
      R->stride = 0;
    }
    if (R->stride == 0 || R->stride > D.needs_stride) {  // (a sampled plan is refined when a pass wants every tile)
      R->stride = std::max<uint32_t>(1, D.needs_stride);
      R->need = tile_needs(B, r, R->stride, rlo, rhi);
      R->q = tile_quantiles(R->need, kTileQuantiles, sizeof(kTileQuantiles) / sizeof(kTileQuantiles[0]));
      R->cap_choice = -1;
    }
    rows = r;
    if (R->cap_choice < 0 || R->cap_key != key) {
      const uint64_t ntl = R->need.size();
      int best = 0;
      uint32_t best_cu = 0, best_lds = 0;
      const double max_split = getenv("KW_TILE_SPLIT") ? atof(getenv("KW_TILE_SPLIT")) : 0.02;  // A/B knob
      for (int k = 0; k < (int)R->q.size(); ++k) {
        const uint32_t cu = per_cu(layout(R->q[k]));
        if (T.lds_bytes > kTileLdsBudget) continue;
        uint64_t over = 0;  // tiles beyond these capacities (split by the descriptors' fit test)
        for (const TileStats& x : R->need) {
          bool o = x.ctr > T.cmax || x.lbl > T.lmax || x.kadd > T.kmax || x.kdrop > T.kmax;
          for (int m = 0; m < (int)NSTR && !o; ++m) o = T.sb_cap[m] && x.bytes[m] > T.sb_cap[m];
          over += o;
        }
        if (getenv("KW_TILE_DEBUG") && (atoi(getenv("KW_TILE_DEBUG")) & 256))
          fprintf(stderr, "[kw tile] rows=%u candidate q=%g lds=%u wg/cu=%u split=%llu/%llu\n", r, kTileQuantiles[k], T.lds_bytes, cu,
                  (unsigned long long)over, (unsigned long long)ntl);
        if (k > 0 && (double)over > max_split * (double)ntl) continue;
        if (cu > best_cu) {
          best = k;
          best_cu = cu;
          best_lds = T.lds_bytes;
        }
      }
      R->cap_key = key;
      R->cap_choice = best;
      R->cap_cu = best_cu;
      R->cap_lds = best_lds;
    }
    return *R;
  };
  // Tile height: KW_SLOT_ROWS when forced; else kSlotRows, or a taller tile (128 down to 96 rows)
  // when the batch has at least 4 tiles per workgroup slot, the taller layout still keeps 4
  // workgroups per CU (its LDS estimated from the 64-row layout first: the per-request part scales
  // with the height), and at most KW_ROUND_SPLIT (2 %) of its tiles hold more items in one P1
  // segment (labels, capability strings, containers / images) than the workgroup has lanes: such a
  // tile sends one wave through the segment twice, and its phase waits for that wave (r03: half of
  // C2 / C3's 128-row tiles had more than 256 images). Taller tiles amortise the per-tile latency
  // (staging, barriers) where the per-request LDS is small: C2 -12 %, C3 -25 % at 128 rows (r02);
  // the C4-C6 layouts need 64 rows for 4 workgroups per CU (r02 sweeps). Per region: a split
  // batch's light region takes the capacities (and occupancy) of its own tiles.
  std::vector<std::pair<uint64_t, uint64_t>> bounds{{0, B.n}};
  if (D.split && D.split < B.n) bounds = {{0, D.split}, {D.split, B.n}};
  plan->regions.clear();
  for (const auto& [lo, hi] : bounds) {
  rlo = lo;
  rhi = hi;
  const DeviceBatch::RowsPlan* pick = nullptr;
  const double round_split = getenv("KW_ROUND_SPLIT") ? atof(getenv("KW_ROUND_SPLIT")) : 0.02;  // A/B knob
  auto two_rounds = [&](const DeviceBatch::RowsPlan& R) {  // share of tiles with a segment beyond one round
    uint64_t over = 0;
    for (const TileStats& x : R.need) {
      uint32_t seg = 0;
      if (any_lbl) seg = std::max(seg, x.lbl);
      if (any_caps) seg = std::max(seg, x.kadd + x.kdrop);
      if (any_ctr || (need & (1u << S_IMG))) seg = std::max(seg, x.ctr);
      over += seg > kSlotThreads;
    }
    return R.need.empty() ? 0.0 : (double)over / (double)R.need.size();
  };
  if (const uint32_t f = slot_rows_forced()) {
    pick = &plan_rows(f);
  } else if (lo > 0) {
    // the heavy region of a split batch: the tallest tile height whose capacities reach the
    // kernel's register-bound occupancy (<= 128 VGPRs: 4 workgroups of 256 threads per CU), else
    // the one with the most workgroups per CU. r05 C5 sweep (profiles/r05_split_ab.txt): at equal
    // occupancy taller tiles win (heavy > 5: 12 rows 6.31 ms, 10 rows 6.85), and a layout one
    // workgroup per CU short loses 10-15 % whatever its height.
    if (const uint32_t h = heavy_rows()) {
      pick = &plan_rows(h);
    } else {
      for (uint32_t r : {64u, 48u, 40u, 32u, 28u, 24u, 20u, 16u, 14u, 12u, 10u, 8u}) {
        const DeviceBatch::RowsPlan& R = plan_rows(r);
        if (!pick || R.cap_cu > pick->cap_cu) pick = &R;
        if (R.cap_cu >= 4) break;
      }
    }
  } else {
    const DeviceBatch::RowsPlan& base = plan_rows(kSlotRows);
    pick = &base;
    const uint32_t fixed = 16 + align(area), per64 = base.cap_lds > fixed ? base.cap_lds - fixed : 0u;
    for (uint32_t r : {128u, 120u, 112u, 104u, 96u}) {
      const uint64_t est = fixed + (uint64_t)per64 * r / kSlotRows;
      if (getenv("KW_TILE_DEBUG") && (atoi(getenv("KW_TILE_DEBUG")) & 256))
        fprintf(stderr, "[kw tile] rows=%u estimated lds=%llu (64-row layout %u, fixed %u) region rows %llu\n", r,
                (unsigned long long)est, base.cap_lds, fixed, (unsigned long long)(rhi - rlo));
      if (per_cu((uint32_t)std::min<uint64_t>(est, 1u << 30)) < 4 || rhi - rlo < (uint64_t)r * 4 * 256 * 4) continue;
      const DeviceBatch::RowsPlan& R = plan_rows(r);
      const double tr = two_rounds(R);
      if (getenv("KW_TILE_DEBUG") && (atoi(getenv("KW_TILE_DEBUG")) & 256))
        fprintf(stderr, "[kw tile] rows=%u workgroups/CU %u, tiles with a segment beyond %u items %.4f\n", r, R.cap_cu,
                kSlotThreads, tr);
      if (R.cap_cu >= 4 && tr <= round_split) {
        pick = &R;
        break;
      }
    }
  }
  rows = pick->rows;
  if (pdbg) fprintf(stderr, "[kw plan] slot chunks %.2f ms, tile needs + capacities %.2f ms\n", t_slots, pms() - t_slots);
  if (const char* fq = getenv("KW_TILE_QUANTILE"))  // tests / diagnostics: force the capacity quantile
    layout(tile_quantile(pick->need, atof(fq)));
  else
    layout(pick->q[pick->cap_choice]);
  if (T.lds_bytes > kTileLdsBudget) return KW_E_ARG;  // policy list too large for one tile
  // next-tile L2 prefetch (compiled in with KW_PREFETCH, kernels.hpp): a gain where several small
  // tiles share a CU, a loss where two large ones do (C5: +2.7 %; r02 A/B); off by default since the
  // descriptor moved to LDS (r02 s60)
  T.prefetch = l2_prefetch() && per_cu(T.lds_bytes) >= 3 ? 1u : 0u;
  // predecessor ranges four loads a round where tiles hold many containers per request (C5 -6 %;
  // C4, two per request, keeps the plain loops: r02 s80)
  T.ctr_ranges = T.cmax > 4u * T.rows ? 1u : 0u;
  PassPlan::Region g;
  g.lo = lo;
  g.hi = hi;
  g.geom = T;
  const uint64_t nt = (hi - lo + T.rows - 1) / T.rows;
  g.grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(nt, 256ull * per_cu(T.lds_bytes)));
  g.dyn = sched_dynamic(nt, g.grid, ldst);
  plan->regions.push_back(g);
  }
  bool any_grp = false;
  for (const SlotChunk& c : plan->chunks) any_grp = any_grp || c.groups;
  // the fields every region shares
  for (PassPlan::Region& rg : plan->regions) {
  T = rg.geom;
  T.feat = ((need & (1u << S_IMG)) ? kFeatImg : 0u) | (any_lbl ? kFeatLbl : 0u) | (any_ctr_fam ? kFeatCtr : 0u) |
           (any_grp ? kFeatGrp : 0u);
  // NFA elements among the classifiers the pass reads: the one instantiation that reads their classes
  const bool nfa_img = (need & (1u << S_IMG)) &&
                       ((H->col[COL_REG].flags | H->col[COL_TAG].flags | H->col[COL_IMG].flags) & 1u);
  const bool nfa_lv = (need & (1u << S_LV)) && (H->col[COL_LV].flags & 1u);
  if (nfa_img || nfa_lv) T.feat = kFeatAll | kFeatNfa;
  // many containers per request (C5's heavy region): the wave-scan instantiation (kernels.hpp kFeatRng)
  if (T.ctr_ranges && ldst && T.feat == (kFeatLbl | kFeatCtr)) T.feat |= kFeatRng;
  T.il = il;
  T.nlv = nlv;
  T.need = need;
  T.lds_tables = ldst ? 1u : 0u;
  T.nlk = H->col[COL_LK].nclass;
  T.bypass_cls = H->bypass_cls;
  T.docker_io_cls = H->docker_io_cls;
  T.latest_cls = H->latest_cls;
  T.rows_mode = plan->rows_mode ? 1u : 0u;
  for (int m = 0; m < (int)NSTR; ++m) {
    T.s_off[m] = D.str[m].off;
    T.s_bytes[m] = D.str[m].bytes;
  }
  // classifiers: blob offsets, and their LDS positions when staged
  {
    uint32_t at = 16;
    std::vector<uint32_t> lds_at(stages.size());
    for (size_t k = 0; k < stages.size(); ++k) {
      lds_at[k] = at;
      at += (stages[k].bytes + 15u) & ~15u;
    }
    T.nstage = 0;
    if (ldst)
      for (size_t k = 0; k < stages.size(); ++k) {
        T.stage_blob[T.nstage] = stages[k].blob;
        T.stage_lds[T.nstage] = lds_at[k];
        T.stage_bytes[T.nstage] = (stages[k].bytes + 15u) & ~15u;
        ++T.nstage;
      }
    for (int c = 0; c < (int)NCOL; ++c) {
      if (lit_of[c]) {
        T.lit_blob[c] = stages[lit_of[c] - 1].blob;
        T.lit_lds[c] = lds_at[lit_of[c] - 1];
      }
      if (dfa_of[c]) {
        T.dfa_blob[c] = stages[dfa_of[c] - 1].blob;
        T.dfa_lds[c] = lds_at[dfa_of[c] - 1];
      }
    }
    if (kv_stage) {
      T.kv_blob = stages[kv_stage - 1].blob;
      T.kv_lds = ldst ? lds_at[kv_stage - 1] : 0u;
    } else if (need & (1u << S_LV)) {  // the value DFAs read from the blob (global memory, L1/L2)
      T.kv_blob = H->kv_off;
      T.kv_lds = 0;
    }
  }
  if (const char* dbg = getenv("KW_TILE_DEBUG")) T.debug = (uint32_t)atoi(dbg);  // phase ablation (diagnostics)
  if (T.debug & 256u)
    fprintf(stderr, "[kw tile] lds_tables=%u rows=%u cmax=%u kmax=%u lmax=%u lds=%u area=%u (classifiers %u) chunks=%zu launches=%zu nim=%u nlv=%u\n",
            T.lds_tables, T.rows, T.cmax, T.kmax, T.lmax, T.lds_bytes, area, table_bytes, plan->chunks.size(), plan->launches.size(), nim,
            nlv);
  if (T.debug & 256u) {
    for (size_t k = 0; k < stages.size(); ++k) fprintf(stderr, "[kw tile]   classifier stage %zu: %u bytes\n", k, stages[k].bytes);
    // the tile's LDS regions (bytes): per-request state, entity classes and sets, the strings / violation-words union
    uint32_t so = 0, sb = 0;
    for (int m = 0; m < (int)NSTR; ++m)
      if (T.o_sb[m]) so += T.o_sb[m] - T.o_so[m], sb += T.sb_cap[m] + 48;
    fprintf(stderr,
            "[kw tile]   layout: headers %u | classes ns %u aa %u img %u caps %u lk %u lv %u | sets vadd %u vl %u vc %u vtr %u | "
            "owners %u | rej/mut/byp %u | union at %u: string offsets %u + bytes %u, violation words %u | total %u\n",
            T.o_ns - T.o_rf, T.o_aa - T.o_ns, T.o_img - T.o_aa, T.o_capadd - T.o_img, T.o_lk - T.o_capadd, T.o_lv - T.o_lk,
            T.o_vadd - T.o_lv, T.o_vl - T.o_vadd, T.o_vc - T.o_vl, T.o_vtr - T.o_vc, T.o_own_c - T.o_vtr, T.o_rej - T.o_own_c,
            T.o_sa - T.o_rej, T.o_vw, so, sb, T.rows * T.vw_stride * 4, T.lds_bytes);
  }
  rg.geom = T;
  }
  T = plan->regions[0].geom;

  // ---- per-launch TileArgs (record pointers filled in at upload, run_pass), region by region
  plan->slot_blob.clear();
  plan->slot_at.clear();
  for (const SlotChunk& c : plan->chunks) {
    plan->slot_at.push_back((uint32_t)plan->slot_blob.size());
    plan->slot_blob.insert(plan->slot_blob.end(), c.rec.begin(), c.rec.end());
  }
  plan->tiles.clear();
  for (const PassPlan::Region& rg : plan->regions)
  for (const auto& [c0, c1] : plan->launches) {
    TileArgs t = rg.geom;
    t.nchunk = c1 - c0;
    uint32_t at = 16 + table_bytes;
    for (uint32_t k = 0; k < t.nchunk; ++k) {
      const SlotChunk& c = plan->chunks[c0 + k];
      ChunkArgs& ca = t.chunk[k];
      memset(&ca, 0, sizeof(ca));
      ca.o_lds = ldst ? at : 0u;
      at += c.staged;
      ca.col0 = c.col0;
      ca.ncols = c.ncols;
      ca.vec4 = (!plan->rows_mode && npol % 4u == 0 && c.col0 % 4u == 0 && c.ncols % 4u == 0) ? 1u : 0u;
      ca.init = ((const SlotHdr*)c.rec.data())->init;
    }
    plan->tiles.push_back(t);
  }

  // ---- evaluation arguments
  EvalArgs& A = plan->args;
  memset(&A, 0, sizeof(A));
  A.blob = (const uint8_t*)E.d_blob;
  A.nrows = B.n;
  A.npol = plan->rows_mode ? 1u : npol;
  A.origin = origin;
  A.req_flags = D.req_flags;
  A.ctr_off = D.ctr_off;
  A.lbl_off = D.lbl_off;
  A.ctr_flags = D.ctr_flags;
  A.capadd_off = D.capadd_off;
  A.capdrop_off = D.capdrop_off;
  A.out = D.verdicts;
  A.nwide = plan->nwide;
  plan->wide_cap_per_row = plan->rows_mode ? 1u : npol;
  // every column the kernel dereferences must be present (a null column is a device fault)
  if (!A.req_flags || !A.ctr_off || !A.lbl_off || !A.ctr_flags || !A.capadd_off || !A.capdrop_off || !A.out) return KW_E_ARG;
  for (int m = 0; m < (int)NSTR; ++m)
    if ((need & (1u << m)) && (!T.s_off[m] || !T.s_bytes[m])) return KW_E_ARG;

  // algorithmic bytes: request headers once, the entity columns and strings the policies read, and
  // the verdict words written
  const double n = (double)B.n;
  double eb = n * (1 + 4 + 4) + 4.0 * n * (double)A.npol;
  if (any_ctr) eb += (double)B.containers() * 1.0;
  if (any_caps) eb += (double)B.containers() * 8.0;
  for (int m = 0; m < (int)NSTR; ++m)
    if (need & (1u << m)) eb += (double)D.str[m].nbytes + 4.0 * (double)D.str[m].n;
  plan->evaluate_bytes = eb;

  plan->grid = plan->regions[0].grid;
  return KW_OK;
}

// Tile descriptors (kernels.hpp TileDesc) and the overflow list of one plan geometry, built from the
// host copy of the batch and uploaded once; reused while the geometry stays the same.
// The descriptors of tiles [t0, t1) of geometry T over rows [lo, hi), in row order, and the requests that exceed the
// capacities alone (overflow); a run that does not fit is halved until its parts do. Tiles in ranges
// of `range` on the host workers. KW_E_ARG when an overflow request index exceeds u32.
int build_descs(const Batch& B, const TileArgs& T, uint64_t lo, uint64_t hi, uint64_t t0, uint64_t t1, uint64_t range,
                std::vector<TileDesc>* desc, std::vector<uint32_t>* ovf) {
  // descriptor of requests [r0, r1); false when it exceeds the capacities
  auto make = [&](uint64_t r0, uint64_t r1, TileDesc* dp) {
    TileDesc& d = *dp;
    memset(&d, 0, sizeof(d));
    d.r0lo = (uint32_t)r0;
    d.r0hi = (uint32_t)(r0 >> 32);
    d.nr = (uint32_t)(r1 - r0);
    d.cb = B.ctr_off[r0];
    d.ce = B.ctr_off[r1];
    d.lb = B.lbl_off[r0];
    d.le = B.lbl_off[r1];
    d.kab = B.capadd_off[d.cb];
    d.kae = B.capadd_off[d.ce];
    d.kdb = B.capdrop_off[d.cb];
    d.kde = B.capdrop_off[d.ce];
    bool fits = d.ce - d.cb <= T.cmax && d.kae - d.kab <= T.kmax && d.kde - d.kdb <= T.kmax && d.le - d.lb <= T.lmax;
    for (int m = 0; m < (int)NSTR; ++m) {
      if (!T.o_sb[m]) continue;
      uint64_t g0, g1;
      str_range(B, m, r0, r1, &g0, &g1);
      const StrCol& c = host_str(B, m);
      d.sa[m] = c.off[g0] & ~15u;
      d.nv[m] = (((c.off[g1] + 15u) & ~15u) - d.sa[m]) / 16u;
      fits = fits && d.nv[m] * 16u <= T.sb_cap[m];
    }
    d.fits = fits ? 1u : 0u;
    return fits;
  };
  const size_t nq = (size_t)((t1 - t0 + range - 1) / range);
  std::vector<std::vector<TileDesc>> qdesc(nq);
  std::vector<std::vector<uint32_t>> qovf(nq);
  std::atomic<bool> too_far{false};
  HostWorkers::get().run(nq, [&](size_t q) {
    std::vector<std::pair<uint64_t, uint64_t>> todo;
    std::vector<TileDesc>& dv = qdesc[q];
    dv.reserve((size_t)range + range / 64);
    for (uint64_t tile = t0 + q * range, te = std::min<uint64_t>(t1, t0 + (q + 1) * range); tile < te; ++tile) {
      todo.assign(1, {lo + tile * T.rows, std::min<uint64_t>(hi, lo + (tile + 1) * T.rows)});
      while (!todo.empty()) {
        const auto [r0, r1] = todo.back();
        todo.pop_back();
        TileDesc d;
        if (make(r0, r1, &d)) {
          dv.push_back(d);
        } else if (r1 - r0 > 1) {
          const uint64_t mid = r0 + (r1 - r0) / 2;
          todo.push_back({mid, r1});
          todo.push_back({r0, mid});
        } else {
          if (r0 > 0xffffffffull) too_far = true;  // overflow list holds u32 request indices
          qovf[q].push_back((uint32_t)r0);
        }
      }
    }
  });
  if (too_far) return KW_E_ARG;
  for (size_t q = 0; q < nq; ++q) {
    desc->insert(desc->end(), qdesc[q].begin(), qdesc[q].end());
    ovf->insert(ovf->end(), qovf[q].begin(), qovf[q].end());
  }
  return KW_OK;
}

int upload_tile_descs(const Batch& B, DeviceBatch* D, const PassPlan& plan, hipStream_t s) {
  uint64_t key = 1469598103934665603ull;
  auto mix = [&](uint64_t v) { key = (key ^ v) * 1099511628211ull; };
  for (const PassPlan::Region& rg : plan.regions) {
    const TileArgs& T = rg.geom;
    mix(rg.lo);
    mix(rg.hi);
    mix(T.rows);
    mix(T.cmax);
    mix(T.kmax);
    mix(T.lmax);
    for (int m = 0; m < (int)NSTR; ++m) {
      mix(T.o_sb[m] != 0);
      mix(T.sb_cap[m]);
    }
  }
  if (D->desc && D->desc_valid && key == D->desc_key) return KW_OK;
  static const bool dbg = getenv("KW_BULK_DEBUG") && atoi(getenv("KW_BULK_DEBUG")) != 0;  // diagnostics
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<TileDesc> desc;
  std::vector<uint32_t> ovf{0};
  if (plan.regions.size() > 2) return KW_E_ARG;
  uint64_t at[2] = {0, 0}, nd[2] = {0, 0};
  for (size_t k = 0; k < plan.regions.size(); ++k) {  // region k's descriptors after region k-1's; one overflow list
    const PassPlan::Region& rg = plan.regions[k];
    const uint64_t ntiles = (rg.hi - rg.lo + rg.geom.rows - 1) / rg.geom.rows;
    at[k] = desc.size();
    desc.reserve(desc.size() + ntiles + ntiles / 64 + 1);
    if (int rc = build_descs(B, rg.geom, rg.lo, rg.hi, 0, ntiles, 4096, &desc, &ovf)) return rc;
    nd[k] = desc.size() - at[k];
  }
  ovf[0] = (uint32_t)(ovf.size() - 1);
  const auto t1 = std::chrono::steady_clock::now();
  HIPCHK(hipStreamSynchronize(s));  // a running pass may still read the previous descriptors
  D->h_desc = std::move(desc);
  D->h_ovf = std::move(ovf);
  if (int rc = ensure(&D->desc, &D->desc_cap, std::max<size_t>(D->h_desc.size(), 1))) return rc;
  if (int rc = ensure(&D->overflow, &D->overflow_cap, D->h_ovf.size())) return rc;
  if (!D->h_desc.empty())
    HIPCHK(hipMemcpyAsync(D->desc, D->h_desc.data(), D->h_desc.size() * sizeof(TileDesc), hipMemcpyHostToDevice, s));
  D->ndesc = D->h_desc.size();
  for (int k = 0; k < 2; ++k) {
    D->reg_desc[k] = at[k];
    D->reg_ndesc[k] = nd[k];
  }
  HIPCHK(hipMemcpyAsync(D->overflow, D->h_ovf.data(), D->h_ovf.size() * sizeof(uint32_t), hipMemcpyHostToDevice, s));
  D->n_overflow = D->h_ovf[0];
  D->desc_key = key;
  D->desc_valid = true;
  if (dbg)
    fprintf(stderr, "[kw descs] %zu descriptors: build %.2f ms, sync + upload %.2f ms\n", D->h_desc.size(),
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
  return KW_OK;
}

// Per-string class arrays of the overflow path (absolute entity indices), one allocation.
int ensure_overflow_classes(const Batch& B, DeviceBatch* D, const TileArgs& T, EvalArgs* A) {
  const uint64_t nim = T.il.n(), nlv = std::max<uint32_t>(T.nlv, 1);
  const uint64_t n_ns = B.n + 1, n_ctr = B.containers() + 1, n_add = B.cap_add.n() + 1, n_drop = B.cap_drop.n() + 1,
                 n_lbl = B.labels() + 1;
  const uint64_t total = n_ns + n_ctr + n_ctr * std::max<uint64_t>(nim, 1) + n_add + n_drop + n_lbl + n_lbl * nlv;
  if (int rc = ensure(&D->g_cls, &D->g_cls_cap, (size_t)total)) return rc;
  uint16_t* p = D->g_cls;
  A->g_ns = p;
  p += n_ns;
  A->g_aa = p;
  p += n_ctr;
  A->g_img = p;
  p += n_ctr * std::max<uint64_t>(nim, 1);
  A->g_capadd = p;
  p += n_add;
  A->g_capdrop = p;
  p += n_drop;
  A->g_lk = (T.need & (1u << S_LK)) ? p : nullptr;
  p += n_lbl;
  A->g_lv = p;
  return KW_OK;
}

// NFA elements of a pass (kwdev.hpp DevNfa): the class arrays the tile kernel reads and the Pike
// VMs' scratch (nfa_classify_kernel, launched first by run_pass).
int ensure_nfa(kw_batch* kb, PassPlan& plan, EvalArgs* A) {
  DeviceBatch& D = *kb->dev;
  const Batch& B = kb->b;
  const TileArgs& T = plan.geom;
  const DevHeader* H = (const DevHeader*)plan.env_blob;
  NfaPass& np = plan.nfa;
  memset(&np, 0, sizeof(np));
  np.nlv = T.nlv;
  np.nim = T.il.n();
  np.nlabels = B.labels();
  np.nctrs = B.containers();
  np.do_lv = (T.need & (1u << S_LV)) && (H->col[COL_LV].flags & 1u) && np.nlv ? 1u : 0u;
  np.do_img = (T.need & (1u << S_IMG)) && ((H->col[COL_REG].flags | H->col[COL_TAG].flags | H->col[COL_IMG].flags) & 1u) && np.nim
                  ? 1u
                  : 0u;
  if (np.do_img && D.max_image_len == 0xffffffffu) {
    uint32_t m = 0;
    for (uint64_t c = 0; c < B.containers(); ++c) m = std::max(m, B.ctr_image.off[c + 1] - B.ctr_image.off[c]);
    D.max_image_len = m;
  }
  np.nfa_words = H->nfa_words;
  np.subj_bytes = np.do_img ? ((D.max_image_len + 64u) & ~3u) : 0u;  // + "docker.io/library/" ":latest"
  np.words_per_thread = np.nfa_words + np.subj_bytes / 4u;
  const uint64_t nlv = std::max<uint32_t>(np.nlv, 1), nim = std::max<uint32_t>(np.nim, 1);
  const uint64_t n_lv = np.do_lv ? np.nlabels * nlv : 0, n_img = np.do_img ? np.nctrs * nim : 0;
  if (int rc = ensure(&D.nfa_cls, &D.nfa_cls_cap, (size_t)(n_lv + n_img + 1))) return rc;
  np.lv = D.nfa_cls;
  np.img = D.nfa_cls + n_lv;
  const uint64_t items = (np.do_lv ? np.nlabels : 0) + (np.do_img ? np.nctrs : 0);
  plan.nfa_threads = nfa_threads(items, np.words_per_thread);
  if (int rc = ensure(&D.nfa_scratch, &D.nfa_scratch_cap, (size_t)(plan.nfa_threads * np.words_per_thread + 1))) return rc;
  np.scratch = D.nfa_scratch;
  A->nfa_lv = np.do_lv ? np.lv : nullptr;
  A->nfa_img = np.do_img ? np.img : nullptr;
  return KW_OK;
}

// Everything a pass's launches need on the device before the first one: the plan's records and
// TileArgs, the rows-mode column map, tile descriptors and overflow list, schedule counters and the
// side-data buffers; *out_args: the launch arguments.
int prepare_pass(kw_batch* kb, PassPlan& plan, hipStream_t s, EvalArgs* out_args, bool descs = true) {
  DeviceBatch& D = *kb->dev;
  const Batch& B = dev_rows(kb);
  if (D.cur && D.cur != s) HIPCHK(hipStreamSynchronize(D.cur));  // order against the previous pass's stream
  D.cur = s;
  // plan upload: records, per-launch TileArgs (with their record pointers), rows-mode column map
  if (int rc = ensure(&D.d_slots, &D.d_slots_cap, plan.slot_blob.size())) return rc;
  if (int rc = ensure(&D.d_tiles, &D.d_tiles_cap, plan.tiles.size())) return rc;
  for (size_t l = 0; l < plan.tiles.size(); ++l)
    for (uint32_t k = 0; k < plan.tiles[l].nchunk; ++k)
      plan.tiles[l].chunk[k].rec = D.d_slots + plan.slot_at[plan.launches[l % plan.launches.size()].first + k];
  if (D.h_slots != plan.slot_blob || D.h_tiles.size() != plan.tiles.size() ||
      (!plan.tiles.empty() && std::memcmp(D.h_tiles.data(), plan.tiles.data(), plan.tiles.size() * sizeof(TileArgs)) != 0)) {
    HIPCHK(hipStreamSynchronize(s));  // a running pass may still read the previous plan
    D.h_slots = plan.slot_blob;
    D.h_tiles = plan.tiles;
    HIPCHK(hipMemcpyAsync(D.d_slots, D.h_slots.data(), D.h_slots.size(), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(D.d_tiles, D.h_tiles.data(), D.h_tiles.size() * sizeof(TileArgs), hipMemcpyHostToDevice, s));
  }
  EvalArgs A = plan.args;
  if (plan.rows_mode) {
    if (D.h_rowcol != plan.rowcol) {
      HIPCHK(hipStreamSynchronize(s));
      D.h_rowcol = plan.rowcol;
      if (int rc = ensure(&D.rowcol, &D.rowcol_cap, D.h_rowcol.size())) return rc;
      HIPCHK(hipMemcpyAsync(D.rowcol, D.h_rowcol.data(), D.h_rowcol.size() * 4, hipMemcpyHostToDevice, s));
    }
    A.rowcol = D.rowcol;
  }
  if (descs) {
    if (int rc = upload_tile_descs(B, &D, plan, s)) return rc;
  } else {  // the caller builds and uploads descriptors per row chunk (kw_validate_host)
    HIPCHK(hipStreamSynchronize(s));  // a running pass may still read the previous descriptors
    D.desc_valid = false;
    D.ndesc = 0;
    D.reg_ndesc[0] = D.reg_ndesc[1] = 0;
    D.n_overflow = 0;
  }
  A.ndesc = D.ndesc;
  // tests: KW_POISON_VERDICTS fills the verdict words with a sentinel no verdict word equals
  // (reason byte 0xA5) before the pass, so a tile the schedule never ran shows up as a mismatch
  // instead of keeping an earlier pass's words
  if (const char* pz = getenv("KW_POISON_VERDICTS"); pz && atoi(pz) != 0)
    HIPCHK(hipMemsetAsync(D.verdicts, 0xA5, D.last_verdicts * sizeof(uint32_t), s));
  // the dynamic tile schedule's per-XCD counters (used by the regions whose plan says so,
  // sched_dynamic; run_pass hands them to those launches only)
  if (!D.sched) {
    void* p = nullptr;
    HIPCHK(dev_pool().alloc(D.device, 512 * sizeof(uint32_t), &p));
    D.sched = (uint32_t*)p;
    HIPCHK(hipMemsetAsync(D.sched, 0, 512 * sizeof(uint32_t), s));
  }
  A.sched = D.sched;
  // side data: dense group causes, the overflow path's class arrays and wide-argument list
  if (plan.nwide) {
    if (int rc = ensure(&D.wide_groups, &D.wide_groups_cap, (size_t)(B.n * plan.nwide))) return rc;
    A.wide_groups = D.wide_groups;
  }
  if (!D.wide_count) {
    void* p = nullptr;
    HIPCHK(dev_pool().alloc(D.device, sizeof(uint32_t), &p));
    D.wide_count = (uint32_t*)p;
  }
  // only the overflow kernels append wide records: a pass without overflow requests leaves the
  // counter alone (no fill launched between back-to-back passes) and has no records to read back
  D.wide_valid = D.n_overflow != 0;
  if (D.wide_valid) HIPCHK(hipMemsetAsync(D.wide_count, 0, sizeof(uint32_t), s));
  A.wide_count = D.wide_count;
  if (D.n_overflow) {
    if (int rc = ensure_overflow_classes(B, &D, plan.geom, &A)) return rc;
    const size_t cap = (size_t)D.n_overflow * plan.wide_cap_per_row;
    if (int rc = ensure(&D.wide_rec, &D.wide_rec_cap, cap)) return rc;
    A.wide_rec = D.wide_rec;
    A.wide_cap = (uint32_t)std::min<size_t>(cap, 0xffffffffu);
  }
  if (plan.geom.feat & kFeatNfa) {
    if (int rc = ensure_nfa(kb, plan, &A)) return rc;
  }
  D.last_nwide = plan.nwide;
  D.last_wide_policy = plan.wide_policy;
  D.last_rows_mode = plan.rows_mode;
  D.last_row_words = plan.args.npol;
  D.last_wide_cap = A.wide_cap;
  *out_args = A;
  return KW_OK;
}

int run_pass(kw_batch* kb, PassPlan& plan, bool timed, hipStream_t s) {
  DeviceBatch& D = *kb->dev;
  EvalArgs A;
  if (int rc = prepare_pass(kb, plan, s, &A)) return rc;
  // diagnostics: per-phase clocks of the tile kernel (KW_TILE_DEBUG & 512), printed per launch
  const bool phases = (plan.geom.debug & 512u) != 0;
  void* d_phase = nullptr;
  uint32_t gmax = 0;
  for (const PassPlan::Region& rg : plan.regions) gmax = std::max(gmax, rg.grid);
  const size_t phase_bytes = (size_t)gmax * kPhaseWords * sizeof(uint64_t);
  if (phases) {
    HIPCHK(hipMalloc(&d_phase, phase_bytes));
    A.phase = (uint64_t*)d_phase;
  }
  if (timed) HIPCHK(hipEventRecord(D.ev[0], s));
  if (plan.geom.feat & kFeatNfa) HIPCHK(launch_nfa_classify(A, D.d_tiles, plan.nfa, plan.nfa_threads, s));
  // region by region (a split batch: the light rows' launches, then the heavy rows'), each over its
  // own descriptors; the overflow kernels after the last region, over the one overflow list
  const size_t nl = plan.launches.size();
  for (size_t l = 0; l < plan.tiles.size(); ++l) {
    const size_t k = l / nl;
    if (phases) HIPCHK(hipMemsetAsync(d_phase, 0, phase_bytes, s));
    const uint32_t grid = plan.regions[k].grid;
    EvalArgs Ak = A;
    Ak.ndesc = D.reg_ndesc[k];
    if (!plan.regions[k].dyn) Ak.sched = nullptr;  // the strided schedule
    HIPCHK(launch_evaluate_tiles(Ak, plan.tiles[l], D.d_tiles + l, D.desc + D.reg_desc[k], grid, s));
    if (phases) {
      std::vector<uint64_t> ph((size_t)grid * kPhaseWords);
      HIPCHK(hipMemcpyAsync(ph.data(), d_phase, ph.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      double sum[kPhaseWords] = {0};
      for (uint32_t g = 0; g < grid; ++g)
        for (uint32_t k = 0; k < kPhaseWords; ++k) sum[k] += (double)ph[(size_t)g * kPhaseWords + k];
      const double tiles = std::max(1.0, sum[5]);
      fprintf(stderr,
              "[kw phase] launch %zu grid %u tiles %.0f: cycles/tile P0 %.0f P1 %.0f D %.0f P2 %.0f P3+next %.0f "
              "(sum %.0f); per workgroup: %.0f cycles, %.2f tiles, table staging %.0f\n",
              l, grid, tiles, sum[0] / tiles, sum[1] / tiles, sum[2] / tiles, sum[3] / tiles, sum[4] / tiles,
              (sum[0] + sum[1] + sum[2] + sum[3] + sum[4]) / tiles, sum[6] / grid, tiles / grid, sum[7] / grid);
      // per wave and tile: P1 / P2 segment cycles, each phase's busy time and its barrier wait
      const double wt = tiles * (double)(kSlotThreads / 64u);
      const double* g = sum + 8;
      fprintf(stderr,
              "[kw seg] per wave-tile: P0 wait %.0f | P1 busy %.0f wait %.0f (label %.0f capstr %.0f ctr %.0f image %.0f req %.0f) "
              "| P2 busy %.0f wait %.0f (ctr %.0f label %.0f req %.0f) | P3 busy %.0f wait %.0f | P0 issue: top %.0f "
              "request arrays %.0f strings %.0f\n",
              g[SG_P0_WAIT] / wt, g[SG_P1_BUSY] / wt, g[SG_P1_WAIT] / wt, g[SG_P1_LABEL] / wt, g[SG_P1_CAPSTR] / wt,
              g[SG_P1_CTR] / wt, g[SG_P1_IMAGE] / wt, g[SG_P1_REQ] / wt, g[SG_P2_BUSY] / wt, g[SG_P2_WAIT] / wt,
              g[SG_P2_CTR] / wt, g[SG_P2_LABEL] / wt, g[SG_P2_REQ] / wt, g[SG_P3_BUSY] / wt, g[SG_P3_WAIT] / wt,
              g[SG_P0_TOP] / wt, g[SG_P0_REQ] / wt, g[SG_P0_STR] / wt);
      // workgroup start times: a grid the CUs do not hold at once starts in waves. The real-time
      // counter is compared only within an XCD (workgroup b runs on XCD b % 8): the XCDs' counters
      // are not synchronised with each other.
      const uint32_t nx = std::min(8u, grid);
      uint32_t late = 0;
      double spread = 0;
      for (uint32_t x = 0; x < nx; ++x) {
        std::vector<uint64_t> st;
        for (uint32_t q = x; q < grid; q += nx) st.push_back(ph[(size_t)q * kPhaseWords + 8 + SG_START]);
        std::sort(st.begin(), st.end());
        for (uint64_t v : st) late += v > st[0] + 2000;  // > 20 us after the XCD's first
        spread = std::max(spread, (double)(st.back() - st[0]) / 100.0);
      }
      fprintf(stderr, "[kw start] launch %zu: %u of %u workgroups started > 20 us after their XCD's first (widest spread %.1f us)\n",
              l, late, grid, spread);
    }
    if (D.n_overflow && k + 1 == plan.regions.size()) HIPCHK(launch_overflow(A, D.d_tiles + l, D.overflow, D.n_overflow, s));
  }
  if (timed) HIPCHK(hipEventRecord(D.ev[2], s));
  if (phases) HIPCHK(hipFree(d_phase));
  return KW_OK;
}

// A planned pass with its wide policy groups (PassPlan::wide): their members first run as a
// separate all-pairs pass into member_words, then the pass itself (wide columns hold a
// placeholder), then the combine kernel writes those columns and their cause bitsets. The member
// pass's own side data (entity indices >= 65535 of members) is not kept: the main pass reuses the
// buffers. `timed`: HIP events bracket the main pass.
int run_validate(const kw_env* env, kw_batch* kb, PassPlan& plan, int origin, bool timed, hipStream_t s) {
  DeviceBatch& D = *kb->dev;
  const PassPlan::Wide& W = plan.wide;
  D.last_big_stride = 0;
  D.last_big_ref.clear();
  if (W.groups.empty()) return run_pass(kb, plan, timed, s);
  const uint64_t n = kb->b.n;
  const size_t nm = W.members.size();
  if (int rc = ensure(&D.member_words, &D.member_words_cap, (size_t)(n * nm))) return rc;
  {
    PassPlan mplan;
    if (int rc = plan_pass(env, kb, W.members.data(), (uint32_t)nm, nullptr, origin, &mplan)) return rc;
    mplan.args.out = D.member_words;
    if (int rc = run_pass(kb, mplan, false, s)) return rc;
  }
  if (int rc = run_pass(kb, plan, timed, s)) return rc;
  // combine: records (the groups', then the split members') | jump code | member maps in one upload
  const size_t g_bytes = (W.groups.size() + W.aux.size()) * sizeof(WideGroupArgs);
  const size_t p_at = g_bytes, m_at = (p_at + W.progs.size() + 15u) & ~(size_t)15u;
  const size_t bytes = m_at + W.midx.size() * 4;
  HIPCHK(hipStreamSynchronize(s));  // the upload buffer may still be read by the previous pass
  if (int rc = ensure(&D.wg_data, &D.wg_data_cap, bytes)) return rc;
  std::vector<uint8_t> h(bytes, 0);
  memcpy(h.data(), W.groups.data(), W.groups.size() * sizeof(WideGroupArgs));
  if (!W.aux.empty()) memcpy(h.data() + W.groups.size() * sizeof(WideGroupArgs), W.aux.data(), W.aux.size() * sizeof(WideGroupArgs));
  memcpy(h.data() + p_at, W.progs.data(), W.progs.size());
  memcpy(h.data() + m_at, W.midx.data(), W.midx.size() * 4);
  HIPCHK(hipMemcpyAsync(D.wg_data, h.data(), bytes, hipMemcpyHostToDevice, s));
  const uint64_t pairs = n * W.groups.size();
  const size_t stack_words = std::max<uint32_t>(W.stack_words, 1);
  // (a script that builds strings or arrays carries a 16 KB arena per thread: the grid keeps the
  // scratch under 1 GiB; every thread loops over its pairs)
  const uint64_t max_grid = std::max<uint64_t>(1, (1ull << 30) / (256ull * 8ull * stack_words));
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({(pairs + 255) / 256, 1024, max_grid}));
  if (int rc = ensure(&D.wg_stack, &D.wg_stack_cap, (size_t)grid * 256 * stack_words)) return rc;
  if (int rc = ensure(&D.big_causes, &D.big_causes_cap, (size_t)(n * W.cause_stride))) return rc;
  HIPCHK(hipMemsetAsync(D.big_causes, 0, (size_t)(n * W.cause_stride) * 8, s));
  WideGroupPass w;
  memset(&w, 0, sizeof(w));
  w.groups = (const WideGroupArgs*)D.wg_data;
  w.ngroups = (uint32_t)W.groups.size();
  w.progs = D.wg_data + p_at;
  w.midx = (const uint32_t*)(D.wg_data + m_at);
  w.member_words = D.member_words;
  w.nmw = (uint32_t)nm;
  w.out = D.verdicts;
  w.npol = plan.args.npol;
  w.rowcol = plan.rows_mode ? D.rowcol : nullptr;
  w.causes = D.big_causes;
  w.cause_stride = W.cause_stride;
  w.stack = D.wg_stack;
  w.stack_words = (uint32_t)stack_words;
  w.nrows = n;
  HIPCHK(launch_wide_groups(w, grid, s));
  D.last_big_stride = W.cause_stride;
  for (size_t k = 0; k < W.groups.size(); ++k)
    D.last_big_ref.push_back({W.policy[k], W.groups[k].cause_off, W.groups[k].cause_words});
  HIPCHK(hipStreamSynchronize(s));  // the host copy `h` is freed on return
  return KW_OK;
}

// The plan cache's key for the diagnostic / A-B settings (tests switch them between passes): the
// values of exactly the KW_* variables that planning reads (plan_pass and the planners it calls),
// looked up by name — no walk over `environ`, which a concurrent setenv could free under it.
uint64_t kw_knob_hash() {
  static const char* const kPlanKnobs[] = {"KW_TILE_DEBUG", "KW_TILE_SPLIT", "KW_ROUND_SPLIT", "KW_L2_PREFETCH",
                                           "KW_KV_GLOBAL", "KW_TILE_QUANTILE", "KW_SPLIT", "KW_SLOT_ROWS",
                                           "KW_SCHED", "KW_HEAVY_ROWS", "KW_HEAVY_CTR", "KW_GLOBAL_TABLES",
                                           "KW_NO_MPACK", "KW_POISON_VERDICTS", "KW_GROUP_FORM"};
  uint64_t h = 1469598103934665603ull;
  for (const char* k : kPlanKnobs) {
    const char* v = getenv(k);
    h = (h ^ (v ? 0x100u : 0x200u)) * 1099511628211ull;
    for (const char* c = v; c && *c; ++c) h = (h ^ (uint8_t)*c) * 1099511628211ull;
  }
  return h;
}

int validate_common(const kw_env* env, kw_batch* kb, const int32_t* policies, uint32_t npol, const int32_t* row_policy,
                    int origin, PassPlan* plan) {
  if (!env || !kb) return KW_E_ARG;
  const Env& E = env->e;
  if (E.device < 0 || !E.d_blob) return KW_E_DEVICE;  // no silent host fallback: the hot path is the GPU
  if (!kb->dev) return KW_E_ARG;                        // batch not resident
  if (kb->dev->device != E.device) return KW_E_ARG;
  if (origin != KW_ORIGIN_VALIDATE && origin != KW_ORIGIN_AUDIT) return KW_E_ARG;
  DeviceBatch& D = *kb->dev;
  HIPCHK(hipSetDevice(D.device));
  const int32_t np = (int32_t)E.nvisible;  // (the hidden parts of split policies are not addressable)
  uint64_t npairs;
  if (row_policy) {
    for (uint64_t r = 0; r < kb->b.n; ++r)
      if (row_policy[r] < 0 || row_policy[r] >= np) return KW_E_ARG;
    npairs = kb->b.n;
  } else {
    if (npol == 0 || !policies) return KW_E_ARG;
    for (uint32_t j = 0; j < npol; ++j)
      if (policies[j] < 0 || policies[j] >= np) return KW_E_ARG;
    npairs = kb->b.n * (uint64_t)npol;
  }
  if (int rc = ensure(&D.verdicts, &D.verdict_cap, npairs)) return rc;
  D.last_verdicts = npairs;
  kb->b.wide.clear();
  if (int rc = plan_pass(env, kb, policies, npol, row_policy, origin, plan)) return rc;
  return (plan->geom.need & ~D.loaded) ? KW_E_ARG : KW_OK;  // a column the upload left out (kw_validate_host)
}

// validate_common for an all-pairs pass through the batch's plan cache (DeviceBatch::plan_cache):
// a repeated pass (same environment, policy list, origin and KW_* settings) skips planning; the
// checks and the verdict buffer are redone every time.
int validate_cached(const kw_env* env, kw_batch* kb, const int32_t* policies, uint32_t npol, int origin, PassPlan** out) {
  DeviceBatch* D = kb && kb->dev ? kb->dev.get() : nullptr;
  const uint64_t knobs = kw_knob_hash();
  if (env && D && D->plan_cache && D->plan_env == env->uid && D->plan_origin == origin && D->plan_knobs == knobs &&
      D->plan_pols.size() == npol && policies && std::equal(policies, policies + npol, D->plan_pols.begin())) {
    PassPlan* plan = (PassPlan*)D->plan_cache.get();
    const Env& E = env->e;
    if (E.device < 0 || !E.d_blob) return KW_E_DEVICE;
    if (D->device != E.device) return KW_E_ARG;
    HIPCHK(hipSetDevice(D->device));
    const uint64_t npairs = kb->b.n * (uint64_t)npol;
    uint32_t* before = D->verdicts;
    if (int rc = ensure(&D->verdicts, &D->verdict_cap, npairs)) return rc;
    if (D->verdicts != before) {  // (reallocated by another pass's larger need: re-plan)
      D->plan_cache.reset();
      return validate_cached(env, kb, policies, npol, origin, out);
    }
    D->last_verdicts = npairs;
    kb->b.wide.clear();
    if (plan->geom.need & ~D->loaded) return KW_E_ARG;
    *out = plan;
    return KW_OK;
  }
  auto plan = std::make_shared<PassPlan>();
  if (D) D->plan_cache.reset();
  if (int rc = validate_common(env, kb, policies, npol, nullptr, origin, plan.get())) return rc;
  D = kb->dev.get();
  D->plan_cache = plan;
  D->plan_env = env->uid;
  D->plan_origin = origin;
  D->plan_knobs = knobs;
  D->plan_pols.assign(policies, policies + npol);
  *out = plan.get();
  return KW_OK;
}

}  // namespace

extern "C" {

const char* kw_version(void) { return "kwgpu 0.2 (gfx950)"; }

int kw_env_build(const char* json, size_t len, const kw_env_options* opts, kw_env** out, char* err, size_t errlen) {
  if (!json || !out) return KW_E_ARG;
  auto env = std::make_unique<kw_env>();
  Status st = build_env(json, len, opts ? opts->continue_on_errors != 0 : false,
                        opts ? opts->always_accept_namespace : nullptr, &env->e);
  if (!st.ok()) {
    put_err(err, errlen, st.message);
    return st.code;
  }
  int dev = opts ? opts->device : -1;
  if (int rc = upload_env(env.get(), dev)) {
    put_err(err, errlen, "cannot upload compiled tables to the device");
    return rc;
  }
  *out = env.release();
  return KW_OK;
}

int kw_env_build_yaml(const char* yaml, size_t len, const kw_env_options* opts, kw_env** out, char* err, size_t errlen) {
  if (!yaml || !out) return KW_E_ARG;
  std::string json, e;
  if (!yaml_to_json(yaml, len, &json, &e)) {  // read_policies_file: serde_yaml error -> boot failure
    put_err(err, errlen, "bootstrap failure: cannot parse policies: " + e);
    return KW_E_BOOTSTRAP;
  }
  return kw_env_build(json.data(), json.size(), opts, out, err, errlen);
}

int kw_yaml_to_json(const char* yaml, size_t len, char* buf, size_t cap, size_t* need) {
  if (!yaml && len) return KW_E_ARG;
  std::string json, e;
  if (!yaml_to_json(yaml, len, &json, &e)) {
    put_out(e, buf, cap, need);
    return KW_E_PAYLOAD;
  }
  return put_out(json, buf, cap, need);
}

int kw_env_serialize(const kw_env* env, void* buf, size_t cap, size_t* need) {
  if (!env) return KW_E_ARG;
  std::vector<uint8_t> s = env_serialize(env->e);
  if (need) *need = s.size();
  if (!buf || cap < s.size()) return KW_E_NOSPACE;
  memcpy(buf, s.data(), s.size());
  return KW_OK;
}

int kw_env_deserialize(const void* blob, size_t len, int device, kw_env** out, char* err, size_t errlen) {
  if (!blob || !out) return KW_E_ARG;
  auto env = std::make_unique<kw_env>();
  Status st = env_from_blob(blob, len, &env->e);
  if (!st.ok()) {
    put_err(err, errlen, st.message);
    return st.code;
  }
  if (int rc = upload_env(env.get(), device)) return rc;
  *out = env.release();
  return KW_OK;
}

void kw_env_destroy(kw_env* env) {
  if (!env) return;
  if (env->e.d_blob) {
    (void)hipSetDevice(env->e.device);
    (void)hipFree(env->e.d_blob);
  }
  delete env;
}

int kw_env_lookup(const kw_env* env, const char* id, size_t len, int32_t* idx) {
  if (!env || !id || !idx) return KW_E_ARG;
  return env_lookup(env->e, std::string(id, len), idx).code;
}

int kw_env_policy_count(const kw_env* env) { return env ? (int)env->e.nvisible : -1; }

int kw_env_policy_id(const kw_env* env, int32_t idx, char* buf, size_t cap) {
  if (!env || idx < 0 || (size_t)idx >= env->e.nvisible) return KW_E_ARG;
  return put_out(env->e.pol[(size_t)idx].id, buf, cap, nullptr);
}

int kw_env_is_group(const kw_env* env, int32_t idx) {
  if (!env || idx < 0 || (size_t)idx >= env->e.nvisible) return -1;
  return env->e.pol[(size_t)idx].is_group ? 1 : 0;
}

int kw_env_get_policy_mode(const kw_env* env, int32_t idx, int* mode) {
  if (!env || !mode || idx < 0 || (size_t)idx >= env->e.nvisible) return KW_E_ARG;
  const PolicyRec& r = env->e.pol[(size_t)idx];
  if (!r.registered) return KW_E_NOT_FOUND;
  *mode = r.mode;
  return KW_OK;
}

int kw_env_get_policy_allowed_to_mutate(const kw_env* env, int32_t idx, int* allowed) {
  if (!env || !allowed || idx < 0 || (size_t)idx >= env->e.nvisible) return KW_E_ARG;
  const PolicyRec& r = env->e.pol[(size_t)idx];
  if (!r.registered) return KW_E_NOT_FOUND;
  *allowed = r.allowed_to_mutate ? 1 : 0;
  return KW_OK;
}

int kw_env_should_always_accept_requests_made_inside_of_namespace(const kw_env* env, const char* ns, size_t len) {
  if (!env || !ns) return 0;
  return env->e.always_ns && *env->e.always_ns == std::string(ns, len) ? 1 : 0;
}

int kw_env_policy_initialization_error(const kw_env* env, int32_t idx, char* buf, size_t cap) {
  if (!env || idx < 0 || (size_t)idx >= env->e.nvisible) return -1;
  const PolicyRec& r = env->e.pol[(size_t)idx];
  if (!r.init_error) return 0;
  put_err(buf, cap, r.init_message);
  return 1;
}

int kw_env_validate_settings(const kw_env* env, int32_t idx, char* buf, size_t cap) {
  if (!env || idx < 0 || (size_t)idx >= env->e.nvisible) return KW_E_ARG;
  Status st = env_validate_settings(env->e, idx);
  if (!st.ok()) put_err(buf, cap, st.message);
  return st.code;
}

int kw_env_group_members(const kw_env* env, int32_t group, int32_t* out, int cap) {
  if (!env || group < 0 || (size_t)group >= env->e.nvisible) return -1;
  const PolicyRec& r = env->e.pol[(size_t)group];
  int n = (int)r.members.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = r.members[(size_t)i];
  return n;
}

int kw_pattern_match(int kind, const char* pat, const char* s, size_t len) {
  if (!pat || (!s && len)) return -1;
  std::vector<Pattern> ps{{(Pattern::Kind)kind, pat}};
  std::vector<Dfa> chain;  // one DFA, or the NFA element a pattern beyond the state budget becomes
  std::string err;
  if (!compile_column(ps, (size_t)1 << 30, kMaxDfaStates, &chain, &err) || chain.size() != 1) return -1;
  return chain[0].run((const uint8_t*)s, len) != 0 ? 1 : 0;
}

int kw_pattern_match_many(int kind, const char* pat, const char* const* subjects, const size_t* lens, size_t n,
                          int32_t* out) {
  if (!pat || (n && (!subjects || !lens || !out))) return -1;
  std::vector<Pattern> ps{{(Pattern::Kind)(kind & 0xff), pat}};
  std::vector<Dfa> chain;
  std::string err;
  if (kind & KW_PATTERN_FORCE_NFA) {
    chain.resize(1);
    if (!compile_nfa(ps[0], &chain[0], &err)) return -1;
  } else if (!compile_column(ps, (size_t)1 << 30, kMaxDfaStates, &chain, &err) || chain.size() != 1) {
    return -1;
  }
  for (size_t i = 0; i < n; ++i) out[i] = chain[0].run((const uint8_t*)subjects[i], lens[i]) != 0 ? 1 : 0;
  return KW_OK;
}

int kw_env_pattern_count(const kw_env* env, int col) {
  if (!env || col < 0 || col >= (int)NCOL) return -1;
  return (int)env->e.cols[col].pats.size();
}

int kw_env_pattern(const kw_env* env, int col, int idx, int* kind, char* buf, size_t cap) {
  if (!env || col < 0 || col >= (int)NCOL || idx < 0 || (size_t)idx >= env->e.cols[col].pats.size()) return KW_E_ARG;
  const Pattern& p = env->e.cols[col].pats[(size_t)idx];
  if (kind) *kind = (int)p.kind;
  return put_out(p.text, buf, cap, nullptr);
}

int kw_env_classify(const kw_env* env, int col, const char* key, size_t klen, const char* s, size_t len, uint32_t* pats,
                    int cap) {
  if (!env || col < 0 || col >= (int)NCOL || (!s && len) || (!key && klen)) return -1;
  const Env& E = env->e;
  std::vector<uint32_t> m;
  if (col == COL_LV) {
    const std::vector<uint32_t> kc = host_classes(E, COL_LK, (const uint8_t*)key, klen);
    const uint32_t k = kc.empty() ? 0u : kc[0];
    for (uint32_t c : host_value_classes(E, k, (const uint8_t*)s, len)) m.insert(m.end(), E.kv[c].matched.begin(), E.kv[c].matched.end());
  } else {
    for (uint32_t c : host_classes(E, (Col)col, (const uint8_t*)s, len))
      m.insert(m.end(), E.cols[col].class_pats[c].begin(), E.cols[col].class_pats[c].end());
  }
  std::sort(m.begin(), m.end());
  m.erase(std::unique(m.begin(), m.end()), m.end());
  for (int i = 0; i < (int)m.size() && i < cap; ++i) pats[i] = m[(size_t)i];
  return (int)m.size();
}

}  // extern "C"

namespace {
// Host restatement of the kernel's image-reference split (kernels.hip parse_image / image_part):
// the registry, effective tag (has_tag false for a digest-only reference) and normalised image.
void host_image_strings(const uint8_t* s, size_t n, std::string* reg, std::string* tag, bool* has_tag, std::string* norm) {
  const size_t NONE = (size_t)-1;
  size_t at = NONE, slash0 = NONE, slash1 = NONE, last_colon = NONE;
  bool dotcolon = false;
  for (size_t q = 0; q < n; ++q) {
    const uint8_t c = s[q];
    if (c == '@') {
      at = q;
      break;
    }
    if (c == '/') {
      if (slash0 == NONE) slash0 = q;
      else if (slash1 == NONE) slash1 = q;
    } else if (c == ':') {
      last_colon = q;
      if (slash0 == NONE) dotcolon = true;
    } else if (c == '.') {
      if (slash0 == NONE) dotcolon = true;
    }
  }
  auto eq = [&](size_t e, const char* lit) { return e == strlen(lit) && memcmp(s, lit, e) == 0; };
  const size_t name_end = at != NONE ? at : n;
  const bool is_reg = slash0 != NONE && (dotcolon || eq(slash0, "localhost"));
  const size_t rest_b = is_reg ? slash0 + 1 : 0;
  const size_t colon = (last_colon != NONE && last_colon >= rest_b) ? last_colon : NONE;
  const size_t path_end = colon != NONE ? colon : name_end;
  const size_t fsr = is_reg ? slash1 : slash0;
  const bool path_slash = fsr != NONE && fsr < path_end;
  const bool is_docker = !is_reg || eq(slash0, "docker.io");
  const bool eff_tag = colon != NONE || at == NONE;
  auto sub = [&](size_t b, size_t e) { return std::string((const char*)s + b, e - b); };
  *reg = is_reg ? sub(0, slash0) : std::string("docker.io");
  *has_tag = colon != NONE || at == NONE;
  *tag = colon != NONE ? sub(colon + 1, name_end) : (at == NONE ? std::string("latest") : std::string());
  *norm = *reg + "/";
  if (is_docker && !path_slash) *norm += "library/";
  *norm += sub(rest_b, path_end);
  if (eff_tag) *norm += ":" + (colon != NONE ? sub(colon + 1, name_end) : std::string("latest"));
  if (at != NONE) *norm += sub(at, n);
}

// Accessor of the sequential walks (slots.hpp) over host class arrays.
struct HostSrc {
  const Batch* b;
  ImgLayout il;
  uint32_t nlv_ = 0;
  std::vector<uint32_t> ns_, aa_, add_, drop_, lk_, lv_, img_;
  uint32_t rf(uint64_t r) const { return b->req_flags[r]; }
  uint32_t coff(uint64_t r) const { return b->ctr_off[r]; }
  uint32_t loff(uint64_t r) const { return b->lbl_off[r]; }
  uint32_t cflags(uint32_t c) const { return b->ctr_flags[c]; }
  uint32_t cadd(uint32_t c) const { return b->capadd_off[c]; }
  uint32_t cdrop(uint32_t c) const { return b->capdrop_off[c]; }
  uint32_t ns(uint64_t r) const { return ns_[r]; }
  uint32_t aa(uint32_t c) const { return aa_[c]; }
  uint32_t capadd(uint32_t k) const { return add_[k]; }
  uint32_t capdrop(uint32_t k) const { return drop_[k]; }
  uint32_t lk(uint32_t l) const { return lk_[l]; }
  uint32_t nlv() const { return nlv_; }
  uint32_t lv(uint32_t l, uint32_t j) const { return lv_[(size_t)l * nlv_ + j]; }
  uint32_t img(uint32_t c, uint32_t j) const { return img_[(size_t)c * il.n() + j]; }
};
}  // namespace

extern "C" {

int kw_debug_host_walk(const kw_env* env, const kw_batch* kb, const int32_t* policies, uint32_t npol, int origin,
                       uint32_t* out) {
  if (!env || !kb || (!policies && npol) || (!out && npol && kb->b.n)) return KW_E_ARG;
  const Env& E = env->e;
  const Batch& B = kb->b;
  const DevHeader* H = (const DevHeader*)E.blob.data();
  std::vector<SlotChunk> chunks;
  Status st = build_slot_chunks(E, policies, npol, origin, false, &chunks);
  if (!st.ok()) return st.code;
  // classification of every string with the blob's tables (env.cpp host_classes)
  HostSrc src;
  src.b = &B;
  src.il = {(H->col[COL_REG].lit_off ? 1u : 0u) + H->col[COL_REG].ndfa, (H->col[COL_TAG].lit_off ? 1u : 0u) + H->col[COL_TAG].ndfa,
            H->col[COL_IMG].ndfa};
  src.nlv_ = H->col[COL_LV].ndfa;
  auto one = [&](Col c, const StrCol& sc, size_t i) {
    const std::vector<uint32_t> v = host_classes(E, c, sc.bytes.data() + sc.off[i], sc.off[i + 1] - sc.off[i]);
    return v.empty() ? 0u : v[0];
  };
  for (size_t r = 0; r < B.n; ++r) src.ns_.push_back(one(COL_NS, B.ns, r));
  for (size_t c = 0; c < B.containers(); ++c) {
    src.aa_.push_back(one(COL_AA, B.ctr_aa, c));
    std::vector<uint32_t> ic;
    if (B.ctr_flags[c] & KW_CTR_HAS_IMAGE) {
      std::string reg, tag, norm;
      bool has_tag;
      host_image_strings(B.ctr_image.bytes.data() + B.ctr_image.off[c], B.ctr_image.off[c + 1] - B.ctr_image.off[c], &reg, &tag,
                         &has_tag, &norm);
      std::vector<uint32_t> r = host_classes(E, COL_REG, (const uint8_t*)reg.data(), reg.size());
      std::vector<uint32_t> t = has_tag ? host_classes(E, COL_TAG, (const uint8_t*)tag.data(), tag.size())
                                        : std::vector<uint32_t>(src.il.ntag, 0u);
      std::vector<uint32_t> m = host_classes(E, COL_IMG, (const uint8_t*)norm.data(), norm.size());
      ic.insert(ic.end(), r.begin(), r.end());
      ic.insert(ic.end(), t.begin(), t.end());
      ic.insert(ic.end(), m.begin(), m.end());
    }
    ic.resize(src.il.n(), 0u);
    src.img_.insert(src.img_.end(), ic.begin(), ic.end());
  }
  for (size_t k = 0; k < B.cap_add.n(); ++k) src.add_.push_back(one(COL_CAP, B.cap_add, k));
  for (size_t k = 0; k < B.cap_drop.n(); ++k) src.drop_.push_back(one(COL_CAP, B.cap_drop, k));
  for (size_t l = 0; l < B.labels(); ++l) {
    const uint32_t k = one(COL_LK, B.lbl_key, l);
    src.lk_.push_back(k);
    std::vector<uint32_t> v = host_value_classes(E, k, B.lbl_val.bytes.data() + B.lbl_val.off[l], B.lbl_val.off[l + 1] - B.lbl_val.off[l]);
    v.resize(src.nlv_, 0xffffu);
    src.lv_.insert(src.lv_.end(), v.begin(), v.end());
  }
  std::vector<uint32_t> vw(kSlots), va(kSlots);
  const ViolSink vs{vw.data(), va.data()};
  for (const SlotChunk& ch : chunks) {
    SlotView sv;
    sv.h = (const SlotHdr*)ch.rec.data();
    sv.base = ch.rec.data();
    const ColInfo* cols = (const ColInfo*)(ch.rec.data() + sv.h->o_cols);
    for (uint64_t r = 0; r < B.n; ++r) {
      const bool byp = is_bypass(B.req_flags[r], src.ns_[r], H->bypass_cls);
      uint64_t mut = 0;
      uint64_t rej = walk_privileged_caps(src, sv, r, vs, &mut);
      rej |= walk_apparmor_images(src, sv, r, vs);
      rej |= walk_labels(src, sv, r, vs);
      rej |= walk_namespace(src, sv, r, vs);
      for (uint32_t j = 0; j < ch.ncols; ++j) {
        uint64_t wide = 0;
        out[r * npol + ch.col0 + j] = byp ? kBypassWord : column_word(cols[j], rej, mut, sv.h->init, vw.data(), ch.rec.data(), &wide);
      }
    }
  }
  // wide groups: their members' words by the same host walk, then the jump code per row
  PassPlan wp;
  plan_wide_groups(E, std::vector<int32_t>(policies, policies + npol), nullptr, origin, &wp);
  const PassPlan::Wide& W = wp.wide;
  if (!W.groups.empty()) {
    const size_t nm = W.members.size();
    std::vector<uint32_t> mw(B.n * nm);
    if (int rc = kw_debug_host_walk(env, kb, W.members.data(), (uint32_t)nm, origin, mw.data())) return rc;
    std::vector<uint64_t> stack(std::max<uint32_t>(W.stack_words, 1));
    for (uint64_t r = 0; r < B.n; ++r)
      for (const WideGroupArgs& g : W.groups) {
        uint32_t* dst = out + r * npol + g.col;
        if (*dst == kBypassWord) continue;
        auto ok = [&](uint32_t m) {
          const uint32_t c = W.midx[g.midx_off + m];
          uint32_t x;
          if (c & kSplitMember) {
            const WideGroupArgs& a = W.aux[c & ~kSplitMember];
            x = combine_parts(a, (const uint32_t*)(W.progs.data() + a.prog_off),
                              [&](uint32_t t) { return mw[r * nm + W.midx[a.midx_off + t]]; });
          } else {
            x = mw[r * nm + c];
          }
          return (x & KW_V_ALLOWED) && !(x & KW_V_MUTATED);
        };
        uint64_t cz = 0;  // (the causes of a group of at most 15 members go into ARG)
        auto cause = [&](uint32_t m) {
          if (m < 64) cz |= 1ull << m;
        };
        auto rej = [&]() { return g.nmem <= 15 ? (g.rejb & 0xffffu) | ((uint32_t)cz << 16) : g.rejb; };
        if (g.kind == 1) {
          const int v = run_script_prog(W.progs.data() + g.prog_off, stack.data(), ok, cause);
          *dst = v == 1 ? g.okw : v == 0 ? rej() : g.errw;
          continue;
        }
        if (g.kind >= 2) {
          *dst = combine_parts(g, (const uint32_t*)(W.progs.data() + g.prog_off),
                               [&](uint32_t m) { return mw[r * nm + W.midx[g.midx_off + m]]; });
          continue;
        }
        const bool v = run_wide_prog(W.progs.data() + g.prog_off, g.prog_len, stack.data(), ok, cause);
        *dst = v ? g.okw : rej();
      }
  }
  return KW_OK;
}

int kw_batch_from_json(const char* const* docs, const size_t* lens, size_t n, int doc_kind, kw_batch** out,
                       int64_t* bad_row, char* err, size_t errlen) {
  if (!out || (n && (!docs || !lens))) return KW_E_ARG;
  auto kb = std::make_unique<kw_batch>();
  // contiguous document ranges flattened by up to KW_FLATTEN_THREADS threads (default: the
  // hardware threads, at most 16), then concatenated in order; the first bad row wins
  uint32_t nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (const char* t = getenv("KW_FLATTEN_THREADS")) nt = (uint32_t)std::max(1, atoi(t));
  nt = (uint32_t)std::min<uint64_t>(nt, std::max<size_t>(1, n / 2048));
  std::vector<Batch> part(nt);
  std::vector<int64_t> bad(nt, -1);
  std::vector<std::string> perr(nt);
  auto work = [&](uint32_t t) {
    const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
    for (size_t i = i0; i < i1; ++i)
      if (!flatten_document(docs[i], lens[i], doc_kind, &part[t], &perr[t])) {
        bad[t] = (int64_t)i;
        return;
      }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  for (uint32_t t = 0; t < nt; ++t)
    if (bad[t] >= 0) {
      if (bad_row) *bad_row = bad[t];
      put_err(err, errlen, perr[t]);
      return KW_E_PAYLOAD;
    }
  if (nt == 1) {
    kb->b = std::move(part[0]);
  } else {
    for (uint32_t t = 0; t < nt; ++t) {
      kb->b.append(part[t]);
      part[t] = Batch();  // release as we go
    }
  }
  kb->b.finalize();
  *out = kb.release();
  return KW_OK;
}

int kw_batch_from_soa(const kw_soa* soa, kw_batch** out) {
  if (!soa || !out) return KW_E_ARG;
  auto kb = std::make_unique<kw_batch>();
  std::string e;
  if (!batch_from_soa(*soa, &kb->b, &e)) return KW_E_ARG;
  kb->b.finalize();
  *out = kb.release();
  return KW_OK;
}

int kw_batch_view(const kw_batch* b, kw_soa* view) {
  if (!b || !view) return KW_E_ARG;
  b->b.view(view);
  return KW_OK;
}

}  // extern "C"

namespace {
// Upload the batch's columns to `device`: one pooled allocation with 256-B aligned sub-arrays,
// assembled in pinned host staging and copied with one async H2D on `stream` (null: a new stream
// owned by the batch); `sync` waits for the copy.
// A column of the device batch image: where its bytes come from and sit, and how a row range maps
// onto it (the bulk path uploads row chunks separately).
enum PieceKind { PK_ROW_U8, PK_ROW_OFF, PK_CTR_U8, PK_CTR_OFF, PK_STR_OFF, PK_STR_BYTES };
struct Piece {
  const void* src;
  size_t bytes;  // source bytes (reserved 256-B aligned in the image)
  size_t at;     // offset in the device image and in the pinned staging
  PieceKind kind;
  int m;         // string column (PK_STR_*), else -1
  bool gather;   // string bytes of a reordered batch (gather_column), src null
};

// Allocates the batch's device image (one pooled allocation, 256-B aligned sub-arrays) and its
// pinned staging block, and points the DeviceBatch views at it; nothing is copied.
// ---- light / heavy split at upload. A batch whose container counts
// are heavy-tailed (C5: Zipf over 1..64 — 14.7 % of the requests hold 63 % of the containers) sizes
// every tile's capacities, and so the occupancy, by the heavy requests scattered through it. The
// device copy instead holds the light requests (<= kHeavyCtr containers) first and the heavy ones
// after them, in batch order within each region; the planner gives each region its own tile
// geometry (plan_pass), and verdicts and side data are scattered back to batch rows on the host.
constexpr uint32_t kHeavyCtr = 5;
constexpr uint64_t kSplitMinRows = 1ull << 18;

// The light region's row count and the device-row order (perm[d] = batch row), or 0 when the batch
// stays in order: the heavy rows must be between 1 % and 50 % of the rows and hold at least 30 % of
// the containers, in a batch of at least kSplitMinRows rows. KW_SPLIT=0 never splits, KW_SPLIT=1
// splits whenever both regions are non-empty (tests).
uint64_t split_rows(const Batch& B, std::vector<uint64_t>* perm) {
  const char* env = getenv("KW_SPLIT");
  const int mode = env ? atoi(env) : -1;
  if (mode == 0 || B.n == 0) return 0;
  const char* hc = getenv("KW_HEAVY_CTR");  // A/B knob: the container count above which a request is heavy
  const uint32_t thr = hc && atoi(hc) > 0 ? (uint32_t)atoi(hc) : kHeavyCtr;
  auto heavy = [&](uint64_t r) { return B.ctr_off[r + 1] - B.ctr_off[r] > thr; };
  uint64_t nh = 0, ch = 0;
  for (uint64_t r = 0; r < B.n; ++r)
    if (heavy(r)) ++nh, ch += B.ctr_off[r + 1] - B.ctr_off[r];
  if (nh == 0 || nh == B.n) return 0;
  if (mode != 1 && (B.n < kSplitMinRows || nh * 100 < B.n || nh * 2 > B.n || ch * 10 < 3ull * B.containers())) return 0;
  perm->resize(B.n);
  uint64_t l = 0, h = B.n - nh;
  for (uint64_t r = 0; r < B.n; ++r) (*perm)[heavy(r) ? h++ : l++] = r;
  return B.n - nh;
}

// Batch rows in `perm` order as a new batch (P's row d = B's row perm[d]). with_bytes false: the
// device string columns get their offsets only — the upload gathers their bytes straight into its
// staging (gather_column) — and the host-only string columns stay empty. *order: the entity maps.
constexpr uint64_t kGatherTask = 1 << 16;
size_t gather_tasks(uint64_t m) { return (size_t)((m + kGatherTask - 1) / kGatherTask); }

void permute_batch(const Batch& B, const std::vector<uint64_t>& perm, Batch* P, bool with_bytes, RowOrder* order) {
  const uint64_t n = B.n;
  RowOrder& o = *order;
  o.perm = &perm;
  // an entity level: the destination offsets per parent and the source entity of each destination one
  auto level = [&](const std::vector<uint32_t>& off, uint64_t np, auto parent, std::vector<uint32_t>* doff,
                   std::vector<uint32_t>* emap) {
    doff->resize(np + 1);
    (*doff)[0] = 0;
    for (uint64_t d = 0; d < np; ++d) {
      const uint64_t p = parent(d);
      (*doff)[d + 1] = (*doff)[d] + (off[p + 1] - off[p]);
    }
    emap->resize((*doff)[np]);
    HostWorkers::get().run(gather_tasks(np), [&](size_t q) {
      for (uint64_t d = q * kGatherTask, e = std::min<uint64_t>(np, (q + 1) * kGatherTask); d < e; ++d) {
        const uint32_t s0 = off[parent(d)];
        for (uint32_t k = 0, c = (*doff)[d + 1] - (*doff)[d]; k < c; ++k) (*emap)[(*doff)[d] + k] = s0 + k;
      }
    });
  };
  auto gather_str = [&](const StrCol& src, uint64_t ne, auto map, StrCol* dst) {
    dst->off.resize(ne + 1);
    dst->off[0] = 0;
    for (uint64_t e = 0; e < ne; ++e) {
      const uint64_t s = map(e);
      dst->off[e + 1] = dst->off[e] + (src.off[s + 1] - src.off[s]);
    }
    if (!with_bytes) return;
    dst->bytes.assign(dst->off[ne], 0);
    HostWorkers::get().run(gather_tasks(ne), [&](size_t q) {
      for (uint64_t e = q * kGatherTask, f = std::min<uint64_t>(ne, (q + 1) * kGatherTask); e < f; ++e) {
        const uint64_t s = map(e);
        memcpy(dst->bytes.data() + dst->off[e], src.bytes.data() + src.off[s], src.off[s + 1] - src.off[s]);
      }
    });
  };
  P->n = n;
  auto row = [&](uint64_t d) { return perm[d]; };
  P->req_flags.resize(n);
  for (uint64_t d = 0; d < n; ++d) P->req_flags[d] = B.req_flags[perm[d]];
  gather_str(B.ns, n, row, &P->ns);
  if (with_bytes)
    for (auto [s, t] : {std::pair<const StrCol*, StrCol*>(&B.uid, &P->uid), std::pair<const StrCol*, StrCol*>(&B.op, &P->op),
                        std::pair<const StrCol*, StrCol*>(&B.kind, &P->kind), std::pair<const StrCol*, StrCol*>(&B.rkind, &P->rkind)})
      gather_str(*s, n, row, t);
  level(B.ctr_off, n, row, &P->ctr_off, &o.cmap);
  level(B.lbl_off, n, row, &P->lbl_off, &o.lmap);
  const uint64_t nc = o.cmap.size(), nl = o.lmap.size();
  auto ctr = [&](uint64_t e) { return (uint64_t)o.cmap[e]; };
  auto lbl = [&](uint64_t e) { return (uint64_t)o.lmap[e]; };
  P->ctr_flags.resize(nc);
  for (uint64_t e = 0; e < nc; ++e) P->ctr_flags[e] = B.ctr_flags[o.cmap[e]];
  gather_str(B.ctr_image, nc, ctr, &P->ctr_image);
  gather_str(B.ctr_aa, nc, ctr, &P->ctr_aa);
  if (with_bytes) gather_str(B.ctr_name, nc, ctr, &P->ctr_name);
  level(B.capadd_off, nc, ctr, &P->capadd_off, &o.amap);
  level(B.capdrop_off, nc, ctr, &P->capdrop_off, &o.dmap);
  gather_str(B.cap_add, o.amap.size(), [&](uint64_t e) { return (uint64_t)o.amap[e]; }, &P->cap_add);
  gather_str(B.cap_drop, o.dmap.size(), [&](uint64_t e) { return (uint64_t)o.dmap[e]; }, &P->cap_drop);
  gather_str(B.lbl_key, nl, lbl, &P->lbl_key);
  gather_str(B.lbl_val, nl, lbl, &P->lbl_val);
  if (with_bytes) P->finalize();
}

// String column m of the reordered batch P into `dst` (a piece of `bytes` bytes of the upload
// staging): every string from B by the entity maps, then the zero tail.
void gather_column(const Batch& B, const Batch& P, const RowOrder& o, int m, uint8_t* dst, size_t bytes) {
  const StrCol &s = host_str(B, m), &d = host_str(P, m);
  const uint64_t ne = d.n();
  HostWorkers::get().run(gather_tasks(ne), [&](size_t q) {
    for (uint64_t e = q * kGatherTask, f = std::min<uint64_t>(ne, (q + 1) * kGatherTask); e < f; ++e) {
      const uint64_t x = o.src(m, e);
      memcpy(dst + d.off[e], s.bytes.data() + s.off[x], s.off[x + 1] - s.off[x]);
    }
  });
  if (bytes > d.off[ne]) memset(dst + d.off[ne], 0, bytes - d.off[ne]);
}

int layout_batch(kw_batch* kb, int device, hipStream_t stream, std::vector<Piece>* pieces, bool may_split = false,
                 bool staging = true) {
  if (!kb || device < 0) return KW_E_ARG;
  HIPCHK(hipSetDevice(device));
  if (kb->dev) kb->dev.reset();  // re-upload: the previous device copy returns to the pools
  auto D = std::make_unique<DeviceBatch>();
  D->device = device;
  if (stream) {
    D->stream = stream;
    D->owns_stream = false;
  } else {
    HIPCHK(stream_pool().get(device, &D->stream));
  }
  kb->b.finalize();
  if (may_split) {
    D->split = split_rows(kb->b, &D->perm);
    if (D->split) {
      D->dev_b = std::make_unique<Batch>();
      D->order = std::make_unique<RowOrder>();
      permute_batch(kb->b, D->perm, D->dev_b.get(), /*with_bytes=*/false, D->order.get());
    } else {
      D->perm.clear();
    }
  }
  const Batch& B = D->dev_b ? *D->dev_b : kb->b;
  pieces->clear();
  size_t total = 0;
  auto add = [&](const void* src, size_t bytes, PieceKind k, int m) {
    size_t at = total;
    pieces->push_back({src, bytes, at, k, m, false});
    total += (bytes + 255) & ~(size_t)255;
    return at;
  };
  size_t o_rf = add(B.req_flags.data(), B.req_flags.size(), PK_ROW_U8, -1);
  size_t o_co = add(B.ctr_off.data(), B.ctr_off.size() * 4, PK_ROW_OFF, -1);
  size_t o_lo = add(B.lbl_off.data(), B.lbl_off.size() * 4, PK_ROW_OFF, -1);
  size_t o_cf = add(B.ctr_flags.data(), B.ctr_flags.size(), PK_CTR_U8, -1);
  size_t o_ca = add(B.capadd_off.data(), B.capadd_off.size() * 4, PK_CTR_OFF, -1);
  size_t o_cd = add(B.capdrop_off.data(), B.capdrop_off.size() * 4, PK_CTR_OFF, -1);
  size_t c_off[NSTR], c_bytes[NSTR];
  for (int m = 0; m < (int)NSTR; ++m) {
    const StrCol& c = host_str(B, m);
    c_off[m] = add(c.off.data(), c.off.size() * 4, PK_STR_OFF, m);
    if (D->order) {  // reordered: gathered into the staging at upload (>= 16 B zero tail, StrCol::pad)
      c_bytes[m] = add(nullptr, ((size_t)c.off.back() + 31) & ~(size_t)15, PK_STR_BYTES, m);
      pieces->back().gather = true;
    } else {
      c_bytes[m] = add(c.bytes.data(), c.bytes.size(), PK_STR_BYTES, m);
    }
  }
  total = std::max<size_t>(total, 256);
  void* dcols = nullptr;
  HIPCHK(dev_pool().alloc(device, total, &dcols));
  D->cols = (uint8_t*)dcols;
  D->cols_bytes = total;
  if (staging) {
    HIPCHK(host_pool().alloc(device, total, &D->staging));
    D->staging_bytes = total;
  }
  D->cur = D->stream;
  D->req_flags = D->cols + o_rf;
  D->ctr_off = (const uint32_t*)(D->cols + o_co);
  D->lbl_off = (const uint32_t*)(D->cols + o_lo);
  D->ctr_flags = D->cols + o_cf;
  D->capadd_off = (const uint32_t*)(D->cols + o_ca);
  D->capdrop_off = (const uint32_t*)(D->cols + o_cd);
  for (int m = 0; m < (int)NSTR; ++m) {
    const StrCol& c = host_str(B, m);
    DeviceBatch::DCol& d = D->str[m];
    d.off = (const uint32_t*)(D->cols + c_off[m]);
    d.bytes = D->cols + c_bytes[m];
    d.n = c.n();
    d.nbytes = c.off.back();
  }
  kb->dev = std::move(D);
  return KW_OK;
}

int upload_batch(kw_batch* kb, int device, hipStream_t stream, bool sync) {
  std::vector<Piece> pieces;
  if (int rc = layout_batch(kb, device, stream, &pieces, /*may_split=*/true)) return rc;
  DeviceBatch& D = *kb->dev;
  uint8_t* st = (uint8_t*)D.staging;
  for (auto& p : pieces) {
    if (!p.bytes) continue;
    if (p.gather)
      gather_column(kb->b, *D.dev_b, *D.order, p.m, st + p.at, p.bytes);
    else
      parallel_copy(st + p.at, p.src, p.bytes);
  }
  D.order.reset();  // (the planner reads the reordered batch's offsets only)
  HIPCHK(hipMemcpyAsync(D.cols, st, D.cols_bytes, hipMemcpyHostToDevice, D.stream));
  if (sync) HIPCHK(hipStreamSynchronize(D.stream));
  D.loaded = ~0u;
  return KW_OK;
}

// Byte range [lo, hi) of piece p that rows [r0, r1) occupy. A chunk's string bytes run 64 bytes past
// its last string (the device's batched reads past a string end stay inside uploaded bytes); the
// first chunk starts at 0 and the last runs to the piece's end (its zero padding).
void piece_range(const Batch& B, const Piece& p, uint64_t r0, uint64_t r1, bool last, size_t* lo, size_t* hi) {
  size_t a = 0, e = 0;
  uint64_t g0 = 0, g1 = 0;
  switch (p.kind) {
    case PK_ROW_U8: a = r0; e = r1; break;
    case PK_ROW_OFF: a = 4 * r0; e = 4 * (r1 + 1); break;
    case PK_CTR_U8: a = B.ctr_off[r0]; e = B.ctr_off[r1]; break;
    case PK_CTR_OFF: a = 4ull * B.ctr_off[r0]; e = 4ull * ((uint64_t)B.ctr_off[r1] + 1); break;
    case PK_STR_OFF: str_range(B, p.m, r0, r1, &g0, &g1); a = 4 * g0; e = 4 * (g1 + 1); break;
    case PK_STR_BYTES: {
      str_range(B, p.m, r0, r1, &g0, &g1);
      const StrCol& c = host_str(B, p.m);
      a = c.off[g0];
      e = (size_t)c.off[g1] + 64;
      break;
    }
  }
  if (r0 == 0) a = 0;
  if (last) e = p.bytes;
  *lo = std::min(a, p.bytes);
  *hi = std::min(std::max(e, a), p.bytes);
}

// The pass's side data into the batch's host copy (kw_batch_wide_arg, the formatter): entity
// indices >= 65535 and > 15-member group causes (kernels.hpp WideRec), after the pass on stream s.
int load_side_data(kw_batch* b, hipStream_t s) {
  DeviceBatch& D = *b->dev;
  WideData& W = b->b.wide;
  W.clear();
  uint32_t nrec = 0;
  if (D.wide_count && D.wide_valid) HIPCHK(hipMemcpyAsync(&nrec, D.wide_count, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  W.nwide = D.last_nwide;
  W.wide_policy = D.last_wide_policy;
  W.rows_mode = D.last_rows_mode;
  if (D.last_big_stride && D.big_causes) {  // wide-group cause bitsets
    W.big_stride = D.last_big_stride;
    W.big_ref = D.last_big_ref;
    W.big.resize(b->b.n * W.big_stride);
    if (!W.big.empty()) HIPCHK(hipMemcpyAsync(W.big.data(), D.big_causes, W.big.size() * 8, hipMemcpyDeviceToHost, s));
  }
  if (W.nwide) {
    W.groups.resize(b->b.n * W.nwide);
    if (!W.groups.empty())
      HIPCHK(hipMemcpyAsync(W.groups.data(), D.wide_groups, W.groups.size() * 8, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  if (D.split) {  // device-row order (light / heavy split) -> batch rows
    auto unperm = [&](std::vector<uint64_t>* v, uint32_t stride) {
      if (v->empty() || !stride) return;
      std::vector<uint64_t> t(v->size());
      for (uint64_t d = 0; d < b->b.n; ++d)
        std::copy_n(v->data() + d * stride, stride, t.data() + D.perm[d] * stride);
      v->swap(t);
    };
    unperm(&W.big, W.big_stride);
    unperm(&W.groups, W.nwide);
  }
  nrec = std::min(nrec, D.last_wide_cap);
  if (nrec) {
    std::vector<WideRec> rec(nrec);
    HIPCHK(hipMemcpy(rec.data(), D.wide_rec, nrec * sizeof(WideRec), hipMemcpyDeviceToHost));
    for (const WideRec& r : rec) {
      const uint64_t d = (uint64_t)r.row_lo | ((uint64_t)r.row_hi << 32);
      W.recs.push_back({D.split ? D.perm[d] : d, (int32_t)r.policy, r.value});
    }
    std::sort(W.recs.begin(), W.recs.end(), [](const WideData::Rec& x, const WideData::Rec& y) {
      return x.row < y.row || (x.row == y.row && x.policy < y.policy);
    });
  }
  return KW_OK;
}

// Bulk host -> host validation (kw_validate_host): the batch's columns are uploaded, evaluated and
// read back in row chunks whose stages overlap: the host workers build chunk k's tile descriptors
// and fill its pinned staging while the copy engines move chunk k-1 in and chunk k-2's verdicts out
// and the tile kernel evaluates in between (three streams ordered by events). Only the string
// columns the pass reads are uploaded. The plan's tile capacities come from a sample of the tile
// needs (every stride-th tile), and each chunk's descriptors are built just before its fill, so the
// first read-back starts after one small chunk rather than after a whole-batch head; a request
// that exceeds the capacities alone runs through the overflow kernels right after its chunk's tile
// launch. Passes with several launches, wide side data or NFA elements run unchunked (upload, pass,
// read-back) with the same result.
int validate_host(const kw_env* env, kw_batch* kb, const int32_t* policies, uint32_t npol, int origin, int device,
                  uint32_t* out, size_t count, uint32_t chunk_rows) {
  if (!env || !kb || !out || !policies || npol == 0) return KW_E_ARG;
  if (env->e.device < 0 || !env->e.d_blob) return KW_E_DEVICE;
  if (device != env->e.device || count != kb->b.n * (uint64_t)npol) return KW_E_ARG;
  // diagnostics (KW_BULK_DEBUG=1): host wall time of each stage, printed at the end
  static const bool dbg = getenv("KW_BULK_DEBUG") && atoi(getenv("KW_BULK_DEBUG")) != 0;
  using clk = std::chrono::steady_clock;
  const auto t_start = clk::now();
  double t_layout = 0, t_plan = 0, t_prep = 0, t_desc = 0, t_fill = 0, t_enq = 0, t_out = 0, t_first = -1;
  auto since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  std::vector<Piece> pieces;
  if (int rc = layout_batch(kb, device, nullptr, &pieces, /*may_split=*/false, /*staging=*/false)) return rc;
  t_layout = since(t_start);
  DeviceBatch& D = *kb->dev;
  const Batch& B = kb->b;
  D.loaded = ~0u;  // (planned as if resident; set to the pass's columns below)
  // tile capacities from about 2048 sampled tiles (KW_BULK_SAMPLE=0: every tile, A/B knob)
  static const bool sample = !(getenv("KW_BULK_SAMPLE") && atoi(getenv("KW_BULK_SAMPLE")) == 0);
  D.needs_stride = sample ? (uint32_t)std::max<uint64_t>(1, B.n / ((uint64_t)kSlotRows * 2048)) : 1u;
  PassPlan plan;
  const int prc = validate_common(env, kb, policies, npol, nullptr, origin, &plan);
  D.needs_stride = 1;
  if (prc) {
    D.loaded = 0;
    return prc;
  }
  const uint32_t need = plan.geom.need;
  t_plan = since(t_start) - t_layout;
  auto wanted = [&](const Piece& p) { return p.m < 0 || ((need >> p.m) & 1u); };
  // columns page-locked in place (kw_batch_pin_host) go to the device by DMA from where they lie;
  // the others through the pinned staging, filled by the host workers
  std::vector<char> dma(pieces.size(), 0);
  if (!kb->host_pinned.empty())
    for (size_t i = 0; i < pieces.size(); ++i) {
      hipPointerAttribute_t pa;
      dma[i] = pieces[i].bytes && hipPointerGetAttributes(&pa, pieces[i].src) == hipSuccess &&
               pa.type == hipMemoryTypeHost;
      (void)hipGetLastError();
    }
  hipStream_t sc = D.stream;
  EvalArgs A;
  // (NFA elements: their pre-pass reads whole columns, so such passes are not chunked)
  const bool chunked = plan.tiles.size() == 1 && plan.wide.groups.empty() && plan.nwide == 0 && !plan.rows_mode &&
                       !(plan.geom.debug & 512u) && !(plan.geom.feat & kFeatNfa) && B.n > 0;
  // the staging image of the whole batch only where it is used: the unchunked path and per-range
  // copies (packed chunks go through their own ring; pinning C5's 3.6 GB image cost 360 ms a call)
  static const bool pack_knob = !(getenv("KW_BULK_PACK") && atoi(getenv("KW_BULK_PACK")) == 0);
  if ((!chunked || !pack_knob) && !D.staging) {
    HIPCHK(host_pool().alloc(device, D.cols_bytes, &D.staging));
    D.staging_bytes = D.cols_bytes;
  }
  uint8_t* st = (uint8_t*)D.staging;
  if (!chunked) {  // one upload, the full pass, one read-back
    std::vector<CopySeg> segs;
    for (size_t i = 0; i < pieces.size(); ++i)
      if (pieces[i].bytes && !dma[i]) segs.push_back({st + pieces[i].at, pieces[i].src, pieces[i].bytes});
    parallel_copy_segs(segs);
    for (const CopySeg& c : segs)
      HIPCHK(hipMemcpyAsync(D.cols + ((uint8_t*)c.dst - st), c.dst, c.bytes, hipMemcpyHostToDevice, sc));
    for (size_t i = 0; i < pieces.size(); ++i)
      if (pieces[i].bytes && dma[i])
        HIPCHK(hipMemcpyAsync(D.cols + pieces[i].at, pieces[i].src, pieces[i].bytes, hipMemcpyHostToDevice, sc));
    if (int rc = run_validate(env, kb, plan, origin, false, sc)) return rc;
    return kw_batch_verdicts(kb, out, count);
  }
  D.last_big_stride = 0;  // (no wide groups in a chunked pass: stale cause bitsets must not be read)
  D.last_big_ref.clear();
  if (int rc = prepare_pass(kb, plan, sc, &A, /*descs=*/false)) {
    D.loaded = 0;
    return rc;
  }
  t_prep = since(t_start) - t_layout - t_plan;
  D.loaded = need;
  const TileArgs& G = plan.geom;
  const uint64_t ntiles = (B.n + G.rows - 1) / G.rows;
  static const uint64_t def_chunk = getenv("KW_BULK_CHUNK") ? std::max(1, atoi(getenv("KW_BULK_CHUNK"))) : 262144;  // A/B knob (profiles/r04_bulk_sweep.txt)
  const uint64_t per = chunk_rows ? chunk_rows : def_chunk;
  // chunk k: tiles [tb[k], tb[k+1]). The read-back stream is the longest (4 B x npol per request
  // out vs the request's columns in), so the first chunks are small (1/16 of `per`, doubling) to
  // start it early; then `per` rows a chunk.
  static const bool ramp = !(getenv("KW_BULK_RAMP") && atoi(getenv("KW_BULK_RAMP")) == 0);  // A/B knob
  // The last chunks shrink the same way (r05): the final chunk's read-back overlaps nothing, so a
  // full-size last chunk left ~1 ms of C4's read-back exposed. At most ~240 chunks (per grows).
  const uint64_t tper = std::max<uint64_t>({1, per / G.rows, (ntiles + 239) / 240});
  std::vector<uint64_t> tb{0};
  {
    std::vector<uint64_t> head, tail;  // chunk sizes in tiles, from the front and from the back
    uint64_t left = ntiles, sh = ramp ? std::max<uint64_t>(1, tper / 16) : tper, st_ = sh;
    while (left) {
      head.push_back(std::min(sh, left));
      left -= head.back();
      sh = std::min(tper, sh * 2);
      if (!left || !ramp) continue;
      tail.push_back(std::min(st_, left));
      left -= tail.back();
      st_ = std::min(tper, st_ * 2);
    }
    for (uint64_t h : head) tb.push_back(tb.back() + h);
    for (auto it = tail.rbegin(); it != tail.rend(); ++it) tb.push_back(tb.back() + *it);
  }
  const uint64_t K = tb.size() - 1;
  auto row_of = [&](uint64_t t) { return std::min<uint64_t>(B.n, t * G.rows); };
  hipPointerAttribute_t attr;
  static const bool direct = !(getenv("KW_BULK_DIRECT") && atoi(getenv("KW_BULK_DIRECT")) == 0);  // A/B knob
  const bool pinned = direct && hipPointerGetAttributes(&attr, out) == hipSuccess && attr.type == hipMemoryTypeHost;
  (void)hipGetLastError();  // a pageable pointer leaves an error state behind
  // pinned output: at most `depth` chunks in flight past the read-back. Unbounded, the host queues
  // every chunk's copies and launch at once and the copies run slower (C4 1M: 16.0-16.7 ms vs
  // 9.7-10.9 at depth 2, profiles/r04_bulk_modes.txt). Staged columns take 3 (the host fills pace
  // the uploads), columns DMA'd in place 2 (at 3 their uploads crowd the read-backs: 11.0 vs
  // 7.1 ms, profiles/r04_bulk_sweep.txt). KW_BULK_DEPTH: A/B knob, 0 = unbounded.
  static const int depth_knob = getenv("KW_BULK_DEPTH") ? std::max(0, atoi(getenv("KW_BULK_DEPTH"))) : -1;
  const bool any_dma = std::count(dma.begin(), dma.end(), 1) > 0;
  const uint64_t depth = depth_knob >= 0 ? (uint64_t)depth_knob : (any_dma ? 2 : 3);
  // (the largest chunk: `per` grows past ~240 chunks)
  uint64_t max_rows = 0;
  for (uint64_t k = 0; k < K; ++k) max_rows = std::max(max_rows, row_of(tb[k + 1]) - row_of(tb[k]));
  const size_t bounce_bytes = (size_t)max_rows * npol * 4;
  void* bounce[2] = {nullptr, nullptr};
  // descriptors: two halves of `dcap` on the device and in pinned host memory (chunk k uses half
  // k & 1; half reuse waits for chunk k-2's kernel on the device and its upload on the host)
  uint64_t dcap = tper + tper / 4 + 64;
  void* hdesc = nullptr;
  size_t hdesc_bytes = 0;
  hipStream_t s_in = nullptr, s_out = nullptr;
  std::vector<hipEvent_t> ev(3 * K, nullptr);
  int rc = KW_OK;  // (a failure below leaves the batch's columns partly uploaded: D.loaded is cleared)
  auto fail = [&](hipError_t e) {
    if (e != hipSuccess && rc == KW_OK) rc = KW_E_DEVICE;
    return e != hipSuccess;
  };
  auto code = [&](int c) {
    if (c != KW_OK && rc == KW_OK) rc = c;
    return c != KW_OK;
  };
  if (!pinned)
    for (auto& b : bounce)
      if (fail(host_pool().alloc(device, bounce_bytes, &b))) break;
  auto alloc_descs = [&]() {
    if (hdesc) host_pool().release(device, hdesc, hdesc_bytes);
    hdesc = nullptr;
    hdesc_bytes = (size_t)(2 * dcap) * sizeof(TileDesc);
    if (fail(host_pool().alloc(device, hdesc_bytes, &hdesc))) return false;
    return !code(ensure(&D.desc, &D.desc_cap, (size_t)(2 * dcap)));
  };
  if (rc == KW_OK) (void)alloc_descs();
  // staged columns: each chunk's ranges packed into one pinned slot, one H2D into the device slot,
  // then the scatter kernel puts them in place (one copy per chunk, not one per column). kRing
  // slots: packing chunk k waits for chunk k - kRing's upload. KW_BULK_PACK=0: a copy per column
  // range (A/B knob, profiles/r05_bulk_copies.txt).
  constexpr uint64_t kRing = 4;
  // (the scatter kernel's argument holds kMaxScatterSegs ranges: a layout with more staged pieces
  // than that — none today, 6 row pieces + 2 per string column — copies each range on its own)
  const bool packed = pack_knob && std::count(dma.begin(), dma.end(), 0) > 0 &&
                      (size_t)std::count(dma.begin(), dma.end(), 0) <= kMaxScatterSegs;
  size_t slot_bytes = 0;
  void *hpack = nullptr, *dland = nullptr;
  if (packed && rc == KW_OK) {
    for (uint64_t k = 0; k < K; ++k) {
      size_t b = 0;
      for (size_t i = 0; i < pieces.size(); ++i) {
        if (!wanted(pieces[i]) || dma[i]) continue;
        size_t lo, hi;
        piece_range(B, pieces[i], row_of(tb[k]), row_of(tb[k + 1]), k + 1 == K, &lo, &hi);
        if (hi > lo) b += (hi - lo) + 32;
      }
      slot_bytes = std::max(slot_bytes, (b + 255) & ~(size_t)255);
    }
    if (!fail(host_pool().alloc(device, kRing * slot_bytes, &hpack))) (void)fail(dev_pool().alloc(device, kRing * slot_bytes, &dland));
  }
  StreamPool& SP = stream_pool();
  if (rc == KW_OK && !fail(SP.get(device, &s_in)) && !fail(SP.get(device, &s_out)))
    for (auto& e : ev)
      if (fail(SP.get(device, &e))) break;
  auto copy_out = [&](uint64_t k) {
    const auto t0 = clk::now();
    if (pinned || rc != KW_OK || fail(hipEventSynchronize(ev[3 * k + 2]))) return;
    const uint64_t r0 = row_of(tb[k]), r1 = row_of(tb[k + 1]);
    parallel_copy_segs({{out + r0 * npol, bounce[k & 1], (size_t)(r1 - r0) * npol * 4}});
    t_out += since(t0);
  };
  // overflow requests (alone beyond the tile capacities): their list, classes and side data
  uint64_t n_ovf = 0;
  std::vector<TileDesc> cd;
  std::vector<uint32_t> co;
  for (uint64_t k = 0; k < K && rc == KW_OK; ++k) {
    const uint64_t r0 = row_of(tb[k]), r1 = row_of(tb[k + 1]);
    if (pinned && depth && k >= depth && fail(hipEventSynchronize(ev[3 * (k - depth) + 2]))) break;
    // the chunk's columns first: their H2D starts at once, and the descriptor build below then
    // reads offsets the fill has just brought into the host caches
    std::vector<CopySeg> segs, dsegs;  // (staged, direct)
    const size_t slot = (size_t)(k % kRing) * slot_bytes;
    ScatterArgs sa;
    sa.dst = D.cols;
    sa.src = (const uint8_t*)dland + slot;
    sa.nseg = 0;
    size_t pk = 0;  // packed bytes of the chunk (each range at its device offset's residue mod 16)
    for (size_t i = 0; i < pieces.size(); ++i) {
      const Piece& p = pieces[i];
      if (!wanted(p)) continue;
      size_t lo, hi;
      piece_range(B, p, r0, r1, k + 1 == K, &lo, &hi);
      if (hi <= lo) continue;
      if (dma[i]) {
        dsegs.push_back({D.cols + p.at + lo, (const uint8_t*)p.src + lo, hi - lo});
      } else if (packed) {
        const size_t at = ((pk + 15) & ~(size_t)15) + ((p.at + lo) & 15);
        segs.push_back({(uint8_t*)hpack + slot + at, (const uint8_t*)p.src + lo, hi - lo});
        sa.seg[sa.nseg++] = {p.at + lo, at, hi - lo};
        pk = at + (hi - lo);
      } else {
        segs.push_back({st + p.at + lo, (const uint8_t*)p.src + lo, hi - lo});
      }
    }
    if (packed && k >= kRing && fail(hipEventSynchronize(ev[3 * (k - kRing)]))) break;  // its slot's upload is done
    const auto t0 = clk::now();
    parallel_copy_segs(segs);
    t_fill += since(t0);
    const auto t1 = clk::now();
    for (const CopySeg& c : dsegs)
      if (fail(hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyHostToDevice, s_in))) break;
    if (packed) {
      if (pk && (fail(hipMemcpyAsync((uint8_t*)dland + slot, (uint8_t*)hpack + slot, pk, hipMemcpyHostToDevice, s_in)) ||
                 fail(launch_scatter(sa, s_in))))
        break;
    } else {
      for (const CopySeg& c : segs)
        if (rc != KW_OK ||
            fail(hipMemcpyAsync(D.cols + ((uint8_t*)c.dst - st), c.dst, c.bytes, hipMemcpyHostToDevice, s_in)))
          break;
    }
    if (rc != KW_OK) break;
    t_enq += since(t1);
    const auto td = clk::now();
    cd.clear();
    co.assign(1, 0u);
    if (code(build_descs(B, G, 0, B.n, tb[k], tb[k + 1], 128, &cd, &co))) break;
    co[0] = (uint32_t)(co.size() - 1);
    if (cd.size() > dcap) {  // more split tiles than the halves hold: wait for every launch, regrow
      if (fail(hipStreamSynchronize(s_in)) || fail(hipStreamSynchronize(sc))) break;
      dcap = cd.size() + cd.size() / 4 + 64;
      if (!alloc_descs()) break;
    } else if (k >= 2 && fail(hipEventSynchronize(ev[3 * (k - 2)]))) {  // host half free: its upload is done
      break;
    }
    TileDesc* hd = (TileDesc*)hdesc + (k & 1) * dcap;
    if (!cd.empty()) memcpy(hd, cd.data(), cd.size() * sizeof(TileDesc));
    t_desc += since(td);
    const auto t2 = clk::now();
    TileDesc* dd = D.desc + (k & 1) * dcap;
    if (k >= 2 && fail(hipStreamWaitEvent(s_in, ev[3 * (k - 2) + 1], 0))) break;  // device half free
    if (!cd.empty() && fail(hipMemcpyAsync(dd, hd, cd.size() * sizeof(TileDesc), hipMemcpyHostToDevice, s_in))) break;
    if (fail(hipEventRecord(ev[3 * k], s_in)) || fail(hipStreamWaitEvent(sc, ev[3 * k], 0))) break;
    EvalArgs Ak = A;
    Ak.ndesc = cd.size();
    if (!sched_dynamic(cd.size(), plan.grid, plan.geom.lds_tables != 0)) Ak.sched = nullptr;
    if (!cd.empty() && fail(launch_evaluate_tiles(Ak, plan.tiles[0], D.d_tiles, dd, plan.grid, sc))) break;
    if (co[0]) {  // rare: synchronous set-up, then the overflow kernels on the chunk's requests
      if (fail(hipStreamSynchronize(sc))) break;
      if (n_ovf == 0 && fail(hipMemsetAsync(D.wide_count, 0, sizeof(uint32_t), sc))) break;  // (first overflow chunk)
      D.wide_valid = true;
      n_ovf += co[0];
      if (code(ensure(&D.overflow, &D.overflow_cap, co.size())) || code(ensure_overflow_classes(B, &D, G, &A))) break;
      const size_t cap = (size_t)n_ovf * plan.wide_cap_per_row;
      if (cap > D.wide_rec_cap || !D.wide_rec) {  // grow, keeping the records earlier chunks wrote
        WideRec* old = D.wide_rec;
        const size_t old_cap = D.wide_rec_cap;
        D.wide_rec = nullptr;
        D.wide_rec_cap = 0;
        if (code(ensure(&D.wide_rec, &D.wide_rec_cap, std::max(cap, 2 * old_cap)))) break;
        if (old && fail(hipMemcpy(D.wide_rec, old, old_cap * sizeof(WideRec), hipMemcpyDeviceToDevice))) break;
        if (old) dev_pool().release(device, old, old_cap * sizeof(WideRec));
      }
      A.wide_rec = D.wide_rec;
      A.wide_cap = (uint32_t)std::min<size_t>(D.wide_rec_cap, 0xffffffffu);
      Ak = A;
      if (fail(hipMemcpy(D.overflow, co.data(), co.size() * sizeof(uint32_t), hipMemcpyHostToDevice))) break;
      if (fail(launch_overflow(Ak, D.d_tiles, D.overflow, co[0], sc))) break;
    }
    if (fail(hipEventRecord(ev[3 * k + 1], sc)) || fail(hipStreamWaitEvent(s_out, ev[3 * k + 1], 0))) break;
    uint32_t* dst = pinned ? out + r0 * npol : (uint32_t*)bounce[k & 1];
    if (fail(hipMemcpyAsync(dst, D.verdicts + r0 * npol, (size_t)(r1 - r0) * npol * 4, hipMemcpyDeviceToHost, s_out))) break;
    if (fail(hipEventRecord(ev[3 * k + 2], s_out))) break;
    t_enq += since(t2);
    if (k == 0) t_first = since(t_start);
    if (k >= 1) copy_out(k - 1);  // (bounce[k & 1] was last read by chunk k - 2's copy-out)
  }
  if (rc == KW_OK) copy_out(K - 1);
  const auto t_w = clk::now();
  if (s_in) (void)hipStreamSynchronize(s_in);
  (void)hipStreamSynchronize(sc);
  if (s_out) (void)hipStreamSynchronize(s_out);
  const double t_wait = since(t_w);
  const auto t_td = clk::now();
  for (auto& e : ev) SP.put(device, e);
  SP.put(device, s_in);
  SP.put(device, s_out);
  for (auto& b : bounce) host_pool().release(device, b, bounce_bytes);
  if (hdesc) host_pool().release(device, hdesc, hdesc_bytes);
  if (hpack) host_pool().release(device, hpack, kRing * slot_bytes);
  if (dland) dev_pool().release(device, dland, kRing * slot_bytes);
  D.last_wide_cap = A.wide_cap;
  D.cur = sc;
  if (rc != KW_OK) {
    D.loaded = 0;
    return rc;
  }
  rc = load_side_data(kb, sc);  // overflow requests' wide arguments (kw_batch_wide_arg)
  if (dbg)
    fprintf(stderr,
            "[kw bulk] rows %llu chunks %llu pinned %d direct-columns %d overflow %llu: layout %.2f plan %.2f prepare %.2f "
            "descs %.2f fill %.2f enqueue %.2f copy-out %.2f first chunk queued at %.2f, final wait %.2f, teardown %.2f, "
            "total %.2f ms\n",
            (unsigned long long)B.n, (unsigned long long)K, pinned ? 1 : 0, (int)std::count(dma.begin(), dma.end(), 1),
            (unsigned long long)n_ovf, t_layout, t_plan, t_prep, t_desc, t_fill, t_enq, t_out, t_first, t_wait, since(t_td),
            since(t_start));
  return rc;
}
}  // namespace

extern "C" {

int kw_batch_to_device(kw_batch* kb, int device) { return upload_batch(kb, device, nullptr, true); }

int kw_batch_to_device_async(kw_batch* kb, int device, void* stream) {
  if (!stream) return KW_E_ARG;
  return upload_batch(kb, device, (hipStream_t)stream, false);
}

int kw_validate_host(const kw_env* env, kw_batch* b, const int32_t* policies, uint32_t npol, int origin, int device,
                     uint32_t* out, size_t count, uint32_t chunk_rows) {
  return validate_host(env, b, policies, npol, origin, device, out, count, chunk_rows);
}

int kw_host_alloc(int device, size_t bytes, void** out) {
  if (!out || device < 0) return KW_E_ARG;
  HIPCHK(hipSetDevice(device));
  *out = nullptr;
  HIPCHK(hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault));
  return KW_OK;
}

void kw_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int kw_stream_create(int device, void** stream) {
  if (!stream || device < 0) return KW_E_ARG;
  HIPCHK(hipSetDevice(device));
  hipStream_t s = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = (void*)s;
  return KW_OK;
}

void kw_stream_destroy(void* stream) {
  if (stream) (void)hipStreamDestroy((hipStream_t)stream);
}

void kw_batch_destroy(kw_batch* b) { delete b; }

int kw_batch_pin_host(kw_batch* kb, int device) {
  if (!kb || device < 0) return KW_E_ARG;
  if (!kb->host_pinned.empty()) return KW_OK;
  HIPCHK(hipSetDevice(device));
  Batch& B = kb->b;
  B.finalize();  // (pads the byte pools now: later passes do not resize what is registered)
  std::vector<std::pair<void*, size_t>> cols = {
      {B.req_flags.data(), B.req_flags.size()},   {B.ctr_off.data(), B.ctr_off.size() * 4},
      {B.lbl_off.data(), B.lbl_off.size() * 4},   {B.ctr_flags.data(), B.ctr_flags.size()},
      {B.capadd_off.data(), B.capadd_off.size() * 4}, {B.capdrop_off.data(), B.capdrop_off.size() * 4}};
  for (int m = 0; m < (int)NSTR; ++m) {
    const StrCol& c = host_str(B, m);
    cols.push_back({(void*)c.off.data(), c.off.size() * 4});
    cols.push_back({(void*)c.bytes.data(), c.bytes.size()});
  }
  // small arrays may share a page with another allocation: they stay pageable (staged), as does
  // any array the runtime declines to register
  for (const auto& [p, n] : cols) {
    if (n < ((size_t)1 << 16)) continue;
    if (hipHostRegister(p, n, hipHostRegisterDefault) == hipSuccess)
      kb->host_pinned.push_back(p);
    else
      (void)hipGetLastError();
  }
  return KW_OK;
}

int kw_validate_batch(const kw_env* env, kw_batch* b, const int32_t* policies, uint32_t npol, int origin, void* stream) {
  PassPlan* plan = nullptr;
  if (int rc = validate_cached(env, b, policies, npol, origin, &plan)) return rc;
  return run_validate(env, b, *plan, origin, false, stream ? (hipStream_t)stream : b->dev->stream);
}

int kw_validate_rows(const kw_env* env, kw_batch* b, const int32_t* row_policy, int origin, void* stream) {
  if (!row_policy) return KW_E_ARG;
  PassPlan plan;
  if (int rc = validate_common(env, b, nullptr, 0, row_policy, origin, &plan)) return rc;
  return run_validate(env, b, plan, origin, false, stream ? (hipStream_t)stream : b->dev->stream);
}

int kw_batch_verdicts(kw_batch* b, uint32_t* host_out, size_t count) {
  if (!b || !b->dev || (!host_out && count)) return KW_E_ARG;
  DeviceBatch& D = *b->dev;
  if (count > D.last_verdicts) return KW_E_ARG;
  HIPCHK(hipSetDevice(D.device));
  hipStream_t s = D.cur ? D.cur : D.stream;
  const size_t vbytes = count * sizeof(uint32_t);
  constexpr size_t kBounce = (size_t)64 << 20;
  if (D.split && count) {
    // rows in device order (light / heavy split): whole device rows through a pinned bounce block,
    // each scattered to its batch row's words below `count`
    const uint64_t rw = std::max<uint32_t>(D.last_row_words, 1), nrows = D.last_verdicts / rw;
    const uint64_t per = std::max<uint64_t>(1, kBounce / (rw * 4));
    void* bounce = nullptr;
    HIPCHK(host_pool().alloc(D.device, kBounce, &bounce));
    for (uint64_t d0 = 0; d0 < nrows; d0 += per) {
      const uint64_t d1 = std::min(nrows, d0 + per);
      HIPCHK(hipMemcpyAsync(bounce, D.verdicts + d0 * rw, (d1 - d0) * rw * 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      const uint32_t* src = (const uint32_t*)bounce;
      HostWorkers::get().run((size_t)((d1 - d0 + 4095) / 4096), [&](size_t q) {
        for (uint64_t d = d0 + q * 4096, e = std::min(d1, d0 + (q + 1) * 4096); d < e; ++d) {
          const uint64_t w0 = D.perm[d] * rw;
          if (w0 < count) memcpy(host_out + w0, src + (d - d0) * rw, std::min<uint64_t>(rw, count - w0) * 4);
        }
      });
    }
    host_pool().release(D.device, bounce, kBounce);
  } else if (vbytes > ((size_t)16 << 20)) {
    // large read-backs through a pinned bounce block (full-rate DMA), fanned out to the caller's
    // (pageable) buffer by several threads
    void* bounce = nullptr;
    HIPCHK(host_pool().alloc(D.device, kBounce, &bounce));
    for (size_t at = 0; at < vbytes; at += kBounce) {
      const size_t n = std::min(kBounce, vbytes - at);
      HIPCHK(hipMemcpyAsync(bounce, (const uint8_t*)D.verdicts + at, n, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      parallel_copy((uint8_t*)host_out + at, bounce, n);
    }
    host_pool().release(D.device, bounce, kBounce);
  } else if (count) {
    HIPCHK(hipMemcpyAsync(host_out, D.verdicts, vbytes, hipMemcpyDeviceToHost, s));
  }
  return load_side_data(b, s);
}

int kw_debug_plan(const kw_env* env, kw_batch* kb, const int32_t* policies, uint32_t npol, int origin, uint32_t* out,
                  int cap) {
  if (!env || !kb || !out || cap < 8 || (!policies && npol)) return KW_E_ARG;
  // plan against a host view of the batch (no device memory, nothing launched), in the device-row
  // order kw_batch_to_device would give it
  std::unique_ptr<DeviceBatch> saved = std::move(kb->dev);
  kb->b.finalize();
  std::vector<uint64_t> perm;
  const uint64_t split = split_rows(kb->b, &perm);
  std::unique_ptr<Batch> P;
  if (split) {
    P = std::make_unique<Batch>();
    RowOrder o;
    permute_batch(kb->b, perm, P.get(), /*with_bytes=*/false, &o);
  }
  const Batch& B = P ? *P : kb->b;
  auto D = std::make_unique<DeviceBatch>();
  D->split = split;
  D->perm = std::move(perm);
  static uint32_t dummy;
  D->req_flags = B.req_flags.data();
  D->ctr_off = B.ctr_off.data();
  D->lbl_off = B.lbl_off.data();
  D->ctr_flags = B.ctr_flags.data();
  D->capadd_off = B.capadd_off.data();
  D->capdrop_off = B.capdrop_off.data();
  for (int m = 0; m < (int)NSTR; ++m) {
    const StrCol& c = host_str(B, m);
    D->str[m] = {c.off.data(), c.bytes.empty() ? (const uint8_t*)&dummy : c.bytes.data(), c.n(), c.off.back()};
  }
  D->verdicts = &dummy;
  D->dev_b = std::move(P);
  kb->dev = std::move(D);
  PassPlan plan;
  int rc = plan_pass(env, kb, policies, npol, nullptr, origin, &plan);
  const TileArgs& T = plan.geom;
  const uint32_t vals[8] = {T.lds_bytes, (uint32_t)plan.launches.size(), (uint32_t)plan.chunks.size(), T.lds_tables,
                            T.rows, T.cmax, T.kmax, T.lmax};
  for (int i = 0; i < 8; ++i) out[i] = rc == KW_OK ? vals[i] : 0u;
  if (cap >= 16) {  // regions: count, light rows, the first region's grid, the heavy region's LDS / rows / cmax / grid, scan regions
    const bool two = rc == KW_OK && plan.regions.size() == 2;
    const TileArgs* H = two ? &plan.regions[1].geom : nullptr;
    uint32_t more[8] = {rc == KW_OK ? (uint32_t)plan.regions.size() : 0u, (uint32_t)split,
                              rc == KW_OK ? plan.regions[0].grid : 0u, H ? H->lds_bytes : 0u, H ? H->rows : 0u,
                              H ? H->cmax : 0u, two ? plan.regions[1].grid : 0u, 0u};
    if (rc == KW_OK)  // regions launched as the wave-scan instantiation (kFeatRng), one bit each
      for (size_t k = 0; k < plan.regions.size() && k < 32; ++k) more[7] |= (plan.regions[k].geom.feat & kFeatRng) ? 1u << k : 0u;
    for (int i = 0; i < 8; ++i) out[8 + i] = more[i];
  }
  kb->dev->verdicts = nullptr;  // host memory: not the DeviceBatch's to free
  kb->dev = std::move(saved);
  return rc;
}

int kw_debug_reorder(const kw_batch* kb, uint64_t* perm, size_t cap, uint64_t* split, kw_batch** out) {
  if (!kb || !split || !out || (!perm && kb->b.n) || cap < kb->b.n) return KW_E_ARG;
  std::vector<uint64_t> p;
  *split = split_rows(kb->b, &p);
  if (!*split) {
    p.resize(kb->b.n);
    for (uint64_t r = 0; r < kb->b.n; ++r) p[r] = r;
  }
  auto nb = std::make_unique<kw_batch>();
  RowOrder o;
  permute_batch(kb->b, p, &nb->b, /*with_bytes=*/true, &o);
  std::copy(p.begin(), p.end(), perm);
  *out = nb.release();
  return KW_OK;
}

int kw_batch_group_causes(const kw_batch* b, uint64_t row, int32_t policy, uint32_t verdict, uint64_t* words,
                          size_t nwords, size_t* needed) {
  if (!b || (!words && nwords)) return KW_E_ARG;
  if (KW_REASON(verdict) != KW_R_GROUP) return KW_E_ARG;
  const WideData& W = b->b.wide;
  uint32_t bw = 0;
  const uint64_t* big = W.lookup_big(row, policy, &bw);
  uint64_t one = KW_ARG(verdict);
  if (!big && KW_ARG(verdict) == kArgWide && !W.lookup(row, policy, &one)) return KW_E_NOT_FOUND;
  const size_t n = big ? bw : 1u;
  if (needed) *needed = n;
  if (nwords < n) return KW_E_NOSPACE;
  for (size_t k = 0; k < n; ++k) words[k] = big ? big[k] : one;
  return KW_OK;
}

int kw_batch_wide_arg(const kw_batch* b, uint64_t row, int32_t policy, uint64_t* value) {
  if (!b || !value) return KW_E_ARG;
  return b->b.wide.lookup(row, policy, value) ? KW_OK : KW_E_NOT_FOUND;
}

int kw_validate_timed(const kw_env* env, kw_batch* b, const int32_t* policies, uint32_t npol, int origin, int warmup,
                      int reps, kw_timing* out) {
  if (!out || reps <= 0) return KW_E_ARG;
  PassPlan plan;
  if (int rc = validate_common(env, b, policies, npol, nullptr, origin, &plan)) return rc;
  DeviceBatch& D = *b->dev;
  for (auto& e : D.ev)
    if (!e) HIPCHK(hipEventCreate(&e));
  for (int i = 0; i < warmup; ++i)
    if (int rc = run_validate(env, b, plan, origin, false, D.stream)) return rc;
  HIPCHK(hipStreamSynchronize(D.stream));
  double ev = 0;
  for (int i = 0; i < reps; ++i) {
    if (int rc = run_validate(env, b, plan, origin, true, D.stream)) return rc;
    HIPCHK(hipEventSynchronize(D.ev[2]));
    float c = 0;
    HIPCHK(hipEventElapsedTime(&c, D.ev[0], D.ev[2]));
    ev += c;
  }
  out->classify_ms = 0;
  out->evaluate_ms = ev / reps;
  out->total_ms = ev / reps;
  out->classify_bytes = 0;
  out->evaluate_bytes = plan.evaluate_bytes;
  return KW_OK;
}

int kw_format_response(const kw_env* env, const kw_batch* b, uint64_t row, int32_t policy, uint32_t verdict,
                       const uint32_t* member_verdicts, char* buf, size_t cap, size_t* need) {
  if (!env || !b || row >= b->b.n || policy < 0 || (size_t)policy >= env->e.nvisible) return KW_E_ARG;
  std::string out;
  Status st = format_response(env->e, b->b, row, policy, verdict, member_verdicts, &out);
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  return put_out(out, buf, cap, need);
}

int kw_format_response_doc(const kw_env* env, const kw_batch* b, uint64_t row, int32_t policy, uint32_t verdict,
                           const uint32_t* member_verdicts, const char* doc, size_t doc_len, int doc_kind, char* buf,
                           size_t cap, size_t* need) {
  if (!env || !b || row >= b->b.n || policy < 0 || (size_t)policy >= env->e.nvisible || (!doc && doc_len))
    return KW_E_ARG;
  std::string out;
  Status st = format_response(env->e, b->b, row, policy, verdict, member_verdicts, &out, doc, doc_len, doc_kind);
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  return put_out(out, buf, cap, need);
}

int kw_evaluate(const kw_env* env, const char* policy_id, const char* doc, size_t doc_len, int doc_kind, int origin,
                char* buf, size_t cap, size_t* need) {
  if (!env || !policy_id || !doc) return KW_E_ARG;
  const Env& E = env->e;
  int32_t idx;
  Status st = env_lookup(E, policy_id, &idx);  // service.rs:37 + PolicyNotFound
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  kw_batch* kb = nullptr;
  char err[512];
  int rc = kw_batch_from_json(&doc, &doc_len, 1, doc_kind, &kb, nullptr, err, sizeof(err));
  if (rc) {
    put_out(err, buf, cap, need);
    return rc;
  }
  std::unique_ptr<kw_batch> hold(kb);
  if (E.device < 0) {
    put_out("engine has no device: the hot path runs only on the GPU", buf, cap, need);
    return KW_E_DEVICE;
  }
  if ((rc = kw_batch_to_device(kb, E.device))) return rc;
  std::vector<int32_t> pols{idx};
  const PolicyRec& P = E.pol[(size_t)idx];
  for (int32_t m : P.members) pols.push_back(m);
  if ((rc = kw_validate_batch(env, kb, pols.data(), (uint32_t)pols.size(), origin, nullptr))) return rc;
  std::vector<uint32_t> v(pols.size());
  if ((rc = kw_batch_verdicts(kb, v.data(), v.size()))) return rc;
  std::string out;
  st = format_response(E, kb->b, 0, idx, v[0], v.size() > 1 ? v.data() + 1 : nullptr, &out, doc, doc_len, doc_kind);
  if (!st.ok()) {
    put_out(st.message, buf, cap, need);
    return st.code;
  }
  return put_out(out, buf, cap, need);
}

int kw_service_constraints(uint32_t in, int mode, int allowed_to_mutate, uint32_t* out_flags) {
  // validation_response_with_constraints (service.rs:160-208); bit0 allowed, bit1 patch, bit2 status
  uint32_t o = in;
  int fst;
  if (mode == KW_MODE_MONITOR) {
    o = 1u;
    fst = KW_FST_NONE;
  } else if ((in & 2u) && !allowed_to_mutate) {
    o = 4u;
    fst = KW_FST_MUTATION_REFUSED;
  } else {
    fst = (in & 4u) ? KW_FST_VANILLA : KW_FST_NONE;
  }
  if (out_flags) *out_flags = o;
  return fst;
}

}  // extern "C"

// ---- metrics (metrics.hpp)
struct kw_metrics {
  kw::Metrics m;
};

kw_metrics* kw_metrics_create(void) { return new (std::nothrow) kw_metrics(); }
void kw_metrics_destroy(kw_metrics* m) { delete m; }

int kw_metrics_record(kw_metrics* m, const kw_env* env, const kw_batch* b, const uint64_t* rows,
                      const int32_t* policies, const uint32_t* verdicts, const uint64_t* latency_ms, size_t n,
                      int origin) {
  if (!m || !env || !b || (n && (!rows || !policies || !verdicts || !latency_ms))) return KW_E_ARG;
  if (origin != KW_ORIGIN_VALIDATE && origin != KW_ORIGIN_AUDIT) return KW_E_ARG;
  for (size_t i = 0; i < n; ++i)
    if (rows[i] >= b->b.n || policies[i] < 0 || (size_t)policies[i] >= env->e.nvisible) return KW_E_ARG;
  for (size_t i = 0; i < n; ++i) m->m.record(env->e, b->b, rows[i], policies[i], verdicts[i], origin, latency_ms[i]);
  return KW_OK;
}

int kw_metrics_render(const kw_metrics* m, char* buf, size_t cap, size_t* need) {
  if (!m) return KW_E_ARG;
  return put_out(m->m.render(), buf, cap, need);
}

void kw_metrics_reset(kw_metrics* m) {
  if (m) m->m.reset();
}
