// Host side of the controller's device aggregation backend (device_agg.h):
// residency bookkeeping, pinned-ring uploads / downloads, tile tables.
#include "engine/device_agg.h"

#include <hip/hip_runtime_api.h>
#include <omp.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <list>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <unordered_map>
#include <unordered_set>

#include "engine/device_agg_kernels.h"

namespace mfl {
namespace {

using namespace devagg;

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string("device aggregation: ") + what + ": " + hipGetErrorString(e));
}

struct Layout {
  std::vector<uint64_t> off, bytes;
  std::vector<uint32_t> len;
  std::vector<int> dtype;
  uint64_t total = 0;
};

Layout make_layout(const ModelT& m) {
  Layout L;
  uint64_t o = 0;
  for (auto& v : m.vars) {
    const uint64_t b = (uint64_t)v.t.length * dtype_size(v.t.dtype);
    if (v.t.value.size() != b) throw std::runtime_error("device aggregation: value size mismatch");
    L.off.push_back(o);
    L.bytes.push_back(b);
    L.len.push_back(v.t.length);
    L.dtype.push_back(v.t.dtype);
    o += (b + kAlign - 1) / kAlign * kAlign;
  }
  L.total = std::max<uint64_t>(o, kAlign);
  return L;
}

bool same_layout(const Layout& a, const Layout& b) {
  return a.bytes == b.bytes && a.dtype == b.dtype;
}

std::vector<Tile> make_tiles(const Layout& L) {
  std::vector<Tile> t;
  for (size_t v = 0; v < L.off.size(); ++v) {
    const uint32_t es = (uint32_t)dtype_size(L.dtype[v]);
    const uint32_t per = kTileBytes / es;
    for (uint64_t b = 0; b < L.len[v]; b += per)
      t.push_back({L.off[v] + b * es, (uint32_t)std::min<uint64_t>(per, L.len[v] - b),
                   (uint32_t)L.dtype[v]});
  }
  return t;
}

// A contiguous host byte range that maps onto [dst, dst + n) of a packed model.
struct Piece {
  const char* src;
  char* dst_host;  // for downloads: destination in host memory
  uint64_t packed_off, n;
};

struct Slot {
  std::string learner;
  std::vector<const char*> ptrs;
  std::vector<size_t> sizes;
  Layout lay;
  char* dev = nullptr;
  hipEvent_t ready = nullptr;
  uint64_t stamp = 0;
  int pins = 0;  // > 0 while an aggregation reads it: never evicted
  uint64_t uid = 0;  // ModelT::uid of the staged model
  bool matches(const ModelT& m) const {
    if (m.uid != uid || m.vars.size() != ptrs.size()) return false;
    for (size_t i = 0; i < ptrs.size(); ++i)
      if (m.vars[i].t.value.data() != ptrs[i] || m.vars[i].t.value.size() != sizes[i]) return false;
    return true;
  }
};

// Every entry point runs on the aggregation device and gives the caller's
// thread its current device back (torch and the engine share one HIP runtime).
struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    hip_check(hipSetDevice(dev), "hipSetDevice");
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

class Impl final : public DeviceAggregator {
 public:
  explicit Impl(int dev) : dev_(dev) {
    hip_check(hipSetDevice(dev_), "hipSetDevice");
    char name[256] = {0};
    hip_check(hipDeviceGetName(name, sizeof(name) - 1, dev_), "hipDeviceGetName");
    stats_.device = dev_;
    stats_.device_name = name;
    hip_check(hipStreamCreateWithFlags(&upload_, hipStreamNonBlocking), "stream");
    hip_check(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking), "stream");
    for (auto& r : ring_) {
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&r.host), kChunk, hipHostMallocDefault),
                "hipHostMalloc");
      hip_check(hipEventCreateWithFlags(&r.done, hipEventDisableTiming), "event");
    }
    hip_check(hipEventCreate(&k0_), "event");
    hip_check(hipEventCreate(&k1_), "event");
    size_t free_b = 0, total_b = 0;
    hip_check(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    budget_ = free_b / 2;
    if (const char* e = std::getenv("METISFL_AMD_DEVICE_AGG_MAX_GB"))
      budget_ = (uint64_t)(std::atof(e) * (double)(1ull << 30));
  }

  ~Impl() override {
    // process teardown: the HIP runtime may already be gone; release nothing.
  }

  void stage(const std::string& learner, const ModelT& m, int keep) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    if (m.vars.empty()) return;
    // a new model invalidates any slot that still names one of its buffers
    // (its previous owner was freed and the allocator reused the address)
    std::unordered_set<const char*> mine;
    for (auto& v : m.vars) mine.insert(v.t.value.data());
    for (auto it = slots_.begin(); it != slots_.end();) {
      bool overlap = false;
      for (auto* p : (*it)->ptrs) overlap = overlap || mine.count(p);
      it = (overlap && !(*it)->pins) ? release(it) : std::next(it);
    }
    int have = 0;
    for (auto& s : slots_) have += s->learner == learner;
    while (keep > 0 && have >= keep) {
      auto oldest = slots_.end();
      for (auto it = slots_.begin(); it != slots_.end(); ++it)
        if ((*it)->learner == learner && (oldest == slots_.end() || (*it)->stamp < (*oldest)->stamp))
          oldest = it;
      if (oldest == slots_.end()) break;
      release(oldest);
      --have;
    }
    Slot* s = upload(m, learner);
    if (s) {
      stats_.staged_models++;
      stats_.staged_bytes += s->lay.total;
    }
  }

  void drop(const std::string& learner) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    for (auto it = slots_.begin(); it != slots_.end();)
      it = (*it)->learner == learner ? release(it) : std::next(it);
  }

  void clear() override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    while (!slots_.empty()) release(slots_.begin());
  }

  bool weighted_sum(ModelT& out, const std::vector<const ModelT*>& models,
                    const std::vector<double>& weights) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    const auto t0 = std::chrono::steady_clock::now();
    if (models.empty()) return false;
    const Layout lay = make_layout(*models.front());
    std::vector<Slot*> in, cold;
    if (!resolve(models, lay, in, cold)) return false;
    char* o = scratch(lay.total);
    upload_tiles(lay);
    hip_check(hipEventRecord(k0_, compute_), "event");
    for (size_t b = 0; b < in.size(); b += kMaxModels) {
      WSumArgs a{};
      a.count = (int)std::min<size_t>(kMaxModels, in.size() - b);
      for (int k = 0; k < a.count; ++k) {
        a.x[k] = in[b + k]->dev;
        a.w[k] = weights[b + k];
      }
      hip_check((hipError_t)launch_wsum(o, tiles_dev_, ntiles_, a, b > 0, compute_), "wsum launch");
    }
    hip_check(hipEventRecord(k1_, compute_), "event");
    download(out, *models.front(), lay, o);
    finish(in, cold);
    float kms = 0;
    hipEventElapsedTime(&kms, k0_, k1_);
    stats_.last_kernel_ms = kms;
    stats_.fedavg_calls++;
    stats_.last_total_ms = ms_since(t0);
    return true;
  }

  int roll_init(const ModelT& m, double w) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    Roll r;
    r.lay = make_layout(m);
    std::vector<Slot*> in, cold;
    if (!resolve({&m}, r.lay, in, cold)) return -1;
    if (hipMalloc(reinterpret_cast<void**>(&r.dev), r.lay.total) != hipSuccess) {
      (void)hipGetLastError();
      finish(in, cold);
      return -1;
    }
    resident_bytes_ += r.lay.total;  // the rolling state counts against the HBM budget
    r.meta.vars.resize(m.vars.size());
    for (size_t v = 0; v < m.vars.size(); ++v) {
      auto& mv = r.meta.vars[v];
      mv.name = m.vars[v].name;
      mv.trainable = m.vars[v].trainable;
      mv.ciphertext = m.vars[v].ciphertext;
      mv.t.length = m.vars[v].t.length;
      mv.t.dims = m.vars[v].t.dims;
      mv.t.dtype = m.vars[v].t.dtype;
      mv.t.byte_order = m.vars[v].t.byte_order;
      mv.t.fortran_order = m.vars[v].t.fortran_order;
    }
    upload_tiles(r.lay);
    roll_(r.dev, in[0]->dev, w, ROLL_MUL);
    finish(in, cold);
    stats_.rolling_calls++;
    const int h = next_roll_++;
    rolls_[h] = std::move(r);
    return h;
  }

  void roll_merge(int h, const ModelT& x, double w, int op) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    Roll& r = roll_at(h);
    std::vector<Slot*> in, cold;
    if (!resolve({&x}, r.lay, in, cold))
      throw std::runtime_error("device aggregation: out of device memory for a rolling merge");
    upload_tiles(r.lay);
    roll_(r.dev, in[0]->dev, w, op);
    finish(in, cold);
    stats_.rolling_calls++;
  }

  void roll_fetch(int h, ModelT& out, double z, int op) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    Roll& r = roll_at(h);
    char* o = scratch(r.lay.total);
    upload_tiles(r.lay);
    roll_(o, r.dev, z, op);
    download(out, r.meta, r.lay, o);
  }

  void roll_free(int h) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    auto it = rolls_.find(h);
    if (it == rolls_.end()) return;
    hipStreamSynchronize(compute_);
    hipFree(it->second.dev);
    resident_bytes_ -= it->second.lay.total;
    rolls_.erase(it);
  }

  bool ckks_pwa(const std::vector<const uint64_t*>& bodies, const std::vector<uint64_t>& wq,
                const std::vector<uint64_t>& wqs, const std::vector<uint64_t>& q, uint32_t L,
                uint32_t N, uint64_t total, uint64_t* out) override {
    std::lock_guard<std::mutex> g(mu_);
    DevGuard dg(dev_);
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t bytes = total * 8;
    // resident ciphertexts: a body that lies inside a staged variable is read in place
    std::vector<const uint64_t*> dptr(bodies.size(), nullptr);
    std::vector<char*> tmp;
    for (size_t i = 0; i < bodies.size(); ++i) {
      dptr[i] = reinterpret_cast<const uint64_t*>(resident_address(bodies[i], bytes));
      if (dptr[i]) {
        stats_.resident_hits++;
        continue;
      }
      char* d = nullptr;
      hip_check(hipMalloc(reinterpret_cast<void**>(&d), bytes), "hipMalloc");
      hip_check(hipMemcpyAsync(d, bodies[i], bytes, hipMemcpyHostToDevice, compute_), "H2D");
      tmp.push_back(d);
      dptr[i] = reinterpret_cast<const uint64_t*>(d);
      stats_.cold_uploads++;
    }
    std::vector<uint64_t> tab(wq.size() * 2);
    for (size_t i = 0; i < wq.size(); ++i) {
      tab[2 * i] = wq[i];
      tab[2 * i + 1] = wqs[i];
    }
    char* aux = nullptr;
    const size_t aux_bytes = tab.size() * 8 + q.size() * 8;
    hip_check(hipMalloc(reinterpret_cast<void**>(&aux), aux_bytes), "hipMalloc");
    hip_check(hipMemcpyAsync(aux, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, compute_), "H2D");
    hip_check(hipMemcpyAsync(aux + tab.size() * 8, q.data(), q.size() * 8, hipMemcpyHostToDevice,
                             compute_),
              "H2D");
    uint64_t* o = reinterpret_cast<uint64_t*>(scratch(bytes));
    hip_check(hipEventRecord(k0_, compute_), "event");
    for (size_t b = 0; b < dptr.size(); b += kMaxModels) {
      PwaArgs a{};
      a.count = (int)std::min<size_t>(kMaxModels, dptr.size() - b);
      a.first = (int)b;
      for (int k = 0; k < a.count; ++k) a.ct[k] = dptr[b + k];
      hip_check((hipError_t)launch_pwa(a, reinterpret_cast<const uint64_t*>(aux),
                                       reinterpret_cast<const uint64_t*>(aux + tab.size() * 8), o, L,
                                       N, total, b > 0, compute_),
                "pwa launch");
    }
    hip_check(hipEventRecord(k1_, compute_), "event");
    hip_check(hipMemcpyAsync(out, o, bytes, hipMemcpyDeviceToHost, compute_), "D2H");
    hip_check(hipStreamSynchronize(compute_), "sync");
    for (auto* d : tmp) hipFree(d);
    hipFree(aux);
    float kms = 0;
    hipEventElapsedTime(&kms, k0_, k1_);
    stats_.last_kernel_ms = kms;
    stats_.pwa_calls++;
    stats_.last_total_ms = ms_since(t0);
    return true;
  }

  DeviceAggStats stats() const override {
    std::lock_guard<std::mutex> g(mu_);
    DeviceAggStats s = stats_;
    s.resident_bytes = resident_bytes_;
    return s;
  }

 private:
  static constexpr uint64_t kChunk = 8ull << 20;  // small enough to pipeline copy-out with D2H
  struct Ring {
    char* host = nullptr;
    hipEvent_t done = nullptr;
  };

  using SlotList = std::list<std::unique_ptr<Slot>>;

  SlotList::iterator release(SlotList::iterator it) {
    Slot* s = it->get();
    if (s->ready) {
      hipEventSynchronize(s->ready);
      hipEventDestroy(s->ready);
    }
    if (s->dev) {
      hipFree(s->dev);
      resident_bytes_ -= s->lay.total;
    }
    return slots_.erase(it);
  }

  void release_ptr(Slot* s) {
    for (auto it = slots_.begin(); it != slots_.end(); ++it)
      if (it->get() == s) {
        release(it);
        return;
      }
  }

  // Pieces of the packed image of `m` that intersect [a, b).
  static std::vector<Piece> pieces_in(const ModelT& m, const Layout& L, uint64_t a, uint64_t b) {
    std::vector<Piece> ps;
    constexpr uint64_t kGrain = 1ull << 20;
    for (size_t v = 0; v < L.off.size(); ++v) {
      const uint64_t lo = std::max(a, L.off[v]), hi = std::min(b, L.off[v] + L.bytes[v]);
      for (uint64_t p = lo; p < hi; p += kGrain) {
        const uint64_t n = std::min(kGrain, hi - p);
        ps.push_back({m.vars[v].t.value.data() + (p - L.off[v]),
                      const_cast<char*>(m.vars[v].t.value.data()) + (p - L.off[v]), p, n});
      }
    }
    return ps;
  }

  // Uploads `m` into a new slot (nullptr when it does not fit the budget).
  Slot* upload(const ModelT& m, const std::string& learner) {
    const auto t0 = std::chrono::steady_clock::now();
    auto s = std::make_unique<Slot>();
    s->learner = learner;
    s->uid = m.uid;
    s->lay = make_layout(m);
    for (auto& v : m.vars) {
      s->ptrs.push_back(v.t.value.data());
      s->sizes.push_back(v.t.value.size());
    }
    while (resident_bytes_ + s->lay.total > budget_) {
      auto oldest = slots_.end();
      for (auto it = slots_.begin(); it != slots_.end(); ++it)
        if (!(*it)->pins && (oldest == slots_.end() || (*it)->stamp < (*oldest)->stamp)) oldest = it;
      if (oldest == slots_.end()) break;
      release(oldest);
    }
    if (resident_bytes_ + s->lay.total > budget_) return nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&s->dev), s->lay.total) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    resident_bytes_ += s->lay.total;
    for (uint64_t a = 0; a < s->lay.total; a += kChunk) {
      Ring& r = ring_[ring_next_++ % kRing];
      hip_check(hipEventSynchronize(r.done), "event sync");
      const uint64_t b = std::min(s->lay.total, a + kChunk);
      const auto ps = pieces_in(m, s->lay, a, b);
#pragma omp parallel for schedule(dynamic, 1)
      for (size_t i = 0; i < ps.size(); ++i) std::memcpy(r.host + (ps[i].packed_off - a), ps[i].src, ps[i].n);
      hip_check(hipMemcpyAsync(s->dev + a, r.host, b - a, hipMemcpyHostToDevice, upload_), "H2D");
      hip_check(hipEventRecord(r.done, upload_), "event");
    }
    hip_check(hipEventCreateWithFlags(&s->ready, hipEventDisableTiming), "event");
    hip_check(hipEventRecord(s->ready, upload_), "event");
    s->stamp = ++clock_;
    stats_.last_upload_ms = ms_since(t0);
    slots_.push_back(std::move(s));
    return slots_.back().get();
  }

  Slot* find(const ModelT& m) {
    for (auto& s : slots_)
      if (s->matches(m)) return s.get();
    return nullptr;
  }

  // Device image of every model (resident or uploaded now into `cold`
  // slots), with the compute stream ordered after the uploads.
  bool resolve(const std::vector<const ModelT*>& models, const Layout& lay, std::vector<Slot*>& in,
               std::vector<Slot*>& cold) {
    for (auto* m : models) {
      Slot* s = find(*m);
      if (s) {
        if (!same_layout(s->lay, lay)) throw std::runtime_error("models have mismatching structure");
        stats_.resident_hits++;
        s->stamp = ++clock_;
      } else {
        const Layout ml = make_layout(*m);
        if (!same_layout(ml, lay)) throw std::runtime_error("models have mismatching structure");
        s = upload(*m, "#cold");
        if (!s) {
          finish(in, cold);
          return false;
        }
        cold.push_back(s);
        stats_.cold_uploads++;
      }
      hip_check(hipStreamWaitEvent(compute_, s->ready, 0), "wait");
      s->pins++;
      in.push_back(s);
    }
    return true;
  }

  // Unpins the inputs of an aggregation and frees its cold uploads (after the
  // compute stream has consumed them).
  void finish(std::vector<Slot*>& in, std::vector<Slot*>& cold) {
    for (auto* s : in) s->pins--;
    if (!cold.empty()) hip_check(hipStreamSynchronize(compute_), "sync");
    for (auto* c : cold) release_ptr(c);
    in.clear();
    cold.clear();
  }

  const char* resident_address(const void* host, uint64_t bytes) {
    const char* p = static_cast<const char*>(host);
    for (auto& s : slots_)
      for (size_t v = 0; v < s->ptrs.size(); ++v)
        if (p >= s->ptrs[v] && p + bytes <= s->ptrs[v] + s->sizes[v]) {
          hip_check(hipStreamWaitEvent(compute_, s->ready, 0), "wait");
          s->stamp = ++clock_;
          return s->dev + s->lay.off[v] + (p - s->ptrs[v]);
        }
    return nullptr;
  }

  char* scratch(uint64_t bytes) {
    if (bytes > scratch_cap_) {
      if (scratch_) {
        hipStreamSynchronize(compute_);
        hipFree(scratch_);
      }
      hip_check(hipMalloc(reinterpret_cast<void**>(&scratch_), bytes), "hipMalloc");
      scratch_cap_ = bytes;
    }
    return scratch_;
  }

  void upload_tiles(const Layout& lay) {
    // the tile table of the previous call is reused when the layout repeats
    // (every op of a round, every rolling merge)
    if (tiles_dev_ && lay.bytes == tiles_bytes_ && lay.dtype == tiles_dtype_) return;
    tiles_bytes_ = lay.bytes;
    tiles_dtype_ = lay.dtype;
    std::vector<Tile> t = make_tiles(lay);
    ntiles_ = (int)t.size();
    const size_t b = std::max<size_t>(1, t.size()) * sizeof(Tile);
    if (b > tiles_cap_) {
      if (tiles_dev_) {
        hipStreamSynchronize(compute_);
        hipFree(tiles_dev_);
      }
      hip_check(hipMalloc(reinterpret_cast<void**>(&tiles_dev_), b), "hipMalloc");
      tiles_cap_ = b;
    }
    if (!t.empty())
      hip_check(hipMemcpyAsync(tiles_dev_, t.data(), t.size() * sizeof(Tile), hipMemcpyHostToDevice,
                               compute_),
                "H2D");
    hip_check(hipStreamSynchronize(compute_), "sync");  // `t` is pageable and dies here
  }

  void roll_(char* y, const char* x, double w, int op) {
    hip_check((hipError_t)launch_roll(y, x, tiles_dev_, ntiles_, w, op, compute_), "roll launch");
  }

  // out = layout of `meta` with the values of device buffer `src`.
  void download(ModelT& out, const ModelT& meta, const Layout& lay, const char* src) {
    const auto t0 = std::chrono::steady_clock::now();
    out.vars.resize(meta.vars.size());
#pragma omp parallel for schedule(dynamic, 1)
    for (size_t v = 0; v < meta.vars.size(); ++v) {
      auto& ov = out.vars[v];
      const auto& sv = meta.vars[v];
      ov.name = sv.name;
      ov.trainable = sv.trainable;
      ov.ciphertext = false;
      ov.t.length = sv.t.length;
      ov.t.dims = sv.t.dims;
      ov.t.dtype = sv.t.dtype;
      ov.t.byte_order = sv.t.byte_order;
      ov.t.fortran_order = sv.t.fortran_order;
      ov.t.value.resize(lay.bytes[v]);
    }
    const uint64_t n = lay.total;
    std::vector<std::pair<uint64_t, uint64_t>> chunks;
    for (uint64_t a = 0; a < n; a += kChunk) chunks.push_back({a, std::min(n, a + kChunk)});
    auto issue = [&](size_t c) {
      Ring& r = ring_[c % kRing];
      hip_check(hipEventSynchronize(r.done), "event sync");
      hip_check(hipMemcpyAsync(r.host, src + chunks[c].first, chunks[c].second - chunks[c].first,
                               hipMemcpyDeviceToHost, compute_),
                "D2H");
      hip_check(hipEventRecord(r.done, compute_), "event");
    };
    for (size_t c = 0; c < std::min<size_t>(kRing, chunks.size()); ++c) issue(c);
    for (size_t c = 0; c < chunks.size(); ++c) {
      Ring& r = ring_[c % kRing];
      hip_check(hipEventSynchronize(r.done), "event sync");
      const auto ps = pieces_in(out, lay, chunks[c].first, chunks[c].second);
#pragma omp parallel for schedule(dynamic, 1)
      for (size_t i = 0; i < ps.size(); ++i)
        std::memcpy(ps[i].dst_host, r.host + (ps[i].packed_off - chunks[c].first), ps[i].n);
      if (c + kRing < chunks.size()) issue(c + kRing);
    }
    ring_next_ = 0;
    stats_.last_download_ms = ms_since(t0);
  }

  static constexpr int kRing = 4;
  mutable std::mutex mu_;
  int dev_;
  hipStream_t upload_ = nullptr, compute_ = nullptr;
  Ring ring_[kRing];
  size_t ring_next_ = 0;
  hipEvent_t k0_ = nullptr, k1_ = nullptr;
  SlotList slots_;
  uint64_t clock_ = 0, resident_bytes_ = 0, budget_ = 0;
  char* scratch_ = nullptr;
  uint64_t scratch_cap_ = 0;
  Tile* tiles_dev_ = nullptr;
  std::vector<uint64_t> tiles_bytes_;
  std::vector<int> tiles_dtype_;
  size_t tiles_cap_ = 0;
  int ntiles_ = 0;
  struct Roll {
    char* dev = nullptr;
    Layout lay;
    ModelT meta;  // names / dtypes / dims, empty values
  };
  Roll& roll_at(int h) {
    auto it = rolls_.find(h);
    if (it == rolls_.end()) throw std::runtime_error("device aggregation: unknown rolling state");
    return it->second;
  }
  std::unordered_map<int, Roll> rolls_;
  int next_roll_ = 0;
  DeviceAggStats stats_;
};

std::once_flag g_once;
std::atomic<DeviceAggregator*> g_dev{nullptr};

}  // namespace

DeviceAggregator* DeviceAggregator::get() {
  std::call_once(g_once, [] {
    const char* mode = std::getenv("METISFL_AMD_DEVICE_AGG");
    const std::string m = mode ? mode : "auto";
    if (m == "0" || m == "off") return;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
      (void)hipGetLastError();
      if (m == "1" || m == "on")
        throw std::runtime_error("METISFL_AMD_DEVICE_AGG=1 but no HIP device is visible");
      return;
    }
    int dev = 0;
    if (const char* d = std::getenv("METISFL_AMD_DEVICE_AGG_DEVICE")) dev = std::atoi(d);
    g_dev = new Impl(std::min(dev, n - 1));  // intentionally leaked (see ~Impl)
  });
  return g_dev;
}

DeviceAggregator* DeviceAggregator::peek() { return g_dev; }

std::atomic<bool> g_on{true};

std::atomic<long long> g_min_bytes{-1};

void DeviceAggregator::set_enabled(bool on, long long min_bytes) {
  g_on = on;
  if (min_bytes >= 0) g_min_bytes = min_bytes;
}

bool DeviceAggregator::enabled_for(size_t model_bytes) {
  if (!g_on) return false;
  if (g_min_bytes < 0) {
    const char* e = std::getenv("METISFL_AMD_DEVICE_AGG_MIN_BYTES");
    g_min_bytes = e ? std::atoll(e) : (1ll << 20);
  }
  return (long long)model_bytes >= g_min_bytes && get() != nullptr;
}

}  // namespace mfl
