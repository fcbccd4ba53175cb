// Controller checkpoint / resume.  The reference keeps all
// controller state in memory (controller.cc:1006-1047): a restarted
// controller loses the federation.  Here the state machine serialises to one
// self-describing blob -- learners (ids, tokens, join requests), task
// templates, local task lineages, the community model and its lineage, the
// runtime-metadata and evaluation lineages, the round counter -- and a new
// controller restores it, then re-dispatches the current round to every
// learner (the learners keep their credentials on disk and rejoin through
// ALREADY_EXISTS, learner.py:96-103 semantics).  The model store (local model
// lineages, an aggregation cache) and the synchronous barrier of the round
// in flight are not persisted: that round restarts.
#include <cstring>

#include "engine/controller.h"

namespace mfl {
namespace {

constexpr char kMagic[8] = {'M', 'F', 'L', 'C', 'K', 'P', 'T', '1'};

struct Out {
  std::string b;
  void raw(const void* p, size_t n) { b.append(static_cast<const char*>(p), n); }
  void u32(uint32_t v) { raw(&v, 4); }
  void i64(int64_t v) { raw(&v, 8); }
  void f64(double v) { raw(&v, 8); }
  void f32(float v) { raw(&v, 4); }
  void str(const std::string& s) {
    u32((uint32_t)s.size());
    raw(s.data(), s.size());
  }
  void strs(const std::vector<std::string>& v) {
    u32((uint32_t)v.size());
    for (auto& s : v) str(s);
  }
  template <typename T>
  void smap(const std::map<std::string, T>& m) {
    u32((uint32_t)m.size());
    for (auto& kv : m) {
      str(kv.first);
      if constexpr (std::is_same_v<T, int64_t>) i64(kv.second);
      else if constexpr (std::is_same_v<T, double>) f64(kv.second);
      else if constexpr (std::is_same_v<T, uint32_t>) u32(kv.second);
      else str(kv.second);
    }
  }
  void f64s(const std::vector<double>& v) {
    u32((uint32_t)v.size());
    for (double x : v) f64(x);
  }
};

struct In {
  std::string_view b;
  size_t p = 0;
  void raw(void* d, size_t n) {
    if (p + n > b.size()) throw StatusError(INVALID_ARGUMENT, "truncated controller checkpoint");
    std::memcpy(d, b.data() + p, n);
    p += n;
  }
  uint32_t u32() { uint32_t v; raw(&v, 4); return v; }
  int64_t i64() { int64_t v; raw(&v, 8); return v; }
  double f64() { double v; raw(&v, 8); return v; }
  float f32() { float v; raw(&v, 4); return v; }
  std::string str() {
    const uint32_t n = u32();
    if (p + n > b.size()) throw StatusError(INVALID_ARGUMENT, "truncated controller checkpoint");
    std::string s(b.data() + p, n);
    p += n;
    return s;
  }
  std::vector<std::string> strs() {
    std::vector<std::string> v(u32());
    for (auto& s : v) s = str();
    return v;
  }
  template <typename T>
  std::map<std::string, T> smap() {
    std::map<std::string, T> m;
    const uint32_t n = u32();
    for (uint32_t i = 0; i < n; ++i) {
      std::string k = str();
      if constexpr (std::is_same_v<T, int64_t>) m[k] = i64();
      else if constexpr (std::is_same_v<T, double>) m[k] = f64();
      else if constexpr (std::is_same_v<T, uint32_t>) m[k] = u32();
      else m[k] = str();
    }
    return m;
  }
  std::vector<double> f64s() {
    std::vector<double> v(u32());
    for (auto& x : v) x = f64();
    return v;
  }
};

}  // namespace

std::string Controller::checkpoint() const {
  std::lock_guard<std::mutex> g(mu_);
  Out o;
  o.raw(kMagic, 8);
  o.u32(global_iteration_);
  o.u32(evicted_);
  o.u32((uint32_t)learners_.size());
  for (auto& kv : learners_) {
    const LearnerRec& l = kv.second;
    o.str(l.id); o.str(l.token); o.str(l.server_entity); o.str(l.dataset_spec);
    o.str(l.hostname); o.u32(l.port); o.f64(l.num_train);
  }
  o.smap(templates_);
  o.u32((uint32_t)local_meta_.size());
  for (auto& kv : local_meta_) {
    o.str(kv.first);
    o.u32((uint32_t)kv.second.size());
    for (const TaskMeta& t : kv.second) {
      o.str(t.raw); o.u32(t.global_iteration); o.u32(t.completed_batches); o.u32(t.batch_size);
      o.f32(t.completed_epochs); o.f32(t.ms_per_epoch); o.f32(t.ms_per_batch);
    }
  }
  o.u32(community_set_ ? 1 : 0);
  o.str(community_set_ ? serialize_federated_model(community_) : std::string());
  o.strs(std::vector<std::string>(community_lineage_.begin(), community_lineage_.end()));
  o.u32((uint32_t)metadata_.size());
  for (const RoundMeta& m : metadata_) {
    o.u32(m.global_iteration); o.i64(m.started_at); o.i64(m.completed_at);
    o.strs(m.assigned); o.strs(m.completed_by);
    o.smap(m.train_submitted); o.smap(m.train_received); o.smap(m.eval_submitted); o.smap(m.eval_received);
    o.smap(m.insertion_ms); o.smap(m.selection_ms);
    o.i64(m.agg_started); o.i64(m.agg_completed); o.f64(m.agg_total_ms);
    o.f64s(m.block_size); o.f64s(m.block_mem_kb); o.f64s(m.block_ms);
    o.u32((uint32_t)m.quantifiers.size());
    for (const Quantifier& q : m.quantifiers) {
      o.i64((int64_t)q.non_zeros); o.i64((int64_t)q.zeros); o.i64((int64_t)q.size_bytes);
    }
  }
  o.u32((uint32_t)evaluations_.size());
  for (const CommEval& e : evaluations_) {
    o.u32(e.global_iteration);
    o.smap(e.evals);
  }
  return o.b;
}

void Controller::restore(const std::string& blob) {
  In in{blob};
  char magic[8];
  in.raw(magic, 8);
  if (std::memcmp(magic, kMagic, 8) != 0) throw StatusError(INVALID_ARGUMENT, "not a controller checkpoint");
  std::lock_guard<std::mutex> g(mu_);
  global_iteration_ = in.u32();
  evicted_ = in.u32();
  learners_.clear();
  for (uint32_t n = in.u32(), i = 0; i < n; ++i) {
    LearnerRec l;
    l.id = in.str(); l.token = in.str(); l.server_entity = in.str(); l.dataset_spec = in.str();
    l.hostname = in.str(); l.port = in.u32(); l.num_train = in.f64();
    learners_[l.id] = l;
  }
  templates_ = in.smap<uint32_t>();
  local_meta_.clear();
  for (uint32_t n = in.u32(), i = 0; i < n; ++i) {
    std::string id = in.str();
    auto& dq = local_meta_[id];
    for (uint32_t k = in.u32(), j = 0; j < k; ++j) {
      TaskMeta t;
      t.raw = in.str(); t.global_iteration = in.u32(); t.completed_batches = in.u32(); t.batch_size = in.u32();
      t.completed_epochs = in.f32(); t.ms_per_epoch = in.f32(); t.ms_per_batch = in.f32();
      dq.push_back(t);
    }
  }
  completed_iter_.clear();
  for (const auto& [id, dq] : local_meta_)
    if (learners_.count(id) && !dq.empty()) completed_iter_[id] = dq.front().global_iteration;
  community_set_ = in.u32() != 0;
  const std::string cm = in.str();
  if (community_set_) community_ = parse_federated_model(cm);
  const auto lin = in.strs();
  community_lineage_.assign(lin.begin(), lin.end());
  metadata_.clear();
  for (uint32_t n = in.u32(), i = 0; i < n; ++i) {
    RoundMeta m;
    m.global_iteration = in.u32(); m.started_at = in.i64(); m.completed_at = in.i64();
    m.assigned = in.strs(); m.completed_by = in.strs();
    m.train_submitted = in.smap<int64_t>(); m.train_received = in.smap<int64_t>();
    m.eval_submitted = in.smap<int64_t>(); m.eval_received = in.smap<int64_t>();
    m.insertion_ms = in.smap<double>(); m.selection_ms = in.smap<double>();
    m.agg_started = in.i64(); m.agg_completed = in.i64(); m.agg_total_ms = in.f64();
    m.block_size = in.f64s(); m.block_mem_kb = in.f64s(); m.block_ms = in.f64s();
    for (uint32_t k = in.u32(), j = 0; j < k; ++j) {
      Quantifier q;
      q.non_zeros = (uint64_t)in.i64(); q.zeros = (uint64_t)in.i64(); q.size_bytes = (uint64_t)in.i64();
      m.quantifiers.push_back(q);
    }
    metadata_.push_back(std::move(m));
  }
  evaluations_.clear();
  for (uint32_t n = in.u32(), i = 0; i < n; ++i) {
    CommEval e;
    e.global_iteration = in.u32();
    e.evals = in.smap<std::string>();
    evaluations_.push_back(std::move(e));
  }
}

Dispatch Controller::resume_dispatch() {
  std::lock_guard<std::mutex> g(mu_);
  Dispatch d;
  if (!community_set_) return d;
  const std::string fm = serialize_federated_model(community_);
  std::map<uint32_t, Payload> cache;
  for (auto& kv : learners_)
    d.run_tasks.emplace_back(kv.first, make_run_task(kv.first, fm, global_iteration_, cache));
  return d;
}

}  // namespace mfl
