#include "engine/controller.h"

#include "engine/device_agg.h"

#include <sys/resource.h>

#include <chrono>
#include <cmath>
#include <sstream>

#include "common/wire.h"

namespace mfl {

using wire::WireMsg;
using wire::Writer;

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::system_clock::now().time_since_epoch())
      .count();
}

long total_memory_kb() {
  rusage u{};
  getrusage(RUSAGE_SELF, &u);
  return u.ru_maxrss;
}

// ---------------------------------------------------------------------------
ControllerConfig ControllerConfig::from_params(std::string_view bytes) {
  ControllerConfig c;
  WireMsg p(bytes);
  if (p.has(1)) {
    WireMsg se = p.msg(1);
    c.hostname = se.str(1);
    c.port = (uint32_t)se.u64(2);
  }
  WireMsg gms = p.msg(2);
  WireMsg rule = gms.msg(1);
  if (rule.has(2)) {
    c.rule = 2;
    c.stride_length = (uint32_t)rule.msg(2).u64(1);
  } else if (rule.has(3)) {
    c.rule = 3;
  } else if (rule.has(4)) {
    c.rule = 4;
    WireMsg he = rule.msg(4).msg(1);
    c.he_ctx_file = he.str(2);
    if (he.has(6)) {
      WireMsg ck = he.msg(6);
      c.he_batch_size = (uint32_t)ck.u64(1, 4096);
      c.he_scaling_bits = (uint32_t)ck.u64(2, 52);
    }
  } else {
    c.rule = 1;
  }
  c.scaling = (int)rule.msg(5).u64(1, SCALE_EXAMPLES);
  if (c.scaling == SCALE_UNKNOWN) c.scaling = SCALE_EXAMPLES;
  c.participation_ratio = gms.f32(2, 1.f);
  WireMsg cs = p.msg(3);
  c.protocol = (int)cs.u64(1, PROTO_SYNC);
  if (c.protocol == PROTO_UNKNOWN) c.protocol = PROTO_SYNC;
  WireMsg ps = cs.msg(2);
  c.semi_sync_lambda = (int)(int32_t)ps.u64(1);
  c.semi_sync_recompute = ps.b(2);
  WireMsg msc = p.msg(4);
  WireMsg specs;
  if (msc.has(2)) {
    c.redis = true;
    WireMsg r = msc.msg(2);
    specs = r.msg(1);
    WireMsg se = r.msg(2);
    if (se.has(1)) c.redis_host = se.str(1);
    if (se.has(2)) c.redis_port = (uint32_t)se.u64(2);
  } else {
    specs = msc.msg(1).msg(1);
  }
  if (specs.has(2)) {
    c.lineage = (int)specs.msg(2).u64(1);
    if (c.lineage == 0) c.lineage = 1;
  } else if (specs.has(1)) {
    c.lineage = -1;
  } else {
    c.lineage = c.rule == 3 ? 2 : 1;
  }
  WireMsg mh = p.msg(5);
  c.batch_size = (uint32_t)mh.u64(1, 100);
  c.epochs = (uint32_t)mh.u64(2, 5);
  c.optimizer_bytes = mh.str(3);
  c.percent_validation = mh.f32(4);
  return c;
}

// ---------------------------------------------------------------------------
std::string RoundMeta::serialize() const {
  Writer w;
  w.u64(1, global_iteration);
  w.timestamp(2, started_at);
  w.timestamp(3, completed_at);
  for (auto& s : assigned) w.bytes(4, s, true);
  for (auto& s : completed_by) w.bytes(5, s, true);
  for (auto& [k, v] : train_submitted) w.map_str_ts(6, k, v);
  for (auto& [k, v] : train_received) w.map_str_ts(7, k, v);
  for (auto& [k, v] : eval_submitted) w.map_str_ts(8, k, v);
  for (auto& [k, v] : eval_received) w.map_str_ts(9, k, v);
  for (auto& [k, v] : insertion_ms) w.map_str_f64(10, k, v);
  for (auto& [k, v] : selection_ms) w.map_str_f64(11, k, v);
  w.timestamp(12, agg_started);
  w.timestamp(13, agg_completed);
  w.f64(14, agg_total_ms);
  w.packed_f64(15, block_size);
  w.packed_f64(16, block_mem_kb);
  w.packed_f64(17, block_ms);
  for (auto& q : quantifiers) {
    Writer t;
    t.u64(1, q.non_zeros, true);
    t.u64(2, q.zeros, true);
    t.u64(3, q.size_bytes);
    w.msg(18, t);
  }
  return w.take();
}

// ---------------------------------------------------------------------------
Controller::Controller(const std::string& params_bytes)
    : cfg_(ControllerConfig::from_params(params_bytes)) {
  if (cfg_.batch_size == 0) throw StatusError(INVALID_ARGUMENT, "batch size cannot be zero");
  if (cfg_.epochs == 0) throw StatusError(INVALID_ARGUMENT, "epochs cannot be zero");
  if (cfg_.protocol == PROTO_ASYNC)
    scheduler_.reset(new AsynchronousScheduler());
  else
    scheduler_.reset(new SynchronousScheduler());
  switch (cfg_.rule) {
    case 2: aggregator_.reset(new FederatedStride()); break;
    case 3: aggregator_.reset(new FederatedRecency()); break;
    case 4:
      aggregator_.reset(new PrivateWeightedAverage(cfg_.he_batch_size, cfg_.he_scaling_bits,
                                                   cfg_.he_ctx_file));
      break;
    default: aggregator_.reset(new FederatedAverage()); break;
  }
  if (cfg_.redis)
    store_.reset(new RedisModelStore(cfg_.lineage, cfg_.redis_host, (int)cfg_.redis_port));
  else
    store_.reset(new HashMapModelStore(cfg_.lineage));
}

// 128 bits from the ChaCha20 stream (keyed with 256 bits of getrandom): an
// observer of other tokens learns nothing about the next one (a 32-bit seeded
// mt19937 could be brute-forced from one token)
std::string Controller::random_token() {
  static const char* hex = "0123456789abcdef";
  std::string t(32, '0');
  for (int w = 0; w < 2; ++w) {
    uint64_t v = rng_.next_u64();
    for (int i = 0; i < 16; ++i, v >>= 4) t[16 * w + i] = hex[v & 15];
  }
  return t;
}

std::vector<std::string> Controller::active_ids_locked() const {
  std::vector<std::string> ids;
  for (auto& [k, _] : learners_) ids.push_back(k);
  return ids;
}

std::vector<std::string> Controller::learner_ids() const {
  std::lock_guard<std::mutex> g(mu_);
  return active_ids_locked();
}

size_t Controller::num_learners() const {
  std::lock_guard<std::mutex> g(mu_);
  return learners_.size();
}

uint32_t Controller::global_iteration() const {
  std::lock_guard<std::mutex> g(mu_);
  return global_iteration_;
}

void Controller::validate(const std::string& id, const std::string& token) const {
  auto it = learners_.find(id);
  if (it == learners_.end()) throw StatusError(NOT_FOUND, "Learner is not part of the federation.");
  if (it->second.token != token) throw StatusError(UNAUTHENTICATED, "Learner token is wrong.");
}

// ---------------------------------------------------------------------------
std::pair<std::string, std::string> Controller::add_learner(const std::string& server_entity,
                                                            const std::string& dataset_spec,
                                                            Dispatch* dispatch) {
  std::lock_guard<std::mutex> g(mu_);
  WireMsg se(server_entity);
  WireMsg ds(dataset_spec);
  const std::string host = se.str(1);
  const uint32_t port = (uint32_t)se.u64(2);
  if (host.empty()) throw StatusError(INVALID_ARGUMENT, "Hostname and port must be provided.");
  const double ntrain = (double)ds.u64(1);
  if (ntrain <= 0) throw StatusError(INVALID_ARGUMENT, "Learner training examples <= 0.");
  const std::string id = host + ":" + std::to_string(port);
  if (learners_.count(id)) throw StatusError(ALREADY_EXISTS, "Learner has already joined.");
  LearnerRec rec;
  rec.id = id;
  rec.token = random_token();
  rec.server_entity = server_entity;
  rec.dataset_spec = dataset_spec;
  rec.hostname = host;
  rec.port = port;
  rec.num_train = ntrain;
  learners_[id] = rec;
  // num_local_updates = epochs * ceil(N_train / batch)  (controller.cc:148-153)
  const uint32_t spe = (uint32_t)std::ceil(ntrain / (double)cfg_.batch_size);
  templates_[id] = cfg_.epochs * spe;
  if (dispatch) schedule_initial_task_locked(id, dispatch);
  return {id, rec.token};
}

Dispatch Controller::remove_learner(const std::string& id, const std::string& token) {
  std::lock_guard<std::mutex> g(mu_);
  validate(id, token);
  store_->erase({id});
  if (auto* d = DeviceAggregator::peek()) d->drop(id);
  learners_.erase(id);
  templates_.erase(id);
  completed_iter_.erase(id);
  const auto active = active_ids_locked();
  auto ready = scheduler_->poll(active);
  if (ready.empty()) return Dispatch{};
  return run_scheduled_locked(ready, active, global_iteration_);
}

void Controller::replace_community_model(const std::string& federated_model) {
  std::lock_guard<std::mutex> g(mu_);
  community_ = parse_federated_model(federated_model);
  community_set_ = true;
  community_lineage_.push_front(federated_model);
  while (community_lineage_.size() > cfg_.community_lineage) community_lineage_.pop_back();
}

std::string Controller::community_model() const {
  std::lock_guard<std::mutex> g(mu_);
  return serialize_federated_model(community_);
}

// ---------------------------------------------------------------------------
Payload Controller::make_run_task(const std::string& id, const std::string& fm_bytes,
                                  uint32_t global_iteration, std::map<uint32_t, Payload>& cache) const {
  auto it = templates_.find(id);
  const uint32_t steps = it == templates_.end() ? 0 : it->second;
  auto hit = cache.find(steps);
  if (hit != cache.end()) return hit->second;
  Writer task;
  task.u64(1, global_iteration);
  task.u64(2, steps);
  task.f32(3, cfg_.percent_validation);
  Writer hp;
  hp.u64(1, cfg_.batch_size);
  if (!cfg_.optimizer_bytes.empty()) hp.bytes(2, cfg_.optimizer_bytes, true);
  Writer req;
  req.bytes(1, fm_bytes, true);
  req.msg(2, task);
  req.msg(3, hp);
  auto p = std::make_shared<const std::string>(req.take());
  cache.emplace(steps, p);
  return p;
}

std::string Controller::make_eval_task(const FederatedModelT& model) const {
  Writer req;
  req.bytes(1, serialize_model(model.model), true);
  req.u64(2, cfg_.batch_size);
  Writer ds;  // packed repeated enum: TRAINING(0), VALIDATION(2), TEST(1)
  ds.varint_raw(0);
  ds.varint_raw(2);
  ds.varint_raw(1);
  req.bytes(3, ds.str(), true);
  return req.take();
}

void Controller::schedule_initial_task_locked(const std::string& id, Dispatch* d) {
  if (!community_set_) return;
  if (metadata_.empty()) {
    RoundMeta m;
    m.global_iteration = ++global_iteration_;
    m.started_at = now_ns();
    metadata_.push_back(m);
  }
  auto& meta = metadata_.back();
  meta.assigned.push_back(id);
  std::map<uint32_t, Payload> cache;
  d->run_tasks.emplace_back(
      id, make_run_task(id, serialize_federated_model(community_), meta.global_iteration, cache));
  meta.train_submitted[id] = now_ns();
}

void Controller::record_train_submitted(const std::string& id, uint32_t metadata_index) {
  std::lock_guard<std::mutex> g(mu_);
  if (metadata_index < metadata_.size()) metadata_[metadata_index].train_submitted[id] = now_ns();
}

Dispatch Controller::learner_completed_task(const std::string& id, const std::string& token,
                                            const std::string& completed_task) {
  std::lock_guard<std::mutex> g(mu_);
  validate(id, token);
  WireMsg task(completed_task);
  WireMsg em = task.msg(2);
  TaskMeta tm;
  tm.raw = std::string(task.bytes(2));
  tm.global_iteration = (uint32_t)em.u64(1);
  tm.completed_epochs = em.f32(3);
  tm.completed_batches = (uint32_t)em.u64(4);
  tm.batch_size = (uint32_t)em.u64(5);
  tm.ms_per_epoch = em.f32(6);
  tm.ms_per_batch = em.f32(7);
  const uint32_t idx = tm.global_iteration == 0 ? 0 : tm.global_iteration - 1;
  const int64_t t0 = now_ns();
  // A duplicate completion (a client retry whose first reply was lost) of a
  // task already recorded is acknowledged and ignored: (learner, global
  // iteration) identifies a task under every protocol -- within one
  // membership of the learner (completed_iter_ is cleared when it leaves).
  auto lc = completed_iter_.find(id);
  if (lc != completed_iter_.end() && tm.global_iteration != 0 && lc->second == tm.global_iteration)
    return Dispatch{};
  if (!metadata_.empty() && idx < metadata_.size()) {
    metadata_[idx].completed_by.push_back(id);
    metadata_[idx].train_received[id] = t0;
  }
  ModelT m = parse_model(task.bytes(1));
  // Device residency: upload now, while the other learners are still
  // training, so the round's aggregation reads HBM only (engine/device_agg.h).
  // The in-memory store keeps `m`'s buffers alive at the same addresses
  // (vector move); the Redis store re-parses on select, so it is not staged.
  if (store_->name() == "InMemoryStore" && DeviceAggregator::enabled_for(m.byte_size()))
    DeviceAggregator::get()->stage(id, m, cfg_.lineage);
  store_->insert(id, std::move(m));
  if (!metadata_.empty() && idx < metadata_.size())
    metadata_[idx].insertion_ms[id] = (double)(now_ns() - t0) / 1e6;
  local_meta_[id].push_front(tm);
  completed_iter_[id] = tm.global_iteration;
  return schedule_tasks_locked(id, tm.global_iteration);
}

Dispatch Controller::schedule_tasks_locked(const std::string& id, uint32_t task_iteration) {
  const auto active = active_ids_locked();
  auto to_schedule = scheduler_->schedule_next(id, active);
  if (to_schedule.empty()) return Dispatch{};
  return run_scheduled_locked(to_schedule, active, task_iteration);
}

// Failure detector hook (no token: the caller is the controller itself).
// Removing a learner that a synchronous barrier was waiting for may complete
// the barrier with the remaining learners -- the reference stalls forever in
// that case; here the round is aggregated right away.
Dispatch Controller::evict_learner(const std::string& id, bool count) {
  std::lock_guard<std::mutex> g(mu_);
  if (!learners_.count(id)) throw StatusError(NOT_FOUND, "learner " + id + " not found");
  store_->erase({id});
  if (auto* d = DeviceAggregator::peek()) d->drop(id);
  learners_.erase(id);
  templates_.erase(id);
  completed_iter_.erase(id);
  if (count) ++evicted_;
  const auto active = active_ids_locked();
  auto ready = scheduler_->poll(active);
  if (ready.empty()) return Dispatch{};
  return run_scheduled_locked(ready, active, global_iteration_);
}

Dispatch Controller::run_scheduled_locked(const std::vector<std::string>& to_schedule,
                                          const std::vector<std::string>& active,
                                          uint32_t task_iteration) {
  Dispatch d;
  const uint32_t idx = task_iteration == 0 ? 0 : task_iteration - 1;
  if (!metadata_.empty() && idx < metadata_.size()) metadata_[idx].completed_at = now_ns();
  // FedRec folds ONE learner's (previous, latest) pair into its running state,
  // so it aggregates the finisher only; the reference hands it every active
  // learner and silently uses whichever comes first (federated_recency.cc:15).
  const auto selected =
      cfg_.rule == 3 ? to_schedule : select_scheduled_cardinality(to_schedule, active);
  FederatedModelT cm = compute_community_model_locked(selected, idx);
  record_quantifiers_locked(cm, idx);
  cm.global_iteration = task_iteration;
  community_ = cm;
  community_set_ = true;
  const std::string cm_bytes = serialize_federated_model(cm);
  community_lineage_.push_front(cm_bytes);
  while (community_lineage_.size() > cfg_.community_lineage) community_lineage_.pop_back();
  CommEval ce;
  ce.global_iteration = task_iteration;
  evaluations_.push_back(ce);
  const uint32_t ce_idx = (uint32_t)evaluations_.size() - 1;
  const Payload eval_req = std::make_shared<const std::string>(make_eval_task(cm));
  for (auto& lid : to_schedule) {
    if (idx < metadata_.size()) metadata_[idx].eval_submitted[lid] = now_ns();
    d.eval_tasks.push_back({lid, eval_req, ce_idx, idx});
  }
  ++global_iteration_;
  update_templates_locked(to_schedule);
  RoundMeta nm;
  nm.global_iteration = global_iteration_;
  nm.started_at = now_ns();
  std::map<uint32_t, Payload> cache;
  for (auto& lid : to_schedule) {
    nm.assigned.push_back(lid);
    d.run_tasks.emplace_back(lid, make_run_task(lid, cm_bytes, global_iteration_, cache));
    nm.train_submitted[lid] = now_ns();
  }
  metadata_.push_back(nm);
  return d;
}

void Controller::update_templates_locked(const std::vector<std::string>& ids) {
  if (cfg_.protocol != PROTO_SEMI_SYNC) return;
  if (!(global_iteration_ == 2 || cfg_.semi_sync_recompute)) return;
  float slowest = 0.f;
  for (auto& id : ids) {
    auto it = local_meta_.find(id);
    if (it == local_meta_.end() || it->second.empty()) continue;
    slowest = std::max(slowest, it->second.front().ms_per_epoch);
  }
  const float t_max = (float)cfg_.semi_sync_lambda * slowest;
  for (auto& id : ids) {
    auto it = local_meta_.find(id);
    if (it == local_meta_.end() || it->second.empty()) continue;
    float mpb = it->second.front().ms_per_batch;
    if (mpb == 0.f) mpb = 1.f;
    templates_[id] = (uint32_t)std::ceil(t_max / mpb);
  }
}

FederatedModelT Controller::compute_community_model_locked(const std::vector<std::string>& ids,
                                                           uint32_t meta_idx) {
  RoundMeta* meta = meta_idx < metadata_.size() ? &metadata_[meta_idx] : nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  if (meta) meta->agg_started = now_ns();
  std::vector<ScalerInput> parts;
  std::vector<std::string> pids;
  for (auto& id : ids) {
    auto it = learners_.find(id);
    if (it == learners_.end()) continue;
    // A learner that has not committed a model yet (e.g. an async federation
    // in its first rounds) cannot contribute: it is excluded before the
    // scaling factors are normalised (the reference would aggregate an empty
    // lineage here, controller.cc:885-903).
    if (store_->lineage_length(id) == 0) continue;
    ScalerInput si;
    si.id = id;
    si.num_training_examples = it->second.num_train;
    auto mt = local_meta_.find(id);
    // Deviation: the reference passes the learner's
    // OLDEST task metadata to the scaler; the newest is used here.
    if (mt != local_meta_.end() && !mt->second.empty())
      si.completed_batches = mt->second.front().completed_batches;
    parts.push_back(si);
    pids.push_back(id);
  }
  auto factors = compute_scaling_factors(cfg_.scaling, learners_.size(), parts);
  uint32_t stride = (uint32_t)pids.size();
  if (cfg_.rule == 2 && cfg_.stride_length > 0) stride = cfg_.stride_length;
  FederatedModelT out;
  std::vector<std::pair<std::string, int>> block;
  for (size_t i = 0; i < pids.size(); ++i) {
    const int have = store_->lineage_length(pids[i]);
    const int need = aggregator_->required_lineage_length();
    block.emplace_back(pids[i], have >= need ? need : have);
    if (block.size() == stride || i + 1 == pids.size()) {
      if (meta) meta->block_size.push_back((double)block.size());
      const auto ts = std::chrono::steady_clock::now();
      auto selected = store_->select(block);
      const double sel_ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts).count();
      AggInput in;
      for (auto& [lid, models] : selected) {
        if (meta) meta->selection_ms[lid] = sel_ms / (double)block.size();
        std::vector<ModelRef> lin;
        for (auto* m : models) lin.push_back({m, factors[lid]});
        in.push_back(std::move(lin));
      }
      const auto ta = std::chrono::steady_clock::now();
      if (!in.empty()) out = aggregator_->aggregate(in);
      if (meta) {
        meta->block_ms.push_back(
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count());
        meta->block_mem_kb.push_back((double)total_memory_kb());
      }
      block.clear();
      store_->reset_state();
    }
  }
  aggregator_->reset();
  if (meta) {
    meta->agg_total_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    meta->agg_completed = now_ns();
  }
  return out;
}

void Controller::record_quantifiers_locked(const FederatedModelT& m, uint32_t meta_idx) {
  if (meta_idx >= metadata_.size()) return;
  auto& q = metadata_[meta_idx].quantifiers;
  q.clear();
  for (auto& v : m.model.vars) q.push_back(quantify(v.t));
}

void Controller::record_evaluation(const std::string& id, uint32_t comm_eval_index,
                                   uint32_t metadata_index, const std::string& model_evaluations) {
  std::lock_guard<std::mutex> g(mu_);
  if (metadata_index < metadata_.size()) metadata_[metadata_index].eval_received[id] = now_ns();
  if (comm_eval_index < evaluations_.size()) evaluations_[comm_eval_index].evals[id] = model_evaluations;
}

// ---------------------------------------------------------------------------
std::map<std::string, double> Controller::scaling_factors(const std::vector<std::string>& ids,
                                                          const std::vector<double>& num_train,
                                                          const std::vector<double>& batches) const {
  std::vector<ScalerInput> parts;
  for (size_t i = 0; i < ids.size(); ++i)
    parts.push_back({ids[i], i < num_train.size() ? num_train[i] : 0.0,
                     i < batches.size() ? batches[i] : 0.0});
  std::lock_guard<std::mutex> g(mu_);
  const size_t n_all = std::max(learners_.size(), ids.size());
  return compute_scaling_factors(cfg_.scaling, n_all, parts);
}

void Controller::record_collective_round(uint32_t global_iteration, const std::vector<std::string>& ids,
                                         int64_t started_ns, int64_t completed_ns,
                                         int64_t agg_started_ns, int64_t agg_completed_ns,
                                         const std::vector<std::string>& task_meta,
                                         const std::vector<uint64_t>& zeros,
                                         const std::vector<uint64_t>& sizes_bytes,
                                         const std::vector<uint64_t>& lengths) {
  std::lock_guard<std::mutex> g(mu_);
  RoundMeta m;
  m.global_iteration = global_iteration;
  m.started_at = started_ns;
  m.completed_at = completed_ns;
  m.agg_started = agg_started_ns;
  m.agg_completed = agg_completed_ns;
  m.agg_total_ms = (double)(agg_completed_ns - agg_started_ns) / 1e6;
  m.block_size.push_back((double)ids.size());
  m.block_ms.push_back(m.agg_total_ms);
  m.block_mem_kb.push_back((double)total_memory_kb());
  for (size_t i = 0; i < ids.size(); ++i) {
    m.assigned.push_back(ids[i]);
    m.completed_by.push_back(ids[i]);
    m.train_submitted[ids[i]] = started_ns;
    m.train_received[ids[i]] = completed_ns;
    if (i < task_meta.size()) {
      TaskMeta tm;
      tm.raw = task_meta[i];
      WireMsg em(tm.raw);
      tm.global_iteration = (uint32_t)em.u64(1);
      tm.completed_epochs = em.f32(3);
      tm.completed_batches = (uint32_t)em.u64(4);
      tm.batch_size = (uint32_t)em.u64(5);
      tm.ms_per_epoch = em.f32(6);
      tm.ms_per_batch = em.f32(7);
      local_meta_[ids[i]].push_front(tm);
    }
  }
  for (size_t v = 0; v < zeros.size(); ++v) {
    Quantifier q;
    q.zeros = zeros[v];
    q.size_bytes = v < sizes_bytes.size() ? sizes_bytes[v] : 0;
    q.non_zeros = v < lengths.size() && lengths[v] >= zeros[v] ? lengths[v] - zeros[v] : 0;
    m.quantifiers.push_back(q);
  }
  metadata_.push_back(m);
  global_iteration_ = std::max(global_iteration_, global_iteration);
}

void Controller::record_community_evaluation(uint32_t global_iteration, const std::vector<std::string>& ids,
                                             const std::vector<std::string>& model_evaluations) {
  std::lock_guard<std::mutex> g(mu_);
  CommEval ce;
  ce.global_iteration = global_iteration;
  for (size_t i = 0; i < ids.size() && i < model_evaluations.size(); ++i) ce.evals[ids[i]] = model_evaluations[i];
  const int64_t t = now_ns();
  for (auto& m : metadata_)
    if (m.global_iteration == global_iteration)
      for (auto& id : ids) {
        m.eval_submitted[id] = t;
        m.eval_received[id] = t;
      }
  evaluations_.push_back(std::move(ce));
}

// ---------------------------------------------------------------------------
std::string Controller::participating_learners() const {
  std::lock_guard<std::mutex> g(mu_);
  Writer w;
  for (auto& [id, rec] : learners_) {
    Writer d;
    d.bytes(1, id, true);
    d.bytes(3, rec.server_entity, true);
    d.bytes(4, rec.dataset_spec, true);
    w.msg(1, d);
  }
  return w.take();
}

std::string Controller::runtime_metadata_lineage(int n) const {
  std::lock_guard<std::mutex> g(mu_);
  Writer w;
  std::ostringstream js;
  js << "[";
  size_t count = 0;
  for (auto& m : metadata_) {
    if (n > 0 && (int)count >= n) break;
    w.bytes(1, m.serialize(), true);
    if (count) js << ",";
    js << "{\"global_iteration\":" << m.global_iteration << ",\"started_at_ns\":" << m.started_at
       << ",\"completed_at_ns\":" << m.completed_at
       << ",\"model_aggregation_total_duration_ms\":" << m.agg_total_ms << "}";
    ++count;
  }
  js << "]";
  w.bytes(2, js.str());
  return w.take();
}

std::string Controller::community_evaluation_lineage(int n) const {
  std::lock_guard<std::mutex> g(mu_);
  Writer w;
  int count = 0;
  for (auto& ce : evaluations_) {
    if (n > 0 && count >= n) break;
    Writer c;
    c.u64(1, ce.global_iteration);
    for (auto& [k, v] : ce.evals) c.map_str_bytes_msg(2, k, v);
    w.msg(1, c);
    ++count;
  }
  return w.take();
}

std::string Controller::local_task_lineage(int n, const std::vector<std::string>& ids) const {
  std::lock_guard<std::mutex> g(mu_);
  Writer w;
  std::vector<std::string> want = ids;
  if (want.empty())
    for (auto& [k, _] : local_meta_) want.push_back(k);
  for (auto& id : want) {
    auto it = local_meta_.find(id);
    if (it == local_meta_.end()) continue;
    Writer lt;
    int count = 0;
    for (auto& tm : it->second) {
      if (n > 0 && count >= n) break;
      lt.bytes(1, tm.raw, true);
      ++count;
    }
    w.map_str_msg(1, id, lt);
  }
  return w.take();
}

std::string Controller::community_model_lineage(int n) const {
  std::lock_guard<std::mutex> g(mu_);
  Writer w;
  int count = 0;
  for (auto& fm : community_lineage_) {
    if (n > 0 && count >= n) break;
    w.bytes(1, fm, true);
    ++count;
  }
  return w.take();
}

std::string Controller::learner_local_model_lineage(int n,
                                                    const std::vector<std::string>& server_entities) {
  std::lock_guard<std::mutex> g(mu_);
  Writer w;
  for (auto& se_bytes : server_entities) {
    WireMsg se(se_bytes);
    const std::string id = se.str(1) + ":" + std::to_string(se.u64(2));
    Writer r;
    r.bytes(1, se_bytes, true);
    const int have = store_->lineage_length(id);
    const int k = n <= 0 ? have : std::min(n, have);
    if (k > 0) {
      auto sel = store_->select({{id, k}});
      for (auto* m : sel[id]) r.bytes(2, serialize_model(*m), true);
    }
    w.msg(1, r);
  }
  store_->reset_state();
  return w.take();
}

}  // namespace mfl
