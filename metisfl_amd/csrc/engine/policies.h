// Scheduling, selection and scaling policies of the controller engine.
//
// Semantics follow the reference controller:
//  * SynchronousScheduler: barrier over the set of active learners
//    (scheduling/synchronous_scheduler.h:13-34); also serves SEMI_SYNCHRONOUS
//    (controller_utils.cc:59-68).
//  * AsynchronousScheduler: re-schedule the finisher immediately
//    (scheduling/asynchronous_scheduler.h:12-18).
//  * ScheduledCardinality selector: fewer than 2 scheduled -> aggregate over
//    every active learner (selection/scheduled_cardinality.h:15-30).
//  * Scalers: NUM_COMPLETED_BATCHES / NUM_PARTICIPANTS / NUM_TRAINING_EXAMPLES
//    (scaling/*.cc) incl. the "single participant among many learners gets
//    its raw value" quirk.
#pragma once
#include <algorithm>
#include <map>
#include <set>
#include <string>
#include <vector>

namespace mfl {

enum Protocol { PROTO_UNKNOWN = 0, PROTO_SYNC = 1, PROTO_ASYNC = 2, PROTO_SEMI_SYNC = 3 };
enum ScalingKind { SCALE_UNKNOWN = 0, SCALE_BATCHES = 1, SCALE_PARTICIPANTS = 2, SCALE_EXAMPLES = 3 };

class Scheduler {
 public:
  virtual ~Scheduler() = default;
  // learner `id` finished; `active` = all learners currently in the federation
  virtual std::vector<std::string> schedule_next(const std::string& id,
                                                 const std::vector<std::string>& active) = 0;
  // membership changed (a learner was evicted): the learners whose round can
  // proceed now, if any
  virtual std::vector<std::string> poll(const std::vector<std::string>&) { return {}; }
  virtual std::string name() const = 0;
};

class SynchronousScheduler : public Scheduler {
 public:
  std::vector<std::string> schedule_next(const std::string& id,
                                         const std::vector<std::string>& active) override {
    done_.insert(id);
    return poll(active);
  }
  std::vector<std::string> poll(const std::vector<std::string>& active) override {
    // only count learners that are still active (a learner that left must not
    // stall the barrier; the reference waits on |active| as well)
    size_t n = 0;
    for (auto& a : active) n += done_.count(a);
    if (n >= active.size() && !active.empty()) {
      std::vector<std::string> out;
      for (auto& a : active)
        if (done_.count(a)) out.push_back(a);
      done_.clear();
      return out;
    }
    return {};
  }
  std::string name() const override { return "SynchronousScheduler"; }

 private:
  std::set<std::string> done_;
};

class AsynchronousScheduler : public Scheduler {
 public:
  std::vector<std::string> schedule_next(const std::string& id,
                                         const std::vector<std::string>&) override {
    return {id};
  }
  std::string name() const override { return "AsynchronousScheduler"; }
};

inline std::vector<std::string> select_scheduled_cardinality(
    const std::vector<std::string>& scheduled, const std::vector<std::string>& active) {
  return scheduled.size() < 2 ? active : scheduled;
}

struct ScalerInput {
  std::string id;
  double num_training_examples = 0;
  double completed_batches = 0;
};

inline std::map<std::string, double> compute_scaling_factors(int kind, size_t num_all_learners,
                                                             const std::vector<ScalerInput>& parts) {
  std::map<std::string, double> out;
  if (parts.empty()) return out;
  if (num_all_learners == 1) {
    for (auto& p : parts) out[p.id] = 1.0;
    return out;
  }
  if (kind == SCALE_PARTICIPANTS) {
    for (auto& p : parts) out[p.id] = parts.size() == 1 ? 1.0 : 1.0 / (double)parts.size();
    return out;
  }
  auto value = [&](const ScalerInput& p) {
    return kind == SCALE_BATCHES ? p.completed_batches : p.num_training_examples;
  };
  if (parts.size() == 1) {
    out[parts[0].id] = value(parts[0]);
    return out;
  }
  long long total = 0;
  for (auto& p : parts) total += (long long)value(p);
  for (auto& p : parts) out[p.id] = total ? value(p) / (double)total : 1.0 / (double)parts.size();
  return out;
}

}  // namespace mfl
