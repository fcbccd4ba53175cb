// The federation controller state machine (native core of the controller
// process).  Reference: metisfl/controller/core/controller.{h,cc}.
//
// Differences in structure (MI355X-first, not a port):
//  * Transport-agnostic: instead of owning gRPC stubs and completion-queue
//    threads (controller.cc:349-793), every state transition returns a
//    `Dispatch` -- the RunTask / EvaluateModel requests (serialized protos)
//    the caller must deliver.  The Python gRPC servicer delivers them over the
//    network; the on-node collective engine needs no model transfer at all.
//  * Single mutex, no detached threads: the reference's data races on
//    `metadata_` / `community_evaluations_` cannot occur.
//  * Auth tokens are 128-bit random 32-hex strings from a ChaCha20 CSPRNG keyed
//    by getrandom (the reference uses "#learners+1",
//    controller.cc:130; its own proto comment asks for a random token).
//  * GetCommunityModelLineage / GetLearnerLocalModelLineage are implemented
//    (declared but missing in the reference servicer, controller.proto:15,19).
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <random>

#include "he/ckks.h"
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "common/model.h"
#include "engine/aggregation.h"
#include "engine/policies.h"
#include "engine/store.h"

namespace mfl {

struct StatusError : std::runtime_error {
  int code;  // grpc.StatusCode numbering
  StatusError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
enum GrpcCode {
  INVALID_ARGUMENT = 3, NOT_FOUND = 5, ALREADY_EXISTS = 6, FAILED_PRECONDITION = 9,
  UNAUTHENTICATED = 16, INTERNAL = 13
};

struct ControllerConfig {
  std::string hostname = "0.0.0.0";
  uint32_t port = 50051;
  int rule = 1;  // 1 FedAvg, 2 FedStride, 3 FedRec, 4 PWA
  uint32_t stride_length = 0;
  int scaling = SCALE_EXAMPLES;
  float participation_ratio = 1.f;
  uint32_t he_batch_size = 4096, he_scaling_bits = 52;
  std::string he_ctx_file;
  int protocol = PROTO_SYNC;
  int semi_sync_lambda = 0;
  bool semi_sync_recompute = false;
  bool redis = false;
  int lineage = 1;  // <= 0 no eviction
  std::string redis_host = "127.0.0.1";
  uint32_t redis_port = 6379;
  uint32_t batch_size = 100, epochs = 5;
  std::string optimizer_bytes;  // serialized OptimizerConfig
  float percent_validation = 0.f;
  uint32_t community_lineage = 16;  // community models kept for GetCommunityModelLineage
  static ControllerConfig from_params(std::string_view controller_params_bytes);
};

// Request payloads are shared: every learner of a round receives the same
// serialized community model, so identical requests are built ONCE and the
// dispatch holds N references (the reference serialises one copy per learner,
// controller.cc:594-604 -- O(N x model) host work per round).
using Payload = std::shared_ptr<const std::string>;

struct EvalTask {
  std::string learner_id;
  Payload request;  // EvaluateModelRequest
  uint32_t comm_eval_index;
  uint32_t metadata_index;
};
struct Dispatch {
  std::vector<std::pair<std::string, Payload>> run_tasks;  // (learner, RunTaskRequest)
  std::vector<EvalTask> eval_tasks;
};

struct LearnerRec {
  std::string id, token, server_entity, dataset_spec;
  std::string hostname;
  uint32_t port = 0;
  double num_train = 0;
};

struct TaskMeta {
  std::string raw;  // serialized TaskExecutionMetadata
  uint32_t global_iteration = 0, completed_batches = 0, batch_size = 0;
  float completed_epochs = 0.f, ms_per_epoch = 0.f, ms_per_batch = 0.f;
};

struct RoundMeta {
  uint32_t global_iteration = 0;
  int64_t started_at = 0, completed_at = 0;
  std::vector<std::string> assigned, completed_by;
  std::map<std::string, int64_t> train_submitted, train_received, eval_submitted, eval_received;
  std::map<std::string, double> insertion_ms, selection_ms;
  int64_t agg_started = 0, agg_completed = 0;
  double agg_total_ms = 0;
  std::vector<double> block_size, block_mem_kb, block_ms;
  std::vector<Quantifier> quantifiers;
  std::string serialize() const;
};

class Controller {
 public:
  explicit Controller(const std::string& params_bytes);
  const ControllerConfig& config() const { return cfg_; }

  // --- membership ---------------------------------------------------------
  // returns (learner_id, auth_token); schedules the initial task in `dispatch`
  std::pair<std::string, std::string> add_learner(const std::string& server_entity,
                                                  const std::string& dataset_spec,
                                                  Dispatch* dispatch);
  // LeaveFederation: a synchronous barrier that waited only for the leaver is
  // released (the returned dispatch runs the round; the reference stalls)
  Dispatch remove_learner(const std::string& id, const std::string& token);
  // failure detector: drop an unresponsive learner; may complete a pending
  // synchronous barrier (returns that round's dispatch)
  // count = false: a membership change the controller itself makes (a
  // collective relaunch re-registering its ranks), not a failure-detector
  // eviction, so evicted() does not move
  Dispatch evict_learner(const std::string& id, bool count = true);
  uint32_t evicted() const { return evicted_; }
  std::vector<std::string> learner_ids() const;

  // --- task flow ------------------------------------------------------------
  Dispatch learner_completed_task(const std::string& id, const std::string& token,
                                  const std::string& completed_task);
  void replace_community_model(const std::string& federated_model);
  void record_train_submitted(const std::string& id, uint32_t metadata_index);
  void record_evaluation(const std::string& id, uint32_t comm_eval_index, uint32_t metadata_index,
                         const std::string& model_evaluations);

  // --- collective (RCCL) path: aggregation happened on device ------------------
  std::map<std::string, double> scaling_factors(const std::vector<std::string>& ids,
                                                const std::vector<double>& num_train,
                                                const std::vector<double>& batches) const;
  void record_collective_round(uint32_t global_iteration, const std::vector<std::string>& ids,
                               int64_t started_ns, int64_t completed_ns, int64_t agg_started_ns,
                               int64_t agg_completed_ns, const std::vector<std::string>& task_meta,
                               const std::vector<uint64_t>& zeros,
                               const std::vector<uint64_t>& sizes_bytes,
                               const std::vector<uint64_t>& lengths);

  // --- queries (serialized response messages) -----------------------------------
  std::string community_model() const;  // FederatedModel
  std::string participating_learners() const;               // GetParticipatingLearnersResponse
  std::string runtime_metadata_lineage(int n) const;        // GetRuntimeMetadataLineageResponse
  // Collective (RCCL) data plane: the learners evaluated the community model
  // of `global_iteration` in place; model_evaluations[i] is learner ids[i]'s
  // serialized ModelEvaluations (controller.cc:469-485 in the reference).
  void record_community_evaluation(uint32_t global_iteration, const std::vector<std::string>& ids,
                                   const std::vector<std::string>& model_evaluations);
  std::string community_evaluation_lineage(int n) const;    // GetCommunityModelEvaluationLineageResponse
  std::string local_task_lineage(int n, const std::vector<std::string>& ids) const;
  std::string community_model_lineage(int n) const;         // GetCommunityModelLineageResponse
  std::string learner_local_model_lineage(int n, const std::vector<std::string>& server_entities);
  uint32_t global_iteration() const;
  size_t num_learners() const;

  // --- checkpoint / resume (checkpoint.cc) -------------------------------------
  std::string checkpoint() const;          // self-describing binary snapshot
  void restore(const std::string& blob);   // into a controller built with the same params
  Dispatch resume_dispatch();              // the current round's RunTask for every learner

 private:
  void validate(const std::string& id, const std::string& token) const;
  // Run-task request for learner `id`; requests that come out identical
  // (same local-step template) share one payload through `cache`.
  Payload make_run_task(const std::string& id, const std::string& fm_bytes, uint32_t global_iteration,
                        std::map<uint32_t, Payload>& cache) const;
  std::string make_eval_task(const FederatedModelT& model) const;
  void schedule_initial_task_locked(const std::string& id, Dispatch* d);
  Dispatch schedule_tasks_locked(const std::string& id, uint32_t task_iteration);
  Dispatch run_scheduled_locked(const std::vector<std::string>& to_schedule,
                                const std::vector<std::string>& active, uint32_t task_iteration);
  FederatedModelT compute_community_model_locked(const std::vector<std::string>& ids,
                                                 uint32_t meta_idx);
  void update_templates_locked(const std::vector<std::string>& ids);
  void record_quantifiers_locked(const FederatedModelT& m, uint32_t meta_idx);
  std::vector<std::string> active_ids_locked() const;
  std::string random_token();

  ControllerConfig cfg_;
  mutable std::mutex mu_;
  std::map<std::string, LearnerRec> learners_;
  std::map<std::string, uint32_t> templates_;
  std::map<std::string, std::deque<TaskMeta>> local_meta_;  // newest first
  // global iteration of each CURRENT member's last recorded completion: the
  // duplicate-completion check.  Cleared when a learner leaves or is evicted
  // (its local_meta_ lineage is kept, as the reference keeps
  // local_tasks_metadata_), so a learner that rejoins under the same
  // host:port in the same round is not mistaken for a retry.
  std::map<std::string, uint32_t> completed_iter_;
  std::unique_ptr<Scheduler> scheduler_;
  std::unique_ptr<AggregationFunction> aggregator_;
  std::unique_ptr<ModelStore> store_;
  FederatedModelT community_;
  bool community_set_ = false;
  std::deque<std::string> community_lineage_;  // serialized FederatedModel, newest first
  std::vector<RoundMeta> metadata_;
  struct CommEval {
    uint32_t global_iteration = 0;
    std::map<std::string, std::string> evals;  // learner -> ModelEvaluations
  };
  std::vector<CommEval> evaluations_;
  uint32_t global_iteration_ = 0;
  uint32_t evicted_ = 0;
  ChaCha20Rng rng_;  // auth tokens: ChaCha20 keyed from getrandom (he/ckks.h)
};

int64_t now_ns();
long total_memory_kb();

}  // namespace mfl
