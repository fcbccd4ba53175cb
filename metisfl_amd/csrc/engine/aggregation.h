// Aggregation rules of the native controller engine.
//
//  * FedAvg     -- sum_i (T)(w_i * x_i), per-term conversion to the tensor
//                  type (integer truncation kept: federated_average.cc:14-37)
//  * FedStride  -- streaming blocks of `stride_length` learners over a
//                  rolling scaled sum (federated_stride.cc:6-64)
//  * FedRec     -- asynchronous recency rule: replace a learner's previous
//                  contribution with its newest (federated_recency.cc:8-100)
//  * PWA        -- private weighted average of CKKS ciphertexts (he/ckks.h)
//
// Deviation (documented): the rolling base implements the
// intended `scaled += w_new * new` when a learner has no previous model; the
// reference reads a just-cleared std::string buffer there.
#pragma once
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "common/model.h"

namespace mfl {

struct ModelRef {
  const ModelT* model;
  double w;
};
// pairs[i] = the lineage (oldest..newest) of learner i with its scaling factor
using AggInput = std::vector<std::vector<ModelRef>>;

class AggregationFunction {
 public:
  virtual ~AggregationFunction() = default;
  virtual FederatedModelT aggregate(const AggInput& pairs) = 0;
  virtual int required_lineage_length() const = 0;
  virtual std::string name() const = 0;
  virtual void reset() {}
};

// Rule-level helpers exposed for tests / Python (host reference kernels).
// out[var] = sum_i (T)(w_i * x_i[var])  over `models` in order.
void weighted_sum_into(ModelT& out, const std::vector<const ModelT*>& models,
                       const std::vector<double>& weights);
// y = y (+|-) (T)(x * w)      op: 0 add, 1 sub
void merge_models(ModelT& y, const ModelT& x, double w, int op);
// y = (T)(y * z) | (T)(y / z)  op: 2 mul, 3 div
void scale_model(ModelT& y, double z, int op);

class FederatedAverage : public AggregationFunction {
 public:
  FederatedModelT aggregate(const AggInput& pairs) override;
  int required_lineage_length() const override { return 1; }
  std::string name() const override { return "FedAvg"; }
};

class RollingAverageBase : public AggregationFunction {
 public:
  ~RollingAverageBase() override;

 protected:
  enum Pending { PENDING_NONE, PENDING_COPY, PENDING_DIV };
  void release_device();
  void fetch_pending();
  void initialize(const ModelT* m, double w);
  void update_scaled(const ModelT* existing, const ModelT* latest, double w_existing, double w_new);
  void update_community();
  ModelT scaled_;
  FederatedModelT community_;
  double z_ = 0.0;
  int dev_ = -1;  // device-resident `scaled` state (DeviceAggregator handle)
  Pending pending_ = PENDING_NONE;
};

class FederatedStride : public RollingAverageBase {
 public:
  FederatedModelT aggregate(const AggInput& pairs) override;
  int required_lineage_length() const override { return 1; }
  std::string name() const override { return "FedStride"; }
  void reset() override;
};

class FederatedRecency : public RollingAverageBase {
 public:
  FederatedModelT aggregate(const AggInput& pairs) override;
  int required_lineage_length() const override { return 2; }
  std::string name() const override { return "FedRec"; }
};

class CKKS;  // he/ckks.h

class PrivateWeightedAverage : public AggregationFunction {
 public:
  PrivateWeightedAverage(uint32_t batch_size, uint32_t scaling_bits, const std::string& ctx_file);
  ~PrivateWeightedAverage() override;
  FederatedModelT aggregate(const AggInput& pairs) override;
  int required_lineage_length() const override { return 1; }
  std::string name() const override { return "PWA"; }

 private:
  std::unique_ptr<CKKS> he_;
};

}  // namespace mfl
