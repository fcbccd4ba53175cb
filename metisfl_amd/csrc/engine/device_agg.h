// Device-resident aggregation backend of the native controller engine.
//
// The reference controller aggregates on the host, one tensor at a time,
// re-deserialising every TensorSpec per step (federated_average.cc:14-37,
// federated_stride.cc:6-64, private_weighted_average.cc:24-82).  When the
// controller process sees a HIP device this backend takes over instead:
//
//  * residency: a learner's model is uploaded when it ARRIVES
//    (Controller::learner_completed_task -> stage()), through a ring of pinned
//    staging chunks on a dedicated upload stream, into one packed device
//    buffer per model (variables 256-B aligned).  By the time the last learner
//    of a synchronous round reports, every other model is already in HBM, so
//    the round's aggregation reads only device memory.
//  * FedAvg (K1): one multi-tensor launch over a tile table covering every
//    variable of every model (dtype per tile), out = SUM_k (T)((double)x_k*w_k)
//    in learner order -- byte-identical to the host rule.
//  * FedStride / FedRec (K2): the rolling `scaled` state lives on the device;
//    merge/scale are launches on it and only the community model comes back.
//  * PWA (K9): CKKS ciphertext limbs are read straight from the staged model
//    buffers (or uploaded when not resident).
//
// All methods are thread-safe (one mutex; the engine itself is serialised by
// the controller lock, PWA calls arrive from an OpenMP loop).  Every entry
// point returns false when the device path does not apply, and the caller
// falls back to the host implementation -- results are identical either way.
//
// Control: METISFL_AMD_DEVICE_AGG = auto (default: use a device if one is
// visible) | 0 (never) | 1 (require a device: get() throws without one);
// METISFL_AMD_DEVICE_AGG_MIN_BYTES (default 1 MiB): smaller models stay on
// the host, where the PCIe round trip would dominate.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

#include "common/model.h"

namespace mfl {

struct DeviceAggStats {
  uint64_t staged_models = 0, staged_bytes = 0;
  uint64_t resident_hits = 0, cold_uploads = 0;
  uint64_t fedavg_calls = 0, rolling_calls = 0, pwa_calls = 0;
  double last_kernel_ms = 0, last_total_ms = 0, last_upload_ms = 0, last_download_ms = 0;
  uint64_t resident_bytes = 0;
  int device = -1;
  std::string device_name;
};

class DeviceAggregator {
 public:
  // nullptr when disabled or no HIP device is visible (never throws unless
  // METISFL_AMD_DEVICE_AGG=1 and no device exists).
  static DeviceAggregator* get();
  static DeviceAggregator* peek();  // the instance if get() already created one
  static bool enabled_for(size_t model_bytes);
  // Process-wide switch (tests compare host and device results in one process).
  // min_bytes >= 0 also overrides METISFL_AMD_DEVICE_AGG_MIN_BYTES.
  static void set_enabled(bool on, long long min_bytes = -1);

  virtual ~DeviceAggregator() = default;

  // Upload `m` (async) and remember it under `learner`; keeps at most
  // `keep` models per learner (the store's lineage length).
  virtual void stage(const std::string& learner, const ModelT& m, int keep) = 0;
  virtual void drop(const std::string& learner) = 0;
  virtual void clear() = 0;

  // out = SUM_k (T)(models[k] * w[k]); `out` must already carry the layout
  // (names / dtypes / lengths) and zero-sized values are allocated here.
  virtual bool weighted_sum(ModelT& out, const std::vector<const ModelT*>& models,
                            const std::vector<double>& weights) = 0;

  // Rolling states (FedStride / FedRec), one per aggregator instance.
  // op: 0 add, 1 sub (merge), 2 mul, 3 div (scale), 4 copy.
  virtual int roll_init(const ModelT& m, double w) = 0;  // new state scaled = (T)(m * w); -1: n/a
  virtual void roll_merge(int h, const ModelT& x, double w, int op) = 0;  // scaled (+|-)= (T)(x*w)
  virtual void roll_fetch(int h, ModelT& out, double z, int op) = 0;      // out = (T)(scaled op z)
  virtual void roll_free(int h) = 0;

  // K9: out[j] = SUM_i w_i * ct_i[j] mod q_limb(j), ciphertext bodies of
  // `total` uint64 words laid out [nct][2][L][N].
  virtual bool ckks_pwa(const std::vector<const uint64_t*>& bodies, const std::vector<uint64_t>& wq,
                        const std::vector<uint64_t>& wqs, const std::vector<uint64_t>& q, uint32_t L,
                        uint32_t N, uint64_t total, uint64_t* out) = 0;

  virtual DeviceAggStats stats() const = 0;
};

}  // namespace mfl
