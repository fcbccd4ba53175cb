#include "engine/aggregation.h"

#include <omp.h>

#include <cstring>
#include <stdexcept>
#include <type_traits>

#include "engine/device_agg.h"
#include "he/ckks.h"

namespace mfl {
namespace {

template <typename T>
inline T add_wrap(T a, T b) {
  if constexpr (std::is_integral_v<T>) {
    using U = std::make_unsigned_t<T>;
    return (T)(U)((U)a + (U)b);
  } else {
    return a + b;
  }
}
template <typename T>
inline T sub_wrap(T a, T b) {
  if constexpr (std::is_integral_v<T>) {
    using U = std::make_unsigned_t<T>;
    return (T)(U)((U)a - (U)b);
  } else {
    return a - b;
  }
}
template <typename T>
inline T term(T x, double w) {
  return (T)((double)x * w);  // (T)(double * double): truncation for integers
}

template <typename F>
void dispatch(int dt, F&& f) {
  switch (dt) {
    case DT_INT8: f((int8_t)0); break;
    case DT_INT16: f((int16_t)0); break;
    case DT_INT32: f((int32_t)0); break;
    case DT_INT64: f((int64_t)0); break;
    case DT_UINT8: f((uint8_t)0); break;
    case DT_UINT16: f((uint16_t)0); break;
    case DT_UINT32: f((uint32_t)0); break;
    case DT_UINT64: f((uint64_t)0); break;
    case DT_FLOAT32: f((float)0); break;
    case DT_FLOAT64: f((double)0); break;
    default: throw std::runtime_error("unsupported tensor data type");
  }
}

// Parallel chunking: large variables are split across threads so a model with
// one huge embedding does not serialise on one core (the reference
// parallelises over variables only, federated_average.cc:101).
struct Chunk {
  size_t var, beg, end;
};
// Small models stay on one thread: an OpenMP team's barrier costs more than
// the whole loop there (and, on oversubscribed or CPU-quota'd hosts, a
// spinning team was measured at 30-60 ms for a 0.4 MB model vs 0.5 ms serial).
constexpr size_t kParallelMinElems = size_t(1) << 20;

size_t total_elems(const ModelT& m) {
  size_t n = 0;
  for (auto& v : m.vars) n += v.t.length;
  return n;
}

std::vector<Chunk> make_chunks(const ModelT& m, size_t grain = 1 << 16) {
  std::vector<Chunk> out;
  for (size_t v = 0; v < m.vars.size(); ++v) {
    const size_t n = m.vars[v].t.length;
    for (size_t b = 0; b < n; b += grain) out.push_back({v, b, std::min(n, b + grain)});
    if (n == 0) out.push_back({v, 0, 0});
  }
  return out;
}

}  // namespace

void weighted_sum_into(ModelT& out, const std::vector<const ModelT*>& models,
                       const std::vector<double>& weights) {
  if (models.empty()) return;
  const ModelT& sample = *models.front();
  for (size_t v = 0; v < sample.vars.size(); ++v) {
    const auto& sv = sample.vars[v];
    if (sv.ciphertext) throw std::runtime_error("Only Plaintext variables are supported.");
    for (auto* m : models)
      if (m->vars.size() != sample.vars.size() || m->vars[v].t.value.size() != sv.t.value.size())
        throw std::runtime_error("models have mismatching structure");
  }
  // K1 on the device when the controller has one (byte-identical result)
  if (DeviceAggregator::enabled_for(sample.byte_size()) &&
      DeviceAggregator::get()->weighted_sum(out, models, weights))
    return;
  out.vars.resize(sample.vars.size());
  for (size_t v = 0; v < sample.vars.size(); ++v) {
    auto& ov = out.vars[v];
    const auto& sv = sample.vars[v];
    ov.name = sv.name;
    ov.trainable = sv.trainable;
    ov.ciphertext = false;
    ov.t.length = sv.t.length;
    ov.t.dims = sv.t.dims;
    ov.t.dtype = sv.t.dtype;
    ov.t.byte_order = sv.t.byte_order;
    ov.t.fortran_order = sv.t.fortran_order;
    ov.t.value.assign((size_t)sv.t.length * dtype_size(sv.t.dtype), '\0');
  }
  const auto chunks = make_chunks(out);
  const bool par = total_elems(out) * models.size() >= kParallelMinElems;
#pragma omp parallel for schedule(dynamic, 1) if (par)
  for (size_t c = 0; c < chunks.size(); ++c) {
    const Chunk ch = chunks[c];
    auto& ov = out.vars[ch.var];
    dispatch(ov.t.dtype, [&](auto zero) {
      using T = decltype(zero);
      T* o = reinterpret_cast<T*>(&ov.t.value[0]);
      for (size_t k = 0; k < models.size(); ++k) {
        const T* x = reinterpret_cast<const T*>(models[k]->vars[ch.var].t.value.data());
        const double w = weights[k];
        for (size_t i = ch.beg; i < ch.end; ++i) o[i] = add_wrap<T>(o[i], term<T>(x[i], w));
      }
    });
  }
}

void merge_models(ModelT& y, const ModelT& x, double w, int op) {
  if (!same_structure(y, x)) throw std::runtime_error("merge: mismatching structure");
  const auto chunks = make_chunks(y);
  const bool par = total_elems(y) >= kParallelMinElems;
#pragma omp parallel for schedule(dynamic, 1) if (par)
  for (size_t c = 0; c < chunks.size(); ++c) {
    const Chunk ch = chunks[c];
    auto& yv = y.vars[ch.var];
    dispatch(yv.t.dtype, [&](auto zero) {
      using T = decltype(zero);
      T* o = reinterpret_cast<T*>(&yv.t.value[0]);
      const T* xi = reinterpret_cast<const T*>(x.vars[ch.var].t.value.data());
      if (op == 0)
        for (size_t i = ch.beg; i < ch.end; ++i) o[i] = add_wrap<T>(o[i], term<T>(xi[i], w));
      else
        for (size_t i = ch.beg; i < ch.end; ++i) o[i] = sub_wrap<T>(o[i], term<T>(xi[i], w));
    });
  }
}

void scale_model(ModelT& y, double z, int op) {
  const auto chunks = make_chunks(y);
  const bool par = total_elems(y) >= kParallelMinElems;
#pragma omp parallel for schedule(dynamic, 1) if (par)
  for (size_t c = 0; c < chunks.size(); ++c) {
    const Chunk ch = chunks[c];
    auto& yv = y.vars[ch.var];
    dispatch(yv.t.dtype, [&](auto zero) {
      using T = decltype(zero);
      T* o = reinterpret_cast<T*>(&yv.t.value[0]);
      if (op == 2)
        for (size_t i = ch.beg; i < ch.end; ++i) o[i] = (T)((double)o[i] * z);
      else
        for (size_t i = ch.beg; i < ch.end; ++i) o[i] = (T)((double)o[i] / z);
    });
  }
}

// ---------------------------------------------------------------------------
FederatedModelT FederatedAverage::aggregate(const AggInput& pairs) {
  FederatedModelT fm;
  if (pairs.empty() || pairs.front().empty()) return fm;
  std::vector<const ModelT*> models;
  std::vector<double> ws;
  for (auto& lineage : pairs) {
    if (lineage.empty()) continue;
    models.push_back(lineage.front().model);
    ws.push_back(lineage.front().w);
  }
  weighted_sum_into(fm.model, models, ws);
  fm.num_contributors = (uint32_t)pairs.size();
  return fm;
}

// ---------------------------------------------------------------------------
// With a device the `scaled` state lives in HBM (dev_ = its handle) and the
// community model is materialised once per aggregate() call (fetch_pending),
// since intermediate community values are overwritten before anyone sees them.
RollingAverageBase::~RollingAverageBase() { release_device(); }

void RollingAverageBase::release_device() {
  if (dev_ >= 0) DeviceAggregator::get()->roll_free(dev_);
  dev_ = -1;
  pending_ = PENDING_NONE;
}

void RollingAverageBase::initialize(const ModelT* m, double w) {
  release_device();
  z_ = w;
  community_.num_contributors = 1;
  if (DeviceAggregator::enabled_for(m->byte_size())) {
    dev_ = DeviceAggregator::get()->roll_init(*m, w);
    if (dev_ >= 0) {
      scaled_ = ModelT();
      pending_ = PENDING_COPY;  // reference keeps the *scaled* model here
      return;
    }
  }
  scaled_ = *m;
  scale_model(scaled_, w, 2);
  community_.model = scaled_;  // reference keeps the *scaled* model here
}

void RollingAverageBase::update_scaled(const ModelT* existing, const ModelT* latest,
                                       double w_existing, double w_new) {
  bool existing_done = !(existing && !existing->empty());
  if (dev_ >= 0) {
    auto* d = DeviceAggregator::get();
    try {
      if (!existing_done) d->roll_merge(dev_, *existing, w_existing, 1);
      existing_done = true;
      d->roll_merge(dev_, *latest, w_new, 0);
      return;
    } catch (const std::runtime_error&) {
      // no room on the device for this merge's operand: the rolling state
      // continues on the host from the device's scaled sum (what the host
      // path holds at this point), so the aggregation does not fail
      d->roll_fetch(dev_, scaled_, 1.0, 4);
      release_device();
    }
  }
  if (!existing_done) merge_models(scaled_, *existing, w_existing, 1);
  merge_models(scaled_, *latest, w_new, 0);
}

void RollingAverageBase::update_community() {
  if (dev_ >= 0) {
    pending_ = PENDING_DIV;
    return;
  }
  community_.model = scaled_;
  scale_model(community_.model, z_, 3);
}

void RollingAverageBase::fetch_pending() {
  if (dev_ < 0 || pending_ == PENDING_NONE) return;
  DeviceAggregator::get()->roll_fetch(dev_, community_.model, pending_ == PENDING_COPY ? 1.0 : z_,
                                      pending_ == PENDING_COPY ? 4 : 3);
  pending_ = PENDING_NONE;
}

FederatedModelT FederatedStride::aggregate(const AggInput& pairs) {
  for (auto& lineage : pairs) {
    if (lineage.empty()) continue;
    const ModelT* latest = lineage.front().model;
    const double w = lineage.front().w;
    if (community_.num_contributors == 0) {
      initialize(latest, w);
    } else {
      z_ += w;
      update_scaled(nullptr, latest, 0.0, w);
      update_community();
      community_.num_contributors += 1;
    }
  }
  fetch_pending();
  return community_;
}

void FederatedStride::reset() {
  release_device();
  z_ = 0.0;
  community_ = FederatedModelT();
  scaled_ = ModelT();
}

FederatedModelT FederatedRecency::aggregate(const AggInput& pairs) {
  if (pairs.empty()) return {};
  const auto& lineage = pairs.front();
  if ((int)lineage.size() > required_lineage_length() || lineage.empty()) return {};
  const ModelT* latest = lineage.back().model;
  const double w_new = lineage.back().w;
  if (community_.num_contributors == 0) {
    initialize(latest, w_new);
  } else if (lineage.size() == 1) {
    z_ += w_new;
    update_scaled(nullptr, latest, 0.0, w_new);
    update_community();
    community_.num_contributors += 1;
  } else {
    const ModelT* existing = lineage.front().model;
    const double w_old = lineage.front().w;
    z_ = z_ - w_old + w_new;
    update_scaled(existing, latest, w_old, w_new);
    update_community();
  }
  fetch_pending();
  return community_;
}

// ---------------------------------------------------------------------------
PrivateWeightedAverage::PrivateWeightedAverage(uint32_t batch_size, uint32_t scaling_bits,
                                               const std::string& ctx_file)
    : he_(new CKKS(batch_size, scaling_bits)) {
  if (!ctx_file.empty()) he_->load_context(ctx_file);
}

PrivateWeightedAverage::~PrivateWeightedAverage() = default;

FederatedModelT PrivateWeightedAverage::aggregate(const AggInput& pairs) {
  FederatedModelT fm;
  if (pairs.empty() || pairs.front().empty()) return fm;
  const ModelT& sample = *pairs.front().front().model;
  std::vector<double> ws;
  for (auto& l : pairs) ws.push_back(pairs.size() == 1 ? 1.0 : l.front().w);
  fm.model.vars.resize(sample.vars.size());
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t v = 0; v < sample.vars.size(); ++v) {
    std::vector<std::string_view> cts;
    for (auto& l : pairs) {
      const auto& var = l.front().model->vars[v];
      if (!var.ciphertext) throw std::runtime_error("PWA expects ciphertext variables");
      cts.push_back(var.t.value);
    }
    auto& out = fm.model.vars[v];
    out = sample.vars[v];
    out.t.value = he_->weighted_average(cts, ws);
  }
  fm.num_contributors = (uint32_t)pairs.size();
  return fm;
}

}  // namespace mfl
