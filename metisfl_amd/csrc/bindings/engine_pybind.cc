// pybind11 module ``metisfl_amd._engine``: the native controller engine and
// the RNS-CKKS scheme.  Counterpart of the reference's ``controller`` and
// ``fhe`` pybind modules (controller_pybind.cc:16-68, ckks_pybind.cc:15-100).
// Protos cross the boundary as serialized bytes.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "common/model.h"
#include "common/tfrecord.h"
#include "engine/aggregation.h"
#include "engine/controller.h"
#include "engine/device_agg.h"
#include "engine/policies.h"
#include "he/ckks.h"
#include "common/chacha20.h"
#include <chrono>
#include <cstdio>
#include <cstring>

namespace py = pybind11;
using namespace mfl;

namespace {

py::bytes B(const std::string& s) { return py::bytes(s); }

// Shared payloads become ONE Python bytes object referenced by every task.
py::dict dispatch_to_py(const Dispatch& d) {
  py::list runs, evals;
  std::map<const std::string*, py::bytes> objs;
  auto obj = [&](const Payload& p) {
    auto it = objs.find(p.get());
    if (it == objs.end()) it = objs.emplace(p.get(), B(*p)).first;
    return it->second;
  };
  for (auto& [id, req] : d.run_tasks) runs.append(py::make_tuple(id, obj(req)));
  for (auto& e : d.eval_tasks)
    evals.append(py::make_tuple(e.learner_id, obj(e.request), e.comm_eval_index, e.metadata_index));
  py::dict out;
  out["run_tasks"] = runs;
  out["eval_tasks"] = evals;
  return out;
}

// Host reference aggregation over serialized models (tests / tools).
std::vector<ModelT> parse_all(const std::vector<std::string>& models) {
  std::vector<ModelT> ms;
  ms.reserve(models.size());
  for (auto& m : models) ms.push_back(parse_model(m));
  return ms;
}

py::bytes aggregate_models(const std::string& rule, const std::vector<std::string>& models,
                           const std::vector<double>& weights, int stride) {
  auto ms = parse_all(models);
  std::unique_ptr<AggregationFunction> agg;
  if (rule == "fed_avg") agg.reset(new FederatedAverage());
  else if (rule == "fed_stride") agg.reset(new FederatedStride());
  else throw std::runtime_error("unknown rule " + rule);
  FederatedModelT out;
  {
    py::gil_scoped_release nogil;
    const size_t s = (rule == "fed_stride" && stride > 0) ? (size_t)stride : ms.size();
    for (size_t b = 0; b < ms.size(); b += s) {
      AggInput in;
      for (size_t i = b; i < std::min(ms.size(), b + s); ++i) in.push_back({{&ms[i], weights[i]}});
      out = agg->aggregate(in);
    }
  }
  return B(serialize_federated_model(out));
}

struct StagedModels {
  std::vector<ModelT> ms;
  double last_aggregate_ms = 0;  // the engine call alone (no serialization)
  StagedModels(const std::vector<std::string>& ids, const std::vector<std::string>& models) {
    for (auto& s : models) ms.push_back(parse_model(s));
    py::gil_scoped_release nogil;
    if (DeviceAggregator::enabled_for(ms.empty() ? 0 : ms[0].byte_size()))
      for (size_t i = 0; i < ms.size(); ++i) DeviceAggregator::get()->stage(ids.at(i), ms[i], 1);
  }
  py::bytes aggregate(const std::string& rule, const std::vector<double>& weights, int stride) {
    std::unique_ptr<AggregationFunction> agg;
    if (rule == "fed_avg") agg.reset(new FederatedAverage());
    else if (rule == "fed_stride") agg.reset(new FederatedStride());
    else throw std::runtime_error("unknown rule " + rule);
    FederatedModelT out;
    {
      py::gil_scoped_release nogil;
      const auto t0 = std::chrono::steady_clock::now();
      const size_t s = (rule == "fed_stride" && stride > 0) ? (size_t)stride : ms.size();
      for (size_t b = 0; b < ms.size(); b += s) {
        AggInput in;
        for (size_t i = b; i < std::min(ms.size(), b + s); ++i) in.push_back({{&ms[i], weights[i]}});
        out = agg->aggregate(in);
      }
      agg->reset();
      last_aggregate_ms =
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return B(serialize_federated_model(out));
  }
};

class PyRecency {
 public:
  // lineage: 1 or 2 (old, new) serialized models with weights
  py::bytes aggregate(const std::vector<std::string>& models, const std::vector<double>& weights) {
    auto ms = parse_all(models);
    AggInput in(1);
    for (size_t i = 0; i < ms.size(); ++i) in[0].push_back({&ms[i], weights[i]});
    FederatedModelT out = agg_.aggregate(in);
    return B(serialize_federated_model(out));
  }

 private:
  FederatedRecency agg_;
};

}  // namespace

PYBIND11_MODULE(_engine, m) {
  m.doc() = "metisfl_amd native controller engine (scheduler, aggregation, model store, CKKS)";

  static py::exception<StatusError> status_exc(m, "EngineStatusError");
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const StatusError& e) {
      // args = (grpc status code, message)
      PyErr_SetObject(status_exc.ptr(), py::make_tuple(e.code, e.what()).ptr());
    }
  });

  py::class_<Controller>(m, "Controller")
      // the GIL is released around everything that may block on the model
      // store (a Redis round trip) or aggregate large models
      .def(py::init([](py::bytes params) {
        std::string p(params);
        py::gil_scoped_release nogil;
        return new Controller(p);
      }))
      .def("add_learner",
           [](Controller& c, py::bytes se, py::bytes ds, bool schedule) {
             // schedule=false: a collective (RCCL data plane) rank -- no
             // RunTask is scheduled and no round is opened for it
             Dispatch d;
             auto r = c.add_learner(std::string(se), std::string(ds), schedule ? &d : nullptr);
             return py::make_tuple(r.first, r.second, dispatch_to_py(d));
           },
           py::arg("server_entity"), py::arg("dataset_spec"), py::arg("schedule") = true)
      .def("remove_learner",
           [](Controller& c, const std::string& id, const std::string& tok) {
             Dispatch d;
             {
               py::gil_scoped_release nogil;
               d = c.remove_learner(id, tok);
             }
             return dispatch_to_py(d);
           })
      .def(
          "evict_learner",
          [](Controller& c, const std::string& id, bool count) {
            Dispatch d;
            {
              py::gil_scoped_release nogil;
              d = c.evict_learner(id, count);
            }
            return dispatch_to_py(d);
          },
          py::arg("id"), py::arg("count") = true)
      .def("checkpoint",
           [](const Controller& c) {
             std::string s;
             {
               py::gil_scoped_release nogil;
               s = c.checkpoint();
             }
             return B(s);
           })
      .def("restore", [](Controller& c, const std::string& blob) { c.restore(blob); })
      .def("resume_dispatch",
           [](Controller& c) {
             Dispatch d;
             {
               py::gil_scoped_release nogil;
               d = c.resume_dispatch();
             }
             return dispatch_to_py(d);
           })
      .def("evicted", &Controller::evicted)
      .def("learner_ids", &Controller::learner_ids)
      .def("num_learners", &Controller::num_learners)
      .def("global_iteration", &Controller::global_iteration)
      .def("learner_completed_task",
           [](Controller& c, const std::string& id, const std::string& tok, py::bytes task) {
             std::string t(task);
             Dispatch d;
             {
               py::gil_scoped_release nogil;
               d = c.learner_completed_task(id, tok, t);
             }
             return dispatch_to_py(d);
           })
      .def("replace_community_model",
           [](Controller& c, py::bytes fm) { c.replace_community_model(std::string(fm)); })
      .def("record_train_submitted", &Controller::record_train_submitted)
      .def("record_evaluation",
           [](Controller& c, const std::string& id, uint32_t ce, uint32_t mi, py::bytes ev) {
             c.record_evaluation(id, ce, mi, std::string(ev));
           })
      .def("scaling_factors", &Controller::scaling_factors)
      .def("record_collective_round",
           [](Controller& c, uint32_t gi, const std::vector<std::string>& ids, int64_t s, int64_t e,
              int64_t as, int64_t ae, const std::vector<py::bytes>& meta,
              const std::vector<uint64_t>& zeros, const std::vector<uint64_t>& sizes,
              const std::vector<uint64_t>& lengths) {
             std::vector<std::string> mm;
             for (auto& b : meta) mm.emplace_back(b);
             c.record_collective_round(gi, ids, s, e, as, ae, mm, zeros, sizes, lengths);
           })
      .def("record_community_evaluation",
           [](Controller& c, uint32_t gi, const std::vector<std::string>& ids, const std::vector<py::bytes>& evs) {
             std::vector<std::string> ee;
             for (auto& b : evs) ee.emplace_back(b);
             c.record_community_evaluation(gi, ids, ee);
           })
      .def("community_model", [](const Controller& c) { return B(c.community_model()); })
      .def("participating_learners", [](const Controller& c) { return B(c.participating_learners()); })
      .def("runtime_metadata_lineage",
           [](const Controller& c, int n) { return B(c.runtime_metadata_lineage(n)); })
      .def("community_evaluation_lineage",
           [](const Controller& c, int n) { return B(c.community_evaluation_lineage(n)); })
      .def("local_task_lineage",
           [](const Controller& c, int n, const std::vector<std::string>& ids) {
             return B(c.local_task_lineage(n, ids));
           })
      .def("community_model_lineage",
           [](const Controller& c, int n) { return B(c.community_model_lineage(n)); })
      .def("learner_local_model_lineage",
           [](Controller& c, int n, const std::vector<py::bytes>& ses) {
             std::vector<std::string> s;
             for (auto& b : ses) s.emplace_back(b);
             std::string out;
             {
               py::gil_scoped_release nogil;
               out = c.learner_local_model_lineage(n, s);
             }
             return B(out);
           })
      .def("config", [](const Controller& c) {
        const auto& k = c.config();
        py::dict d;
        d["hostname"] = k.hostname;
        d["port"] = k.port;
        d["rule"] = k.rule;
        d["stride_length"] = k.stride_length;
        d["scaling"] = k.scaling;
        d["protocol"] = k.protocol;
        d["semi_sync_lambda"] = k.semi_sync_lambda;
        d["semi_sync_recompute"] = k.semi_sync_recompute;
        d["lineage"] = k.lineage;
        d["redis"] = k.redis;
        d["batch_size"] = k.batch_size;
        d["epochs"] = k.epochs;
        d["he_batch_size"] = k.he_batch_size;
        d["he_scaling_bits"] = k.he_scaling_bits;
        return d;
      });

  m.def("scaling_factors",
        [](int kind, size_t n_all, const std::vector<std::string>& ids,
           const std::vector<double>& ntrain, const std::vector<double>& batches) {
          std::vector<ScalerInput> parts;
          for (size_t i = 0; i < ids.size(); ++i) parts.push_back({ids[i], ntrain[i], batches[i]});
          return compute_scaling_factors(kind, n_all, parts);
        });
  m.def("set_device_aggregation", &DeviceAggregator::set_enabled, py::arg("enabled"),
        py::arg("min_bytes") = -1,
        "Process-wide switch of the controller's device aggregation backend.");
  m.def("device_aggregation_available", [] {
    py::gil_scoped_release nogil;
    return DeviceAggregator::get() != nullptr;
  });
  m.def("device_aggregation_stats", [] {
    py::dict d;
    auto* a = DeviceAggregator::peek();
    d["available"] = a != nullptr;
    if (!a) return d;
    const DeviceAggStats s = a->stats();
    d["device"] = s.device;
    d["device_name"] = s.device_name;
    d["staged_models"] = s.staged_models;
    d["staged_bytes"] = s.staged_bytes;
    d["resident_bytes"] = s.resident_bytes;
    d["resident_hits"] = s.resident_hits;
    d["cold_uploads"] = s.cold_uploads;
    d["fedavg_calls"] = s.fedavg_calls;
    d["rolling_calls"] = s.rolling_calls;
    d["pwa_calls"] = s.pwa_calls;
    d["last_kernel_ms"] = s.last_kernel_ms;
    d["last_total_ms"] = s.last_total_ms;
    d["last_upload_ms"] = s.last_upload_ms;
    d["last_download_ms"] = s.last_download_ms;
    return d;
  });
  // TFRecord container I/O (datasets/tfrecord.py builds tf.train.Example on top)
  m.def("crc32c", [](py::bytes b) {
    std::string_view s = b;
    return crc32c(s.data(), s.size());
  });
  m.def("tfrecord_read", [](const std::string& path, bool verify) {
    std::vector<std::string> recs;
    {
      py::gil_scoped_release nogil;
      recs = tfrecord_read(path, verify);
    }
    py::list out;
    for (auto& r : recs) out.append(py::bytes(r));
    return out;
  }, py::arg("path"), py::arg("verify") = true);
  m.def("tfrecord_write", [](const std::string& path, const std::vector<py::bytes>& records, bool append) {
    std::vector<std::string_view> v;
    for (auto& r : records) v.emplace_back(r);  // views into the caller's bytes objects
    py::gil_scoped_release nogil;
    tfrecord_write(path, v, append);
  }, py::arg("path"), py::arg("records"), py::arg("append") = false);
  // Benchmark / test helper: models parsed and staged exactly like
  // Controller::learner_completed_task does, then aggregated in place.
  py::class_<StagedModels>(m, "StagedModels")
      .def(py::init<const std::vector<std::string>&, const std::vector<std::string>&>(),
           py::arg("ids"), py::arg("models"))
      .def("aggregate", &StagedModels::aggregate, py::arg("rule"), py::arg("weights"),
           py::arg("stride") = 0)
      .def_readonly("last_aggregate_ms", &StagedModels::last_aggregate_ms);
  m.def("aggregate_models", &aggregate_models, py::arg("rule"), py::arg("models"),
        py::arg("weights"), py::arg("stride") = 0);
  py::class_<PyRecency>(m, "FedRec").def(py::init<>()).def("aggregate", &PyRecency::aggregate);
  m.def("quantify_model", [](py::bytes model) {
    auto mm = parse_model(std::string(model));
    py::list out;
    for (auto& v : mm.vars) {
      auto q = quantify(v.t);
      out.append(py::make_tuple(q.non_zeros, q.zeros, q.size_bytes));
    }
    return out;
  });
  // Checkpoint writers that run with the GIL released (parallel/checkpoint.py:
  // a background writer thread must not starve the training thread's launch
  // loop): the community model as a serialized FederatedModel, and tensors
  // in the safetensors layout (8-byte little-endian header length, JSON
  // header, raw little-endian data), read back with safetensors' own loader.
  m.def("write_federated_model", [](const std::string& path, py::buffer flat, const std::vector<std::string>& names,
                                    const std::vector<std::vector<int64_t>>& shapes,
                                    const std::vector<int64_t>& offsets, const std::vector<bool>& trainable,
                                    uint32_t num_contributors, uint32_t global_iteration) {
    py::buffer_info bi = flat.request();
    if (bi.itemsize != 4 || bi.format != py::format_descriptor<float>::format())
      throw std::invalid_argument("write_federated_model: float32 buffer expected");
    const float* base = static_cast<const float*>(bi.ptr);
    const int64_t n = bi.size;
    if (names.size() != shapes.size() || names.size() != offsets.size() || names.size() != trainable.size())
      throw std::invalid_argument("write_federated_model: ragged variable lists");
    py::gil_scoped_release nogil;
    FederatedModelT fm;
    fm.num_contributors = num_contributors;
    fm.global_iteration = global_iteration;
    fm.model.vars.resize(names.size());
    for (size_t i = 0; i < names.size(); ++i) {
      VariableT& v = fm.model.vars[i];
      v.name = names[i];
      v.trainable = trainable[i];
      int64_t numel = 1;
      for (int64_t d : shapes[i]) numel *= d;
      if (offsets[i] < 0 || offsets[i] + numel > n) throw std::out_of_range("variable outside the flat buffer");
      v.t.length = (uint32_t)numel;
      v.t.dims = shapes[i];
      v.t.dtype = DT_FLOAT32;
      v.t.byte_order = BO_LITTLE;
      v.t.value.assign(reinterpret_cast<const char*>(base + offsets[i]), (size_t)numel * 4);
    }
    const std::string bytes = serialize_federated_model(fm);
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot open " + tmp);
    const size_t w = std::fwrite(bytes.data(), 1, bytes.size(), f);
    if (std::fclose(f) != 0 || w != bytes.size()) throw std::runtime_error("short write " + tmp);
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename " + tmp);
  });
  m.def("write_safetensors", [](const std::string& path, const std::vector<std::string>& names,
                                const std::vector<py::buffer>& bufs, const std::vector<std::string>& dtypes,
                                const std::vector<std::vector<int64_t>>& shapes) {
    if (names.size() != bufs.size() || names.size() != dtypes.size() || names.size() != shapes.size())
      throw std::invalid_argument("write_safetensors: ragged lists");
    std::vector<std::pair<const char*, size_t>> data;
    std::string header = "{";
    size_t off = 0;
    for (size_t i = 0; i < names.size(); ++i) {
      py::buffer_info bi = bufs[i].request();
      const size_t nb = (size_t)bi.size * (size_t)bi.itemsize;
      data.emplace_back(static_cast<const char*>(bi.ptr), nb);
      if (i) header += ",";
      header += "\"" + names[i] + "\":{\"dtype\":\"" + dtypes[i] + "\",\"shape\":[";
      for (size_t k = 0; k < shapes[i].size(); ++k) header += (k ? "," : "") + std::to_string(shapes[i][k]);
      header += "],\"data_offsets\":[" + std::to_string(off) + "," + std::to_string(off + nb) + "]}";
      off += nb;
    }
    header += "}";
    while (header.size() % 8) header += " ";  // 8-byte aligned data section
    py::gil_scoped_release nogil;
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot open " + tmp);
    const uint64_t hl = header.size();
    bool ok = std::fwrite(&hl, 8, 1, f) == 1 && std::fwrite(header.data(), 1, header.size(), f) == header.size();
    for (auto& [p, nb] : data) ok = ok && (nb == 0 || std::fwrite(p, 1, nb, f) == nb);
    if (std::fclose(f) != 0 || !ok) throw std::runtime_error("short write " + tmp);
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("rename " + tmp);
  });
  m.def("roundtrip_model", [](py::bytes model) {
    return B(serialize_model(parse_model(std::string(model))));
  });

  // RFC 8439 block function (known-answer tests; same code as the device side)
  m.def("chacha20_block", [](py::bytes key, uint32_t counter, py::bytes nonce) {
    const std::string k = key, n = nonce;
    if (k.size() != 32 || n.size() != 12) throw std::invalid_argument("key 32 bytes, nonce 12 bytes");
    uint32_t kw[8], nw[3], out[16];
    std::memcpy(kw, k.data(), 32);
    std::memcpy(nw, n.data(), 12);
    chacha20_block(kw, counter, nw, out);
    return py::bytes(reinterpret_cast<const char*>(out), 64);
  });
  py::class_<CKKS>(m, "CKKS")
      .def(py::init<uint32_t, uint32_t>(), py::arg("batch_size"), py::arg("scaling_factor_bits"))
      .def("gen_crypto_context_and_keys", &CKKS::gen_crypto_context_and_keys,
           py::call_guard<py::gil_scoped_release>())
      .def("get_crypto_params_files",
           [](const CKKS& c) {
             auto f = c.files();
             py::dict d;
             d["crypto_context_file"] = f.crypto_context_file;
             d["public_key_file"] = f.public_key_file;
             d["private_key_file"] = f.private_key_file;
             d["eval_mult_key_file"] = f.eval_mult_key_file;
             return d;
           })
      .def("load_crypto_context_from_file", &CKKS::load_context)
      .def("load_public_key_from_file", &CKKS::load_public_key)
      .def("load_private_key_from_file", &CKKS::load_private_key)
      .def("load_context_and_keys_from_files", &CKKS::load_context_and_keys)
      .def("encrypt",
           [](CKKS& c, py::array_t<double, py::array::c_style | py::array::forcecast> a) {
             std::vector<double> v(a.data(), a.data() + a.size());
             std::string ct;
             {
               py::gil_scoped_release nogil;
               ct = c.encrypt(v);
             }
             return B(ct);
           })
      .def("compute_weighted_average",
           [](const CKKS& c, const std::vector<py::bytes>& cts, const std::vector<double>& w) {
             std::vector<std::string> owned;
             for (auto& b : cts) owned.emplace_back(b);
             std::vector<std::string_view> views(owned.begin(), owned.end());
             std::string out;
             {
               py::gil_scoped_release nogil;
               out = c.weighted_average(views, w);
             }
             return B(out);
           })
      .def("decrypt",
           [](const CKKS& c, py::bytes ct, size_t n) {
             std::string s(ct);
             std::vector<double> v;
             {
               py::gil_scoped_release nogil;
               v = c.decrypt(s, n);
             }
             return py::array_t<double>(v.size(), v.data());
           })
      .def("encode_decode_roundtrip", &CKKS::encode_decode_roundtrip)
      .def("debug_sample", &CKKS::debug_sample, py::arg("kind"), py::arg("n"),
           "sampler output for statistical tests: 0 ternary secret, 1 Gaussian error, 2 uniform mod q_0")
      .def_property_readonly("ring_dim", &CKKS::ring_dim)
      .def_property_readonly("slots", &CKKS::slots)
      .def_property_readonly("moduli", &CKKS::moduli)
      .def_property_readonly("scaling_bits", &CKKS::scaling_bits)
      .def("device_tables",
           [](const CKKS& c) {
             // flat numpy copies of everything the HIP encrypt / decrypt path
             // needs (encryption/device.py uploads them once)
             auto u64 = [](const std::vector<uint64_t>& v) {
               return py::array_t<uint64_t>(v.size(), v.data());
             };
             auto u64_2d = [](const std::vector<std::vector<uint64_t>>& v) {
               std::vector<uint64_t> flat;
               for (auto& r : v) flat.insert(flat.end(), r.begin(), r.end());
               return py::array_t<uint64_t>(flat.size(), flat.data());
             };
             py::dict d;
             d["moduli"] = u64(c.moduli());
             d["psi"] = u64_2d(c.psi_rev());
             d["psi_shoup"] = u64_2d(c.psi_rev_shoup());
             d["ipsi"] = u64_2d(c.ipsi_rev());
             d["ipsi_shoup"] = u64_2d(c.ipsi_rev_shoup());
             d["n_inv"] = u64(c.n_inv());
             d["n_inv_shoup"] = u64(c.n_inv_shoup());
             d["rot"] = u64(c.rot());
             d["ksi_re"] = py::array_t<double>(c.ksi_re().size(), c.ksi_re().data());
             d["ksi_im"] = py::array_t<double>(c.ksi_im().size(), c.ksi_im().data());
             if (c.has_public_key()) {
               d["pk_b"] = u64(c.pk_b());
               d["pk_a"] = u64(c.pk_a());
             }
             if (c.has_private_key()) d["sk"] = u64(c.sk());
             return d;
           });
}
