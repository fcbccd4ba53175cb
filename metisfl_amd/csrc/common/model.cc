#include "common/model.h"

#include <atomic>

#include <algorithm>
#include <stdexcept>

#include "common/wire.h"

namespace mfl {

size_t dtype_size(int dt) {
  switch (dt) {
    case DT_INT8: case DT_UINT8: return 1;
    case DT_INT16: case DT_UINT16: return 2;
    case DT_INT32: case DT_UINT32: case DT_FLOAT32: return 4;
    case DT_INT64: case DT_UINT64: case DT_FLOAT64: return 8;
    default: throw std::runtime_error("unsupported tensor dtype");
  }
}

size_t ModelT::byte_size() const {
  size_t n = 0;
  for (auto& v : vars) n += v.t.value.size();
  return n;
}

TensorT parse_tensor_spec(std::string_view bytes) {
  wire::WireMsg m(bytes);
  TensorT t;
  t.length = (uint32_t)m.u64(1);
  t.dims = m.i64s(2);
  wire::WireMsg dt = m.msg(3);
  t.dtype = (int)dt.u64(1);
  t.byte_order = (int)dt.u64(2);
  t.fortran_order = dt.b(3);
  t.value = m.str(4);
  const size_t es = dtype_size(t.dtype);
  if (t.byte_order == BO_BIG && es > 1) {
    for (size_t i = 0; i + es <= t.value.size(); i += es) std::reverse(&t.value[i], &t.value[i] + es);
    t.byte_order = BO_LITTLE;
  }
  return t;
}

std::string serialize_tensor_spec(const TensorT& t) {
  wire::Writer w;
  w.u64(1, t.length);
  w.packed_i64(2, t.dims);
  wire::Writer dt;
  dt.u64(1, (uint64_t)t.dtype);
  dt.u64(2, (uint64_t)(dtype_size(t.dtype) == 1 ? t.byte_order : BO_LITTLE));
  dt.boolean(3, t.fortran_order);
  w.msg(3, dt);
  w.bytes(4, t.value);
  return w.take();
}

VariableT parse_variable(std::string_view bytes) {
  wire::WireMsg vm(bytes);
  VariableT v;
  v.name = vm.str(1);
  v.trainable = vm.b(2);
  if (vm.has(3)) {
    v.ciphertext = false;
    v.t = parse_tensor_spec(vm.msg(3).bytes(1));
  } else if (vm.has(4)) {
    v.ciphertext = true;
    v.t = parse_tensor_spec(vm.msg(4).bytes(1));
  }
  return v;
}

std::string serialize_variable(const VariableT& v) {
  wire::Writer vw;
  vw.bytes(1, v.name);
  vw.boolean(2, v.trainable);
  wire::Writer tw;
  tw.bytes(1, serialize_tensor_spec(v.t), true);
  vw.msg(v.ciphertext ? 4 : 3, tw);
  return vw.take();
}

ModelT parse_model(std::string_view bytes) {
  static std::atomic<uint64_t> next_uid{1};
  wire::WireMsg m(bytes);
  ModelT out;
  for (auto sv : m.strs(1)) out.vars.push_back(parse_variable(sv));
  out.uid = next_uid.fetch_add(1, std::memory_order_relaxed);
  return out;
}

std::string serialize_model(const ModelT& m) {
  wire::Writer w;
  for (auto& v : m.vars) w.bytes(1, serialize_variable(v), true);
  return w.take();
}

FederatedModelT parse_federated_model(std::string_view bytes) {
  wire::WireMsg m(bytes);
  FederatedModelT fm;
  fm.num_contributors = (uint32_t)m.u64(1);
  fm.global_iteration = (uint32_t)m.u64(2);
  fm.model = parse_model(m.bytes(3));
  return fm;
}

std::string serialize_federated_model(const FederatedModelT& fm) {
  wire::Writer w;
  w.u64(1, fm.num_contributors);
  w.u64(2, fm.global_iteration);
  w.bytes(3, serialize_model(fm.model), true);
  return w.take();
}

template <typename T>
static void count_zeros_t(const std::string& v, uint64_t& z) {
  const T* p = reinterpret_cast<const T*>(v.data());
  const size_t n = v.size() / sizeof(T);
  uint64_t c = 0;
  for (size_t i = 0; i < n; ++i) c += (p[i] == T(0));
  z = c;
}

Quantifier quantify(const TensorT& t) {
  Quantifier q;
  q.size_bytes = t.value.size();
  uint64_t z = 0;
  switch (t.dtype) {
    case DT_INT8: count_zeros_t<int8_t>(t.value, z); break;
    case DT_INT16: count_zeros_t<int16_t>(t.value, z); break;
    case DT_INT32: count_zeros_t<int32_t>(t.value, z); break;
    case DT_INT64: count_zeros_t<int64_t>(t.value, z); break;
    case DT_UINT8: count_zeros_t<uint8_t>(t.value, z); break;
    case DT_UINT16: count_zeros_t<uint16_t>(t.value, z); break;
    case DT_UINT32: count_zeros_t<uint32_t>(t.value, z); break;
    case DT_UINT64: count_zeros_t<uint64_t>(t.value, z); break;
    case DT_FLOAT32: count_zeros_t<float>(t.value, z); break;
    case DT_FLOAT64: count_zeros_t<double>(t.value, z); break;
    default: break;
  }
  q.zeros = z;
  q.non_zeros = t.length >= z ? t.length - z : 0;
  return q;
}

bool same_structure(const ModelT& a, const ModelT& b) {
  if (a.vars.size() != b.vars.size()) return false;
  for (size_t i = 0; i < a.vars.size(); ++i) {
    if (a.vars[i].t.dtype != b.vars[i].t.dtype) return false;
    if (a.vars[i].t.value.size() != b.vars[i].t.value.size()) return false;
  }
  return true;
}

}  // namespace mfl
