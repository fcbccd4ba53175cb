// Host-side model representation of the native controller engine.
//
// Mirrors the `Model` / `TensorSpec` wire messages (model.proto) but keeps
// each variable's values as one contiguous little-endian byte buffer, so the
// aggregators work on raw arrays (the reference re-deserialises every tensor
// per aggregation step: proto_tensor_serde.h:14-32, federated_average.cc).
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace mfl {

enum DTypeCode {
  DT_INT8 = 0, DT_INT16 = 1, DT_INT32 = 2, DT_INT64 = 3, DT_UINT8 = 4, DT_UINT16 = 5,
  DT_UINT32 = 6, DT_UINT64 = 7, DT_FLOAT32 = 8, DT_FLOAT64 = 9
};
enum ByteOrderCode { BO_NA = 0, BO_BIG = 1, BO_LITTLE = 2 };

size_t dtype_size(int dt);

struct TensorT {
  uint32_t length = 0;
  std::vector<int64_t> dims;
  int dtype = DT_FLOAT32;
  int byte_order = BO_LITTLE;
  bool fortran_order = false;
  std::string value;  // native (little-endian) bytes, length * dtype_size
};

struct VariableT {
  std::string name;
  bool trainable = true;
  bool ciphertext = false;
  TensorT t;
};

struct ModelT {
  std::vector<VariableT> vars;
  // process-unique identity, assigned when a model is parsed: a device-staged
  // copy is matched by (uid, buffer addresses), so a later model that the
  // allocator places at a freed model's addresses never aliases its slot
  uint64_t uid = 0;
  size_t byte_size() const;
  bool empty() const { return vars.empty(); }
};

struct FederatedModelT {
  uint32_t num_contributors = 0;
  uint32_t global_iteration = 0;
  ModelT model;
};

struct Quantifier {
  uint64_t non_zeros = 0, zeros = 0, size_bytes = 0;
};

VariableT parse_variable(std::string_view bytes);
std::string serialize_variable(const VariableT& v);
ModelT parse_model(std::string_view bytes);
std::string serialize_model(const ModelT& m);
FederatedModelT parse_federated_model(std::string_view bytes);
std::string serialize_federated_model(const FederatedModelT& fm);
std::string serialize_tensor_spec(const TensorT& t);
TensorT parse_tensor_spec(std::string_view bytes);
Quantifier quantify(const TensorT& t);

// Shallow structural equality (same variable names / dtypes / lengths).
bool same_structure(const ModelT& a, const ModelT& b);

}  // namespace mfl
