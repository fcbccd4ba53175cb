// Model stores of the controller engine (reference: metisfl/controller/store).
//
//  * HashMapModelStore: per-learner lineage of models kept in host memory,
//    oldest first, with NoEviction or LineageLength(k) eviction
//    (hash_map_model_store.cc:8-121).
//  * RedisModelStore: same lineage semantics, models kept in an external
//    Redis: key "<learner_id>_<counter>", one RPUSH'd serialized
//    Model.Variable per list element (redis_model_store.cc:60-241).  Speaks
//    RESP over a plain TCP socket (hiredis is not in the image) and fails
//    with an exception instead of exit(1) when Redis is unreachable.
//
// select(learner, k): the last k models, ascending commit order; k <= 0 ->
// all; k > lineage -> empty (reference semantics).
#pragma once
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common/model.h"

namespace mfl {

class ModelStore {
 public:
  explicit ModelStore(int lineage_length) : lineage_(lineage_length) {}
  virtual ~ModelStore() = default;
  virtual void insert(const std::string& learner, ModelT model) = 0;
  virtual std::map<std::string, std::vector<const ModelT*>> select(
      const std::vector<std::pair<std::string, int>>& req) = 0;
  virtual int lineage_length(const std::string& learner) = 0;
  virtual void erase(const std::vector<std::string>& learners) = 0;
  virtual void expunge() = 0;
  virtual void reset_state() {}
  virtual std::string name() const = 0;
  // <= 0 means no eviction
  int eviction_lineage() const { return lineage_; }

 protected:
  int lineage_;
};

class HashMapModelStore : public ModelStore {
 public:
  using ModelStore::ModelStore;
  void insert(const std::string& learner, ModelT model) override;
  std::map<std::string, std::vector<const ModelT*>> select(
      const std::vector<std::pair<std::string, int>>& req) override;
  int lineage_length(const std::string& learner) override;
  void erase(const std::vector<std::string>& learners) override;
  void expunge() override;
  std::string name() const override { return "InMemoryStore"; }

 private:
  std::map<std::string, std::vector<ModelT>> cache_;
};

class RespClient;

class RedisModelStore : public ModelStore {
 public:
  RedisModelStore(int lineage_length, const std::string& host, int port);
  ~RedisModelStore() override;
  void insert(const std::string& learner, ModelT model) override;
  std::map<std::string, std::vector<const ModelT*>> select(
      const std::vector<std::pair<std::string, int>>& req) override;
  int lineage_length(const std::string& learner) override;
  void erase(const std::vector<std::string>& learners) override;
  void expunge() override;
  void reset_state() override;
  std::string name() const override { return "RedisDBStore"; }

 private:
  std::unique_ptr<RespClient> redis_;
  std::map<std::string, std::vector<std::string>> keys_;  // learner -> model keys (oldest first)
  std::map<std::string, uint64_t> counter_;
  std::map<std::string, ModelT> cache_;                    // key -> parsed model (per selection)
  std::mutex mu_;
};

// Minimal RESP2 client (blocking TCP).
class RespClient {
 public:
  RespClient(const std::string& host, int port, double timeout_s = 1.5);
  ~RespClient();
  struct Reply {
    char type = 0;  // '+', '-', ':', '$', '*'
    long long integer = 0;
    std::string str;
    bool nil = false;
    std::vector<Reply> elems;
  };
  Reply command(const std::vector<std::string>& args);

 private:
  void send_all(const std::string& s);
  Reply read_reply();
  std::string read_line();
  std::string read_n(size_t n);
  int fd_ = -1;
  std::string buf_;
};

}  // namespace mfl
