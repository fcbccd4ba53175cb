#include "engine/store.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstring>
#include <stdexcept>

namespace mfl {

// ---------------------------------------------------------------------------
void HashMapModelStore::insert(const std::string& learner, ModelT model) {
  auto& lin = cache_[learner];
  if (lineage_ > 0 && (int)lin.size() >= lineage_) lin.erase(lin.begin());
  lin.push_back(std::move(model));
}

std::map<std::string, std::vector<const ModelT*>> HashMapModelStore::select(
    const std::vector<std::pair<std::string, int>>& req) {
  std::map<std::string, std::vector<const ModelT*>> out;
  for (auto& [id, k0] : req) {
    auto& lin = cache_[id];
    const int size = (int)lin.size();
    int k = k0;
    auto& dst = out[id];
    if (k > size) continue;
    if (k <= 0) k = size;
    for (int h = k; h > 0; --h) dst.push_back(&lin[size - h]);
  }
  return out;
}

int HashMapModelStore::lineage_length(const std::string& learner) {
  auto it = cache_.find(learner);
  return it == cache_.end() ? 0 : (int)it->second.size();
}

void HashMapModelStore::erase(const std::vector<std::string>& learners) {
  for (auto& l : learners) cache_.erase(l);
}

void HashMapModelStore::expunge() { cache_.clear(); }

// ---------------------------------------------------------------------------
RespClient::RespClient(const std::string& host, int port, double timeout_s) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  const std::string ps = std::to_string(port);
  if (getaddrinfo(host.c_str(), ps.c_str(), &hints, &res) != 0 || !res)
    throw std::runtime_error("redis: cannot resolve " + host);
  for (addrinfo* p = res; p; p = p->ai_next) {
    fd_ = ::socket(p->ai_family, p->ai_socktype, p->ai_protocol);
    if (fd_ < 0) continue;
    timeval tv{(time_t)timeout_s, (suseconds_t)((timeout_s - (long)timeout_s) * 1e6)};
    setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    int one = 1;
    setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    if (::connect(fd_, p->ai_addr, p->ai_addrlen) == 0) break;
    ::close(fd_);
    fd_ = -1;
  }
  freeaddrinfo(res);
  if (fd_ < 0) throw std::runtime_error("redis: cannot connect to " + host + ":" + ps);
  // generous timeout for large transfers once connected
  timeval tv{60, 0};
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

RespClient::~RespClient() {
  if (fd_ >= 0) ::close(fd_);
}

void RespClient::send_all(const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t n = ::send(fd_, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n <= 0) throw std::runtime_error("redis: send failed");
    off += (size_t)n;
  }
}

std::string RespClient::read_n(size_t n) {
  while (buf_.size() < n) {
    char tmp[1 << 16];
    const ssize_t r = ::recv(fd_, tmp, sizeof(tmp), 0);
    if (r <= 0) throw std::runtime_error("redis: connection closed");
    buf_.append(tmp, (size_t)r);
  }
  std::string out = buf_.substr(0, n);
  buf_.erase(0, n);
  return out;
}

std::string RespClient::read_line() {
  size_t pos;
  while ((pos = buf_.find("\r\n")) == std::string::npos) {
    char tmp[1 << 16];
    const ssize_t r = ::recv(fd_, tmp, sizeof(tmp), 0);
    if (r <= 0) throw std::runtime_error("redis: connection closed");
    buf_.append(tmp, (size_t)r);
  }
  std::string line = buf_.substr(0, pos);
  buf_.erase(0, pos + 2);
  return line;
}

RespClient::Reply RespClient::read_reply() {
  Reply r;
  const std::string line = read_line();
  if (line.empty()) throw std::runtime_error("redis: empty reply");
  r.type = line[0];
  const std::string body = line.substr(1);
  switch (r.type) {
    case '+': r.str = body; break;
    case '-': r.str = body; break;
    case ':': r.integer = std::stoll(body); break;
    case '$': {
      const long long n = std::stoll(body);
      if (n < 0) {
        r.nil = true;
      } else {
        r.str = read_n((size_t)n);
        read_n(2);
      }
      break;
    }
    case '*': {
      const long long n = std::stoll(body);
      if (n < 0) {
        r.nil = true;
      } else {
        for (long long i = 0; i < n; ++i) r.elems.push_back(read_reply());
      }
      break;
    }
    default: throw std::runtime_error("redis: bad reply type");
  }
  return r;
}

RespClient::Reply RespClient::command(const std::vector<std::string>& args) {
  std::string msg = "*" + std::to_string(args.size()) + "\r\n";
  for (auto& a : args) {
    msg += "$" + std::to_string(a.size()) + "\r\n";
    msg += a;
    msg += "\r\n";
  }
  send_all(msg);
  Reply r = read_reply();
  if (r.type == '-') throw std::runtime_error("redis error: " + r.str);
  return r;
}

// ---------------------------------------------------------------------------
RedisModelStore::RedisModelStore(int lineage_length, const std::string& host, int port)
    : ModelStore(lineage_length), redis_(new RespClient(host, port)) {
  redis_->command({"PING"});
}

RedisModelStore::~RedisModelStore() = default;

void RedisModelStore::insert(const std::string& learner, ModelT model) {
  std::lock_guard<std::mutex> g(mu_);
  auto& keys = keys_[learner];
  if (lineage_ > 0 && (int)keys.size() >= lineage_) {
    redis_->command({"DEL", keys.front()});
    cache_.erase(keys.front());
    keys.erase(keys.begin());
  }
  const std::string key = learner + "_" + std::to_string(counter_[learner]++);
  // one variable per list element (scales to large models, pipelined)
  std::vector<std::string> args{"RPUSH", key};
  for (auto& v : model.vars) args.push_back(serialize_variable(v));
  if (args.size() > 2) redis_->command(args);
  keys.push_back(key);
}

std::map<std::string, std::vector<const ModelT*>> RedisModelStore::select(
    const std::vector<std::pair<std::string, int>>& req) {
  std::lock_guard<std::mutex> g(mu_);
  std::map<std::string, std::vector<const ModelT*>> out;
  for (auto& [id, k0] : req) {
    auto& keys = keys_[id];
    auto& dst = out[id];
    const int size = (int)keys.size();
    int k = k0;
    if (k > size) continue;
    if (k <= 0) k = size;
    for (int h = k; h > 0; --h) {
      const std::string& key = keys[size - h];
      auto it = cache_.find(key);
      if (it == cache_.end()) {
        auto rep = redis_->command({"LRANGE", key, "0", "-1"});
        ModelT m;
        for (auto& e : rep.elems) m.vars.push_back(parse_variable(e.str));
        it = cache_.emplace(key, std::move(m)).first;
      }
      dst.push_back(&it->second);
    }
  }
  return out;
}

int RedisModelStore::lineage_length(const std::string& learner) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = keys_.find(learner);
  return it == keys_.end() ? 0 : (int)it->second.size();
}

void RedisModelStore::erase(const std::vector<std::string>& learners) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& l : learners) {
    for (auto& k : keys_[l]) {
      redis_->command({"DEL", k});
      cache_.erase(k);
    }
    keys_.erase(l);
  }
}

void RedisModelStore::expunge() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& [l, ks] : keys_)
    for (auto& k : ks) redis_->command({"DEL", k});
  keys_.clear();
  cache_.clear();
}

void RedisModelStore::reset_state() {
  std::lock_guard<std::mutex> g(mu_);
  cache_.clear();
}

}  // namespace mfl
