// Minimal protobuf wire-format reader/writer for the native controller engine.
//
// The image has no C++ protobuf/gRPC, so the engine speaks the
// `metisfl` wire format directly: WireMsg indexes a serialized message by
// field number (zero-copy string_views into the caller's buffer) and Writer
// emits fields in ascending order.  Only the encodings the schema uses are
// supported: varint (0), fixed64 (1), length-delimited (2), fixed32 (5),
// including packed repeated scalars.
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace mfl::wire {

struct Field {
  int wt;             // wire type
  uint64_t u;         // varint / fixed payload
  std::string_view s; // length-delimited payload
};

inline uint64_t read_varint(const char*& p, const char* end) {
  uint64_t v = 0;
  int shift = 0;
  while (p < end) {
    const uint8_t b = static_cast<uint8_t>(*p++);
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return v;
    shift += 7;
    if (shift > 63) break;
  }
  throw std::runtime_error("malformed varint");
}

class WireMsg {
 public:
  WireMsg() = default;
  explicit WireMsg(std::string_view buf) { parse(buf); }

  void parse(std::string_view buf) {
    fields_.clear();
    const char* p = buf.data();
    const char* end = p + buf.size();
    while (p < end) {
      const uint64_t key = read_varint(p, end);
      const int fn = (int)(key >> 3);
      const int wt = (int)(key & 7);
      Field f{wt, 0, {}};
      switch (wt) {
        case 0: f.u = read_varint(p, end); break;
        case 1:
          if (end - p < 8) throw std::runtime_error("truncated fixed64");
          std::memcpy(&f.u, p, 8);
          p += 8;
          break;
        case 2: {
          const uint64_t n = read_varint(p, end);
          if ((uint64_t)(end - p) < n) throw std::runtime_error("truncated bytes field");
          f.s = std::string_view(p, n);
          p += n;
          break;
        }
        case 5: {
          if (end - p < 4) throw std::runtime_error("truncated fixed32");
          uint32_t v;
          std::memcpy(&v, p, 4);
          f.u = v;
          p += 4;
          break;
        }
        default: throw std::runtime_error("unsupported wire type");
      }
      fields_[fn].push_back(f);
    }
  }

  bool has(int fn) const { return fields_.count(fn) > 0; }
  const std::vector<Field>* all(int fn) const {
    auto it = fields_.find(fn);
    return it == fields_.end() ? nullptr : &it->second;
  }
  uint64_t u64(int fn, uint64_t def = 0) const {
    auto* v = all(fn);
    return v ? v->back().u : def;
  }
  int64_t i64(int fn, int64_t def = 0) const { return (int64_t)u64(fn, (uint64_t)def); }
  bool b(int fn) const { return u64(fn) != 0; }
  float f32(int fn, float def = 0.f) const {
    auto* v = all(fn);
    if (!v) return def;
    uint32_t x = (uint32_t)v->back().u;
    float f;
    std::memcpy(&f, &x, 4);
    return f;
  }
  double f64(int fn, double def = 0.0) const {
    auto* v = all(fn);
    if (!v) return def;
    double d;
    uint64_t x = v->back().u;
    std::memcpy(&d, &x, 8);
    return d;
  }
  std::string_view bytes(int fn) const {
    auto* v = all(fn);
    return v ? v->back().s : std::string_view();
  }
  std::string str(int fn) const { return std::string(bytes(fn)); }
  WireMsg msg(int fn) const { return WireMsg(bytes(fn)); }
  std::vector<WireMsg> msgs(int fn) const {
    std::vector<WireMsg> out;
    if (auto* v = all(fn))
      for (auto& f : *v) out.emplace_back(f.s);
    return out;
  }
  std::vector<std::string_view> strs(int fn) const {
    std::vector<std::string_view> out;
    if (auto* v = all(fn))
      for (auto& f : *v) out.push_back(f.s);
    return out;
  }
  // repeated int64 (packed or not)
  std::vector<int64_t> i64s(int fn) const {
    std::vector<int64_t> out;
    if (auto* v = all(fn))
      for (auto& f : *v) {
        if (f.wt == 2) {
          const char* p = f.s.data();
          const char* e = p + f.s.size();
          while (p < e) out.push_back((int64_t)read_varint(p, e));
        } else {
          out.push_back((int64_t)f.u);
        }
      }
    return out;
  }

 private:
  std::map<int, std::vector<Field>> fields_;
};

class Writer {
 public:
  void varint_raw(uint64_t v) {
    while (v >= 0x80) {
      buf_.push_back((char)((v & 0x7f) | 0x80));
      v >>= 7;
    }
    buf_.push_back((char)v);
  }
  void key(int fn, int wt) { varint_raw(((uint64_t)fn << 3) | (uint64_t)wt); }
  // proto3: default values are not emitted unless `force`
  void u64(int fn, uint64_t v, bool force = false) {
    if (!v && !force) return;
    key(fn, 0);
    varint_raw(v);
  }
  void i64(int fn, int64_t v, bool force = false) { u64(fn, (uint64_t)v, force); }
  void boolean(int fn, bool v) { u64(fn, v ? 1 : 0); }
  void f32(int fn, float v, bool force = false) {
    if (v == 0.f && !force) return;
    key(fn, 5);
    char b[4];
    std::memcpy(b, &v, 4);
    buf_.append(b, 4);
  }
  void f64(int fn, double v, bool force = false) {
    if (v == 0.0 && !force) return;
    key(fn, 1);
    char b[8];
    std::memcpy(b, &v, 8);
    buf_.append(b, 8);
  }
  void bytes(int fn, std::string_view s, bool force = false) {
    if (s.empty() && !force) return;
    key(fn, 2);
    varint_raw(s.size());
    buf_.append(s.data(), s.size());
  }
  void msg(int fn, const Writer& w, bool force = true) { bytes(fn, w.buf_, force); }
  void packed_i64(int fn, const std::vector<int64_t>& v) {
    if (v.empty()) return;
    Writer t;
    for (auto x : v) t.varint_raw((uint64_t)x);
    bytes(fn, t.buf_);
  }
  void packed_f64(int fn, const std::vector<double>& v) {
    if (v.empty()) return;
    std::string s(v.size() * 8, '\0');
    std::memcpy(&s[0], v.data(), s.size());
    bytes(fn, s);
  }
  // Timestamp from ns since epoch
  void timestamp(int fn, int64_t ns) {
    if (ns <= 0) return;
    Writer t;
    t.i64(1, ns / 1000000000LL);
    t.i64(2, ns % 1000000000LL);
    msg(fn, t);
  }
  // map<string, V> entries
  void map_str_msg(int fn, std::string_view k, const Writer& v) {
    Writer e;
    e.bytes(1, k, true);
    e.msg(2, v);
    msg(fn, e);
  }
  void map_str_bytes_msg(int fn, std::string_view k, std::string_view vbytes) {
    Writer e;
    e.bytes(1, k, true);
    e.bytes(2, vbytes, true);
    msg(fn, e);
  }
  void map_str_f64(int fn, std::string_view k, double v) {
    Writer e;
    e.bytes(1, k, true);
    e.f64(2, v, true);
    msg(fn, e);
  }
  void map_str_ts(int fn, std::string_view k, int64_t ns) {
    Writer e;
    e.bytes(1, k, true);
    e.timestamp(2, ns);
    msg(fn, e);
  }
  const std::string& str() const { return buf_; }
  std::string take() { return std::move(buf_); }
  void append_raw(std::string_view s) { buf_.append(s.data(), s.size()); }

 private:
  std::string buf_;
};

}  // namespace mfl::wire
