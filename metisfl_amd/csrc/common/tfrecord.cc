#include "common/tfrecord.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace mfl {
namespace {

struct Table {
  uint32_t t[8][256];
  Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};

uint32_t crc_sw(const uint8_t* p, size_t n, uint32_t c) {
  static const Table T;
  while (n >= 8) {  // slicing-by-8
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= c;
    c = T.t[7][v & 0xff] ^ T.t[6][(v >> 8) & 0xff] ^ T.t[5][(v >> 16) & 0xff] ^
        T.t[4][(v >> 24) & 0xff] ^ T.t[3][(v >> 32) & 0xff] ^ T.t[2][(v >> 40) & 0xff] ^
        T.t[1][(v >> 48) & 0xff] ^ T.t[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ T.t[0][(c ^ *p++) & 0xff];
  return c;
}

__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n, uint32_t c) {
  uint64_t c64 = c;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c64 = __builtin_ia32_crc32di(c64, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c64;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return c32;
}

uint32_t load_u32(const char* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

}  // namespace

uint32_t crc32c(const void* data, size_t n, uint32_t crc) {
  static const bool hw = __builtin_cpu_supports("sse4.2");
  const uint8_t* p = static_cast<const uint8_t*>(data);
  crc = ~crc;
  crc = hw ? crc_hw(p, n, crc) : crc_sw(p, n, crc);
  return ~crc;
}

std::vector<std::string> tfrecord_read(const std::string& path, bool verify) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("tfrecord: cannot open " + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    throw std::runtime_error("tfrecord: cannot stat " + path);
  }
  const size_t size = (size_t)st.st_size;
  std::vector<std::string> out;
  if (size == 0) {
    ::close(fd);
    return out;
  }
  void* m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) throw std::runtime_error("tfrecord: cannot map " + path);
  madvise(m, size, MADV_SEQUENTIAL);
  const char* p = static_cast<const char*>(m);
  size_t off = 0;
  try {
    while (off < size) {
      if (size - off < 12) throw std::runtime_error("tfrecord: truncated record header in " + path);
      uint64_t len;
      std::memcpy(&len, p + off, 8);
      if (verify && masked_crc32c(p + off, 8) != load_u32(p + off + 8))
        throw std::runtime_error("tfrecord: corrupted length at offset " + std::to_string(off));
      off += 12;
      if (len > size - off || size - off - len < 4)
        throw std::runtime_error("tfrecord: truncated record data in " + path);
      if (verify && masked_crc32c(p + off, len) != load_u32(p + off + len))
        throw std::runtime_error("tfrecord: corrupted data at offset " + std::to_string(off));
      out.emplace_back(p + off, len);
      off += len + 4;
    }
  } catch (...) {
    munmap(m, size);
    throw;
  }
  munmap(m, size);
  return out;
}

void tfrecord_write(const std::string& path, const std::vector<std::string_view>& records, bool append) {
  FILE* f = std::fopen(path.c_str(), append ? "ab" : "wb");
  if (!f) throw std::runtime_error("tfrecord: cannot open " + path + " for writing");
  bool ok = true;
  for (auto r : records) {
    char hdr[12];
    const uint64_t len = r.size();
    std::memcpy(hdr, &len, 8);
    const uint32_t lc = masked_crc32c(hdr, 8);
    std::memcpy(hdr + 8, &lc, 4);
    const uint32_t dc = masked_crc32c(r.data(), r.size());
    ok = ok && std::fwrite(hdr, 1, 12, f) == 12;
    ok = ok && std::fwrite(r.data(), 1, r.size(), f) == r.size();
    ok = ok && std::fwrite(&dc, 1, 4, f) == 4;
  }
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error("tfrecord: write failed for " + path);
}

}  // namespace mfl
