// TFRecord container I/O (the on-disk format of tf.data.TFRecordDataset /
// tf.io.TFRecordWriter that the reference's neuroimaging example uses,
// examples/keras/neuroimaging.py:96-128, 219-225):
//
//   uint64 length | uint32 masked_crc32c(length) | byte data[length] | uint32 masked_crc32c(data)
//
// little-endian, masked crc = ((crc >> 15) | (crc << 17)) + 0xa282ead8.
// CRC32C runs on the SSE4.2 crc32 instruction (8 B per step) when the CPU has
// it, a slicing table otherwise.  Reads are one pass over an mmap of the file.
#pragma once
#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace mfl {

uint32_t crc32c(const void* data, size_t n, uint32_t crc = 0);
inline uint32_t masked_crc32c(const void* data, size_t n) {
  const uint32_t c = crc32c(data, n);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// Every record of `path`; throws on truncation or (verify) a CRC mismatch.
std::vector<std::string> tfrecord_read(const std::string& path, bool verify = true);
void tfrecord_write(const std::string& path, const std::vector<std::string_view>& records, bool append = false);

}  // namespace mfl
