// Launch interface between the host-side device aggregator (device_agg.cc,
// g++ + OpenMP) and its kernels (device_agg_kernels.hip, hipcc gfx950).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace mfl {
namespace devagg {

constexpr int kMaxModels = 32;          // inputs per launch (more: accumulate launches)
constexpr uint32_t kTileBytes = 16384;  // 256 lanes x 16 B x 4
constexpr uint64_t kAlign = 256;        // variable alignment inside a packed model

struct Tile {
  uint64_t off;    // byte offset of the tile inside the packed model
  uint32_t n;      // elements
  uint32_t dtype;  // DTypeCode
};

struct WSumArgs {
  const char* x[kMaxModels];
  double w[kMaxModels];
  int count;
};

struct PwaArgs {
  const uint64_t* ct[kMaxModels];
  int count;
  int first;  // index of ct[0] in the weight table
};

enum RollOp { ROLL_ADD = 0, ROLL_SUB = 1, ROLL_MUL = 2, ROLL_DIV = 3, ROLL_COPY = 4 };

int launch_wsum(char* out, const Tile* tiles, int ntiles, const WSumArgs& a, bool accumulate,
                hipStream_t s);
int launch_roll(char* y, const char* x, const Tile* tiles, int ntiles, double w, int op,
                hipStream_t s);
int launch_pwa(const PwaArgs& a, const uint64_t* wtab, const uint64_t* q, uint64_t* out, uint32_t L,
               uint32_t N, uint64_t total, bool accumulate, hipStream_t s);

}  // namespace devagg
}  // namespace mfl
