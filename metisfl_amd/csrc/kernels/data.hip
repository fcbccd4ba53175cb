// Device-resident data pipeline: gathers one mini-batch of a learner's shard
// through a per-epoch permutation.  The step counter is read from device
// memory, so the gather sits inside the captured training-step hipGraph and
// the host never touches the data path (the reference instead unpickles
// dataset recipes and re-loads .npz files per task: learner.py:173-182).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace mfl {

// One workgroup per sample; rows are copied in 16-B units.  xp (fp32 shards
// only, optional): also the packed bf16x3 split of the batch -- the stem
// convolution's operand on the bf16x3 fp32 path (no separate pack launch).
__global__ __launch_bounds__(256) void gather_kernel(const uint16_t* __restrict__ shard,
                                                     const int* __restrict__ labels,
                                                     const int* __restrict__ perm,
                                                     const int* __restrict__ step, int spe, int B,
                                                     int64_t row_vec, uint16_t* __restrict__ xb,
                                                     int* __restrict__ yb, uint32_t* __restrict__ xp) {
  const int b = blockIdx.x;
  const int s = step[0] % spe;
  const int src = perm[(int64_t)s * B + b];
  const uint4* in = reinterpret_cast<const uint4*>(shard) + (int64_t)src * row_vec;
  uint4* out = reinterpret_cast<uint4*>(xb) + (int64_t)b * row_vec;
  uint4* outp = reinterpret_cast<uint4*>(xp) + (int64_t)b * row_vec;
  for (int64_t i = threadIdx.x; i < row_vec; i += blockDim.x) {
    const uint4 v = in[i];
    out[i] = v;
    if (xp)  // uniform
      outp[i] = make_uint4(split_pack(__uint_as_float(v.x)), split_pack(__uint_as_float(v.y)),
                           split_pack(__uint_as_float(v.z)), split_pack(__uint_as_float(v.w)));
  }
  if (threadIdx.x == 0) yb[b] = labels[src];
}

void launch_gather_batch(const uint16_t* shard, const int* labels, const int* perm,
                         const int* step, int steps_per_epoch, int B, int64_t row_elems,
                         uint16_t* xb, int* yb, hipStream_t s, uint32_t* xp) {
  gather_kernel<<<B, 256, 0, s>>>(shard, labels, perm, step, steps_per_epoch, B, row_elems / 8, xb,
                                  yb, xp);
}

}  // namespace mfl
