// Device-resident data pipeline: gathers one mini-batch of a learner's shard
// through a per-epoch permutation.  The step counter is read from device
// memory, so the gather sits inside the captured training-step hipGraph and
// the host never touches the data path (the reference instead unpickles
// dataset recipes and re-loads .npz files per task: learner.py:173-182).
#include "kernels/common.h"
#include "kernels/launchers.h"

namespace mfl {

// `parts` workgroups per sample, each a contiguous slice of its row copied in
// 16-B units (one vector per thread at the CIFAR row sizes: the step -> perm
// -> row chain of dependent loads is paid once per thread, not once per
// loop trip of a single 256-thread workgroup per sample).  xp (fp32 shards
// only, optional): also the packed bf16x3 split of the batch -- the stem
// convolution's operand on the bf16x3 fp32 path (no separate pack launch).
__global__ __launch_bounds__(256) void gather_kernel(const uint16_t* __restrict__ shard,
                                                     const int* __restrict__ labels,
                                                     const int* __restrict__ perm,
                                                     const int* __restrict__ step, int spe, int B, int parts,
                                                     int64_t row_vec, uint16_t* __restrict__ xb,
                                                     int* __restrict__ yb, uint32_t* __restrict__ xp) {
  const int b = blockIdx.x / parts, part = blockIdx.x - b * parts;
  const int s = step[0] % spe;
  const int src = perm[(int64_t)s * B + b];
  const int64_t per = (row_vec + parts - 1) / parts;
  const int64_t beg = part * per, end = beg + per < row_vec ? beg + per : row_vec;
  const uint4* in = reinterpret_cast<const uint4*>(shard) + (int64_t)src * row_vec;
  uint4* out = reinterpret_cast<uint4*>(xb) + (int64_t)b * row_vec;
  uint4* outp = reinterpret_cast<uint4*>(xp) + (int64_t)b * row_vec;
  for (int64_t i = beg + threadIdx.x; i < end; i += blockDim.x) {
    const uint4 v = in[i];
    out[i] = v;
    if (xp)  // uniform
      outp[i] = make_uint4(split_pack(__uint_as_float(v.x)), split_pack(__uint_as_float(v.y)),
                           split_pack(__uint_as_float(v.z)), split_pack(__uint_as_float(v.w)));
  }
  if (part == 0 && threadIdx.x == 0) yb[b] = labels[src];
}

void launch_gather_batch(const uint16_t* shard, const int* labels, const int* perm,
                         const int* step, int steps_per_epoch, int B, int64_t row_elems,
                         uint16_t* xb, int* yb, hipStream_t s, uint32_t* xp) {
  const int64_t row_vec = row_elems / 8;
  int64_t parts = row_vec / 256;  // ~one 16-B vector per thread
  if (parts < 1) parts = 1;
  if (parts > 16) parts = 16;
  gather_kernel<<<(unsigned)(B * parts), 256, 0, s>>>(shard, labels, perm, step, steps_per_epoch, B, (int)parts,
                                                      row_vec, xb, yb, xp);
}

}  // namespace mfl
