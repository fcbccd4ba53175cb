// K7: dense bf16 GEMM  C = A . B^T  on the MFMA implicit-GEMM core of conv.hip
// (a 1x1 convolution over an M x 1 x 1 "image" is exactly an NT GEMM with
// both operands K-contiguous), followed by a fused vectorised epilogue.
#include "kernels/common.h"
#include "kernels/conv.h"
#include "kernels/gemm.h"

namespace mfl {

template <int EPI>
__global__ __launch_bounds__(256) void gemm_epilogue_kernel(uint16_t* __restrict__ c,
                                                            const float* __restrict__ bias,
                                                            const uint16_t* __restrict__ aux,
                                                            int64_t nvec, int N) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int vpr = N / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int cb = (int)(i % vpr) * 8;
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(c)[i], f);
    float r[8];
    if (EPI == EPI_BIAS_RESIDUAL) unpack8(reinterpret_cast<const uint4*>(aux)[i], r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = f[k] + bias[cb + k];
      if (EPI == EPI_BIAS_GELU) {
        const float u = 0.7978845608f * (v + 0.044715f * v * v * v);
        v = 0.5f * v * (1.f + tanhf(u));
      }
      if (EPI == EPI_BIAS_RESIDUAL) v += r[k];
      f[k] = v;
    }
    reinterpret_cast<uint4*>(c)[i] = pack8(f);
  }
}

void launch_gemm_nt(const uint16_t* a, const uint16_t* b, uint16_t* c, const float* bias,
                    const uint16_t* aux, int M, int N, int K, int epilogue, hipStream_t s) {
  ConvGeom g{};
  g.N = M; g.H = 1; g.W = 1; g.C = K;
  g.P = 1; g.Q = 1; g.R = 1; g.S = 1; g.stride = 1; g.pad = 0;
  g.M = M; g.K = K; g.Ng = N;
  ConvPlan p = plan_conv_gemm(g);
  p.splits = 1;  // no workspace on this path
  p.kchunk = ((K + 63) / 64) * 64;
  launch_conv_gemm(g, false, p, a, b, c, nullptr, nullptr, nullptr, false, s);
  if (epilogue != EPI_NONE && bias) {
    const int64_t nvec = (int64_t)M * N / 8;
    const unsigned grid = stream_grid(nvec);
    if (epilogue == EPI_BIAS) gemm_epilogue_kernel<EPI_BIAS><<<grid, 256, 0, s>>>(c, bias, aux, nvec, N);
    else if (epilogue == EPI_BIAS_GELU) gemm_epilogue_kernel<EPI_BIAS_GELU><<<grid, 256, 0, s>>>(c, bias, aux, nvec, N);
    else gemm_epilogue_kernel<EPI_BIAS_RESIDUAL><<<grid, 256, 0, s>>>(c, bias, aux, nvec, N);
  }
}

}  // namespace mfl
