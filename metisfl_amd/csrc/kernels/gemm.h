// Dense bf16 GEMM entry points (BERT-base path, classifier heads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels/conv.h"

namespace mfl {

enum GemmEpilogue { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RESIDUAL = 3 };

ConvPlan plan_gemm(int M, int N, int K);

// C[M][N] = A[M][K] . B[N][K]^T  with an optional fused epilogue
// (bias, bias+GELU(erf) in place, bias+residual(aux)).
void launch_gemm_nt(const uint16_t* a, const uint16_t* b, uint16_t* c, const float* bias,
                    const uint16_t* aux, int M, int N, int K, int epilogue, hipStream_t s);

// Linear layer GEMMs (W is [N][K], K-contiguous):
//   y = x W^T + bias (+ resid);  act_out = gelu(y) when given; with act_grad
//   (and act_out) y holds gelu'(x W^T + bias) instead, for a backward that
//   multiplies by it (launch_gemm_dgrad_gelu pre)
void launch_gemm_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                     const uint16_t* resid, uint16_t* act_out, int M, int N, int K, hipStream_t s,
                     int act_grad = 0);
//   dx (+)= dy W  (+ resid: dx = dy W + resid, the residual branch's gradient
//   read in the epilogue instead of a copy of it accumulated into)
//   ws: optional split-K slab workspace of gemm_dgrad_workspace(M, N, K) fp32
//   elements (long reductions over few output tiles: the MLM decoder)
void launch_gemm_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int N, int K,
                       bool accumulate, hipStream_t s, float* ws = nullptr, const uint16_t* resid = nullptr);
int64_t gemm_dgrad_workspace(int M, int N, int K);
//   dw = dy^T x, or dw += with accumulate (fp32 atomics; split-K plans always
//   add, so dw must be zero on entry unless accumulating on purpose)
//   ws: optional split-K slab workspace of gemm_wgrad_workspace(M, N, K) fp32
//   elements -- the slices store partials and one reduce launch sums them
//   (then dw needs no zeroing); without it split plans add with atomics
void launch_gemm_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int N, int K,
                       bool accumulate, hipStream_t s, float* ws = nullptr);
bool gemm_wgrad_splits(int M, int N, int K);
int64_t gemm_wgrad_workspace(int M, int N, int K);

// Large-tile path (gemm_big.hip): 256x256 tiles, exact-tiling shapes only.
bool gemm_big_ok(int M, int N, int K);
void launch_gemm_big_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                         const uint16_t* resid, uint16_t* act_out, int M, int N, int K, hipStream_t s,
                         int act_grad = 0);
void launch_gemm_big_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int N, int K,
                           bool accumulate, hipStream_t s, float* ws = nullptr, const uint16_t* resid = nullptr);
int gemm_big_dgrad_splits(int M, int N, int K);
int64_t gemm_big_dgrad_workspace(int M, int N, int K);
void launch_gemm_big_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int N, int K,
                           bool accumulate, hipStream_t s, float* ws = nullptr);
int gemm_big_wgrad_splits(int M, int N, int K);
int64_t gemm_big_wgrad_workspace(int M, int N, int K);
// two weight gradients over the same M in one launch (zeroed dW0 / dW1);
// set_gemm_wgrad2_splits: run-time slice count (0: the default plan)
void set_gemm_wgrad2_splits(int splits);
// ping-pong tile width: 0 = per-shape plan, 192 / 256 forced (co-located regime)
void set_gemm_width(int w);
bool gemm_big_wgrad2_ok(int M, int N0, int K0, int N1, int K1);
int64_t gemm_big_wgrad2_workspace(int M, int N0, int K0, int N1, int K1);
void launch_gemm_big_wgrad2(const uint16_t* x0, const uint16_t* dy0, float* dw0, int N0, int K0, const uint16_t* x1,
                            const uint16_t* dy1, float* dw1, int N1, int K1, int M, hipStream_t s, float* ws);
void launch_gemm_big_dgrad_gelu(const uint16_t* dy, const uint16_t* w, uint16_t* dz, const uint16_t* z,
                                float* dbias, int M, int N, int K, hipStream_t s, int pre = 0);
// dz[M][K] = (dy W) * gelu'(z) (exact erf), dbias[K] += column sums of dz:
// the FFN1 backward in one launch on the large-tile path (else dgrad + gelu_bwd);
// pre: z holds gelu'(z) already (the forward's act_grad)
void launch_gemm_dgrad_gelu(const uint16_t* dy, const uint16_t* w, uint16_t* dz, const uint16_t* z,
                            float* dbias, int M, int N, int K, hipStream_t s, int pre = 0);  // > 1: adds into dw (atomics)
// 1 (default; env MFL_GEMM_BIG=0 turns it off): eligible shapes take the large-tile path
void set_gemm_big(int on);
int gemm_big_enabled();

}  // namespace mfl
