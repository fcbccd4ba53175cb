// Dense bf16 GEMM entry points (BERT-base path, classifier heads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {

enum GemmEpilogue { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_BIAS_RESIDUAL = 3 };

// C[M][N] = A[M][K] . B[N][K]^T  with an optional fused epilogue
// (bias, bias+GELU(tanh), bias+residual(aux)).
void launch_gemm_nt(const uint16_t* a, const uint16_t* b, uint16_t* c, const float* bias,
                    const uint16_t* aux, int M, int N, int K, int epilogue, hipStream_t s);

}  // namespace mfl
