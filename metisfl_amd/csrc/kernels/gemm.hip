// K7: dense bf16 GEMMs on the MFMA implicit-GEMM core of conv.hip.  A 1x1
// convolution over an M x 1 x 1 "image" is exactly a GEMM with both operands
// K-contiguous, so the three training GEMMs of a Linear layer map onto the
// three conv kernels with no new tiling code:
//   forward  Y[M][N]  = X[M][K] . W[N][K]^T  (+bias, +residual, GELU copy:
//                       fused into the tile epilogue, no extra pass)
//   dgrad    dX[M][K] = dY[M][N] . W[N][K]   (conv dgrad, W read through
//                       transposing LDS reads -- no weight transpose)
//   wgrad    dW[N][K] += dY^T . X            (conv wgrad, fp32 accumulation
//                       into the flat gradient buffer)
// Reference: the Keras Dense layers of the example models
// (examples/keras/models/fashion_mnist_fc.py:19-21, cifar_cnn.py:38-41) and
// the BERT-base FFN / attention projections of SURVEY §2.10 K7.
#include "kernels/common.h"
#include "kernels/conv.h"
#include "kernels/gemm.h"
#include "kernels/bert.h"

namespace mfl {

static ConvGeom dense_geom(int M, int Nout, int K) {
  ConvGeom g{};
  g.N = M; g.H = 1; g.W = 1; g.C = K;
  g.P = 1; g.Q = 1; g.R = 1; g.S = 1; g.stride = 1; g.pad = 0;
  g.M = M; g.K = K; g.Ng = Nout;
  return g;
}

// Tile plan for a dense GEMM with M rows, N columns, K reduction.  Bigger
// tiles re-read fewer operand bytes per FLOP (a 128x128 tile does twice the
// MFMA work per staged byte of a 128x64 one) but give fewer workgroups; take
// the biggest tile that still puts >= 2 workgroups on each of the 256 CUs,
// and never split K (the BERT GEMMs have >= 768 tiles of work already).
ConvPlan plan_gemm(int M, int N, int K) {
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  ConvPlan p;
  if (blocks(128, 128) >= 512) {
    p.bm = 128; p.bn = 128;
  } else if (blocks(128, 64) >= 256) {
    p.bm = 128; p.bn = 64;
  } else {
    p.bm = 64; p.bn = 64;
  }
  p.bk = (K >= 512 && !(p.bm == 128 && p.bn == 128)) ? 128 : 64;
  p.splits = 1;
  p.kchunk = ((K + p.bk - 1) / p.bk) * p.bk;
  p.stats_rows = 0;
  return p;
}

static int g_big = -1;
void set_gemm_big(int on) { g_big = on ? 1 : 0; }
int gemm_big_enabled() {
  if (g_big < 0) {
    const char* v = getenv("MFL_GEMM_BIG");
    g_big = (v && *v == '0') ? 0 : 1;
  }
  return g_big;
}

void launch_gemm_fwd(const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                     const uint16_t* resid, uint16_t* act_out, int M, int N, int K, hipStream_t s,
                     int act_grad) {
  if (gemm_big_enabled() && gemm_big_ok(M, N, K)) {
    launch_gemm_big_fwd(x, w, y, bias, resid, act_out, M, N, K, s, act_grad);
    return;
  }
  const ConvGeom g = dense_geom(M, N, K);
  GemmEpilogueArgs e;
  e.bias = bias;
  e.resid = resid;
  e.act_out = act_out;
  launch_conv_gemm_epi(g, plan_gemm(M, N, K), x, w, y, nullptr, nullptr, e, s);
  if (act_out && act_grad) launch_gelu_grad_inplace(y, (int64_t)M * N, s);  // conv-core path: y -> gelu'(y)
}

void launch_gemm_dgrad(const uint16_t* dy, const uint16_t* w, uint16_t* dx, int M, int N, int K,
                       bool accumulate, hipStream_t s, float* ws, const uint16_t* resid) {
  if (gemm_big_enabled() && gemm_big_ok(M, K, N)) {
    launch_gemm_big_dgrad(dy, w, dx, M, N, K, accumulate, s, ws, resid);
    return;
  }
  if (resid) {  // small shapes (conv-core path): dx = resid, then accumulate
    (void)hipMemcpyAsync(dx, resid, (size_t)M * K * 2, hipMemcpyDeviceToDevice, s);
    accumulate = true;
  }
  // dgrad geometry: "dY" has C = N channels, the output dX has Ng = K columns
  ConvGeom g = dense_geom(M, K, N);
  ConvPlan p = plan_gemm(M, K, N);
  launch_conv_gemm(g, true, p, dy, w, dx, nullptr, nullptr, nullptr, accumulate, s);
}

void launch_gemm_dgrad_gelu(const uint16_t* dy, const uint16_t* w, uint16_t* dz, const uint16_t* z,
                            float* dbias, int M, int N, int K, hipStream_t s, int pre) {
  if (gemm_big_enabled() && gemm_big_ok(M, K, N)) {
    launch_gemm_big_dgrad_gelu(dy, w, dz, z, dbias, M, N, K, s, pre);
    return;
  }
  launch_gemm_dgrad(dy, w, dz, M, N, K, false, s);
  launch_gelu_bwd(dz, z, dz, dbias, M, K, s, pre);  // in place: each element read then written by one thread
}

void launch_gemm_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int M, int N, int K,
                       bool accumulate, hipStream_t s, float* ws) {
  if (gemm_big_enabled() && gemm_big_ok(N, K, M)) {
    launch_gemm_big_wgrad(x, dy, dw, M, N, K, accumulate, s, ws);
    return;
  }
  const ConvGeom g = dense_geom(M, N, K);
  launch_conv_wgrad(g, plan_conv_wgrad(g), x, dy, dw, s, accumulate);
}

int64_t gemm_dgrad_workspace(int M, int N, int K) {
  return (gemm_big_enabled() && gemm_big_ok(M, K, N)) ? gemm_big_dgrad_workspace(M, N, K) : 0;
}

int64_t gemm_wgrad_workspace(int M, int N, int K) {
  return (gemm_big_enabled() && gemm_big_ok(N, K, M)) ? gemm_big_wgrad_workspace(M, N, K) : 0;
}

bool gemm_wgrad_splits(int M, int N, int K) {
  if (gemm_big_enabled() && gemm_big_ok(N, K, M)) return gemm_big_wgrad_splits(M, N, K) > 1;
  return plan_conv_wgrad(dense_geom(M, N, K)).splits > 1; }

void launch_gemm_nt(const uint16_t* a, const uint16_t* b, uint16_t* c, const float* bias,
                    const uint16_t* aux, int M, int N, int K, int epilogue, hipStream_t s) {
  if (gemm_big_enabled() && gemm_big_ok(M, N, K)) {
    launch_gemm_big_fwd(a, b, c, epilogue != EPI_NONE ? bias : nullptr,
                        epilogue == EPI_BIAS_RESIDUAL ? aux : nullptr,
                        epilogue == EPI_BIAS_GELU ? c : nullptr, M, N, K, s);
    return;
  }
  GemmEpilogueArgs e;
  if (epilogue != EPI_NONE) e.bias = bias;
  if (epilogue == EPI_BIAS_RESIDUAL) e.resid = aux;
  // GELU in place: the same thread stores the pre-activation, then gelu()
  if (epilogue == EPI_BIAS_GELU) e.act_out = c;
  launch_conv_gemm_epi(dense_geom(M, N, K), plan_gemm(M, N, K), a, b, c, nullptr, nullptr, e, s);
}

}  // namespace mfl
