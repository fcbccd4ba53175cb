// BERT-base kernel entry points (bert.hip).  All launchers take the stream
// explicitly and allocate nothing (hipGraph-capturable).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfl {

struct LnFwdArgs {
  const uint16_t* x = nullptr;  // [M][H] LN input (non-embedding variant)
  // embedding variant: x = word[tok] + pos[t] + type[0], stored to xsave
  const int* tokens = nullptr;
  int tok_stride = 0, T = 1;
  const uint16_t* word = nullptr;
  const uint16_t* pos = nullptr;
  const uint16_t* type = nullptr;
  uint16_t* xsave = nullptr;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  uint16_t* y = nullptr;
  float* mean = nullptr;
  float* rstd = nullptr;
  int M = 0;
  float eps = 1e-12f;
};

struct LnBwdArgs {
  const uint16_t* dy = nullptr;
  const uint16_t* x = nullptr;  // LN input
  const float* mean = nullptr;
  const float* rstd = nullptr;
  const float* gamma = nullptr;
  uint16_t* dx = nullptr;
  uint16_t* dx2 = nullptr;        // optional second copy (residual branch)
  float* dgamma = nullptr;
  float* dbeta = nullptr;
  float* dbias_prev = nullptr;    // optional: += column sums of dx
  // embedding variant: dx scattered into the tables (fp32 grads)
  const int* tokens = nullptr;
  int tok_stride = 0, T = 1;
  float* dword = nullptr;
  float* dpos = nullptr;
  float* dtype = nullptr;
  int B = 1, pos_reduced = 0;  // see ln_bwd_kernel
  // contention-free word-table gradient (optional): dx rows go to demb
  // [M][H] fp32 and (token, row) pairs to keys / vals [M]; launch_emb_word_grad
  // then sorts by token and reduces each token's rows (no same-address
  // atomics for frequent tokens such as [MASK] / [CLS])
  float* demb = nullptr;
  int* keys = nullptr;
  int* vals = nullptr;
  int rows = 16;               // rows per block (set by the launcher)
  int dbg = 0;                 // timing experiments (MFL_LN_BWD_DEBUG): bit0 skip global column atomics, bit1 skip LDS reduction
  int M = 0;
};

// Word-embedding gradient from the demb / keys / vals scratch written by the
// embedding LN backward: radix sort of (token, row) pairs (hipCUB) into
// skeys / svals, then a chunked segmented reduction -- each token's rows are
// summed in registers, only segments that straddle a 64-row chunk boundary
// use atomics.  tmp: emb_sort_temp_bytes(M, key_bits) bytes.
size_t emb_sort_temp_bytes(int M, int key_bits);
void launch_emb_word_grad(const float* demb, const int* keys, const int* vals, int* skeys, int* svals,
                          void* tmp, size_t tmp_bytes, int M, int H, int key_bits, float* dword,
                          hipStream_t s);

struct AttnArgs {
  const uint16_t* qkv = nullptr;  // [B*T][3H]: q | k | v, head h at columns h*64
  uint16_t* ctx = nullptr;        // [B*T][H] (forward output)
  float* lse = nullptr;           // [B][heads][T] natural-log softmax normaliser
  const uint16_t* dctx = nullptr;
  uint16_t* dqkv = nullptr;
  float* dbias = nullptr;         // optional [3H] qkv bias gradient (+=)
  int batch = 0, heads = 0;
  float scale = 0.125f;
};

struct VocabXentArgs {
  const uint16_t* logits = nullptr;  // [R][Vp]
  uint16_t* dlogits = nullptr;       // optional [R][Vp]
  const int* rec = nullptr;          // batch records (labels inside)
  int rec_stride = 0, T = 0, P = 0;
  int R = 0, V = 0, Vp = 0;
  float* stats = nullptr;            // [loss, correct, count]
};

void launch_ln_fwd(const LnFwdArgs& a, int H, bool emb, hipStream_t s);
void launch_ln_bwd(const LnBwdArgs& a, int H, bool emb, hipStream_t s);
// pre: z holds gelu'(z) already (dz = dh * z)
void launch_gelu_bwd(const uint16_t* dh, const uint16_t* z, uint16_t* dz, float* dbias, int M, int N,
                     hipStream_t s, int pre = 0);
// y <- gelu'(y) in place, n % 8 == 0
void launch_gelu_grad_inplace(uint16_t* y, int64_t n, hipStream_t s);
void launch_colsum(const uint16_t* dy, float* dbias, int M, int N, hipStream_t s);
size_t attn_fwd_lds();
size_t attn_bwd_lds();
void launch_attn_fwd(const AttnArgs& a, hipStream_t s);
void launch_attn_bwd(const AttnArgs& a, hipStream_t s);
void launch_mlm_gather(const uint16_t* x, const int* rec, int rec_stride, int B, int T, int P, int H,
                       uint16_t* out, hipStream_t s);
void launch_mlm_scatter(const uint16_t* dsel, const int* rec, int rec_stride, int B, int T, int P, int H,
                        uint16_t* dx, hipStream_t s);
void launch_vocab_xent(const VocabXentArgs& a, hipStream_t s);

}  // namespace mfl
