// torch binding for the BERT-base path: Linear-layer GEMMs (gemm.hip) and the
// encoder kernels (bert.hip).  Shapes are validated here before any launch.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "kernels/bert.h"
#include "kernels/gemm.h"

namespace {

hipStream_t stream_of(const torch::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}
uint16_t* bfp(const torch::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

void need(const torch::Tensor& t, torch::ScalarType dt, int64_t numel, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == dt, nm, " has the wrong dtype");
  TORCH_CHECK(numel < 0 || t.numel() == numel, nm, " has ", t.numel(), " elements, expected ", numel);
}
void need_min(const torch::Tensor& t, torch::ScalarType dt, int64_t numel, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.scalar_type() == dt, nm, " has the wrong dtype");
  TORCH_CHECK(t.numel() >= numel, nm, " too small");
}
template <typename T>
T* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void dense_dims(int64_t M, int64_t N, int64_t K) {
  TORCH_CHECK(M > 0 && N % 8 == 0 && K % 8 == 0, "GEMM N and K must be multiples of 8");
  TORCH_CHECK(M * std::max(N, K) < (1LL << 31), "GEMM operand too large for 32-bit indexing");
}

// y[M][N] = x[M][K] w[N][K]^T (+ bias) (+ resid); act_out = gelu(y);
// act_grad (with act_out): y holds gelu'(.) of the pre-activation instead
void gemm_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor y, c10::optional<torch::Tensor> bias,
              c10::optional<torch::Tensor> resid, c10::optional<torch::Tensor> act_out, int64_t M, int64_t N,
              int64_t K, bool act_grad) {
  dense_dims(M, N, K);
  need(x, torch::kBFloat16, M * K, "x");
  need(w, torch::kBFloat16, N * K, "w");
  need(y, torch::kBFloat16, M * N, "y");
  if (bias.has_value() && bias->defined()) need_min(*bias, torch::kFloat32, N, "bias");
  if (resid.has_value() && resid->defined()) need(*resid, torch::kBFloat16, M * N, "resid");
  if (act_out.has_value() && act_out->defined()) need(*act_out, torch::kBFloat16, M * N, "act_out");
  TORCH_CHECK(!act_grad || (act_out.has_value() && act_out->defined()), "gemm_fwd: act_grad needs act_out");
  TORCH_CHECK(!act_grad || N % 8 == 0, "gemm_fwd: act_grad width");
  mfl::launch_gemm_fwd(bfp(x), bfp(w), bfp(y), opt_ptr<const float>(bias), opt_ptr<const uint16_t>(resid),
                       opt_ptr<uint16_t>(act_out), (int)M, (int)N, (int)K, stream_of(x), act_grad ? 1 : 0);
}

// dx[M][K] (+)= dy[M][N] w[N][K].  Long reductions over few output tiles
// run split-K through an fp32 slab workspace taken from the caching
// allocator on the current stream (stream-ordered: co-located learners on
// their own streams, and graph capture, get their own).
// resid: dx = dy w + resid (the residual branch's gradient added in the
// output stage; not together with accumulate)
void gemm_dgrad(torch::Tensor dy, torch::Tensor w, torch::Tensor dx, int64_t M, int64_t N, int64_t K,
                bool accumulate, c10::optional<torch::Tensor> resid) {
  dense_dims(M, N, K);
  need(dy, torch::kBFloat16, M * N, "dy");
  need(w, torch::kBFloat16, N * K, "w");
  need(dx, torch::kBFloat16, M * K, "dx");
  const uint16_t* rp = nullptr;
  if (resid.has_value()) {
    TORCH_CHECK(!accumulate, "gemm_dgrad: resid and accumulate are exclusive");
    need(*resid, torch::kBFloat16, M * K, "resid");
    TORCH_CHECK(resid->data_ptr() != dx.data_ptr(), "gemm_dgrad: resid must not alias dx");
    rp = bfp(*resid);
  }
  const int64_t wsn = mfl::gemm_dgrad_workspace((int)M, (int)N, (int)K);
  torch::Tensor ws;
  if (wsn > 0) ws = torch::empty({wsn}, dy.options().dtype(torch::kFloat32));
  mfl::launch_gemm_dgrad(bfp(dy), bfp(w), bfp(dx), (int)M, (int)N, (int)K, accumulate, stream_of(dy),
                         wsn > 0 ? ws.data_ptr<float>() : nullptr, rp);
}

// dz = (dy w) * gelu'(z); dbias += colsum(dz)  (FFN1 backward, one launch)
// pre: z holds gelu'(z) (the forward's act_grad): dz = (dy w) * z
void gemm_dgrad_gelu(torch::Tensor dy, torch::Tensor w, torch::Tensor dz, torch::Tensor z,
                     c10::optional<torch::Tensor> dbias, int64_t M, int64_t N, int64_t K, bool pre) {
  dense_dims(M, N, K);
  need(dy, torch::kBFloat16, M * N, "dy");
  need(w, torch::kBFloat16, N * K, "w");
  need(dz, torch::kBFloat16, M * K, "dz");
  need(z, torch::kBFloat16, M * K, "z");
  if (dbias.has_value() && dbias->defined()) need(*dbias, torch::kFloat32, K, "dbias");
  mfl::launch_gemm_dgrad_gelu(bfp(dy), bfp(w), bfp(dz), bfp(z), opt_ptr<float>(dbias), (int)M, (int)N,
                              (int)K, stream_of(dy), pre ? 1 : 0);
}

// dw[N][K] (+)= dy^T x  (fp32)
// zeroed: dw is known to be zero on entry (the training step's gradient
// buffer, re-zeroed by the optimizer launch) -> no memset before split plans
void gemm_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, int64_t M, int64_t N, int64_t K,
                bool accumulate, bool zeroed) {
  dense_dims(M, N, K);
  need(x, torch::kBFloat16, M * K, "x");
  need(dy, torch::kBFloat16, M * N, "dy");
  need(dw, torch::kFloat32, N * K, "dw");
  // split-K slabs from the caching allocator: stream-ordered, and legal inside
  // graph capture (the block comes from the capture's private pool)
  const int64_t ws_n = mfl::gemm_wgrad_workspace((int)M, (int)N, (int)K);
  torch::Tensor ws;
  if (ws_n > 0) ws = torch::empty({ws_n}, dw.options());
  else if (!accumulate && !zeroed && mfl::gemm_wgrad_splits((int)M, (int)N, (int)K))
    (void)hipMemsetAsync(dw.data_ptr<float>(), 0, dw.numel() * sizeof(float), stream_of(x));
  mfl::launch_gemm_wgrad(bfp(x), bfp(dy), dw.data_ptr<float>(), (int)M, (int)N, (int)K, accumulate,
                         stream_of(x), ws_n > 0 ? ws.data_ptr<float>() : nullptr);
}

// dw0 = dy0^T x0 and dw1 = dy1^T x1 over the same M rows, both zeroed on
// entry, in one grouped launch (gemm_big.hip gemm_pp_group_kernel); two
// ordinary launches where the pair does not fit it.  -> whether grouped.
bool gemm_wgrad2(torch::Tensor x0, torch::Tensor dy0, torch::Tensor dw0, int64_t N0, int64_t K0, torch::Tensor x1,
                 torch::Tensor dy1, torch::Tensor dw1, int64_t N1, int64_t K1, int64_t M) {
  dense_dims(M, N0, K0);
  dense_dims(M, N1, K1);
  need(x0, torch::kBFloat16, M * K0, "x0");
  need(dy0, torch::kBFloat16, M * N0, "dy0");
  need(dw0, torch::kFloat32, N0 * K0, "dw0");
  need(x1, torch::kBFloat16, M * K1, "x1");
  need(dy1, torch::kBFloat16, M * N1, "dy1");
  need(dw1, torch::kFloat32, N1 * K1, "dw1");
  if (!mfl::gemm_big_enabled() || !mfl::gemm_big_wgrad2_ok((int)M, (int)N0, (int)K0, (int)N1, (int)K1)) {
    gemm_wgrad(x0, dy0, dw0, M, N0, K0, false, true);
    gemm_wgrad(x1, dy1, dw1, M, N1, K1, false, true);
    return false;
  }
  const int64_t ws_n = mfl::gemm_big_wgrad2_workspace((int)M, (int)N0, (int)K0, (int)N1, (int)K1);
  torch::Tensor ws;
  if (ws_n > 0) ws = torch::empty({ws_n}, dw0.options());
  mfl::launch_gemm_big_wgrad2(bfp(x0), bfp(dy0), dw0.data_ptr<float>(), (int)N0, (int)K0, bfp(x1), bfp(dy1),
                              dw1.data_ptr<float>(), (int)N1, (int)K1, (int)M, stream_of(x0),
                              ws_n > 0 ? ws.data_ptr<float>() : nullptr);
  return true;
}

void ln_dims(int64_t H) {
  TORCH_CHECK(H % 256 == 0 && H <= 1024, "LayerNorm width must be 256, 512, 768 or 1024");
}

void ln_fwd(torch::Tensor x, torch::Tensor gamma, torch::Tensor beta, torch::Tensor y, torch::Tensor mean,
            torch::Tensor rstd, int64_t M, int64_t H, double eps) {
  ln_dims(H);
  need(x, torch::kBFloat16, M * H, "x");
  need(y, torch::kBFloat16, M * H, "y");
  need(gamma, torch::kFloat32, H, "gamma");
  need(beta, torch::kFloat32, H, "beta");
  need_min(mean, torch::kFloat32, M, "mean");
  need_min(rstd, torch::kFloat32, M, "rstd");
  mfl::LnFwdArgs a;
  a.x = bfp(x);
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.y = bfp(y);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.M = (int)M;
  a.eps = (float)eps;
  mfl::launch_ln_fwd(a, (int)H, false, stream_of(x));
}

void emb_ln_fwd(torch::Tensor rec, int64_t rec_stride, int64_t B, int64_t T, torch::Tensor word,
                torch::Tensor pos, torch::Tensor type, torch::Tensor xsave, torch::Tensor gamma,
                torch::Tensor beta, torch::Tensor y, torch::Tensor mean, torch::Tensor rstd, int64_t H,
                double eps) {
  ln_dims(H);
  const int64_t M = B * T;
  need_min(rec, torch::kInt32, B * rec_stride, "rec");
  TORCH_CHECK(rec_stride >= T, "record stride");
  TORCH_CHECK(word.numel() % H == 0 && pos.numel() >= T * H && type.numel() >= H, "embedding tables");
  need(word, torch::kBFloat16, -1, "word");
  need(pos, torch::kBFloat16, -1, "pos");
  need(type, torch::kBFloat16, -1, "type");
  need(xsave, torch::kBFloat16, M * H, "xsave");
  need(y, torch::kBFloat16, M * H, "y");
  need(gamma, torch::kFloat32, H, "gamma");
  need(beta, torch::kFloat32, H, "beta");
  need_min(mean, torch::kFloat32, M, "mean");
  need_min(rstd, torch::kFloat32, M, "rstd");
  mfl::LnFwdArgs a;
  a.tokens = rec.data_ptr<int>();
  a.tok_stride = (int)rec_stride;
  a.T = (int)T;
  a.word = bfp(word);
  a.pos = bfp(pos);
  a.type = bfp(type);
  a.xsave = bfp(xsave);
  a.gamma = gamma.data_ptr<float>();
  a.beta = beta.data_ptr<float>();
  a.y = bfp(y);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.M = (int)M;
  a.eps = (float)eps;
  mfl::launch_ln_fwd(a, (int)H, true, stream_of(y));
}

void ln_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor mean, torch::Tensor rstd, torch::Tensor gamma,
            torch::Tensor dx, c10::optional<torch::Tensor> dx2, torch::Tensor dgamma, torch::Tensor dbeta,
            c10::optional<torch::Tensor> dbias_prev, int64_t M, int64_t H) {
  ln_dims(H);
  need(dy, torch::kBFloat16, M * H, "dy");
  need(x, torch::kBFloat16, M * H, "x");
  need(dx, torch::kBFloat16, M * H, "dx");
  if (dx2.has_value() && dx2->defined()) need(*dx2, torch::kBFloat16, M * H, "dx2");
  need(gamma, torch::kFloat32, H, "gamma");
  need(dgamma, torch::kFloat32, H, "dgamma");
  need(dbeta, torch::kFloat32, H, "dbeta");
  if (dbias_prev.has_value() && dbias_prev->defined()) need(*dbias_prev, torch::kFloat32, H, "dbias_prev");
  need_min(mean, torch::kFloat32, M, "mean");
  need_min(rstd, torch::kFloat32, M, "rstd");
  mfl::LnBwdArgs a;
  a.dy = bfp(dy);
  a.x = bfp(x);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.gamma = gamma.data_ptr<float>();
  a.dx = bfp(dx);
  a.dx2 = opt_ptr<uint16_t>(dx2);
  a.dgamma = dgamma.data_ptr<float>();
  a.dbeta = dbeta.data_ptr<float>();
  a.dbias_prev = opt_ptr<float>(dbias_prev);
  a.M = (int)M;
  mfl::launch_ln_bwd(a, (int)H, false, stream_of(dy));
}

void emb_ln_bwd(torch::Tensor dy, torch::Tensor xsave, torch::Tensor mean, torch::Tensor rstd,
                torch::Tensor gamma, torch::Tensor rec, int64_t rec_stride, int64_t B, int64_t T,
                torch::Tensor dword, torch::Tensor dpos, torch::Tensor dtype, torch::Tensor dgamma,
                torch::Tensor dbeta, int64_t H, c10::optional<torch::Tensor> demb,
                c10::optional<torch::Tensor> idx, c10::optional<torch::Tensor> tmp) {
  ln_dims(H);
  const int64_t M = B * T;
  need(dy, torch::kBFloat16, M * H, "dy");
  need(xsave, torch::kBFloat16, M * H, "xsave");
  need(gamma, torch::kFloat32, H, "gamma");
  need(dgamma, torch::kFloat32, H, "dgamma");
  need(dbeta, torch::kFloat32, H, "dbeta");
  need_min(rec, torch::kInt32, B * rec_stride, "rec");
  need(dword, torch::kFloat32, -1, "dword");
  need_min(dpos, torch::kFloat32, T * H, "dpos");
  need_min(dtype, torch::kFloat32, H, "dtype");
  TORCH_CHECK(dword.numel() % H == 0, "dword shape");
  need_min(mean, torch::kFloat32, M, "mean");
  need_min(rstd, torch::kFloat32, M, "rstd");
  mfl::LnBwdArgs a;
  a.dy = bfp(dy);
  a.x = bfp(xsave);
  a.mean = mean.data_ptr<float>();
  a.rstd = rstd.data_ptr<float>();
  a.gamma = gamma.data_ptr<float>();
  a.dgamma = dgamma.data_ptr<float>();
  a.dbeta = dbeta.data_ptr<float>();
  a.tokens = rec.data_ptr<int>();
  a.tok_stride = (int)rec_stride;
  a.T = (int)T;
  a.dword = dword.data_ptr<float>();
  a.dpos = dpos.data_ptr<float>();
  a.dtype = dtype.data_ptr<float>();
  a.B = (int)B;
  a.pos_reduced = (B % 16 == 0) ? 1 : 0;  // bert.hip kLnBwdRows
  a.M = (int)M;
  const bool sorted = demb.has_value() && demb->defined();
  const int64_t V = dword.numel() / H;
  int bits = 1;
  while ((1LL << bits) < V) ++bits;
  if (sorted) {
    need(*demb, torch::kFloat32, M * H, "demb");
    TORCH_CHECK(idx.has_value() && idx->defined() && tmp.has_value() && tmp->defined(),
                "emb_ln_bwd: demb needs idx and tmp scratch");
    need(*idx, torch::kInt32, 4 * M, "idx");
    TORCH_CHECK(tmp->is_cuda() && (size_t)tmp->numel() >= mfl::emb_sort_temp_bytes((int)M, bits),
                "emb_ln_bwd: tmp scratch too small (emb_sort_temp_bytes)");
    a.demb = demb->data_ptr<float>();
    a.keys = idx->data_ptr<int>();
    a.vals = a.keys + M;
  }
  mfl::launch_ln_bwd(a, (int)H, true, stream_of(dy));
  if (sorted)
    mfl::launch_emb_word_grad(a.demb, a.keys, a.vals, a.keys + 2 * M, a.keys + 3 * M, tmp->data_ptr(),
                              (size_t)tmp->numel(), (int)M, (int)H, bits, a.dword, stream_of(dy));
}

void gelu_bwd(torch::Tensor dh, torch::Tensor z, torch::Tensor dz, c10::optional<torch::Tensor> dbias,
              int64_t M, int64_t N) {
  TORCH_CHECK(N % 8 == 0, "gelu_bwd width");
  need(dh, torch::kBFloat16, M * N, "dh");
  need(z, torch::kBFloat16, M * N, "z");
  need(dz, torch::kBFloat16, M * N, "dz");
  if (dbias.has_value() && dbias->defined()) need(*dbias, torch::kFloat32, N, "dbias");
  mfl::launch_gelu_bwd(bfp(dh), bfp(z), bfp(dz), opt_ptr<float>(dbias), (int)M, (int)N, stream_of(dh));
}

void colsum(torch::Tensor dy, torch::Tensor dbias, int64_t M, int64_t N) {
  TORCH_CHECK(N % 8 == 0, "colsum width");
  need(dy, torch::kBFloat16, M * N, "dy");
  need(dbias, torch::kFloat32, N, "dbias");
  mfl::launch_colsum(bfp(dy), dbias.data_ptr<float>(), (int)M, (int)N, stream_of(dy));
}

void attn_dims(const torch::Tensor& qkv, int64_t B, int64_t heads) {
  TORCH_CHECK(heads > 0 && B > 0, "attention dims");
  need(qkv, torch::kBFloat16, B * 128 * 3 * heads * 64, "qkv (seq 128, head dim 64)");
}

void attn_fwd(torch::Tensor qkv, torch::Tensor ctx, torch::Tensor lse, int64_t B, int64_t heads, double scale) {
  attn_dims(qkv, B, heads);
  need(ctx, torch::kBFloat16, B * 128 * heads * 64, "ctx");
  need_min(lse, torch::kFloat32, B * heads * 128, "lse");
  mfl::AttnArgs a;
  a.qkv = bfp(qkv);
  a.ctx = bfp(ctx);
  a.lse = lse.data_ptr<float>();
  a.batch = (int)B;
  a.heads = (int)heads;
  a.scale = (float)scale;
  mfl::launch_attn_fwd(a, stream_of(qkv));
}

void attn_bwd(torch::Tensor qkv, torch::Tensor ctx, torch::Tensor lse, torch::Tensor dctx, torch::Tensor dqkv,
              c10::optional<torch::Tensor> dbias, int64_t B, int64_t heads, double scale) {
  attn_dims(qkv, B, heads);
  need(ctx, torch::kBFloat16, B * 128 * heads * 64, "ctx");
  need(dctx, torch::kBFloat16, B * 128 * heads * 64, "dctx");
  need(dqkv, torch::kBFloat16, qkv.numel(), "dqkv");
  need_min(lse, torch::kFloat32, B * heads * 128, "lse");
  if (dbias.has_value() && dbias->defined()) need(*dbias, torch::kFloat32, 3 * heads * 64, "dbias");
  mfl::AttnArgs a;
  a.qkv = bfp(qkv);
  a.ctx = bfp(ctx);
  a.lse = lse.data_ptr<float>();
  a.dctx = bfp(dctx);
  a.dqkv = bfp(dqkv);
  a.dbias = opt_ptr<float>(dbias);
  a.batch = (int)B;
  a.heads = (int)heads;
  a.scale = (float)scale;
  mfl::launch_attn_bwd(a, stream_of(qkv));
}

void rec_dims(const torch::Tensor& rec, int64_t rec_stride, int64_t B, int64_t T, int64_t P) {
  need_min(rec, torch::kInt32, B * rec_stride, "rec");
  TORCH_CHECK(rec_stride >= 2 * T + 2 * P, "record stride < 2T + 2P");
}

void mlm_gather(torch::Tensor x, torch::Tensor rec, int64_t rec_stride, int64_t B, int64_t T, int64_t P,
                torch::Tensor out, int64_t H) {
  rec_dims(rec, rec_stride, B, T, P);
  TORCH_CHECK(H % 8 == 0, "width");
  need(x, torch::kBFloat16, B * T * H, "x");
  need(out, torch::kBFloat16, B * P * H, "out");
  mfl::launch_mlm_gather(bfp(x), rec.data_ptr<int>(), (int)rec_stride, (int)B, (int)T, (int)P, (int)H, bfp(out),
                         stream_of(x));
}

void mlm_scatter(torch::Tensor dsel, torch::Tensor rec, int64_t rec_stride, int64_t B, int64_t T, int64_t P,
                 torch::Tensor dx, int64_t H) {
  rec_dims(rec, rec_stride, B, T, P);
  TORCH_CHECK(H % 8 == 0, "width");
  need(dsel, torch::kBFloat16, B * P * H, "dsel");
  need(dx, torch::kBFloat16, B * T * H, "dx");
  mfl::launch_mlm_scatter(bfp(dsel), rec.data_ptr<int>(), (int)rec_stride, (int)B, (int)T, (int)P, (int)H,
                          bfp(dx), stream_of(dx));
}

void vocab_xent(torch::Tensor logits, c10::optional<torch::Tensor> dlogits, torch::Tensor rec, int64_t rec_stride,
                int64_t B, int64_t T, int64_t P, int64_t V, int64_t Vp, torch::Tensor stats) {
  rec_dims(rec, rec_stride, B, T, P);
  TORCH_CHECK(Vp % 8 == 0 && V <= Vp, "vocab padding");
  need(logits, torch::kBFloat16, B * P * Vp, "logits");
  if (dlogits.has_value() && dlogits->defined()) need(*dlogits, torch::kBFloat16, B * P * Vp, "dlogits");
  need_min(stats, torch::kFloat32, 3, "stats");
  mfl::VocabXentArgs a;
  a.logits = bfp(logits);
  a.dlogits = opt_ptr<uint16_t>(dlogits);
  a.rec = rec.data_ptr<int>();
  a.rec_stride = (int)rec_stride;
  a.T = (int)T;
  a.P = (int)P;
  a.R = (int)(B * P);
  a.V = (int)V;
  a.Vp = (int)Vp;
  a.stats = stats.data_ptr<float>();
  mfl::launch_vocab_xent(a, stream_of(logits));
}

}  // namespace

void register_bert(pybind11::module& m) {
  m.def("gemm_fwd", &gemm_fwd, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("bias"),
        pybind11::arg("resid"), pybind11::arg("act_out"), pybind11::arg("M"), pybind11::arg("N"),
        pybind11::arg("K"), pybind11::arg("act_grad") = false);
  m.def("set_gemm_big", [](bool on) { mfl::set_gemm_big(on ? 1 : 0); });
  m.def("gemm_big_enabled", []() { return mfl::gemm_big_enabled() != 0; });
  m.def("gemm_dgrad", &gemm_dgrad, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("dx"), pybind11::arg("M"),
        pybind11::arg("N"),
        pybind11::arg("K"), pybind11::arg("accumulate"), pybind11::arg("resid") = pybind11::none());
  m.def("gemm_dgrad_workspace",
        [](int64_t M, int64_t N, int64_t K) { return mfl::gemm_dgrad_workspace((int)M, (int)N, (int)K); });
  m.def("gemm_dgrad_gelu", &gemm_dgrad_gelu, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("dz"),
        pybind11::arg("z"), pybind11::arg("dbias"), pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("K"),
        pybind11::arg("pre") = false);
  m.def("gemm_wgrad", &gemm_wgrad);
  m.def("gemm_wgrad2", &gemm_wgrad2);
  m.def("set_gemm_wgrad2_splits", [](int64_t s) { mfl::set_gemm_wgrad2_splits((int)s); });
  m.def("set_gemm_width", [](int64_t w) { mfl::set_gemm_width((int)w); });
  m.def("ln_fwd", &ln_fwd);
  m.def("emb_ln_fwd", &emb_ln_fwd);
  m.def("ln_bwd", &ln_bwd);
  m.def("emb_ln_bwd", &emb_ln_bwd, pybind11::arg("dy"), pybind11::arg("xsave"), pybind11::arg("mean"),
        pybind11::arg("rstd"), pybind11::arg("gamma"), pybind11::arg("rec"), pybind11::arg("rec_stride"),
        pybind11::arg("B"), pybind11::arg("T"), pybind11::arg("dword"), pybind11::arg("dpos"),
        pybind11::arg("dtype"), pybind11::arg("dgamma"), pybind11::arg("dbeta"), pybind11::arg("H"),
        pybind11::arg("demb") = pybind11::none(), pybind11::arg("idx") = pybind11::none(),
        pybind11::arg("tmp") = pybind11::none());
  m.def("emb_sort_temp_bytes", [](int64_t M, int64_t V) {
    int bits = 1;
    while ((1LL << bits) < V) ++bits;
    return (int64_t)mfl::emb_sort_temp_bytes((int)M, bits);
  });
  m.def("gelu_bwd", &gelu_bwd);
  m.def("colsum", &colsum);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
  m.def("mlm_gather", &mlm_gather);
  m.def("mlm_scatter", &mlm_scatter);
  m.def("vocab_xent", &vocab_xent);
}
