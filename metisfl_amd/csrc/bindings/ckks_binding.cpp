// torch binding for the device RNS-CKKS kernels (kernels/ckks.hip).  The
// tables arrive as a fixed-order list of device tensors built once by
// metisfl_amd/encryption/device.py; shapes are validated here, on the host,
// before any launch (the kernels index [nct][2][L][N] with no bounds checks).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <cstring>

#include "kernels/ckks.h"

namespace {

enum {
  kQ, kOneSh, kPsi, kPsiSh, kIpsi, kIpsiSh, kNinv, kNinvSh, kPkB, kPkBSh, kPkA, kPkASh, kSk, kSkSh,
  kGarner, kRot, kKsiRe, kKsiIm, kNumTables
};

hipStream_t cur_stream(const torch::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

template <typename T>
const T* ptr(const std::vector<torch::Tensor>& v, int i, int64_t numel, const char* nm) {
  const auto& t = v[i];
  if (t.numel() == 0) return nullptr;
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "ckks table ", nm, " must be a contiguous device tensor");
  TORCH_CHECK(t.numel() == numel, "ckks table ", nm, " has ", t.numel(), " elements, expected ", numel);
  TORCH_CHECK(t.element_size() == sizeof(T), "ckks table ", nm, " element size");
  return reinterpret_cast<const T*>(t.data_ptr());
}

mfl::CkksTables tables(const std::vector<torch::Tensor>& v, int64_t N, int64_t L) {
  TORCH_CHECK((int)v.size() == kNumTables, "ckks: expected ", (int)kNumTables, " tables");
  TORCH_CHECK(N >= 16 && N <= 8192 && (N & (N - 1)) == 0, "ckks: ring dimension must be a power of two <= 8192");
  TORCH_CHECK(L >= 1 && L <= mfl::kCkksMaxLimbs, "ckks: 1..", mfl::kCkksMaxLimbs, " limbs");
  mfl::CkksTables T{};
  T.N = (int)N;
  T.S = (int)(N / 2);
  T.L = (int)L;
  const int64_t LN = L * N;
  T.q = ptr<uint64_t>(v, kQ, L, "q");
  T.one_sh = ptr<uint64_t>(v, kOneSh, L, "one_sh");
  T.psi = ptr<uint64_t>(v, kPsi, LN, "psi");
  T.psi_sh = ptr<uint64_t>(v, kPsiSh, LN, "psi_sh");
  T.ipsi = ptr<uint64_t>(v, kIpsi, LN, "ipsi");
  T.ipsi_sh = ptr<uint64_t>(v, kIpsiSh, LN, "ipsi_sh");
  T.ninv = ptr<uint64_t>(v, kNinv, L, "ninv");
  T.ninv_sh = ptr<uint64_t>(v, kNinvSh, L, "ninv_sh");
  T.pk_b = ptr<uint64_t>(v, kPkB, LN, "pk_b");
  T.pk_b_sh = ptr<uint64_t>(v, kPkBSh, LN, "pk_b_sh");
  T.pk_a = ptr<uint64_t>(v, kPkA, LN, "pk_a");
  T.pk_a_sh = ptr<uint64_t>(v, kPkASh, LN, "pk_a_sh");
  T.sk = ptr<uint64_t>(v, kSk, LN, "sk");
  T.sk_sh = ptr<uint64_t>(v, kSkSh, LN, "sk_sh");
  T.garner = ptr<uint64_t>(v, kGarner, mfl::kCkksMaxLimbs * mfl::kCkksMaxLimbs * 2, "garner");
  T.rot = ptr<uint32_t>(v, kRot, N / 2, "rot");
  T.ksi_re = ptr<double>(v, kKsiRe, 2 * N + 1, "ksi_re");
  T.ksi_im = ptr<double>(v, kKsiIm, 2 * N + 1, "ksi_im");
  TORCH_CHECK(T.q && T.one_sh && T.psi && T.psi_sh && T.ipsi && T.ipsi_sh && T.ninv && T.ninv_sh &&
                  T.garner && T.rot && T.ksi_re && T.ksi_im,
              "ckks: context tables missing");
  return T;
}

void check_u64(const torch::Tensor& t, int64_t numel, const char* nm) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kInt64, nm,
              " must be a contiguous int64 (u64 bits) device tensor");
  TORCH_CHECK(t.numel() == numel, nm, " has ", t.numel(), " elements, expected ", numel);
}

int64_t num_ct(int64_t n, int64_t S) { return std::max<int64_t>(1, (n + S - 1) / S); }

mfl::CkksKey key_from(const std::string& k) {
  TORCH_CHECK(k.size() == 32, "ckks: the encryption key must be 32 bytes");
  mfl::CkksKey key;
  std::memcpy(key.w, k.data(), 32);
  return key;
}

void ckks_encrypt_dev(std::vector<torch::Tensor> tabs, int64_t N, int64_t L, torch::Tensor x,
                      torch::Tensor ct, torch::Tensor u, double delta, pybind11::bytes key32) {
  auto T = tables(tabs, N, L);
  TORCH_CHECK(T.pk_a && T.pk_b && T.pk_a_sh && T.pk_b_sh, "ckks encrypt: public key not loaded");
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == torch::kFloat32, "x fp32");
  const int64_t nct = num_ct(x.numel(), T.S);
  check_u64(ct, nct * 2 * L * N, "ct");
  check_u64(u, nct * L * N, "u scratch");
  mfl::launch_ckks_encrypt(T, x.data_ptr<float>(), x.numel(), nct, delta, key_from(key32),
                           reinterpret_cast<uint64_t*>(ct.data_ptr()),
                           reinterpret_cast<uint64_t*>(u.data_ptr()), cur_stream(x));
}

void ckks_decrypt_dev(std::vector<torch::Tensor> tabs, int64_t N, int64_t L, torch::Tensor ct,
                      torch::Tensor m, torch::Tensor out, double inv_scale) {
  auto T = tables(tabs, N, L);
  TORCH_CHECK(T.sk && T.sk_sh, "ckks decrypt: private key not loaded");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() &&
                  (out.scalar_type() == torch::kFloat32 || out.scalar_type() == torch::kFloat64),
              "out must be a contiguous fp32 / fp64 device tensor");
  const bool f64 = out.scalar_type() == torch::kFloat64;
  const int64_t nct = num_ct(out.numel(), T.S);
  check_u64(ct, nct * 2 * L * N, "ct");
  check_u64(m, nct * L * N, "m scratch");
  mfl::launch_ckks_decrypt(T, reinterpret_cast<const uint64_t*>(ct.data_ptr()), nct, inv_scale,
                           reinterpret_cast<uint64_t*>(m.data_ptr()),
                           f64 ? nullptr : out.data_ptr<float>(), f64 ? out.data_ptr<double>() : nullptr,
                           out.numel(), cur_stream(out));
}

void ckks_ntt_dev(std::vector<torch::Tensor> tabs, int64_t N, int64_t L, torch::Tensor rows, bool inverse) {
  auto T = tables(tabs, N, L);
  TORCH_CHECK(rows.numel() % (N * L) == 0, "rows must hold whole [L][N] groups");
  check_u64(rows, rows.numel(), "rows");
  mfl::launch_ckks_ntt(T, reinterpret_cast<uint64_t*>(rows.data_ptr()), rows.numel() / N, inverse,
                       cur_stream(rows));
}

void ckks_scale_dev(std::vector<torch::Tensor> tabs, int64_t N, int64_t L, torch::Tensor x, torch::Tensor wq) {
  auto T = tables(tabs, N, L);
  TORCH_CHECK(x.numel() % (N * L) == 0, "x must hold whole [L][N] groups");
  check_u64(x, x.numel(), "x");
  check_u64(wq, 2 * L, "wq");
  mfl::launch_ckks_scale(T, reinterpret_cast<uint64_t*>(x.data_ptr()),
                         reinterpret_cast<const uint64_t*>(wq.data_ptr()), x.numel(), cur_stream(x));
}

void ckks_reduce_dev(std::vector<torch::Tensor> tabs, int64_t N, int64_t L, torch::Tensor x) {
  auto T = tables(tabs, N, L);
  TORCH_CHECK(x.numel() % (N * L) == 0, "x must hold whole [L][N] groups");
  check_u64(x, x.numel(), "x");
  mfl::launch_ckks_reduce(T, reinterpret_cast<uint64_t*>(x.data_ptr()), x.numel(), cur_stream(x));
}

}  // namespace

// RFC 8439 known-answer / stream checks on the device
torch::Tensor chacha20_blocks_dev(pybind11::bytes key32, int64_t counter0, pybind11::bytes nonce12, int64_t nblocks,
                                  torch::Tensor like) {
  const std::string n = nonce12;
  TORCH_CHECK(n.size() == 12 && nblocks > 0 && nblocks < (1 << 24), "nonce 12 bytes, 0 < nblocks < 2^24");
  uint32_t nw[3];
  std::memcpy(nw, n.data(), 12);
  auto out = torch::empty({nblocks * 16}, like.options().dtype(torch::kInt32));
  mfl::launch_chacha_blocks(key_from(key32), (uint32_t)counter0, nw, (int)nblocks,
                            reinterpret_cast<uint32_t*>(out.data_ptr()), cur_stream(like));
  return out;
}
torch::Tensor ckks_noise_dump_dev(pybind11::bytes key32, int64_t c, int64_t n, torch::Tensor like) {
  TORCH_CHECK(n > 0 && n < (1 << 26), "0 < n < 2^26");
  auto out = torch::empty({3 * n}, like.options().dtype(torch::kInt64));
  mfl::launch_ckks_noise_dump(key_from(key32), c, (int)n, out.data_ptr<int64_t>(), cur_stream(like));
  return out;
}

void register_ckks(pybind11::module& m) {
  m.def("chacha20_blocks", &chacha20_blocks_dev);
  m.def("ckks_noise_dump", &ckks_noise_dump_dev);
  m.def("ckks_encrypt", &ckks_encrypt_dev);
  m.def("ckks_decrypt", &ckks_decrypt_dev);
  m.def("ckks_ntt", &ckks_ntt_dev);
  m.def("ckks_scale", &ckks_scale_dev);
  m.def("ckks_reduce", &ckks_reduce_dev);
}
