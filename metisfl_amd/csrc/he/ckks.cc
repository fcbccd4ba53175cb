#include "he/ckks.h"

#include "engine/device_agg.h"

#include <sys/random.h>

#include <cerrno>
#include <cmath>

#include "common/chacha20.h"

#include <omp.h>
#include <sys/stat.h>

#include <cmath>
#include <complex>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace mfl {
namespace {

using u128 = unsigned __int128;

inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)((u128)a * b % q); }
inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) {
  const uint64_t s = a + b;
  return s >= q ? s - q : s;
}
inline uint64_t submod(uint64_t a, uint64_t b, uint64_t q) { return a >= b ? a - b : a + q - b; }
inline uint64_t shoup(uint64_t w, uint64_t q) { return (uint64_t)(((u128)w << 64) / q); }
inline uint64_t mulsh(uint64_t a, uint64_t w, uint64_t wp, uint64_t q) {
  const uint64_t hi = (uint64_t)(((u128)a * wp) >> 64);
  const uint64_t r = a * w - hi * q;
  return r >= q ? r - q : r;
}
uint64_t powmod(uint64_t b, uint64_t e, uint64_t q) {
  uint64_t r = 1;
  b %= q;
  while (e) {
    if (e & 1) r = mulmod(r, b, q);
    b = mulmod(b, b, q);
    e >>= 1;
  }
  return r;
}
bool is_prime(uint64_t n) {
  if (n < 2) return false;
  for (uint64_t p : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull})
    if (n % p == 0) return n == p;
  uint64_t d = n - 1;
  int s = 0;
  while (!(d & 1)) {
    d >>= 1;
    ++s;
  }
  for (uint64_t a : {2ull, 3ull, 5ull, 7ull, 11ull, 13ull, 17ull, 19ull, 23ull, 29ull, 31ull, 37ull}) {
    uint64_t x = powmod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool comp = true;
    for (int r = 1; r < s; ++r) {
      x = mulmod(x, x, n);
      if (x == n - 1) {
        comp = false;
        break;
      }
    }
    if (comp) return false;
  }
  return true;
}
uint32_t bitrev(uint32_t x, int bits) {
  uint32_t r = 0;
  for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
  return r;
}
template <typename T>
void put(std::string& s, T v) {
  s.append(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <typename T>
T get(const char*& p, const char* end) {
  if (end - p < (long)sizeof(T)) throw std::runtime_error("CKKS: truncated buffer");
  T v;
  std::memcpy(&v, p, sizeof(T));
  p += sizeof(T);
  return v;
}
std::string read_file(const std::string& f) {
  std::ifstream in(f, std::ios::binary);
  if (!in) throw std::runtime_error("CKKS: cannot open " + f);
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}
void write_file(const std::string& f, const std::string& data) {
  std::ofstream out(f, std::ios::binary | std::ios::trunc);
  if (!out) throw std::runtime_error("CKKS: cannot write " + f);
  out.write(data.data(), (std::streamsize)data.size());
}

// Mixed-radix (Garner) CRT -> centred long double, exact before the final cast.
struct Crt {
  std::vector<uint64_t> q;
  std::vector<std::vector<uint64_t>> inv;  // inv[i][j] = q_i^{-1} mod q_j (i < j)
  explicit Crt(const std::vector<uint64_t>& mods) : q(mods) {
    const size_t L = q.size();
    inv.assign(L, std::vector<uint64_t>(L, 0));
    for (size_t i = 0; i < L; ++i)
      for (size_t j = i + 1; j < L; ++j) inv[i][j] = powmod(q[i] % q[j], q[j] - 2, q[j]);
  }
  // words little-endian multiword integer ops
  static void mul_add(std::vector<uint64_t>& x, uint64_t m, uint64_t a) {
    u128 carry = a;
    for (auto& w : x) {
      const u128 t = (u128)w * m + carry;
      w = (uint64_t)t;
      carry = t >> 64;
    }
    if (carry) x.push_back((uint64_t)carry);
  }
  static int cmp(const std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {
    const size_t n = std::max(a.size(), b.size());
    for (size_t i = n; i-- > 0;) {
      const uint64_t x = i < a.size() ? a[i] : 0, y = i < b.size() ? b[i] : 0;
      if (x != y) return x < y ? -1 : 1;
    }
    return 0;
  }
  static std::vector<uint64_t> sub(const std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {
    std::vector<uint64_t> r(a.size());
    uint64_t borrow = 0;
    for (size_t i = 0; i < a.size(); ++i) {
      const uint64_t y = (i < b.size() ? b[i] : 0);
      const u128 t = (u128)a[i] - (u128)y - (u128)borrow;
      r[i] = (uint64_t)t;
      borrow = (uint64_t)(t >> 64) ? 1 : 0;
    }
    return r;
  }
  static long double to_ld(const std::vector<uint64_t>& x) {
    long double r = 0.0L;
    for (size_t i = x.size(); i-- > 0;) r = r * 18446744073709551616.0L + (long double)x[i];
    return r;
  }
  std::vector<uint64_t> Q() const {
    std::vector<uint64_t> r{1};
    for (auto m : q) mul_add(r, m, 0);
    return r;
  }
  long double centred(const uint64_t* a) const {  // a[j] residues
    const size_t L = q.size();
    std::vector<uint64_t> v(L);
    for (size_t j = 0; j < L; ++j) {
      uint64_t t = a[j] % q[j];
      for (size_t i = 0; i < j; ++i) t = mulmod(submod(t, v[i] % q[j], q[j]), inv[i][j], q[j]);
      v[j] = t;
    }
    std::vector<uint64_t> x;
    // Horner: x = v[L-1]; x = x*q[L-2] + v[L-2]; ... x = x*q0 + v0
    x.assign(1, v[L - 1]);
    for (size_t j = L - 1; j-- > 0;) mul_add(x, q[j], v[j]);
    static thread_local std::vector<uint64_t> Qc, halfQ;
    if (Qc.empty() || Qc != Q()) {
      Qc = Q();
      halfQ = Qc;
      uint64_t carry = 0;
      for (size_t i = halfQ.size(); i-- > 0;) {
        const uint64_t w = halfQ[i];
        halfQ[i] = (w >> 1) | (carry << 63);
        carry = w & 1;
      }
    }
    if (cmp(x, halfQ) > 0) {
      auto y = sub(Qc, x);
      return -to_ld(y);
    }
    return to_ld(x);
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// ChaCha20Rng
void ChaCha20Rng::os_random(void* buf, size_t n) {
  uint8_t* p = static_cast<uint8_t*>(buf);
  while (n) {
    const ssize_t r = getrandom(p, n, 0);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error("getrandom failed");
    }
    p += r;
    n -= (size_t)r;
  }
}

ChaCha20Rng::ChaCha20Rng() {
  os_random(key_, sizeof(key_));
  nonce_[0] = nonce_[1] = 0;
  nonce_[2] = kChaKeygen;
}

ChaCha20Rng::ChaCha20Rng(const uint32_t key[8], uint64_t stream, uint32_t domain) {
  for (int i = 0; i < 8; ++i) key_[i] = key[i];
  nonce_[0] = (uint32_t)stream;
  nonce_[1] = (uint32_t)(stream >> 32);
  nonce_[2] = domain;
}

void ChaCha20Rng::refill() {
  chacha20_block(key_, ctr_, nonce_, buf_);
  if (++ctr_ == 0) {  // 2^32 blocks (256 GiB) on one nonce: move to the next
    if (++nonce_[0] == 0) ++nonce_[1];
  }
  pos_ = 0;
}

uint64_t ChaCha20Rng::next_u64() {
  if (pos_ > 14) refill();
  const uint64_t v = chacha_u64(buf_ + pos_);
  pos_ += 2;
  return v;
}

uint64_t ChaCha20Rng::below(uint64_t q) {
  const uint64_t lim = (~0ULL / q) * q;  // largest multiple of q <= 2^64 - 1
  for (;;) {
    const uint64_t v = next_u64();
    if (v < lim) return v % q;
  }
}

int ChaCha20Rng::ternary() {
  for (;;) {  // exact: reject 3 of a 2-bit draw
    const uint64_t v = next_u64();
    for (int i = 0; i < 32; ++i) {
      const int t = (int)((v >> (2 * i)) & 3u);
      if (t != 3) return t - 1;
    }
  }
}

double ChaCha20Rng::gauss(double sigma) {
  if (has_spare_) {
    has_spare_ = false;
    return spare_ * sigma;
  }
  const double u1 = chacha_unit_open0(next_u64()), u2 = chacha_unit(next_u64());
  const double r = std::sqrt(-2.0 * std::log(u1));
  spare_ = r * std::sin(2.0 * M_PI * u2);
  has_spare_ = true;
  return r * std::cos(2.0 * M_PI * u2) * sigma;
}

void ChaCha20Rng::derive_key(uint32_t out[8]) {
  for (int i = 0; i < 4; ++i) {
    const uint64_t v = next_u64();
    out[2 * i] = (uint32_t)v;
    out[2 * i + 1] = (uint32_t)(v >> 32);
  }
}

CKKS::CKKS(uint32_t batch_size, uint32_t scaling_bits)
    : batch_(batch_size), bits_(scaling_bits) {
  if (batch_size == 0 || (batch_size & (batch_size - 1)))
    throw std::runtime_error("CKKS batch_size must be a power of two");
  if (scaling_bits < 20 || scaling_bits > 58) throw std::runtime_error("CKKS scaling bits in [20,58]");
  N_ = 2 * batch_size;
  slots_ = batch_size;
  setup_primes();
  precompute();
}

void CKKS::setup_primes() {
  const uint64_t M = 2ull * N_;
  auto find_below = [&](int bits, uint64_t below) {
    uint64_t c = ((below - 1) / M) * M + 1;
    if (c >= below) c -= M;
    (void)bits;
    while (!is_prime(c)) c -= M;
    return c;
  };
  q_.clear();
  q_.push_back(find_below(60, 1ull << 60));
  uint64_t b = 1ull << bits_;
  for (int i = 0; i < 2; ++i) {
    uint64_t p = find_below((int)bits_, b);
    if (p == q_[0]) p = find_below((int)bits_, p);
    q_.push_back(p);
    b = p;
  }
}

void CKKS::precompute() {
  const int L = (int)q_.size();
  int logN = 0;
  while ((1u << logN) < N_) ++logN;
  psi_rev_.assign(L, {});
  psi_rev_sh_.assign(L, {});
  ipsi_rev_.assign(L, {});
  ipsi_rev_sh_.assign(L, {});
  ninv_.assign(L, 0);
  ninv_sh_.assign(L, 0);
  for (int l = 0; l < L; ++l) {
    const uint64_t q = q_[l];
    uint64_t psi = 0;
    for (uint64_t x = 2; x < 1000000; ++x) {
      const uint64_t g = powmod(x, (q - 1) / (2ull * N_), q);
      if (powmod(g, N_, q) == q - 1) {
        psi = g;
        break;
      }
    }
    if (!psi) throw std::runtime_error("CKKS: no 2N-th root of unity");
    const uint64_t ipsi = powmod(psi, q - 2, q);
    psi_rev_[l].resize(N_);
    ipsi_rev_[l].resize(N_);
    psi_rev_sh_[l].resize(N_);
    ipsi_rev_sh_[l].resize(N_);
    for (uint32_t k = 0; k < N_; ++k) {
      const uint32_t r = bitrev(k, logN);
      psi_rev_[l][k] = powmod(psi, r, q);
      ipsi_rev_[l][k] = powmod(ipsi, r, q);
      psi_rev_sh_[l][k] = shoup(psi_rev_[l][k], q);
      ipsi_rev_sh_[l][k] = shoup(ipsi_rev_[l][k], q);
    }
    ninv_[l] = powmod(N_, q - 2, q);
    ninv_sh_[l] = shoup(ninv_[l], q);
  }
  // canonical embedding tables (M = 2N)
  const uint64_t M = 2ull * N_;
  rot_.resize(slots_);
  uint64_t r = 1;
  for (uint32_t j = 0; j < slots_; ++j) {
    rot_[j] = r;
    r = (r * 5) % M;
  }
  ksi_re_.resize(M + 1);
  ksi_im_.resize(M + 1);
  for (uint64_t k = 0; k <= M; ++k) {
    const long double a = 2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)M;
    ksi_re_[k] = (double)cosl(a);
    ksi_im_[k] = (double)sinl(a);
  }
}

void CKKS::ntt(uint64_t* a, int l) const {
  const uint64_t q = q_[l];
  const auto& W = psi_rev_[l];
  const auto& Ws = psi_rev_sh_[l];
  uint32_t t = N_;
  for (uint32_t m = 1; m < N_; m <<= 1) {
    t >>= 1;
    for (uint32_t i = 0; i < m; ++i) {
      const uint32_t j1 = 2 * i * t;
      const uint64_t S = W[m + i], Sp = Ws[m + i];
      for (uint32_t j = j1; j < j1 + t; ++j) {
        const uint64_t U = a[j];
        const uint64_t V = mulsh(a[j + t], S, Sp, q);
        a[j] = addmod(U, V, q);
        a[j + t] = submod(U, V, q);
      }
    }
  }
}

void CKKS::intt(uint64_t* a, int l) const {
  const uint64_t q = q_[l];
  const auto& W = ipsi_rev_[l];
  const auto& Ws = ipsi_rev_sh_[l];
  uint32_t t = 1;
  for (uint32_t m = N_; m > 1; m >>= 1) {
    uint32_t j1 = 0;
    const uint32_t h = m >> 1;
    for (uint32_t i = 0; i < h; ++i) {
      const uint64_t S = W[h + i], Sp = Ws[h + i];
      for (uint32_t j = j1; j < j1 + t; ++j) {
        const uint64_t U = a[j], V = a[j + t];
        a[j] = addmod(U, V, q);
        a[j + t] = mulsh(submod(U, V, q), S, Sp, q);
      }
      j1 += 2 * t;
    }
    t <<= 1;
  }
  for (uint32_t j = 0; j < N_; ++j) a[j] = mulsh(a[j], ninv_[l], ninv_sh_[l], q);
}

// HEAAN-style special FFT for the canonical embedding over the slots.
void CKKS::encode(const double* z, size_t n, std::vector<double>& coeffs) const {
  const size_t S = slots_;
  const uint64_t M = 2ull * N_;
  std::vector<std::complex<double>> v(S, {0.0, 0.0});
  for (size_t i = 0; i < n && i < S; ++i) v[i] = {z[i], 0.0};
  for (size_t len = S; len >= 1; len >>= 1) {
    for (size_t i = 0; i < S; i += len) {
      const size_t lenh = len >> 1, lenq = len << 2;
      const uint64_t gap = M / lenq;
      for (size_t j = 0; j < lenh; ++j) {
        const uint64_t idx = (lenq - (rot_[j] % lenq)) * gap;
        const std::complex<double> u = v[i + j] + v[i + j + lenh];
        std::complex<double> w = v[i + j] - v[i + j + lenh];
        w *= std::complex<double>(ksi_re_[idx], ksi_im_[idx]);
        v[i + j] = u;
        v[i + j + lenh] = w;
      }
    }
    if (len == 1) break;
  }
  int bits = 0;
  while ((1u << bits) < S) ++bits;
  for (size_t i = 0; i < S; ++i) {
    const size_t r = bitrev((uint32_t)i, bits);
    if (i < r) std::swap(v[i], v[r]);
  }
  coeffs.assign(N_, 0.0);
  for (size_t i = 0; i < S; ++i) {
    coeffs[i] = v[i].real() / (double)S;
    coeffs[i + S] = v[i].imag() / (double)S;
  }
}

void CKKS::decode(const std::vector<long double>& coeffs, double scale, double* out, size_t n) const {
  const size_t S = slots_;
  const uint64_t M = 2ull * N_;
  std::vector<std::complex<double>> v(S);
  for (size_t i = 0; i < S; ++i)
    v[i] = {(double)(coeffs[i] / scale), (double)(coeffs[i + S] / scale)};
  int bits = 0;
  while ((1u << bits) < S) ++bits;
  for (size_t i = 0; i < S; ++i) {
    const size_t r = bitrev((uint32_t)i, bits);
    if (i < r) std::swap(v[i], v[r]);
  }
  for (size_t len = 2; len <= S; len <<= 1) {
    for (size_t i = 0; i < S; i += len) {
      const size_t lenh = len >> 1, lenq = len << 2;
      const uint64_t gap = M / lenq;
      for (size_t j = 0; j < lenh; ++j) {
        const uint64_t idx = (rot_[j] % lenq) * gap;
        const std::complex<double> u = v[i + j];
        const std::complex<double> w = v[i + j + lenh] * std::complex<double>(ksi_re_[idx], ksi_im_[idx]);
        v[i + j] = u + w;
        v[i + j + lenh] = u - w;
      }
    }
  }
  for (size_t i = 0; i < n; ++i) out[i] = v[i].real();
}

std::vector<double> CKKS::encode_decode_roundtrip(const std::vector<double>& x) const {
  std::vector<double> c;
  encode(x.data(), x.size(), c);
  std::vector<long double> cl(c.begin(), c.end());
  std::vector<double> out(std::min<size_t>(x.size(), slots_));
  decode(cl, 1.0, out.data(), out.size());
  return out;
}

uint64_t CKKS::reduce_signed(long double x, int l) const {
  const long double q = (long double)q_[l];
  long double r = fmodl(x, q);
  if (r < 0) r += q;
  uint64_t u = (uint64_t)r;
  if (u >= q_[l]) u -= q_[l];
  return u;
}

void CKKS::sample_ternary(std::vector<int64_t>& v) {
  for (auto& x : v) x = rng_.ternary();
}

static int64_t clip_round(double g) {
  g = g > 19.2 ? 19.2 : (g < -19.2 ? -19.2 : g);  // 6 sigma
  return (int64_t)llround(g);
}

void CKKS::sample_gauss(std::vector<int64_t>& v) {
  for (auto& x : v) x = clip_round(rng_.gauss(3.2));
}

std::vector<int64_t> CKKS::debug_sample(int kind, size_t n) {
  std::vector<int64_t> v(n);
  if (kind == 0) sample_ternary(v);
  else if (kind == 1) sample_gauss(v);
  else for (auto& x : v) x = (int64_t)rng_.below(q_.empty() ? 1000003ULL : q_[0]) ;
  return v;
}

// ---------------------------------------------------------------------------
void CKKS::gen_crypto_context_and_keys(const std::string& dir) {
  mkdir(dir.c_str(), 0755);
  const int L = (int)q_.size();
  std::vector<int64_t> s(N_), e(N_);
  sample_ternary(s);
  sample_gauss(e);
  sk_.assign((size_t)L * N_, 0);
  pk_a_.assign((size_t)L * N_, 0);
  pk_b_.assign((size_t)L * N_, 0);
  for (int l = 0; l < L; ++l) {
    const uint64_t q = q_[l];
    uint64_t* sl = &sk_[(size_t)l * N_];
    uint64_t* al = &pk_a_[(size_t)l * N_];
    uint64_t* bl = &pk_b_[(size_t)l * N_];
    std::vector<uint64_t> el(N_);
    for (uint32_t i = 0; i < N_; ++i) {
      sl[i] = s[i] < 0 ? q - 1 : (uint64_t)s[i];
      el[i] = e[i] < 0 ? q - (uint64_t)(-e[i]) : (uint64_t)e[i];
      al[i] = rng_.below(q);
    }
    ntt(sl, l);
    ntt(el.data(), l);
    for (uint32_t i = 0; i < N_; ++i) bl[i] = submod(el[i], mulmod(al[i], sl[i], q), q);
  }
  has_pk_ = has_sk_ = true;
  files_.crypto_context_file = dir + "/cryptocontext.txt";
  files_.public_key_file = dir + "/key-public.txt";
  files_.private_key_file = dir + "/key-private.txt";
  files_.eval_mult_key_file = dir + "/key-eval-mult.txt";
  std::string ctx("MCKC");
  put<uint32_t>(ctx, N_);
  put<uint32_t>(ctx, bits_);
  put<uint32_t>(ctx, (uint32_t)L);
  for (auto q : q_) put<uint64_t>(ctx, q);
  write_file(files_.crypto_context_file, ctx);
  auto keyfile = [&](const char* magic, const std::vector<std::vector<uint64_t>*>& polys) {
    std::string k(magic);
    put<uint32_t>(k, N_);
    put<uint32_t>(k, (uint32_t)L);
    for (auto q : q_) put<uint64_t>(k, q);
    for (auto* p : polys) k.append(reinterpret_cast<const char*>(p->data()), p->size() * 8);
    return k;
  };
  write_file(files_.public_key_file, keyfile("MCKP", {&pk_b_, &pk_a_}));
  write_file(files_.private_key_file, keyfile("MCKS", {&sk_}));
  // PWA needs no ciphertext x ciphertext product, hence no relinearisation key;
  // the file is kept for layout parity with the reference (key-eval-mult.txt).
  write_file(files_.eval_mult_key_file, keyfile("MCKE", {}));
}

void CKKS::load_context(const std::string& file) {
  const std::string d = read_file(file);
  const char* p = d.data();
  const char* e = p + d.size();
  if (d.size() < 4 || d.compare(0, 4, "MCKC") != 0) throw std::runtime_error("CKKS: bad context file");
  p += 4;
  const uint32_t N = get<uint32_t>(p, e), bits = get<uint32_t>(p, e), L = get<uint32_t>(p, e);
  std::vector<uint64_t> q(L);
  for (auto& x : q) x = get<uint64_t>(p, e);
  if (N != N_ || bits != bits_ || q != q_) throw std::runtime_error("CKKS: context does not match parameters");
  files_.crypto_context_file = file;
}

static void load_polys(const std::string& file, const char* magic, uint32_t N,
                       const std::vector<uint64_t>& q, std::vector<std::vector<uint64_t>*> outs) {
  const std::string d = read_file(file);
  const char* p = d.data();
  const char* e = p + d.size();
  if (d.size() < 4 || d.compare(0, 4, magic) != 0) throw std::runtime_error("CKKS: bad key file " + file);
  p += 4;
  const uint32_t n = get<uint32_t>(p, e), L = get<uint32_t>(p, e);
  std::vector<uint64_t> qq(L);
  for (auto& x : qq) x = get<uint64_t>(p, e);
  if (n != N || qq != q) throw std::runtime_error("CKKS: key does not match context");
  for (auto* o : outs) {
    o->resize((size_t)L * N);
    const size_t bytes = o->size() * 8;
    if ((size_t)(e - p) < bytes) throw std::runtime_error("CKKS: truncated key");
    std::memcpy(o->data(), p, bytes);
    p += bytes;
  }
}

void CKKS::load_public_key(const std::string& file) {
  load_polys(file, "MCKP", N_, q_, {&pk_b_, &pk_a_});
  has_pk_ = true;
  files_.public_key_file = file;
}

void CKKS::load_private_key(const std::string& file) {
  load_polys(file, "MCKS", N_, q_, {&sk_});
  has_sk_ = true;
  files_.private_key_file = file;
}

void CKKS::load_context_and_keys(const std::string& ctx, const std::string& pk,
                                 const std::string& sk) {
  load_context(ctx);
  if (!pk.empty()) load_public_key(pk);
  if (!sk.empty()) load_private_key(sk);
}

std::string CKKS::encrypt(const std::vector<double>& values) {
  if (!has_pk_) throw std::runtime_error("CKKS: public key not loaded");
  const int L = (int)q_.size();
  const size_t nct = std::max<size_t>(1, (values.size() + slots_ - 1) / slots_);
  std::string out("MCK1");
  put<uint32_t>(out, N_);
  put<uint32_t>(out, (uint32_t)L);
  put<uint32_t>(out, (uint32_t)nct);
  put<double>(out, (double)bits_);
  for (auto q : q_) put<uint64_t>(out, q);
  const size_t hdr = out.size();
  const size_t per_ct = (size_t)2 * L * N_;
  out.resize(hdr + nct * per_ct * 8);
  uint64_t* body = reinterpret_cast<uint64_t*>(&out[hdr]);
  uint32_t ekey[8];  // fresh per encryption; one ChaCha20 stream per ciphertext
  rng_.derive_key(ekey);
  const long double delta = ldexpl(1.0L, (int)bits_);
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t c = 0; c < nct; ++c) {
    ChaCha20Rng rng(ekey, (uint64_t)c, kChaEncrypt);
    auto gauss = [&]() { return clip_round(rng.gauss(3.2)); };
    const size_t off = c * slots_;
    const size_t n = std::min<size_t>(slots_, values.size() > off ? values.size() - off : 0);
    std::vector<double> coeffs;
    encode(values.data() + off, n, coeffs);
    std::vector<int64_t> u(N_), e0(N_), e1(N_);
    for (auto& x : u) x = rng.ternary();
    for (auto& x : e0) x = gauss();
    for (auto& x : e1) x = gauss();
    uint64_t* c0 = body + c * per_ct;
    uint64_t* c1 = c0 + (size_t)L * N_;
    std::vector<uint64_t> ul(N_), t0(N_), t1(N_);
    for (int l = 0; l < L; ++l) {
      const uint64_t q = q_[l];
      for (uint32_t i = 0; i < N_; ++i) {
        ul[i] = u[i] < 0 ? q - 1 : (uint64_t)u[i];
        const long double m = roundl((long double)coeffs[i] * delta) + (long double)e0[i];
        t0[i] = reduce_signed(m, l);
        t1[i] = e1[i] < 0 ? q - (uint64_t)(-e1[i]) : (uint64_t)e1[i];
      }
      ntt(ul.data(), l);
      ntt(t0.data(), l);
      ntt(t1.data(), l);
      const uint64_t* b = &pk_b_[(size_t)l * N_];
      const uint64_t* a = &pk_a_[(size_t)l * N_];
      uint64_t* o0 = c0 + (size_t)l * N_;
      uint64_t* o1 = c1 + (size_t)l * N_;
      for (uint32_t i = 0; i < N_; ++i) {
        o0[i] = addmod(mulmod(b[i], ul[i], q), t0[i], q);
        o1[i] = addmod(mulmod(a[i], ul[i], q), t1[i], q);
      }
    }
  }
  return out;
}

namespace {
struct CtView {
  uint32_t N, L, nct;
  double logscale;
  std::vector<uint64_t> q;
  const uint64_t* body;
};
CtView parse_ct(std::string_view s) {
  const char* p = s.data();
  const char* e = p + s.size();
  if (s.size() < 4 || s.substr(0, 4) != "MCK1") throw std::runtime_error("CKKS: not a ciphertext");
  p += 4;
  CtView v;
  v.N = get<uint32_t>(p, e);
  v.L = get<uint32_t>(p, e);
  v.nct = get<uint32_t>(p, e);
  v.logscale = get<double>(p, e);
  v.q.resize(v.L);
  for (auto& x : v.q) x = get<uint64_t>(p, e);
  const size_t need = (size_t)v.nct * 2 * v.L * v.N * 8;
  if ((size_t)(e - p) != need) throw std::runtime_error("CKKS: ciphertext size mismatch");
  if (((uintptr_t)p & 7) != 0) throw std::runtime_error("CKKS: misaligned ciphertext buffer");
  v.body = reinterpret_cast<const uint64_t*>(p);
  return v;
}
}  // namespace

std::string CKKS::weighted_average(const std::vector<std::string_view>& cts,
                                   const std::vector<double>& weights) const {
  if (cts.empty() || cts.size() != weights.size()) throw std::runtime_error("CKKS: bad PWA inputs");
  std::vector<std::string> aligned;  // copy if the protobuf buffer is not 8-B aligned
  std::vector<CtView> v;
  for (auto& c : cts) {
    try {
      v.push_back(parse_ct(c));
    } catch (const std::runtime_error& err) {
      if (std::string(err.what()).find("misaligned") == std::string::npos) throw;
      aligned.emplace_back(c);
      v.push_back(parse_ct(aligned.back()));
    }
  }
  const CtView& h = v[0];
  for (auto& x : v)
    if (x.N != h.N || x.L != h.L || x.nct != h.nct || x.q != h.q || x.logscale != h.logscale)
      throw std::runtime_error("CKKS: ciphertexts have different parameters");
  std::string out("MCK1");
  put<uint32_t>(out, h.N);
  put<uint32_t>(out, h.L);
  put<uint32_t>(out, h.nct);
  put<double>(out, h.logscale + kWeightBits);
  for (auto q : h.q) put<uint64_t>(out, q);
  const size_t hdr = out.size();
  const size_t total = (size_t)h.nct * 2 * h.L * h.N;
  out.resize(hdr + total * 8);
  uint64_t* o = reinterpret_cast<uint64_t*>(&out[hdr]);
  // w_ij = round(w_i * 2^30) mod q_j with Shoup precomputation (K9 host path)
  std::vector<uint64_t> wq(v.size() * h.L), wqs(v.size() * h.L);
  for (size_t i = 0; i < v.size(); ++i) {
    const long double w = roundl((long double)weights[i] * ldexpl(1.0L, kWeightBits));
    for (uint32_t l = 0; l < h.L; ++l) {
      const long double qq = (long double)h.q[l];
      long double r = fmodl(w, qq);
      if (r < 0) r += qq;
      wq[i * h.L + l] = (uint64_t)r;
      wqs[i * h.L + l] = shoup(wq[i * h.L + l], h.q[l]);
    }
  }
  // K9 on the controller's device (residency: limbs of staged models are read in place)
  if (DeviceAggregator::enabled_for(total * 8 * v.size())) {
    std::vector<const uint64_t*> bodies;
    for (auto& x : v) bodies.push_back(x.body);
    if (DeviceAggregator::get()->ckks_pwa(bodies, wq, wqs, h.q, h.L, h.N, total, o)) return out;
  }
#pragma omp parallel for schedule(static)
  for (size_t k = 0; k < total; k += h.N) {
    const uint32_t limb = (uint32_t)((k / h.N) % h.L);
    const uint64_t q = h.q[limb];
    for (size_t j = k; j < k + h.N; ++j) {
      uint64_t acc = 0;
      for (size_t i = 0; i < v.size(); ++i)
        acc = addmod(acc, mulsh(v[i].body[j], wq[i * h.L + limb], wqs[i * h.L + limb], q), q);
      o[j] = acc;
    }
  }
  return out;
}

std::vector<double> CKKS::decrypt(std::string_view ct, size_t n) const {
  if (!has_sk_) throw std::runtime_error("CKKS: private key not loaded");
  std::string aligned;
  CtView v;
  try {
    v = parse_ct(ct);
  } catch (const std::runtime_error& err) {
    if (std::string(err.what()).find("misaligned") == std::string::npos) throw;
    aligned.assign(ct);
    v = parse_ct(aligned);
  }
  if (v.N != N_ || v.q != q_) throw std::runtime_error("CKKS: ciphertext from another context");
  const int L = (int)v.L;
  std::vector<double> out(n, 0.0);
  const double scale = std::ldexp(1.0, (int)v.logscale);
  Crt crt(q_);
#pragma omp parallel for schedule(dynamic, 1)
  for (size_t c = 0; c < v.nct; ++c) {
    const size_t off = c * slots_;
    if (off >= n) continue;
    const uint64_t* c0 = v.body + c * 2 * L * N_;
    const uint64_t* c1 = c0 + (size_t)L * N_;
    std::vector<uint64_t> m((size_t)L * N_);
    for (int l = 0; l < L; ++l) {
      const uint64_t q = q_[l];
      const uint64_t* s = &sk_[(size_t)l * N_];
      uint64_t* ml = &m[(size_t)l * N_];
      for (uint32_t i = 0; i < N_; ++i) ml[i] = addmod(c0[(size_t)l * N_ + i], mulmod(c1[(size_t)l * N_ + i], s[i], q), q);
      intt(ml, l);
    }
    std::vector<long double> coeffs(N_);
    std::vector<uint64_t> res(L);
    for (uint32_t i = 0; i < N_; ++i) {
      for (int l = 0; l < L; ++l) res[l] = m[(size_t)l * N_ + i];
      coeffs[i] = crt.centred(res.data());
    }
    decode(coeffs, scale, out.data() + off, std::min<size_t>(slots_, n - off));
  }
  return out;
}

}  // namespace mfl
