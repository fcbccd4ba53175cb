// ChaCha20 (RFC 8439) -- the CSPRNG behind CKKS key generation and
// encryption noise, on the host (he/ckks.cc) and on the device
// (kernels/ckks.hip), replacing the mt19937_64 / splitmix64 generators of
// round 1.  The reference gets this from Palisade's internal PRNG
// (metisfl/encryption/palisade/ckks_scheme.cc:36 KeyGen, :142 Encrypt).
//
// One block function, compiled for both sides (hipcc marks it host+device;
// g++ sees a plain inline function).  Usage pattern:
//   * a 256-bit key drawn from the kernel's entropy pool (getrandom) seeds a
//     host generator per CKKS context;
//   * every encryption draws a FRESH 256-bit key from that generator; each
//     ciphertext c is its own stream (nonce word 0/1 = c, word 2 = domain),
//     and coefficient k of it reads block counter k -- so the device can
//     sample every (c, k) independently and in parallel (counter mode).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MFL_HD __host__ __device__ __forceinline__
#else
#define MFL_HD inline
#endif

namespace mfl {

MFL_HD uint32_t chacha_rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }

#define MFL_CHACHA_QR(a, b, c, d) \
  a += b; d ^= a; d = chacha_rotl(d, 16); \
  c += d; b ^= c; b = chacha_rotl(b, 12); \
  a += b; d ^= a; d = chacha_rotl(d, 8);  \
  c += d; b ^= c; b = chacha_rotl(b, 7);

// RFC 8439 section 2.3: 64-byte block for (key, 32-bit counter, 96-bit nonce)
MFL_HD void chacha20_block(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                    counter, nonce[0], nonce[1], nonce[2]};
  uint32_t x[16];
  for (int i = 0; i < 16; ++i) x[i] = s[i];
  for (int r = 0; r < 10; ++r) {
    MFL_CHACHA_QR(x[0], x[4], x[8], x[12])
    MFL_CHACHA_QR(x[1], x[5], x[9], x[13])
    MFL_CHACHA_QR(x[2], x[6], x[10], x[14])
    MFL_CHACHA_QR(x[3], x[7], x[11], x[15])
    MFL_CHACHA_QR(x[0], x[5], x[10], x[15])
    MFL_CHACHA_QR(x[1], x[6], x[11], x[12])
    MFL_CHACHA_QR(x[2], x[7], x[8], x[13])
    MFL_CHACHA_QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}
#undef MFL_CHACHA_QR

// Stream domains (nonce word 2): which quantity a stream samples.
enum ChaChaDomain : uint32_t { kChaKeygen = 0x6b657967u, kChaEncrypt = 0x656e6372u };

MFL_HD uint64_t chacha_u64(const uint32_t* w) { return (uint64_t)w[0] | ((uint64_t)w[1] << 32); }
// 53-bit uniform in (0, 1] / [0, 1)
MFL_HD double chacha_unit_open0(uint64_t v) { return ((double)(v >> 11) + 1.0) * (1.0 / 9007199254740992.0); }
MFL_HD double chacha_unit(uint64_t v) { return (double)(v >> 11) * (1.0 / 9007199254740992.0); }
// {-1, 0, 1} from a 64-bit uniform (bias < 2^-62)
MFL_HD int chacha_ternary(uint64_t v) { return (int)(v % 3u) - 1; }

}  // namespace mfl
