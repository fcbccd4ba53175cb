// LDS-DMA operand staging + MFMA fragment helpers shared by the implicit-GEMM
// convolution (conv.hip) and the large-tile dense GEMM (gemm_big.hip).
// Derivations of the swizzles: conv.hip header comment and swz_* below.
#pragma once
#include "kernels/common.h"

namespace mfl {

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}


// ---- buffer descriptors / LDS-DMA --------------------------------------------
constexpr uint32_t kOOB = 0xFFFFFFF0u;  // offset past every range: reads zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
typedef __attribute__((address_space(3))) void lds_void;
// 16 bytes per lane from `rsrc + off` into LDS at lds_base + 16 * lane
// (lds_base wave-uniform).  Counted by vmcnt, invisible to hipcc's ds waits.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint8_t* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_base, 16, (int)off, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---- swizzles ------------------------------------------------------------------
// Row-major LDS tiles, 16-byte chunks; physical chunk = logical ^ swz(row).
// b128 fragment reads (A of fwd/dgrad, B of fwd): 16 lanes read 16 consecutive
// rows at one logical chunk; 128-B rows -> bank slot (16 B) = 8*(row&1) +
// phys.  swz = (row>>1)&7 makes the 16 slots distinct.
// 256-B rows (BK = 128): one row spans the whole 64-bank window, slot = phys:
// swz = row & 15.
template <int ROWB = 128>
__device__ __forceinline__ int swz_b128(int row) {
  static_assert(ROWB == 64 || ROWB == 128 || ROWB == 256, "b128 swizzle defined for 64/128/256-B rows");
  if constexpr (ROWB == 64) {
    // 64-B rows (BK = 32, gemm_big.hip): slot = 4*(row&3) + phys.  A b128
    // lane group takes 4 rows of each residue class mod 4 at chunks
    // {c, c, c^1, c^1} (e.g. rows 0,12 at c and rows 4,8 at c^1); the key
    // {0,2,3,1}[(row>>2)&3] sends those four to distinct slots for every c.
    return (0x78 >> (2 * ((row >> 2) & 3))) & 3;
  } else if constexpr (ROWB == 128) {
    return (row >> 1) & 7;
  } else {
    return row & 15;
  }
}
// ds_read_b64_tr_b16 reads: 32 lanes per LDS cycle cover rows {R..R+3,
// R+8..R+11} (R % 4 == 0), two 16-B chunks (c0 even, c0+1) each.
//   128-B rows (8 chunks): parity classes of rows need the 4 rows of each
//   class to get distinct even XOR keys: swz = 2*bit1(row) + 4*bit3(row).
//   256-B rows (16 chunks): all 8 rows share one bank window: swz =
//   2*(row&3) + 8*bit3(row).  512-B rows (32 chunks, gemm_big.hip's k-major
//   256-column tiles): bank slot = chunk mod 16, so the same low-4-bit key.
template <int ROWB>
__device__ __forceinline__ int swz_tr(int row) {
  if constexpr (ROWB == 128) return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2);
  else return ((row & 3) << 1) | (((row >> 3) & 1) << 3);
}

typedef short v4s __attribute__((ext_vector_type(4)));
// MFMA B/A fragment from a [k][col] tile via transposing reads: lane gets
// column (col0 + lane%16), k = 8*(lane/16) + 0..7 of the 32-k slice at kk.
//
// The reads are issued through inline asm, NOT __builtin_amdgcn_ds_read_tr16_b64:
// hipcc's waitcnt pass treats the builtin as possibly aliasing every LDS-DMA
// write still in flight and emits s_waitcnt vmcnt(0) in front of the first
// one -- inside a k-loop that drains the whole DMA ring each step (measured:
// conv dgrad / wgrad ran with zero tiles in flight).  The tile being read was
// already made visible by the caller's counted vmcnt + barrier.  The price:
// the compiler no longer tracks these reads, so every fragment must pass
// frags_ready() (an lgkmcnt(0) wait tied to its registers) before use.
__device__ __forceinline__ v4s ds_read_tr_b64(const uint8_t* p) {
  v4s r;
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
template <int ROWB>
__device__ __forceinline__ bf16x8 tr_frag(const uint8_t* tile, int kk, int col0, int lane) {
  const int grp = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int col = col0 + 4 * tp;
  bf16x8 out;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = kk + 8 * grp + 4 * h + tq;
    const int off = row * ROWB + ((((col >> 3) ^ swz_tr<ROWB>(row))) << 4) + ((col & 4) << 1);
    const v4s v = ds_read_tr_b64(tile + off);
    out[4 * h + 0] = v[0];
    out[4 * h + 1] = v[1];
    out[4 * h + 2] = v[2];
    out[4 * h + 3] = v[3];
  }
  return out;
}
// Wait for every outstanding LDS read of this wave, then pin the fragments
// behind the wait (their consumers cannot be scheduled above it).
template <int N>
__device__ __forceinline__ void frags_ready(bf16x8 (&f)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}
// fragment from a [row][k] tile (ROWB-byte rows): lane reads row r0 + lane%16,
// k-chunk (kk/8 + lane/16).
template <int ROWB>
__device__ __forceinline__ bf16x8 b128_frag(const uint8_t* tile, int kk, int r0, int lane) {
  const int row = r0 + (lane & 15);
  const int ch = (kk >> 3) + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(tile + row * ROWB + ((ch ^ swz_b128<ROWB>(row)) << 4));
}

}  // namespace mfl
