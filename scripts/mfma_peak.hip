// Achieved fp32-MFMA rate on this chip: v_mfma_f32_32x32x2_f32 and
// v_mfma_f32_16x16x4_f32 with C independent accumulator chains per wave and
// W waves per SIMD, no memory traffic.  Calibrates the conv32 kernels'
// ceiling (dependent-accumulator latency, clocks under sustained MFMA load).
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma_peak.hip -o build/tools/mfma_peak
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int C>
__global__ __launch_bounds__(256) void k32(float* out, int iters, float a, float b) {
  f32x16 acc[C];
  for (int c = 0; c < C; ++c)
    for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
  float x = a + threadIdx.x, y = b - threadIdx.x;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[c], 0, 0, 0);
  float s = 0.f;
  for (int c = 0; c < C; ++c)
    for (int e = 0; e < 16; ++e) s += acc[c][e];
  if (s == 123.456f) out[threadIdx.x] = s;
}

template <int C>
__global__ __launch_bounds__(256) void k16(float* out, int iters, float a, float b) {
  f32x4 acc[C];
  for (int c = 0; c < C; ++c)
    for (int e = 0; e < 4; ++e) acc[c][e] = 0.f;
  float x = a + threadIdx.x, y = b - threadIdx.x;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, acc[c], 0, 0, 0);
  float s = 0.f;
  for (int c = 0; c < C; ++c)
    for (int e = 0; e < 4; ++e) s += acc[c][e];
  if (s == 123.456f) out[threadIdx.x] = s;
}

// Co-issue probe: do the f32 matrix pipe and the f32 VALU (v_pk_fma_f32) run
// at the same time?  512-thread workgroups put two waves on every SIMD; with
// `mode` 0 both run MFMA chains, 1 both run VALU chains, 2 wave 0-3 MFMA and
// waves 4-7 VALU.  Every wave does the same instruction count.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(512) void kmix(float* out, int iters, float a, float b, int mode) {
  const int w = threadIdx.x >> 6;
  const bool mm = mode == 0 || (mode == 2 && w < 4);
  float s = 0.f;
  if (mm) {
    f32x16 acc[4];
    for (int c = 0; c < 4; ++c)
      for (int e = 0; e < 16; ++e) acc[c][e] = 0.f;
    float x = a + threadIdx.x, y = b - threadIdx.x;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[c], 0, 0, 0);
    for (int c = 0; c < 4; ++c)
      for (int e = 0; e < 16; ++e) s += acc[c][e];
  } else {
    // 16 packed FMAs per MFMA-slot (64 cycles of VALU = 16 v_pk_fma_f32), 8 chains
    f32x2 acc[8];
    for (int c = 0; c < 8; ++c) acc[c] = f32x2{(float)c, (float)-c};
    const f32x2 x = {a + threadIdx.x, b}, y = {b - threadIdx.x, a};
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = __builtin_elementwise_fma(acc[c], x, y);
    for (int c = 0; c < 8; ++c) s += acc[c][0] + acc[c][1];
  }
  if (s == 123.456f) out[threadIdx.x] = s;
}

void run_mix() {
  float* out;
  (void)hipMalloc(&out, 1024 * sizeof(float));
  const int iters = 2048, grid = 256;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[3] = {"mfma+mfma", "valu+valu", "mfma+valu"};
  for (int mode = 0; mode < 3; ++mode) {
    kmix<<<grid, 512>>>(out, 16, 1.f, 2.f, mode);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) kmix<<<grid, 512>>>(out, iters, 1.f, 2.f, mode);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // per wave per iter: 4 MFMA x 4096 flop, or 64 v_pk_fma x 64 lanes x 4 flop (= same 16384)
    const double flop = 5.0 * grid * 8 * (double)iters * 16384.0;
    printf("%-10s (2 waves/SIMD): %8.1f TF/s  %.3f ms\n", names[mode], flop / (ms * 1e-3) / 1e12, ms / 5);
  }
  (void)hipFree(out);
}

template <typename K>
void run(const char* name, K kern, int blocks_per_cu, int chains, double flop_per_mfma) {
  float* out;
  (void)hipMalloc(&out, 1024 * sizeof(float));
  const int iters = 4096;
  const int grid = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  kern<<<grid, 256>>>(out, 16, 1.f, 2.f);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) kern<<<grid, 256>>>(out, iters, 1.f, 2.f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flop = 5.0 * grid * 4.0 * iters * chains * flop_per_mfma;
  printf("%-10s waves/SIMD %d chains %d: %8.1f TF/s\n", name, blocks_per_cu, chains, flop / (ms * 1e-3) / 1e12);
  (void)hipFree(out);
}

int main() {
  run_mix();
  for (int w = 1; w <= 2; ++w) {
    run("32x32x2", k32<1>, w, 1, 32.0 * 32 * 2 * 2);
    run("32x32x2", k32<2>, w, 2, 32.0 * 32 * 2 * 2);
    run("32x32x2", k32<4>, w, 4, 32.0 * 32 * 2 * 2);
    run("16x16x4", k16<1>, w, 1, 16.0 * 16 * 4 * 2);
    run("16x16x4", k16<2>, w, 2, 16.0 * 16 * 4 * 2);
    run("16x16x4", k16<4>, w, 4, 16.0 * 16 * 4 * 2);
  }
  return 0;
}
