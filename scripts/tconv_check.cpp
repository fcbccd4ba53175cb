// Stand-alone numerics + timing harness for the throughput-regime backward
// convolutions (kernels/tconv.hip): random fp32 operands, packed as the fp32
// path packs them (hi << 16 | lo), sampled outputs of every tile
// configuration against an fp64 reference, then per-call device time at the
// ResNet-18 CIFAR 3x3 shapes: one stream, and the co-located regime (8
// learners' buffers, launches dealt over 4 streams -- the HIP default
// hardware-queue count).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -Imetisfl_amd/csrc \
//     scripts/tconv_check.cpp metisfl_amd/csrc/kernels/tconv.hip -o build/bench/tconv_check
//   build/tconv_check [batch] [iters] [shape index or -1] [sweep 0/1]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

#include "kernels/tconv.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

static uint16_t bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
static float bf16_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static uint32_t split_pack(float a) {
  const uint16_t h = bf16_rne(a);
  const uint16_t l = bf16_rne(a - bf16_f(h));
  return ((uint32_t)h << 16) | l;
}

constexpr int kL = 8, kS = 4;  // co-located learners, streams

struct Bufs {
  uint32_t *xp, *dyp, *wp;
  float *dw, *dx, *ws;
  int* cnt;
};

int main(int argc, char** argv) {
  const int batch = argc > 1 ? atoi(argv[1]) : 32;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  const int only = argc > 3 ? atoi(argv[3]) : -1;
  const int sweep = argc > 4 ? atoi(argv[4]) : 1;
  // profile mode: argv[5] = "w" / "d", argv[6] = cfg, argv[7] = splits: only
  // that kernel, `iters` launches on one stream (for rocprofv3 --pmc passes)
  const char* prof = argc > 5 ? argv[5] : nullptr;
  const int pcfg = argc > 6 ? atoi(argv[6]) : 0, psplit = argc > 7 ? atoi(argv[7]) : 0;
  const int shp[4][2] = {{32, 64}, {16, 128}, {8, 256}, {4, 512}};
  std::mt19937 rng(1234);
  std::normal_distribution<float> nd(0.f, 1.f);
  int fails = 0;
  hipStream_t st[kS];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int si = 0; si < 4; ++si) {
    if (only >= 0 && si != only) continue;
    const int H = shp[si][0], C = shp[si][1];
    mfl::tc::Geom g{batch, H, H, C, C, 3, 1, 1, H, H};
    const int64_t M = (int64_t)g.N * g.P * g.Q;
    const int64_t nx = (int64_t)g.N * g.H * g.W * g.C, ndy = M * g.Co, nw = (int64_t)g.Co * 9 * g.C;
    std::vector<float> x(nx), dy(ndy), w(nw);
    for (auto& v : x) v = nd(rng);
    for (auto& v : dy) v = nd(rng) * 0.01f;
    for (auto& v : w) v = nd(rng) * 0.05f;
    std::vector<uint32_t> xp(nx), dyp(ndy), wp(nw);
    for (int64_t i = 0; i < nx; ++i) xp[i] = split_pack(x[i]);
    for (int64_t i = 0; i < ndy; ++i) dyp[i] = split_pack(dy[i]);
    for (int64_t i = 0; i < nw; ++i) wp[i] = split_pack(w[i]);
    const int64_t wsn = 64 << 20;  // floats, generous for any split plan
    Bufs b[kL];
    for (int l = 0; l < kL; ++l) {
      CK(hipMalloc(&b[l].xp, nx * 4));
      CK(hipMalloc(&b[l].dyp, ndy * 4));
      CK(hipMalloc(&b[l].wp, nw * 4));
      CK(hipMalloc(&b[l].dw, nw * 4));
      CK(hipMalloc(&b[l].dx, nx * 4));
      CK(hipMalloc(&b[l].ws, wsn * 4));
      CK(hipMalloc(&b[l].cnt, 65536 * 4));
      CK(hipMemset(b[l].cnt, 0, 65536 * 4));
      CK(hipMemcpy(b[l].xp, xp.data(), nx * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(b[l].dyp, dyp.data(), ndy * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(b[l].wp, wp.data(), nw * 4, hipMemcpyHostToDevice));
    }
    std::uniform_int_distribution<int64_t> pw(0, nw - 1), px(0, nx - 1);
    auto check_w = [&](const std::vector<float>& dw, int ns) {
      double e = 0;
      for (int sdx = 0; sdx < ns; ++sdx) {
        const int64_t k = sdx < 4 ? (sdx * (nw - 1)) / 3 : pw(rng);
        const int co = (int)(k / (9 * g.C)), rem = (int)(k % (9 * g.C));
        const int r = rem / (3 * g.C), s = (rem / g.C) % 3, c = rem % g.C;
        double ref = 0, mag = 0;
        for (int n = 0; n < g.N; ++n)
          for (int oy = 0; oy < g.P; ++oy)
            for (int ox = 0; ox < g.Q; ++ox) {
              const int iy = oy - 1 + r, ix = ox - 1 + s;
              if (iy < 0 || iy >= g.H || ix < 0 || ix >= g.W) continue;
              const double t = (double)dy[((int64_t)(n * g.P + oy) * g.Q + ox) * g.Co + co] *
                               (double)x[((int64_t)(n * g.H + iy) * g.W + ix) * g.C + c];
              ref += t;
              mag += fabs(t);
            }
        e = std::max(e, fabs(dw[k] - ref) / (mag + 1e-30));
      }
      return e;
    };
    auto check_d = [&](const std::vector<float>& dx, int ns) {
      double e = 0;
      for (int sdx = 0; sdx < ns; ++sdx) {
        const int64_t k = sdx < 4 ? (sdx * (nx - 1)) / 3 : px(rng);
        const int ci = (int)(k % g.C);
        const int64_t pix = k / g.C;
        const int n = (int)(pix / (g.H * g.W)), y = (int)((pix / g.W) % g.H), xx = (int)(pix % g.W);
        double ref = 0, mag = 0;
        for (int r = 0; r < 3; ++r)
          for (int s = 0; s < 3; ++s) {
            const int oy = y + 1 - r, ox = xx + 1 - s;
            if (oy < 0 || oy >= g.P || ox < 0 || ox >= g.Q) continue;
            for (int co = 0; co < g.Co; ++co) {
              const double t = (double)dy[((int64_t)(n * g.P + oy) * g.Q + ox) * g.Co + co] *
                               (double)w[((int64_t)co * 9 + r * 3 + s) * g.C + ci];
              ref += t;
              mag += fabs(t);
            }
          }
        e = std::max(e, fabs(dx[k] - ref) / (mag + 1e-30));
      }
      return e;
    };
    hipEvent_t e0, e1, es[kS];
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& e : es) CK(hipEventCreate(&e));
    // time `fn(l, stream)`: one stream (learner 0), then kL learners over kS streams
    auto timeit = [&](const std::function<void(int, hipStream_t)>& fn, float& single, float& conc) {
      for (int i = 0; i < 3; ++i) fn(0, st[0]);
      CK(hipEventRecord(e0, st[0]));
      for (int i = 0; i < iters; ++i) fn(0, st[0]);
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&single, e0, e1));
      single = single * 1e3f / iters;
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, st[0]));
      for (int s = 1; s < kS; ++s) CK(hipStreamWaitEvent(st[s], e0, 0));
      for (int i = 0; i < iters; ++i)
        for (int l = 0; l < kL; ++l) fn(l, st[l % kS]);
      for (int s = 1; s < kS; ++s) {
        CK(hipEventRecord(es[s], st[s]));
        CK(hipStreamWaitEvent(st[0], es[s], 0));
      }
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&conc, e0, e1));
      conc = conc * 1e3f / (iters * kL);
    };
    const double flop = 2.0 * (double)M * g.Co * 9 * g.C;  // real fp32 FLOP per GEMM
    if (prof) {
      for (int i = 0; i < iters; ++i) {
        if (prof[0] == 'w')
          mfl::tc::launch_wgrad(g, b[0].xp, b[0].dyp, b[0].dw, psplit, st[0], pcfg);
        else
          mfl::tc::launch_dgrad(g, b[0].dyp, b[0].wp, b[0].dx, false, nullptr, b[0].ws, b[0].cnt, psplit, st[0], pcfg);
      }
      CK(hipDeviceSynchronize());
      printf("profiled %s cfg %d splits %d x %d\n", prof, pcfg, psplit, iters);
      continue;
    }
    auto pct = [&](float us) { return 100.0 * 4 * flop / us * 1e-6 / 2500.0; };
    const int targets[] = {64, 128, 256, 512};
    // ---- wgrad ----
    for (int cfg = 0; cfg < mfl::tc::num_wgrad_cfgs(); ++cfg) {
      if (!mfl::tc::wgrad_cfg_fits(g, cfg)) continue;
      CK(hipMemset(b[0].dw, 0, nw * 4));
      mfl::tc::launch_wgrad(g, b[0].xp, b[0].dyp, b[0].dw, 0, st[0], cfg);
      CK(hipDeviceSynchronize());
      std::vector<float> dw(nw);
      CK(hipMemcpy(dw.data(), b[0].dw, nw * 4, hipMemcpyDeviceToHost));
      const double err = check_w(dw, 60);
      fails += err > 1e-5;
      for (int ti = 0; ti < (sweep ? 4 : 1); ++ti) {
        const int M32 = (int)(M / 32);
        int sp = sweep ? std::max(1, targets[ti] / 1) : 0;
        if (sweep) {
          // splits so that tiles x splits ~ target
          CK(hipDeviceSynchronize());
          setenv("MFL_TC_WG_TARGET", std::to_string(targets[ti]).c_str(), 1);
          sp = mfl::tc::wgrad_default_splits(g, cfg);
        }
        (void)M32;
        float t1, tc;
        timeit([&](int l, hipStream_t s) { mfl::tc::launch_wgrad(g, b[l].xp, b[l].dyp, b[l].dw, sp, s, cfg); }, t1,
               tc);
        printf("N=%d %2dx%-2d C=%3d wgrad cfg %d splits %3d | 1-stream %7.2f us (%3.0f%%) | 8 on 4 streams %7.2f us "
               "(%3.0f%%) | err %.1e\n",
               g.N, g.H, g.W, g.C, cfg, sp ? sp : mfl::tc::wgrad_default_splits(g, cfg), t1, pct(t1), tc, pct(tc),
               err);
        fflush(stdout);
      }
    }
    unsetenv("MFL_TC_WG_TARGET");
    // ---- dgrad ----
    for (int cfg = 0; cfg < mfl::tc::num_dgrad_cfgs(); ++cfg) {
      if (!mfl::tc::dgrad_cfg_fits(g, cfg)) continue;
      const int dsp0 = mfl::tc::dgrad_default_splits(g, cfg);
      mfl::tc::launch_dgrad(g, b[0].dyp, b[0].wp, b[0].dx, false, nullptr, b[0].ws, b[0].cnt, dsp0, st[0], cfg);
      CK(hipDeviceSynchronize());
      std::vector<float> dx(nx);
      CK(hipMemcpy(dx.data(), b[0].dx, nx * 4, hipMemcpyDeviceToHost));
      const double err = check_d(dx, 200);
      fails += err > 1e-5;
      for (int ti = 0; ti < (sweep ? 4 : 1); ++ti) {
        if (sweep) setenv("MFL_TC_DG_TARGET", std::to_string(targets[ti]).c_str(), 1);
        const int sp = mfl::tc::dgrad_default_splits(g, cfg);
        float t1, tc;
        timeit(
            [&](int l, hipStream_t s) {
              mfl::tc::launch_dgrad(g, b[l].dyp, b[l].wp, b[l].dx, false, nullptr, b[l].ws, b[l].cnt, sp, s, cfg);
            },
            t1, tc);
        printf("N=%d %2dx%-2d C=%3d dgrad cfg %d splits %3d | 1-stream %7.2f us (%3.0f%%) | 8 on 4 streams %7.2f us "
               "(%3.0f%%) | err %.1e\n",
               g.N, g.H, g.W, g.C, cfg, sp, t1, pct(t1), tc, pct(tc), err);
        fflush(stdout);
      }
    }
    unsetenv("MFL_TC_DG_TARGET");
    for (int l = 0; l < kL; ++l) {
      CK(hipFree(b[l].xp));
      CK(hipFree(b[l].dyp));
      CK(hipFree(b[l].wp));
      CK(hipFree(b[l].dw));
      CK(hipFree(b[l].dx));
      CK(hipFree(b[l].ws));
      CK(hipFree(b[l].cnt));
    }
  }
  printf("%s\n", fails ? "SOME FAILED" : "ALL OK");
  return fails ? 1 : 0;
}
