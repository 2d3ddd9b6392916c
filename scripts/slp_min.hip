// Minimal stand-alone reproducer for the SLP question: the row-block
// GEMM's LayerNorm-in-registers prologue followed by MFMAs on those registers, with
// nothing else -- no LDS, no DMA, no inline asm, no barriers.  Each wave loads 32 rows x
// 320 bf16 into registers, normalises them in place ((x - mean) * rstd as fmaf, which
// SLP packs into v_pk_fma_f32 with op_sel), then multiplies by 64 W rows read straight
// from global memory with v_mfma_f32_16x16x32_bf16 and stores fp32.  The host checks
// every element against a CPU reference (same bf16 rounding of the normalised rows)
// over repeated launches.
// Modes (argv[2]) bisect the failure:
//   0  LayerNorm in registers, then MFMAs on those registers (the row-block prologue)
//   1  LayerNorm in registers, stored straight back as bf16 (no MFMA)
//   2  as 0, but the LayerNorm written as explicit float2 pair arithmetic (no op_sel broadcast)
//   3  as 0, with a scheduling barrier between the LayerNorm and the first MFMA
//   4  as 2, with rstd / -mean*rstd read as duplicated pairs from memory (no op_sel)
//   5  v_pk_fma_f32 written out (inline asm), low-half broadcast: op_sel_hi:[1,0,0]
//   6  v_pk_fma_f32 written out, high-half broadcast: op_sel:[0,1,1] op_sel_hi:[1,1,1]
//   7  v_pk_fma_f32 written out with the compiler's failing form: op_sel:[0,1,0] op_sel_hi:[1,1,0]
//   hipcc --offload-arch=gfx950 -O3 [-fslp-vectorize | -fno-slp-vectorize] slp_min.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int K = 320, KT = K / 32, N = 64, FM = 2;

template <int MODE>
__global__ void __launch_bounds__(512) ln_mfma(const unsigned short* x, const float2* stats, const unsigned short* w,
                                               float* y, unsigned short* xn, const float4* st4) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, l16 = lane & 15, lg = lane >> 4;
  const long m0 = (long)blockIdx.x * 256 + wid * 32;
  bf16x8 ar[FM][KT];
  float2 st[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    st[i] = stats[m0 + i * 16 + l16];
#pragma unroll
    for (int s = 0; s < KT; ++s) ar[i][s] = *(const bf16x8*)(x + (m0 + i * 16 + l16) * K + s * 32 + lg * 8);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const float rstd = st[i].y, nmr = -st[i].x * st[i].y;
    float4 q4 = {rstd, rstd, nmr, nmr};
    if constexpr (MODE == 4) q4 = st4[m0 + i * 16 + l16];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      bf16x8 v = ar[i][s];
      if constexpr (MODE >= 5) {
        const f32x2 lo_r = {rstd, 0.f}, lo_n = {nmr, 0.f}, hi_r = {0.f, rstd}, hi_n = {0.f, nmr};
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          f32x2 t = {(float)v[e], (float)v[e + 1]}, u;
          if constexpr (MODE == 5)
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(u) : "v"(t), "v"(lo_r), "v"(lo_n));
          else if constexpr (MODE == 6)
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[1,1,1]" : "=v"(u) : "v"(t), "v"(hi_r), "v"(hi_n));
          else
            asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,0]" : "=v"(u) : "v"(t), "v"(hi_r), "v"(lo_n));
          v[e] = (__bf16)u[0];
          v[e + 1] = (__bf16)u[1];
        }
      } else if constexpr (MODE == 2 || MODE == 4) {
        const f32x2 r2 = {q4.x, q4.y}, n2 = {q4.z, q4.w};
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          f32x2 t = {(float)v[e], (float)v[e + 1]};
          t = __builtin_elementwise_fma(t, r2, n2);
          v[e] = (__bf16)t[0];
          v[e + 1] = (__bf16)t[1];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (__bf16)fmaf((float)v[e], rstd, nmr);
      }
      ar[i][s] = v;
    }
  }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int s = 0; s < KT; ++s) *(bf16x8*)(xn + (m0 + i * 16 + l16) * K + s * 32 + lg * 8) = ar[i][s];
    return;
  }
  if constexpr (MODE == 3) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < N / 16; ++j) {
    f32x4 acc[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      const bf16x8 bw = *(const bf16x8*)(w + (j * 16 + l16) * K + s * 32 + lg * 8);
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw, ar[i][s], acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) y[(m0 + i * 16 + l16) * N + j * 16 + 4 * lg + r] = acc[i][r];
  }
}

static unsigned short f2bf(float f) {  // round to nearest even
  unsigned u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
static float bf2f(unsigned short h) {
  unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

int main(int argc, char** argv) {
  const int M = 65536, runs = argc > 1 ? atoi(argv[1]) : 16, mode = argc > 2 ? atoi(argv[2]) : 0;
  std::vector<unsigned short> hx((size_t)M * K), hw((size_t)N * K);
  std::vector<float2> hs(M);
  srand(1);
  auto rnd = [] { return (float)rand() / (float)RAND_MAX * 2.f - 1.f; };
  for (auto& v : hx) v = f2bf(rnd() * 3.f + 2.f);
  for (auto& v : hw) v = f2bf(rnd() * 0.1f);
  for (int m = 0; m < M; ++m) {
    double s1 = 0, s2 = 0;
    for (int k = 0; k < K; ++k) { double v = bf2f(hx[(size_t)m * K + k]); s1 += v; s2 += v * v; }
    const double mean = s1 / K, var = s2 / K - mean * mean;
    hs[m] = make_float2((float)mean, (float)(1.0 / sqrt(var + 1e-5)));
  }
  // reference: the normalised rows rounded to bf16 as the kernel does, fp64 dot products
  std::vector<float> ref((size_t)M * N);
  std::vector<unsigned short> refn((size_t)M * K);
  std::vector<float> a(K);
  for (int m = 0; m < M; ++m) {
    const float rstd = hs[m].y, nmr = -hs[m].x * hs[m].y;
    for (int k = 0; k < K; ++k) {
      refn[(size_t)m * K + k] = f2bf(fmaf(bf2f(hx[(size_t)m * K + k]), rstd, nmr));
      a[k] = bf2f(refn[(size_t)m * K + k]);
    }
    for (int n = 0; n < N; ++n) {
      double t = 0;
      for (int k = 0; k < K; ++k) t += (double)a[k] * bf2f(hw[(size_t)n * K + k]);
      ref[(size_t)m * N + n] = (float)t;
    }
  }
  unsigned short *dx, *dw, *dn;
  float2* ds;
  float* dy;
  (void)hipMalloc(&dx, hx.size() * 2);
  (void)hipMalloc(&dw, hw.size() * 2);
  (void)hipMalloc(&ds, M * sizeof(float2));
  (void)hipMalloc(&dy, (size_t)M * N * 4);
  (void)hipMalloc(&dn, hx.size() * 2);
  std::vector<float4> h4(M);
  for (int m = 0; m < M; ++m) h4[m] = make_float4(hs[m].y, hs[m].y, -hs[m].x * hs[m].y, -hs[m].x * hs[m].y);
  float4* d4;
  (void)hipMalloc(&d4, M * sizeof(float4));
  (void)hipMemcpy(d4, h4.data(), M * sizeof(float4), hipMemcpyHostToDevice);
  (void)hipMemcpy(dx, hx.data(), hx.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dw, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, hs.data(), M * sizeof(float2), hipMemcpyHostToDevice);
  std::vector<float> hy((size_t)M * N), first;
  std::vector<unsigned short> hn(hx.size()), firstn;
  long bad_total = 0, diff_total = 0;
  for (int r = 0; r < runs; ++r) {
    if (mode == 0) ln_mfma<0><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    else if (mode == 1) ln_mfma<1><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    else if (mode == 2) ln_mfma<2><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    else if (mode == 3) ln_mfma<3><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    else if (mode == 4) ln_mfma<4><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    else if (mode == 5) ln_mfma<5><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    else if (mode == 6) ln_mfma<6><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    else ln_mfma<7><<<M / 256, 512>>>(dx, ds, dw, dy, dn, d4);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    long bad = 0;
    if (mode == 1) {
      (void)hipMemcpy(hn.data(), dn, hn.size() * 2, hipMemcpyDeviceToHost);
      for (size_t i = 0; i < hn.size(); ++i) bad += hn[i] != refn[i];
      if (firstn.empty()) firstn = hn;
      else for (size_t i = 0; i < hn.size(); ++i) diff_total += hn[i] != firstn[i];
    } else {
      (void)hipMemcpy(hy.data(), dy, hy.size() * 4, hipMemcpyDeviceToHost);
      for (size_t i = 0; i < hy.size(); ++i)
        if (!(fabsf(hy[i] - ref[i]) <= 1e-3f + 1e-3f * fabsf(ref[i]))) ++bad;
      if (first.empty()) first = hy;
      else for (size_t i = 0; i < hy.size(); ++i) diff_total += hy[i] != first[i];
    }
    bad_total += bad;
  }
  printf("mode %d, %d runs x %d rows: elements off the reference %ld, run-to-run differing %ld\n", mode, runs, M, bad_total,
         diff_total);
  return bad_total || diff_total ? 1 : 0;
}
