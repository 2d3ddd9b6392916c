// Probe: (1) a v_mfma_f32_16x16x32_bf16 result fed straight into a dependent
// v_mfma_f32_16x16x16_bf16 as its accumulator (the d = 40 QK^T split tried in round 3),
// checked against a CPU dot product; (2) cycles per instruction of the two shapes,
// back-to-back on independent accumulators, one wave per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 -o build/mfma_mix_probe scripts/mfma_mix_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static unsigned short f2bf_host(float f) {
  unsigned int u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (unsigned short)(u >> 16);
}
static float bf2f_host(unsigned short h) {
  unsigned int u = (unsigned int)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// A: 16 x 48 (row-major), B: 48 x 16 given as Bt 16 x 48 (row-major, Bt[j][k] = B[k][j]).
// out[i][j] = sum_k A[i][k] B[k][j]; dims 0..31 on 16x16x32, 32..47 on 16x16x16.
// mode 0: chained (16x16x16 reads the 16x16x32 result as srcC); mode 1: separate accumulators
// added on the VALU; mode 2: 16x16x16 first, then 16x16x32 reads it as srcC.
__global__ void mix_kernel(const unsigned short* A, const unsigned short* Bt, float* out, int mode) {
  const int lane = threadIdx.x, lq = lane & 15, lg = lane >> 4;
  uint4 a32 = *(const uint4*)(A + lq * 48 + lg * 8);
  uint4 b32 = *(const uint4*)(Bt + lq * 48 + lg * 8);
  uint2 a16 = *(const uint2*)(A + lq * 48 + 32 + lg * 4);
  uint2 b16 = *(const uint2*)(Bt + lq * 48 + 32 + lg * 4);
  const bf16x8 af = __builtin_bit_cast(bf16x8, a32), bf = __builtin_bit_cast(bf16x8, b32);
  const v4i16 ah = __builtin_bit_cast(v4i16, a16), bh = __builtin_bit_cast(v4i16, b16);
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 c;
  if (mode == 0) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, z, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, c, 0, 0, 0);
  } else if (mode == 1) {
    const f32x4 c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, z, 0, 0, 0);
    const f32x4 c2 = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, z, 0, 0, 0);
    c = c1 + c2;
  } else {
    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, z, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, c, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) out[(4 * lg + r) * 16 + lq] = c[r];
}

template <int SHAPE>  // 0: 16x16x32, 1: 16x16x16
__global__ void __launch_bounds__(256) rate_kernel(float* sink, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a8;
  v4i16 a4;
  for (int e = 0; e < 8; ++e) a8[e] = (__bf16)(0.001f * (lane + e));
  for (int e = 0; e < 4; ++e) a4[e] = (short)(0x3c00 + lane + e);
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (SHAPE == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, a8, acc[i], 0, 0, 0);
      else acc[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, a4, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  unsigned short hA[16 * 48], hB[16 * 48];
  srand(7);
  for (int i = 0; i < 16 * 48; ++i) {
    hA[i] = f2bf_host((rand() / (float)RAND_MAX) * 2.f - 1.f);
    hB[i] = f2bf_host((rand() / (float)RAND_MAX) * 2.f - 1.f);
  }
  double ref[256];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 48; ++k) s += (double)bf2f_host(hA[i * 48 + k]) * bf2f_host(hB[j * 48 + k]);
      ref[i * 16 + j] = s;
    }
  unsigned short *dA, *dB;
  float* dO;
  CK(hipMalloc(&dA, sizeof hA));
  CK(hipMalloc(&dB, sizeof hB));
  CK(hipMalloc(&dO, 256 * 4));
  CK(hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice));
  const char* names[3] = {"chained 32->16", "separate + add", "chained 16->32"};
  for (int mode = 0; mode < 3; ++mode) {
    mix_kernel<<<1, 64>>>(dA, dB, dO, mode);
    CK(hipGetLastError());
    float o[256];
    CK(hipMemcpy(o, dO, sizeof o, hipMemcpyDeviceToHost));
    double maxerr = 0;
    for (int i = 0; i < 256; ++i) maxerr = fmax(maxerr, fabs(o[i] - ref[i]));
    printf("%-16s max |err| vs fp64 dot = %.3e  (%s)\n", names[mode], maxerr, maxerr < 1e-3 ? "ok" : "WRONG");
  }
  int dev;
  hipDeviceProp_t p;
  CK(hipGetDevice(&dev));
  CK(hipGetDeviceProperties(&p, dev));
  const int blocks = p.multiProcessorCount, iters = 20000;
  float* sink;
  CK(hipMalloc(&sink, (size_t)blocks * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int shape = 0; shape < 2; ++shape) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (shape == 0) rate_kernel<0><<<blocks, 256>>>(sink, iters);
      else rate_kernel<1><<<blocks, 256>>>(sink, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double per_simd = (double)iters * 8;  // MFMAs per wave = per SIMD
      const double ns = ms * 1e6 / per_simd;
      if (rep == 1)
        printf("%s: %.3f ms for %d x 8 MFMAs per SIMD -> %.2f ns per MFMA (%.1f cycles at %.2f GHz clock rate)\n",
               shape == 0 ? "16x16x32_bf16" : "16x16x16_bf16", ms, iters, ns, ns * p.clockRate * 1e-6, p.clockRate * 1e-6);
    }
  }
  return 0;
}
