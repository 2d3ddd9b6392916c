// GroupNorm statistics (-> per-(sample, channel) affine consumed by the conv/GEMM
// prologue) and LayerNorm, for gfx950.
//
// GroupNorm: numerically robust single read pass.  Block = (split, sample); each
// thread owns a fixed 16-B channel chunk and walks pixels, accumulating shifted
// sums S1 = sum(x - k_c), S2 = sum((x - k_c)^2) with k_c the block's first pixel
// (no catastrophic cancellation when |mean| >> std).  The block folds its
// per-channel sums into per-group (n, mean, M2) in double; the finalize kernel
// merges the splits with Chan's formula and emits scale/shift per channel.
#include "ls_common.h"

namespace ls {

constexpr int GN_THREADS = 256;

struct GnPart { double n, mean, m2, pad; };

__global__ void __launch_bounds__(GN_THREADS)
gn_partial_kernel(const u16* __restrict__ x1, const u16* __restrict__ x2, int C1, int C2, long pps, int nsplit,
                  int groups, GnPart* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float gsh[];  // [R][C] S1 then [R][C] S2 then k[C]
  const int C = C1 + C2, CC = C / 8;
  const int split = blockIdx.x, s = blockIdx.y;
  const int tid = threadIdx.x;
  const long p0 = pps * split / nsplit, p1 = pps * (split + 1) / nsplit;
  const long base = (long)s * pps;
  int R, nchunk;
  if (CC <= GN_THREADS) { R = GN_THREADS / CC; nchunk = 1; } else { R = 1; nchunk = (CC + GN_THREADS - 1) / GN_THREADS; }
  float* S1 = gsh;
  float* S2 = gsh + (long)R * C;
  float* kk = gsh + 2L * R * C;
  for (int c = tid; c < C; c += GN_THREADS) {
    const long pix = base + p0;
    kk[c] = (p1 > p0) ? bf2f(c < C1 ? x1[pix * C1 + c] : x2[pix * C2 + (c - C1)]) : 0.f;
  }
  __syncthreads();
  for (int q = 0; q < nchunk; ++q) {
    int cc, r;
    if (nchunk == 1) { cc = tid % CC; r = tid / CC; } else { cc = tid + q * GN_THREADS; r = 0; }
    const bool active = (nchunk == 1) ? (tid < R * CC) : (cc < CC);
    float a1[8], a2[8], k8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a1[j] = 0.f; a2[j] = 0.f; }
    if (active) {
      const int c = cc * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) k8[j] = kk[c + j];
      const u16* src; int ld;
      if (c < C1) { src = x1 + c; ld = C1; } else { src = x2 + (c - C1); ld = C2; }
      for (long p = p0 + r; p < p1; p += R) {
        float f[8];
        unpack8(*(const uint4*)(src + (base + p) * ld), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = f[j] - k8[j]; a1[j] += d; a2[j] += d * d; }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { S1[(long)r * C + c + j] = a1[j]; S2[(long)r * C + c + j] = a2[j]; }
    }
  }
  __syncthreads();
  // per group: combine channels (each channel over R thread rows) in double
  const int cpg = C / groups;
  const double n_c = (double)(p1 - p0);
  for (int g = tid; g < groups; g += GN_THREADS) {
    double tot = 0.0;
    for (int j = 0; j < cpg; ++j) {
      const int c = g * cpg + j;
      double s1 = 0.0;
      for (int r = 0; r < R; ++r) s1 += S1[(long)r * C + c];
      tot += n_c * kk[c] + s1;
    }
    const double n = n_c * cpg;
    const double mean = n > 0 ? tot / n : 0.0;
    double m2 = 0.0;
    for (int j = 0; j < cpg; ++j) {
      const int c = g * cpg + j;
      double s1 = 0.0, s2 = 0.0;
      for (int r = 0; r < R; ++r) { s1 += S1[(long)r * C + c]; s2 += S2[(long)r * C + c]; }
      const double dk = mean - (double)kk[c];
      m2 += s2 - 2.0 * dk * s1 + n_c * dk * dk;
    }
    GnPart o; o.n = n; o.mean = mean; o.m2 = m2; o.pad = 0;
    part[((long)s * nsplit + split) * groups + g] = o;
  }
}

__global__ void gn_finalize_kernel(const GnPart* __restrict__ part, int nsplit, int groups, int C, float eps,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ float mean_s[64], rstd_s[64];
  const int s = blockIdx.x;
  for (int g = threadIdx.x; g < groups; g += blockDim.x) {
    double n = 0.0, mean = 0.0, m2 = 0.0;
    for (int i = 0; i < nsplit; ++i) {
      const GnPart p = part[((long)s * nsplit + i) * groups + g];
      if (p.n <= 0) continue;
      const double nt = n + p.n;
      const double d = p.mean - mean;
      mean += d * p.n / nt;
      m2 += p.m2 + d * d * n * p.n / nt;
      n = nt;
    }
    const double var = n > 0 ? m2 / n : 0.0;
    mean_s[g] = (float)mean;
    rstd_s[g] = (float)(1.0 / sqrt(var + (double)eps));
  }
  __syncthreads();
  const int cpg = C / groups;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const int g = c / cpg;
    const float sc = (gamma ? gamma[c] : 1.f) * rstd_s[g];
    scale[(long)s * C + c] = sc;
    shift[(long)s * C + c] = (beta ? beta[c] : 0.f) - mean_s[g] * sc;
  }
}

static int gn_nsplit(int n_samples, long pps) {
  int ns = cdiv(512, n_samples);
  ns = (int)std::min<long>(ns, std::max<long>(1, pps / 16));
  return std::max(1, std::min(ns, 256));
}

__global__ void affine_act_kernel(const u16* __restrict__ x, long n_chunks, int C, long pps,
                                  const float* __restrict__ scale, const float* __restrict__ shift, int silu_on,
                                  u16* __restrict__ y) {
  const int CC = C / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n_chunks; i += (long)gridDim.x * blockDim.x) {
    const long pix = i / CC;
    const int c = (int)(i - pix * CC) * 8;
    const long s = pix / pps;
    float f[8];
    unpack8(*(const uint4*)(x + pix * C + c), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = f[j] * scale[s * C + c + j] + shift[s * C + c + j];
      f[j] = silu_on ? silu(t) : t;
    }
    *(uint4*)(y + pix * C + c) = pack8(f);
  }
}

// LayerNorm: one wave per row, row cached in registers (C <= 2048), two-pass.
constexpr int LN_MAXCH = 4;  // 16-B chunks per lane -> C <= 64*8*4 = 2048

__global__ void __launch_bounds__(256)
layernorm_kernel(const u16* __restrict__ x, long rows, int C, float eps, const float* __restrict__ gamma,
                 const float* __restrict__ beta, const float* __restrict__ pe, int pe_rpf, int pe_frames,
                 u16* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int CC = C / 8;
  const u16* xr = x + row * C;
  float v[LN_MAXCH][8];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < LN_MAXCH; ++q) {
    const int cc = lane + 64 * q;
    if (cc < CC) {
      unpack8(*(const uint4*)(xr + cc * 8), v[q]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[q][j];
    }
  }
  const float mean = wave_sum(s) / C;
  float s2 = 0.f;
#pragma unroll
  for (int q = 0; q < LN_MAXCH; ++q) {
    const int cc = lane + 64 * q;
    if (cc < CC) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[q][j] - mean; s2 += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(s2) / C + eps);
  const float* per = pe ? pe + (long)((row / pe_rpf) % pe_frames) * C : nullptr;
#pragma unroll
  for (int q = 0; q < LN_MAXCH; ++q) {
    const int cc = lane + 64 * q;
    if (cc < CC) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = cc * 8 + j;
        o[j] = (v[q][j] - mean) * rstd * gamma[c] + beta[c];
        if (per) o[j] += per[c];
      }
      *(uint4*)(y + row * C + cc * 8) = pack8(o);
    }
  }
}

}  // namespace ls

using namespace ls;

extern "C" size_t ls_groupnorm_workspace_bytes(int32_t n_samples, int32_t groups) {
  return (size_t)n_samples * 256 * groups * sizeof(GnPart);
}

extern "C" int ls_groupnorm(const uint16_t* x1, const uint16_t* x2, int32_t C1, int32_t C2, int32_t n_samples,
                            int64_t pps, int32_t groups, float eps, const float* gamma, const float* beta,
                            float* scale, float* shift, void* workspace, size_t workspace_bytes, void* stream) {
  const int C = C1 + C2;
  if (!x1 || !scale || !shift || n_samples <= 0 || pps <= 0 || groups <= 0)
    return fail(LS_ERR_INVALID, "ls_groupnorm: bad arguments");
  if (C1 % 8 || C2 % 8 || C % groups || groups > 64 || (C2 && !x2))
    return fail(LS_ERR_INVALID, "ls_groupnorm: channels must be multiples of 8 and groups <= 64");
  const int ns = gn_nsplit(n_samples, pps);
  const size_t need = (size_t)n_samples * ns * groups * sizeof(GnPart);
  if (!workspace || workspace_bytes < need) return fail(LS_ERR_WORKSPACE, "ls_groupnorm: workspace too small");
  const int CC = C / 8;
  const int R = CC <= GN_THREADS ? GN_THREADS / CC : 1;
  const size_t shm = (2 * (size_t)R * C + C) * sizeof(float);
  if (shm > 64 * 1024) return fail(LS_ERR_INVALID, "ls_groupnorm: too many channels");
  hipStream_t s = (hipStream_t)stream;
  gn_partial_kernel<<<dim3(ns, n_samples), GN_THREADS, shm, s>>>(x1, x2, C1, C2, pps, ns, groups, (GnPart*)workspace);
  int rc = check_launch("gn_partial_kernel");
  if (rc) return rc;
  gn_finalize_kernel<<<n_samples, 256, 0, s>>>((const GnPart*)workspace, ns, groups, C, eps, gamma, beta, scale, shift);
  return check_launch("gn_finalize_kernel");
}

extern "C" int ls_affine_act(const uint16_t* x, int64_t n_pix, int32_t C, int64_t pps, const float* scale,
                             const float* shift, int32_t silu_on, uint16_t* y, void* stream) {
  if (!x || !y || C % 8 || n_pix <= 0) return fail(LS_ERR_INVALID, "ls_affine_act: bad arguments");
  const long n = n_pix * (C / 8);
  affine_act_kernel<<<(int)std::min<long>(cdiv(n, 256), 8192), 256, 0, (hipStream_t)stream>>>(x, n, C, pps, scale, shift,
                                                                                             silu_on, y);
  return check_launch("affine_act_kernel");
}

extern "C" int ls_layernorm(const uint16_t* x, int64_t rows, int32_t C, float eps, const float* gamma,
                            const float* beta, const float* pe, int32_t pe_rpf, int32_t pe_frames, uint16_t* y,
                            void* stream) {
  if (!x || !y || !gamma || !beta || C % 8 || C > 64 * 8 * LN_MAXCH || rows <= 0)
    return fail(LS_ERR_INVALID, "ls_layernorm: bad arguments (C % 8 == 0, C <= 2048)");
  if (pe && (pe_rpf <= 0 || pe_frames <= 0)) return fail(LS_ERR_INVALID, "ls_layernorm: bad pe geometry");
  layernorm_kernel<<<cdiv(rows, 4), 256, 0, (hipStream_t)stream>>>(x, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y);
  return check_launch("layernorm_kernel");
}
