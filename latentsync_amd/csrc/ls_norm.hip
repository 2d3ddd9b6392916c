// GroupNorm statistics (-> per-(sample, channel) affine consumed by the conv/GEMM
// prologue) and LayerNorm, for gfx950.
//
// GroupNorm: numerically robust single read pass.  Every (sample, group) uses one
// shift k_g = x[first pixel of the sample][first channel of the group], so the
// shifted sums S1 = sum(x - k_g), S2 = sum((x - k_g)^2) of all blocks simply add
// (no cancellation when |mean| >> std, no pairwise merges).  Block = (split,
// sample): threads own 16-B channel chunks and walk pixels with 8 loads in
// flight (enough blocks that the whole tensor is in flight at once); the block
// reduces its per-thread sums to per-group fp64 (S1, S2) in parallel (8 lanes
// per group + shuffles) and adds them into a per-(sample, group) fp64
// accumulator with agent-scope atomics; the last-arriving block of the sample
// (arrival ticket) reads the accumulator, re-zeroes it and writes the
// per-channel affine.  (fp64 sums: the atomic order changes results only at the
// 1e-16 level.)
#include "ls_common.h"

namespace ls {

constexpr int GN_THREADS = 256;
constexpr int GN_MAX_SAMPLES = 1024;
constexpr size_t GN_COUNTER_BYTES = 4096;  // per-sample arrival tickets at the workspace start

struct GnPart { double s1, s2; };  // per-(sample, group) accumulator, zero between calls

__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  const long long b = __double_as_longlong(v);
  const int lo = __shfl_xor((int)(b & 0xffffffffLL), m, 64), hi = __shfl_xor((int)(b >> 32), m, 64);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__global__ void __launch_bounds__(GN_THREADS)
gn_stats_kernel(const u16* __restrict__ x1, const u16* __restrict__ x2, int C1, int C2, long pps, int nsplit,
                int groups, float eps, const float* __restrict__ gamma, const float* __restrict__ beta,
                GnPart* part, unsigned* counters, float* __restrict__ scale, float* __restrict__ shift) {
  extern __shared__ __attribute__((aligned(16))) float gsh[];  // [R][C] S1, [R][C] S2
  __shared__ float kg[64];
  __shared__ float mean_s[64], rstd_s[64];
  __shared__ int is_last;
  const int C = C1 + C2, CC = C / 8;
  const int cpg = C / groups;
  const int split = blockIdx.x, s = blockIdx.y;
  const int tid = threadIdx.x;
  const long p0 = pps * split / nsplit, p1 = pps * (split + 1) / nsplit;
  const long base = (long)s * pps;
  int R, nchunk;
  if (CC <= GN_THREADS) { R = GN_THREADS / CC; nchunk = 1; } else { R = 1; nchunk = (CC + GN_THREADS - 1) / GN_THREADS; }
  float* S1 = gsh;
  float* S2 = gsh + (long)R * C;
  if (tid < groups) {
    const int c = tid * cpg;
    kg[tid] = bf2f(c < C1 ? x1[base * C1 + c] : x2[base * C2 + (c - C1)]);
  }
  __syncthreads();
  for (int q = 0; q < nchunk; ++q) {
    int cc, r;
    if (nchunk == 1) { cc = tid % CC; r = tid / CC; } else { cc = tid + q * GN_THREADS; r = 0; }
    const bool active = (nchunk == 1) ? (tid < R * CC) : (cc < CC);
    if (!active) continue;
    const int c = cc * 8;
    float a1[8], a2[8], k8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a1[j] = 0.f; a2[j] = 0.f; k8[j] = kg[(c + j) / cpg]; }
    const u16* src; int ld;
    if (c < C1) { src = x1 + c; ld = C1; } else { src = x2 + (c - C1); ld = C2; }
    long p = p0 + r;
    for (; p + 7 * R < p1; p += 8 * R) {  // 8 independent loads in flight per thread
      uint4 u[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) u[t] = *(const uint4*)(src + (base + p + t * R) * ld);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        float f[8];
        unpack8(u[t], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = f[j] - k8[j]; a1[j] += d; a2[j] += d * d; }
      }
    }
    for (; p < p1; p += R) {
      float f[8];
      unpack8(*(const uint4*)(src + (base + p) * ld), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = f[j] - k8[j]; a1[j] += d; a2[j] += d * d; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { S1[(long)r * C + c + j] = a1[j]; S2[(long)r * C + c + j] = a2[j]; }
  }
  __syncthreads();
  // ---- block partial per group: L lanes per group, strided over (row, channel) entries
  const int L = groups > 32 ? 4 : 8;
  const int g = tid / L, j = tid % L;
  const int Rv = (nchunk == 1) ? R : 1;
  double b1 = 0.0, b2 = 0.0;
  if (g < groups) {
    const int ne = Rv * cpg;
    for (int e = j; e < ne; e += L) {
      const int r = e / cpg, c = g * cpg + (e - r * cpg);
      b1 += (double)S1[(long)r * C + c];
      b2 += (double)S2[(long)r * C + c];
    }
  }
  for (int off = 1; off < L; off <<= 1) { b1 += shfl_xor_d(b1, off); b2 += shfl_xor_d(b2, off); }
  if (g < groups && j == 0) {
    GnPart* d = &part[(long)s * groups + g];
    __hip_atomic_fetch_add(&d->s1, b1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&d->s2, b2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // ---- the adds are complete (vmcnt drained by every wave), then one lane takes the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(counters + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = (t == (unsigned)(nsplit - 1));
  }
  __syncthreads();
  if (!is_last) return;
  if (tid == 0) __hip_atomic_store(counters + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  if (tid < groups) {
    GnPart* d = &part[(long)s * groups + tid];
    const double t1 = ld_wt(&d->s1), t2 = ld_wt(&d->s2);
    st_wt(&d->s1, 0.0);  // re-zero for the next call
    st_wt(&d->s2, 0.0);
    const double n = (double)pps * cpg;
    const double m1 = t1 / n;
    const double var = fmax(t2 / n - m1 * m1, 0.0);
    mean_s[tid] = (float)((double)kg[tid] + m1);
    rstd_s[tid] = (float)(1.0 / sqrt(var + (double)eps));
  }
  __syncthreads();
  for (int c = tid; c < C; c += GN_THREADS) {
    const int gg = c / cpg;
    const float sc = (gamma ? gamma[c] : 1.f) * rstd_s[gg];
    scale[(long)s * C + c] = sc;
    shift[(long)s * C + c] = (beta ? beta[c] : 0.f) - mean_s[gg] * sc;
  }
}

static int gn_nsplit(int n_samples, long pps, int C) {
  // Every block adds its per-group fp64 partials into one accumulator per (sample,
  // group) with memory-side atomics, which serialise per address: aim for ~512
  // blocks in total (2 per CU keep ~12 MB of loads in flight), i.e. as many pixel
  // rows per thread as that allows (>= 8, one batch of 8 loads).  Measured on the
  // UNet / VAE shapes this halves the 32x32 stats pass (59 -> 28 us, 8 windows).
  const int CC = C / 8;
  const int R = CC <= GN_THREADS ? GN_THREADS / CC : 1;
  long ns = cdiv(512, n_samples);
  ns = std::min<long>(ns, pps / (8L * R));
  return (int)std::max<long>(1, std::min<long>(ns, 4096));
}

// GroupNorm statistics from producer column sums (ls_conv_desc.gn_colsum_out):
// block = (group, sample); the slot sums of the group's channels over the sample's
// slots are added in fp64 (fixed order per thread, then a fixed-shape tree), so
// the result does not depend on scheduling.
__global__ void __launch_bounds__(256)
gn_colsum_finalize_kernel(const float* __restrict__ cs1, const float* __restrict__ cs2, int C1, int C2,
                          long slots_per_sample, int groups, float eps, const float* __restrict__ gamma,
                          const float* __restrict__ beta, float* __restrict__ scale, float* __restrict__ shift) {
  __shared__ double r1[4], r2[4];
  const int C = C1 + C2, cpg = C / groups;
  const int g = blockIdx.x, s = blockIdx.y, tid = threadIdx.x;
  // thread = (channel of the group, slot lane): no integer division in the loop
  const int lanes = 256 / cpg, cl = tid % cpg, sl = tid / cpg;
  double t1 = 0.0, t2 = 0.0;
  if (sl < lanes) {
    const int c = g * cpg + cl;
    const int n = c < C1 ? C1 : C2;
    const float* p = (c < C1 ? cs1 + c : cs2 + (c - C1)) + (long)s * slots_per_sample * 2 * n;
    for (long q = sl; q < slots_per_sample; q += lanes) {
      t1 += (double)p[q * 2 * n];
      t2 += (double)p[q * 2 * n + n];
    }
  }
  for (int off = 32; off > 0; off >>= 1) { t1 += shfl_xor_d(t1, off); t2 += shfl_xor_d(t2, off); }
  if ((tid & 63) == 0) { r1[tid >> 6] = t1; r2[tid >> 6] = t2; }
  __syncthreads();
  if (tid < cpg) {
    const double s1 = (r1[0] + r1[1]) + (r1[2] + r1[3]), s2 = (r2[0] + r2[1]) + (r2[2] + r2[3]);
    const double n = (double)slots_per_sample * LS_GN_SLOT_ROWS * cpg;
    const double mean = s1 / n;
    const double var = fmax(s2 / n - mean * mean, 0.0);
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const int c = g * cpg + tid;
    const float sc = (gamma ? gamma[c] : 1.f) * rstd;
    scale[(long)s * C + c] = sc;
    shift[(long)s * C + c] = (beta ? beta[c] : 0.f) - (float)mean * sc;
  }
}

// Materialised GroupNorm apply (+SiLU) over an optional channel concat.  A thread keeps
// one 8-channel chunk for its whole grid-stride walk over pixels (ppb pixels per block
// pass, C / 8 threads each), so the loop has no 64-bit index division, and it re-reads
// its scale / shift only when the walk crosses into the next sample.
__global__ void __launch_bounds__(256) gn_apply_kernel(const u16* __restrict__ x1, const u16* __restrict__ x2, int C1,
                                                       int C2, long n_pix, long pps, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int silu_on,
                                                       u16* __restrict__ y, int ppb, int ccb) {
  // ppb pixels per block pass, ccb chunks of 8 channels per pixel (blockIdx.y selects which)
  const int C = C1 + C2, CC = C / 8;
  const int pl = threadIdx.x / ccb, cc = blockIdx.y * ccb + threadIdx.x - pl * ccb;
  if (pl >= ppb || cc >= CC) return;
  const int c = cc * 8;
  const u16* src = c < C1 ? x1 + c : x2 + (c - C1);
  const int lds = c < C1 ? C1 : C2;
  long s_cur = -1, s_end = 0;
  float sc[8], sh[8];
  const long step = (long)gridDim.x * ppb;
  for (long pix = (long)blockIdx.x * ppb + pl; pix < n_pix; pix += step) {
    if (pix >= s_end || s_cur < 0) {  // entered another sample (rare: samples span many passes)
      s_cur = pix / pps;
      s_end = (s_cur + 1) * pps;
      const float4 s0 = *(const float4*)(scale + s_cur * C + c), s1 = *(const float4*)(scale + s_cur * C + c + 4);
      const float4 h0 = *(const float4*)(shift + s_cur * C + c), h1 = *(const float4*)(shift + s_cur * C + c + 4);
      sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
      sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
    }
    float f[8];
    unpack8(*(const uint4*)(src + pix * lds), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = fmaf(f[j], sc[j], sh[j]);
      f[j] = silu_on ? silu(t) : t;
    }
    *(uint4*)(y + pix * C + c) = pack8(f);
  }
}

// The same apply with U independent 16-B loads in flight per thread.  gn_apply_kernel's
// grid-stride walk had one load outstanding per thread (~32 KB per CU: latency-bound at
// ~4 TB/s), and its stride (gridDim * ppb pixels) crossed a sample boundary on almost
// every step, so the "rare" scale / shift reload ran every iteration.  Here a block owns
// U * ppb consecutive pixels (thread: pixels base + k ppb + pl, k < U, coalesced rows),
// issues all U loads first, and looks the sample up once per thread (a block spans at
// most a few samples: the host keeps U * ppb <= pps).
template <int U>
__global__ void __launch_bounds__(256) gn_apply_u_kernel(const u16* __restrict__ x1, const u16* __restrict__ x2, int C1,
                                                         int C2, long n_pix, long pps, const float* __restrict__ scale,
                                                         const float* __restrict__ shift, int silu_on,
                                                         u16* __restrict__ y, int ppb, int ccb) {
  const int C = C1 + C2, CC = C / 8;
  const int pl = threadIdx.x / ccb, cc = blockIdx.y * ccb + threadIdx.x - pl * ccb;
  if (pl >= ppb || cc >= CC) return;
  const int c = cc * 8;
  const u16* src = c < C1 ? x1 + c : x2 + (c - C1);
  const int lds = c < C1 ? C1 : C2;
  const long p0 = (long)blockIdx.x * ppb * U + pl;
  uint4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const long pix = p0 + (long)k * ppb;
    v[k] = pix < n_pix ? *(const uint4*)(src + pix * lds) : make_uint4(0, 0, 0, 0);
  }
  long s_cur = p0 / pps, s_end = (s_cur + 1) * pps;
  float sc[8], sh[8];
  load8f(scale + s_cur * C + c, sc);
  load8f(shift + s_cur * C + c, sh);
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const long pix = p0 + (long)k * ppb;
    if (pix >= n_pix) break;
    if (pix >= s_end) {  // (a block's range crossed into the next sample)
      s_cur = pix / pps;
      s_end = (s_cur + 1) * pps;
      load8f(scale + s_cur * C + c, sc);
      load8f(shift + s_cur * C + c, sh);
    }
    float f[8];
    unpack8(v[k], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = fmaf(f[j], sc[j], sh[j]);
      f[j] = silu_on ? silu(t) : t;
    }
    *(uint4*)(y + pix * C + c) = pack8(f);
  }
}

// LayerNorm: 16 lanes per row (4 rows per wave, 16 per block), row cached in
// registers, two-pass mean / variance, 16-lane shuffle reductions.
template <int NCH>
__global__ void __launch_bounds__(256)
layernorm_kernel(const u16* __restrict__ x, long ldx, long rows, int C, float eps, const float* __restrict__ gamma,
                 const float* __restrict__ beta, const float* __restrict__ pe, int pe_rpf, int pe_frames,
                 u16* __restrict__ y, float* __restrict__ stats) {
  const int sub = threadIdx.x & 15;
  const long row = (long)blockIdx.x * 16 + (threadIdx.x >> 4);
  const bool live = row < rows;
  const int CC = C / 8;
  const u16* xr = x + (live ? row : 0) * ldx;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int cc = sub + 16 * q;
    if (cc < CC) {
      unpack8(*(const uint4*)(xr + cc * 8), v[q]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[q][j];
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
  const float mean = s / C;
  float s2 = 0.f;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int cc = sub + 16 * q;
    if (cc < CC) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[q][j] - mean; s2 += d * d; }
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 16);
  const float rstd = rsqrtf(s2 / C + eps);
  if (!live) return;
  if (stats) {  // statistics only (LayerNorm folded into the consumer GEMM)
    if (sub == 0) *(float2*)(stats + 2 * row) = make_float2(mean, rstd);
    return;
  }
  const float* per = pe ? pe + (long)((row / pe_rpf) % pe_frames) * C : nullptr;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int cc = sub + 16 * q;
    if (cc < CC) {
      const int c = cc * 8;
      float g[8], b[8], o[8];
      const float4 g0 = *(const float4*)(gamma + c), g1 = *(const float4*)(gamma + c + 4);
      const float4 b0 = *(const float4*)(beta + c), b1 = *(const float4*)(beta + c + 4);
      g[0] = g0.x; g[1] = g0.y; g[2] = g0.z; g[3] = g0.w; g[4] = g1.x; g[5] = g1.y; g[6] = g1.z; g[7] = g1.w;
      b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (v[q][j] - mean) * rstd * g[j] + b[j];
        if (per) o[j] += per[c + j];
      }
      *(uint4*)(y + row * C + c) = pack8(o);
    }
  }
}

}  // namespace ls

using namespace ls;

extern "C" size_t ls_groupnorm_workspace_bytes(int32_t n_samples, int32_t groups) {
  return GN_COUNTER_BYTES + (size_t)n_samples * groups * sizeof(GnPart);
}

extern "C" int ls_groupnorm(const uint16_t* x1, const uint16_t* x2, int32_t C1, int32_t C2, int32_t n_samples,
                            int64_t pps, int32_t groups, float eps, const float* gamma, const float* beta,
                            float* scale, float* shift, void* workspace, size_t workspace_bytes, void* stream) {
  const int C = C1 + C2;
  if (!x1 || !scale || !shift || n_samples <= 0 || pps <= 0 || groups <= 0)
    return fail(LS_ERR_INVALID, "ls_groupnorm: bad arguments");
  if (C1 % 8 || C2 % 8 || C % groups || groups > 64 || (C2 && !x2))
    return fail(LS_ERR_INVALID, "ls_groupnorm: channels must be multiples of 8 and groups <= 64");
  if (n_samples > GN_MAX_SAMPLES)
    return fail(LS_ERR_INVALID, "ls_groupnorm: too many samples");
  const int ns = gn_nsplit(n_samples, pps, C);
  const size_t need = ls_groupnorm_workspace_bytes(n_samples, groups);
  if (!workspace || workspace_bytes < need) return fail(LS_ERR_WORKSPACE, "ls_groupnorm: workspace too small");
  const int CC = C / 8;
  const int R = CC <= GN_THREADS ? GN_THREADS / CC : 1;
  const size_t shm = 2 * (size_t)R * C * sizeof(float);
  if (shm > 60 * 1024) return fail(LS_ERR_INVALID, "ls_groupnorm: too many channels");
  unsigned* counters = (unsigned*)workspace;  // zero-initialised by the caller once; re-armed by each call
  GnPart* part = (GnPart*)((char*)workspace + GN_COUNTER_BYTES);
  gn_stats_kernel<<<dim3(ns, n_samples), GN_THREADS, shm, (hipStream_t)stream>>>(
      x1, x2, C1, C2, pps, ns, groups, eps, gamma, beta, part, counters, scale, shift);
  return check_launch("gn_stats_kernel");
}

extern "C" int ls_groupnorm_colsum(const float* cs1, const float* cs2, int32_t C1, int32_t C2, int32_t n_samples,
                                   int64_t pps, int32_t groups, float eps, const float* gamma, const float* beta,
                                   float* scale, float* shift, void* stream) {
  const int C = C1 + C2;
  if (!cs1 || !scale || !shift || n_samples <= 0 || pps <= 0 || groups <= 0 || C1 <= 0 || C2 < 0 || (C2 && !cs2))
    return fail(LS_ERR_INVALID, "ls_groupnorm_colsum: bad arguments");
  if (C % groups || C / groups > 256 || pps % LS_GN_SLOT_ROWS)
    return fail(LS_ERR_INVALID, "ls_groupnorm_colsum: C % groups == 0, C / groups <= 256, pix_per_sample % 128 == 0");
  gn_colsum_finalize_kernel<<<dim3(groups, n_samples), 256, 0, (hipStream_t)stream>>>(
      cs1, cs2, C1, C2, pps / LS_GN_SLOT_ROWS, groups, eps, gamma, beta, scale, shift);
  return check_launch("gn_colsum_finalize_kernel");
}

extern "C" int ls_groupnorm_apply(const uint16_t* x1, const uint16_t* x2, int32_t C1, int32_t C2, int64_t n_pix,
                                  int64_t pps, const float* scale, const float* shift, int32_t silu_on, uint16_t* y,
                                  void* stream) {
  if (!x1 || !y || !scale || !shift || (C1 + C2) % 8 || C1 % 8 || n_pix <= 0 || pps <= 0 || (C2 && !x2))
    return fail(LS_ERR_INVALID, "ls_groupnorm_apply: bad arguments");
  const int CC = (C1 + C2) / 8;
  const int ccb = std::min(CC, 256);
  const int ppb = std::max(1, 256 / ccb);
  const int threads = (ppb * ccb + 63) / 64 * 64;  // 1280 channels: 3 waves, 160 live lanes
  static const bool v1 = ls_env("LS_GN_APPLY_V1") != nullptr;  // A/B switch: the grid-stride kernel
  constexpr int U = 4;
  const long ublocks = (n_pix + (long)U * ppb - 1) / ((long)U * ppb);
  // (C >= 1280 -- one pixel per block pass -- stays on the grid-stride kernel: 37 vs 41 us
  // at 8x8 / 32 windows; C <= 640 and the VAE 12-17 % faster, profiles/r03c_gn_apply_ab.txt)
  if (!v1 && ppb >= 2 && (((uintptr_t)scale | (uintptr_t)shift) & 15) == 0 && (long)U * ppb <= pps &&
      ublocks < 0x7fffffffL) {
    gn_apply_u_kernel<U><<<dim3((unsigned)ublocks, cdiv(CC, ccb)), threads, 0, (hipStream_t)stream>>>(
        x1, x2, C1, C2, n_pix, pps, scale, shift, silu_on, y, ppb, ccb);
    return check_launch("gn_apply_u_kernel");
  }
  const long blocks = std::min<long>(cdiv(n_pix, ppb), 16384);
  gn_apply_kernel<<<dim3((unsigned)blocks, cdiv(CC, ccb)), threads, 0, (hipStream_t)stream>>>(
      x1, x2, C1, C2, n_pix, pps, scale, shift, silu_on, y, ppb, ccb);
  return check_launch("gn_apply_kernel");
}

template <int NCH>
static void launch_ln(const uint16_t* x, int64_t ldx, int64_t rows, int32_t C, float eps, const float* gamma, const float* beta,
                      const float* pe, int32_t pe_rpf, int32_t pe_frames, uint16_t* y, hipStream_t s,
                      float* stats = nullptr) {
  layernorm_kernel<NCH><<<cdiv(rows, 16), 256, 0, s>>>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y,
                                                        stats);
}

extern "C" int ls_layernorm(const uint16_t* x, int64_t ldx, int64_t rows, int32_t C, float eps,
                            const float* gamma, const float* beta, const float* pe, int32_t pe_rpf, int32_t pe_frames, uint16_t* y,
                            void* stream) {
  if (!x || !y || !gamma || !beta || C % 8 || C > 16 * 8 * 16 || rows <= 0 || ldx < C || ldx % 8)
    return fail(LS_ERR_INVALID, "ls_layernorm: bad arguments (C % 8 == 0, C <= 2048, ldx >= C, ldx % 8 == 0)");
  if (pe && (pe_rpf <= 0 || pe_frames <= 0)) return fail(LS_ERR_INVALID, "ls_layernorm: bad pe geometry");
  hipStream_t s = (hipStream_t)stream;
  const int nch = cdiv(C / 8, 16);
  if (nch <= 1) launch_ln<1>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  else if (nch <= 2) launch_ln<2>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  else if (nch <= 3) launch_ln<3>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  else if (nch <= 5) launch_ln<5>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  else if (nch <= 8) launch_ln<8>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  else if (nch <= 10) launch_ln<10>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  else if (nch <= 12) launch_ln<12>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  else launch_ln<16>(x, ldx, rows, C, eps, gamma, beta, pe, pe_rpf, pe_frames, y, s);
  return check_launch("layernorm_kernel");
}

extern "C" int ls_row_stats(const uint16_t* x, int64_t ldx, int64_t rows, int32_t C, float eps, float* stats,
                            void* stream) {
  if (!x || !stats || C % 8 || C > 16 * 8 * 16 || rows <= 0 || ldx < C || ldx % 8)
    return fail(LS_ERR_INVALID, "ls_row_stats: bad arguments (C % 8 == 0, C <= 2048, ldx >= C, ldx % 8 == 0)");
  hipStream_t s = (hipStream_t)stream;
  const int nch = cdiv(C / 8, 16);
  if (nch <= 1) launch_ln<1>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  else if (nch <= 2) launch_ln<2>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  else if (nch <= 3) launch_ln<3>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  else if (nch <= 5) launch_ln<5>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  else if (nch <= 8) launch_ln<8>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  else if (nch <= 10) launch_ln<10>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  else if (nch <= 12) launch_ln<12>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  else launch_ln<16>(x, ldx, rows, C, eps, nullptr, nullptr, nullptr, 1, 1, nullptr, s, stats);
  return check_launch("layernorm_kernel(stats)");
}
