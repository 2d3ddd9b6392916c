// Paste-back warp on gfx950: LipsyncPipeline.restore_video
// (latentsync/pipelines/lipsync_pipeline.py:343-358) and AlignRestore.restore_img
// (latentsync/utils/affine_transform.py:85-115), batched over the frames of a clip.
//
// The reference runs this per frame on the host: torchvision resize, then OpenCV
// warpAffine (Lanczos4 + bilinear), two erodes, a Gaussian blur and a blend, all
// over the whole video frame.  Here every frame is one z-slice of each launch and
// the work is confined to a per-frame region of interest (the face's footprint in
// the frame plus the erode/blur reach, computed by the host from the affine
// matrix); pixels outside it are the frame unchanged (soft mask 0), so the frames
// are updated in place.  All of it is HBM/L2-bound integer and fp32 work:
//   face_resize_kernel     torchvision resize(antialias=True) + u8, (N,fh,fw,3)
//   restore_mask_kernel    warped-ones bilinear mask -> 2x2 erode -> mask_e, area
//   erode_rows/cols        (2 w_edge)^2 rectangular erode (separable min)
//   blur_rows_kernel       Gaussian row pass (BORDER_REFLECT_101)
//   blur_cols_blend_kernel Gaussian column pass + Lanczos4 face sample + blend
// Arithmetic follows OpenCV's fixed-point warp (AB_BITS 10, 32 sub-pixel steps,
// 15-bit Lanczos coefficients) and its float32 operation order, so the kernels
// reproduce the CPU restatement (oracle/restore_cpu.py) bit for bit.
#include "ls_common.h"

#include <cmath>
#include <vector>

// HIP compiles with -ffp-contract=fast-honor-pragmas: without this, a*b + c pairs of the
// blur / blend are
// fused into FMAs and the float results drift by an ulp from OpenCV's separate
// multiply-add order (1-LSB uint8 flips where a blend lands on an integer).  Explicit
// fmaf() (the torch resize) is unaffected.
#pragma clang fp contract(off)

namespace ls {

constexpr int RS_TAB = 32;              // INTER_TAB_SIZE
constexpr int RS_LANCZOS_BYTES = RS_TAB * RS_TAB * 64 * 2;

// ---------------------------------------------------------------- host tables

// cv::interpolateLanczos4
static void lanczos4_coeffs(float x, float* c) {
  if (x < 1.1920928955078125e-07f) {
    for (int i = 0; i < 8; ++i) c[i] = 0.f;
    c[3] = 1.f;
    return;
  }
  const double s45 = 0.70710678118654752440084436210485;
  const double cs[8][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
  const double y0 = -((double)x + 3) * M_PI * 0.25, s0 = std::sin(y0), c0 = std::cos(y0);
  float sum = 0.f;
  for (int i = 0; i < 8; ++i) {
    const double yy = (double)x + 3 - i;
    if (std::fabs(yy) >= 1e-6) {
      const double y = -yy * M_PI * 0.25;
      c[i] = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (y * y));
    } else {
      c[i] = 1e30f;
    }
    sum += c[i];
  }
  const float inv = 1.f / sum;
  for (int i = 0; i < 8; ++i) c[i] *= inv;
}

// initInterTab2D(INTER_LANCZOS4, fixed point): [fy*32+fx][k1*8+k2] int16, each
// 64-tap kernel nudged to sum exactly 1 << 15.
static void lanczos4_tab(int16_t* out) {
  float t1[RS_TAB][8];
  for (int i = 0; i < RS_TAB; ++i) lanczos4_coeffs((float)i * (1.f / RS_TAB), t1[i]);
  for (int i = 0; i < RS_TAB; ++i)
    for (int j = 0; j < RS_TAB; ++j) {
      int it[64], isum = 0;
      for (int k1 = 0; k1 < 8; ++k1)
        for (int k2 = 0; k2 < 8; ++k2) {
          const float v = t1[i][k1] * t1[j][k2];
          int r = (int)std::nearbyint((double)v * 32768.0);
          r = r < -32768 ? -32768 : (r > 32767 ? 32767 : r);
          it[k1 * 8 + k2] = r;
          isum += r;
        }
      if (isum != 32768) {
        const int diff = isum - 32768;
        int mk1 = 4, mk2 = 4, Mk1 = 4, Mk2 = 4;
        for (int k1 = 4; k1 < 6; ++k1)
          for (int k2 = 4; k2 < 6; ++k2) {
            if (it[k1 * 8 + k2] < it[mk1 * 8 + mk2]) {
              mk1 = k1; mk2 = k2;
            } else if (it[k1 * 8 + k2] > it[Mk1 * 8 + Mk2]) {
              Mk1 = k1; Mk2 = k2;
            }
          }
        if (diff < 0) it[Mk1 * 8 + Mk2] -= diff;
        else it[mk1 * 8 + mk2] -= diff;
      }
      for (int k = 0; k < 64; ++k) out[(i * RS_TAB + j) * 64 + k] = (int16_t)it[k];
    }
}

// getGaussianKernel(n, 0, CV_32F) (getGaussianKernelBitExact's formula, libm exp)
static void gaussian_kernel(int n, float* g) {
  static const float small[4][7] = {{1.f},
                                    {0.25f, 0.5f, 0.25f},
                                    {0.0625f, 0.25f, 0.375f, 0.25f, 0.0625f},
                                    {0.03125f, 0.109375f, 0.21875f, 0.28125f, 0.21875f, 0.109375f, 0.03125f}};
  if ((n & 1) && n <= 7) {
    for (int i = 0; i < n; ++i) g[i] = small[n >> 1][i];
    return;
  }
  const double sigma = n * 0.15 + 0.35, scale2x = -0.125 / (sigma * sigma);
  const int n2 = (n - 1) / 2;
  std::vector<double> vals(n2 + 1);
  double s = 0.0;
  for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
    vals[i] = std::exp((double)(x * x) * scale2x);
    s += vals[i];
  }
  s = s * 2 + 1.0;
  if (!(n & 1)) s += 1.0;
  const double mul = 1.0 / s;
  for (int i = 0; i < n2; ++i) g[i] = g[n - 1 - i] = (float)(vals[i] * mul);
  g[n2] = (float)mul;
  if (!(n & 1)) g[n2 + 1] = g[n2];
}

static size_t gauss_stride(int w_max) { return (size_t)(2 * w_max + 1); }

// ---------------------------------------------------------------- device helpers

struct WarpPt {
  int sx, sy, fxy;
};

// WarpAffineInvoker (imgwarp.cpp): X = (round((M1 y + M2) 2^10) + 16 + round(M0 x 2^10)) >> 5,
// integer part saturated to int16, 5-bit fractions -> table index fy*32 + fx.
// Double ops are written out (no FMA contraction) to match the host.
__device__ __forceinline__ WarpPt warp_point(const double* M, int x, int y) {
  const int X0 = __double2int_rn((((M[1] * (double)y) + M[2]) * 1024.0)) + 16;
  const int Y0 = __double2int_rn((((M[4] * (double)y) + M[5]) * 1024.0)) + 16;
  const int X = (X0 + __double2int_rn(((M[0] * (double)x) * 1024.0))) >> 5;
  const int Y = (Y0 + __double2int_rn(((M[3] * (double)x) * 1024.0))) >> 5;
  WarpPt p;
  p.sx = min(max(X >> 5, -32768), 32767);
  p.sy = min(max(Y >> 5, -32768), 32767);
  p.fxy = (Y & 31) * 32 + (X & 31);
  return p;
}

// cv2.warpAffine(ones(fh, fw) f32, ., INTER_LINEAR, BORDER_CONSTANT 0) at (x, y):
// sum of the bilinear weights of the in-source taps (every product and partial sum
// is a multiple of 2^-10 <= 1: exact in any order).
__device__ __forceinline__ float warped_ones(const double* M, int x, int y, int fh, int fw) {
  const WarpPt p = warp_point(M, x, y);
  const float fx = (float)(p.fxy & 31) * (1.f / 32), fy = (float)(p.fxy >> 5) * (1.f / 32);
  const float wx[2] = {1.f - fx, fx}, wy[2] = {1.f - fy, fy};
  float acc = 0.f;
#pragma unroll
  for (int dy = 0; dy < 2; ++dy)
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const bool ok = (unsigned)(p.sy + dy) < (unsigned)fh && (unsigned)(p.sx + dx) < (unsigned)fw;
      acc = acc + (ok ? wy[dy] * wx[dx] : 0.f);
    }
  return acc;
}

__device__ __forceinline__ int reflect101(int p, int n) {
  p = p < 0 ? -p : p;
  return p >= n ? 2 * n - p - 2 : p;
}

struct RoiView {
  int x0, y0, w, h;
};

__device__ __forceinline__ RoiView roi_of(const int32_t* roi, int n) {
  const int4 r = ((const int4*)roi)[n];
  RoiView v;
  v.x0 = r.x; v.y0 = r.y; v.w = r.z - r.x; v.h = r.w - r.y;
  return v;
}

// w_edge = int(sqrt(area)) // 20 (affine_transform.py:103), capped by the host bound
__device__ __forceinline__ int w_edge_of(const double* area, int n, int w_max) {
  const float a = (float)area[n];
  return min((int)__fsqrt_rn(a) / 20, w_max);
}

// ---------------------------------------------------------------- kernels

// torchvision resize(face, (out_h, out_w), antialias=True) == aten
// _upsample_bilinear2d_aa (separable: width pass, then height pass, float), then
// (x / 2 + 0.5).clamp(0, 1) * 255 -> uint8 (lipsync_pipeline.py:351-354).
// Weight arithmetic mirrors aten's _compute_weights_aa (float, with its double
// promotions of the +0.5 terms); accumulation t = src0 w0, t = fma(src_j, w_j, t).
constexpr int AA_MAXT = 16;

__device__ int aa_weights(int i, int in_size, int out_size, float* w, int* xmin_out) {
  const float scale = (float)in_size / (float)out_size;
  const float support = scale >= 1.f ? scale : 1.f;  // interp_size 2 * 0.5 * scale
  const float center = (float)((double)scale * ((double)i + 0.5));
  const float invscale = scale >= 1.f ? 1.f / scale : 1.f;
  const int xmin = max((int)((double)(center - support) + 0.5), 0);
  int xsize = min((int)((double)(center + support) + 0.5), in_size) - xmin;
  xsize = min(max(xsize, 0), AA_MAXT);
  float total = 0.f;
  for (int j = 0; j < xsize; ++j) {
    float x = (float)(((double)((float)(j + xmin) - center) + 0.5) * (double)invscale);
    x = fabsf(x);
    const float v = x < 1.f ? 1.f - x : 0.f;
    w[j] = v;
    total += v;
  }
  if (total != 0.f)
    for (int j = 0; j < xsize; ++j) w[j] /= total;
  *xmin_out = xmin;
  return xsize;
}

__global__ void __launch_bounds__(256) face_resize_kernel(const float* __restrict__ faces, int in_h, int in_w,
                                                          int out_h, int out_w, uint8_t* __restrict__ out) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int n = blockIdx.z;
  if (x >= out_w || y >= out_h) return;
  float wx[AA_MAXT], wy[AA_MAXT];
  int x0, y0, nx, ny;
  if (in_w != out_w) {
    nx = aa_weights(x, in_w, out_w, wx, &x0);
  } else {
    nx = 1; x0 = x; wx[0] = 1.f;
  }
  if (in_h != out_h) {
    ny = aa_weights(y, in_h, out_h, wy, &y0);
  } else {
    ny = 1; y0 = y; wy[0] = 1.f;
  }
  const bool hpass = in_w != out_w, vpass = in_h != out_h;
  uint8_t res[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float* src = faces + ((long)n * 3 + c) * in_h * in_w;
    float v = 0.f;
    for (int j = 0; j < ny; ++j) {
      const float* row = src + (long)(y0 + j) * in_w + x0;
      float h = row[0];
      if (hpass) {
        h = row[0] * wx[0];
        for (int i = 1; i < nx; ++i) h = fmaf(row[i], wx[i], h);
      }
      if (!vpass) v = h;
      else v = j == 0 ? h * wy[0] : fmaf(h, wy[j], v);
    }
    float f = v / 2.f + 0.5f;
    f = fminf(fmaxf(f, 0.f), 1.f) * 255.f;
    res[c] = (uint8_t)(int)f;
  }
  uint8_t* o = out + (((long)n * out_h + y) * out_w + x) * 3;
  o[0] = res[0]; o[1] = res[1]; o[2] = res[2];
}

// mask_e = erode2x2(warpAffine(ones)) over the ROI (affine_transform.py:96-100), and
// area[n] += sum(mask_e) (fp64; the reference sums in float32).
__global__ void __launch_bounds__(256) restore_mask_kernel(const double* __restrict__ warp,
                                                           const int32_t* __restrict__ roi, int H, int W, int fh,
                                                           int fw, int ld_w, int ld_h, float* __restrict__ mask_e,
                                                           double* __restrict__ area) {
  const int n = blockIdx.z;
  const RoiView r = roi_of(roi, n);
  const int lx = blockIdx.x * 64 + (threadIdx.x & 63), ly = blockIdx.y * 4 + (threadIdx.x >> 6);
  const double* M = warp + 6 * n;
  float v = 0.f;
  if (lx < r.w && ly < r.h) {
    const int x = r.x0 + lx, y = r.y0 + ly;
    // 2x2 kernel, anchor (1,1): taps (x-1..x, y-1..y); out-of-image taps ignored
    v = 3.4e38f;
#pragma unroll
    for (int dy = -1; dy <= 0; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 0; ++dx)
        if (x + dx >= 0 && y + dy >= 0) v = fminf(v, warped_ones(M, x + dx, y + dy, fh, fw));
    mask_e[((long)n * ld_h + ly) * ld_w + lx] = v;
  }
  double s = (double)v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = part[0] + part[1] + part[2] + part[3];
    if (t != 0.0) atomicAdd(area + n, t);
  }
}

// Rectangular erode by k = 2 w_edge (k = 0 -> OpenCV's default 3x3), anchor k/2:
// dst(x) = min src(x - a .. x - a + k - 1); out-of-image taps ignored, in-image taps
// outside the ROI are 0 (the mask is 0 there).
template <bool ROWS>
__global__ void __launch_bounds__(256) erode_kernel(const float* __restrict__ src, const int32_t* __restrict__ roi,
                                                    const double* __restrict__ area, int w_max, int H, int W,
                                                    int ld_w, int ld_h, float* __restrict__ dst) {
  const int n = blockIdx.z;
  const RoiView r = roi_of(roi, n);
  const int lx = blockIdx.x * 64 + (threadIdx.x & 63), ly = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (lx >= r.w || ly >= r.h) return;
  const int we = w_edge_of(area, n, w_max);
  const int k = we == 0 ? 3 : 2 * we, a = k / 2;
  const float* s = src + (long)n * ld_h * ld_w;
  float v = 3.4e38f;
  if (ROWS) {
    const int x = r.x0 + lx;
    for (int j = 0; j < k; ++j) {
      const int xx = x - a + j;
      if (xx < 0 || xx >= W) continue;
      const int l = xx - r.x0;
      v = fminf(v, (l >= 0 && l < r.w) ? s[(long)ly * ld_w + l] : 0.f);
    }
  } else {
    const int y = r.y0 + ly;
    for (int j = 0; j < k; ++j) {
      const int yy = y - a + j;
      if (yy < 0 || yy >= H) continue;
      const int l = yy - r.y0;
      v = fminf(v, (l >= 0 && l < r.h) ? s[(long)l * ld_w + lx] : 0.f);
    }
  }
  dst[((long)n * ld_h + ly) * ld_w + lx] = v;
}

// Gaussian row pass of sepFilter2D: s = sum_k g[k] x[reflect101(x + k - a)], k ascending.
__global__ void __launch_bounds__(256) blur_rows_kernel(const float* __restrict__ src, const int32_t* __restrict__ roi,
                                                        const double* __restrict__ area, const float* __restrict__ gtab,
                                                        int w_max, int W, int ld_w, int ld_h,
                                                        float* __restrict__ dst) {
  const int n = blockIdx.z;
  const RoiView r = roi_of(roi, n);
  const int lx = blockIdx.x * 64 + (threadIdx.x & 63), ly = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (lx >= r.w || ly >= r.h) return;
  const int we = w_edge_of(area, n, w_max);
  const int ks = 2 * we + 1, a = we;
  const float* g = gtab + (size_t)we * (2 * w_max + 1);
  const float* s = src + ((long)n * ld_h + ly) * ld_w;
  const int x = r.x0 + lx;
  float acc = 0.f;
  for (int k = 0; k < ks; ++k) {
    const int l = reflect101(x + k - a, W) - r.x0;
    const float v = (l >= 0 && l < r.w) ? s[l] : 0.f;
    acc = (acc + (g[k] * v));
  }
  dst[((long)n * ld_h + ly) * ld_w + lx] = acc;
}

// Gaussian column pass (symmetric: g[a] x[y] + sum_k g[a+k] (x[y+k] + x[y-k])) -> soft,
// then the blend of affine_transform.py:108-114:
//   out = trunc(soft * (mask_e * lanczos(face)) + (1 - soft) * frame)
// The Lanczos4 sample (remapLanczos4 fixed point, border 0) is taken only where
// mask_e > 0 (elsewhere the pasted term is exactly 0).
__global__ void __launch_bounds__(256) blur_cols_blend_kernel(
    const float* __restrict__ rows, const float* __restrict__ mask_e, const int32_t* __restrict__ roi,
    const double* __restrict__ area, const float* __restrict__ gtab, int w_max, const double* __restrict__ warp,
    const uint8_t* __restrict__ face, int fh, int fw, const int16_t* __restrict__ ltab, int H, int W, int ld_w,
    int ld_h, uint8_t* __restrict__ frames) {
  const int n = blockIdx.z;
  const RoiView r = roi_of(roi, n);
  const int lx = blockIdx.x * 64 + (threadIdx.x & 63), ly = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (lx >= r.w || ly >= r.h) return;
  const int we = w_edge_of(area, n, w_max);
  const float* g = gtab + (size_t)we * (2 * w_max + 1) + we;  // centred
  const float* s = rows + (long)n * ld_h * ld_w + lx;
  const int x = r.x0 + lx, y = r.y0 + ly;
  auto at = [&](int yy) {
    const int l = reflect101(yy, H) - r.y0;
    return (l >= 0 && l < r.h) ? s[(long)l * ld_w] : 0.f;
  };
  float soft = (g[0] * s[(long)ly * ld_w]);
  for (int k = 1; k <= we; ++k) soft = (soft + (g[k] * (at(y + k) + at(y - k))));
  const float me = mask_e[((long)n * ld_h + ly) * ld_w + lx];
  float pasted[3] = {0.f, 0.f, 0.f};
  if (me > 0.f) {
    const WarpPt p = warp_point(warp + 6 * n, x, y);
    const int sx = p.sx - 3, sy = p.sy - 3;
    const int16_t* w = ltab + p.fxy * 64;
    const uint8_t* fc = face + (long)n * fh * fw * 3;
    int acc[3] = {0, 0, 0};
    if ((unsigned)sx < (unsigned)max(fw - 7, 0) && (unsigned)sy < (unsigned)max(fh - 7, 0)) {
      for (int rr = 0; rr < 8; ++rr) {
        const uint8_t* row = fc + ((long)(sy + rr) * fw + sx) * 3;
#pragma unroll
        for (int cc = 0; cc < 8; ++cc) {
          const int ww = w[rr * 8 + cc];
          acc[0] += row[cc * 3 + 0] * ww;
          acc[1] += row[cc * 3 + 1] * ww;
          acc[2] += row[cc * 3 + 2] * ww;
        }
      }
    } else {
      for (int rr = 0; rr < 8; ++rr) {
        const int yy = sy + rr;
        if ((unsigned)yy >= (unsigned)fh) continue;
        for (int cc = 0; cc < 8; ++cc) {
          const int xx = sx + cc;
          if ((unsigned)xx >= (unsigned)fw) continue;
          const int ww = w[rr * 8 + cc];
          const uint8_t* px = fc + ((long)yy * fw + xx) * 3;
          acc[0] += px[0] * ww;
          acc[1] += px[1] * ww;
          acc[2] += px[2] * ww;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int v = min(max((acc[c] + (1 << 14)) >> 15, 0), 255);
      pasted[c] = (me * (float)v);
    }
  }
  uint8_t* o = frames + (((long)n * H + y) * W + x) * 3;
  const float inv = (1.f - soft);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v = ((soft * pasted[c]) + (inv * (float)o[c]));
    o[c] = (uint8_t)min((int)v, 255);
  }
}

// ---------------------------------------------------------------- cv2.resize INTER_LANCZOS4
// resize.cpp's own interpolateLanczos4 (no FLT_EPSILON guard: x ~ 0 is caught by the
// 1e30 centre tap); (x + 3) and (x + 3 - i) are float sums, as in the C++ source.
static void resize_lanczos4_coeffs(float x, float* c) {
  const double s45 = 0.70710678118654752440084436210485;
  const double cs[8][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
  const float x3 = x + 3.f;
  const double y0 = ((double)(-x3) * M_PI) * 0.25, s0 = std::sin(y0), c0 = std::cos(y0);
  float sum = 0.f;
  for (int i = 0; i < 8; ++i) {
    const float yy = x3 - (float)i;
    if (std::fabs(yy) >= 1e-6f) {
      const double y = ((double)(-yy) * M_PI) * 0.25;
      c[i] = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (y * y));
    } else {
      c[i] = 1e30f;
    }
    sum += c[i];
  }
  const float inv = 1.f / sum;
  for (int i = 0; i < 8; ++i) c[i] *= inv;
}

// resizeGeneric_ per-axis tables: f = (float)((d + 0.5) * scale - 0.5), s = floor(f),
// scale = 1 / (dst / src) in double; 8 int16 coefficients saturate_cast(c * 2048).
static void resize_axis(int sn, int dn, int32_t* ofs, int16_t* coef) {
  const double inv_scale = (double)dn / sn, scale = 1. / inv_scale;
  for (int d = 0; d < dn; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    const int s = (int)std::floor(f);
    f -= (float)s;
    float c[8];
    resize_lanczos4_coeffs(f, c);
    ofs[d] = s;
    for (int k = 0; k < 8; ++k) {
      long r = std::lrint(c[k] * 2048.f);
      coef[d * 8 + k] = (int16_t)(r < -32768 ? -32768 : (r > 32767 ? 32767 : r));
    }
  }
}

// HResizeLanczos4 (int row sums of u8 * int16, taps clamped to the row) then
// VResizeLanczos4 (int sums of the 8 clamped rows * int16) and
// FixedPtCast<int, uchar, 22>: (v + 2^21) >> 22, saturated.
__global__ void __launch_bounds__(256) resize_lanczos4_kernel(const uint8_t* __restrict__ src, int sh, int sw, int C,
                                                              uint8_t* __restrict__ dst, int dh, int dw,
                                                              const int32_t* __restrict__ ofs_x,
                                                              const int32_t* __restrict__ ofs_y,
                                                              const int16_t* __restrict__ ax,
                                                              const int16_t* __restrict__ ay) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int n = blockIdx.z;
  if (x >= dw || y >= dh) return;
  const int sx = ofs_x[x] - 3, sy = ofs_y[y] - 3;
  int xi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) xi[j] = min(max(sx + j, 0), sw - 1) * C;
  const uint8_t* img = src + (long)n * sh * sw * C;
  int acc[4] = {0, 0, 0, 0};
  for (int k = 0; k < 8; ++k) {
    const uint8_t* row = img + (long)min(max(sy + k, 0), sh - 1) * sw * C;
    const int b = ay[y * 8 + k];
    for (int c = 0; c < C; ++c) {
      int h = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) h += (int)row[xi[j] + c] * (int)ax[x * 8 + j];
      acc[c] += h * b;
    }
  }
  uint8_t* o = dst + (((long)n * dh + y) * dw + x) * C;
  for (int c = 0; c < C; ++c) o[c] = (uint8_t)min(max((acc[c] + (1 << 21)) >> 22, 0), 255);
}

// cv2.warpAffine(frame, M, (out_w, out_h), INTER_LANCZOS4, BORDER_CONSTANT, border) --
// AlignRestore.align_warp_face (affine_transform.py:53-70).  remapLanczos4 fixed point:
// sum = border 2^15 + sum over in-image taps (S - border) w, i.e. taps outside read the
// border value (the 64 taps sum to exactly 2^15); (sum + 2^14) >> 15 saturated.
__global__ void __launch_bounds__(256) align_warp_kernel(const uint8_t* __restrict__ frames, int H, int W,
                                                         const double* __restrict__ warp,
                                                         const int16_t* __restrict__ ltab, int oh, int ow,
                                                         int border, uint8_t* __restrict__ out) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int n = blockIdx.z;
  if (x >= ow || y >= oh) return;
  const WarpPt p = warp_point(warp + 6 * n, x, y);
  const int sx = p.sx - 3, sy = p.sy - 3;
  const int16_t* w = ltab + p.fxy * 64;
  const uint8_t* fr = frames + (long)n * H * W * 3;
  int acc[3] = {0, 0, 0};
  for (int rr = 0; rr < 8; ++rr) {
    const int yy = sy + rr;
    const bool rin = (unsigned)yy < (unsigned)H;
#pragma unroll
    for (int cc = 0; cc < 8; ++cc) {
      const int xx = sx + cc;
      const int ww = w[rr * 8 + cc];
      if (rin && (unsigned)xx < (unsigned)W) {
        const uint8_t* px = fr + ((long)yy * W + xx) * 3;
        acc[0] += px[0] * ww;
        acc[1] += px[1] * ww;
        acc[2] += px[2] * ww;
      } else {
        acc[0] += border * ww;
        acc[1] += border * ww;
        acc[2] += border * ww;
      }
    }
  }
  uint8_t* o = out + (((long)n * oh + y) * ow + x) * 3;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[c] = (uint8_t)min(max((acc[c] + (1 << 14)) >> 15, 0), 255);
}

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace ls

using namespace ls;

extern "C" {

size_t ls_restore_tables_bytes(int32_t w_edge_max) {
  if (w_edge_max < 0) return 0;
  return RS_LANCZOS_BYTES + sizeof(float) * (size_t)(w_edge_max + 1) * gauss_stride(w_edge_max);
}

int ls_restore_init_tables(void* tables, int32_t w_edge_max, void* stream) {
  if (!tables || w_edge_max < 0 || w_edge_max > 4096) return fail(LS_ERR_INVALID, "ls_restore_init_tables: bad args");
  const size_t gs = gauss_stride(w_edge_max);
  std::vector<uint8_t> host(ls_restore_tables_bytes(w_edge_max), 0);
  lanczos4_tab((int16_t*)host.data());
  float* g = (float*)(host.data() + RS_LANCZOS_BYTES);
  for (int we = 0; we <= w_edge_max; ++we) gaussian_kernel(2 * we + 1, g + (size_t)we * gs);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemcpyAsync(tables, host.data(), host.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(LS_ERR_LAUNCH, "ls_restore_init_tables: copy failed");
  return LS_OK;
}

int ls_face_resize_u8(const float* faces, int32_t N, int32_t in_h, int32_t in_w, int32_t out_h, int32_t out_w,
                      uint8_t* out, void* stream) {
  if (!faces || !out || N < 0 || in_h <= 0 || in_w <= 0 || out_h <= 0 || out_w <= 0)
    return fail(LS_ERR_INVALID, "ls_face_resize_u8: bad args");
  // support taps: ceil(2 * max(scale, 1)) + 1 must fit AA_MAXT
  if ((double)in_w / out_w > (AA_MAXT - 2) / 2.0 || (double)in_h / out_h > (AA_MAXT - 2) / 2.0)
    return fail(LS_ERR_INVALID, "ls_face_resize_u8: downscale factor above 7");
  if (N == 0) return LS_OK;
  hipLaunchKernelGGL(face_resize_kernel, dim3(cdiv(out_w, 64), cdiv(out_h, 4), N), dim3(256), 0,
                     (hipStream_t)stream, faces, in_h, in_w, out_h, out_w, out);
  return check_launch("face_resize_kernel");
}

size_t ls_restore_workspace_bytes(int32_t N, int32_t roi_h, int32_t roi_w) {
  if (N < 0 || roi_h < 0 || roi_w < 0) return 0;
  return align256(sizeof(double) * (size_t)N) + 3 * align256(sizeof(float) * (size_t)N * roi_h * roi_w);
}

int ls_restore_frames(uint8_t* frames, int32_t N, int32_t H, int32_t W, const uint8_t* faces, int32_t fh, int32_t fw,
                      const double* warp, const int32_t* roi, int32_t roi_h, int32_t roi_w, int32_t w_edge_max,
                      const void* tables, void* workspace, size_t workspace_bytes, void* stream) {
  if (!frames || !faces || !warp || !roi || !tables || N < 0 || H <= 0 || W <= 0 || fh <= 0 || fw <= 0 ||
      roi_h < 0 || roi_w < 0 || roi_h > H || roi_w > W || w_edge_max < 0)
    return fail(LS_ERR_INVALID, "ls_restore_frames: bad args");
  if (((uintptr_t)roi & 15) != 0) return fail(LS_ERR_INVALID, "ls_restore_frames: roi must be 16-byte aligned");
  if (!workspace || workspace_bytes < ls_restore_workspace_bytes(N, roi_h, roi_w))
    return fail(LS_ERR_WORKSPACE, "ls_restore_frames: workspace too small");
  if (N == 0 || roi_h == 0 || roi_w == 0) return LS_OK;
  hipStream_t s = (hipStream_t)stream;
  const size_t plane = align256(sizeof(float) * (size_t)N * roi_h * roi_w);
  double* area = (double*)workspace;
  float* mask_e = (float*)((char*)workspace + align256(sizeof(double) * (size_t)N));
  float* tmp = (float*)((char*)mask_e + plane);
  float* center = (float*)((char*)tmp + plane);
  const int16_t* ltab = (const int16_t*)tables;
  const float* gtab = (const float*)((const char*)tables + RS_LANCZOS_BYTES);
  if (hipMemsetAsync(area, 0, sizeof(double) * N, s) != hipSuccess)
    return fail(LS_ERR_LAUNCH, "ls_restore_frames: memset failed");
  const dim3 grid(cdiv(roi_w, 64), cdiv(roi_h, 4), N), blk(256);
  hipLaunchKernelGGL(restore_mask_kernel, grid, blk, 0, s, warp, roi, H, W, fh, fw, roi_w, roi_h, mask_e, area);
  hipLaunchKernelGGL(erode_kernel<true>, grid, blk, 0, s, mask_e, roi, area, w_edge_max, H, W, roi_w, roi_h, tmp);
  hipLaunchKernelGGL(erode_kernel<false>, grid, blk, 0, s, tmp, roi, area, w_edge_max, H, W, roi_w, roi_h, center);
  hipLaunchKernelGGL(blur_rows_kernel, grid, blk, 0, s, center, roi, area, gtab, w_edge_max, W, roi_w, roi_h, tmp);
  hipLaunchKernelGGL(blur_cols_blend_kernel, grid, blk, 0, s, tmp, mask_e, roi, area, gtab, w_edge_max, warp, faces,
                     fh, fw, ltab, H, W, roi_w, roi_h, frames);
  return check_launch("ls_restore_frames");
}

size_t ls_resize_lanczos4_workspace_bytes(int32_t dst_h, int32_t dst_w) {
  if (dst_h <= 0 || dst_w <= 0) return 0;
  return align256(sizeof(int32_t) * (size_t)(dst_h + dst_w)) + align256(16 * (size_t)(dst_h + dst_w));
}

int ls_resize_lanczos4_u8(const uint8_t* src, int32_t N, int32_t src_h, int32_t src_w, int32_t C, uint8_t* dst,
                          int32_t dst_h, int32_t dst_w, void* workspace, size_t workspace_bytes, void* stream) {
  if (!src || !dst || N < 0 || src_h <= 0 || src_w <= 0 || dst_h <= 0 || dst_w <= 0 || C < 1 || C > 4)
    return fail(LS_ERR_INVALID, "ls_resize_lanczos4_u8: bad args (C in 1..4)");
  hipStream_t s = (hipStream_t)stream;
  if (N == 0) return LS_OK;
  if (src_h == dst_h && src_w == dst_w) {  // cv::resize copies when dsize == ssize
    if (hipMemcpyAsync(dst, src, (size_t)N * src_h * src_w * C, hipMemcpyDeviceToDevice, s) != hipSuccess)
      return fail(LS_ERR_LAUNCH, "ls_resize_lanczos4_u8: copy failed");
    return LS_OK;
  }
  const size_t need = ls_resize_lanczos4_workspace_bytes(dst_h, dst_w);
  if (!workspace || workspace_bytes < need) return fail(LS_ERR_WORKSPACE, "ls_resize_lanczos4_u8: workspace");
  std::vector<uint8_t> host(need, 0);
  int32_t* ofs_x = (int32_t*)host.data();
  int32_t* ofs_y = ofs_x + dst_w;
  int16_t* ax = (int16_t*)(host.data() + align256(sizeof(int32_t) * (size_t)(dst_h + dst_w)));
  int16_t* ay = ax + 8 * (size_t)dst_w;
  resize_axis(src_w, dst_w, ofs_x, ax);
  resize_axis(src_h, dst_h, ofs_y, ay);
  if (hipMemcpyAsync(workspace, host.data(), need, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return fail(LS_ERR_LAUNCH, "ls_resize_lanczos4_u8: table copy failed");
  const uint8_t* ws = (const uint8_t*)workspace;
  const int32_t* d_ofs_x = (const int32_t*)ws;
  const int16_t* d_ax = (const int16_t*)(ws + ((const uint8_t*)ax - host.data()));
  hipLaunchKernelGGL(resize_lanczos4_kernel, dim3(cdiv(dst_w, 64), cdiv(dst_h, 4), N), dim3(256), 0, s, src, src_h,
                     src_w, C, dst, dst_h, dst_w, d_ofs_x, d_ofs_x + dst_w, d_ax, d_ax + 8 * (size_t)dst_w);
  return check_launch("resize_lanczos4_kernel");
}

int ls_align_warp_u8(const uint8_t* frames, int32_t N, int32_t H, int32_t W, const double* warp, int32_t out_h,
                     int32_t out_w, int32_t border_value, const void* tables, uint8_t* out, void* stream) {
  if (!frames || !warp || !tables || !out || N < 0 || H <= 0 || W <= 0 || out_h <= 0 || out_w <= 0 ||
      border_value < 0 || border_value > 255)
    return fail(LS_ERR_INVALID, "ls_align_warp_u8: bad args");
  if (N == 0) return LS_OK;
  hipLaunchKernelGGL(align_warp_kernel, dim3(cdiv(out_w, 64), cdiv(out_h, 4), N), dim3(256), 0, (hipStream_t)stream,
                     frames, H, W, warp, (const int16_t*)tables, out_h, out_w, border_value, out);
  return check_launch("align_warp_kernel");
}

}  // extern "C"
