// Small / elementwise kernels of the window loop (gfx950): timestep embedding,
// small-M fp32 linear (TimestepEmbedding + batched time_emb_proj), fused
// CFG + DDIM step, VAE posterior sampling, pixel prep, UNet input packing,
// latent scaling and paste-back.  All HBM-bound; 16-B vector accesses where the
// layout allows.
#include "ls_common.h"

#include <mutex>

namespace ls {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
int fail(ls_status code, const std::string& msg) { set_error(msg); return code; }
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(LS_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  return LS_OK;
}

// diffusers get_timestep_embedding (unet.py:95,376)
__global__ void timestep_embed_kernel(const int* ts, const int* step, int B, int dim, int flip, float shift,
                                      float* out) {
  const int half = dim / 2;
  const float t = (float)ts[*step];
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float e = expf(-9.210340371976184f * (float)i / ((float)half - shift));  // -ln(10000)
    const float arg = t * e;
    const float sn = sinf(arg), cs = cosf(arg);
    for (int b = 0; b < B; ++b) {
      float* o = out + (long)b * dim;
      if (flip) { o[i] = cs; o[half + i] = sn; } else { o[i] = sn; o[half + i] = cs; }
    }
  }
}

// The same embedding for one fp32 timestep per sample (blockIdx.x = sample): forward()'s
// float timesteps and distinct per-sample values, which the reference broadcasts over the
// batch (unet.py:361-376; get_timestep_embedding casts t to fp32 before the product).
__global__ void timestep_embed_f32_kernel(const float* ts, int dim, int flip, float shift, float* out) {
  const int half = dim / 2;
  const float t = ts[blockIdx.x];
  float* o = out + (long)blockIdx.x * dim;
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float e = expf(-9.210340371976184f * (float)i / ((float)half - shift));
    const float arg = t * e;
    const float sn = sinf(arg), cs = cosf(arg);
    if (flip) { o[i] = cs; o[half + i] = sn; } else { o[i] = sn; o[half + i] = cs; }
  }
}

// y[m, n] = sum_k act(x[m, k]) * W[n, k] + b[n]; one wave per output column n,
// rows in chunks of SL_ROWS per block (grid.y), the chunk's x cached in LDS.
constexpr int SL_ROWS = 8;
__global__ void __launch_bounds__(256) small_linear_kernel(const float* __restrict__ x, int M, int K,
                                                          const u16* __restrict__ w, const float* __restrict__ bias,
                                                          int N, int silu_in, float* __restrict__ y) {
  extern __shared__ float xs[];  // [SL_ROWS][K]
  const int m0 = blockIdx.y * SL_ROWS;
  const int mr = min(SL_ROWS, M - m0);
  for (int i = threadIdx.x; i < mr * K; i += blockDim.x) {
    const float v = x[(long)m0 * K + i];
    xs[i] = silu_in ? silu(v) : v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  float acc[SL_ROWS];
#pragma unroll
  for (int mm = 0; mm < SL_ROWS; ++mm) acc[mm] = 0.f;
  const u16* wr = w + (long)n * K;
  for (int k = lane * 8; k < K; k += 512) {
    float f[8];
    unpack8(*(const uint4*)(wr + k), f);
#pragma unroll
    for (int mm = 0; mm < SL_ROWS; ++mm) {
      if (mm < mr) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += f[j] * xs[mm * K + k + j];
        acc[mm] += s;
      }
    }
  }
#pragma unroll
  for (int mm = 0; mm < SL_ROWS; ++mm) {
    if (mm < mr) {
      const float s = wave_sum(acc[mm]);
      if (lane == 0) y[(long)(m0 + mm) * N + n] = s + (bias ? bias[n] : 0.f);
    }
  }
}

// CFG + DDIM step (eta = 0); re-packs channels 0..3 of every UNet batch copy.
__global__ void ddim_cfg_kernel(const u16* __restrict__ eps, int ld_eps, int Bu, long P, float guidance,
                                float* __restrict__ lat, const float* __restrict__ coef, const int* __restrict__ step,
                                u16* __restrict__ unet_in, int ld_in) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const float4 cf = *(const float4*)(coef + 4 * (*step));  // sqrt(a_t), sqrt(1-a_t), sqrt(a_prev), sqrt(1-a_prev)
  float e[4], x[4];
  const float4 l4 = *(const float4*)(lat + 4 * p);
  x[0] = l4.x; x[1] = l4.y; x[2] = l4.z; x[3] = l4.w;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float v = bf2f(eps[p * ld_eps + c]);
    if (Bu == 2) {
      const float a = bf2f(eps[(P + p) * ld_eps + c]);
      v = v + guidance * (a - v);  // noise_pred_uncond + g * (audio - uncond)
    }
    e[c] = v;
  }
  float o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float x0 = (x[c] - cf.y * e[c]) / cf.x;
    o[c] = cf.z * x0 + cf.w * e[c];
  }
  *(float4*)(lat + 4 * p) = make_float4(o[0], o[1], o[2], o[3]);
  const uint2 pk = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
  for (int b = 0; b < Bu; ++b) *(uint2*)(unet_in + (b * P + p) * ld_in) = pk;
}

__global__ void step_advance_kernel(int* step) { *step += 1; }

// ImageProcessor.preprocess_fixed_mask_image at native resolution
__global__ void prep_pixels_kernel(const uint8_t* __restrict__ faces, int F, int R, const float* __restrict__ mask,
                                   u16* __restrict__ pix, u16* __restrict__ masked, int ld) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long RR = (long)R * R;
  if (i >= F * RR) return;
  const long f = i / RR, yx = i - f * RR;
  const float mk = mask[yx];
  float pv[8], mv[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) { pv[c] = 0.f; mv[c] = 0.f; }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float u = (float)faces[(f * 3 + c) * RR + yx];
    const float p = (u / 255.0f - 0.5f) / 0.5f;
    pv[c] = p;
    mv[c] = p * mk;
  }
  if (ld == 8) {
    *(uint4*)(pix + i * 8) = pack8(pv);
    *(uint4*)(masked + i * 8) = pack8(mv);
  } else {
    for (int c = 0; c < ld; ++c) {
      pix[i * ld + c] = f2bf(c < 8 ? pv[c] : 0.f);
      masked[i * ld + c] = f2bf(c < 8 ? mv[c] : 0.f);
    }
  }
}

// DiagonalGaussianDistribution.sample() * scaling
__global__ void vae_sample_kernel(const float* __restrict__ mom, int ld_m, const float* __restrict__ eps, long P,
                                  float scaling, float shift, u16* __restrict__ dst, int ld_dst, int c_off) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float mean = mom[p * ld_m + c];
    float lv = mom[p * ld_m + 4 + c];
    lv = fminf(fmaxf(lv, -30.f), 20.f);
    const float z = mean + expf(0.5f * lv) * eps[p * 4 + c];
    dst[p * ld_dst + c_off + c] = f2bf((z - shift) * scaling);
  }
}

// UNet input = cat([latents, mask, masked_latents, ref_latents]) (lipsync_pipeline.py:547-549)
__global__ void pack_unet_input_kernel(const float* __restrict__ lat, const u16* __restrict__ cond,
                                       const float* __restrict__ mask, int F, int R, int h, int Bu,
                                       u16* __restrict__ unet_in, int ld_in) {
  const long P = (long)F * h * h;
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  const int yx = (int)(p % ((long)h * h));
  const int y = yx / h, x = yx - y * h;
  const int sy = (int)((long)y * R / h), sx = (int)((long)x * R / h);  // F.interpolate nearest
  float v[16];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = lat[p * 4 + c];
  v[4] = mask[(long)sy * R + sx];
#pragma unroll
  for (int c = 5; c < 13; ++c) v[c] = bf2f(cond[p * 16 + c]);
#pragma unroll
  for (int c = 13; c < 16; ++c) v[c] = 0.f;
  const uint4 lo = pack8(v), hi = pack8(v + 8);
  for (int b = 0; b < Bu; ++b) {
    u16* d = unet_in + (b * P + p) * ld_in;
    *(uint4*)d = lo;
    *(uint4*)(d + 8) = hi;
  }
}

__global__ void scale_latents_kernel(const float* __restrict__ lat, long P, float inv_s, float shift,
                                     u16* __restrict__ z, int ld) {
  const long p = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  float v[8];
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = lat[p * 4 + c] * inv_s + shift;
#pragma unroll
  for (int c = 4; c < 8; ++c) v[c] = 0.f;
  if (ld == 8) *(uint4*)(z + p * 8) = pack8(v);
  else for (int c = 0; c < ld; ++c) z[p * ld + c] = f2bf(c < 8 ? v[c] : 0.f);
}

// paste_surrounding_pixels_back + pixel_values_to_images
__global__ void paste_back_kernel(const u16* __restrict__ dec, int ld_dec, const u16* __restrict__ pix, int ld_pix,
                                  const float* __restrict__ mask, int F, int R, float* __restrict__ out,
                                  uint8_t* __restrict__ out_u8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long RR = (long)R * R;
  if (i >= F * RR) return;
  const long f = i / RR, yx = i - f * RR;
  const float keep = mask[yx];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float d = bf2f(dec[i * ld_dec + c]);
    const float p = bf2f(pix[i * ld_pix + c]);
    const float v = d * (1.f - keep) + p * keep;
    if (out) out[(f * 3 + c) * RR + yx] = v;
    if (out_u8) {
      const float u = fminf(fmaxf(v / 2.f + 0.5f, 0.f), 1.f) * 255.f;
      out_u8[i * 3 + c] = (uint8_t)u;
    }
  }
}

__global__ void add_rows_kernel(const u16* __restrict__ x, long rows, int C, int ldx, const float* __restrict__ t,
                                int trows, u16* __restrict__ y, int ldy) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * C) return;
  const long r = i / C;
  const int c = (int)(i - r * C);
  y[r * ldy + c] = f2bf(bf2f(x[r * ldx + c]) + t[(r % trows) * C + c]);
}

}  // namespace ls

using namespace ls;

extern "C" int ls_abi_version(void) { return LS_ABI_VERSION; }
extern "C" const char* ls_last_error(void) { return g_err.c_str(); }

extern "C" int ls_timestep_embed(const int32_t* ts, const int32_t* step, int32_t B, int32_t dim, int32_t flip,
                                 float shift, float* out, void* stream) {
  if (!ts || !step || !out || dim % 2 || B <= 0) return fail(LS_ERR_INVALID, "ls_timestep_embed: bad arguments");
  timestep_embed_kernel<<<1, 256, 0, (hipStream_t)stream>>>(ts, step, B, dim, flip, shift, out);
  return check_launch("timestep_embed_kernel");
}

extern "C" int ls_timestep_embed_f32(const float* ts, int32_t B, int32_t dim, int32_t flip, float shift, float* out,
                                     void* stream) {
  if (!ts || !out || dim % 2 || B <= 0) return fail(LS_ERR_INVALID, "ls_timestep_embed_f32: bad arguments");
  timestep_embed_f32_kernel<<<B, 256, 0, (hipStream_t)stream>>>(ts, dim, flip, shift, out);
  return check_launch("timestep_embed_f32_kernel");
}

extern "C" int ls_small_linear(const float* x, int32_t M, int32_t K, const uint16_t* w, const float* bias, int32_t N,
                               int32_t silu_in, float* y, void* stream) {
  if (!x || !w || !y || M <= 0 || M > 1024 || K % 8 || K > 2048 || N <= 0)
    return fail(LS_ERR_INVALID, "ls_small_linear: 0 < M <= 1024, K % 8 == 0, K <= 2048");
  const int rows = std::min(M, SL_ROWS);
  small_linear_kernel<<<dim3(cdiv(N, 4), cdiv(M, SL_ROWS)), 256, rows * K * sizeof(float), (hipStream_t)stream>>>(
      x, M, K, w, bias, N, silu_in, y);
  return check_launch("small_linear_kernel");
}

extern "C" int ls_ddim_cfg_step(const uint16_t* eps, int32_t ld_eps, int32_t Bu, int64_t P, float guidance,
                                float* lat, const float* coef, int32_t* step, uint16_t* unet_in, int32_t ld_in,
                                void* stream) {
  if (!eps || !lat || !coef || !step || !unet_in || (Bu != 1 && Bu != 2) || ld_eps < 4 || ld_in < 4 || ld_in % 4)
    return fail(LS_ERR_INVALID, "ls_ddim_cfg_step: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  ddim_cfg_kernel<<<cdiv(P, 256), 256, 0, s>>>(eps, ld_eps, Bu, P, guidance, lat, coef, step, unet_in, ld_in);
  int rc = check_launch("ddim_cfg_kernel");
  if (rc) return rc;
  step_advance_kernel<<<1, 1, 0, s>>>(step);
  return check_launch("step_advance_kernel");
}

extern "C" int ls_prep_pixels(const uint8_t* faces, int32_t F, int32_t R, const float* mask, uint16_t* pix,
                              uint16_t* masked, int32_t ld, void* stream) {
  if (!faces || !mask || !pix || !masked || ld < 3) return fail(LS_ERR_INVALID, "ls_prep_pixels: bad arguments");
  const long n = (long)F * R * R;
  prep_pixels_kernel<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(faces, F, R, mask, pix, masked, ld);
  return check_launch("prep_pixels_kernel");
}

extern "C" int ls_vae_sample(const float* moments, int32_t ld_m, const float* eps, int64_t P, float scaling,
                             float shift, uint16_t* dst, int32_t ld_dst, int32_t c_off, void* stream) {
  if (!moments || !eps || !dst || ld_m < 8) return fail(LS_ERR_INVALID, "ls_vae_sample: bad arguments");
  vae_sample_kernel<<<cdiv(P, 256), 256, 0, (hipStream_t)stream>>>(moments, ld_m, eps, P, scaling, shift, dst, ld_dst,
                                                                    c_off);
  return check_launch("vae_sample_kernel");
}

extern "C" int ls_pack_unet_input(const float* lat, const uint16_t* cond, const float* mask, int32_t F, int32_t R,
                                  int32_t h, int32_t Bu, uint16_t* unet_in, int32_t ld_in, void* stream) {
  if (!lat || !cond || !mask || !unet_in || ld_in % 8 || ld_in < 16) return fail(LS_ERR_INVALID, "ls_pack_unet_input");
  const long P = (long)F * h * h;
  pack_unet_input_kernel<<<cdiv(P, 256), 256, 0, (hipStream_t)stream>>>(lat, cond, mask, F, R, h, Bu, unet_in, ld_in);
  return check_launch("pack_unet_input_kernel");
}

extern "C" int ls_scale_latents(const float* lat, int64_t P, float inv_s, float shift, uint16_t* z, int32_t ld,
                                void* stream) {
  if (!lat || !z || ld < 4) return fail(LS_ERR_INVALID, "ls_scale_latents: bad arguments");
  scale_latents_kernel<<<cdiv(P, 256), 256, 0, (hipStream_t)stream>>>(lat, P, inv_s, shift, z, ld);
  return check_launch("scale_latents_kernel");
}

extern "C" int ls_paste_back(const uint16_t* dec, int32_t ld_dec, const uint16_t* pix, int32_t ld_pix,
                             const float* mask, int32_t F, int32_t R, float* out, uint8_t* out_u8, void* stream) {
  if (!dec || !pix || !mask || (!out && !out_u8)) return fail(LS_ERR_INVALID, "ls_paste_back: bad arguments");
  const long n = (long)F * R * R;
  paste_back_kernel<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(dec, ld_dec, pix, ld_pix, mask, F, R, out, out_u8);
  return check_launch("paste_back_kernel");
}

extern "C" int ls_add_rows(const uint16_t* x, int64_t rows, int32_t C, int32_t ldx, const float* table,
                           int32_t table_rows, uint16_t* y, int32_t ldy, void* stream) {
  if (!x || !table || !y || table_rows <= 0) return fail(LS_ERR_INVALID, "ls_add_rows: bad arguments");
  const long n = rows * C;
  add_rows_kernel<<<cdiv(n, 256), 256, 0, (hipStream_t)stream>>>(x, rows, C, ldx, table, table_rows, y, ldy);
  return check_launch("add_rows_kernel");
}
