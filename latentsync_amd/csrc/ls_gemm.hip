// Fused implicit-GEMM convolution / linear layer for gfx950 (bf16 MFMA 16x16x32).
//
// One kernel family covers every dense contraction of the UNet / SD-VAE / Whisper
// path: InflatedConv3d 3x3 (s1, s2, fused nearest-x2 upsample), 1x1 convs and
// nn.Linear (ksize 1).  The A operand is gathered straight from the NHWC
// activation (optionally two tensors = fused torch.cat, optionally through the
// GroupNorm affine + SiLU prologue); W is pre-packed [N][K] K-contiguous.
//
// Tile: BM x BN x 64, 4 waves (256 threads) of (BM/WM) x (BN/WN) each, fp32
// accumulators in registers, register-staged double-buffered LDS (one barrier
// per K-tile: the next tile's global loads are issued before the MFMAs of the
// current one).  LDS rows are 128 B (64 bf16) and XOR-swizzled at 16-B chunk
// granularity (chunk ^ ((row >> 1) & 7)) so the ds_read_b128 fragment reads of
// a 16-lane group hit 16 distinct 4-bank slots.
#include "ls_common.h"

namespace ls {

struct ConvArgs {
  const u16* x1; const u16* x2;
  int C1, C2, Cin, ld1, ld2;
  int n_img, H, W, Ho, Wo, stride, pad, upsample;
  const float* aff_scale; const float* aff_shift; int pix_per_sample; int silu_in;
  const u16* w; int K, N, M, CC;
  const float* bias; const float* rowvec; int rows_per_vec, rowvec_ld;
  const u16* res; int ldr; float out_scale; int act;
  void* y; int ldy; int y_f32;
  int ktiles, kt_per_split, split; float* partial;
  int ntm, ntn;
};

// ---------------------------------------------------------------- epilogue
__device__ __forceinline__ float epi_value(const ConvArgs& a, int row, int col, float v) {
  if (a.bias) v += a.bias[col];
  if (a.rowvec) v += a.rowvec[(long)(row / a.rows_per_vec) * a.rowvec_ld + col];
  if (a.res) v += bf2f(a.res[(long)row * a.ldr + col]);
  v *= a.out_scale;
  if (a.act == LS_ACT_GELU) v = gelu_erf(v);
  else if (a.act == LS_ACT_SILU) v = silu(v);
  return v;
}

__device__ __forceinline__ void epi_store(const ConvArgs& a, int row, int col, float v) {
  if (a.y_f32) ((float*)a.y)[(long)row * a.ldy + col] = v;
  else ((u16*)a.y)[(long)row * a.ldy + col] = f2bf(v);
}

// GEGLU: packed column 32b+i holds h_{16b+i}, 32b+16+i holds g_{16b+i}.
__device__ __forceinline__ void epi_geglu(const ConvArgs& a, int row, int pcol_h, float h, float g) {
  if (a.bias) { h += a.bias[pcol_h]; g += a.bias[pcol_h + 16]; }
  const int ocol = (pcol_h >> 5) * 16 + (pcol_h & 15);
  epi_store(a, row, ocol, h * gelu_erf(g));
}

// ---------------------------------------------------------------- A gather
template <int KS, bool TAPU>
__device__ __forceinline__ uint4 load_a_chunk(const ConvArgs& a, int kt, int ch, int m, int n, int yo, int xo) {
  if (m >= a.M) return make_uint4(0, 0, 0, 0);
  int c, tap;
  if (KS == 1) {
    tap = 0;
    c = kt * 64 + ch * 8;
    if (c >= a.Cin) return make_uint4(0, 0, 0, 0);
  } else if (TAPU) {
    tap = (kt * 64) / a.Cin;  // uniform across the tile
    c = kt * 64 - tap * a.Cin + ch * 8;
  } else {
    const int kc = kt * 8 + ch;
    tap = kc / a.CC;
    c = (kc - tap * a.CC) * 8;
    if (tap >= 9) return make_uint4(0, 0, 0, 0);
  }
  long pix;
  if (KS == 1) {
    pix = m;
  } else {
    const int kh = tap / 3, kw = tap - kh * 3;
    int yy = yo * a.stride + kh - a.pad;
    int xx = xo * a.stride + kw - a.pad;
    if (a.upsample) {
      if (yy < 0 || xx < 0 || yy >= 2 * a.H || xx >= 2 * a.W) return make_uint4(0, 0, 0, 0);
      yy >>= 1; xx >>= 1;
    } else {
      if (yy < 0 || xx < 0 || yy >= a.H || xx >= a.W) return make_uint4(0, 0, 0, 0);
    }
    pix = ((long)n * a.H + yy) * a.W + xx;
  }
  uint4 v;
  if (c < a.C1) v = *(const uint4*)(a.x1 + pix * a.ld1 + c);
  else v = *(const uint4*)(a.x2 + pix * a.ld2 + (c - a.C1));
  if (a.aff_scale) {
    const long s = pix / a.pix_per_sample;
    const float4* sc = (const float4*)(a.aff_scale + s * a.Cin + c);
    const float4* sh = (const float4*)(a.aff_shift + s * a.Cin + c);
    const float4 s0 = sc[0], s1 = sc[1], h0 = sh[0], h1 = sh[1];
    const float scl[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float shf[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = f[j] * scl[j] + shf[j];
      f[j] = a.silu_in ? silu(t) : t;
    }
    v = pack8(f);
  }
  return v;
}

__device__ __forceinline__ int swz(int row, int ch) { return row * 8 + (ch ^ ((row >> 1) & 7)); }

template <int BM, int BN, int WM, int WN, int KS, bool TAPU>
__global__ void __launch_bounds__(256) conv_gemm_kernel(ConvArgs a) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int AL = BM / 32, BL = BN / 32;  // 16-B chunks per thread per K-tile
  __shared__ uint4 lds[2][(BM + BN) * 8];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  int bid = blockIdx.x;
  const int nt = a.ntm * a.ntn;
  const int z = bid / nt;
  bid -= z * nt;
  const int tm = bid / a.ntn, tn = bid - tm * a.ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = z * a.kt_per_split;
  const int kt1 = min(a.ktiles, kt0 + a.kt_per_split);

  // per-thread fixed A rows
  const int ch = tid & 7;
  int rm[AL], rn[AL], ryo[AL], rxo[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    rm[i] = m;
    if (KS == 3) {
      const int hw = a.Ho * a.Wo;
      const int n = m / hw, r = m - n * hw;
      rn[i] = n; ryo[i] = r / a.Wo; rxo[i] = r - ryo[i] * a.Wo;
    } else {
      rn[i] = 0; ryo[i] = 0; rxo[i] = 0;
    }
  }

  uint4 ra[AL], rb[BL];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < AL; ++i) ra[i] = load_a_chunk<KS, TAPU>(a, kt, ch, rm[i], rn[i], ryo[i], rxo[i]);
#pragma unroll
    for (int j = 0; j < BL; ++j) {
      const int n = n0 + (tid >> 3) + 32 * j;
      rb[j] = (n < a.N) ? *(const uint4*)(a.w + (long)n * a.K + kt * 64 + ch * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AL; ++i) lds[buf][swz((tid >> 3) + 32 * i, ch)] = ra[i];
#pragma unroll
    for (int j = 0; j < BL; ++j) lds[buf][BM * 8 + swz((tid >> 3) + 32 * j, ch)] = rb[j];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    gload(kt0);
    sstore(0);
    __syncthreads();
    int cur = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) gload(kt + 1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + (lane >> 4);
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = __builtin_bit_cast(bf16x8, lds[cur][swz(wm * WTM + i * 16 + (lane & 15), c)]);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = __builtin_bit_cast(bf16x8, lds[cur][BM * 8 + swz(wn * WTN + j * 16 + (lane & 15), c)]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      if (more) sstore(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  // ---------------------------------------------------------------- epilogue
  const int rbase = m0 + wm * WTM + (lane >> 4) * 4;
  const int cbase = n0 + wn * WTN + (lane & 15);
  if (a.split > 1) {
    float* P = a.partial + (long)z * a.M * a.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + r, col = cbase + j * 16;
          if (row < a.M && col < a.N) P[(long)row * a.N + col] = acc[i][j][r];
        }
    return;
  }
  if (a.act == LS_ACT_GEGLU) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; j += 2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rbase + i * 16 + r, col = cbase + j * 16;
          if (row < a.M && col < a.N) epi_geglu(a, row, col, acc[i][j][r], acc[i][j + 1][r]);
        }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + i * 16 + r, col = cbase + j * 16;
        if (row < a.M && col < a.N) epi_store(a, row, col, epi_value(a, row, col, acc[i][j][r]));
      }
}

// split-K reduction + epilogue: one thread per output element
__global__ void splitk_reduce_kernel(ConvArgs a) {
  const int nout = (a.act == LS_ACT_GEGLU) ? a.N / 2 : a.N;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)a.M * nout) return;
  const int row = idx / nout, oc = idx - (long)row * nout;
  const long MN = (long)a.M * a.N;
  if (a.act == LS_ACT_GEGLU) {
    const int ph = (oc >> 4) * 32 + (oc & 15);
    float h = 0.f, g = 0.f;
    for (int z = 0; z < a.split; ++z) {
      h += a.partial[z * MN + (long)row * a.N + ph];
      g += a.partial[z * MN + (long)row * a.N + ph + 16];
    }
    epi_geglu(a, row, ph, h, g);
  } else {
    float v = 0.f;
    for (int z = 0; z < a.split; ++z) v += a.partial[z * MN + (long)row * a.N + oc];
    epi_store(a, row, oc, epi_value(a, row, oc, v));
  }
}

// ---------------------------------------------------------------- host side
struct TileCfg { int bm, bn; };

static TileCfg pick_tile(long M, int N) {
  if (N <= 32) return {128, 32};
  const long t128 = (long)cdiv(M, 128) * cdiv(N, 128);
  if (t128 >= 240) return {128, 128};
  if ((long)cdiv(M, 128) * cdiv(N, 64) >= 240) return {128, 64};
  return {64, 64};
}

template <int BM, int BN, int WM, int WN>
static void launch_cfg(const ConvArgs& a, int ks, bool tapu, int grid, hipStream_t s) {
  if (ks == 1) conv_gemm_kernel<BM, BN, WM, WN, 1, false><<<grid, 256, 0, s>>>(a);
  else if (tapu) conv_gemm_kernel<BM, BN, WM, WN, 3, true><<<grid, 256, 0, s>>>(a);
  else conv_gemm_kernel<BM, BN, WM, WN, 3, false><<<grid, 256, 0, s>>>(a);
}

static int build_args(const ls_conv_desc* d, ConvArgs& a, TileCfg& t, int& split) {
  if (!d || !d->x1 || !d->w || !d->y) return fail(LS_ERR_INVALID, "ls_conv2d: null pointer");
  if (d->ksize != 1 && d->ksize != 3) return fail(LS_ERR_INVALID, "ls_conv2d: ksize must be 1 or 3");
  const int Cin = d->C1 + d->C2;
  if (d->C1 % 8 || d->C2 % 8 || Cin <= 0) return fail(LS_ERR_INVALID, "ls_conv2d: channels must be multiples of 8");
  if (d->C2 && !d->x2) return fail(LS_ERR_INVALID, "ls_conv2d: C2 > 0 needs x2");
  if (d->ld1 % 8 || (d->C2 && d->ld2 % 8)) return fail(LS_ERR_INVALID, "ls_conv2d: pixel pitch must be a multiple of 8");
  const long Kneed = (long)d->ksize * d->ksize * Cin;
  if (d->K % 64 || d->K < Kneed || d->K - Kneed >= 64 + (d->ksize == 3 ? 0 : 0))
    return fail(LS_ERR_INVALID, "ls_conv2d: K must be ksize^2*Cin rounded up to 64");
  if (d->ksize == 1 && (d->Ho != d->H || d->Wo != d->W || d->stride != 1 || d->upsample))
    return fail(LS_ERR_INVALID, "ls_conv2d: ksize 1 must be stride 1 with no resampling");
  if (d->act == LS_ACT_GEGLU && (d->N % 32)) return fail(LS_ERR_INVALID, "ls_conv2d: GEGLU needs N % 32 == 0");
  if (d->aff_scale && (!d->aff_shift || d->imgs_per_sample <= 0))
    return fail(LS_ERR_INVALID, "ls_conv2d: affine prologue needs shift and imgs_per_sample");
  if (d->rowvec && d->rows_per_vec <= 0) return fail(LS_ERR_INVALID, "ls_conv2d: rowvec needs rows_per_vec");
  const long M = (long)d->n_img * d->Ho * d->Wo;
  if (M <= 0 || M >= (1L << 31)) return fail(LS_ERR_INVALID, "ls_conv2d: bad M");
  a.x1 = d->x1; a.x2 = d->x2; a.C1 = d->C1; a.C2 = d->C2; a.Cin = Cin; a.ld1 = d->ld1; a.ld2 = d->ld2;
  a.n_img = d->n_img; a.H = d->H; a.W = d->W; a.Ho = d->Ho; a.Wo = d->Wo;
  a.stride = d->stride; a.pad = d->pad; a.upsample = d->upsample;
  a.aff_scale = d->aff_scale; a.aff_shift = d->aff_shift;
  a.pix_per_sample = d->imgs_per_sample * d->H * d->W; a.silu_in = d->silu_in;
  a.w = d->w; a.K = d->K; a.N = d->N; a.M = (int)M; a.CC = Cin / 8;
  a.bias = d->bias; a.rowvec = d->rowvec; a.rows_per_vec = d->rows_per_vec;
  a.rowvec_ld = d->rowvec_ld > 0 ? d->rowvec_ld : d->N;
  a.res = d->res; a.ldr = d->ldr; a.out_scale = d->out_scale == 0.f ? 1.f : d->out_scale; a.act = d->act;
  a.y = d->y; a.ldy = d->ldy; a.y_f32 = d->y_f32;
  a.ktiles = d->K / 64;
  t = pick_tile(M, d->N);
  a.ntm = cdiv(M, t.bm); a.ntn = cdiv(d->N, t.bn);
  split = d->split_k;
  if (split <= 0) {
    split = 1;
    const long tiles = (long)a.ntm * a.ntn;
    if (tiles < 160 && a.ktiles >= 16) split = (int)std::min<long>(a.ktiles / 8, cdiv(320, tiles));
    if (split < 1) split = 1;
  }
  split = std::min(split, a.ktiles);
  a.kt_per_split = cdiv(a.ktiles, split);
  split = cdiv(a.ktiles, a.kt_per_split);
  a.split = split;
  a.partial = nullptr;
  return LS_OK;
}

}  // namespace ls

using namespace ls;

extern "C" size_t ls_conv_workspace_bytes(const ls_conv_desc* d) {
  ConvArgs a; TileCfg t; int split;
  if (build_args(d, a, t, split) != LS_OK) return 0;
  return split > 1 ? (size_t)split * a.M * a.N * sizeof(float) : 0;
}

extern "C" int ls_conv2d(const ls_conv_desc* d, void* stream) {
  ConvArgs a; TileCfg t; int split;
  int rc = build_args(d, a, t, split);
  if (rc != LS_OK) return rc;
  if (split > 1) {
    const size_t need = (size_t)split * a.M * a.N * sizeof(float);
    if (!d->workspace || d->workspace_bytes < need) {
      // fall back to fewer splits that fit the workspace
      const size_t per = (size_t)a.M * a.N * sizeof(float);
      int fit = d->workspace ? (int)(d->workspace_bytes / per) : 0;
      if (fit < 2) { split = 1; } else { split = std::min(split, fit); }
      a.kt_per_split = cdiv(a.ktiles, split);
      split = cdiv(a.ktiles, a.kt_per_split);
      a.split = split;
    }
    if (split > 1) a.partial = (float*)d->workspace;
  }
  hipStream_t s = (hipStream_t)stream;
  const bool tapu = (d->ksize == 3) && (a.Cin % 64 == 0);
  const int grid = a.ntm * a.ntn * a.split;
  if (t.bm == 128 && t.bn == 128) launch_cfg<128, 128, 2, 2>(a, d->ksize, tapu, grid, s);
  else if (t.bm == 128 && t.bn == 64) launch_cfg<128, 64, 2, 2>(a, d->ksize, tapu, grid, s);
  else if (t.bm == 128 && t.bn == 32) launch_cfg<128, 32, 4, 1>(a, d->ksize, tapu, grid, s);
  else launch_cfg<64, 64, 2, 2>(a, d->ksize, tapu, grid, s);
  if ((rc = check_launch("conv_gemm_kernel")) != LS_OK) return rc;
  if (a.split > 1) {
    const long nout = (long)a.M * ((a.act == LS_ACT_GEGLU) ? a.N / 2 : a.N);
    splitk_reduce_kernel<<<cdiv(nout, 256), 256, 0, s>>>(a);
    if ((rc = check_launch("splitk_reduce_kernel")) != LS_OK) return rc;
  }
  return LS_OK;
}
