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
#include <type_traits>

#include "ls_common.h"

namespace ls {

struct ConvArgs {
  const u16* x1; const u16* x2;
  int C1, C2, Cin, ld1, ld2;
  int n_img, H, W, Ho, Wo, stride, pad, upsample;
  const float* aff_scale; const float* aff_shift; int pix_per_sample; int silu_in;
  const u16* w; int K, N, M, CC;
  const float* bias; const float* rowvec; int rows_per_vec, rowvec_ld, rowvec_mod;
  const float* ln_mr; const float* ln_cs;
  const u16* res; int ldr; float out_scale; int act;
  void* y; int ldy; int y_f32;
  int ktiles, kt_per_split, split; float* partial;
  int ntm, ntn;
  float* stats_out; float stats_eps;  // row (mean, rstd) of y (row-block epilogue or a trailing row_stats)
  float* cs_out;  // GroupNorm column sums of y: [M / CS_ROWS][2][N] fp32 (sum, sum of squares per slot)
  int ablate;  // tuning only (bits): 2 = skip operand DMA, 4 = skip epilogue stores, 8 = skip epilogue,
               // 16 = skip MFMAs (DMA kernel)
  int ccm;     // 3x3 with Cin % 64 == 0: K is channel-chunk-major, taps innermost (see tap_of)
  int gm;      // tile raster: groups of gm row-blocks x all column tiles, row-block fastest (tile_of)
};

// Logical tile index -> (row-block, column-block), grouped: gm row-blocks x all ntn column
// tiles per group, the row-block index fastest.  Tiles running together on an XCD (xcd_remap
// gives every XCD a contiguous logical range) then share gm A row-bands and ~(concurrent /
// gm) W column panels instead of one A band and a W panel per tile: the wide linears
// (GEGLU W1, fused q|k|v) re-fetched their whole W per row-band (profiles/r03e_pmc_per_kernel.txt).
// gm = 1 is the plain column-fastest order.
__device__ __forceinline__ void tile_of(const ConvArgs& a, int bid, int& tm, int& tn) {
  const int gsz = a.gm * a.ntn, g = bid / gsz, r = bid - g * gsz;
  const int first = g * a.gm, rows = min(a.ntm - first, a.gm);
  tm = first + r % rows;
  tn = r / rows;
}

// K order of a 3x3 weight with Cin % 64 == 0 (packing.py): k = (ci / 64) * 576 + tap * 64 +
// ci % 64 -- the 9 taps of one 64-channel chunk are consecutive K-tiles, so a block reads
// a pixel chunk's 3x3 neighbourhood in 9 back-to-back K-tiles and the re-reads hit L2
// (tap-major, the 9 re-reads of a pixel were Cin / 64 K-tiles apart and, with 64 blocks
// per XCD streaming operands in between, missed: profiles/r03e_pmc_per_kernel.txt).
// Returns the tap and sets c0 = the K-tile's first input channel (k0 = a 64-aligned or,
// for BK 32, 32-aligned K offset).
__device__ __forceinline__ int tap_of(const ConvArgs& a, int k0, int& c0) {
  if (a.ccm) {
    const int chunk = k0 / 576, rem = k0 - chunk * 576;
    c0 = chunk * 64 + (rem & 63);
    return rem >> 6;
  }
  const int tap = k0 / a.Cin;
  c0 = k0 - tap * a.Cin;
  return tap;
}

// ---------------------------------------------------------------- epilogue
// Vectorised epilogue on 8 consecutive output columns (16-B bf16 / 32-B fp32
// stores).  All global loads of a chunk are issued before its stores.
struct Chunk8 { float v[8]; };


__device__ __forceinline__ float act_fn(int act, float v) {
  if (act == LS_ACT_GELU) return gelu_erf(v);
  if (act == LS_ACT_SILU) return silu(v);
  return v;
}

// v[8] = accumulators of packed columns [col, col+8) of `row`; applies bias,
// rowvec, residual, scale, activation and stores.  vec = all 8 in range and aligned.
__device__ __forceinline__ long rv_row(const ConvArgs& a, int row) {
  const int r = row / a.rows_per_vec;
  return (long)(a.rowvec_mod ? r % a.rowvec_mod : r) * a.rowvec_ld;
}

// LayerNorm fold: acc = rstd * (acc - mean * colsum[c])
__device__ __forceinline__ void ln_fold8(const ConvArgs& a, int row, int col, float* v, bool vec) {
  const float2 mr = *(const float2*)(a.ln_mr + 2L * row);
  if (vec) {
    float cs[8];
    load8f(a.ln_cs + col, cs);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = mr.y * (v[j] - mr.x * cs[j]);
  } else {
    for (int j = 0; j < 8 && col + j < a.N; ++j) v[j] = mr.y * (v[j] - mr.x * a.ln_cs[col + j]);
  }
}

__device__ __forceinline__ void epi_chunk(const ConvArgs& a, int row, int col, float* v, bool vec) {
  if (row >= a.M) return;
  if (a.ln_mr) ln_fold8(a, row, col, v, vec);
  if (vec) {
    float b[8], rv[8], rs[8];
    if (a.bias) load8f(a.bias + col, b); else for (int j = 0; j < 8; ++j) b[j] = 0.f;
    if (a.rowvec) load8f(a.rowvec + rv_row(a, row) + col, rv);
    else for (int j = 0; j < 8; ++j) rv[j] = 0.f;
    if (a.res) unpack8(*(const uint4*)(a.res + (long)row * a.ldr + col), rs);
    else for (int j = 0; j < 8; ++j) rs[j] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = act_fn(a.act, (v[j] + b[j] + rv[j] + rs[j]) * a.out_scale);
    if (a.y_f32) {
      float* y = (float*)a.y + (long)row * a.ldy + col;
      *(float4*)y = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(y + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      *(uint4*)((u16*)a.y + (long)row * a.ldy + col) = pack8(v);
    }
  } else {
    for (int j = 0; j < 8; ++j) {
      const int c = col + j;
      if (c >= a.N) break;
      float t = v[j];
      if (a.bias) t += a.bias[c];
      if (a.rowvec) t += a.rowvec[rv_row(a, row) + c];
      if (a.res) t += bf2f(a.res[(long)row * a.ldr + c]);
      t = act_fn(a.act, t * a.out_scale);
      if (a.y_f32) ((float*)a.y)[(long)row * a.ldy + c] = t;
      else ((u16*)a.y)[(long)row * a.ldy + c] = f2bf(t);
    }
  }
}

// GEGLU chunk: h[8] = packed cols [ph, ph+8), g[8] = [ph+16, ph+24) -> out cols [oc, oc+8)
__device__ __forceinline__ void epi_geglu8(const ConvArgs& a, int row, int ph, float* h, float* g, bool vec) {
  if (row >= a.M) return;
  const int oc = (ph >> 5) * 16 + (ph & 15);
  if (a.ln_mr) {
    ln_fold8(a, row, ph, h, true);
    ln_fold8(a, row, ph + 16, g, true);
  }
  float bh[8], bg[8];
  if (a.bias) { load8f(a.bias + ph, bh); load8f(a.bias + ph + 16, bg); }
  else for (int j = 0; j < 8; ++j) { bh[j] = 0.f; bg[j] = 0.f; }
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (h[j] + bh[j]) * gelu_erf(g[j] + bg[j]);
  if (vec && !a.y_f32) *(uint4*)((u16*)a.y + (long)row * a.ldy + oc) = pack8(h);
  else
    for (int j = 0; j < 8; ++j) {
      if (a.y_f32) ((float*)a.y)[(long)row * a.ldy + oc + j] = h[j];
      else ((u16*)a.y)[(long)row * a.ldy + oc + j] = f2bf(h[j]);
    }
}

// ---------------------------------------------------------------- A gather
// Per-row geometry precomputed once per thread: pixel base of the image, and
// the top-left input coordinate of the 3x3 window (or a sentinel for m >= M).
struct RowGeo { int pb, yb, xb; };

template <int KS, bool TAPU>
__device__ __forceinline__ uint4 load_a_chunk(const ConvArgs& a, int kt, int ch, int m, const RowGeo& g) {
  int c, tap = 0;
  if (KS == 1) {
    c = kt * 64 + ch * 8;
    if (m >= a.M || c >= a.Cin) return make_uint4(0, 0, 0, 0);
  } else if (TAPU) {
    tap = tap_of(a, kt * 64, c);
    c += ch * 8;
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
    int yy = g.yb + kh, xx = g.xb + kw;
    if (a.upsample) {
      if ((unsigned)yy >= (unsigned)(2 * a.H) || (unsigned)xx >= (unsigned)(2 * a.W)) return make_uint4(0, 0, 0, 0);
      yy >>= 1; xx >>= 1;
    } else {
      if ((unsigned)yy >= (unsigned)a.H || (unsigned)xx >= (unsigned)a.W) return make_uint4(0, 0, 0, 0);
    }
    pix = (long)g.pb + yy * a.W + xx;
  }
  uint4 v;
  if (c < a.C1) v = *(const uint4*)(a.x1 + pix * a.ld1 + c);
  else v = *(const uint4*)(a.x2 + pix * a.ld2 + (c - a.C1));
  if (a.aff_scale) {
    const long s = pix / a.pix_per_sample;
    float scl[8], shf[8], f[8];
    load8f(a.aff_scale + s * a.Cin + c, scl);
    load8f(a.aff_shift + s * a.Cin + c, shf);
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = f[j] * scl[j] + shf[j];
      f[j] = a.silu_in ? silu(t) : t;
    }
    v = pack8(f);
  }
  return v;
}

__device__ __forceinline__ int swz(int row, int ch) { return row * 8 + (ch ^ ((row >> 1) & 7)); }

// Accumulators of wave-row p -> LDS staging (fp32, pitch BN + 4).
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void stage_acc(f32x4 (&acc)[BM / WM / 16][BN / WN / 16], float* st, int p, int tid) {
  constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16, SP = BN + 4;
  const int lane = tid & 63, wid = tid >> 6;
  if (wid / WN != p) return;
  const int wn = wid % WN;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        st[(i * 16 + (lane >> 4) * 4 + r) * SP + wn * WTN + j * 16 + (lane & 15)] = acc[i][j][r];
}

// Vectorised single-pass epilogue (N % 8 == 0, no split-K).  Every thread owns
// ONE 8-column chunk of the tile for the whole epilogue, so the per-column side
// inputs (bias, LayerNorm colsum) are loaded once, before the first barrier; the
// per-row side inputs (residual, row vector, LayerNorm row stats) of all of a
// thread's rows in a wave-row pass are issued together before any is consumed --
// one L2/HBM round trip per pass instead of one per chunk.
// GroupNorm statistics from the producer (a.cs_out): per CS_ROWS-row slot and column,
// the sum and the sum of squares of the STORED (bf16-rounded) values, fp32 over the
// slot -- what gn_stats_kernel would read back; ls_groupnorm_colsum merges the slots
// of a sample in fp64.  The store loop writes the rounded values back over its fp32
// staging; after the pass barrier one thread per column adds the pass's rows from LDS
// (2 registers across passes), then a barrier before the next pass re-stages.  A
// slot's sums go out with its last pass.  128-row tiles only (cs_tile_fits).
constexpr int CS_ROWS = LS_GN_SLOT_ROWS;

template <int BM, int BN, int WM, int WN>
__host__ __device__ constexpr bool cs_tile_fits() {
  return BM != 256 && BM % CS_ROWS == 0 && CS_ROWS % (BM / WM) == 0 && WM * WN * 64 >= BN;
}

// Thread geometry of the single-pass epilogue: a thread owns one 8-column chunk of the
// tile (CPRW chunk columns per row), RPI rows per iteration, ITER iterations per wave-row pass.
template <int BM, int BN, int WM, int WN>
struct EpiGeo {
  static constexpr int NT = WM * WN * 64, WTM = BM / WM, CPRW = BN / 8, RPI = NT / CPRW;
  static constexpr int ITER = (WTM + RPI - 1) / RPI;
};
// the residual chunks of one wave-row pass (the per-row side input worth prefetching; the
// LayerNorm row statistics of a folded GEMM are loaded in the pass)
template <int ITER>
struct EpiSide {
  uint4 rs[ITER];
};

// tile-local row -> output row (RW: see store_tile_plain)
template <int RW>
__device__ __forceinline__ int epi_out_row(const ConvArgs& a, int m0, long m0r, int lr) {
  if constexpr (RW > 0) return (int)(m0r + (long)(lr / RW) * a.Wo + lr % RW);
  else return m0 + lr;
}

// issue the residual loads of wave-row pass p (global loads into registers; the consumer's
// s_waitcnt is the compiler's): one HBM round trip per pass, issued a pass (or, from the
// DMA kernel's last K-tile, the whole final K-tile) before it is consumed
template <int BM, int BN, int WM, int WN, int RW = 0>
__device__ __forceinline__ void epi_side_load(const ConvArgs& a, int m0, int n0, long m0r, int tid, int p,
                                              EpiSide<EpiGeo<BM, BN, WM, WN>::ITER>& sd) {
  using G = EpiGeo<BM, BN, WM, WN>;
  const int c8 = (tid % G::CPRW) * 8, r0 = tid / G::CPRW;
  const int col = n0 + c8;
  const bool cok = (r0 < G::RPI) && col < a.N;
#pragma unroll
  for (int it = 0; it < G::ITER; ++it) {
    const int rl = r0 + it * G::RPI, row = epi_out_row<RW>(a, m0, m0r, p * G::WTM + rl);
    const bool ok = cok && rl < G::WTM && row < a.M;
    sd.rs[it] = make_uint4(0, 0, 0, 0);
    if (ok && a.res) sd.rs[it] = *(const uint4*)(a.res + (long)row * a.ldr + col);
  }
}

// CSF: the column sums also for a 256-row tile whose wave rows are 64 (the halo conv);
// RW > 0: the tile's rows are BM / RW segments of RW consecutive output pixels, one per
// image row (the halo conv's TH x TW tiles); m0 is then the tile's VIRTUAL first row
// (GroupNorm slots) and m0r the real first row.  PRE: pass 0's side inputs were loaded by
// the caller (epi_side_load during its last K-tile) into `pre`.  Pass p + 1's side inputs
// are issued right after pass p's staging barrier, so only the first pass waits on HBM.
// CSG > 1 (round 6, the halo convs): the column sums are kept per thread in registers -- its
// 8-column chunk summed over the rows it stores, across the passes of a 128-row slot -- and
// only at the slot's end do the RPI threads of a chunk column meet through LDS (the staging
// image; a fixed order).  The per-pass form wrote every stored value back to the staging image
// and had BN threads re-read all WTM rows: 10-14 % of the 16x16 halo conv (scripts/cs_cost.py).
// (The caller guarantees (NT / (BN / 8)) x BN x 2 floats of LDS at st.)
template <int BM, int BN, int WM, int WN, bool GEN, bool CSF = false, int RW = 0, bool PRE = false, bool PIPE = true,
          int CSG = 1>
__device__ __forceinline__ void store_tile_plain_pre(const ConvArgs& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                                     float* st, int m0, int n0, long m0r, int tid_in,
                                                     const EpiSide<EpiGeo<BM, BN, WM, WN>::ITER>& pre) {
  constexpr int NT = WM * WN * 64, WTM = BM / WM, SP = BN + 4;
  constexpr int CPRW = BN / 8;                 // chunk columns per tile row
  constexpr int RPI = NT / CPRW;               // rows per iteration
  constexpr int ITER = (WTM + RPI - 1) / RPI;  // iterations per wave-row pass
  constexpr bool CSOK = CSF || cs_tile_fits<BM, BN, WM, WN>();
  static_assert(!CSF || (CS_ROWS % WTM == 0 && NT >= BN), "column-sum slots of whole wave rows");
  // tile-local row -> output row
  auto out_row = [&](int lr) -> int { return epi_out_row<RW>(a, m0, m0r, lr); };
  const int tid = tid_in >= 0 ? tid_in : (int)threadIdx.x;  // (a caller in a loop passes an opaque copy)
  const int c8 = (tid % CPRW) * 8, r0 = tid / CPRW;
  const int col = n0 + c8;
  const bool cok = (r0 < RPI) && col < a.N;
  const bool cs_on = CSOK && a.cs_out != nullptr;
  float g1 = 0.f, g2 = 0.f;  // column tid's sums over the slot's passes so far
  float q1[8], q2[8];        // (CSG > 1) this thread's chunk sums over its stored rows of the slot
#pragma unroll
  for (int j = 0; j < 8; ++j) { q1[j] = 0.f; q2[j] = 0.f; }
  // row vector (per-frame temb / positional-encoding rows): one row for the whole
  // tile in the common case (rows_per_vec >= the tile's row span), folded into
  // the per-column constants; otherwise looked up per row.
  const bool rv_tile = a.rowvec && out_row(0) / a.rows_per_vec == (RW > 0 ? out_row(BM - 1)
                                                                           : min(m0 + BM, a.M) - 1) / a.rows_per_vec;
  float bb[8], cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bb[j] = 0.f; cs[j] = 0.f; }
  if (cok && a.bias) load8f(a.bias + col, bb);
  if (cok && rv_tile) {
    float rv[8];
    load8f(a.rowvec + rv_row(a, out_row(0)) + col, rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) bb[j] += rv[j];
  }
  if (cok && a.ln_mr) load8f(a.ln_cs + col, cs);
  // no LayerNorm fold, no per-row row vector, unit output scale: the short path
  const bool plain = !a.ln_mr && !(a.rowvec && !rv_tile) && a.out_scale == 1.f && !(a.ablate & 8);
  EpiSide<ITER> cur;
  if constexpr (PRE) cur = pre;
  else if constexpr (PIPE) epi_side_load<BM, BN, WM, WN, RW>(a, m0, n0, m0r, tid, 0, cur);
#pragma unroll 1
  for (int p = 0; p < WM; ++p) {
    stage_acc<BM, BN, WM, WN>(acc, st, p, tid);
    // (no pipelining: this pass's residual after its staging writes, as the accumulators
    // it staged are dead -- the 256 x 256 tile has no registers to spare before that)
    if constexpr (!PIPE && !PRE) epi_side_load<BM, BN, WM, WN, RW>(a, m0, n0, m0r, tid, p, cur);
    float2 mr[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int rl = r0 + it * RPI, row = out_row(p * WTM + rl);
      mr[it] = make_float2(0.f, 1.f);
      if (cok && rl < WTM && row < a.M && a.ln_mr) mr[it] = *(const float2*)(a.ln_mr + 2L * row);
    }
    __syncthreads();
    EpiSide<ITER> nxt;
    if (PIPE && p + 1 < WM) epi_side_load<BM, BN, WM, WN, RW>(a, m0, n0, m0r, tid, p + 1, nxt);
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int rl = r0 + it * RPI, row = out_row(p * WTM + rl);
      if (!(cok && rl < WTM && row < a.M)) continue;
      const float* s = st + rl * SP + c8;
      const float4 s0 = *(const float4*)s, s1 = *(const float4*)(s + 4);
      float v[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      float r8[8];
      unpack8(cur.rs[it], r8);
      if (plain) {  // (block-uniform) bias (+ the tile's row vector) + residual: 2 VALU per value
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (v[j] + bb[j]) + r8[j];
      } else {
        float rv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) rv[j] = 0.f;
        if (a.rowvec && !rv_tile) load8f(a.rowvec + rv_row(a, row) + col, rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = mr[it].y * (v[j] - mr[it].x * cs[j]);
          v[j] = (x + bb[j] + rv[j] + r8[j]) * a.out_scale;
        }
      }
      if (GEN) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = act_fn(a.act, v[j]);
      }
      if (a.ablate & 4) {
        if (v[0] == 12345.f) ((float*)a.y)[0] = v[1];
      } else if (GEN && a.y_f32) {
        float* y = (float*)a.y + (long)row * a.ldy + col;
        *(float4*)y = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(y + 4) = make_float4(v[4], v[5], v[6], v[7]);
      } else {
        const uint4 pk = pack8(v);
        *(uint4*)((u16*)a.y + (long)row * a.ldy + col) = pk;
        if (cs_on) {
          float b[8];
          unpack8(pk, b);
          if constexpr (CSG > 1) {  // sums of the stored (bf16) values, in registers
#pragma unroll
            for (int j = 0; j < 8; ++j) { q1[j] += b[j]; q2[j] = fmaf(b[j], b[j], q2[j]); }
          } else {  // the stored values replace their fp32 staging
            float* sw = st + rl * SP + c8;
            *(float4*)sw = make_float4(b[0], b[1], b[2], b[3]);
            *(float4*)(sw + 4) = make_float4(b[4], b[5], b[6], b[7]);
          }
        }
      }
    }
    __syncthreads();
    if (cs_on && CSG > 1) {  // (block-uniform) the slot's end: the RPI chunk partials of a column meet
      if (((p + 1) * WTM) % CS_ROWS == 0) {
        float2* const part = (float2*)st;  // [RPI][BN] (sum, sum of squares)
        if (cok) {
#pragma unroll
          for (int j = 0; j < 8; ++j) part[r0 * BN + c8 + j] = make_float2(q1[j], q2[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) { q1[j] = 0.f; q2[j] = 0.f; }
        __syncthreads();
        if (tid < BN && n0 + tid < a.N) {
          float t1 = 0.f, t2 = 0.f;
#pragma unroll 5
          for (int r = 0; r < RPI; ++r) {
            const float2 v = part[r * BN + tid];
            t1 += v.x;
            t2 += v.y;
          }
          float* o = a.cs_out + (m0 + (long)p * WTM) / CS_ROWS * 2 * a.N + n0 + tid;
          o[0] = t1;
          o[a.N] = t2;
        }
        __syncthreads();  // the next pass stages into st
      }
    } else if (cs_on) {  // (block-uniform)
      const bool mine = tid < BN && n0 + tid < a.N;
      if (mine) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll 8
        for (int r = 0; r < WTM; ++r) {
          const float x = st[r * SP + tid];
          t1 += x;
          t2 = fmaf(x, x, t2);
        }
        g1 += t1;
        g2 += t2;
      }
      if (((p + 1) * WTM) % CS_ROWS == 0) {  // the slot is complete
        if (mine) {
          float* o = a.cs_out + (m0 + (long)p * WTM) / CS_ROWS * 2 * a.N + n0 + tid;
          o[0] = g1;
          o[a.N] = g2;
        }
        g1 = 0.f;
        g2 = 0.f;
      }
      __syncthreads();
    }
    if constexpr (PIPE) {
      if (p + 1 < WM) cur = nxt;
    }
  }
}

template <int BM, int BN, int WM, int WN, bool GEN, bool CSF = false, int RW = 0, int CSG = 1>
__device__ __forceinline__ void store_tile_plain(const ConvArgs& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                                 float* st, int m0, int n0, long m0r = 0, int tid_in = -1) {
  // (the 8-wave 256 x 256 tile runs at the 256-VGPR limit: its next pass's residual loads
  // would spill, so they stay in the pass)
  EpiSide<EpiGeo<BM, BN, WM, WN>::ITER> none;
  store_tile_plain_pre<BM, BN, WM, WN, GEN, CSF, RW, false, !(BM == 256 && WM == 2), CSG>(a, acc, st, m0, n0, m0r,
                                                                                          tid_in, none);
}

// GEGLU variant: a thread owns one 8-wide OUTPUT chunk, i.e. packed columns
// [ph, ph+8) (h) and [ph+16, ph+24) (g) of the 16-row-interleaved W1.
template <int BM, int BN, int WM, int WN, bool GEN>
__device__ __forceinline__ void store_tile_geglu(const ConvArgs& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                                 float* st, int m0, int n0) {
  constexpr int NT = WM * WN * 64, WTM = BM / WM, SP = BN + 4;
  constexpr int CPRW = BN / 16;
  constexpr int RPI = NT / CPRW;
  constexpr int ITER = (WTM + RPI - 1) / RPI;
  const int tid = threadIdx.x;
  const int o8 = (tid % CPRW) * 8, r0 = tid / CPRW;
  const int ph = (o8 >> 4) * 32 + (o8 & 15);
  const int col = n0 + ph;                       // packed column of h
  const int oc = (col >> 5) * 16 + (col & 15);   // output column
  const bool cok = (r0 < RPI) && col < a.N;
  float bh[8], bg[8], ch[8], cg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bh[j] = 0.f; bg[j] = 0.f; ch[j] = 0.f; cg[j] = 0.f; }
  if (cok && a.bias) { load8f(a.bias + col, bh); load8f(a.bias + col + 16, bg); }
  if (cok && a.ln_mr) { load8f(a.ln_cs + col, ch); load8f(a.ln_cs + col + 16, cg); }
#pragma unroll 1
  for (int p = 0; p < WM; ++p) {
    stage_acc<BM, BN, WM, WN>(acc, st, p, tid);
    const int rbase = m0 + p * WTM;
    float2 mr[ITER];
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int rl = r0 + it * RPI, row = rbase + rl;
      mr[it] = make_float2(0.f, 1.f);
      if (cok && rl < WTM && row < a.M && a.ln_mr) mr[it] = *(const float2*)(a.ln_mr + 2L * row);
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int rl = r0 + it * RPI, row = rbase + rl;
      if (!(cok && rl < WTM && row < a.M)) continue;
      const float* s = st + rl * SP + ph;
      float h[8], g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        h[j] = mr[it].y * (s[j] - mr[it].x * ch[j]) + bh[j];
        g[j] = mr[it].y * (s[16 + j] - mr[it].x * cg[j]) + bg[j];
        h[j] *= gelu_erf(g[j]);
      }
      if (GEN && a.y_f32) {
        float* y = (float*)a.y + (long)row * a.ldy + oc;
        *(float4*)y = make_float4(h[0], h[1], h[2], h[3]);
        *(float4*)(y + 4) = make_float4(h[4], h[5], h[6], h[7]);
      } else {
        *(uint4*)((u16*)a.y + (long)row * a.ldy + oc) = pack8(h);
      }
    }
    __syncthreads();
  }
}

// Stage the accumulator tile through LDS one wave-row (WTM rows) at a time, then
// each thread handles whole 8-column chunks (split-K slab / GEGLU / plain).
// EPI selects the epilogue compiled into a kernel instance (host: epi_kind()), so
// the common instances carry only the code they run -- the fully general
// epilogue is ~40 KB of code, and fetching it per tile cost more than the
// MFMAs of a K = 320 tile.
//   EPI_PLAIN: vectorised, no split-K, no activation, bf16 out (bias / rowvec /
//              residual / LayerNorm fold as runtime options);
//   EPI_GEGLU: the same for the GEGLU epilogue;
//   EPI_ANY:   everything (split-K slabs, GELU/SiLU, fp32 out, ragged N).
enum { EPI_PLAIN = 0, EPI_GEGLU = 1, EPI_ANY = 2 };

template <int BM, int BN, int WM, int WN, int EPI = EPI_ANY>
__device__ __forceinline__ void store_tile(const ConvArgs& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16], float* st,
                                           int m0, int n0, int z) {
  if constexpr (EPI == EPI_PLAIN) {
    // (the 4 x 2-wave 256-row tile keeps 64-row wave rows: column sums in its epilogue too)
    store_tile_plain<BM, BN, WM, WN, false, BM == 256 && WM == 4>(a, acc, st, m0, n0);
    return;
  } else if constexpr (EPI == EPI_GEGLU) {
    store_tile_geglu<BM, BN, WM, WN, false>(a, acc, st, m0, n0);
    return;
  }
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int SP = BN + 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const bool vec = (a.N % 8 == 0) && (a.ldy % 8 == 0) && (!a.res || a.ldr % 8 == 0);
  const bool geglu = a.act == LS_ACT_GEGLU;
  if (a.split == 1 && vec) {
    if (geglu) store_tile_geglu<BM, BN, WM, WN, true>(a, acc, st, m0, n0);
    else store_tile_plain<BM, BN, WM, WN, true>(a, acc, st, m0, n0);
    return;
  }
#pragma unroll 1
  for (int p = 0; p < WM; ++p) {
    if (wm == p) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            st[(i * 16 + (lane >> 4) * 4 + r) * SP + wn * WTN + j * 16 + (lane & 15)] = acc[i][j][r];
    }
    __syncthreads();
    const int rbase = m0 + p * WTM;
    if (a.split > 1) {
      float* P = a.partial + (long)z * a.M * a.N;
      for (int q = tid; q < WTM * (BN / 8); q += NT) {
        const int r = q / (BN / 8), c8 = (q - r * (BN / 8)) * 8;
        const int row = rbase + r, col = n0 + c8;
        if (row >= a.M || col >= a.N) continue;
        const float* s = st + r * SP + c8;
        if (vec) {
          *(float4*)(P + (long)row * a.N + col) = *(const float4*)s;
          *(float4*)(P + (long)row * a.N + col + 4) = *(const float4*)(s + 4);
        } else {
          for (int j = 0; j < 8 && col + j < a.N; ++j) P[(long)row * a.N + col + j] = s[j];
        }
      }
    } else if (geglu) {
      for (int q = tid; q < WTM * (BN / 16); q += NT) {
        const int r = q / (BN / 16), o8 = (q - r * (BN / 16)) * 8;
        const int ph = (o8 >> 4) * 32 + (o8 & 15);
        const int row = rbase + r, col = n0 + ph;
        if (col >= a.N) continue;
        float h[8], g[8];
        const float* s = st + r * SP + ph;
#pragma unroll
        for (int j = 0; j < 8; ++j) { h[j] = s[j]; g[j] = s[16 + j]; }
        epi_geglu8(a, row, col, h, g, vec);
      }
    } else {
      for (int q = tid; q < WTM * (BN / 8); q += NT) {
        const int r = q / (BN / 8), c8 = (q - r * (BN / 8)) * 8;
        const int row = rbase + r, col = n0 + c8;
        if (col >= a.N) continue;
        float v[8];
        const float* s = st + r * SP + c8;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = s[j];
        epi_chunk(a, row, col, v, vec && col + 8 <= a.N);
      }
    }
    __syncthreads();
  }
}

template <int BM, int BN, int WM, int WN, int KS, bool TAPU>
__global__ void __launch_bounds__(256) conv_gemm_kernel(ConvArgs a) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int AL = BM / 32, BL = BN / 32;  // 16-B chunks per thread per K-tile
  constexpr int SP = BN + 4;                 // epilogue staging pitch (floats)
  static_assert(WTM * SP * 4 <= 2 * (BM + BN) * 8 * 16, "staging must fit the LDS ring");
  __shared__ uint4 lds[2][(BM + BN) * 8];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  int bid = blockIdx.x;
  const int nt = a.ntm * a.ntn;
  const int z = bid / nt;
  bid -= z * nt;
  int tm, tn;
  tile_of(a, bid, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = z * a.kt_per_split;
  const int kt1 = min(a.ktiles, kt0 + a.kt_per_split);

  const int ch = tid & 7;
  int rm[AL];
  RowGeo geo[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    rm[i] = m;
    if (KS == 3) {
      const int hw = a.Ho * a.Wo;
      const int n = m / hw, r = m - n * hw;
      const int yo = r / a.Wo, xo = r - yo * a.Wo;
      geo[i].pb = n * a.H * a.W;
      geo[i].yb = (m < a.M) ? (a.upsample ? yo - a.pad : yo * a.stride - a.pad) : -(1 << 28);
      geo[i].xb = a.upsample ? xo - a.pad : xo * a.stride - a.pad;
    } else {
      geo[i].pb = 0; geo[i].yb = 0; geo[i].xb = 0;
    }
  }

  uint4 ra[AL], rb[BL];
  auto gload = [&](int kt) {
#pragma unroll
    for (int i = 0; i < AL; ++i) ra[i] = load_a_chunk<KS, TAPU>(a, kt, ch, rm[i], geo[i]);
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

  store_tile<BM, BN, WM, WN>(a, acc, (float*)&lds[0][0], m0, n0, z);
}


// ------------------------------------------------------------------ DMA path
// Same tiles / LDS image / epilogue, but both operands stream global -> LDS with
// global_load_lds_dwordx4 (no VGPR staging, no ds_write).  The LDS image is
// written lane-linearly, so the XOR swizzle is applied on the per-lane SOURCE
// address (logical chunk = physical chunk ^ ((row >> 1) & 7)).  Out-of-range /
// padding taps read a zero page.  Two LDS buffers: tile k+1's DMA overlaps tile
// k's MFMAs; counted vmcnt + raw s_barrier so the in-flight tile is not drained.
__device__ uint4 ls_zero_page[2];


template <int KS, bool TAPU, int BK = 64>
__device__ __forceinline__ const void* a_src(const ConvArgs& a, int kt, int c, int m, const RowGeo& g) {
  // branch-free: compute the candidate address, then select it or the zero page
  int cg, tap = 0;
  bool ok;
  if (KS == 1) {
    cg = kt * BK + c * 8;
    ok = (m < a.M) & (cg < a.Cin);
  } else if (TAPU) {
    tap = tap_of(a, kt * BK, cg);
    cg += c * 8;
    ok = true;
  } else {
    const int kc = kt * (BK / 8) + c;
    tap = kc / a.CC;
    cg = (kc - tap * a.CC) * 8;
    ok = tap < 9;
  }
  int pix;
  if (KS == 1) {
    pix = m;
  } else {
    const int kh = tap / 3, kw = tap - kh * 3;
    int yy = g.yb + kh, xx = g.xb + kw;
    const int lim_y = a.upsample ? 2 * a.H : a.H, lim_x = a.upsample ? 2 * a.W : a.W;
    ok &= ((unsigned)yy < (unsigned)lim_y) & ((unsigned)xx < (unsigned)lim_x);
    yy >>= a.upsample;
    xx >>= a.upsample;
    pix = g.pb + yy * a.W + xx;
  }
  const bool second = cg >= a.C1;
  const u16* base = second ? a.x2 : a.x1;
  const long off = (long)pix * (second ? a.ld2 : a.ld1) + (second ? cg - a.C1 : cg);
  return ok ? (const void*)(base + off) : (const void*)ls_zero_page;
}

// XCD-aware block order: blocks b and b+8 share an XCD under round-robin
// dispatch, so give every XCD a contiguous range of tiles (shared A rows /
// 3x3 halos / weight panels stay in one L2).  Bijective for any grid size.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}


// Operand DMA through buffer descriptors for a BM x BN x 64 tile whose threads each
// move AI A pieces and BI B pieces of 16 B per K-tile (LDS images lane-linear per
// wave, 64 pieces per wave-instruction; the XOR swizzle is folded into the chunk
// offsets ach / bch).  See conv_gemm_dma_kernel's BUF note.
__device__ i32x4 ls_raw_buffer_load_v4(i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4i32");

template <int BM, int BN, int AI, int BI, int KS>
struct BufDma {
  i32x4 rs_a1, rs_a2, rs_b;
  int avo1[AI], avo2[AI], bvo[BI];
  unsigned amask[AI];
  int tap = 0, c0 = 0;  // 3x3: tap / channel offset of the next K-tile (next())

  // arow / brow: tile-relative row of each piece; ach / bch: its logical 16-B chunk
  __device__ __forceinline__ void init(const ConvArgs& a, int m0, int n0, const int* arow, const int* ach,
                                       const int* brow, const int* bch) {
    const long cap = 0x7FFFFFFFL;
    if (KS == 1) {  // (rows of one tile: the concat halves share the row index)
      rs_a1 = buffer_rsrc(a.x1 + (long)m0 * a.ld1, (uint32_t)min((long)(a.M - m0) * a.ld1 * 2, cap));
      rs_a2 = a.C2 ? buffer_rsrc(a.x2 + (long)m0 * a.ld2, (uint32_t)min((long)(a.M - m0) * a.ld2 * 2, cap)) : rs_a1;
#pragma unroll
      for (int p = 0; p < AI; ++p) {
        avo1[p] = (arow[p] * a.ld1 + ach[p] * 8) * 2;
        avo2[p] = (arow[p] * a.ld2 + ach[p] * 8) * 2;
        amask[p] = 0x1FF;
      }
    } else if (a.upsample) {
      // nearest x2 then 3x3 pad 1: upsampled (yo - 1 + kh, xo - 1 + kw) reads input
      // (i - 1 + r, j - 1 + c), i = yo >> 1, r = (py + kh + 1) >> 1 (py = yo & 1), likewise
      // c: the tap's uniform shift r0 W + c0 (py = px = 0) plus W / 1 pixel for the odd
      // rows / columns of taps kh / kw != 1 (parity bits 9 / 10 of amask)
      const int HWi = a.H * a.W, HWo = a.Ho * a.Wo;
      const long base_pix = (long)(m0 / HWo) * HWi - a.W - 1;
      const long tot_pix = (long)a.n_img * HWi;
      rs_a1 = buffer_rsrc(a.x1 + base_pix * a.ld1, (uint32_t)min((tot_pix - base_pix) * a.ld1 * 2, cap));
      rs_a2 = a.C2 ? buffer_rsrc(a.x2 + base_pix * a.ld2, (uint32_t)min((tot_pix - base_pix) * a.ld2 * 2, cap))
                   : rs_a1;
#pragma unroll
      for (int p = 0; p < AI; ++p) {
        const int m = m0 + arow[p];
        const int n = m / HWo, r = m - n * HWo;
        const int yo = r / a.Wo, xo = r - yo * a.Wo;
        const int win = (int)((long)n * HWi + (long)((yo >> 1) - 1) * a.W + ((xo >> 1) - 1) - base_pix);
        avo1[p] = (win * a.ld1 + ach[p] * 8) * 2;
        avo2[p] = (win * a.ld2 + ach[p] * 8) * 2;
        unsigned mk = ((unsigned)(yo & 1) << 9) | ((unsigned)(xo & 1) << 10);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const bool ok = m < a.M && (unsigned)(yo - 1 + kh) < (unsigned)a.Ho && (unsigned)(xo - 1 + kw) < (unsigned)a.Wo;
            mk |= (ok ? 1u : 0u) << (kh * 3 + kw);
          }
        amask[p] = mk;
      }
    } else {  // output pixel (yo, xo) reads input (yo s - pad + kh, xo s - pad + kw)
      const int HWi = a.H * a.W, HWo = a.Ho * a.Wo;
      const long base_pix = (long)(m0 / HWo) * HWi - (long)a.pad * a.W - a.pad;
      const long tot_pix = (long)a.n_img * HWi;
      rs_a1 = buffer_rsrc(a.x1 + base_pix * a.ld1, (uint32_t)min((tot_pix - base_pix) * a.ld1 * 2, cap));
      rs_a2 = a.C2 ? buffer_rsrc(a.x2 + base_pix * a.ld2, (uint32_t)min((tot_pix - base_pix) * a.ld2 * 2, cap))
                   : rs_a1;
#pragma unroll
      for (int p = 0; p < AI; ++p) {
        const int m = m0 + arow[p];
        const int n = m / HWo, r = m - n * HWo;
        const int yo = r / a.Wo, xo = r - yo * a.Wo;
        const int yt = yo * a.stride - a.pad, xt = xo * a.stride - a.pad;  // window top-left
        const int win = (int)((long)n * HWi + (long)yt * a.W + xt - base_pix);
        avo1[p] = (win * a.ld1 + ach[p] * 8) * 2;
        avo2[p] = (win * a.ld2 + ach[p] * 8) * 2;
        unsigned mk = 0;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const bool ok = m < a.M && (unsigned)(yt + kh) < (unsigned)a.H && (unsigned)(xt + kw) < (unsigned)a.W;
            mk |= (ok ? 1u : 0u) << (kh * 3 + kw);
          }
        amask[p] = mk;
      }
    }
    rs_b = buffer_rsrc(a.w + (long)n0 * a.K, (uint32_t)min((long)(a.N - n0) * a.K * 2, cap));
#pragma unroll
    for (int p = 0; p < BI; ++p) bvo[p] = (brow[p] * a.K + bch[p] * 8) * 2;
  }

  // uniform per-K-tile offsets.  next(): K-tiles requested in increasing order from the
  // first (3x3: the tap / channel offset advance; the first of a split divides once)
  struct KTile { int soff_a, soff_b, tap, dy, dx; bool two; };
  __device__ __forceinline__ KTile next(const ConvArgs& a, int kt) {
    KTile k;
    k.soff_b = kt * 128;
    k.dy = 0;
    k.dx = 0;
    if (KS == 1) {
      k.tap = 0;
      k.two = a.C2 && kt * 64 >= a.C1;  // concat: a K-tile lies in one source (host: C1 % 64 == 0)
      k.soff_a = k.two ? (kt * 64 - a.C1) * 2 : kt * 128;
    } else {
      if (c0 == 0 && tap == 0 && kt != 0) tap = tap_of(a, kt * 64, c0);
      const int kh = tap / 3, kw = tap - kh * 3;
      k.tap = tap;
      k.two = c0 >= a.C1;
      const int ld = k.two ? a.ld2 : a.ld1;
      if (a.upsample) {
        k.soff_a = ((((kh + 1) >> 1) * a.W + ((kw + 1) >> 1)) * ld + (k.two ? c0 - a.C1 : c0)) * 2;
        k.dy = kh != 1 ? a.W * ld * 2 : 0;
        k.dx = kw != 1 ? ld * 2 : 0;
      } else {
        k.soff_a = ((kh * a.W + kw) * ld + (k.two ? c0 - a.C1 : c0)) * 2;
      }
      if (a.ccm) {
        if (++tap == 9) { tap = 0; c0 += 64; }
      } else {
        c0 += 64;
        if (c0 == a.Cin) { c0 = 0; ++tap; }
      }
    }
    return k;
  }

  __device__ __forceinline__ void load_a(int p, uint4* dst, const KTile& k, bool ups = false) const {
    int v = k.two ? avo2[p] : avo1[p];
    if (KS == 3 && ups) v += ((amask[p] >> 9) & 1u ? k.dy : 0) + ((amask[p] >> 10) & 1u ? k.dx : 0);
    const int vo = KS == 1 ? v : (((amask[p] >> k.tap) & 1u) ? v : (int)0x80000000);
    ls_raw_buffer_load_lds(k.two ? rs_a2 : rs_a1, (__attribute__((address_space(3))) void*)dst, 16, vo, k.soff_a, 0, 0);
  }
  __device__ __forceinline__ void load_b(int p, uint4* dst, const KTile& k) const {
    ls_raw_buffer_load_lds(rs_b, (__attribute__((address_space(3))) void*)dst, 16, bvo[p], k.soff_b, 0, 0);
  }
  // the same pieces into registers (register-staged variant: buffer_load_dwordx4 + ds_write_b128)
  __device__ __forceinline__ uint4 reg_a(int p, const KTile& k, bool ups = false) const {
    int v = k.two ? avo2[p] : avo1[p];
    if (KS == 3 && ups) v += ((amask[p] >> 9) & 1u ? k.dy : 0) + ((amask[p] >> 10) & 1u ? k.dx : 0);
    const int vo = KS == 1 ? v : (((amask[p] >> k.tap) & 1u) ? v : (int)0x80000000);
    return __builtin_bit_cast(uint4, ls_raw_buffer_load_v4(k.two ? rs_a2 : rs_a1, vo, k.soff_a, 0));
  }
  __device__ __forceinline__ uint4 reg_b(int p, const KTile& k) const {
    return __builtin_bit_cast(uint4, ls_raw_buffer_load_v4(rs_b, bvo[p], k.soff_b, 0));
  }

  // the whole K-tile kt into the A / B images of a stage (pieces lane-linear per wave)
  __device__ __forceinline__ void issue(const ConvArgs& a, int kt, uint4* a_img, uint4* b_img, int wid_u) {
    const KTile k = next(a, kt);
    if (KS == 3 && a.upsample) {  // (uniform branch: the parity adds only where they apply)
#pragma unroll
      for (int p = 0; p < AI; ++p) load_a(p, a_img + (wid_u * AI + p) * 64, k, true);
    } else {
#pragma unroll
      for (int p = 0; p < AI; ++p) load_a(p, a_img + (wid_u * AI + p) * 64, k);
    }
#pragma unroll
    for (int p = 0; p < BI; ++p) load_b(p, b_img + (wid_u * BI + p) * 64, k);
  }
};

// BUF: operand DMA through buffer descriptors (host: buf_dma_ok) -- every per-thread
// byte offset is computed once; a K-tile only changes the uniform soffset (and, for
// a 3x3 tap, one select per piece between the precomputed window offset and an
// out-of-range offset that reads zeros), so the K loop carries no 64-bit address
// arithmetic: ~90-125 VALU per K-tile less than the global_load_lds path, which
// competes with the MFMAs for vector issue.  1x1: A rows of the tile from a
// descriptor at row m0 (rows past M read zeros), B rows from one at column n0.
// 3x3 (stride 1 / 2, pad 0 / 1, C1 % 64 == 0): the descriptor starts pad (W + 1)
// pixels before the tile's first input image, so every window's top-left pixel has
// a non-negative offset; the tap's (kh W + kw) pixel shift and channel offset go in
// soffset, taps outside the image select an offset past the descriptor (zeros).
template <int BM, int BN, int WM, int WN, int KS, bool TAPU, int NST, int BK, int EPI, bool BUF = false>
__global__ void __launch_bounds__(WM * WN * 64) conv_gemm_dma_kernel(ConvArgs a) {
  constexpr int NT = WM * WN * 64;                    // 256 (4 waves) or 512 (8 waves, 256-row tiles)
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int CPR = BK / 8;                         // 16-B chunks per row
  constexpr int AI = BM * CPR / NT, BI = BN * CPR / NT;  // DMA wave-instructions per wave per K-tile
  static_assert((BM * CPR) % NT == 0 && (BN * CPR) % NT == 0, "operand pieces must divide over the threads");
  constexpr int L = AI + BI;
  constexpr int KSTEPS = BK / 32;
  constexpr int STAGE = (BM + BN) * CPR;              // uint4 per stage
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  uint4* lds = lds_dyn;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nt = a.ntm * a.ntn;
  int bid = xcd_remap(blockIdx.x, nt * a.split);
  const int z = bid / nt;
  bid -= z * nt;
  int tm, tn;
  tile_of(a, bid, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ktiles = a.K / BK;
  const int kps = a.kt_per_split * (64 / BK);
  const int kt0 = z * kps;
  const int kt1 = min(ktiles, kt0 + kps);

  int arow[AI], ach[AI], brow[BI], bch[BI];
  RowGeo geo[AI];
#pragma unroll
  for (int p = 0; p < AI; ++p) {
    const int q = (wid * AI + p) * 64 + lane;
    const int row = q / CPR;
    const int pc = q % CPR;
    arow[p] = m0 + row;
    ach[p] = swz_bk<BK>(row, pc) - row * CPR;  // logical chunk stored at physical chunk pc (involution)
    if (KS == 3) {
      const int m = m0 + row;
      const int hw = a.Ho * a.Wo;
      const int n = m / hw, r = m - n * hw;
      const int yo = r / a.Wo, xo = r - yo * a.Wo;
      geo[p].pb = n * a.H * a.W;
      geo[p].yb = (m < a.M) ? (a.upsample ? yo - a.pad : yo * a.stride - a.pad) : -(1 << 28);
      geo[p].xb = a.upsample ? xo - a.pad : xo * a.stride - a.pad;
    } else {
      geo[p].pb = 0; geo[p].yb = 0; geo[p].xb = 0;
    }
  }
#pragma unroll
  for (int p = 0; p < BI; ++p) {
    const int q = (wid * BI + p) * 64 + lane;
    const int row = q / CPR;
    brow[p] = n0 + row;
    bch[p] = swz_bk<BK>(row, q % CPR) - row * CPR;
  }
  static_assert(!BUF || (BK == 64 && (KS == 1 || TAPU)), "buffer DMA: BK 64, 1x1 or tap-major 3x3");
  BufDma<BM, BN, AI, BI, KS> bd;  // BUF (dead code otherwise)
  if constexpr (BUF) {
    int ar[AI], br[BI];
#pragma unroll
    for (int p = 0; p < AI; ++p) ar[p] = arow[p] - m0;
#pragma unroll
    for (int p = 0; p < BI; ++p) br[p] = brow[p] - n0;
    bd.init(a, m0, n0, ar, ach, br, bch);
  }
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  auto issue = [&](int kt, int stage) {
    uint4* base = lds + stage * STAGE;
    if constexpr (BUF) {
      bd.issue(a, kt, base, base + BM * CPR, wid_u);
    } else {
#pragma unroll
      for (int p = 0; p < AI; ++p)
        glds16(a_src<KS, TAPU, BK>(a, kt, ach[p], arow[p], geo[p]), base + (wid * AI + p) * 64);
#pragma unroll
      for (int p = 0; p < BI; ++p) {
        const void* src = brow[p] < a.N ? (const void*)(a.w + (long)brow[p] * a.K + kt * BK + bch[p] * 8)
                                        : (const void*)ls_zero_page;
        glds16(src, base + BM * CPR + (wid * BI + p) * 64);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const bool do_dma = !(a.ablate & 2);
#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (kt0 + t < kt1 && do_dma) issue(kt0 + t, t);
  // ILV (2-stage buffer-descriptor path): the next K-tile's DMA is issued after this
  // K-tile's barrier, its wave-instructions spread between the MFMAs (sched_group_barrier)
  // instead of one burst before the wait -- an LDS-DMA instruction costs ~60 issue cycles
  // among MFMAs but 100-185 in a burst beside the fragment reads (MI355X_MICROARCH.md).  Its
  // stage was last read in K-tile kt - 1, whose trailing barrier every wave has passed.
  constexpr bool ILV = false;  // (A/B: BUF && NST == 2)
  constexpr bool ILV_SGB = false;  // explicit interleave (sched_group_barrier): see DESIGN
  int stage = 0;
  // the plain epilogue's first-pass side inputs (residual / LayerNorm rows), loaded during
  // the last K-tile so their HBM latency hides under its MFMAs
  EpiSide<EpiGeo<BM, BN, WM, WN>::ITER> pre;
  // one K-tile; IS: issue the next K-tile's DMA inside it (ILV).  (Peeling the last K-tile so
  // that the DMA and the MFMAs share one basic block made the register allocator rotate the
  // accumulators through AGPR moves, ~90 per K-tile: not kept.)
  auto ktile = [&](int kt, auto is_tag) {
    constexpr bool IS = decltype(is_tag)::value;
    if (!ILV && kt + NST - 1 < kt1 && do_dma) issue(kt + NST - 1, (stage + NST - 1) % NST);
    const int ahead = ILV ? 0 : min(NST - 1, kt1 - 1 - kt);
    if (NST >= 4 && ahead >= 3) wait_vm<3 * L>();
    else if (NST >= 3 && ahead >= 2) wait_vm<2 * L>();
    else if (ahead >= 1) wait_vm<L>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (EPI == EPI_PLAIN) {
      if (kt == kt1 - 1) epi_side_load<BM, BN, WM, WN>(a, m0, n0, 0, tid, 0, pre);
    }
    const uint4* cur = lds + stage * STAGE;
    bf16x8 af[KSTEPS][FM], bfr[KSTEPS][FN];
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks) {
      const int c = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[ks][i] = __builtin_bit_cast(bf16x8, cur[swz_bk<BK>(wm * WTM + i * 16 + (lane & 15), c)]);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[ks][j] = __builtin_bit_cast(bf16x8, cur[BM * CPR + swz_bk<BK>(wn * WTN + j * 16 + (lane & 15), c)]);
    }
    if (ILV && IS && kt + 1 < kt1 && do_dma) issue(kt + 1, stage ^ 1);
#ifdef LS_GEMM_ABLATE
    if (!(a.ablate & 16))
#endif
    {
#pragma unroll
      for (int ks = 0; ks < KSTEPS; ++ks)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[i][j], 0, 0, 0);
    }
    if constexpr (ILV && IS && ILV_SGB) {  // fragment reads first, then L x (one DMA, MFMAs), the rest
      constexpr int NMF = KSTEPS * FM * FN, PER = NMF / (L + 1) > 0 ? NMF / (L + 1) : 1;
      __builtin_amdgcn_sched_group_barrier(0x100, KSTEPS * (FM + FN), 0);
#pragma unroll
      for (int r = 0; r < L; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NMF - L * PER > 0 ? NMF - L * PER : 0, 0);
    }
#ifdef LS_GEMM_ABLATE
    else if (a.ablate & 32) {
      acc[0][0][0] += (float)af[0][0][0] + (float)bfr[0][0][0];
    }
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stage = stage + 1 == NST ? 0 : stage + 1;
  };
  for (int kt = kt0; kt < kt1; ++kt) ktile(kt, std::true_type{});
#ifdef LS_GEMM_ABLATE  // diagnostic build only (hipcc -DLS_GEMM_ABLATE): it costs registers
  if (a.ablate & 8) {  // tuning: no epilogue at all (keep the accumulators live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][3];
    if (t == 12345.f) ((float*)a.y)[tid] = t;
    return;
  }
#endif
  if constexpr (EPI == EPI_PLAIN) {
    if (kt0 < kt1) {
      store_tile_plain_pre<BM, BN, WM, WN, false, BM == 256 && WM == 4, 0, true>(a, acc, (float*)lds, m0, n0, 0, -1,
                                                                                 pre);
      return;
    }
  }
  store_tile<BM, BN, WM, WN, EPI>(a, acc, (float*)lds, m0, n0, z);
}

#ifdef LS_DIAG_KERNELS  // measured and rejected: diagnostics build only
// Register-staged variant of conv_gemm_dma_kernel's BUF path (A/B switch LS_GEMM_RS=1):
// the same buffer-descriptor offsets, but each 16-B operand piece goes through a VGPR
// (buffer_load_dwordx4, then ds_write_b128 into the slot the LDS-DMA would have written)
// instead of buffer_load ... lds.  MI355X_MICROARCH.md prices an LDS-DMA wave-instruction
// at ~60 issue cycles beside MFMAs; a VMEM load + a 16-B LDS store are a fraction of that,
// at the cost of 4 VGPRs per piece held across the K-tile's MFMAs.  Loads of K-tile t+1
// are issued right after the barrier of K-tile t and stored after its MFMAs.
template <int BM, int BN, int WM, int WN, int KS, int EPI>
__global__ void __launch_bounds__(WM * WN * 64) conv_gemm_rs_kernel(ConvArgs a) {
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int CPR = 8;
  constexpr int AI = BM * CPR / NT, BI = BN * CPR / NT;
  static_assert((BM * CPR) % NT == 0 && (BN * CPR) % NT == 0, "operand pieces must divide over the threads");
  constexpr int STAGE = (BM + BN) * CPR;
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  uint4* lds = lds_dyn;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nt = a.ntm * a.ntn;
  int bid = xcd_remap(blockIdx.x, nt);
  int tm, tn;
  tile_of(a, bid, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt1 = a.ktiles;

  int ar[AI], ach[AI], br[BI], bch[BI];
#pragma unroll
  for (int p = 0; p < AI; ++p) {
    const int q = (wid * AI + p) * 64 + lane;
    const int row = q / CPR;
    ar[p] = row;
    ach[p] = swz_bk<64>(row, q % CPR) - row * CPR;
  }
#pragma unroll
  for (int p = 0; p < BI; ++p) {
    const int q = (wid * BI + p) * 64 + lane;
    const int row = q / CPR;
    br[p] = row;
    bch[p] = swz_bk<64>(row, q % CPR) - row * CPR;
  }
  BufDma<BM, BN, AI, BI, KS> bd;
  bd.init(a, m0, n0, ar, ach, br, bch);
  uint4 ra[AI], rb[BI];
  auto gload = [&](int kt) {
    const auto k = bd.next(a, kt);
    const bool ups = KS == 3 && a.upsample;
#pragma unroll
    for (int p = 0; p < AI; ++p) ra[p] = bd.reg_a(p, k, ups);
#pragma unroll
    for (int p = 0; p < BI; ++p) rb[p] = bd.reg_b(p, k);
  };
  auto lstore = [&](int stage) {
    uint4* base = lds + stage * STAGE;
#pragma unroll
    for (int p = 0; p < AI; ++p) base[(wid * AI + p) * 64 + lane] = ra[p];
#pragma unroll
    for (int p = 0; p < BI; ++p) base[BM * CPR + (wid * BI + p) * 64 + lane] = rb[p];
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  gload(0);
  lstore(0);
  int stage = 0;
  for (int kt = 0; kt < kt1; ++kt) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = kt + 1 < kt1;
    if (more) gload(kt + 1);
    const uint4* cur = lds + stage * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + (lane >> 4);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = __builtin_bit_cast(bf16x8, cur[swz_bk<64>(wm * WTM + i * 16 + (lane & 15), c)]);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = __builtin_bit_cast(bf16x8, cur[BM * CPR + swz_bk<64>(wn * WTN + j * 16 + (lane & 15), c)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) lstore(stage ^ 1);  // stage ^ 1 was read in K-tile kt - 1, before this barrier
    stage ^= 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  store_tile<BM, BN, WM, WN, EPI>(a, acc, (float*)lds, m0, n0, 0);
}

// 1x1 GEMM with the A operand straight into registers (A/B switch LS_GEMM_AREG / tuning key
// 14): a lane's A fragment of a 32-wide k-step is 8 consecutive channels of one row -- 16
// contiguous bytes of the NHWC activation -- so it is one buffer_load_dwordx4 into the MFMA
// operand registers, no LDS.  Only B (the weights) goes through an LDS-DMA ring (3 stages,
// 20 KB each at BN 160): per K-tile a wave issues BN/32 LDS-DMA instructions instead of
// (BM + BN)/32, the rest of the operand traffic being plain vector loads (each A element is
// read by the WN waves of its row band, from L1 / L2).  A of K-tile kt + 1 is loaded during
// K-tile kt (two register sets, the K loop unrolled by 2 so the sets are static).
template <int BM, int BN, int WM, int WN, int EPI>
__global__ void __launch_bounds__(WM * WN * 64) conv_gemm_areg_kernel(ConvArgs a) {
  constexpr int NT = WM * WN * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  constexpr int BI = BN * 8 / NT;
  static_assert((BN * 8) % NT == 0, "B pieces must divide over the threads");
  constexpr int STAGE = BN * 8;  // uint4 per B stage
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  uint4* lds = lds_dyn;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int wm = wid / WN, wn = wid % WN;
  const int nt = a.ntm * a.ntn;
  int bid = xcd_remap(blockIdx.x, nt);
  int tm, tn;
  tile_of(a, bid, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt1 = a.K / 64;
  const long cap = 0x7FFFFFFFL;

  // A: rows past M read zeros (descriptor size); concat K-tiles from x2 (host: C1 % 64 == 0)
  const i32x4 rs_a1 = buffer_rsrc(a.x1 + (long)m0 * a.ld1, (uint32_t)min((long)(a.M - m0) * a.ld1 * 2, cap));
  const i32x4 rs_a2 =
      a.C2 ? buffer_rsrc(a.x2 + (long)m0 * a.ld2, (uint32_t)min((long)(a.M - m0) * a.ld2 * 2, cap)) : rs_a1;
  int avo1[FM], avo2[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int r = wm * WTM + i * 16 + l16;
    avo1[i] = (r * a.ld1 + lg * 8) * 2;
    avo2[i] = (r * a.ld2 + lg * 8) * 2;
  }
  // B: pieces lane-linear per wave, 16-B chunks XOR-swizzled as in the LDS-DMA kernels
  const i32x4 rs_b = buffer_rsrc(a.w + (long)n0 * a.K, (uint32_t)min((long)(a.N - n0) * a.K * 2, cap));
  int bvo[BI];
#pragma unroll
  for (int p = 0; p < BI; ++p) {
    const int q = (wid * BI + p) * 64 + lane, row = q / 8;
    const int lc = swz_bk<64>(row, q % 8) - row * 8;  // logical chunk stored at physical chunk q % 8
    bvo[p] = (row * a.K + lc * 8) * 2;
  }
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  auto issue_b = [&](int kt) {
    uint4* base = lds + (kt % 3) * STAGE;
#pragma unroll
    for (int p = 0; p < BI; ++p)
      ls_raw_buffer_load_lds(rs_b, (__attribute__((address_space(3))) void*)(base + (wid_u * BI + p) * 64), 16, bvo[p],
                             kt * 128, 0, 0);
  };
  bf16x8 ar[2][2][FM];  // [register set][k-step][fragment]
  auto load_a = [&](int kt, bf16x8 (&r)[2][FM]) {
    const bool two = a.C2 && kt * 64 >= a.C1;
    const int soff = (two ? kt * 64 - a.C1 : kt * 64) * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
        r[ks][i] = __builtin_bit_cast(bf16x8, ls_raw_buffer_load_v4(two ? rs_a2 : rs_a1, two ? avo2[i] : avo1[i],
                                                                    soff + ks * 64, 0));
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  issue_b(0);
  if (kt1 > 1) issue_b(1);
  load_a(0, ar[0]);
  // K-tile kt from register set CUR; B of kt lands in stage kt % 3 (issued two K-tiles ahead)
  auto body = [&](int kt, auto cur_tag) {
    constexpr int CUR = decltype(cur_tag)::value;
    if (kt + 2 < kt1) issue_b(kt + 2);
    if (kt + 1 < kt1) load_a(kt + 1, ar[CUR ^ 1]);
    // B(kt) and A(kt) landed: the VMEM instructions younger than A(kt) are B(kt + 2) and A(kt + 1)
    if (kt + 2 < kt1) wait_vm<BI + 2 * FM>();
    else if (kt + 1 < kt1) wait_vm<2 * FM>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const uint4* cur = lds + (kt % 3) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = __builtin_bit_cast(bf16x8, cur[swz_bk<64>(wn * WTN + j * 16 + l16, ks * 4 + lg)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[CUR][ks][i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage kt % 3 free for B(kt + 3)
    asm volatile("" ::: "memory");
  };
  int kt = 0;
  for (; kt + 1 < kt1; kt += 2) {
    body(kt, std::integral_constant<int, 0>{});
    body(kt + 1, std::integral_constant<int, 1>{});
  }
  if (kt < kt1) body(kt, std::integral_constant<int, 0>{});
  store_tile<BM, BN, WM, WN, EPI>(a, acc, (float*)lds, m0, n0, 0);
}

#endif  // LS_DIAG_KERNELS

// 256-row tile, 8 waves (2 M x 4 N), each wave 128 x BN/4 (FM = 8 fragments of
// 16 rows x FN of 16 cols): 1.5x the MFMAs per LDS fragment read of the 4-wave
// 64 x 64 wave tile.  One block per CU (128 KB of LDS: two 64-KB stages at
// BN = 256), glds operand DMA into XOR-swizzled lane-linear images, one raw
// barrier per K-tile; the next tile's DMA is issued right after the barrier so
// it has a whole K-tile of MFMAs to land.  MFMA runs are bracketed by
// s_setprio(1) so the co-resident wave's fragment reads interleave.
template <int BN, int KS, bool TAPU, int EPI, bool BUF = false>
__global__ void __launch_bounds__(512) conv_gemm_big_kernel(ConvArgs a) {
  constexpr int BM = 256, BK = 64, WM = 2, WN = 4;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16, FH = FM / 2;
  constexpr int CPR = BK / 8;
  constexpr int AI = BM * CPR / 512, BI = BN * CPR / 512;
  constexpr int STAGE = (BM + BN) * CPR;
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  uint4* lds = lds_dyn;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nt = a.ntm * a.ntn;
  int bid = xcd_remap(blockIdx.x, nt * a.split);
  const int z = bid / nt;
  bid -= z * nt;
  int tm, tn;
  tile_of(a, bid, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = z * a.kt_per_split;
  const int kt1 = min(a.ktiles, kt0 + a.kt_per_split);

  int arow[AI], ach[AI], brow[BI], bch[BI];
  RowGeo geo[AI];
#pragma unroll
  for (int p = 0; p < AI; ++p) {
    const int q = (wid * AI + p) * 64 + lane;
    const int row = q / CPR;
    arow[p] = m0 + row;
    ach[p] = swz_bk<BK>(row, q % CPR) - row * CPR;
    if (KS == 3) {
      const int m = m0 + row;
      const int hw = a.Ho * a.Wo;
      const int n = m / hw, r = m - n * hw;
      const int yo = r / a.Wo, xo = r - yo * a.Wo;
      geo[p].pb = n * a.H * a.W;
      geo[p].yb = (m < a.M) ? (a.upsample ? yo - a.pad : yo * a.stride - a.pad) : -(1 << 28);
      geo[p].xb = a.upsample ? xo - a.pad : xo * a.stride - a.pad;
    } else {
      geo[p].pb = 0; geo[p].yb = 0; geo[p].xb = 0;
    }
  }
#pragma unroll
  for (int p = 0; p < BI; ++p) {
    const int q = (wid * BI + p) * 64 + lane;
    const int row = q / CPR;
    brow[p] = n0 + row;
    bch[p] = swz_bk<BK>(row, q % CPR) - row * CPR;
  }
  static_assert(!BUF || KS == 1 || TAPU, "buffer DMA: 1x1 or tap-major 3x3");
  BufDma<BM, BN, AI, BI, KS> bd;  // BUF (dead code otherwise)
  if constexpr (BUF) {
    int ar[AI], br[BI];
#pragma unroll
    for (int p = 0; p < AI; ++p) ar[p] = arow[p] - m0;
#pragma unroll
    for (int p = 0; p < BI; ++p) br[p] = brow[p] - n0;
    bd.init(a, m0, n0, ar, ach, br, bch);
  }
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  auto issue = [&](int kt, int stage) {
    uint4* base = lds + stage * STAGE;
    if constexpr (BUF) {
      bd.issue(a, kt, base, base + BM * CPR, wid_u);
      return;
    }
#pragma unroll
    for (int p = 0; p < AI; ++p)
      glds16(a_src<KS, TAPU, BK>(a, kt, ach[p], arow[p], geo[p]), base + (wid * AI + p) * 64);
#pragma unroll
    for (int p = 0; p < BI; ++p) {
      const void* src = brow[p] < a.N ? (const void*)(a.w + (long)brow[p] * a.K + kt * BK + bch[p] * 8)
                                      : (const void*)ls_zero_page;
      glds16(src, base + BM * CPR + (wid * BI + p) * 64);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) issue(kt0, 0);
  int stage = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    wait_vm<0>();  // this wave's share of tile kt has landed
    __builtin_amdgcn_s_barrier();  // ... everyone's, and stage^1 is no longer read
    asm volatile("" ::: "memory");
    if (kt + 1 < kt1) issue(kt + 1, stage ^ 1);
    const uint4* cur = lds + stage * STAGE;
    bf16x8 bfr[2][FN], af[2][FH];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[ks][j] = __builtin_bit_cast(bf16x8, cur[BM * CPR + swz_bk<BK>(wn * WTN + j * 16 + (lane & 15), c)]);
#pragma unroll
      for (int i = 0; i < FH; ++i)
        af[ks][i] = __builtin_bit_cast(bf16x8, cur[swz_bk<BK>(wm * WTM + i * 16 + (lane & 15), c)]);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 an[2][FH];
      if (h == 0) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + (lane >> 4);
#pragma unroll
          for (int i = 0; i < FH; ++i)
            an[ks][i] = __builtin_bit_cast(bf16x8, cur[swz_bk<BK>(wm * WTM + (FH + i) * 16 + (lane & 15), c)]);
        }
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < FH; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[h * FH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[ks][j], acc[h * FH + i][j],
                                                                          0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      if (h == 0) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < FH; ++i) af[ks][i] = an[ks][i];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage ^= 1;
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  store_tile<BM, BN, WM, WN, EPI>(a, acc, (float*)lds, m0, n0, z);
}

#ifdef LS_DIAG_KERNELS  // measured and rejected: diagnostics build only
// 256 x 256 x 64 tile, 8 waves (2 M x 4 N, 128 x 64 per wave), phased schedule
// (after the guide's 8-phase template): each K-tile runs as 4 phases, one per
// 64 x 32 quadrant of the wave tile (16 MFMAs).  A phase issues the fragment
// reads it needs (A quadrant rows and/or B quadrant cols), ONE half-tile of
// operand DMA (2 glds per thread; half-tiles A0 A1 B0 B1 = 128 rows x 64 k)
// D = 5 half-tiles ahead, barrier, waits for its reads (they overlap the
// barrier), MFMAs at raised priority, barrier.  The DMA for tile t+1 is retired
// by a counted vmcnt(2) in phase 3 of tile t, so operand loads span barriers and
// never drain in the main loop.  Hazards (g = 4t + phase): half g+5 overwrites
// half g-3 -- A0(t) last read by row 0 at 4t+2, re-staged at 4t+3 after that
// row retired the reads in its own phase 4t+2; A1 at 4t+4, B0 at 4t+5, B1 at
// 4t+6 (B last read at 4t+1).  Row 1 runs one barrier behind row 0.
template <int KS, bool TAPU>
__global__ void __launch_bounds__(512) conv_gemm_p8_kernel(ConvArgs a) {
  constexpr int BM = 256, BN = 256, BK = 64, CPR = 8;
  constexpr int HALF = 128 * CPR;         // uint4 per half-tile (16 KB)
  constexpr int BUF = 4 * HALF;           // A0 A1 B0 B1
  constexpr int D = 5;                    // half-tiles of DMA issued ahead
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  uint4* lds = lds_dyn;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int nt = a.ntm * a.ntn;
  int bid = xcd_remap(blockIdx.x, nt * a.split);
  const int z = bid / nt;
  bid -= z * nt;
  int tm, tn;
  tile_of(a, bid, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = z * a.kt_per_split;
  const int nk = min(a.ktiles, kt0 + a.kt_per_split) - kt0;
  const int nhalf = 4 * nk;

  // per-thread DMA geometry: instruction i (0, 1) of each half covers rows (wid*2+i)*8 + lane/8
  int arow[4], ach[4], brow[4], bch[4];
  RowGeo geo[4];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = (wid * 2 + i) * 64 + lane;
      const int row = q / CPR, pc = q % CPR;
      const int lc = swz_bk<BK>(row, pc) - row * CPR;
      const int p = hh * 2 + i;
      arow[p] = m0 + hh * 128 + row;
      ach[p] = lc;
      brow[p] = n0 + hh * 128 + row;
      bch[p] = lc;
      if (KS == 3) {
        const int m = arow[p];
        const int hw = a.Ho * a.Wo;
        const int n = m / hw, r = m - n * hw;
        const int yo = r / a.Wo, xo = r - yo * a.Wo;
        geo[p].pb = n * a.H * a.W;
        geo[p].yb = (m < a.M) ? (a.upsample ? yo - a.pad : yo * a.stride - a.pad) : -(1 << 28);
        geo[p].xb = a.upsample ? xo - a.pad : xo * a.stride - a.pad;
      } else {
        geo[p].pb = 0; geo[p].yb = 0; geo[p].xb = 0;
      }
    }
  // issue half-tile s (tile s/4, half s%4: A0 A1 B0 B1) into its buffer
  auto issue_half = [&](int s) {
    if (s >= nhalf) return;
    const int t = s >> 2, h = s & 3;
    const int kt = kt0 + t;
    uint4* dst = lds + (t & 1) * BUF + h * HALF + wid * 2 * 64;
    if (h < 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int p = (h & 1) * 2 + i;
        glds16(a_src<KS, TAPU, BK>(a, kt, ach[p], arow[p], geo[p]), dst + i * 64);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int p = (h & 1) * 2 + i;
        const void* src = brow[p] < a.N ? (const void*)(a.w + (long)brow[p] * a.K + kt * BK + bch[p] * 8)
                                        : (const void*)ls_zero_page;
        glds16(src, dst + i * 64);
      }
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: half-tiles 0 .. D-1 in flight, tile 0 landed
#pragma unroll
  for (int s = 0; s < D; ++s) issue_half(s);
  if (nhalf > 4) wait_vm<2>(); else wait_vm<0>();  // tile 0 (halves 0..3) landed, half 4 in flight
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // ping-pong: the two wave rows (one wave of each per SIMD) run one barrier
  // apart, so one wave's MFMA section overlaps the other's load section
  if (wr == 1) __builtin_amdgcn_s_barrier();
  bf16x8 af[2][4], b0[2][2], b1[2][2];
  const int arow_w = wr * 128;            // this wave's rows inside the A tile (= its A half)
  const int bh = wc >> 1, bcol = (wc & 1) * 64;  // B half + column offset inside it
  for (int t = 0; t < nk; ++t) {
    const uint4* buf = lds + (t & 1) * BUF;
    const uint4* Ah = buf + wr * HALF;
    const uint4* Bh = buf + (2 + bh) * HALF;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int qm = (ph == 0 || ph == 1) ? 0 : 1;
      const int qn = (ph == 0 || ph == 3) ? 0 : 1;
      // fragment reads this phase needs
      if (ph == 0 || ph == 3) {
        if (ph == 0) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              b0[ks][j] = __builtin_bit_cast(
                  bf16x8, Bh[swz_bk<BK>(bcol + j * 16 + (lane & 15), ks * 4 + (lane >> 4))]);
        }
      } else if (ph == 1) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            b1[ks][j] = __builtin_bit_cast(
                bf16x8, Bh[swz_bk<BK>(bcol + 32 + j * 16 + (lane & 15), ks * 4 + (lane >> 4))]);
      }
      if (ph == 0 || ph == 2) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            af[ks][i] = __builtin_bit_cast(
                bf16x8, Ah[swz_bk<BK>(qm * 64 + i * 16 + (lane & 15), ks * 4 + (lane >> 4))]);
      }
      (void)arow_w;
      // one half-tile of DMA, D ahead
      issue_half(4 * t + ph + D);
      if (ph == 3) {  // retire tile t+1 (issued up to 4t+8 now; t+1 ends at 4t+7)
        if (4 * t + 3 + D < nhalf) wait_vm<2>();
        else wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this phase's reads, overlapped with the barrier
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bf16x8 bv = qn == 0 ? b0[ks][j] : b1[ks][j];
            acc[qm * 4 + i][qn * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bv, acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
          }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the rows before the LDS is reused
  asm volatile("" ::: "memory");
  store_tile<BM, BN, 2, 4>(a, acc, (float*)lds, m0, n0, z);
}

// 256 x 256 tile, 8 waves (128 x 64 per wave), BK = 32 with a 4-stage LDS ring
// (4 x 32 KB): the DMA runs three K-tiles ahead of the MFMAs behind a counted
// vmcnt, one raw barrier per K-tile.  For operand streams that come from the
// Infinity Cache / HBM rather than L2 (the 2-stage BK = 64 ring can only cover
// one K-tile of latency).
template <int KS, bool TAPU>
__global__ void __launch_bounds__(512) conv_gemm_big4_kernel(ConvArgs a) {
  constexpr int BM = 256, BN = 256, BK = 32, NST = 4, WM = 2, WN = 4;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16, FH = FM / 2;
  constexpr int CPR = BK / 8;
  constexpr int AI = BM * CPR / 512, BI = BN * CPR / 512;  // 2 + 2 glds per thread per stage
  constexpr int L = AI + BI;
  constexpr int STAGE = (BM + BN) * CPR;
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  uint4* lds = lds_dyn;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nt = a.ntm * a.ntn;
  int bid = xcd_remap(blockIdx.x, nt * a.split);
  const int z = bid / nt;
  bid -= z * nt;
  int tm, tn;
  tile_of(a, bid, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kps = a.kt_per_split * 2;  // 32-wide K-tiles per split
  const int kt0 = z * kps;
  const int kt1 = min(a.ktiles * 2, kt0 + kps);

  int arow[AI], ach[AI], brow[BI], bch[BI];
  RowGeo geo[AI];
#pragma unroll
  for (int p = 0; p < AI; ++p) {
    const int q = (wid * AI + p) * 64 + lane;
    const int row = q / CPR;
    arow[p] = m0 + row;
    ach[p] = swz_bk<BK>(row, q % CPR) - row * CPR;
    if (KS == 3) {
      const int m = m0 + row;
      const int hw = a.Ho * a.Wo;
      const int n = m / hw, r = m - n * hw;
      const int yo = r / a.Wo, xo = r - yo * a.Wo;
      geo[p].pb = n * a.H * a.W;
      geo[p].yb = (m < a.M) ? (a.upsample ? yo - a.pad : yo * a.stride - a.pad) : -(1 << 28);
      geo[p].xb = a.upsample ? xo - a.pad : xo * a.stride - a.pad;
    } else {
      geo[p].pb = 0; geo[p].yb = 0; geo[p].xb = 0;
    }
  }
#pragma unroll
  for (int p = 0; p < BI; ++p) {
    const int q = (wid * BI + p) * 64 + lane;
    const int row = q / CPR;
    brow[p] = n0 + row;
    bch[p] = swz_bk<BK>(row, q % CPR) - row * CPR;
  }
  auto issue = [&](int kt, int stage) {
    uint4* base = lds + stage * STAGE;
#pragma unroll
    for (int p = 0; p < AI; ++p)
      glds16(a_src<KS, TAPU, BK>(a, kt, ach[p], arow[p], geo[p]), base + (wid * AI + p) * 64);
#pragma unroll
    for (int p = 0; p < BI; ++p) {
      const void* src = brow[p] < a.N ? (const void*)(a.w + (long)brow[p] * a.K + kt * BK + bch[p] * 8)
                                      : (const void*)ls_zero_page;
      glds16(src, base + BM * CPR + (wid * BI + p) * 64);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < NST - 1; ++t)
    if (kt0 + t < kt1) issue(kt0 + t, t);
  int stage = 0;
  for (int kt = kt0; kt < kt1; ++kt) {
    // tile kt landed for this wave: later tiles (up to 2) may stay in flight
    const int ahead = min(NST - 2, kt1 - 1 - kt);
    if (ahead >= 2) wait_vm<2 * L>();
    else if (ahead == 1) wait_vm<L>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // everyone's tile kt landed; stage of kt-1 free
    asm volatile("" ::: "memory");
    if (kt + NST - 1 < kt1) issue(kt + NST - 1, (stage + NST - 1) & (NST - 1));
    const uint4* cur = lds + stage * STAGE;
    const int c = lane >> 4;
    bf16x8 bfr[FN], a0[FH], a1[FH];
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[j] = __builtin_bit_cast(bf16x8, cur[BM * CPR + swz_bk<BK>(wn * WTN + j * 16 + (lane & 15), c)]);
#pragma unroll
    for (int i = 0; i < FH; ++i) a0[i] = __builtin_bit_cast(bf16x8, cur[swz_bk<BK>(wm * WTM + i * 16 + (lane & 15), c)]);
#pragma unroll
    for (int i = 0; i < FH; ++i)
      a1[i] = __builtin_bit_cast(bf16x8, cur[swz_bk<BK>(wm * WTM + (FH + i) * 16 + (lane & 15), c)]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FH; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], bfr[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < FH; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[FH + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], bfr[j], acc[FH + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    stage = (stage + 1) & (NST - 1);
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  store_tile<BM, BN, WM, WN>(a, acc, (float*)lds, m0, n0, z);
}

#endif  // LS_DIAG_KERNELS

// split-K reduction + epilogue: one thread per 8 output columns
__global__ void splitk_reduce_kernel(ConvArgs a) {
  const bool geglu = a.act == LS_ACT_GEGLU;
  const int nout = geglu ? a.N / 2 : a.N;
  const int cpr = (nout + 7) / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)a.M * cpr) return;
  const int row = idx / cpr, o8 = (int)(idx - (long)row * cpr) * 8;
  const long MN = (long)a.M * a.N;
  const bool vec = (a.N % 8 == 0) && (a.ldy % 8 == 0) && (!a.res || a.ldr % 8 == 0);
  if (geglu) {
    const int ph = (o8 >> 4) * 32 + (o8 & 15);
    float h[8], g[8], t[8];
    for (int j = 0; j < 8; ++j) { h[j] = 0.f; g[j] = 0.f; }
    for (int z = 0; z < a.split; ++z) {
      load8f(a.partial + z * MN + (long)row * a.N + ph, t);
      for (int j = 0; j < 8; ++j) h[j] += t[j];
      load8f(a.partial + z * MN + (long)row * a.N + ph + 16, t);
      for (int j = 0; j < 8; ++j) g[j] += t[j];
    }
    epi_geglu8(a, row, ph, h, g, vec);
  } else {
    float v[8];
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    for (int z = 0; z < a.split; ++z) {
      const float* p = a.partial + z * MN + (long)row * a.N + o8;
      if (vec) {
        float t[8];
        load8f(p, t);
        for (int j = 0; j < 8; ++j) v[j] += t[j];
      } else {
        for (int j = 0; j < 8 && o8 + j < a.N; ++j) v[j] += p[j];
      }
    }
    epi_chunk(a, row, o8, v, vec && o8 + 8 <= a.N);
  }
}

// GroupNorm column sums of a stored bf16 [M][ldy] tensor by a separate read pass
// (producers whose epilogue does not emit them: split-K, the row-block kernel, the
// small tiles).  Block = (slot, 32 column chunks of 8); thread = (chunk, row lane of
// 8); same fp32-per-slot sums as the epilogue (the order of the adds differs).
__global__ void __launch_bounds__(256) colsum_pass_kernel(const u16* __restrict__ y, long ldy, int N,
                                                          float* __restrict__ out) {
  __shared__ float red[8][32][17];
  const int lane = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const long slot = blockIdx.x;
  const int cc = blockIdx.y * 32 + lane;
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  if (cc * 8 < N) {
    const u16* src = y + slot * CS_ROWS * ldy + cc * 8;
#pragma unroll 4
    for (int r = rl; r < CS_ROWS; r += 8) {
      float f[8];
      unpack8(*(const uint4*)(src + (long)r * ldy), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s1[j] += f[j]; s2[j] = fmaf(f[j], f[j], s2[j]); }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[rl][lane][j] = s1[j]; red[rl][lane][8 + j] = s2[j]; }
  __syncthreads();
  if (rl == 0 && cc * 8 < N) {
    float t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) t[j] = red[0][lane][j];
    for (int k = 1; k < 8; ++k)
#pragma unroll
      for (int j = 0; j < 16; ++j) t[j] += red[k][lane][j];
    float* o = out + slot * 2 * N + cc * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) { o[j] = t[j]; o[N + j] = t[8 + j]; }
  }
}

static int launch_colsum_pass(const u16* y, long ldy, long M, int N, float* out, hipStream_t s) {
  if (!y || !out || M <= 0 || M % CS_ROWS || N <= 0 || N % 8 || ldy % 8)
    return fail(LS_ERR_INVALID, "gn column sums: M % 128 == 0, N % 8 == 0, ldy % 8 == 0");
  colsum_pass_kernel<<<dim3((unsigned)(M / CS_ROWS), cdiv(N / 8, 32)), 256, 0, s>>>(y, ldy, N, out);
  return check_launch("colsum_pass_kernel");
}

// ------------------------------------------------------------ row-block GEMM
// The short-K linears of the 32x32 level (K = Cin = 320: Transformer/motion
// proj_in/out, fused q|k|v, q, out-proj, GEGLU W1) are epilogue/bandwidth bound
// on the tiled kernels: every 128x160 tile pays a full prologue + LDS-staged
// epilogue for only 5 K-tiles of MFMAs, and re-reads its A rows once per N tile.
// Here one workgroup (8 waves, 2 per SIMD) owns 256 rows x a range of N:
//   * each wave keeps its 32 A rows x K in registers for the whole kernel
//     (2 x KT bf16x8 fragments = 80 VGPRs at K = 320): A is read once;
//   * W streams through LDS in 64-column chunks (all of K per chunk, 2-stage
//     ring, global_load_lds DMA into the XOR-swizzled 64-wide images);
//   * the product is computed transposed, C^T = W A^T (MFMA A operand = W rows,
//     B operand = A rows), so a lane's accumulator holds 4 consecutive output
//     columns of one row and the epilogue stores 8 B per lane straight from
//     registers -- no LDS staging, no barrier -- and runs in the same basic
//     block as the next chunk's MFMAs (double-buffered accumulators), so its
//     VALU work and stores overlap the matrix pipe.
// FLAGS: RB_LN LayerNorm fold (ln_rowstats/ln_colsum), RB_RES residual,
// RB_RV row vector (positional-encoding rows), RB_GEGLU GEGLU epilogue.  With RB_LN the
// register-resident A rows are normalised in place (the host folds gamma / beta).
// Host contract (rowblock_ok): ksize 1, no x2 / affine prologue, K = 32*KT = Cin
// (320 with FM = 2: 256 rows per block; 640 with FM = 1: 128 rows, A still 80 VGPRs),
// M % BM == 0, N % 64 == 0, no split-K, bf16 output with 4-aligned pitches.
enum { RB_LN = 1, RB_RES = 2, RB_RV = 4, RB_GEGLU = 8, RB_STATS = 16, RB_GNCS = 32, RB_AFF = 64 };

// sum over the 16 lanes of a DPP row (all 16 receive it): quad butterflies, then
// rotations by 4 and 8 within the row
__device__ __forceinline__ float row16_sum(float v) {
  auto dpp = [](float x, int ctrl) -> float {
    switch (ctrl) {  // dpp_ctrl must be a constant
      case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));
      case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));
      case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x124, 0xF, 0xF, false));
      default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));
    }
  };
  v += dpp(v, 0);
  v += dpp(v, 1);
  v += dpp(v, 2);
  v += dpp(v, 3);
  return v;
}

template <int KT, int FM, int FN, int FLAGS>
__global__ void __launch_bounds__(512) gemm_rowblock_kernel(ConvArgs a) {
  constexpr int BN = 16 * FN;
  constexpr int BM = 8 * 16 * FM;             // rows per workgroup (8 waves x FM fragments of 16)
  constexpr int KTILES = KT / 2;              // 64-wide LDS images per chunk
  constexpr int WIMG = BN * KTILES * 8;       // uint4 of the W images of a chunk
  constexpr bool LN = FLAGS & RB_LN, RES = FLAGS & RB_RES, RV = FLAGS & RB_RV, GG = FLAGS & RB_GEGLU;
  // residual tile of a chunk (BM rows x BN columns bf16) DMA'd with its W images, so it is
  // in flight two chunks ahead of its epilogue with no registers held (the register
  // residual, one chunk ahead, left the short-K residual GEMMs latency-bound on HBM)
  constexpr int RIMG = RES ? BM * BN / 8 : 0;  // uint4
  constexpr int RPT = RIMG / 512;
  constexpr int STAGE = WIMG + 48 + RIMG;     // + bias / colsum / row-vector columns (3 x 64 fp32) + residual
  constexpr bool AF = FLAGS & RB_AFF;  // GroupNorm affine (+SiLU) prologue on the register-resident A rows
  constexpr bool ST = (FLAGS & RB_STATS) && !GG;  // row statistics of the output (host: one N range per block)
  // GroupNorm column sums (a.cs_out): per chunk a wave's 16 FM rows are summed over its
  // lanes (DPP) into LDS; after the chunk's barrier the CS_ROWS / (16 FM) waves of a
  // slot are added in a fixed order and written (host: BM % CS_ROWS == 0)
  constexpr bool CS = (FLAGS & RB_GNCS) && !GG;
  constexpr int WPS = CS_ROWS / (16 * FM);  // waves per 128-row slot
  constexpr int NSTORE = GG ? FM * FN / 2 : FM * FN;
  constexpr int PPT = (WIMG + 511) / 512;     // 16-B DMA pieces per thread per chunk
  static_assert(KT % 2 == 0 && WIMG % 256 == 0, "K must be a multiple of 64");
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int rb = blockIdx.x / a.ntn, ns = blockIdx.x - rb * a.ntn;
  const int nch = a.N / BN;
  const int c0 = (int)((long)nch * ns / a.ntn), c1 = (int)((long)nch * (ns + 1) / a.ntn);
  const int mw = rb * BM + wid * 16 * FM;  // this wave's first row

  // chunk c -> LDS stage: W rows [64c, 64c + 64) x all K as KTILES swizzled 64-wide
  // images, then the chunk's 64 bias, colsum and row-vector values (wave 0).
  // piece q = p * 512 + tid of a chunk's images: image t = q / (8 BN), row (q / 8) % BN, chunk q % 8
  const long rv_base = RV ? rv_row(a, rb * BM) : 0;  // host: rows_per_vec % BM == 0
#ifdef LS_DIAG_KERNELS  // timing ablations (LS_GEMM_ABLATE): 2 no chunk DMA past the first two, 4 no
  // stores, 64 no A-row loads (zeros) -- results are garbage; profiles/r05l_ablate.txt
  const int abl = a.ablate;
#else
  constexpr int abl = 0;
#endif
  // W / residual DMA through buffer descriptors (round 6): the per-thread byte offsets are
  // fixed over the chunks, a chunk moves only the uniform soffset, and the LDS destinations
  // are LDS-space addresses -- one s_add to M0 per DMA instead of a 64-bit global address,
  // a readfirstlane and the M0 copy (the same change took the ff_chain kernel 5-8 % faster)
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  __builtin_assume(wid_u >= 0 && wid_u < 8);
  const uint32_t cap = 0x7FFFFFFFu;
  const i32x4 rs_w = buffer_rsrc(a.w, (uint32_t)min((long)a.N * a.K * 2, (long)cap));
  const i32x4 rs_r = RES ? buffer_rsrc(a.res + (long)rb * BM * a.ldr, (uint32_t)min((long)BM * a.ldr * 2, (long)cap)) : rs_w;
  int wvo[PPT], rvo[RPT > 0 ? RPT : 1];
#pragma unroll
  for (int p = 0; p < PPT; ++p) {
    const int q = p * 512 + tid, t = q / (8 * BN), row = (q >> 3) % BN, pc = q & 7;
    const int lc = pc ^ ((row >> 1) & 7);  // logical 16-B chunk stored at physical chunk pc
    wvo[p] = (row * a.K + t * 64 + lc * 8) * 2;
  }
#pragma unroll
  for (int p = 0; p < RPT; ++p) {  // residual piece q: row q / (BN / 8), 16-B column chunk q % (BN / 8)
    const int q = p * 512 + tid, row = q / (BN / 8), ch = q % (BN / 8);
    rvo[p] = (row * a.ldr + ch * 8) * 2;
  }
  lds_u4* const lbase = (lds_u4*)lds_dyn;
  auto issue = [&](int c, int stage) {
    if ((abl & 2) && c > c0 + 1) return;
    lds_u4* const dst = lbase + stage * STAGE;
#pragma unroll
    for (int p = 0; p < PPT; ++p) {
      if (WIMG % 512 == 0 || p * 512 + wid_u * 64 < WIMG)  // (wave-uniform)
        ls_raw_buffer_load_lds(rs_w, (__attribute__((address_space(3))) void*)(dst + p * 512 + wid_u * 64), 16, wvo[p],
                               c * BN * a.K * 2, 0, 0);
    }
    if (wid == 0 && lane < 48 && (lane & 15) * 4 < BN) {
      const int q = lane >> 4, e = (lane & 15) * 4;
      const float* base = q == 0 ? a.bias : q == 1 ? nullptr : (RV ? a.rowvec + rv_base : nullptr);
      const void* ps = base ? (const void*)(base + c * BN + e) : (const void*)ls_zero_page;
      glds16(ps, lds_dyn + stage * STAGE + WIMG);
    }
#pragma unroll
    for (int p = 0; p < RPT; ++p)
      ls_raw_buffer_load_lds(rs_r, (__attribute__((address_space(3))) void*)(dst + WIMG + 48 + p * 512 + wid_u * 64), 16,
                             rvo[p], c * BN * 2, 0, 0);
  };

  if (c0 >= c1) return;
  float2 mrow[FM];  // LayerNorm (mean, rstd) of this lane's two rows
  if (LN) {
#pragma unroll
    for (int i = 0; i < FM; ++i) mrow[i] = *(const float2*)(a.ln_mr + 2L * (mw + i * 16 + l16));
  }
  issue(c0, 0);
  // A rows -> registers (B operand of C^T = W A^T: lane = row l16, k = 8 lg .. + 7 of each 32-wide step)
  bf16x8 ar[FM][KT];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const u16* src = a.x1 + (long)(mw + i * 16 + l16) * a.ld1 + lg * 8;
#pragma unroll
    for (int s = 0; s < KT; ++s) ar[i][s] = (abl & 64) ? bf16x8{} : *(const bf16x8*)(src + s * 32);
  }
  if (LN) {
    // LayerNorm applied to the register-resident A rows once ((x - mean) * rstd, rounded
    // to bf16 like the reference's normalised activations); gamma / beta are folded
    // into W and the bias on the host, so the epilogue needs no per-column colsum.
    wait_vm<0>();
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const float rstd = mrow[i].y, nmr = -mrow[i].x * mrow[i].y;
#pragma unroll
      for (int s = 0; s < KT; ++s) {
        bf16x8 v = ar[i][s];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (__bf16)fmaf((float)v[e], rstd, nmr);
        ar[i][s] = v;
      }
    }
  }
  if (AF) {
    // x * scale[s][c] + shift[s][c], rounded to bf16 like ls_groupnorm_apply's materialised
    // output; the block's rows lie in one sample (host: pix_per_sample % BM == 0).  A SiLU
    // after the affine goes to the register-staged kernel (rowblock_ok): beside the 80 A
    // registers its unrolled form spills.
    const long sb = (long)((rb * BM) / a.pix_per_sample) * a.Cin + lg * 8;
    wait_vm<0>();
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      float sc[8], sh[8];
      load8f(a.aff_scale + sb + s * 32, sc);
      load8f(a.aff_shift + sb + s * 32, sh);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        bf16x8 v = ar[i][s];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (__bf16)fmaf((float)v[e], sc[e], sh[e]);
        // pin the result here: sunk past the barrier, every step's scale / shift would
        // stay live beside the A rows and spill
        asm volatile("" : "+v"(v));
        ar[i][s] = v;
      }
    }
  }
  wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  f32x4 acc0[FM][FN], acc1[FM][FN];
  // column parameters (bias + row vector) of chunk c from its LDS stage, read before
  // the next DMA is issued (an LDS read after it would wait for the DMA); the chunk's
  // accumulators start at them
  auto load_prm = [&](int stage, float4 (&bb)[FN]) {
    const float4* prm = (const float4*)(lds_dyn + stage * STAGE + WIMG);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      bb[j] = prm[lg + 4 * j];
      if (RV) {
        const float4 r4 = prm[32 + lg + 4 * j];  // (FN 2 uses the first 8 of each 16)
        bb[j].x += r4.x; bb[j].y += r4.y; bb[j].z += r4.z; bb[j].w += r4.w;
      }
    }
  };
  const bool unit_scale = a.out_scale == 1.f;
  double S1[FM], S2[FM];  // running row sums of the output (ST), per lane: its 4-column slices
#pragma unroll
  for (int i = 0; i < FM; ++i) { S1[i] = 0.0; S2[i] = 0.0; }
  auto epilogue = [&](int c, f32x4 (&acc)[FM][FN], int stage) {
    const int nb = c * BN + 4 * lg;  // packed column of fragment j: nb + 16 j
    const u16* rtile = (const u16*)(lds_dyn + stage * STAGE + WIMG + 48);  // [BM][BN] residual of chunk c
    float cs1[FM], cs2[FM];  // this chunk's partial sums (fp32 over 4*FN values), folded into S in fp64
    float gcs[FM][FN][4];    // stored values of this chunk (CS)
#pragma unroll
    for (int i = 0; i < FM; ++i) { cs1[i] = 0.f; cs2[i] = 0.f; }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      u16* yrow = (u16*)a.y + (long)(mw + i * 16 + l16) * a.ldy;
      if (GG) {
#pragma unroll
        for (int p = 0; p < FN / 2; ++p) {
          float h[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) h[r] = acc[i][2 * p][r] * gelu_erf(acc[i][2 * p + 1][r]);
          *(uint2*)(yrow + c * (BN / 2) + 16 * p + 4 * lg) = make_uint2(pack2(h[0], h[1]), pack2(h[2], h[3]));
        }
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float o[4];
          float r4[4] = {0.f, 0.f, 0.f, 0.f};
          if (RES) {
            const uint2 rs = *(const uint2*)(rtile + (wid * 16 * FM + i * 16 + l16) * BN + 4 * lg + 16 * j);
            r4[0] = __uint_as_float(rs.x << 16); r4[1] = __uint_as_float(rs.x & 0xffff0000u);
            r4[2] = __uint_as_float(rs.y << 16); r4[3] = __uint_as_float(rs.y & 0xffff0000u);
          }
          if (unit_scale) {  // (block-uniform)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = acc[i][j][r] + r4[r];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (acc[i][j][r] + r4[r]) * a.out_scale;
          }
          const uint2 pk = make_uint2(pack2(o[0], o[1]), pack2(o[2], o[3]));
          if (!(abl & 4) || pk.x == 0x12345u) *(uint2*)(yrow + nb + 16 * j) = pk;
          if (CS) {
            gcs[i][j][0] = __uint_as_float(pk.x << 16); gcs[i][j][1] = __uint_as_float(pk.x & 0xffff0000u);
            gcs[i][j][2] = __uint_as_float(pk.y << 16); gcs[i][j][3] = __uint_as_float(pk.y & 0xffff0000u);
          }
          if (ST) {  // statistics of the stored (bf16-rounded) values, like ls_row_stats reads them:
            // v_dot2c_f32_bf16 on the packed pairs (4 instructions for 4 values instead of 11)
            typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
            const bf2 one2 = {(__bf16)1.0f, (__bf16)1.0f};
            const bf2 px = __builtin_bit_cast(bf2, pk.x), py = __builtin_bit_cast(bf2, pk.y);
            cs1[i] = __builtin_amdgcn_fdot2_f32_bf16(py, one2, __builtin_amdgcn_fdot2_f32_bf16(px, one2, cs1[i], false), false);
            cs2[i] = __builtin_amdgcn_fdot2_f32_bf16(py, py, __builtin_amdgcn_fdot2_f32_bf16(px, px, cs2[i], false), false);
          }
        }
      }
    }
    if (ST) {
#pragma unroll
      for (int i = 0; i < FM; ++i) { S1[i] += (double)cs1[i]; S2[i] += (double)cs2[i]; }
    }
    if (CS) {  // column sums of this wave's rows -> LDS part[c & 1][wave][64]
      float* part = (float*)(lds_dyn + 3 * STAGE) + (c & 1) * 512 + wid * 64;
      float mine = 0.f;
#pragma unroll
      for (int v = 0; v < 16; ++v) {  // v = kind * 8 + j * 4 + r
        const int j = (v >> 2) & 1, r = v & 3;
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const float b = gcs[i][j][r];
          t += (v >> 3) ? b * b : b;
        }
        t = row16_sum(t);
        mine = (l16 == v) ? t : mine;
      }
      // lane (lg, l16): column 4 lg + 16 j + r of the chunk, value kind
      const int v = l16, col = 4 * lg + 16 * ((v >> 2) & 1) + (v & 3);
      part[col * 2 + (v >> 3)] = mine;
    }
  };
  // slots of this block's rows: add the WPS waves of each for chunk cc and write them
  auto merge_cs = [&](int cc) {
    const float* part = (const float*)(lds_dyn + 3 * STAGE) + (cc & 1) * 512;
    for (int q = tid; q < (BM / CS_ROWS) * 64; q += 512) {
      const int sl = q >> 6, e = q & 63;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WPS; ++w) t += part[(sl * WPS + w) * 64 + e];
      const long slot = (long)rb * (BM / CS_ROWS) + sl;
      a.cs_out[slot * 2 * a.N + (e & 1) * a.N + cc * BN + (e >> 1)] = t;
    }
  };
  // b0: the chunk's bias (+ row vector), read by the caller before its DMA issue; the
  // accumulators start there, so the epilogue has no bias add
  auto mfma_chunk = [&](int stage, f32x4 (&acc)[FM][FN], const float4 (&b0)[FN]) {
    const uint4* cur = lds_dyn + stage * STAGE;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){b0[j].x, b0[j].y, b0[j].z, b0[j].w};
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      bf16x8 bw[FN];
      const int ch = (s & 1) * 4 + lg;
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bw[j] = __builtin_bit_cast(bf16x8, cur[(s >> 1) * (8 * BN) + swz_bk<64>(j * 16 + l16, ch)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], ar[i][s], acc[i][j], 0, 0, 0);
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // 3-stage ring: chunk c computes from stage c%3 while chunk c-1's parameters stay in
  // (c-1)%3 for its epilogue and chunk c+1 lands in (c+1)%3.  Past the last chunk the DMA
  // re-loads the last chunk into the spare stage, so the steady-state body is branch-free.
  // The residual tile of chunk c travels with the chunk's W images (stage c % 3).
  auto body = [&](int c, f32x4 (&acc)[FM][FN], f32x4 (&prev)[FM][FN]) {
    const int st = (c - c0) % 3;
    const int sp = st == 0 ? 2 : st - 1;
    float4 bn[FN];
    load_prm(st, bn);
    issue(min(c + 1, c1 - 1), st == 2 ? 0 : st + 1);
    if (CS && c - 2 >= c0) merge_cs(c - 2);  // written two epilogues ago, past a barrier
    mfma_chunk(st, acc, bn);
    epilogue(c - 1, prev, sp);
    wait_vm<NSTORE>();                                       // the DMA (older than the stores) landed
    sync();
  };
  // first chunk: no epilogue
  {
    float4 bn[FN];
    load_prm(0, bn);
    issue(min(c0 + 1, c1 - 1), 1);
    mfma_chunk(0, acc0, bn);
  }
  wait_vm<0>();
  sync();
  int c = c0 + 1;
  for (; c + 1 < c1; c += 2) {
    body(c, acc1, acc0);
    body(c + 1, acc0, acc1);
  }
  if (c < c1) {
    body(c, acc1, acc0);
    epilogue(c, acc1, (c - c0) % 3);
  } else {
    epilogue(c1 - 1, acc0, (c1 - 1 - c0) % 3);
  }
  if (CS) {  // the last two chunks' column sums
    __syncthreads();
    for (int cc = max(c0, c1 - 2); cc < c1; ++cc) merge_cs(cc);
  }
  if (ST) {  // the 4 lane groups of a row hold disjoint column slices: combine, then lane group 0 writes
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      double s1 = S1[i], s2 = S2[i];
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
      if (lg == 0) {
        const double n = (double)a.N, mean = s1 / n;
        const double var = fmax(s2 / n - mean * mean, 0.0);
        *(float2*)(a.stats_out + 2L * (mw + i * 16 + l16)) =
            make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.stats_eps)));
      }
    }
  }
}

// ------------------------------------------------------------- halo-tile 3x3 conv
// conv3x3_halo_kernel: 3x3 / stride 1 / pad 1 convolutions with Cin % 64 == 0 whose A
// operand comes from an LDS HALO TILE.  The implicit-GEMM kernels above gather A per tap:
// a 64-channel chunk of every output pixel's 3x3 window is DMA'd 9 times (9 K-tiles), so
// at N = 128 / 160 the operand DMA -- about 60 issue cycles per 1-KB wave-instruction --
// outweighs the MFMAs it feeds (the VAE's 128-channel convs at 256^2 ran at 0.34 of the
// bf16 peak), and a GroupNorm affine + SiLU on the input had to be materialised by its
// own pass (ls_groupnorm_apply) because applying it in the gather would repeat it 9 times.
// Here a block owns a TH x TW patch of one image (256 output pixels; 128 in the 16 x 8
// form below) x BN output channels:
//   * per 64-channel chunk, the (TH + 2) x (TW + 2) input pixels of the patch are loaded
//     ONCE (buffer loads into registers; pixels outside the image read zeros), optionally
//     put through y = silu?(x * scale + shift) (the GroupNorm affine of the pixel's sample)
//     and stored to a halo image in LDS: 128 B per pixel, the 16-B chunks XOR-swizzled by
//     (pixel & 7) -- conflict-free ds_read_b128 fragment reads at ANY pixel offset, which
//     the 9 taps need (brute-forced over the lane groups; the GEMMs' ((row >> 1) & 7)
//     swizzle is 2-way there).  Halo rows are TW + 8 pixels long (== 0 mod 8), so the
//     swizzle phase of every fragment of a wave equals its first fragment's: one address
//     computation per (tap, k-step) and lane, fragment offsets are immediates (the compact
//     TW + 2 row with a column-based swizzle frees 28 KB of LDS, but the third weight slot
//     at BN 160 that room was for spills 30 VGPRs; the 16 x 8 form uses it to fit 2 blocks);
//   * the 9 taps of the chunk then run from that image: tap (kh, kw) shifts the read by
//     kh P + kw pixels (P the row pitch); the weight K-tile of each tap ([BN][64], channel-chunk-major
//     packing) streams through an NSW-slot LDS ring by LDS-DMA, NSW - 1 taps ahead;
//   * the halo of chunk c + 1 is loaded into registers at tap 0 of chunk c and written to
//     the other halo image at tap 8 (so the input affine's VALU work overlaps the MFMAs
//     of 8 taps); every wait is one constant vmcnt (padded dummy DMAs).
// 8 waves as 4 (pixels) x 2 (channels), 64 x BN/2 per wave; the epilogue is
// store_tile_plain (bias, per-frame row vector, residual, scale, GroupNorm column sums
// of the output) with the patch's rows mapped back to image rows.
// TH = 256 / TW: 16 x 16 patches, 8 waves, one block per CU (the shipped UNet form).
// TH = 8 (round 5, BN 128: the VAE's convs): 16 x 8 patches, 4 waves as 2 (pixels) x 2
// (channels), compact halo rows (TW + 2 pixels, chunks swizzled by the halo COLUMN & 7 --
// conflict-free at any row / column offset, brute-forced -- so fragments one patch row
// apart still share the swizzle phase) and a 2-slot weight ring: 80 KB of LDS, TWO blocks
// per CU, so one block's halo prologue, chunk transitions and epilogue overlap the other's
// MFMAs (the 1-block form waited 44.5 % of its wave time, profiles/r05a_h128_summary.txt).
template <int TW, int BN, int TH_ = 256 / TW>
struct HaloCfg {
  static constexpr int TH = TH_;
  // channel waves: 2 (BN / 2 columns each); 1 for the narrow tile (BN 16: the VAE decoder's
  // conv_out, 3 used output channels, where the conv is bound by the halo transform and HBM)
  static constexpr int WNW = BN >= 64 ? 2 : 1;
  static constexpr int NT = (TH / 4) * WNW * 64;         // threads: (TH / 4) pixel waves x WNW channel waves
  static constexpr bool COMPACT = TH < 16;
  static constexpr int P = COMPACT ? TW + 2 : TW + 8;    // halo row pitch (pixels); padded: 0 mod 8
  static constexpr int HALO = (TH + 2) * P * 8;          // uint4 per halo image
  static constexpr int WSLOT = BN * 8;                   // uint4 per weight ring slot (BN x 64 k)
  // weight ring slots (3 at BN 160 spills 30 VGPRs; the 2-block form has LDS for 2)
  static constexpr int NSW = COMPACT ? 2 : BN <= 128 ? 3 : 2;
  static constexpr int DPT = (WSLOT + NT - 1) / NT;      // weight DMAs per thread per tap
  static constexpr int FN = BN / WNW / 16;               // 16-column fragments per wave
  static constexpr size_t SHM = ((size_t)2 * HALO + (size_t)NSW * WSLOT + 64 + 64) * 16;  // + dummy, affine
  static_assert(SHM <= (COMPACT ? 81920 : 163840), "halo conv LDS (compact: two blocks per CU)");
  static_assert((size_t)64 * (BN + 4) * 4 <= (size_t)2 * HALO * 16, "epilogue staging fits the halo images");
  static_assert(TW == 16 && (TH == 16 || TH == 8), "16-pixel patch rows, 16 or 8 of them");
  static_assert(BN % (16 * WNW) == 0, "whole 16-column fragments per wave");
  static constexpr int MINB = BN >= 64 ? 16 / TH : 2;    // launch bounds: blocks per CU
};


// halo loads of a chunk in 3 batches (pieces [hb_lo(b), hb_lo(b + 1))): loaded at taps 0 /
// 3 / 6 of the previous chunk and stored at taps 3 / 6 / 8, so at most 3 pieces (12 VGPRs)
// are in flight per thread
__host__ __device__ constexpr int hb_lo(int b, int nhl) { return b == 0 ? 0 : b == 1 ? (nhl + 2) / 3 : b == 2 ? (2 * nhl + 2) / 3 : nhl; }
// VMEM instructions a thread issues after the weight DMA at tap t (0..8) of a chunk:
// the halo batch loaded there (+ its 4 affine loads) when a next chunk exists
// the halo batch loaded there (+ at tap 0 the chunk's affine parameters, one float4 per thread)
__host__ __device__ constexpr int halo_issue(int t, int nhl, bool gn) {
  return t == 0 ? hb_lo(1, nhl) + (gn ? 1 : 0) : t == 3 ? hb_lo(2, nhl) - hb_lo(1, nhl) : t == 6 ? nhl - hb_lo(2, nhl) : 0;
}

// Halo pieces: the (TH + 2) x (TW + 2) pixels the taps read x 8 16-B chunks (2592 pieces at
// 16 x 16: 5.06 per thread); piece j of a thread has its own LDS slot hdst[j].
template <int TW, int BN, bool GN, bool CSF, int TH_ = 256 / TW>
__global__ void __launch_bounds__((HaloCfg<TW, BN, TH_>::NT), (HaloCfg<TW, BN, TH_>::MINB)) conv3x3_halo_kernel(ConvArgs a) {
  using HC = HaloCfg<TW, BN, TH_>;
  constexpr int TH = HC::TH, P = HC::P, HALO = HC::HALO, WSLOT = HC::WSLOT, NSW = HC::NSW, NT = HC::NT;
  constexpr int WNW = HC::WNW;
  constexpr bool COMPACT = HC::COMPACT;
  constexpr int NPC = (TH + 2) * (TW + 2) * 8;  // pieces per chunk (the read pixels)
  constexpr int NHL = (NPC + NT - 1) / NT, DPT = HC::DPT, FM = 4, FN = HC::FN, WTN = BN / WNW;
  constexpr int HB = (NHL + 2) / 3;  // largest batch
  extern __shared__ __attribute__((aligned(16))) uint4 lds_dyn[];
  uint4* const hbuf = lds_dyn;                 // [2][HALO]
  uint4* const wbuf = lds_dyn + 2 * HALO;      // [NSW][WSLOT]
  uint4* const dummy = wbuf + NSW * WSLOT;     // 1 KB: padding DMAs land here
  float4* const gpar = (float4*)(dummy + 64);  // [2 chunk parities][scale 16 | shift 16] float4

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WNW, wn = wid % WNW;
  const int l16 = lane & 15, lg = lane >> 4;
  const int ntn = (a.N + BN - 1) / BN, tpr = a.W / TW, tpc = a.H / TH;
  // (measured, not kept: a persistent grid issuing the next tile's weights and halo loads
  // before this tile's epilogue -- 30-90 VGPRs of spills in every instance)
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % ntn;
  bid /= ntn;
  const int txb = bid % tpr;
  bid /= tpr;
  const int tyb = bid % tpc;
  const int img = bid / tpc;
  const int y0 = tyb * TH, x0 = txb * TW, n0 = tn * BN;
  const long HW = (long)a.H * a.W;  // the OUTPUT image (for an upsample conv the launch passes the output dims)
  // nearest x2 upsample (round 6): halo pixel (y, x) of the output image reads input pixel
  // (y >> 1, x >> 1) -- the LDS halo image, the taps and the epilogue are those of a plain conv
  const int ups = a.upsample;
  const int Wi = a.W >> ups;
  const long HWi = HW >> (2 * ups);
  const int nchunk = a.Cin / 64;
  const int G = 9 * nchunk;  // taps in all

  // ---- this thread's halo pieces: q = j*NT + tid -> read pixel q / 8 (row-major over the
  // (TH + 2) x (TW + 2) pixels the taps read), logical 16-B chunk tid & 7; its slot in the
  // padded image: row hr, column hcol + 3, the chunk swizzled by (slot & 7); compact: row
  // hr, column hcol, swizzled by (hcol & 7)
  const int hc8 = tid & 7;
  int hpix[NHL];  // pixel index within the image, or -1 (outside: zeros)
  int hdst[NHL];
#pragma unroll
  for (int j = 0; j < NHL; ++j) {
    const int q = j * NT + tid, hp = q >> 3;
    const int hr = hp / (TW + 2), hcol = hp - hr * (TW + 2);
    if constexpr (COMPACT) {  // row hr, column hcol, the chunk swizzled by the column
      hdst[j] = (hr * P + hcol) * 8 + (hc8 ^ (hcol & 7));
    } else {
      const int slot = hr * P + hcol + 3;
      hdst[j] = slot * 8 + (hc8 ^ (slot & 7));
    }
  }
  const uint32_t cap = 0x7FFFFFFFu;
#pragma unroll
  for (int j = 0; j < NHL; ++j) {
    const int q = j * NT + tid, hp = q >> 3;
    const int hr = hp / (TW + 2), hcol = hp - hr * (TW + 2);
    const int y = y0 - 1 + hr, x = x0 - 1 + hcol;
    hpix[j] = q < NPC && y >= 0 && y < a.H && x >= 0 && x < a.W ? (y >> ups) * Wi + (x >> ups) : -1;
  }
  const i32x4 rs1 = buffer_rsrc(a.x1 + img * HWi * a.ld1, (uint32_t)min((long)HWi * a.ld1 * 2, (long)cap));
  const i32x4 rs2 = a.C2 ? buffer_rsrc(a.x2 + img * HWi * a.ld2, (uint32_t)min((long)HWi * a.ld2 * 2, (long)cap)) : rs1;
  const long aff0 = (long)img * HW / a.pix_per_sample * a.Cin;
  // weight descriptor from column n0 (rows n0 + BN > N -- the narrow tile over N = 8 -- lie
  // past it and read zeros)
  const i32x4 rs_w = buffer_rsrc(a.w + (long)n0 * a.K, (uint32_t)min((long)min(BN, a.N - n0) * a.K * 2, (long)cap));
  uint4 hreg[HB];
  float4 gp;
  // the affine parameters of chunk ci (64 scales, 64 shifts): every thread loads one float4
  // (the same count per wave), threads 0..31 keep theirs in LDS for store_halo
  auto load_par = [&](int ci) {
    const int k = tid & 31;
    gp = *(const float4*)((k < 16 ? a.aff_scale : a.aff_shift) + aff0 + ci * 64 + (k & 15) * 4);
  };
  auto store_par = [&](int ci) {  // scale and shift times log2(e): store_halo applies silu_log2
    constexpr float L2E = 1.4426950408889634f;
    if (tid < 32) gpar[(ci & 1) * 32 + tid] = make_float4(gp.x * L2E, gp.y * L2E, gp.z * L2E, gp.w * L2E);
  };
  auto load_halo = [&](int ci, int b) {
    const bool two = ci * 64 >= a.C1;
    const int ld = two ? a.ld2 : a.ld1;
    const int soff = (two ? ci * 64 - a.C1 : ci * 64) * 2;
    const int j0 = hb_lo(b, NHL), j1 = hb_lo(b + 1, NHL);
#pragma unroll
    for (int j = j0; j < j1; ++j) {
      const int vo = hpix[j] >= 0 ? hpix[j] * ld * 2 + hc8 * 16 : (int)0x80000000;
      hreg[j - j0] = __builtin_bit_cast(uint4, ls_raw_buffer_load_v4(two ? rs2 : rs1, vo, soff, 0));
    }
    if constexpr (GN) {
      if (b == 0 && ci > 0) load_par(ci);
    }
  };
  // pieces [j0, j1) of a chunk's halo image buf from v[j - j0] (+ the affine + SiLU)
  auto put_halo = [&](int buf, int j0, int j1, const uint4* v_in) __attribute__((always_inline)) {
    uint4* const hb0 = hbuf + buf * HALO;
    float4 gsc[2], gsh[2];
    if constexpr (GN) {  // this thread's 8 channels (chunk parity buf)
      const float4* gq = gpar + buf * 32 + hc8 * 2;
      gsc[0] = gq[0]; gsc[1] = gq[1]; gsh[0] = gq[16]; gsh[1] = gq[17];
    }
#pragma unroll
    for (int j = j0; j < j1; ++j) {
      if (j * NT + tid >= NPC) continue;
      uint4 v = v_in[j - j0];
      if constexpr (GN) {
        if (hpix[j] >= 0) {  // zero padding stays zero: the conv pads the ACTIVATED input
          float f[8];
          unpack8(v, f);
          const float scl[8] = {gsc[0].x, gsc[0].y, gsc[0].z, gsc[0].w, gsc[1].x, gsc[1].y, gsc[1].z, gsc[1].w};
          const float shf[8] = {gsh[0].x, gsh[0].y, gsh[0].z, gsh[0].w, gsh[1].x, gsh[1].y, gsh[1].z, gsh[1].w};
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = silu_log2(fmaf(f[e], scl[e], shf[e]));  // (host: GN implies SiLU)
          v = pack8(f);
        }
      }
      hb0[hdst[j]] = v;
    }
  };
  auto store_halo = [&](int buf, int b) { put_halo(buf, hb_lo(b, NHL), hb_lo(b + 1, NHL), hreg); };

  // ---- weight DMA: tap g = 9 ci + t is K-tile g of the channel-chunk-major packing
  // (buffer-descriptor DMA from column n0: per thread one byte offset, per tap the uniform
  // soffset g * 128 -- no 64-bit address arithmetic in the tap loop)
  int wvo[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const int q = j * NT + tid, row = q >> 3, pc = q & 7;
    const int lc = pc ^ ((row >> 1) & 7);
    wvo[j] = ((q < WSLOT ? row : 0) * a.K + lc * 8) * 2;
  }
  // ring slot of tap g: with 3 slots, (9 ci + t) % 3 == t % 3 is known per tap at compile time
  // (2 slots: (9 ci + t) % 2 == (ci + t) % 2, so with the chunk parity par = ci & 1 computed
  // once per chunk the slot of every tap is one of two per-chunk values -- no per-tap g % 2)
  auto wslot = [&](int par, int t) { return NSW == 3 ? t % 3 : (t & 1) ^ par; };
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  __builtin_assume(wid_u >= 0 && wid_u < NT / 64);
  // (LDS destinations as 32-bit LDS-space addresses: a generic-pointer select cast to LDS
  // costs a null check per DMA, and with WSLOT % NT == 0 no DMA is a padding one)
  lds_u4* const wbuf_l = (lds_u4*)lds_dyn + 2 * HALO;
  lds_u4* const dummy_l = wbuf_l + NSW * WSLOT;
  auto issue_w = [&](int g, int sl) {
    lds_u4* slot = wbuf_l + sl * WSLOT + wid_u * 64;
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      const bool live = WSLOT % NT == 0 || j * NT + wid_u * 64 < WSLOT;  // wave-uniform
      ls_raw_buffer_load_lds(rs_w, (__attribute__((address_space(3))) void*)(live ? slot + j * NT : dummy_l), 16, wvo[j],
                             g * 128, 0, 0);
    }
  };

  // ---- A fragment addressing: output pixel p = 64 wm + 16 i + l16 of the patch (TW 16:
  // fragment i is patch row 4 wm + i, column l16)
  static_assert(TW == 16, "fragment i = one patch row");
  const int p0 = 64 * wm + l16;
  const int hp0 = (p0 / TW) * P + (p0 % TW) + (COMPACT ? 0 : 3);  // halo pixel of fragment 0 at tap (0, 0)

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: weights of taps 0 .. NSW - 2, the chunk-0 affine row, and every chunk-0 halo
  // piece into registers at once (one HBM round trip, not one per batch), then the image
  // (chunk 0 reads source 1: host C1 % 64 == 0, C1 > 0)
  for (int g = 0; g < NSW - 1 && g < G; ++g) issue_w(g, g % NSW);
  {
    uint4 hpre[NHL];
    if constexpr (GN) load_par(0);
#pragma unroll
    for (int j = 0; j < NHL; ++j) {
      const int vo = hpix[j] >= 0 ? hpix[j] * a.ld1 * 2 + hc8 * 16 : (int)0x80000000;
      hpre[j] = __builtin_bit_cast(uint4, ls_raw_buffer_load_v4(rs1, vo, 0, 0));
    }
    if constexpr (GN) {
      store_par(0);
      __syncthreads();
    }
    put_halo(0, 0, NHL, hpre);  // (the compiler waits for the loads)
  }

  bf16x8 apf[2][FM];  // A fragments of the current tap (both k-steps)
  auto read_a = [&](const uint4* hb, int tt) {  // (tt compile-time after inlining)
    const int hpt = hp0 + (tt / 3) * P + tt % 3;
    // the swizzle phase, shared by the wave's fragments: padded rows (P == 0 mod 8) the
    // pixel's, compact rows the halo column's (l16 + kw)
    const int sw = COMPACT ? (l16 + tt % 3) & 7 : hpt & 7;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int base = hpt * 8 + ((ks * 4 + lg) ^ sw);
#pragma unroll
      for (int i = 0; i < FM; ++i)  // fragment i: + ((16 i) / TW) rows, + (16 i) % TW pixels
        apf[ks][i] = __builtin_bit_cast(bf16x8, hb[base + 8 * (((16 * i) / TW) * P + (16 * i) % TW)]);
    }
  };
  auto tap = [&](int ci, int par, auto t_tag, auto last_tag) {
    constexpr int t = decltype(t_tag)::value;
    constexpr bool LAST = decltype(last_tag)::value;  // no next chunk
    const int g = 9 * ci + t;
    // the weight DMA of tap g landed: VMEM instructions younger than it are the weights
    // of the NSW - 2 later taps and the halo batches issued at taps t - NSW + 1 .. t - 1
    constexpr int HY = LAST ? 0 : (t - 1 >= 0 ? halo_issue(t - 1, NHL, GN) : 0) +
                                  (NSW >= 3 && t - 2 >= 0 ? halo_issue(t - 2, NHL, GN) : 0);
    if (g + NSW - 2 >= G) wait_vm<0>();  // the ring's tail
    else wait_vm<(NSW - 2) * DPT + HY>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (g + NSW - 1 < G) issue_w(g + NSW - 1, wslot(par, t + NSW - 1));
    if constexpr (!LAST) {
      if constexpr (GN && t == 1) store_par(ci + 1);  // read at taps 3 / 6 / 8, past a barrier
      if constexpr (t == 3 || t == 6) store_halo(par ^ 1, t / 3 - 1);
      if constexpr (t == 0 || t == 3 || t == 6) load_halo(ci + 1, t / 3);
    }
    const uint4* hb = hbuf + par * HALO;
    const uint4* wb = wbuf + wslot(par, t) * WSLOT;
    // A fragments of tap t: at t = 0 read here; for t > 0 read at the end of tap t - 1 (the
    // halo image is stable within a chunk), so after this tap's barrier only the weight
    // fragments stand between the wave and its MFMAs, and the LDS array serves 10 reads per
    // wave there instead of 18
    if constexpr (t == 0) read_a(hb, 0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = __builtin_bit_cast(bf16x8, wb[swz_bk<64>(wn * WTN + j * 16 + l16, ks * 4 + lg)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(apf[ks][i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (t < 8) read_a(hb, t + 1);
    if constexpr (!LAST && t == 8) store_halo(par ^ 1, 2);
  };
  using I0 = std::integral_constant<int, 0>; using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>; using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>; using I5 = std::integral_constant<int, 5>;
  using I6 = std::integral_constant<int, 6>; using I7 = std::integral_constant<int, 7>;
  using I8 = std::integral_constant<int, 8>;
  auto chunk = [&](int ci, auto last) {
    const int par = ci & 1;
    tap(ci, par, I0{}, last); tap(ci, par, I1{}, last); tap(ci, par, I2{}, last);
    tap(ci, par, I3{}, last); tap(ci, par, I4{}, last); tap(ci, par, I5{}, last);
    tap(ci, par, I6{}, last); tap(ci, par, I7{}, last); tap(ci, par, I8{}, last);
  };
  for (int ci = 0; ci + 1 < nchunk; ++ci) chunk(ci, std::false_type{});
  chunk(nchunk - 1, std::true_type{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // epilogue: virtual rows (GroupNorm slots) = the patch's index within its image x 256
  const int m0v = (int)(img * HW) + (tyb * tpr + txb) * (TH * TW);
  const long m0r = img * HW + (long)y0 * a.W + x0;
  // column sums from per-thread register partials (CSG = 2: store_tile_plain_pre's slot-end form)
  static_assert((size_t)(NT / (BN / 8)) * BN * 2 * 4 <= (size_t)2 * HALO * 16, "column-sum partials fit the halo images");
  store_tile_plain<TH * TW, BN, TH / 4, WNW, false, CSF, TW, 2>(a, acc, (float*)lds_dyn, m0v, n0, m0r);
}

// ---------------------------------------------------------------- host side
static bool g_force_regstage = ls_env("LS_GEMM_REGSTAGE") != nullptr;
// A/B switch: 3x3 weights packed tap-major (packing.py reads the same variable)
static const int g_gemm_gm = ls_env("LS_GEMM_GM") ? atoi(ls_env("LS_GEMM_GM")) : 0;  // A/B switch: tile raster
static const bool g_gm_shortk = ls_env("LS_GEMM_GM_SHORTK") == nullptr || atoi(ls_env("LS_GEMM_GM_SHORTK")) != 0;
static int g_force_tile = 0, g_force_split = 0, g_bk = 64;
// ablation bits (diagnostics; tuning key 4 or LS_GEMM_ABLATE): 1 no MFMA, 2 no operand DMA,
// 4 no output store, 8 the general epilogue arithmetic even where the short path applies
static int g_ablate = ls_env("LS_GEMM_ABLATE") ? atoi(ls_env("LS_GEMM_ABLATE")) : 0;

struct TileCfg { int bm, bn, split; };
// A/B switch (LS_GEMM_BIG1280=0): the N = 1280 linears back on 128 x 160 tiles
static bool g_big1280 = ls_env("LS_GEMM_BIG1280") == nullptr || atoi(ls_env("LS_GEMM_BIG1280")) != 0;

// Tile + split-K choice by a small cost model.  A CU runs up to R blocks of a tile
// at once (LDS-limited: 2 for the 4-wave 128-row tiles, 1 for the 8-wave 256x256);
// the grid takes ceil(blocks / CUs) block-durations per CU, and a 4-wave tile alone
// on a CU runs at ~0.75 of its throughput with a second block beside it (measured,
// scripts/splitk_sweep.py: 128x160 at 256 blocks 685 TF/s, at 512 blocks 838).
// eff = relative MFMA throughput of the tile; split-K adds its fp32 slab write + read
// (~1.5 MAC-units per slab element, calibrated on the 4x4-level convs and FF2).
static TileCfg pick_tile(long M, int N, int ktiles, bool allow_split, bool big_ok, int ksize) {
  struct Cand { int bm, bn; double eff; int waves, resident; };
  const Cand cands[] = {{128, 128, 1.0, 4, 2}, {128, 160, 1.2, 4, 2}, {128, 64, 0.72, 4, 2}, {64, 64, 0.42, 4, 4},
                        {128, 32, 0.36, 4, 4}, {256, 256, 1.5, 8, 1}};
  TileCfg best{128, 128, 1};
  double best_t = 1e300;
  for (const Cand& c : cands) {
    if (c.bn == 32 && N > 32) continue;
    if (N <= 32 && c.bn != 32) continue;
    if (c.bm == 256) {
      if (!big_ok || N < 256) continue;
      // linears: 256x256 only on wide N (GEGLU W1, fused q|k|v, and N = 1280: the 8x8 / 4x4
      // levels' projections, FF2 and shortcuts, 7-16 % faster than 128x160 on every one of
      // them, profiles/r05c_n1280.txt) or when 160 does not divide N (the VAE's 512); 3x3
      // convs: the cost model decides
      if (ksize == 1 && ((N % 256 != 0 && N < 1920) || (N < 1280 && N % 160 == 0) ||
                         (N == 1280 && !g_big1280)))
        continue;
    }
    if (c.bn == 160 && N % 160 != 0) continue;  // the UNet's widths are all multiples of 160
    const long tiles = (long)cdiv(M, c.bm) * cdiv(N, c.bn);
    for (int split = 1; split <= 16; ++split) {
      // split-K only to fill the chip (grids of fewer tiles than CUs)
      if (split > 1 && (!allow_split || ktiles / split < 4 || tiles >= 256)) break;
      const long blocks = tiles * split;
      const long per_cu = (blocks + 255) / 256;
      const long conc = std::min<long>(c.resident, per_cu);
      const double f = (c.waves * conc >= 8) ? 1.0 : 0.75;
      const double per_block = (double)c.bm * c.bn * 64.0 * cdiv(ktiles, split) / c.eff;
      double t = per_cu * per_block / f;
      if (split > 1) t += (double)M * N * split * 1.5;
      if (t < best_t * 0.97) { best_t = t; best = {c.bm, c.bn, split}; }
    }
  }
  return best;
}

// ---- row-block GEMM dispatch (gemm_rowblock_kernel)
static bool g_rowblock = ls_env("LS_GEMM_NO_ROWBLOCK") == nullptr;
static bool g_rowblock640 = ls_env("LS_GEMM_NO_ROWBLOCK640") == nullptr;
static bool g_rb640_res = ls_env("LS_GEMM_RB640_RES") != nullptr;  // A/B switch: K = 640 residual GEMMs too

static bool rowblock_ok(const ls_conv_desc* d, const ConvArgs& a) {
  if (!g_rowblock || g_force_tile || g_force_regstage || d->ksize != 1 || a.C2) return false;
  // GroupNorm affine prologue: one sample per block, and not together with the LayerNorm fold
  if (a.aff_scale && (a.ln_mr || a.silu_in || a.pix_per_sample % (a.Cin == 320 ? 256 : 128) ||
                      ((uintptr_t)a.aff_scale | (uintptr_t)a.aff_shift) & 15))
    return false;
  // K = 640 only without a residual (the tiled kernel is faster there: 48 vs 53 us at 16x16)
  if (!((a.Cin == 320 && a.K == 320 && a.M % 256 == 0) ||
        (g_rowblock640 && a.Cin == 640 && a.K == 640 && a.M % 128 == 0 && (!a.res || g_rb640_res))))
    return false;
  if (a.N % 64 || a.split != 1 || a.y_f32) return false;
  if (a.act != LS_ACT_NONE && a.act != LS_ACT_GEGLU) return false;
  if (a.ldy % 4 || (a.res && a.ldr % 8) || (a.rowvec && (a.rowvec_ld % 4 || a.rows_per_vec % 256))) return false;
  if (((uintptr_t)a.y & 7) || ((uintptr_t)a.res & 15)) return false;  // 8-B output pieces, 16-B residual DMA
  return (((uintptr_t)a.x1 | (uintptr_t)a.bias | (uintptr_t)a.ln_cs | (uintptr_t)a.rowvec) & 15) == 0;
}

// FN = 2 (32-column chunks): the FN = 4 variant needs > 256 VGPRs and spills, and a
// spill's scratch traffic would break the kernel's counted vmcnt waits.
template <int KT, int FM, int FLAGS>
static void launch_rowblock2(const ConvArgs& a, int grid, hipStream_t s) {
  constexpr int FN = 2;
  constexpr int BM = 8 * 16 * FM;
  const size_t shm = (size_t)3 * (16 * FN * (KT / 2) * 8 + 48 + ((FLAGS & RB_RES) ? BM * 16 * FN / 8 : 0)) * 16 +
                     ((FLAGS & RB_GNCS) ? 4096 : 0);
  LS_SET_MAX_DYN_SHM((gemm_rowblock_kernel<KT, FM, FN, FLAGS>), (int)shm);
  gemm_rowblock_kernel<KT, FM, FN, FLAGS><<<grid, 512, shm, s>>>(a);
}

// K = 640 with two 16-row fragments per wave (256-row blocks, half the W-fragment LDS reads
// per MFMA, 160 A registers): default since r04x (step 215.3 -> 212.2 ms at 48 windows, three
// same-box alternations); tuning key 15 / LS_RB640_FM2=0: one fragment per wave
static bool g_rb640_fm2 = ls_env("LS_RB640_FM2") == nullptr || atoi(ls_env("LS_RB640_FM2")) != 0;

static bool rb640_fm2(int flags);

template <int FLAGS>
static void launch_rowblock1(const ConvArgs& a, int grid, hipStream_t s) {
  if (a.K == 320) {
    launch_rowblock2<10, 2, FLAGS>(a, grid, s);
    return;
  }
  if constexpr (!(FLAGS & (RB_STATS | RB_GNCS | RB_AFF))) {  // (the statistics epilogues spill at FM 2)
    if (rb640_fm2(FLAGS)) {
      launch_rowblock2<20, 2, FLAGS>(a, grid, s);
      return;
    }
  }
  launch_rowblock2<20, 1, FLAGS>(a, grid, s);
}

// returns false when no instance matches (the caller then uses the tiled kernels)
// compiled row-block instances (FLAGS combinations)
static const int kRowblockInstances[] = {0, RB_LN, RB_LN | RB_RV, RB_RES, RB_LN | RB_RES, RB_LN | RB_GEGLU, RB_GEGLU,
                                         RB_STATS, RB_RES | RB_STATS, RB_RES | RB_GNCS, RB_AFF, RB_AFF | RB_STATS};

// the row-block instance flags for this call, or -1; the row-block grid goes to
// *ntm / *ntn only (the caller's tiled grid in a.ntm / a.ntn stays valid for a fallback)
// (not with the GroupNorm affine: a block looks its sample up once, and rowblock_ok only
// guarantees pix_per_sample % 128 == 0 at K = 640)
static bool rb640_fm2(int flags) { return g_rb640_fm2 && !(flags & (RB_STATS | RB_GNCS | RB_AFF)); }

static int rowblock_flags(const ConvArgs& a, int* ntm_out, int* ntn_out) {
  const int flags = (a.ln_mr ? RB_LN : 0) | (a.res ? RB_RES : 0) | (a.rowvec ? RB_RV : 0) |
                    (a.act == LS_ACT_GEGLU ? RB_GEGLU : 0) | (a.stats_out ? RB_STATS : 0) | (a.cs_out ? RB_GNCS : 0) |
                    (a.aff_scale ? RB_AFF : 0);
  const int bm = a.K == 320 || rb640_fm2(flags) ? 256 : 128;
  if (a.M % bm) return -1;
  const int ntm = a.M / bm, nch = a.N / 32;
  const int ntn = std::max(1, std::min(nch, (256 + ntm - 1) / ntm));
  if (a.stats_out && ntn != 1) return -1;  // fused statistics need whole rows per block
  if (a.cs_out && (bm % CS_ROWS || ntn != 1)) return -1;
  for (int f : kRowblockInstances)
    if (f == flags) {
      *ntm_out = ntm;
      *ntn_out = ntn;
      return flags;
    }
  return -1;
}

// returns false when no instance matches (the caller then uses the tiled kernels with
// its own, untouched a.ntm / a.ntn)
static bool launch_rowblock(const ConvArgs& a0, hipStream_t s) {
  int ntm = 0, ntn = 0;
  const int flags = rowblock_flags(a0, &ntm, &ntn);
  if (flags < 0) return false;
  ConvArgs a = a0;
  a.ntm = ntm;
  a.ntn = ntn;
  const int grid = ntm * ntn;
  switch (flags) {
    case 0: launch_rowblock1<0>(a, grid, s); return true;
    case RB_LN: launch_rowblock1<RB_LN>(a, grid, s); return true;
    case RB_LN | RB_RV: launch_rowblock1<RB_LN | RB_RV>(a, grid, s); return true;
    case RB_RES: launch_rowblock1<RB_RES>(a, grid, s); return true;
    case RB_LN | RB_RES: launch_rowblock1<RB_LN | RB_RES>(a, grid, s); return true;
    case RB_LN | RB_GEGLU: launch_rowblock1<RB_LN | RB_GEGLU>(a, grid, s); return true;
    case RB_GEGLU: launch_rowblock1<RB_GEGLU>(a, grid, s); return true;
    case RB_STATS: launch_rowblock1<RB_STATS>(a, grid, s); return true;
    case RB_RES | RB_STATS: launch_rowblock1<RB_RES | RB_STATS>(a, grid, s); return true;
    case RB_RES | RB_GNCS: launch_rowblock1<RB_RES | RB_GNCS>(a, grid, s); return true;
    case RB_AFF: launch_rowblock1<RB_AFF>(a, grid, s); return true;
    case RB_AFF | RB_STATS: launch_rowblock1<RB_AFF | RB_STATS>(a, grid, s); return true;
    default: return false;
  }
}

// epilogue variant of a launch (see store_tile)
static int epi_kind(const ConvArgs& a) {
  const bool vec = (a.N % 8 == 0) && (a.ldy % 8 == 0) && (!a.res || a.ldr % 8 == 0);
  if (a.split != 1 || !vec || a.y_f32) return EPI_ANY;
  if (a.act == LS_ACT_NONE) return EPI_PLAIN;
  if (a.act == LS_ACT_GEGLU) return EPI_GEGLU;
  return EPI_ANY;
}

template <int BM, int BN, int WM, int WN, int KS, bool TAPU, int NST, int BK, int EPI, bool BUF = false>
static void launch_dma1(const ConvArgs& a, int grid, hipStream_t s) {
  // staging for the epilogue must fit too
  const size_t shm = std::max<size_t>((size_t)NST * (BM + BN) * (BK / 8) * 16, (size_t)(BM / WM) * (BN + 4) * 4);
  LS_SET_MAX_DYN_SHM((conv_gemm_dma_kernel<BM, BN, WM, WN, KS, TAPU, NST, BK, EPI, BUF>), (int)shm);
  conv_gemm_dma_kernel<BM, BN, WM, WN, KS, TAPU, NST, BK, EPI, BUF><<<grid, WM * WN * 64, shm, s>>>(a);
}

static bool g_no_buf_dma = ls_env("LS_GEMM_GLDS") != nullptr;  // A/B switch: global_load_lds addressing
#ifdef LS_DIAG_KERNELS  // measured and rejected: diagnostics build only
static int g_rs = ls_env("LS_GEMM_RS") ? atoi(ls_env("LS_GEMM_RS")) : 0;  // A/B switch: register-staged buffer loads

template <int BM, int BN, int WM, int WN, int KS, int EPI>
static void launch_rs(const ConvArgs& a, int grid, hipStream_t s) {
  const size_t shm = std::max<size_t>((size_t)2 * (BM + BN) * 8 * 16, (size_t)(BM / WM) * (BN + 4) * 4);
  LS_SET_MAX_DYN_SHM((conv_gemm_rs_kernel<BM, BN, WM, WN, KS, EPI>), (int)shm);
  conv_gemm_rs_kernel<BM, BN, WM, WN, KS, EPI><<<grid, WM * WN * 64, shm, s>>>(a);
}
static bool g_areg = ls_env("LS_GEMM_AREG") ? atoi(ls_env("LS_GEMM_AREG")) != 0 : false;  // A/B switch: 1x1 A in registers

template <int BM, int BN, int WM, int WN, int EPI>
static void launch_areg(const ConvArgs& a, int grid, hipStream_t s) {
  const size_t shm = std::max<size_t>((size_t)3 * BN * 8 * 16, (size_t)(BM / WM) * (BN + 4) * 4);
  LS_SET_MAX_DYN_SHM((conv_gemm_areg_kernel<BM, BN, WM, WN, EPI>), (int)shm);
  conv_gemm_areg_kernel<BM, BN, WM, WN, EPI><<<grid, WM * WN * 64, shm, s>>>(a);
}
#endif  // LS_DIAG_KERNELS

static bool g_no_buf_ups = ls_env("LS_GEMM_UPS_GLDS") != nullptr;  // A/B switch: ... for upsampling convs only

// operand DMA through buffer descriptors: 1x1 with K == Cin, Cin % 64 == 0; tap-major 3x3,
// stride 1 or 2, pad 0 or 1, or nearest-x2 upsample with pad 1; C1 % 64 == 0 (a K-tile never straddles the
// concat); byte offsets of a tile's window must fit 31 bits (they do: < 16 MB)
static bool buf_dma_ok(const ConvArgs& a, int ks) {
  if (g_no_buf_dma || a.aff_scale) return false;
  if (ks == 1) return a.Cin % 64 == 0 && a.C1 % 64 == 0 && a.K == a.Cin;
  if (a.upsample) return !g_no_buf_ups && a.Cin % 64 == 0 && a.C1 % 64 == 0 && a.stride == 1 && a.pad == 1;
  return a.Cin % 64 == 0 && a.C1 % 64 == 0 && (a.stride == 1 || a.stride == 2) && (a.pad == 0 || a.pad == 1);
}

template <int BM, int BN, int WM, int WN, int KS, bool TAPU>
static void launch_dma(const ConvArgs& a, int grid, hipStream_t s) {
  // (BK 32 tuning mode: only tiles whose 16-B operand pieces divide over the threads --
  // 128 x 160 has 640 B pieces for 256 threads and would leave B rows unloaded)
#ifdef LS_DIAG_KERNELS
  if constexpr (BN >= 64 && (BN * 4) % (WM * WN * 64) == 0 && (BM * 4) % (WM * WN * 64) == 0) {
    if (g_bk == 32) { launch_dma1<BM, BN, WM, WN, KS, TAPU, 4, 32, EPI_ANY>(a, grid, s); return; }
  }
#endif
  if constexpr (KS == 1 || TAPU) {
#ifdef LS_DIAG_KERNELS
    if constexpr (KS == 1) {
      if (g_areg && buf_dma_ok(a, 1) && a.split == 1) {
        switch (epi_kind(a)) {
          case EPI_PLAIN: launch_areg<BM, BN, WM, WN, EPI_PLAIN>(a, grid, s); return;
          case EPI_GEGLU: launch_areg<BM, BN, WM, WN, EPI_GEGLU>(a, grid, s); return;
          default: launch_areg<BM, BN, WM, WN, EPI_ANY>(a, grid, s); return;
        }
      }
    }
    if (g_rs && buf_dma_ok(a, KS) && a.split == 1) {
      switch (epi_kind(a)) {
        case EPI_PLAIN: launch_rs<BM, BN, WM, WN, KS, EPI_PLAIN>(a, grid, s); return;
        case EPI_GEGLU: launch_rs<BM, BN, WM, WN, KS, EPI_GEGLU>(a, grid, s); return;
        default: launch_rs<BM, BN, WM, WN, KS, EPI_ANY>(a, grid, s); return;
      }
    }
#endif
    if (buf_dma_ok(a, KS)) {
      switch (epi_kind(a)) {
        case EPI_PLAIN: launch_dma1<BM, BN, WM, WN, KS, TAPU, 2, 64, EPI_PLAIN, true>(a, grid, s); return;
        case EPI_GEGLU: launch_dma1<BM, BN, WM, WN, KS, TAPU, 2, 64, EPI_GEGLU, true>(a, grid, s); return;
        default: launch_dma1<BM, BN, WM, WN, KS, TAPU, 2, 64, EPI_ANY, true>(a, grid, s); return;
      }
    }
  }
  switch (epi_kind(a)) {
    case EPI_PLAIN: launch_dma1<BM, BN, WM, WN, KS, TAPU, 2, 64, EPI_PLAIN>(a, grid, s); break;
    case EPI_GEGLU: launch_dma1<BM, BN, WM, WN, KS, TAPU, 2, 64, EPI_GEGLU>(a, grid, s); break;
    default: launch_dma1<BM, BN, WM, WN, KS, TAPU, 2, 64, EPI_ANY>(a, grid, s);
  }
}

template <int BN, int KS, bool TAPU, int EPI, bool BUF = false>
static void launch_big2(const ConvArgs& a, int grid, hipStream_t s) {
  const size_t shm = std::max<size_t>((size_t)2 * (256 + BN) * 8 * 16, (size_t)128 * (BN + 4) * 4);
  LS_SET_MAX_DYN_SHM((conv_gemm_big_kernel<BN, KS, TAPU, EPI, BUF>), (int)shm);
  conv_gemm_big_kernel<BN, KS, TAPU, EPI, BUF><<<grid, 512, shm, s>>>(a);
}

template <int BN, int KS, bool TAPU>
static void launch_big1(const ConvArgs& a, int grid, hipStream_t s) {
  if constexpr (KS == 1 || TAPU) {
    if (buf_dma_ok(a, KS)) {
      switch (epi_kind(a)) {
        case EPI_PLAIN: launch_big2<BN, KS, TAPU, EPI_PLAIN, true>(a, grid, s); return;
        case EPI_GEGLU: launch_big2<BN, KS, TAPU, EPI_GEGLU, true>(a, grid, s); return;
        default: launch_big2<BN, KS, TAPU, EPI_ANY, true>(a, grid, s); return;
      }
    }
  }
  switch (epi_kind(a)) {
    case EPI_PLAIN: launch_big2<BN, KS, TAPU, EPI_PLAIN>(a, grid, s); break;
    case EPI_GEGLU: launch_big2<BN, KS, TAPU, EPI_GEGLU>(a, grid, s); break;
    default: launch_big2<BN, KS, TAPU, EPI_ANY>(a, grid, s);
  }
}

#ifdef LS_DIAG_KERNELS  // measured and rejected: diagnostics build only
template <int KS, bool TAPU>
static void launch_big4(const ConvArgs& a, int grid, hipStream_t s) {
  const size_t shm = std::max<size_t>((size_t)4 * (256 + 256) * 4 * 16, (size_t)128 * (256 + 4) * 4);
  LS_SET_MAX_DYN_SHM((conv_gemm_big4_kernel<KS, TAPU>), (int)shm);
  conv_gemm_big4_kernel<KS, TAPU><<<grid, 512, shm, s>>>(a);
}

template <int KS, bool TAPU>
static void launch_p8_1(const ConvArgs& a, int grid, hipStream_t s) {
  const size_t shm = std::max<size_t>((size_t)2 * 4 * 128 * 8 * 16, (size_t)128 * (256 + 4) * 4);
  LS_SET_MAX_DYN_SHM((conv_gemm_p8_kernel<KS, TAPU>), (int)shm);
  conv_gemm_p8_kernel<KS, TAPU><<<grid, 512, shm, s>>>(a);
}

#endif  // LS_DIAG_KERNELS

template <int BN>
static void launch_big(const ConvArgs& a, int ks, bool tapu, int grid, hipStream_t s) {
  if (ks == 1) launch_big1<BN, 1, false>(a, grid, s);
  else if (tapu) launch_big1<BN, 3, true>(a, grid, s);
  else launch_big1<BN, 3, false>(a, grid, s);
}

template <int BM, int BN, int WM, int WN>
static void launch_cfg(const ConvArgs& a, int ks, bool tapu, int grid, hipStream_t s) {
  if (a.aff_scale || g_force_regstage) {  // prologue needs the register path
    if (ks == 1) conv_gemm_kernel<BM, BN, WM, WN, 1, false><<<grid, 256, 0, s>>>(a);
    else if (tapu) conv_gemm_kernel<BM, BN, WM, WN, 3, true><<<grid, 256, 0, s>>>(a);
    else conv_gemm_kernel<BM, BN, WM, WN, 3, false><<<grid, 256, 0, s>>>(a);
  } else {
    if (ks == 1) launch_dma<BM, BN, WM, WN, 1, false>(a, grid, s);
    else if (tapu) launch_dma<BM, BN, WM, WN, 3, true>(a, grid, s);
    else launch_dma<BM, BN, WM, WN, 3, false>(a, grid, s);
  }
}

// ---- halo-tile 3x3 conv dispatch (conv3x3_halo_kernel)
static bool g_halo = ls_env("LS_HALO") == nullptr || atoi(ls_env("LS_HALO")) != 0;  // A/B switch: LS_HALO=0
// the nearest-x2 upsample convs on the halo kernel too (tuning key 18; off: the tiled gather)
static bool g_halo_ups = ls_env("LS_HALO_UPS") == nullptr || atoi(ls_env("LS_HALO_UPS")) != 0;
// A/B switch (tuning key 13): 128-channel tiles where both divide N (3-slot weight ring
// instead of 2 at BN 160)
static bool g_halo_bn128 = ls_env("LS_HALO_BN128") != nullptr;

// the narrow 16-column tile for N <= 16 (tuning key 19; off: the tiled GEMM's 128 x 32 tile)
static bool g_halo_narrow = true;

// patch width of the halo conv for this call (0: not taken)
static int halo_tw(const ls_conv_desc* d, const ConvArgs& a) {
  if (!g_halo || g_force_tile || g_force_regstage || d->ksize != 3 || a.stride != 1 || a.pad != 1 ||
      !a.ccm || a.Cin % 64 || a.C1 % 64 || a.K != 9 * a.Cin || a.y_f32 || a.act != LS_ACT_NONE ||
      a.ln_mr || a.stats_out || a.ldy % 8 || (a.res && a.ldr % 8))
    return 0;
  // nearest x2 upsample (Upsample3D, resnet.py:53-71; round 6): no input affine (the UNet's
  // upsampler conv has none); the halo image is built in output space from the input pixels
  if (a.upsample ? (!g_halo_ups || a.aff_scale || a.Ho != 2 * a.H || a.Wo != 2 * a.W) : (a.Ho != a.H || a.Wo != a.W))
    return 0;
  // N <= 640: with more output channels the patch is re-loaded and re-transformed per N tile
  // and the tiled 256x256 kernel wins (VAE 512 channels at 32^2: 3667 vs 3409 us; 128 at
  // 256^2: 18660 vs 23610 us incl. the materialised GroupNorm; profiles/r04f_ab_t256_halo.txt)
  // (N = 8 / 16: the narrow tile -- conv_out of the VAE decoder / encoder, N padded to 8)
  const bool narrow = a.N % 8 == 0 && a.N <= 16 && a.H % 8 == 0 && g_halo_narrow;
  if (((a.N % 160 && a.N % 128) || a.N > 640) && !narrow) return 0;
  if (a.aff_scale && (!a.silu_in || a.pix_per_sample % (a.H * a.W) || ((uintptr_t)a.aff_scale | (uintptr_t)a.aff_shift) & 15))
    return 0;  // (the kernel's input transform is the GroupNorm affine + SiLU of a ResnetBlock)
  if (((uintptr_t)a.x1 | (uintptr_t)a.x2 | (uintptr_t)a.w) & 15 || a.ld1 % 8 || (a.C2 && a.ld2 % 8)) return 0;
  // 16 x 16 patches everywhere: the smallest halo overhead ((16 + 2)^2 / 256 = 1.27 input
  // pixels per output pixel; 32 x 8: 1.33, 64 x 4: 1.55) and no register spills
  const int tw = (a.Wo % 16 == 0 && a.Ho % 16 == 0) ? 16 : 0;
  if (!tw) return 0;
  if ((long)a.H * a.W * a.ld1 * 2 >= (1L << 31) || (a.C2 && (long)a.H * a.W * a.ld2 * 2 >= (1L << 31)))
    return 0;  // per-image buffer descriptors
  return tw;
}

template <int TW, int BN, bool GN, bool CSF, int TH>
static void launch_halo3(const ConvArgs& a, hipStream_t s) {
  using HC = HaloCfg<TW, BN, TH>;
  const int ntile = a.n_img * (a.H / HC::TH) * (a.W / TW) * ((a.N + BN - 1) / BN);
  LS_SET_MAX_DYN_SHM((conv3x3_halo_kernel<TW, BN, GN, CSF, TH>), HC::SHM);
  conv3x3_halo_kernel<TW, BN, GN, CSF, TH><<<ntile, HC::NT, HC::SHM, s>>>(a);
}

template <int TW, int BN, int TH = 256 / TW>
static void launch_halo2(const ConvArgs& a, hipStream_t s) {
  if (a.aff_scale) {
    if (a.cs_out) launch_halo3<TW, BN, true, true, TH>(a, s);
    else launch_halo3<TW, BN, true, false, TH>(a, s);
  } else {
    if (a.cs_out) launch_halo3<TW, BN, false, true, TH>(a, s);
    else launch_halo3<TW, BN, false, false, TH>(a, s);
  }
}

// 16 x 8 patches, two blocks per CU for the 128-column tiles of convs with at most 4 input
// chunks (Cin <= 256), where a block's halo prologue and epilogue are a large share of its
// time: VAE 128 ch at 256^2 17.67 -> 17.23 ms, 128 -> 256 at 128^2 8.74 -> 8.43 ms, 256 at
// 128^2 a tie; at Cin 512 (8 chunks) the 2-slot weight ring loses to the 1-block form's 3
// slots (13.12 -> 13.55 ms at 64^2), profiles/r05k_halo_ab.txt.  A/B switch LS_HALO_TH8=0.
static bool g_halo_th8 = ls_env("LS_HALO_TH8") == nullptr || atoi(ls_env("LS_HALO_TH8")) != 0;

template <int TW>
static void launch_halo1(const ConvArgs& a, hipStream_t s) {
  if (a.N <= 16) launch_halo2<TW, 16, 8>(a, s);
  else if (a.N % 160 == 0 && !(g_halo_bn128 && a.N % 128 == 0)) launch_halo2<TW, 160>(a, s);
  else if (g_halo_th8 && a.H % 8 == 0 && a.Cin <= 256) launch_halo2<TW, 128, 8>(a, s);
  else launch_halo2<TW, 128>(a, s);
}

static void launch_halo(const ConvArgs& a, int tw, hipStream_t s) {
  (void)tw;  // (16: the only patch width compiled)
  if (a.upsample) {  // the kernel works in output space: H, W = the output image
    ConvArgs o = a;
    o.H = a.Ho;
    o.W = a.Wo;
    launch_halo1<16>(o, s);
    return;
  }
  launch_halo1<16>(a, s);
}

#ifdef LS_DIAG_KERNELS  // measured and rejected: diagnostics build only
// 256 x 128 tiles (8 waves as 4 x 2, 64 x 64 each) with a 3-stage LDS ring (147 KB) for the
// short-K linears (K <= 1280, N % 128 == 0): two K-tiles of operand DMA in flight instead of
// one.  (A/B switch LS_GEMM_T256=0/1; tile id 260.  256 x 160 would leave 2.5 B pieces per thread.)
static int g_t256 = ls_env("LS_GEMM_T256") ? atoi(ls_env("LS_GEMM_T256")) : 0;

#endif  // LS_DIAG_KERNELS

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
  a.bias = d->bias; a.rowvec = d->rowvec; a.rows_per_vec = d->rows_per_vec; a.rowvec_mod = d->rowvec_mod;
  a.ln_mr = d->ln_rowstats; a.ln_cs = d->ln_colsum;
  if (a.ln_mr && (!a.ln_cs || d->ksize != 1)) return fail(LS_ERR_INVALID, "ls_conv2d: ln_rowstats needs ln_colsum, ksize 1");
  a.rowvec_ld = d->rowvec_ld > 0 ? d->rowvec_ld : d->N;
  a.res = d->res; a.ldr = d->ldr; a.out_scale = d->out_scale == 0.f ? 1.f : d->out_scale; a.act = d->act;
  a.y = d->y; a.ldy = d->ldy; a.y_f32 = d->y_f32;
  a.stats_out = d->row_stats_out;
  a.stats_eps = d->row_stats_eps > 0.f ? d->row_stats_eps : 1e-5f;
  if (a.stats_out && (d->ksize != 1 || d->act == LS_ACT_GEGLU || d->y_f32))
    return fail(LS_ERR_INVALID, "ls_conv2d: row_stats_out needs ksize 1, bf16 output, no GEGLU");
  a.cs_out = d->gn_colsum_out;
  if (a.cs_out && (M % CS_ROWS || d->N % 8 || d->ldy % 8 || d->act == LS_ACT_GEGLU || d->y_f32))
    return fail(LS_ERR_INVALID, "ls_conv2d: gn_colsum_out needs M % 128 == 0, N % 8 == 0, bf16 output, no GEGLU");
  a.ablate = g_ablate;
  a.ccm = (d->ksize == 3 && Cin % 64 == 0) ? 1 : 0;
  a.gm = 1;  // (set with the tile below)
  a.ktiles = d->K / 64;
  t = pick_tile(M, d->N, a.ktiles, d->split_k <= 0 && d->workspace != nullptr,
                !d->aff_scale && !g_force_regstage && (d->ksize == 1 || Cin % 64 == 0), d->ksize);
  if (g_force_tile) {
    static const int tb[11][2] = {{0, 0}, {128, 128}, {128, 64}, {64, 64}, {128, 32}, {256, 256}, {256, 128},
                                  {257, 256}, {258, 256}, {128, 160}, {259, 160}};
    t.bm = tb[g_force_tile][0]; t.bn = tb[g_force_tile][1]; t.split = g_force_split ? g_force_split : 1;
  }
#ifdef LS_DIAG_KERNELS
  if (g_t256 && !g_force_tile && d->ksize == 1 && a.ktiles <= 20 && d->N % 128 == 0 && !d->aff_scale &&
      M % 256 == 0 && d->K == Cin && Cin % 64 == 0 && d->C1 % 64 == 0)
    t = {260, 128, 1};
#endif
  a.ntm = cdiv(M, t.bm > 256 ? 256 : t.bm); a.ntn = cdiv(d->N, t.bn);  // 257..260 = 256-row kernel variants
  // grouped raster (LS_GEMM_GM=g, g row-bands per group): it cuts the wide linears' L2-miss
  // fetch (GEGLU W1 at 8x8 3.6 -> 1.3 GB per call) but measured +0.4 ms per 32-window step
  // against the column-fastest order over three alternated same-box rounds
  // (profiles/r03i_locality_sweep.txt), so the default stays column-fastest (gm = 1)
  a.gm = g_gemm_gm > 0 ? g_gemm_gm : 1;
  // round 5: 4 row bands per group for 256x256 1x1 tiles with K <= 1920 (out2 181 -> 173 us,
  // sc2b -1 %, profiles/r05s_gm_ab.txt; at K = 5120 the grouping loses); A/B switch
  // LS_GEMM_GM_SHORTK=0
  if (g_gemm_gm <= 0 && g_gm_shortk && t.bm == 256 && t.bn == 256 && d->ksize == 1 && d->K <= 1920) a.gm = 4;
  a.gm = std::max(1, std::min(a.gm, a.ntm));
  split = d->split_k > 0 ? d->split_k : t.split;
  split = std::min(split, a.ktiles);
  a.kt_per_split = cdiv(a.ktiles, split);
  split = cdiv(a.ktiles, a.kt_per_split);
  a.split = split;
  a.partial = nullptr;
  return LS_OK;
}

}  // namespace ls

using namespace ls;

namespace ls { void attn_set_attn6(bool on); }

extern int g_ff_chain_fmr;  // ls_ff.hip

extern "C" int ls_set_tuning(int32_t key, int32_t value) {
  switch (key) {
    case 18: g_halo_ups = value != 0; return LS_OK;
    case 19: g_halo_narrow = value != 0; return LS_OK;
    case 20: g_rb640_res = value != 0; return LS_OK;
    case 17:
#ifndef LS_DIAG_KERNELS
      if (value == 2) return fail(LS_ERR_INVALID, "ls_ff_chain at 32 rows per wave: diagnostics build only");
#endif
      if (value != 1 && value != 2) return fail(LS_ERR_INVALID, "ls_ff_chain rows per wave: 1 (16) or 2 (32)");
      g_ff_chain_fmr = value;
      return LS_OK;
    case 1: g_force_regstage = value != 0; return LS_OK;
    case 2:
#ifndef LS_DIAG_KERNELS
      if (value == 7 || value == 8) return fail(LS_ERR_INVALID, "tile ids 7 / 8: diagnostics build only");
#endif
      if (value < 0 || value > 9) return fail(LS_ERR_INVALID, "tile id 0..9");
      g_force_tile = value;
      return LS_OK;
    case 3: g_force_split = value; return LS_OK;
    case 4: g_ablate = value; return LS_OK;
#ifdef LS_DIAG_KERNELS
    case 5: if (value != 32 && value != 64) return fail(LS_ERR_INVALID, "BK 32 or 64"); g_bk = value; return LS_OK;
#endif
    case 6: g_rowblock = value != 0; return LS_OK;
    case 7: g_rowblock640 = value != 0; return LS_OK;
    case 8: g_halo = value != 0; return LS_OK;
    case 12:  // (the padded-row halo image is gone since the compact image, round 5)
      if (!value) return fail(LS_ERR_INVALID, "LS_HALO_RP=0 (padded halo rows) no longer exists");
      return LS_OK;
    case 13: g_halo_bn128 = value != 0; return LS_OK;
    case 15: g_rb640_fm2 = value != 0; return LS_OK;
    case 16: g_halo_th8 = value != 0; return LS_OK;
    case 9:
#ifndef LS_DIAG_KERNELS
      if (value) return fail(LS_ERR_INVALID, "attn6: diagnostics build only");
#endif
      attn_set_attn6(value != 0);
      return LS_OK;
#ifdef LS_DIAG_KERNELS
    case 10: g_t256 = value; return LS_OK;
    case 11: g_rs = value; return LS_OK;
    case 14: g_areg = value != 0; return LS_OK;
#endif
    default: return fail(LS_ERR_INVALID, "ls_set_tuning: unknown key");
  }
}

template <typename K>
static int occ(K kern, int threads, size_t shm) {
  int n = 0;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, threads, shm) != hipSuccess) return -1;
  return n;
}

extern "C" int ls_gemm_occupancy(int32_t which) {
  switch (which) {
    case 1: return occ(conv_gemm_dma_kernel<128, 160, 2, 2, 1, false, 2, 64, EPI_PLAIN>, 256,
                       (size_t)2 * (128 + 160) * 8 * 16);
    case 2: return occ(conv_gemm_big_kernel<256, 1, false, EPI_PLAIN>, 512, (size_t)2 * (256 + 256) * 8 * 16);
    case 3: return occ(conv_gemm_dma_kernel<128, 128, 2, 2, 1, false, 2, 64, EPI_PLAIN>, 256,
                       (size_t)2 * (128 + 128) * 8 * 16);
    default: return fail(LS_ERR_INVALID, "ls_gemm_occupancy: which 1..3");
  }
}

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
  if (const int tw = halo_tw(d, a)) {  // 3x3 from an LDS halo tile, input affine fused, with the column sums
    launch_halo(a, tw, s);
    return check_launch("conv3x3_halo_kernel");
  }
  float* cs = a.cs_out;  // GroupNorm column sums: epilogue (tiled / row-block) or a trailing read pass
  if (rowblock_ok(d, a)) {
    if (launch_rowblock(a, s)) return check_launch("gemm_rowblock_kernel");  // with cs_out if given
    a.cs_out = nullptr;  // no row-block instance with the sums: without them, then a read pass
    if (cs && launch_rowblock(a, s)) {
      if ((rc = check_launch("gemm_rowblock_kernel")) != LS_OK) return rc;
      return launch_colsum_pass((const u16*)d->y, d->ldy, a.M, d->N, cs, s);
    }
  }
  a.cs_out = nullptr;
  if (a.stats_out) {  // tiled path: the GEMM, then LayerNorm statistics of y in a second pass
    float* so = a.stats_out;
    a.stats_out = nullptr;
    ls_conv_desc d2 = *d;
    d2.row_stats_out = nullptr;
    if ((rc = ls_conv2d(&d2, stream)) != LS_OK) return rc;
    return ls_row_stats((const uint16_t*)d->y, d->ldy, a.M, d->N, a.stats_eps, so, stream);
  }
  const bool tapu = (d->ksize == 3) && (a.Cin % 64 == 0);
  const int grid = a.ntm * a.ntn * a.split;
  // epilogue column sums: single-pass vectorised epilogue and a tile whose staging
  // buffer holds the per-thread partials (cs_tile_fits; not 128x32 / 64x64)
  const bool vec = (a.N % 8 == 0) && (a.ldy % 8 == 0) && (!a.res || a.ldr % 8 == 0);
  // (not the 256-row kernels: compiled in, the sums cost their main loop ~12 % -- they run
  // at the 256-VGPR limit -- against a ~15 us read pass; same-box A/B, scripts/ab_lib.sh)
  const bool cs_epi = cs && a.split == 1 && vec && !(t.bm == 128 && t.bn == 32) && t.bm != 64 &&
                      (t.bm < 256 || (t.bm == 260 && epi_kind(a) == EPI_PLAIN));
  if (cs_epi) a.cs_out = cs;
#ifdef LS_DIAG_KERNELS
  if (t.bm == 260) {  // 256 x 128, 3-stage ring (short-K linears)
    switch (epi_kind(a)) {
      case EPI_PLAIN: launch_dma1<256, 128, 4, 2, 1, false, 3, 64, EPI_PLAIN, true>(a, grid, s); break;
      case EPI_GEGLU: launch_dma1<256, 128, 4, 2, 1, false, 3, 64, EPI_GEGLU, true>(a, grid, s); break;
      default: launch_dma1<256, 128, 4, 2, 1, false, 3, 64, EPI_ANY, true>(a, grid, s);
    }
  } else if (t.bm == 257 && !a.aff_scale && !g_force_regstage && (d->ksize == 1 || tapu)) {  // phased 256x256
    if (d->ksize == 1) launch_p8_1<1, false>(a, grid, s);
    else launch_p8_1<3, true>(a, grid, s);
  } else if (t.bm == 258 && !a.aff_scale && !g_force_regstage && (d->ksize == 1 || tapu)) {  // 4-stage BK 32
    if (d->ksize == 1) launch_big4<1, false>(a, grid, s);
    else launch_big4<3, true>(a, grid, s);
  } else
#endif
  if (t.bm == 256 && !a.aff_scale && !g_force_regstage) {
    if (t.bn == 256) launch_big<256>(a, d->ksize, tapu, grid, s);
    else launch_big<128>(a, d->ksize, tapu, grid, s);
  } else if (t.bm == 128 && t.bn == 128) launch_cfg<128, 128, 2, 2>(a, d->ksize, tapu, grid, s);
  else if (t.bm == 128 && t.bn == 160) launch_cfg<128, 160, 2, 2>(a, d->ksize, tapu, grid, s);

  else if (t.bm == 128 && t.bn == 64) launch_cfg<128, 64, 2, 2>(a, d->ksize, tapu, grid, s);
  else if (t.bm == 128 && t.bn == 32) launch_cfg<128, 32, 4, 1>(a, d->ksize, tapu, grid, s);
  else launch_cfg<64, 64, 2, 2>(a, d->ksize, tapu, grid, s);
  if ((rc = check_launch("conv_gemm_kernel")) != LS_OK) return rc;
  if (a.split > 1) {
    const long nchunk = (long)a.M * ((((a.act == LS_ACT_GEGLU) ? a.N / 2 : a.N) + 7) / 8);
    splitk_reduce_kernel<<<cdiv(nchunk, 256), 256, 0, s>>>(a);
    if ((rc = check_launch("splitk_reduce_kernel")) != LS_OK) return rc;
  }
  if (cs && !cs_epi) return launch_colsum_pass((const u16*)d->y, d->ldy, a.M, d->N, cs, s);
  return LS_OK;
}

extern "C" int ls_conv_path(const ls_conv_desc* d) {
  ConvArgs a; TileCfg t; int split;
  if (build_args(d, a, t, split) != LS_OK) return -1;
  a.cs_out = nullptr;  // (the column sums never change the path)
  int ntm, ntn;
  if (rowblock_ok(d, a) && rowblock_flags(a, &ntm, &ntn) >= 0) return 1;
  if (halo_tw(d, a)) return 3;
  return (a.aff_scale || g_force_regstage) ? 2 : 0;
}

extern "C" int ls_gn_colsum(const uint16_t* y, int64_t ldy, int64_t M, int32_t N, float* out, void* stream) {
  return launch_colsum_pass(y, ldy, M, N, out, (hipStream_t)stream);
}
