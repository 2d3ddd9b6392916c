// FeedForward of BasicTransformerBlock / TemporalTransformerBlock at C = 320 fused into
// one gfx950 kernel (diffusers FeedForward(dim, activation_fn="geglu"): GEGLU proj
// C -> 2*4C, h * gelu(g), Linear 4C -> C; attention.py:174-199 norm3 + ff,
// motion_module.py:240-313 ff_norm + ff), with the LayerNorm folded in and the
// residual added:
//
//   y = x + W2 GEGLU(W1 LN(x) + b1) + b2
//
// Before this kernel the 4C-wide GEGLU output went to HBM and came back (1.3 GB each
// way per call at 32 windows): the W1 row-block GEMM (VALU-bound on its GELU epilogue)
// and the W2 tiled GEMM (memory-bound) ran 1.0 + 0.59 ms.
//
// A workgroup owns 128 rows (8 waves x 16); a wave keeps its 16 rows of LN(x) in
// registers (40 VGPRs; LayerNorm applied in place from the producer's row statistics,
// gamma / beta folded into W1 / b1 on the host) and the C^T = W2 G^T accumulator of all C
// output columns (20 tiles, 80 VGPRs).  The inner dimension streams in chunks of 32
// GEGLU columns: per chunk the 64 interleaved W1 rows (h, g tiles, 40 KB) and the W2
// columns (C x 32, 20 KB) arrive by LDS DMA into one of two stages while the previous
// chunk computes:
//   * GEMM1: C^T = W1 A^T (16x16x32), four 16-row tiles h0 g0 h1 g1 -- a lane holds 4
//     consecutive GEGLU columns of its row in each;
//   * GEGLU on the accumulators -> 8 bf16 per lane: columns 4 lg .. + 3 and 16 + 4 lg .. + 3
//     of the chunk;
//   * GEMM2: those 8 values ARE the B operand of out^T += W2 G^T for k-slots lg*8 .. + 7,
//     because the host packs each W2 chunk with its 32 columns permuted the same way
//     (slot (lg, i) -> column i < 4 ? 4 lg + i : 16 + 4 lg + i - 4): the intermediate
//     never leaves the registers.
// W2 chunk images are [C rows][4 x 16 B] with the 16-B pieces XOR-swizzled by
// ((row >> 3) & 1) << 1 (host-side), which makes every ds_read_b128 lane group hit
// 64 distinct banks; W1 images use the row-block kernel's 64-wide swizzle.
#include "ls_common.h"

namespace ls {

struct FFArgs {
  const u16* x;       // [M][ldx] FF input (pre-LayerNorm), also the residual
  const float* ln_mr; // [M][2] (mean, rstd) of x rows
  const u16* w1;      // [2I][C] GEGLU W1, rows interleaved in 16-blocks (h, g), LN gamma folded
  const float* b1;    // [2I] its bias (+ W1 beta), same interleave
  const u16* w2;      // [I/32][C][32] W2 chunks, columns permuted + pieces swizzled (see above)
  const float* b2;    // [C]
  u16* y;             // [M][ldy]
  long M;
  int ldx, ldy;
};

template <int C, int I, int PD1 = 2, int PD2 = 6>
__global__ void __launch_bounds__(512, 1) ff_fused_kernel(FFArgs a) {
  constexpr int KT = C / 32;              // GEMM1 k-steps
  constexpr int NCH = I / 32;             // inner chunks
  constexpr int WIMG = 64 * (C / 64) * 8; // uint4: W1 chunk, C/64 images of [64 rows][8 pieces]
  constexpr int W2IMG = C * 4;            // uint4: W2 chunk, [C rows][4 pieces]
  constexpr int STAGE = WIMG + W2IMG;
  constexpr int NT2 = C / 16;             // output tiles
  constexpr int PW1 = WIMG / 512;         // W1 pieces per thread per chunk
  constexpr int UW2 = W2IMG / 64;         // W2 wave-instructions per chunk
  static_assert(WIMG % 512 == 0 && W2IMG % 64 == 0 && C % 64 == 0 && I % 32 == 0, "ff_fused shape");
  static_assert(PD1 >= 1 && PD1 <= KT && PD2 >= PD1 && PD2 <= NT2, "prefetch depths");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // [2][STAGE], then b1 (2I fp32)
  float* b1s = (float*)(lds + 2 * STAGE);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const long row = (long)blockIdx.x * 128 + wid * 16 + l16;
  const bool live = row < a.M;

  for (int i = tid; i < 2 * I / 4; i += 512) ((float4*)b1s)[i] = ((const float4*)a.b1)[i];

  auto issue = [&](int c, int st) __attribute__((always_inline)) {
    uint4* dst = lds + st * STAGE;
#pragma unroll
    for (int p = 0; p < PW1; ++p) {  // piece q: image p (k 64p .. 64p + 63), row (q / 8) % 64, physical chunk q % 8
      const int q = p * 512 + tid, r = (q >> 3) & 63, pc = q & 7;
      const int lc = pc ^ ((r >> 1) & 7);
      glds16(a.w1 + (long)(c * 64 + r) * C + p * 64 + lc * 8, dst + p * 512 + wid * 64);
    }
    for (int u = wid; u < UW2; u += 8)  // W2 chunk: a contiguous copy (host-packed layout)
      glds16(a.w2 + ((long)c * W2IMG + u * 64 + lane) * 8, dst + WIMG + u * 64);
  };
  issue(0, 0);

  // A rows -> registers, LayerNorm in place (bf16, like the reference's normalised rows)
  bf16x8 ar[KT];
  {
    const u16* src = a.x + (live ? row : 0) * a.ldx + lg * 8;
#pragma unroll
    for (int s = 0; s < KT; ++s) ar[s] = live ? *(const bf16x8*)(src + s * 32) : __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
    const float2 mr = live ? *(const float2*)(a.ln_mr + 2 * row) : make_float2(0.f, 0.f);
    const float rstd = mr.y, nmr = -mr.x * mr.y;
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      bf16x8 v = ar[s];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)fmaf((float)v[e], rstd, nmr);
      ar[s] = v;
    }
  }

  f32x4 out[NT2];
#pragma unroll
  for (int t = 0; t < NT2; ++t) out[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int p2 = lg ^ (((l16 >> 3) & 1) << 1);  // this lane's physical W2 piece

  for (int c = 0; c < NCH; ++c) {
    wait_vm<0>();  // this wave's DMA of chunk c (and the A rows) landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone's; the other stage (chunk c - 1) is no longer read
    asm volatile("" ::: "memory");
    if (c + 1 < NCH) issue(c + 1, (c + 1) & 1);
    const uint4* cur = lds + (c & 1) * STAGE;

    // GEMM1: the chunk's 4 W1 tiles (h0 g0 h1 g1)
    f32x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto frag = [&](int s, int t) {
      return __builtin_bit_cast(bf16x8, cur[(s >> 1) * 512 + swz_bk<64>(t * 16 + l16, (s & 1) * 4 + lg)]);
    };
    // W1 fragments PD1 k-steps ahead, the first PD2 W2 fragments issued under GEMM1 (an
    // LDS read one MFMA ahead left each W2 MFMA waiting out the read's latency)
    const uint4* w2 = cur + WIMG;
    bf16x8 wf[PD1][4];
#pragma unroll
    for (int p = 0; p < PD1; ++p)
#pragma unroll
      for (int t = 0; t < 4; ++t) wf[p][t] = frag(p, t);
    uint4 w2q[PD2];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      const int sl = s % PD1;
      bf16x8 cw[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) cw[t] = wf[sl][t];
      if (s + PD1 < KT) {
#pragma unroll
        for (int t = 0; t < 4; ++t) wf[sl][t] = frag(s + PD1, t);
      } else if (s + PD1 - KT < PD2) {
        w2q[s + PD1 - KT] = w2[((s + PD1 - KT) * 16 + l16) * 4 + p2];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[t], ar[s], acc[t], 0, 0, 0);
    }
#pragma unroll
    for (int q = PD1; q < PD2; ++q) w2q[q] = w2[(q * 16 + l16) * 4 + p2];
    // GEGLU -> the B operand of GEMM2 (k-slot order matches the host's W2 permutation)
    const float* bb = b1s + c * 64 + 4 * lg;
    const float4 bh0 = *(const float4*)(bb), bg0 = *(const float4*)(bb + 16);
    const float4 bh1 = *(const float4*)(bb + 32), bg1 = *(const float4*)(bb + 48);
    const float hb0[4] = {bh0.x, bh0.y, bh0.z, bh0.w}, gb0[4] = {bg0.x, bg0.y, bg0.z, bg0.w};
    const float hb1[4] = {bh1.x, bh1.y, bh1.z, bh1.w}, gb1[4] = {bg1.x, bg1.y, bg1.z, bg1.w};
    bf16x8 gv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      gv[r] = (__bf16)((acc[0][r] + hb0[r]) * gelu_erf(acc[1][r] + gb0[r]));
      gv[4 + r] = (__bf16)((acc[2][r] + hb1[r]) * gelu_erf(acc[3][r] + gb1[r]));
    }
    // GEMM2: out^T[16 t + 4 lg + r][row] += W2[16 t + l16][chunk k-slots] . G^T, W2
    // fragments PD2 tiles ahead
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const bf16x8 wv = __builtin_bit_cast(bf16x8, w2q[t % PD2]);
      if (t + PD2 < NT2) w2q[t % PD2] = w2[((t + PD2) * 16 + l16) * 4 + p2];
      out[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, gv, out[t], 0, 0, 0);
    }
  }

  // y = out + b2 + x (the residual: FF input rows, re-read -- the registers hold LN(x))
  if (live) {
    const u16* xr = a.x + row * a.ldx;
    u16* yr = a.y + row * a.ldy;
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const int col = 16 * t + 4 * lg;
      const float4 b = *(const float4*)(a.b2 + col);
      const uint2 rs = *(const uint2*)(xr + col);
      const float o0 = out[t][0] + b.x + __uint_as_float(rs.x << 16);
      const float o1 = out[t][1] + b.y + __uint_as_float(rs.x & 0xffff0000u);
      const float o2 = out[t][2] + b.z + __uint_as_float(rs.y << 16);
      const float o3 = out[t][3] + b.w + __uint_as_float(rs.y & 0xffff0000u);
      *(uint2*)(yr + col) = make_uint2(pack2(o0, o1), pack2(o2, o3));
    }
  }
}

// ---------------------------------------------------------------------------------------
// ff_chain_kernel (round 6, ABI 14 ls_ff_chain): the 32x32-level tail of a Transformer3D /
// motion block in ONE launch -- the attention branch's out-projection + residual, the
// LayerNorm, the GEGLU FeedForward + residual, proj_out + the block input, and the
// GroupNorm column sums of the result for the next GroupNorm:
//
//   h2 = o Wo^T + bo + h1                     attn2 (attn1 without audio) to_out + residual
//                                             (attention.py:174-199); the motion block's last
//                                             attention to_out (motion_module.py:262-313)
//   y  = h2 + W2 GEGLU(W1 LN(h2) + b1) + b2   norm3 + ff / ff_norm + ff, as ff_fused_kernel
//   z  = y Wp^T + bp + xb                     proj_out + the block input (attention.py:110-118,
//                                             motion_module.py:126-151)
//
// Unfused, h2 and y each make a round trip through HBM (write + read: 2 GB per call at 48
// windows) and the two K = C projections run as separate latency-bound row-block GEMMs
// (390 us each at 48 windows, profiles/r05f2_step_calls.txt).  Here they are two more
// GEMM phases of the FeedForward kernel on the registers it already holds:
//   * phase A (GEMM0): the wave's 16 o rows are the B operand (40 VGPRs, natural k order),
//     the 20 accumulator tiles of all C outputs (80 VGPRs) start at bo; Wo streams through
//     the LDS stages in k-step images [C rows][32 k] (a 60-KB stage holds three);
//   * + h1, rounded to bf16 (the values the unfused path stores), the row's LayerNorm
//     statistics (two-pass, fp32, across the 4 lane groups of a row by cross-row swaps) and
//     LN(h2) into the GEMM1 operand registers -- in ACCUMULATOR order: k-slot (lg, e) of
//     k-step s is column 32 s + (e < 4 ? 4 lg + e : 16 + 4 lg + e - 4), so the host packs
//     W1's columns with that permutation (pack_ff_w2's order); the FeedForward's
//     accumulators start at h2 + b2 (the residual);
//   * phase B: the FeedForward chunk loop of ff_fused_kernel;
//   * y rounded to bf16 into the operand registers (accumulator order again: Wp packed
//     permuted), the accumulators restart at bp, phase C (GEMM3) streams Wp like Wo;
//   * + xb, bf16; the block's 128 x C result goes through LDS once: coalesced 16-B row
//     stores, and the GroupNorm column sums of the stored values for the block's 128-row
//     slot (ls_conv_desc.gn_colsum_out's layout) -- so the consumer's ls_groupnorm_colsum
//     needs no read pass.
// Per row it reads o, h1, xb and writes z; the GEMM work grows by 2 x 2 C^2 flop per row
// (+17 % over the FeedForward's 2 x 3 x 2 C I).
struct FFChainArgs {
  const u16* o;       // [M][ldo]  attention output (GEMM0's operand)
  const u16* wo;      // [C/32][C][32]  Wo k-step images (natural k order, pieces swizzled)
  const float* bo;    // [C]
  const u16* h1;      // [M][ldh]  GEMM0's residual
  const u16* w1;      // [2I][C]   GEGLU W1: rows interleaved (h, g), LN gamma folded, k permuted
  const float* b1;    // [2I]
  const u16* w2;      // [I/32][C][32] (pack_ff_w2)
  const float* b2;    // [C]
  const u16* wp;      // [C/32][C][32]  Wp k-step images (k permuted, pieces swizzled)
  const float* bp;    // [C]
  const u16* xb;      // [M][ldxb] proj_out's residual (the block input)
  u16* z;             // [M][ldz]
  float* cs_out;      // [M/128][2][C] GroupNorm column sums of z, or null
  long M;
  int ldo, ldh, ldxb, ldz;
  float eps;          // the LayerNorm's eps
};

// FMR = 16-row fragments per wave: 1 -> 8 waves of 16 rows (two per SIMD, <= 256 registers);
// 2 -> 4 waves of 32 rows, one per SIMD (up to 512 registers, the accumulators in AGPRs):
// every W fragment read from LDS then feeds two MFMAs -- at one fragment per MFMA the
// FeedForward's fragment reads alone fill the LDS array (1 KB per 16-cycle MFMA per SIMD =
// 256 B/clk/CU), which had left it at 0.34 of the MFMA peak.
template <int C, int I, int FMR>
__global__ void __launch_bounds__(512 / FMR, 1) ff_chain_kernel(FFChainArgs a) {
  constexpr int NW = 8 / FMR;             // waves per block (128 rows)
  constexpr int NT = 64 * NW;
  constexpr int KT = C / 32;              // k-steps of every C-wide contraction
  constexpr int NCH = I / 32;             // FeedForward inner chunks
  constexpr int WIMG = 64 * (C / 64) * 8; // uint4: W1 chunk
  constexpr int W2IMG = C * 4;            // uint4: one [C][32] k-step image (W2 chunk, Wo / Wp k-step)
  constexpr int STAGE = WIMG + W2IMG;
  constexpr int KPS = STAGE / W2IMG;      // k-step images per stage in phases A / C
  constexpr int NA = (KT + KPS - 1) / KPS;  // stages of phase A (and of phase C)
  constexpr int NT2 = C / 16;             // output tiles
  constexpr int PW1 = WIMG / NT;
  constexpr int UW2 = W2IMG / 64;
  constexpr int PD1 = 2, PD2 = 6;
  constexpr int ZP = C + 8;               // LDS pitch (bf16) of the block's result image
  constexpr int RG = NT >= C ? 4 : 2;     // row groups of the column-sum pass
  static_assert(STAGE % W2IMG == 0 && KPS >= 1 && WIMG % NT == 0, "ff_chain stage layout");
  static_assert(2 * STAGE * 16 >= 128 * ZP * 2 + RG * (C / 4) * 8 * 4, "ff_chain epilogue LDS");
  static_assert(C == 320 && I == 1280 && (FMR == 1 || FMR == 2), "ff_chain shape");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // [2][STAGE], then b1 (2I fp32)
  float* b1s = (float*)(lds + 2 * STAGE);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const long row0 = (long)blockIdx.x * 128;
  const int wr0 = wid * 16 * FMR + l16;   // block row of fragment 0 (fragment f: + 16 f); host: M % 128 == 0

  for (int i = tid; i < 2 * I / 4; i += NT) ((float4*)b1s)[i] = ((const float4*)a.b1)[i];

  // chunk g of the launch: [0, NA) Wo stages, [NA, NA + NCH) FeedForward chunks, then Wp stages.
  // Buffer-descriptor DMA: every per-thread byte offset is fixed over the chunks (W1 piece p:
  // row (q >> 3) & 63 of the chunk, image q >> 9, swizzled chunk; W2 / Wo / Wp: slot u of the
  // image), a chunk only moves the uniform soffset, and the LDS destinations are LDS-space
  // addresses (one s_add to M0 per DMA instead of a 64-bit global address + readfirstlane).
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  __builtin_assume(wid_u >= 0 && wid_u < NW);
  const i32x4 rs_w1 = buffer_rsrc(a.w1, (uint32_t)(2L * I * C * 2));
  const i32x4 rs_w2 = buffer_rsrc(a.w2, (uint32_t)((long)I * C * 2));
  const i32x4 rs_wo = buffer_rsrc(a.wo, (uint32_t)((long)C * C * 2));
  const i32x4 rs_wp = buffer_rsrc(a.wp, (uint32_t)((long)C * C * 2));
  int vo1[PW1];
#pragma unroll
  for (int p = 0; p < PW1; ++p) {  // piece q: image q >> 9, row (q >> 3) & 63, physical chunk q & 7
    const int q = p * NT + tid, r = (q >> 3) & 63, pc = q & 7;
    const int lc = pc ^ ((r >> 1) & 7);
    vo1[p] = (r * C + (q >> 9) * 64 + lc * 8) * 2;
  }
  const int vol = (wid_u * 64 + lane) * 16;  // slot u = wid + k NW of a [C][32] image: vol + k NW 1 KB
  lds_u4* const lbase = (lds_u4*)lds;
  auto issue = [&](int g, int st) __attribute__((always_inline)) {
    lds_u4* const dst = lbase + st * STAGE;
    if (g < NA || g >= NA + NCH) {
      const bool o = g < NA;
      const int q = o ? g : g - NA - NCH;
      const int nk = min(KPS, KT - q * KPS);
      const int so = q * KPS * W2IMG * 16;
      for (int k = 0; wid_u + k * NW < nk * UW2; ++k)
        ls_raw_buffer_load_lds(o ? rs_wo : rs_wp, (__attribute__((address_space(3))) void*)(dst + (wid_u + k * NW) * 64),
                               16, vol + k * NW * 1024, so, 0, 0);
    } else {
      const int c = g - NA;
#pragma unroll
      for (int p = 0; p < PW1; ++p)
        ls_raw_buffer_load_lds(rs_w1, (__attribute__((address_space(3))) void*)(dst + p * NT + wid_u * 64), 16, vo1[p],
                               c * 64 * C * 2, 0, 0);
      for (int k = 0; wid_u + k * NW < UW2; ++k)
        ls_raw_buffer_load_lds(rs_w2, (__attribute__((address_space(3))) void*)(dst + WIMG + (wid_u + k * NW) * 64), 16,
                               vol + k * NW * 1024, c * W2IMG * 16, 0, 0);
    }
  };
  auto top = [&](int g) __attribute__((always_inline)) {  // chunk g's DMA landed everywhere; refill the other stage
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (g + 1 < 2 * NA + NCH) issue(g + 1, (g + 1) & 1);
    return (const uint4*)(lds + (g & 1) * STAGE);
  };
  issue(0, 0);

  const int p2 = lg ^ (((l16 >> 3) & 1) << 1);  // this lane's physical piece of a [C][32] image
  bf16x8 ar[FMR][KT];   // the B operand of the current phase: o rows, LN(h2), y
  f32x4 out[FMR][NT2];  // C^T accumulators: out[f][t][r] = column 16 t + 4 lg + r of row 16 f + l16
  auto init_cols = [&](const float* v) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const float4 b = *(const float4*)(v + 16 * t + 4 * lg);
#pragma unroll
      for (int f = 0; f < FMR; ++f) out[f][t] = (f32x4){b.x, b.y, b.z, b.w};
    }
  };
  // GEMM0 / GEMM3 over the NA stages of a [C][C] weight, operand ar (compile-time k-steps)
  auto proj = [&](int g0) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NA; ++q) {
      const uint4* cur = top(g0 + q);
      const int nk = (q + 1) * KPS <= KT ? KPS : KT - q * KPS;
      // per-image lane offsets, laundered so that the two projections' (same-valued) LDS
      // addresses are not shared across the FeedForward loop (kept live there, they spilled);
      // a tile's offset within an image is an instruction immediate
      int lo[KPS];
#pragma unroll
      for (int j = 0; j < KPS; ++j) {
        lo[j] = j * W2IMG + l16 * 4 + p2;
        asm volatile("" : "+v"(lo[j]));
      }
      uint4 wq[PD2];
#pragma unroll
      for (int i = 0; i < PD2; ++i) wq[i] = cur[lo[i / NT2] + (i % NT2) * 64];
#pragma unroll
      for (int j = 0; j < KPS; ++j) {
        if (j < nk) {
          const int k = q * KPS + j < KT ? q * KPS + j : 0;
#pragma unroll
          for (int t = 0; t < NT2; ++t) {
            const int i = j * NT2 + t;
            const bf16x8 wv = __builtin_bit_cast(bf16x8, wq[i % PD2]);
            const int n = i + PD2;
            if (n < nk * NT2) wq[i % PD2] = cur[lo[n / NT2 < KPS ? n / NT2 : 0] + (n % NT2) * 64];
#pragma unroll
            for (int f = 0; f < FMR; ++f)
              out[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, ar[f][k], out[f][t], 0, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);  // one k-step at a time: hoisted fragment reads spill
        }
      }
    }
  };
  // accumulators (bf16-rounded values) -> the operand registers in accumulator k order
  auto acc_to_operand = [&](int f, float mean, float rstd) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)((out[f][2 * s + (e >> 2)][e & 3] - mean) * rstd);
      ar[f][s] = v;
    }
  };

  // ---- phase A: h2 = o Wo^T + bo + h1 ----
#pragma unroll
  for (int f = 0; f < FMR; ++f) {
    const u16* src = a.o + (row0 + wr0 + 16 * f) * a.ldo + lg * 8;
#pragma unroll
    for (int s = 0; s < KT; ++s) ar[f][s] = *(const bf16x8*)(src + s * 32);
  }
  init_cols(a.bo);
  proj(0);
#pragma unroll
  for (int f = 0; f < FMR; ++f) {
    uint2 xr[NT2];
    const u16* hr = a.h1 + (row0 + wr0 + 16 * f) * a.ldh + 4 * lg;
#pragma unroll
    for (int t = 0; t < NT2; ++t) xr[t] = *(const uint2*)(hr + 16 * t);
    float s1 = 0.f;
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const uint2 rs = xr[t];
      const uint32_t pk0 = pack2(out[f][t][0] + __uint_as_float(rs.x << 16), out[f][t][1] + __uint_as_float(rs.x & 0xffff0000u));
      const uint32_t pk1 = pack2(out[f][t][2] + __uint_as_float(rs.y << 16), out[f][t][3] + __uint_as_float(rs.y & 0xffff0000u));
      out[f][t] = (f32x4){__uint_as_float(pk0 << 16), __uint_as_float(pk0 & 0xffff0000u),
                          __uint_as_float(pk1 << 16), __uint_as_float(pk1 & 0xffff0000u)};
      s1 += (out[f][t][0] + out[f][t][1]) + (out[f][t][2] + out[f][t][3]);
    }
    const float mean = xor16_32_sum(s1) * (1.0f / C);
    float s2 = 0.f;
#pragma unroll
    for (int t = 0; t < NT2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = out[f][t][r] - mean;
        s2 = fmaf(d, d, s2);
      }
    const float rstd = rsqrtf(xor16_32_sum(s2) * (1.0f / C) + a.eps);
    acc_to_operand(f, mean, rstd);  // LN(h2), gamma / beta folded into W1 / b1
  }
#pragma unroll
  for (int t = 0; t < NT2; ++t) {  // the FeedForward's accumulators start at its residual + b2
    const float4 b = *(const float4*)(a.b2 + 16 * t + 4 * lg);
#pragma unroll
    for (int f = 0; f < FMR; ++f) {
      out[f][t][0] += b.x; out[f][t][1] += b.y; out[f][t][2] += b.z; out[f][t][3] += b.w;
    }
  }

  // ---- phase B: the FeedForward ----
  // GELU of the chunk's 32 inner columns from the GEMM1 accumulators (biases from LDS)
  auto gelu_val = [&](f32x4 (&ac)[FMR][4], int c, int f, int hh, int r) __attribute__((always_inline)) {
    const float* bb = b1s + c * 64 + 32 * hh + 4 * lg;
    return (__bf16)((ac[f][2 * hh][r] + bb[r]) * gelu_erf(ac[f][2 * hh + 1][r] + bb[16 + r]));
  };
  if constexpr (FMR == 2) {
    // One wave per SIMD, software-pipelined: iteration c runs GEMM1 of chunk c + 1 with the
    // GELUs of chunk c between its MFMAs, then GEMM2 of chunk c -- a lone wave would
    // otherwise wait out every MFMA -> GELU -> MFMA dependency.  W1 of chunk c sits in W1
    // slot c & 1 (the first WIMG of stage c & 1), W2 of chunk c in W2 slot c & 1: W1 runs
    // one chunk ahead of W2, so at barrier T(c) W1(c + 2) refills the W1 slot GEMM1(c) left and
    // W2(c + 1) the W2 slot GEMM2(c - 1) left.  (Phase A's last barrier issued W1(0) + W2(0).)
    auto issue_w1 = [&](int c) __attribute__((always_inline)) {
      uint4* dst = lds + (c & 1) * STAGE;
#pragma unroll
      for (int p = 0; p < PW1; ++p) {
        const int q = p * NT + tid, r = (q >> 3) & 63, pc = q & 7;
        const int lc = pc ^ ((r >> 1) & 7);
        glds16(a.w1 + (long)(c * 64 + r) * C + (q >> 9) * 64 + lc * 8, dst + p * NT + wid * 64);
      }
    };
    auto issue_w2 = [&](int c) __attribute__((always_inline)) {
      uint4* dst = lds + (c & 1) * STAGE + WIMG;
      for (int u = wid; u < UW2; u += NW) glds16(a.w2 + ((long)c * W2IMG + u * 64 + lane) * 8, dst + u * 64);
    };
    auto bar = [&]() __attribute__((always_inline)) {
      wait_vm<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    // GEMM1 of chunk cn into nx; with GL the GELUs of chunk cn - 1 (from cu) between its k-steps
    auto gemm1 = [&](int cn, f32x4 (&nx)[FMR][4], f32x4 (&cu)[FMR][4], bf16x8 (&gv)[FMR], auto gl_tag)
        __attribute__((always_inline)) {
      constexpr bool GL = decltype(gl_tag)::value;
      const uint4* cur = lds + (cn & 1) * STAGE;
      auto frag = [&](int s, int t) {
        return __builtin_bit_cast(bf16x8, cur[(s >> 1) * 512 + swz_bk<64>(t * 16 + l16, (s & 1) * 4 + lg)]);
      };
#pragma unroll
      for (int f = 0; f < FMR; ++f)
#pragma unroll
        for (int t = 0; t < 4; ++t) nx[f][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
      bf16x8 wf[PD1][4];
#pragma unroll
      for (int p = 0; p < PD1; ++p)
#pragma unroll
        for (int t = 0; t < 4; ++t) wf[p][t] = frag(p, t);
#pragma unroll
      for (int s = 0; s < KT; ++s) {
        const int sl = s % PD1;
        bf16x8 cw[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) cw[t] = wf[sl][t];
        if (s + PD1 < KT) {
#pragma unroll
          for (int t = 0; t < 4; ++t) wf[sl][t] = frag(s + PD1, t);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int f = 0; f < FMR; ++f) nx[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[t], ar[f][s], nx[f][t], 0, 0, 0);
        if constexpr (GL) {  // two of the 16 GELUs (f, hh, r) per k-step
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int v = 2 * s + u;
            if (v < 8 * FMR) gv[v >> 3][v & 7] = gelu_val(cu, cn - 1, v >> 3, (v >> 2) & 1, v & 3);
          }
        }
      }
    };
    auto gemm2 = [&](int c, bf16x8 (&gv)[FMR]) __attribute__((always_inline)) {
      const uint4* w2 = lds + (c & 1) * STAGE + WIMG;
      uint4 w2q[PD2];
#pragma unroll
      for (int q = 0; q < PD2; ++q) w2q[q] = w2[(q * 16 + l16) * 4 + p2];
#pragma unroll
      for (int t = 0; t < NT2; ++t) {
        const bf16x8 wv = __builtin_bit_cast(bf16x8, w2q[t % PD2]);
        if (t + PD2 < NT2) w2q[t % PD2] = w2[((t + PD2) * 16 + l16) * 4 + p2];
#pragma unroll
        for (int f = 0; f < FMR; ++f) out[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, gv[f], out[f][t], 0, 0, 0);
      }
    };
    f32x4 accA[FMR][4], accB[FMR][4];
    bf16x8 gv[FMR];
    bar();  // T(-1): W1(0), W2(0) landed; phase A's stages are free
    issue_w1(1);
    gemm1(0, accA, accB, gv, std::false_type{});
    // iteration c: T(c) (W1(c + 1), W2(c) landed), issue W1(c + 2), W2(c + 1),
    // GEMM1(c + 1) with GELU(c), GEMM2(c)
    auto iter = [&](int c, f32x4 (&cu)[FMR][4], f32x4 (&nx)[FMR][4]) __attribute__((always_inline)) {
      bar();
      if (c + 2 < NCH) issue_w1(c + 2);
      if (c + 1 < NCH) issue_w2(c + 1);
      if (c + 1 < NCH) {
        gemm1(c + 1, nx, cu, gv, std::true_type{});
      } else {
#pragma unroll
        for (int v = 0; v < 8 * FMR; ++v) gv[v >> 3][v & 7] = gelu_val(cu, c, v >> 3, (v >> 2) & 1, v & 3);
      }
      gemm2(c, gv);
    };
    static_assert(NCH % 2 == 0, "ff_chain: an even chunk count");
    for (int c = 0; c < NCH; c += 2) {
      iter(c, accA, accB);
      iter(c + 1, accB, accA);
    }
    // phase C's first stage into stage 0 once every wave is done with the FeedForward's slots
    __syncthreads();
    issue(NA + NCH, (NA + NCH) & 1);
  } else {
    for (int c = 0; c < NCH; ++c) {
      const uint4* cur = top(NA + c);
      // (the GEGLU biases are added after GEMM1: loaded into the accumulators before it, their
      // LDS latency stood in front of the first MFMA -- 2623-2644 vs 2950-2970 us per call,
      // profiles/r06n_chain_variants.txt)
      f32x4 acc[FMR][4];
      const float* bb = b1s + c * 64 + 4 * lg;
  #pragma unroll
      for (int f = 0; f < FMR; ++f)
  #pragma unroll
        for (int t = 0; t < 4; ++t) acc[f][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
      auto frag = [&](int s, int t) {
        return __builtin_bit_cast(bf16x8, cur[(s >> 1) * 512 + swz_bk<64>(t * 16 + l16, (s & 1) * 4 + lg)]);
      };
      const uint4* w2 = cur + WIMG;
      bf16x8 wf[PD1][4];
  #pragma unroll
      for (int p = 0; p < PD1; ++p)
  #pragma unroll
        for (int t = 0; t < 4; ++t) wf[p][t] = frag(p, t);
      uint4 w2q[PD2];
  #pragma unroll
      for (int s = 0; s < KT; ++s) {
        const int sl = s % PD1;
        bf16x8 cw[4];
  #pragma unroll
        for (int t = 0; t < 4; ++t) cw[t] = wf[sl][t];
        if (s + PD1 < KT) {
  #pragma unroll
          for (int t = 0; t < 4; ++t) wf[sl][t] = frag(s + PD1, t);
        } else if (s + PD1 - KT < PD2) {
          w2q[s + PD1 - KT] = w2[((s + PD1 - KT) * 16 + l16) * 4 + p2];
        }
  #pragma unroll
        for (int t = 0; t < 4; ++t)
  #pragma unroll
          for (int f = 0; f < FMR; ++f) acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cw[t], ar[f][s], acc[f][t], 0, 0, 0);
      }
  #pragma unroll
      for (int q = PD1; q < PD2; ++q) w2q[q] = w2[(q * 16 + l16) * 4 + p2];
      bf16x8 gv[FMR];
  #pragma unroll
      for (int f = 0; f < FMR; ++f)
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          gv[f][r] = (__bf16)((acc[f][0][r] + bb[r]) * gelu_erf(acc[f][1][r] + bb[16 + r]));
          gv[f][4 + r] = (__bf16)((acc[f][2][r] + bb[32 + r]) * gelu_erf(acc[f][3][r] + bb[48 + r]));
        }
  #pragma unroll
      for (int t = 0; t < NT2; ++t) {
        const bf16x8 wv = __builtin_bit_cast(bf16x8, w2q[t % PD2]);
        if (t + PD2 < NT2) w2q[t % PD2] = w2[((t + PD2) * 16 + l16) * 4 + p2];
  #pragma unroll
        for (int f = 0; f < FMR; ++f) out[f][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, gv[f], out[f][t], 0, 0, 0);
      }
    }

  }

  // ---- phase C: z = y Wp^T + bp + xb ----
#pragma unroll
  for (int f = 0; f < FMR; ++f) acc_to_operand(f, 0.f, 1.f);  // y, rounded to bf16 as the unfused path stores it
  init_cols(a.bp);
  proj(NA + NCH);

  // ---- epilogue: + xb, the block's 128 x C result through LDS: row stores + column sums ----
  __syncthreads();  // every wave is past its last stage reads
  u16* zimg = (u16*)lds;
#pragma unroll
  for (int f = 0; f < FMR; ++f) {
    uint2 xr[NT2];
    const u16* src = a.xb + (row0 + wr0 + 16 * f) * a.ldxb + 4 * lg;
#pragma unroll
    for (int t = 0; t < NT2; ++t) xr[t] = *(const uint2*)(src + 16 * t);
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const uint2 rs = xr[t];
      const float o0 = out[f][t][0] + __uint_as_float(rs.x << 16), o1 = out[f][t][1] + __uint_as_float(rs.x & 0xffff0000u);
      const float o2 = out[f][t][2] + __uint_as_float(rs.y << 16), o3 = out[f][t][3] + __uint_as_float(rs.y & 0xffff0000u);
      *(uint2*)(zimg + (wr0 + 16 * f) * ZP + 16 * t + 4 * lg) = make_uint2(pack2(o0, o1), pack2(o2, o3));
    }
  }
  __syncthreads();
  constexpr int PCS = C / 8;  // 16-B pieces per row
  for (int q = tid; q < 128 * PCS; q += NT) {
    const int r = q / PCS, ch = q - r * PCS;
    *(uint4*)(a.z + (row0 + r) * a.ldz + ch * 8) = *(const uint4*)(zimg + r * ZP + ch * 8);
  }
  if (a.cs_out) {
    constexpr int RPG = 128 / RG;  // rows per group
    float* part = (float*)(zimg + 128 * ZP);  // [RG row groups][C / 4 quads][8]
    if (tid < RG * (C / 4)) {  // thread: columns 4 cq .. + 3 over rows RPG rg .. + RPG - 1
      const int cq = tid % (C / 4), rg = tid / (C / 4);
      float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < RPG; ++r) {
        const uint2 v = *(const uint2*)(zimg + (RPG * rg + r) * ZP + 4 * cq);
        const float fv[4] = {__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                             __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
#pragma unroll
        for (int e = 0; e < 4; ++e) { s1[e] += fv[e]; s2[e] = fmaf(fv[e], fv[e], s2[e]); }
      }
      float4* pp = (float4*)(part + (rg * (C / 4) + cq) * 8);
      pp[0] = make_float4(s1[0], s1[1], s1[2], s1[3]);
      pp[1] = make_float4(s2[0], s2[1], s2[2], s2[3]);
    }
    __syncthreads();
    for (int col = tid; col < C; col += NT) {
      const int cq = col >> 2, e = col & 3;
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        t1 += part[(rg * (C / 4) + cq) * 8 + e];
        t2 += part[(rg * (C / 4) + cq) * 8 + 4 + e];
      }
      a.cs_out[(long)blockIdx.x * 2 * C + col] = t1;
      a.cs_out[(long)blockIdx.x * 2 * C + C + col] = t2;
    }
  }
}

#ifdef LS_DIAG_KERNELS  // measured and rejected: diagnostics build only
// ff_pair_kernel (round 5, measured and rejected: 2630 vs 2460 us per call, step +3 ms,
// profiles/r05g_ff.txt, r05g_step_ab.txt -- the exchange barrier lines every wave up mid-chunk, and the
// two waves of a SIMD then run their GEMM1 / GELU / GEMM2 phases in step instead of beside
// each other): the same FeedForward with each W fragment read from LDS feeding TWO MFMAs.  ff_fused_kernel's waves own 16 rows, so every 1-KB W1 / W2 fragment it reads
// serves one 16x16x32 MFMA: 480 KB of LDS reads per chunk and CU against 1920 MFMA cycles
// per SIMD, and with the fragment-read -> MFMA dependency neither the matrix pipe (38 %
// busy) nor the LDS (40 %) is kept full (PMC, profiles/r05d_ff_pmc.txt).  Here a PAIR of
// waves owns 32 rows (two 16-row fragments, A in registers for both: 80 VGPRs) and splits
// the work by columns:
//   * GEMM1: wave h of the pair computes the h / g tiles of inner columns 16 h .. 16 h + 15
//     of the chunk (W1 tiles 2h, 2h + 1) for both row fragments: 20 fragment reads, 40 MFMAs;
//   * GEGLU -> 4 bf16 per lane and row fragment: inner columns 16 h + 4 lg .. + 3;
//   * the pair exchanges them through LDS (8 B per lane and row fragment), so each wave
//     holds GEMM2's full 32-wide B operand -- k-slots 4 lg .. + 3 from wave 0 and 16 + 4 lg
//     .. + 3 from wave 1, the order pack_ff_w2 already puts the W2 columns in;
//   * GEMM2: wave h accumulates output columns 160 h .. 160 h + 159 (10 tiles) for both row
//     fragments: 10 fragment reads, 20 MFMAs.
// 0.5 KB of LDS reads per MFMA instead of 1, the same MFMAs, GELUs and W DMA per row.  The
// exchange's barrier is also where W1 of chunk c + 2 is issued into the stage just read (as
// the W1 images of the stage just read).
template <int C, int I, int PD1 = 2, int PD2 = 6>
__global__ void __launch_bounds__(512, 1) ff_pair_kernel(FFArgs a) {
  constexpr int KT = C / 32;              // GEMM1 k-steps
  constexpr int NCH = I / 32;             // inner chunks
  constexpr int WIMG = 64 * (C / 64) * 8; // uint4: W1 chunk, C/64 images of [64 rows][8 pieces]
  constexpr int W2IMG = C * 4;            // uint4: W2 chunk, [C rows][4 pieces]
  constexpr int STAGE = WIMG + W2IMG;
  constexpr int NT2 = C / 32;             // output tiles per wave (half of C / 16)
  constexpr int PW1 = WIMG / 512;         // W1 pieces per thread per chunk
  constexpr int UW2 = W2IMG / 64;         // W2 wave-instructions per chunk
  static_assert(WIMG % 512 == 0 && W2IMG % 64 == 0 && C % 64 == 0 && I % 32 == 0, "ff_pair shape");
  static_assert(PD1 >= 1 && PD1 <= KT && PD2 >= PD1 && PD2 <= NT2, "prefetch depths");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // [2][STAGE], b1 (2I fp32), exchange
  float* b1s = (float*)(lds + 2 * STAGE);
  uint2* xch = (uint2*)(b1s + 2 * I);    // [4 pairs][2 halves][2 row fragments][64 lanes]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int pr = wid >> 1, h = wid & 1;  // pair, half
  const long row0 = (long)blockIdx.x * 128 + pr * 32 + l16;  // row of fragment 0 (fragment 1: + 16)

  for (int i = tid; i < 2 * I / 4; i += 512) ((float4*)b1s)[i] = ((const float4*)a.b1)[i];

  auto issue_w1 = [&](int c, int st) {
    uint4* dst = lds + st * STAGE;
#pragma unroll
    for (int p = 0; p < PW1; ++p) {
      const int q = p * 512 + tid, r = (q >> 3) & 63, pc = q & 7;
      const int lc = pc ^ ((r >> 1) & 7);
      glds16(a.w1 + (long)(c * 64 + r) * C + p * 64 + lc * 8, dst + p * 512 + wid * 64);
    }
  };
  auto issue_w2 = [&](int c, int st) {
    uint4* dst = lds + st * STAGE;
    for (int u = wid; u < UW2; u += 8) glds16(a.w2 + ((long)c * W2IMG + u * 64 + lane) * 8, dst + WIMG + u * 64);
  };
  issue_w1(0, 0);
  issue_w2(0, 0);

  // A rows of both fragments -> registers, LayerNorm in place
  bf16x8 ar[2][KT];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const long row = row0 + 16 * f;
    const bool live = row < a.M;
    const u16* src = a.x + (live ? row : 0) * a.ldx + lg * 8;
#pragma unroll
    for (int s = 0; s < KT; ++s)
      ar[f][s] = live ? *(const bf16x8*)(src + s * 32) : __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
    const float2 mr = live ? *(const float2*)(a.ln_mr + 2 * row) : make_float2(0.f, 0.f);
    const float rstd = mr.y, nmr = -mr.x * mr.y;
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      bf16x8 v = ar[f][s];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)fmaf((float)v[e], rstd, nmr);
      ar[f][s] = v;
    }
  }
  if (NCH > 1) issue_w1(1, 1);  // W1 runs a half chunk ahead of W2: refilled at the exchange barrier

  f32x4 out[NT2][2];
#pragma unroll
  for (int t = 0; t < NT2; ++t) out[t][0] = out[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int p2 = lg ^ (((l16 >> 3) & 1) << 1);  // this lane's physical W2 piece
  uint2* const xmine = xch + ((pr * 2 + h) * 2) * 64 + lane;
  const uint2* const xpart = xch + ((pr * 2 + (h ^ 1)) * 2) * 64 + lane;

  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) wait_vm<PW1>();  // W1 + W2 of chunk c landed; W1 of c + 1 may fly
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone's; the other stage's W2 (chunk c - 1) is no longer read
    asm volatile("" ::: "memory");
    if (c + 1 < NCH) issue_w2(c + 1, (c + 1) & 1);
    const uint4* cur = lds + (c & 1) * STAGE;

    // GEMM1: tiles 2h (h) and 2h + 1 (g) of the chunk, both row fragments
    f32x4 acc[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[t][0] = acc[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto frag = [&](int s, int t) {
      return __builtin_bit_cast(bf16x8, cur[(s >> 1) * 512 + swz_bk<64>((2 * h + t) * 16 + l16, (s & 1) * 4 + lg)]);
    };
    const uint4* w2 = cur + WIMG + (size_t)(h * NT2 * 16) * 4;  // this wave's 160 output rows of W2
    bf16x8 wf[PD1][2];
#pragma unroll
    for (int q = 0; q < PD1; ++q)
#pragma unroll
      for (int t = 0; t < 2; ++t) wf[q][t] = frag(q, t);
    uint4 w2q[PD2];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      const int sl = s % PD1;
      const bf16x8 c0 = wf[sl][0], c1 = wf[sl][1];
      if (s + PD1 < KT) {
        wf[sl][0] = frag(s + PD1, 0);
        wf[sl][1] = frag(s + PD1, 1);
      } else if (s + PD1 - KT < PD2) {
        w2q[s + PD1 - KT] = w2[((s + PD1 - KT) * 16 + l16) * 4 + p2];
      }
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        acc[0][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c0, ar[f][s], acc[0][f], 0, 0, 0);
        acc[1][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c1, ar[f][s], acc[1][f], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = PD1; q < PD2; ++q) w2q[q] = w2[(q * 16 + l16) * 4 + p2];
    // GEGLU of inner columns 16 h + 4 lg .. + 3 -> this wave's half of the B operand
    const float* bb = b1s + c * 64 + 32 * h + 4 * lg;
    const float4 bh = *(const float4*)(bb), bg = *(const float4*)(bb + 16);
    const float hb[4] = {bh.x, bh.y, bh.z, bh.w}, gb[4] = {bg.x, bg.y, bg.z, bg.w};
    uint2 mine[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      float g4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) g4[r] = (acc[0][f][r] + hb[r]) * gelu_erf(acc[1][f][r] + gb[r]);
      mine[f] = make_uint2(pack2(g4[0], g4[1]), pack2(g4[2], g4[3]));
      xmine[f * 64] = mine[f];
    }
    // the pair's exchange; every wave's GEMM1 reads of this stage's W1 images have retired too,
    // so they are refilled with chunk c + 2
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c + 2 < NCH) issue_w1(c + 2, c & 1);
    bf16x8 gv[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const uint2 other = xpart[f * 64];
      const uint4 q = h == 0 ? make_uint4(mine[f].x, mine[f].y, other.x, other.y)
                             : make_uint4(other.x, other.y, mine[f].x, mine[f].y);
      gv[f] = __builtin_bit_cast(bf16x8, q);
    }
    // GEMM2: out^T[160 h + 16 t + 4 lg + r][row] += W2[160 h + 16 t + l16][chunk k-slots] . G^T
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const bf16x8 wv = __builtin_bit_cast(bf16x8, w2q[t % PD2]);
      if (t + PD2 < NT2) w2q[t % PD2] = w2[((t + PD2) * 16 + l16) * 4 + p2];
      out[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, gv[0], out[t][0], 0, 0, 0);
      out[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, gv[1], out[t][1], 0, 0, 0);
    }
  }

  // y = out + b2 + x for this wave's 160 columns of both row fragments
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const long row = row0 + 16 * f;
    if (row >= a.M) continue;
    const u16* xr = a.x + row * a.ldx;
    u16* yr = a.y + row * a.ldy;
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
      const int col = C / 2 * h + 16 * t + 4 * lg;
      const float4 b = *(const float4*)(a.b2 + col);
      const uint2 rs = *(const uint2*)(xr + col);
      const float o0 = out[t][f][0] + b.x + __uint_as_float(rs.x << 16);
      const float o1 = out[t][f][1] + b.y + __uint_as_float(rs.x & 0xffff0000u);
      const float o2 = out[t][f][2] + b.z + __uint_as_float(rs.y << 16);
      const float o3 = out[t][f][3] + b.w + __uint_as_float(rs.y & 0xffff0000u);
      *(uint2*)(yr + col) = make_uint2(pack2(o0, o1), pack2(o2, o3));
    }
  }
}

#endif  // LS_DIAG_KERNELS

}  // namespace ls

using namespace ls;

// rows per wave of ls_ff_chain: 16 (1, the default) or, in the diagnostics build, 32 (2) --
// ls_set_tuning key 17.  Measured and rejected (profiles/r06c_kernel.txt, same box, M = 786432):
// 32 rows, one wave per SIMD 3058 us straight / 5120 us software-pipelined (AGPR traffic and
// scratch in the chunk loop) against 2695 us at 16 rows
int g_ff_chain_fmr = 1;

extern "C" int ls_ff_chain(const ls_ff_chain_desc* d, void* stream) {
  if (!d || !d->o || !d->wo || !d->bo || !d->h1 || !d->w1 || !d->b1 || !d->w2 || !d->b2 || !d->wp || !d->bp ||
      !d->xb || !d->z)
    return fail(LS_ERR_INVALID, "ls_ff_chain: null pointer");
  if (d->C != 320 || d->inner != 1280) return fail(LS_ERR_INVALID, "ls_ff_chain: C = 320, inner = 1280 only");
  if (d->M <= 0 || d->M % 128 || (d->M / 128) > 0x7fffffffL)
    return fail(LS_ERR_INVALID, "ls_ff_chain: M a positive multiple of 128");
  if (d->ldo < d->C || d->ldh < d->C || d->ldxb < d->C || d->ldz < d->C || d->ldo % 8 || d->ldh % 4 ||
      d->ldxb % 4 || d->ldz % 8)
    return fail(LS_ERR_INVALID, "ls_ff_chain: pitches >= C (o, z: % 8; h1, xb: % 4)");
  if ((((uintptr_t)d->o | (uintptr_t)d->wo | (uintptr_t)d->w1 | (uintptr_t)d->w2 | (uintptr_t)d->wp |
        (uintptr_t)d->b1 | (uintptr_t)d->b2 | (uintptr_t)d->bo | (uintptr_t)d->bp | (uintptr_t)d->z |
        (uintptr_t)d->cs_out) & 15) || (((uintptr_t)d->h1 | (uintptr_t)d->xb) & 7))
    return fail(LS_ERR_INVALID, "ls_ff_chain: operands 16-B aligned (h1 / xb 8-B)");
  FFChainArgs a;
  a.o = (const u16*)d->o; a.wo = (const u16*)d->wo; a.bo = d->bo; a.h1 = (const u16*)d->h1;
  a.w1 = (const u16*)d->w1; a.b1 = d->b1; a.w2 = (const u16*)d->w2; a.b2 = d->b2;
  a.wp = (const u16*)d->wp; a.bp = d->bp; a.xb = (const u16*)d->xb; a.z = (u16*)d->z; a.cs_out = d->cs_out;
  a.M = d->M; a.ldo = d->ldo; a.ldh = d->ldh; a.ldxb = d->ldxb; a.ldz = d->ldz; a.eps = d->eps;
  constexpr int C = 320, I = 1280;
  const size_t shm = (size_t)2 * (64 * (C / 64) * 8 + C * 4) * 16 + 2 * I * sizeof(float);
#ifdef LS_DIAG_KERNELS
  if (g_ff_chain_fmr == 2) {
    LS_SET_MAX_DYN_SHM((ff_chain_kernel<C, I, 2>), (int)shm);
    ff_chain_kernel<C, I, 2><<<(unsigned)(d->M / 128), 256, shm, (hipStream_t)stream>>>(a);
    return check_launch("ff_chain_kernel");
  }
#endif
  LS_SET_MAX_DYN_SHM((ff_chain_kernel<C, I, 1>), (int)shm);
  ff_chain_kernel<C, I, 1><<<(unsigned)(d->M / 128), 512, shm, (hipStream_t)stream>>>(a);
  return check_launch("ff_chain_kernel");
}

extern "C" int ls_feedforward(const ls_ff_desc* d, void* stream) {
  if (!d || !d->x || !d->ln_rowstats || !d->w1 || !d->b1 || !d->w2 || !d->b2 || !d->y)
    return fail(LS_ERR_INVALID, "ls_feedforward: null pointer");
  if (d->C != 320 || d->inner != 1280) return fail(LS_ERR_INVALID, "ls_feedforward: C = 320, inner = 1280 only");
  if (d->M <= 0 || d->ldx < d->C || d->ldy < d->C || d->ldx % 8 || d->ldy % 4)
    return fail(LS_ERR_INVALID, "ls_feedforward: bad rows / pitches (ldx % 8, ldy % 4, >= C)");
  if ((((uintptr_t)d->x | (uintptr_t)d->w1 | (uintptr_t)d->w2 | (uintptr_t)d->b1 | (uintptr_t)d->b2) & 15) ||
      (((uintptr_t)d->y | (uintptr_t)d->ln_rowstats) & 7))
    return fail(LS_ERR_INVALID, "ls_feedforward: x / w1 / w2 / b1 / b2 16-B aligned, y / ln_rowstats 8-B aligned");
  if ((d->M + 127) / 128 > 0x7fffffffL) return fail(LS_ERR_INVALID, "ls_feedforward: too many rows");
  FFArgs a;
  a.x = (const u16*)d->x; a.ln_mr = d->ln_rowstats; a.w1 = (const u16*)d->w1; a.b1 = d->b1;
  a.w2 = (const u16*)d->w2; a.b2 = d->b2; a.y = (u16*)d->y; a.M = d->M; a.ldx = d->ldx; a.ldy = d->ldy;
  constexpr int C = 320, I = 1280;
#ifdef LS_DIAG_KERNELS
  static const bool pair = ls_env("LS_FF_PAIR") != nullptr && atoi(ls_env("LS_FF_PAIR")) != 0;  // A/B switch
  if (pair) {
    const size_t shm = (size_t)2 * (64 * (C / 64) * 8 + C * 4) * 16 + 2 * I * sizeof(float) + 4 * 2 * 2 * 64 * 8;
    LS_SET_MAX_DYN_SHM((ff_pair_kernel<C, I>), (int)shm);
    ff_pair_kernel<C, I><<<(unsigned)((d->M + 127) / 128), 512, shm, (hipStream_t)stream>>>(a);
    return check_launch("ff_pair_kernel");
  }
#endif
  const size_t shm = (size_t)2 * (64 * (C / 64) * 8 + C * 4) * 16 + 2 * I * sizeof(float);
  LS_SET_MAX_DYN_SHM((ff_fused_kernel<C, I>), (int)shm);
  ff_fused_kernel<C, I><<<(unsigned)((d->M + 127) / 128), 512, shm, (hipStream_t)stream>>>(a);
  return check_launch("ff_fused_kernel");
}
