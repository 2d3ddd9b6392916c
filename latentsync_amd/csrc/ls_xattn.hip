// The audio cross-attention branch of BasicTransformerBlock at C = 320 in one gfx950
// launch (attention.py:174-199 norm2 + attn2; Attention.forward :250-280 with the
// Whisper chunk as encoder_hidden_states):
//
//   y = x + Wo softmax(Q K^T / sqrt(d)) V + bo,   Q = Wq LN(x) + bq,   8 heads x d = 40
//
// plus the LayerNorm row statistics of y (for norm3's fold into the FeedForward).  The
// three launches this replaces (the LN-folded q GEMM, the SDPA over the 50 audio tokens,
// the residual out-projection) moved q and o through HBM: at 48 windows 4 x 0.5 GB per
// call beside the 2 x 0.5 GB of x in / y out that remain.
//
// A workgroup owns 128 rows (8 waves x 16) of ONE image, so it shares that image's 50
// audio keys / values, staged once in LDS ([64 keys][C] each, keys >= L zero; row
// pitches chosen for conflict-free fragment reads: K 656 B (= 16 x odd: the 16 keys of
// a ds_read_b64 half land on distinct 16-B slots), V 672 B (= 32 x odd: the 8 keys of a
// ds_read_b64_tr_b16 half on distinct 32-B slots)).  A wave keeps its 16 rows of LN(x)
// in registers (40 VGPRs, as ff_fused) and walks the heads:
//   * q_h^T = Wq_h LN(x)^T + bq_h (16x16x32, Wq streamed per head through a 2-stage LDS
//     ring: [48 rows][C], rows 40..47 zero, LN gamma and log2(e)/sqrt(d) folded on the
//     host) -> a lane holds q dims 16t + 4lg + r of its row;
//   * those accumulators ARE the B operand of S^T = K_h q_h^T: k-step 0 takes dims
//     {4lg..+3, 16+4lg..+3}, k-step 1 dims {32+4lg..+3} (+ zeros), and the K fragment
//     reads the same dims (two 8-B reads per k-step);
//   * softmax over the 64 key slots (keys >= L masked) in registers + two cross-row
//     swaps; P is the B operand of O^T = V_h^T P^T (V^T by ds_read_b64_tr_b16), the row
//     sum taken from the same bf16 P;
//   * O / l -> bf16 -> the B operand of the out-projection: per head pair 3 k-steps
//     (each head's dims 0..31, then both heads' dims 32..39 side by side), i.e. 12 k-steps
//     (48 VGPRs) over all heads; the host permutes Wo's columns into that k-slot order
//     and zeroes the slots that carry padding.
// Then out^T = Wo o^T streams Wo in 32-column chunks through the same ring, and the
// epilogue adds bo and the residual, stores y (8 B per lane and tile) and accumulates
// the row statistics of the stored bf16 values (double across chunks, as the row-block
// GEMM's RB_STATS).
#include "ls_common.h"

typedef short v4i16 __attribute__((ext_vector_type(4)));

namespace ls {

struct XAArgs {
  const u16* x;         // [M][ldx] block input h (norm2 input and the residual)
  const float* ln_mr;   // [M][2] (mean, rstd) of x rows
  const u16* wq;        // [8][5][48][8] uint4 pieces: per head 5 k-images of [48 rows][8 x 16 B], swizzled
  const float* bq;      // [8][48]
  const u16* kv;        // [n_img * L] rows of k | v, pitch ldkv
  const u16* wo;        // [10][2][12][16][4] uint4 pieces (see packing.pack_xattn_wo)
  const float* bo;      // [320]
  u16* y;               // [M][ldy]
  float* stats_out;     // [M][2] (mean, rstd) of y, eps
  long M;
  int ldx, ldy, ldkv, L, hw;
  float eps;
};

constexpr int XA_C = 320, XA_H = 8, XA_KP = 328, XA_VP = 336;
constexpr int XA_WQIMG = 5 * 48 * 8;         // uint4 per head of Wq
constexpr int XA_WOIMG = 2 * 12 * 16 * 4;    // uint4 per 32-column chunk of Wo
constexpr int XA_SLOT = XA_WQIMG;            // ring slot (uint4), the larger of the two
constexpr size_t XA_SHM = (size_t)64 * XA_KP * 2 + (size_t)64 * XA_VP * 2 + (size_t)2 * XA_SLOT * 16;

__global__ void __launch_bounds__(512, 1) xattn_fused_kernel(XAArgs a) {
  constexpr int C = XA_C, KP = XA_KP, VP = XA_VP;
  static_assert(XA_WOIMG <= XA_SLOT, "ring slot");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  u16* Ks = (u16*)lds;                    // [64][KP]
  u16* Vs = Ks + 64 * KP;                 // [64][VP]
  uint4* ring = (uint4*)(Vs + 64 * VP);   // [2][XA_SLOT]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const long row0 = (long)blockIdx.x * 128;
  const long row = row0 + wid * 16 + l16;
  const bool live = row < a.M;
  const long img = row0 / a.hw;

  // ring items: 0..7 = Wq of head h, 8..17 = Wo chunk c - 8; item i goes to slot i & 1
  auto issue = [&](int item) {
    uint4* dst = ring + (item & 1) * XA_SLOT;
    if (item < 8) {
      const u16* src = a.wq + (long)item * XA_WQIMG * 8;
      for (int q = tid; q < XA_WQIMG; q += 512) glds16(src + q * 8, dst + q);
    } else {
      const u16* src = a.wo + (long)(item - 8) * XA_WOIMG * 8;
      for (int q = tid; q < XA_WOIMG; q += 512) glds16(src + q * 8, dst + q);
    }
  };
  issue(0);

  // the image's keys / values -> LDS (register-staged: the padded rows and the zero
  // keys >= L are written in the same pass)
  for (int q = tid; q < 64 * 83; q += 512) {
    const int r = q / 83, pc = q - r * 83;
    const bool isv = pc >= 41;
    const int c = isv ? pc - 41 : pc;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < a.L && c < 40) v = *(const uint4*)(a.kv + (img * a.L + r) * a.ldkv + (isv ? C : 0) + c * 8);
    if (isv) *(uint4*)(Vs + r * VP + c * 8) = v;
    else *(uint4*)(Ks + r * KP + c * 8) = v;
  }

  // LN(x) rows -> registers (B operand of the q projection: lane holds k 32s + 8lg .. +8)
  bf16x8 ar[10];
  {
    const u16* src = a.x + (live ? row : 0) * a.ldx + lg * 8;
#pragma unroll
    for (int s = 0; s < 10; ++s)
      ar[s] = live ? *(const bf16x8*)(src + s * 32) : __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
    const float2 mr = live ? *(const float2*)(a.ln_mr + 2 * row) : make_float2(0.f, 0.f);
    const float rstd = mr.y, nmr = -mr.x * mr.y;
#pragma unroll
    for (int s = 0; s < 10; ++s) {
      bf16x8 v = ar[s];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (__bf16)fmaf((float)v[e], rstd, nmr);
      ar[s] = v;
    }
  }

  auto sync = [&]() {
    wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  bf16x8 ofr[12];  // o^T B operand of the out-projection, k-steps 3j + {0, 1, 2}
  const int qq = l16 >> 2, pp = l16 & 3;
#pragma unroll 1
  for (int h = 0; h < 8; ++h) {
    sync();  // Wq_h landed for everyone; the other slot (and at h = 0: K / V) free / written
    issue(h + 1);
    const uint4* w = ring + (h & 1) * XA_SLOT;
    // q_h^T: 3 tiles of 16 dims x 10 k-steps
    f32x4 qa[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) qa[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 10; ++s)
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const bf16x8 wf = __builtin_bit_cast(bf16x8, w[(s >> 1) * 384 + swz_bk<64>(t * 16 + l16, (s & 1) * 4 + lg)]);
        qa[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, ar[s], qa[t], 0, 0, 0);
      }
    bf16x8 qk0, qk1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float* bq = a.bq + h * 48 + 4 * lg + r;
      qk0[r] = (__bf16)(qa[0][r] + bq[0]);
      qk0[4 + r] = (__bf16)(qa[1][r] + bq[16]);
      qk1[r] = (__bf16)(qa[2][r] + bq[32]);
      qk1[4 + r] = (__bf16)0.f;
    }
    // S^T = K_h q_h^T over 4 tiles of 16 key slots: s[f][r] = key 16f + 4lg + r
    f32x4 s[4];
    const u16* kh = Ks + 40 * h + 4 * lg;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const u16* kr = kh + (16 * f + l16) * KP;
      const uint2 k0 = *(const uint2*)kr, k1 = *(const uint2*)(kr + 16), k2 = *(const uint2*)(kr + 32);
      const bf16x8 ka = __builtin_bit_cast(bf16x8, make_uint4(k0.x, k0.y, k1.x, k1.y));
      const bf16x8 kb = __builtin_bit_cast(bf16x8, make_uint4(k2.x, k2.y, 0u, 0u));
      s[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qk0, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      s[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kb, qk1, s[f], 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (16 * f + 4 * lg + r >= a.L) s[f][r] = -INFINITY;
        mx = __builtin_elementwise_maximum(mx, s[f][r]);
      }
    mx = xor16_32_max(mx);
    bf16x8 pb[2];
    float ps = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const __bf16 p0 = (__bf16)fast_exp2(s[2 * c][r] - mx), p1 = (__bf16)fast_exp2(s[2 * c + 1][r] - mx);
        pb[c][r] = p0;
        pb[c][4 + r] = p1;
        ps += (float)p0 + (float)p1;  // the denominator sums the bf16 P that P V consumes
      }
    const float inv = 1.f / xor16_32_sum(ps);
    // O^T = V_h^T P^T: 3 tiles of 16 dims x 2 steps of 32 keys
    f32x4 o[3];
#pragma unroll
    for (int nd = 0; nd < 3; ++nd) {
      o[nd] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const u16* va = Vs + (32 * c + 4 * lg + qq) * VP + 40 * h + 16 * nd + 4 * pp;
        const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)va);
        const v4i16 hi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(va + 16 * VP));
        const short __attribute__((ext_vector_type(8))) av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av), pb[c], o[nd], 0, 0, 0);
      }
    }
    // O / l -> the out-projection's B operand (k-step order of packing.pack_xattn_wo)
    const int ja = 3 * (h >> 1) + (h & 1), jb = 3 * (h >> 1) + 2, eb = (h & 1) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ofr[ja][r] = (__bf16)(o[0][r] * inv);
      ofr[ja][4 + r] = (__bf16)(o[1][r] * inv);
      ofr[jb][eb + r] = (__bf16)(o[2][r] * inv);
    }
  }

  // out^T = Wo o^T in 10 chunks of 32 columns, + bo + residual; row statistics of y
  double S1 = 0.0, S2 = 0.0;
  const int p2 = lg ^ (((l16 >> 3) & 1) << 1);  // this lane's physical Wo piece
  const u16* xr = a.x + (live ? row : 0) * a.ldx;
  u16* yr = a.y + (live ? row : 0) * a.ldy;
#pragma unroll 1
  for (int c = 0; c < 10; ++c) {
    const int item = 8 + c;
    sync();
    if (c < 9) issue(item + 1);
    const uint4* w = ring + (item & 1) * XA_SLOT;
    uint2 rs[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) rs[t] = live ? *(const uint2*)(xr + 32 * c + 16 * t + 4 * lg) : make_uint2(0, 0);
    f32x4 acc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 12; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16x8 wf = __builtin_bit_cast(bf16x8, w[((t * 12 + ks) * 16 + l16) * 4 + p2]);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, ofr[ks], acc[t], 0, 0, 0);
      }
    float c1 = 0.f, c2 = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int col = 32 * c + 16 * t + 4 * lg;
      const float4 b = *(const float4*)(a.bo + col);
      const float y0 = acc[t][0] + b.x + __uint_as_float(rs[t].x << 16);
      const float y1 = acc[t][1] + b.y + __uint_as_float(rs[t].x & 0xffff0000u);
      const float y2 = acc[t][2] + b.z + __uint_as_float(rs[t].y << 16);
      const float y3 = acc[t][3] + b.w + __uint_as_float(rs[t].y & 0xffff0000u);
      const uint2 pk = make_uint2(pack2(y0, y1), pack2(y2, y3));
      if (live) *(uint2*)(yr + col) = pk;
      const float b0 = __uint_as_float(pk.x << 16), b1 = __uint_as_float(pk.x & 0xffff0000u);
      const float b2 = __uint_as_float(pk.y << 16), b3 = __uint_as_float(pk.y & 0xffff0000u);
      c1 += (b0 + b1) + (b2 + b3);
      c2 = fmaf(b0, b0, fmaf(b1, b1, fmaf(b2, b2, fmaf(b3, b3, c2))));
    }
    S1 += (double)c1;
    S2 += (double)c2;
  }
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    S1 += __shfl_xor(S1, o, 64);
    S2 += __shfl_xor(S2, o, 64);
  }
  if (lg == 0 && live) {
    const double mean = S1 / C, var = fmax(S2 / C - mean * mean, 0.0);
    *(float2*)(a.stats_out + 2 * row) = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)a.eps)));
  }
}

}  // namespace ls

using namespace ls;

extern "C" int ls_cross_attention_block(const ls_xattn_desc* d, void* stream) {
  if (!d || !d->x || !d->ln_rowstats || !d->wq || !d->bq || !d->kv || !d->wo || !d->bo || !d->y || !d->stats_out)
    return fail(LS_ERR_INVALID, "ls_cross_attention_block: null pointer");
  if (d->C != XA_C || d->heads != XA_H)
    return fail(LS_ERR_INVALID, "ls_cross_attention_block: C = 320, 8 heads only");
  if (d->L < 1 || d->L > 64) return fail(LS_ERR_INVALID, "ls_cross_attention_block: 1..64 audio tokens");
  if (d->M <= 0 || d->hw <= 0 || d->hw % 128 || d->M % d->hw)
    return fail(LS_ERR_INVALID, "ls_cross_attention_block: M a multiple of hw, hw a multiple of 128");
  if (d->ldx < XA_C || d->ldy < XA_C || d->ldx % 8 || d->ldy % 4 || d->ldkv < 2 * XA_C || d->ldkv % 8)
    return fail(LS_ERR_INVALID, "ls_cross_attention_block: pitches (ldx % 8, ldy % 4, ldkv % 8)");
  if ((((uintptr_t)d->x | (uintptr_t)d->wq | (uintptr_t)d->wo | (uintptr_t)d->kv | (uintptr_t)d->bo) & 15) ||
      (((uintptr_t)d->y | (uintptr_t)d->ln_rowstats | (uintptr_t)d->stats_out | (uintptr_t)d->bq) & 7))
    return fail(LS_ERR_INVALID, "ls_cross_attention_block: alignment (x, wq, wo, kv, bo 16 B; y, stats 8 B)");
  if (d->M / 128 > 0x7fffffffL) return fail(LS_ERR_INVALID, "ls_cross_attention_block: too many rows");
  XAArgs a;
  a.x = (const u16*)d->x; a.ln_mr = d->ln_rowstats; a.wq = (const u16*)d->wq; a.bq = d->bq;
  a.kv = (const u16*)d->kv; a.wo = (const u16*)d->wo; a.bo = d->bo; a.y = (u16*)d->y; a.stats_out = d->stats_out;
  a.M = d->M; a.ldx = d->ldx; a.ldy = d->ldy; a.ldkv = d->ldkv; a.L = d->L; a.hw = d->hw; a.eps = d->eps;
  LS_SET_MAX_DYN_SHM(xattn_fused_kernel, XA_SHM);
  xattn_fused_kernel<<<(unsigned)(d->M / 128), 512, XA_SHM, (hipStream_t)stream>>>(a);
  return check_launch("xattn_fused_kernel");
}
