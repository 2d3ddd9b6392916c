// Flash-style multi-head attention for gfx950 (bf16 MFMA 16x16x32, fp32 online
// softmax).
//
// Each wave owns 16 queries of one (batch, head); the waves of a block share the
// K/V tiles staged in LDS.  The score tile is computed TRANSPOSED, S^T = K Q^T
// (A = K rows from LDS via ds_read_b128, B = Q^T held in registers), so the
// accumulator has the key on the register/row axis and the query on the lane.
// That makes (a) the softmax max/sum per query a 4-register + 2-shuffle
// reduction, and (b) the probabilities already the B operand of the next MFMA,
// O^T = V^T P^T, with no LDS round trip: the MFMA's k index is permuted
// identically on both operands (keys 32c+4h+j and 32c+16+4h+j for lane group h),
// and V^T comes from the row-major V tile through ds_read_b64_tr_b16.
//
// Kernels (dispatch in ls_attention):
//   attn_seqm_kernel short sequences (the temporal attention over a window's frames), MFMA
//                    (d = 80 / 160: a sequence's heads split over two blocks)
//   attn_seq_kernel  the same with packed-bf16 dot products (d = 160, A/B baseline)
//   attn5_kernel     d = 40 self attention: DMA-fed K/V planes, 64 queries per wave
//   attn3_kernel     other long sequences (register-staged K/V tiles)
//   attn_kernel      everything else (nk <= 32, d > 160: the VAE mid attention)
// attn3/attn5 share the softmax scheme: Q pre-scaled to log2 units, the running max
// subtracted by the MFMA's C operand, lazy rescaling, bf16 P.
#include <type_traits>

#include "ls_common.h"

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef int v8i32 __attribute__((ext_vector_type(8)));

namespace ls {

struct AttnArgs {
  const u16* q; const u16* k; const u16* v; u16* o;
  long q_sb1, q_sb2, q_si, q_sh;
  long k_sb1, k_sb2, k_si, k_sh;
  long v_sb1, v_sb2, v_si, v_sh;
  long o_sb1, o_sb2, o_si, o_sh;
  int z2, nq, nk, D;
  float scale_log2;
  int o16;  // o rows and head slices 16-B aligned: epilogues may store 8 dims per lane
};

// up to 8 bf16 from a possibly unaligned address, zero beyond `n`
__device__ __forceinline__ uint4 load_partial(const u16* p, int n) {
  u16 e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = j < n ? p[j] : (u16)0;
  return make_uint4(e[0] | (uint32_t)e[1] << 16, e[2] | (uint32_t)e[3] << 16, e[4] | (uint32_t)e[5] << 16,
                    e[6] | (uint32_t)e[7] << 16);
}

template <int DP, int NKF>
__global__ void __launch_bounds__(256) attn_kernel(AttnArgs a) {
  constexpr int KC = DP / 32;   // 32-wide d chunks (QK^T k-steps)
  constexpr int ND = DP / 16;   // 16-row O^T fragments
  constexpr int KT = 16 * NKF;  // keys per tile
  constexpr int PITCH = DP + 8; // LDS row pitch (elements), 16-B aligned
  extern __shared__ __attribute__((aligned(16))) u16 sm[];
  u16* Ks = sm;
  u16* Vs = sm + KT * PITCH;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = blockDim.x >> 6;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const long b1 = b / a.z2, b2 = b - b1 * a.z2;
  const u16* qb = a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)h * a.q_sh;
  const u16* kb = a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + (long)h * a.k_sh;
  const u16* vb = a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + (long)h * a.v_sh;
  u16* ob = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)h * a.o_sh;
  const int q0 = (blockIdx.x * nw + wid) * 16;
  const int lq = lane & 15, lg = lane >> 4;

  // Q^T fragments (B operand): lane holds Q[q0+lq][32kc + 8lg .. +8]
  bf16x8 qf[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    const int d = kc * 32 + lg * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (q0 + lq < a.nq && d < a.D) {
      const u16* src = qb + (long)(q0 + lq) * a.q_si + d;
      if ((a.D & 7) == 0) v = *(const uint4*)src;
      else v = load_partial(src, a.D - d);
    }
    qf[kc] = __builtin_bit_cast(bf16x8, v);
  }

  f32x4 oacc[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) oacc[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  const int cpr = DP / 8;  // 16-B chunks per row
  for (int t0 = 0; t0 < a.nk; t0 += KT) {
    __syncthreads();
    for (int i = tid; i < KT * cpr; i += blockDim.x) {
      const int r = i / cpr, c = (i - r * cpr) * 8;
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (t0 + r < a.nk && c < a.D) {
        if ((a.D & 7) == 0) {
          kv = *(const uint4*)(kb + (long)(t0 + r) * a.k_si + c);
          vv = *(const uint4*)(vb + (long)(t0 + r) * a.v_si + c);
        } else {  // head_dim not a multiple of 8 (reduced-width test configs)
          kv = load_partial(kb + (long)(t0 + r) * a.k_si + c, a.D - c);
          vv = load_partial(vb + (long)(t0 + r) * a.v_si + c, a.D - c);
        }
      }
      *(uint4*)(Ks + r * PITCH + c) = kv;
      *(uint4*)(Vs + r * PITCH + c) = vv;
    }
    __syncthreads();

    // S^T = K Q^T : s[f][r] = score(key t0 + 16f + 4lg + r, query q0 + lq)
    f32x4 s[NKF];
#pragma unroll
    for (int f = 0; f < NKF; ++f) {
      s[f] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const bf16x8 kf = __builtin_bit_cast(bf16x8, *(const uint4*)(Ks + (16 * f + lq) * PITCH + kc * 32 + lg * 8));
        s[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kc], s[f], 0, 0, 0);
      }
    }
    float mt = -INFINITY;
#pragma unroll
    for (int f = 0; f < NKF; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = t0 + 16 * f + 4 * lg + r;
        const float x = key < a.nk ? s[f][r] * a.scale_log2 : -INFINITY;
        s[f][r] = x;
        mt = fmaxf(mt, x);
      }
    mt = fmaxf(mt, __shfl_xor(mt, 16, 64));
    mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
    const float mn = fmaxf(m, mt);
    const float alpha = fast_exp2(m - mn);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int f = 0; f < NKF; ++f)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = fast_exp2(s[f][r] - mn);
        s[f][r] = p;
        ps += p;
      }
    l = l * alpha + ps;
#pragma unroll
    for (int i = 0; i < ND; ++i) oacc[i] *= alpha;

    // O^T += V^T P^T over 32-key chunks
#pragma unroll
    for (int c = 0; c < NKF / 2; ++c) {
      bf16x8 pb;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pb[r] = (__bf16)s[2 * c][r];
        pb[4 + r] = (__bf16)s[2 * c + 1][r];
      }
      const int qq = lq >> 2, pp = lq & 3;
      const u16* va = Vs + (32 * c + 4 * lg + qq) * PITCH + 4 * pp;
      const u16* vb2 = va + 16 * PITCH;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4i16*)(va + nd * 16));
        const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4i16*)(vb2 + nd * 16));
        const short __attribute__((ext_vector_type(8))) av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        oacc[nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av), pb, oacc[nd], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  const int q = q0 + lq;
  if (q < a.nq) {
    u16* orow = ob + (long)q * a.o_si;
#pragma unroll
    for (int nd = 0; nd < ND; ++nd)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = nd * 16 + 4 * lg + r;
        if (d < a.D) orow[d] = f2bf(oacc[nd][r] * inv);
      }
  }
}

// attn3: long-sequence flash attention (nk > 32).  Every wave owns 32 queries (two Q
// fragments share each K/V fragment read), 64-key tiles double-buffered in LDS with
// the next tile's global loads issued into registers before the current tile's
// MFMAs (one barrier per tile), QK^T over KC 32-wide d chunks, PV over ND = ceil(D/16)
// output fragments (d = 40 pays 48, not 64).  The softmax costs ~2 VALU instructions
// per score (round 1's kernel spent ~215 VALU instructions per 64-key tile at d = 40
// against 28 MFMAs):
//   * Q is pre-scaled by scale*log2(e) once (bf16), so a score leaves the MFMA in
//     log2 units;
//   * the running max m is SUBTRACTED BY THE MFMA: the first QK^T step of every
//     fragment accumulates onto C = -m (a 4-register splat), so p = exp2(s) with no
//     FMA per score;
//   * lazy rescaling: m is only moved (and O, l rescaled) when a tile's max exceeds
//     it by more than TAU = 10 (p <= 2^10 is exact enough in bf16/fp32); the check
//     is one wave-uniform ballot per tile, the rescale path is rare after tile 0;
//   * DSUM = D with D % 16 != 0 (d = 40): the row sum l comes out of the PV MFMA --
//     V's padding column D is set to 1.0 once, so O^T row D accumulates sum_k p_k
//     (of the same bf16 p the numerator uses) and the 16 adds per score row go away.
// ONE: the key set fits one 64-key tile (the 50 audio tokens, the 8x8 / 4x4 levels' self
// attention): a single LDS stage and no prefetch registers, so d = 160 runs two blocks per CU.
// With a 16-B aligned o the epilogue stores 8 dims per lane (fragment pairs swapped across
// lane groups): 253 -> 233 us for the audio cross attention at d = 40, 252 -> 242 us for the
// 16x16-level self attention at d = 80 (32 windows).
template <int KC, int ND, int DSUM, bool ONE = false>
__global__ void __launch_bounds__(256, (KC >= 5 && !ONE) ? 1 : 2) attn3_kernel(AttnArgs a) {
  constexpr int DP = KC * 32;
  constexpr int KT = 64;
  constexpr int PITCH = DP + 8;
  constexpr int TILE = KT * PITCH;
  constexpr int CPR = ND * 2;
  constexpr int LPT = (KT * CPR + 255) / 256;
  constexpr float TAU = 10.f;
  static_assert(DSUM == 0 || (DSUM % 8 == 0 && DSUM < 16 * ND), "sum column must be a padding column");
  extern __shared__ __attribute__((aligned(16))) u16 sm[];  // [2][K, V]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = blockIdx.y;
  const int b = blockIdx.z;
  const long b1 = b / a.z2, b2 = b - b1 * a.z2;
  const u16* qb = a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)h * a.q_sh;
  const u16* kb = a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + (long)h * a.k_sh;
  const u16* vb = a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + (long)h * a.v_sh;
  u16* ob = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)h * a.o_sh;
  const int q0 = (blockIdx.x * 4 + wid) * 32;
  const int lq = lane & 15, lg = lane >> 4;
  const int cpr = (a.D + 7) >> 3;

  // K d-padding zeroed in both buffers; with DSUM, V[:, DSUM] = 1 and the rest of the
  // padding 0 (the per-tile stores never touch chunks >= cpr)
  for (int i = tid; i < (ONE ? 1 : 2) * KT; i += 256) {
    u16* krow = sm + (i / KT) * 2 * TILE + (i % KT) * PITCH;
    for (int c = cpr * 8; c < DP; c += 8) *(uint4*)(krow + c) = make_uint4(0, 0, 0, 0);
    if (DSUM) {
      u16* vrow = krow + TILE;
      for (int c = cpr * 8; c < 16 * ND; c += 8)
        *(uint4*)(vrow + c) = make_uint4(c == DSUM ? 0x3F80u : 0u, 0, 0, 0);
    }
  }

  const float c2 = a.scale_log2;
  bf16x8 qf[2][KC];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int d = kc * 32 + lg * 8;
      const int q = q0 + g * 16 + lq;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (q < a.nq && d < a.D) v = *(const uint4*)(qb + (long)q * a.q_si + d);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= c2;
      qf[g][kc] = __builtin_bit_cast(bf16x8, pack8(f));
    }

  uint4 kr[LPT], vr[LPT];
  auto gload = [&](int t0) {
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int i = tid + u * 256;
      const int r = i / CPR, c = i - r * CPR;
      kr[u] = make_uint4(0, 0, 0, 0);
      vr[u] = make_uint4(0, 0, 0, 0);
      if (i < KT * CPR && c < cpr && t0 + r < a.nk) {
        kr[u] = *(const uint4*)(kb + (long)(t0 + r) * a.k_si + c * 8);
        vr[u] = *(const uint4*)(vb + (long)(t0 + r) * a.v_si + c * 8);
      }
    }
  };
  auto lstore = [&](int buf) {
    u16* Ks = sm + buf * 2 * TILE;
    u16* Vs = Ks + TILE;
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
      const int i = tid + u * 256;
      const int r = i / CPR, c = i - r * CPR;
      if (i < KT * CPR && c < cpr) {
        *(uint4*)(Ks + r * PITCH + c * 8) = kr[u];
        *(uint4*)(Vs + r * PITCH + c * 8) = vr[u];
      }
    }
  };

  f32x4 oacc[2][ND];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int i = 0; i < ND; ++i) oacc[g][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[2] = {0.f, 0.f}, l[2] = {0.f, 0.f};
  f32x4 negm[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};

  gload(0);
  __syncthreads();  // padding written
  lstore(0);
  const int ntile = (a.nk + KT - 1) / KT;
  auto tile = [&](int t, auto partial_tag) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    const int t0 = t * KT;
    __syncthreads();
    if (!ONE && t + 1 < ntile) gload(t0 + KT);
    const u16* Ks = sm + (t & 1) * 2 * TILE;
    const u16* Vs = Ks + TILE;
    // S^T - m = K Q^T + (-m): scores relative to the running max, log2 units
    f32x4 s[2][4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const bf16x8 kf = __builtin_bit_cast(bf16x8, *(const uint4*)(Ks + (16 * f + lq) * PITCH + kc * 32 + lg * 8));
        s[0][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[0][kc], kc == 0 ? negm[0] : s[0][f], 0, 0, 0);
        s[1][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[1][kc], kc == 0 ? negm[1] : s[1][f], 0, 0, 0);
      }
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (PARTIAL) {
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t0 + 16 * f + 4 * lg + r >= a.nk) s[g][f][r] = -INFINITY;
      }
      float mt = __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][0][0], s[g][0][1]),
                                               __builtin_elementwise_maximum(s[g][0][2], s[g][0][3]));
#pragma unroll
      for (int f = 1; f < 4; ++f)
        mt = __builtin_elementwise_maximum(
            mt, __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][f][0], s[g][f][1]),
                                              __builtin_elementwise_maximum(s[g][f][2], s[g][f][3])));
      mt = xor16_32_max(mt);
      // move the reference max only when needed (always on the first tile, which
      // starts from m = 0 with nothing accumulated)
      const bool need = t == 0 || mt > TAU;
      if (__builtin_amdgcn_ballot_w64(need)) {
        const float dlt = need ? mt : 0.f;
        const float alpha = t == 0 ? 0.f : fast_exp2(-dlt);
        m[g] += dlt;
        negm[g] = (f32x4){-m[g], -m[g], -m[g], -m[g]};
#pragma unroll
        for (int f = 0; f < 4; ++f) s[g][f] -= dlt;
#pragma unroll
        for (int i = 0; i < ND; ++i) oacc[g][i] *= alpha;
        l[g] *= alpha;
      }
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[g][f][r] = fast_exp2(s[g][f][r]);
      if (!DSUM) {
        float ps = 0.f;
#pragma unroll
        for (int f = 0; f < 4; ++f) ps += (s[g][f][0] + s[g][f][1]) + (s[g][f][2] + s[g][f][3]);
        l[g] += ps;
      }
    }
    // O^T += V^T P^T over 32-key chunks
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8 pb[2];
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pb[g][r] = (__bf16)s[g][2 * c][r];
          pb[g][4 + r] = (__bf16)s[g][2 * c + 1][r];
        }
      const int qq = lq >> 2, pp = lq & 3;
      const u16* va = Vs + (32 * c + 4 * lg + qq) * PITCH + 4 * pp;
      const u16* vb2 = va + 16 * PITCH;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(va + nd * 16));
        const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(vb2 + nd * 16));
        const short __attribute__((ext_vector_type(8))) av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 vf = __builtin_bit_cast(bf16x8, av);
        oacc[0][nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[0], oacc[0][nd], 0, 0, 0);
        oacc[1][nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[1], oacc[1][nd], 0, 0, 0);
      }
    }
    if (!ONE && t + 1 < ntile) lstore((t + 1) & 1);
  };
  const int nfull = a.nk / KT;
  for (int t = 0; t < nfull; ++t) tile(t, std::false_type{});
  if (nfull < ntile) tile(nfull, std::true_type{});
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float lt;
    if (DSUM) {
      // O^T row DSUM (fragment DSUM/16, lane group (DSUM%16)/4, register DSUM%4) holds l
      constexpr int NDL = DSUM / 16, LGL = (DSUM % 16) / 4, RL = DSUM % 4;
      lt = __shfl(oacc[g][NDL][RL], LGL * 16 + lq, 64);
    } else {
      lt = xor16_32_sum(l[g]);
    }
    const float inv = 1.f / lt;
    const int q = q0 + g * 16 + lq;
    if (a.o16 && a.D % 8 == 0) {
      // 16-B stores: fragments 2p, 2p+1 trade halves across lane groups (as attn_seqm)
      uint2 w[ND + 1];
#pragma unroll
      for (int nd = 0; nd < ND; ++nd)
        w[nd] = make_uint2(pack2(oacc[g][nd][0] * inv, oacc[g][nd][1] * inv),
                           pack2(oacc[g][nd][2] * inv, oacc[g][nd][3] * inv));
      w[ND] = make_uint2(0, 0);
      u16* orow = ob + (long)(q < a.nq ? q : 0) * a.o_si;
#pragma unroll
      for (int p = 0; p < (ND + 1) / 2; ++p) {
        const auto rx = __builtin_amdgcn_permlane16_swap(w[2 * p].x, w[2 * p + 1].x, false, false);
        const auto ry = __builtin_amdgcn_permlane16_swap(w[2 * p].y, w[2 * p + 1].y, false, false);
        const int d = 32 * p + 16 * (lg & 1) + 4 * (lg & 2);
        if (q < a.nq && d < a.D) *(uint4*)(orow + d) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
      }
    } else if (q < a.nq) {
      u16* orow = ob + (long)q * a.o_si;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        const int d = nd * 16 + 4 * lg;
        if (d + 3 < a.D) {
          uint2 w;
          w.x = pack2(oacc[g][nd][0] * inv, oacc[g][nd][1] * inv);
          w.y = pack2(oacc[g][nd][2] * inv, oacc[g][nd][3] * inv);
          *(uint2*)(orow + d) = w;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (d + r < a.D) orow[d + r] = f2bf(oacc[g][nd][r] * inv);
        }
      }
    }
  }
}

// attn5: attn3's arithmetic with the K/V tiles moved by buffer_load ... lds DMA.
// attn3's register-staged tile copy cost ~60 VALU per tile (64-bit address math,
// exec-masked tails, ds_writes) beside the softmax, and its 144-B-pitch image had
// 2-way bank conflicts.  Here every K/V tile is stored "chunk-plane major": plane c
// holds the 16-B chunk c (head dims 8c .. 8c+7) of the tile's 64 keys, one
// wave-instruction of DMA per plane (lane = key).  The per-lane byte offset
// (key * row stride + 16 c) is fixed for the whole kernel and the tile advances
// through the uniform soffset, so a tile costs no VALU at all; keys >= nk fall
// outside the buffer descriptor's range and load zeros.  Planes past the head dim
// are written once: K's are zero, V's plane D/8 holds the 1.0 sum column (DSUM).
// K fragment reads (ds_read_b128, 16 keys x one plane per 16-lane group) are
// conflict-free; V planes are stored with a rotation of 8 keys per plane so the
// transposed PV reads (ds_read_b64_tr_b16 over two adjacent planes) are too.

template <int N>
__device__ __forceinline__ void attn_wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// XCD-aware order (blocks b and b + 8 share an XCD under round-robin dispatch): every
// XCD gets a contiguous range of logical blocks, so the query blocks of one (batch,
// head) -- which read the same K/V tiles -- run together on one L2.
__device__ __forceinline__ int attn_xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

template <int KC, int ND, int DSUM, int QG>
__global__ void __launch_bounds__(256, 2) attn5_kernel(AttnArgs a, int nqb, int heads) {
  constexpr int KT = 64;
  constexpr int NST = 3;                   // LDS ring: tile t computed while t+1, t+2 land
  constexpr int KPL = KC * 4;              // K planes (32-wide d chunks x 4)
  constexpr int VPL = ND * 2;              // V planes (16-wide d fragments x 2)
  constexpr int PLANE = KT * 8;            // elements per plane (64 keys x 8)
  constexpr int STAGE = (KPL + VPL) * PLANE;
  constexpr int QW = 16 * QG;              // queries per wave
  constexpr float TAU = 10.f;
  static_assert(DSUM == 0 || (DSUM % 8 == 0 && DSUM < 16 * ND), "sum column must be a padding column");
  extern __shared__ __attribute__((aligned(16))) u16 sm[];  // [NST][K planes, V planes] + dummy plane

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lb = attn_xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lb % nqb, pair = lb / nqb;
  const int h = pair % heads;
  const int b = pair / heads;
  const long b1 = b / a.z2, b2 = b - b1 * a.z2;
  const u16* qb = a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)h * a.q_sh;
  const u16* kb = a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + (long)h * a.k_sh;
  const u16* vb = a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + (long)h * a.v_sh;
  u16* ob = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)h * a.o_sh;
  const int q0 = (qblk * 4 + wid) * QW;
  const int lq = lane & 15, lg = lane >> 4;
  const int cpr = (a.D + 7) >> 3;           // planes that carry data

  // constant planes of every stage: K's zero, V's sum column / zero
  for (int i = tid; i < NST * (KPL + VPL) * KT; i += 256) {
    const int r = i % KT, c = (i / KT) % (KPL + VPL), st = i / (KT * (KPL + VPL));
    const bool isv = c >= KPL;
    const int cc = isv ? c - KPL : c;
    if (cc >= cpr)
      *(uint4*)(sm + st * STAGE + c * PLANE + r * 8) = make_uint4(isv && DSUM && cc * 8 == DSUM ? 0x3F80u : 0u, 0, 0, 0);
  }

  const float c2 = a.scale_log2;
  bf16x8 qf[QG][KC];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int d = kc * 32 + lg * 8;
      const int q = q0 + g * 16 + lq;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (q < a.nq && d < a.D) v = *(const uint4*)(qb + (long)q * a.q_si + d);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= c2;
      qf[g][kc] = __builtin_bit_cast(bf16x8, pack8(f));
    }

  // DMA: the 2 cpr plane loads of a tile are dealt round-robin to the 4 waves, padded
  // to the same count per wave (extra loads re-fetch plane 0 of K into a dummy plane)
  // so every wave's wait is one constant vmcnt
  const uint32_t kst = (uint32_t)a.k_si * 2, vst = (uint32_t)a.v_si * 2;
  const i32x4 krs = buffer_rsrc(kb, (uint32_t)(a.nk - 1) * kst + cpr * 16);
  const i32x4 vrs = buffer_rsrc(vb, (uint32_t)(a.nk - 1) * vst + cpr * 16);
  constexpr int NDMA = (2 * ((KC * 32 < ND * 16 ? KC * 32 : ND * 16) / 8) + 3) / 4;  // per wave, upper bound
  u16* dummy = sm + NST * STAGE;
  auto issue = [&](int t) {
    const int t0 = t * KT;
    u16* st = sm + (t % NST) * STAGE;
#pragma unroll
    for (int u = 0; u < NDMA; ++u) {
      const int j = wid + 4 * u;  // wave-uniform
      const bool live = j < 2 * cpr;
      const bool isv = live && j >= cpr;
      const int c = !live ? 0 : (isv ? j - cpr : j);
      const int key = isv ? ((lane - 8 * c) & 63) : lane;
      u16* dst = live ? st + ((isv ? KPL : 0) + c) * PLANE : dummy;
      ls_raw_buffer_load_lds(isv ? vrs : krs, (__attribute__((address_space(3))) void*)dst, 16,
                             key * (int)(isv ? vst : kst) + c * 16, t0 * (int)(isv ? vst : kst), 0, 0);
    }
  };

  f32x4 oacc[QG][ND];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int i = 0; i < ND; ++i) oacc[g][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[QG], l[QG];
  f32x4 negm[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    m[g] = 0.f;
    l[g] = 0.f;
    negm[g] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  const int ntile = (a.nk + KT - 1) / KT;
  issue(0);
  if (ntile > 1) issue(1);
  auto tile = [&](int t, auto partial_tag) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    const int t0 = t * KT;
    if (t + 1 < ntile) attn_wait_vm<NDMA>();  // this wave's DMA of tile t landed (t+1's may fly)
    else attn_wait_vm<0>();
    __syncthreads();                          // everyone's; slot (t+2) % 3 free
    if (t + 2 < ntile) issue(t + 2);
    const u16* Ks = sm + (t % NST) * STAGE;
    const u16* Vs = Ks + KPL * PLANE;
    f32x4 s[QG][4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const bf16x8 kf = __builtin_bit_cast(bf16x8, *(const uint4*)(Ks + (kc * 4 + lg) * PLANE + (16 * f + lq) * 8));
#pragma unroll
        for (int g = 0; g < QG; ++g)
          s[g][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[g][kc], kc == 0 ? negm[g] : s[g][f], 0, 0, 0);
      }
    }
    float mt[QG];
    bool need_any = t == 0;
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      if (PARTIAL) {
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t0 + 16 * f + 4 * lg + r >= a.nk) s[g][f][r] = -INFINITY;
      }
      float x = __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][0][0], s[g][0][1]),
                                              __builtin_elementwise_maximum(s[g][0][2], s[g][0][3]));
#pragma unroll
      for (int f = 1; f < 4; ++f)
        x = __builtin_elementwise_maximum(
            x, __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][f][0], s[g][f][1]),
                                             __builtin_elementwise_maximum(s[g][f][2], s[g][f][3])));
      mt[g] = xor16_32_max(x);
      need_any |= mt[g] > TAU;
    }
    // one wave-uniform check per tile: move the reference max of the rows whose tile
    // max exceeds it by TAU (every row on the first tile)
    if (__builtin_amdgcn_ballot_w64(need_any)) {
#pragma unroll
      for (int g = 0; g < QG; ++g) {
        const bool need = t == 0 || mt[g] > TAU;
        const float dlt = need ? mt[g] : 0.f;
        const float alpha = t == 0 ? 0.f : fast_exp2(-dlt);
        m[g] += dlt;
        negm[g] = (f32x4){-m[g], -m[g], -m[g], -m[g]};
#pragma unroll
        for (int f = 0; f < 4; ++f) s[g][f] -= dlt;
#pragma unroll
        for (int i = 0; i < ND; ++i) oacc[g][i] *= alpha;
        l[g] *= alpha;
      }
    }
#pragma unroll
    for (int g = 0; g < QG; ++g) {
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[g][f][r] = fast_exp2(s[g][f][r]);
      if (!DSUM) {
        float ps = 0.f;
#pragma unroll
        for (int f = 0; f < 4; ++f) ps += (s[g][f][0] + s[g][f][1]) + (s[g][f][2] + s[g][f][3]);
        l[g] += ps;
      }
    }
    // O^T += V^T P^T over 32-key chunks; a lane reads 4 dims of one key from plane
    // 2 nd + pp/2 (rows rotated by 8 keys per plane)
    const int qq = lq >> 2, pp = lq & 3;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8 pb[QG];
#pragma unroll
      for (int g = 0; g < QG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          pb[g][r] = (__bf16)s[g][2 * c][r];
          pb[g][4 + r] = (__bf16)s[g][2 * c + 1][r];
        }
      const int key = 32 * c + 4 * lg + qq;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        const int pl = 2 * nd + (pp >> 1);
        const u16* plane = Vs + pl * PLANE + (pp & 1) * 4;
        const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4i16*)(plane + ((key + 8 * pl) & 63) * 8));
        const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) v4i16*)(plane + ((key + 16 + 8 * pl) & 63) * 8));
        const short __attribute__((ext_vector_type(8))) av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const bf16x8 vf = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int g = 0; g < QG; ++g)
          oacc[g][nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[g], oacc[g][nd], 0, 0, 0);
      }
    }
  };
  const int nfull = a.nk / KT;
  for (int t = 0; t < nfull; ++t) tile(t, std::false_type{});
  if (nfull < ntile) tile(nfull, std::true_type{});
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    float lt;
    if (DSUM) {
      constexpr int NDL = DSUM / 16, LGL = (DSUM % 16) / 4, RL = DSUM % 4;
      lt = __shfl(oacc[g][NDL][RL], LGL * 16 + lq, 64);
    } else {
      lt = xor16_32_sum(l[g]);
    }
    const float inv = 1.f / lt;
    const int q = q0 + g * 16 + lq;
    if (q < a.nq) {
      u16* orow = ob + (long)q * a.o_si;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        const int d = nd * 16 + 4 * lg;
        if (d + 3 < a.D) {
          uint2 w;
          w.x = pack2(oacc[g][nd][0] * inv, oacc[g][nd][1] * inv);
          w.y = pack2(oacc[g][nd][2] * inv, oacc[g][nd][3] * inv);
          *(uint2*)(orow + d) = w;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (d + r < a.D) orow[d + r] = f2bf(oacc[g][nd][r] * inv);
        }
      }
    }
  }
}

template <int KC, int ND, int DSUM, int QG = 2>
static int launch_attn5(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  const int nqb = cdiv(a.nq, 4 * 16 * QG);
  const long nblk = (long)nqb * heads * batch;
  if (nblk > 0x7fffffff) return fail(LS_ERR_INVALID, "ls_attention: grid too large");
  const size_t shm = (3 * (size_t)(KC * 4 + ND * 2) + 1) * 64 * 8 * sizeof(u16);
  if (shm > 64 * 1024) {
    LS_SET_MAX_DYN_SHM((attn5_kernel<KC, ND, DSUM, QG>), (int)shm);
  }
  attn5_kernel<KC, ND, DSUM, QG><<<(int)nblk, 256, shm, s>>>(a, nqb, heads);
  return check_launch("attn5_kernel");
}

#ifdef LS_DIAG_KERNELS  // measured and rejected: diagnostics build only
// attn6: the d = 40 self attention (UNet 32x32 level; 64x64 at configs[4]) on
// v_mfma_f32_32x32x16_bf16.  attn5 is issue-bound, not MFMA-bound: per 64-key tile and
// wave it issues 64 v_exp_f32 (8 cycles each) beside 56 16x16x32 MFMAs that each hold the
// SIMD's vector issue for 8 of their 16 cycles (448 cycles), so the ~1350 issue cycles of
// a tile exceed its 896 MFMA cycles.  The 32x32x16 form holds issue 8 of 32 cycles: the
// same 896 MFMA cycles (QK^T: 2 query x 2 key tiles x 3 k-steps over d padded to 48;
// P V: 2 query x 2 d tiles x 4 key steps over d padded to 64, row 40 = the sum column)
// cost 224 issue cycles instead of 448.
//   * S^T = K Q^T per (query tile qt, key tile kt): a lane holds query r32 = lane & 31
//     and 16 keys (i & 3) + 8 (i >> 2) + 4 hh of the tile (hh = lane >> 5), so the row
//     max is 31 maxima + one permlane32 swap; C = -m (a 16-register splat per qt).
//   * The accumulator IS the next MFMA's B operand (cdna_hip_programming.md §3, "an
//     accumulator tile as the next MFMA's operand"): registers 8s .. 8s+7 of S^T are
//     k-step s of O^T += V^T P^T with element j = key 16s + 8(j>>2) + 4hh + (j&3); the V^T
//     fragment takes the same key order by two ds_read_b64_tr_b16 (4 keys each).
//   * V plane c stores key k at position k ^ 4 (c & 3) (attn5 rotates by 8 keys per plane)
//     so the 32-lane halves of those transposed reads, which span 4 planes, hit 32 distinct
//     8-B bank slots; the XOR leaves bit 5 alone, so the second 32-key half of a tile is a
//     uniform offset.
// Same DMA ring, lazy rescale and XCD-aware block order as attn5.
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float swap32_max(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_elementwise_maximum(__uint_as_float(a[0]), __uint_as_float(a[1]));
}

template <int DSUM>
__global__ void __launch_bounds__(256, 2) attn6_kernel(AttnArgs a, int nqb, int heads) {
  constexpr int KT = 64;
  constexpr int NST = 3;
  constexpr int KPL = 6;        // K planes: d 0..47 (3 k-steps of 16)
  constexpr int VPL = 8;        // V planes: d 0..63 (two 32-row O^T tiles)
  constexpr int PLANE = KT * 8;
  constexpr int STAGE = (KPL + VPL) * PLANE;
  constexpr float TAU = 10.f;
  static_assert(DSUM == 40, "attn6 is the d = 40 kernel (sum column at d = 40)");
  extern __shared__ __attribute__((aligned(16))) u16 sm[];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lb = attn_xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lb % nqb, pair = lb / nqb;
  const int h = pair % heads;
  const int b = pair / heads;
  const long b1 = b / a.z2, b2 = b - b1 * a.z2;
  const u16* qb = a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)h * a.q_sh;
  const u16* kb = a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + (long)h * a.k_sh;
  const u16* vb = a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + (long)h * a.v_sh;
  u16* ob = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)h * a.o_sh;
  const int q0 = (qblk * 4 + wid) * 64;
  const int r32 = lane & 31, hh = lane >> 5;
  const int cpr = (a.D + 7) >> 3;  // planes that carry data (5)

  // constant planes of every stage: K's zero, V's sum column / zero (a constant plane
  // reads the same under any key rotation)
  for (int i = tid; i < NST * (KPL + VPL) * KT; i += 256) {
    const int r = i % KT, c = (i / KT) % (KPL + VPL), st = i / (KT * (KPL + VPL));
    const bool isv = c >= KPL;
    const int cc = isv ? c - KPL : c;
    if (cc >= cpr)
      *(uint4*)(sm + st * STAGE + c * PLANE + r * 8) = make_uint4(isv && cc * 8 == DSUM ? 0x3F80u : 0u, 0, 0, 0);
  }

  // Q^T fragments (B operand): lane (r32, hh) holds Q[q0 + 32 qt + r32][16 ks + 8 hh .. + 8]
  const float c2 = a.scale_log2;
  bf16x8 qf[2][3];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int d = ks * 16 + hh * 8;
      const int q = q0 + qt * 32 + r32;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (q < a.nq && d < a.D) v = *(const uint4*)(qb + (long)q * a.q_si + d);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= c2;
      qf[qt][ks] = __builtin_bit_cast(bf16x8, pack8(f));
    }

  const uint32_t kst = (uint32_t)a.k_si * 2, vst = (uint32_t)a.v_si * 2;
  const i32x4 krs = buffer_rsrc(kb, (uint32_t)(a.nk - 1) * kst + cpr * 16);
  const i32x4 vrs = buffer_rsrc(vb, (uint32_t)(a.nk - 1) * vst + cpr * 16);
  constexpr int NDMA = 3;  // ceil(2 * 5 planes / 4 waves); extra loads go to the dummy plane
  u16* dummy = sm + NST * STAGE;
  auto issue = [&](int t) {
    const int t0 = t * KT;
    u16* st = sm + (t % NST) * STAGE;
#pragma unroll
    for (int u = 0; u < NDMA; ++u) {
      const int j = wid + 4 * u;  // wave-uniform
      const bool live = j < 2 * cpr;
      const bool isv = live && j >= cpr;
      const int c = !live ? 0 : (isv ? j - cpr : j);
      const int key = isv ? (lane ^ (4 * (c & 3))) : lane;  // V: position p holds key p ^ 4 (c & 3)
      u16* dst = live ? st + ((isv ? KPL : 0) + c) * PLANE : dummy;
      ls_raw_buffer_load_lds(isv ? vrs : krs, (__attribute__((address_space(3))) void*)dst, 16,
                             key * (int)(isv ? vst : kst) + c * 16, t0 * (int)(isv ? vst : kst), 0, 0);
    }
  };

  f32x16 oacc[2][2];
  f32x16 negm[2];
  float m[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    m[qt] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      oacc[qt][0][i] = 0.f;
      oacc[qt][1][i] = 0.f;
      negm[qt][i] = 0.f;
    }
  }

  // per-lane LDS element offsets of the V^T fragment reads (tile-invariant): group
  // g = lane >> 4 reads keys 4 (g >> 1) + q, d = 32 dt + 16 (g & 1) + 4 p (lane 4q + p)
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3, gg = lane >> 4;
  int voff[2][2][2];  // [dt][s][half of the key step]
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    const int pl = 4 * dt + 2 * (gg & 1) + (tp >> 1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int key = 16 * s + 8 * e + 4 * (gg >> 1) + tq;  // within a 32-key tile (+ 32 kt below)
        voff[dt][s][e] = pl * PLANE + (key ^ (4 * (pl & 3))) * 8 + (tp & 1) * 4;
      }
  }

  const int ntile = (a.nk + KT - 1) / KT;
  issue(0);
  if (ntile > 1) issue(1);
  auto tile = [&](int t, auto partial_tag) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    const int t0 = t * KT;
    if (t + 1 < ntile) attn_wait_vm<NDMA>();
    else attn_wait_vm<0>();
    __syncthreads();
    if (t + 2 < ntile) issue(t + 2);
    const u16* Ks = sm + (t % NST) * STAGE;
    const u16* Vs = Ks + KPL * PLANE;
    f32x16 s[2][2];  // [qt][kt]
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const bf16x8 kf =
            __builtin_bit_cast(bf16x8, *(const uint4*)(Ks + (2 * ks + hh) * PLANE + (32 * kt + r32) * 8));
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
          s[qt][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[qt][ks], ks == 0 ? negm[qt] : s[qt][kt], 0, 0, 0);
      }
    }
    float mt[2];
    bool need_any = t == 0;
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      if (PARTIAL) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (t0 + 32 * kt + (i & 3) + 8 * (i >> 2) + 4 * hh >= a.nk) s[qt][kt][i] = -INFINITY;
      }
      float x = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; i += 2)
          x = __builtin_elementwise_maximum(x, __builtin_elementwise_maximum(s[qt][kt][i], s[qt][kt][i + 1]));
      mt[qt] = swap32_max(x);
      need_any |= mt[qt] > TAU;
    }
    if (__builtin_amdgcn_ballot_w64(need_any)) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        const bool need = t == 0 || mt[qt] > TAU;
        const float dlt = need ? mt[qt] : 0.f;
        const float alpha = t == 0 ? 0.f : fast_exp2(-dlt);
        m[qt] += dlt;
#pragma unroll
        for (int i = 0; i < 16; ++i) negm[qt][i] = -m[qt];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) s[qt][kt] -= dlt;
        oacc[qt][0] *= alpha;
        oacc[qt][1] *= alpha;
      }
    }
    // P = exp2(S^T - m), then O^T += V^T P^T over 4 key steps of 16
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[qt][kt][i] = fast_exp2(s[qt][kt][i]);
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pb[2];
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[qt][j] = (__bf16)s[qt][kt][8 * st + j];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const u16* vk = Vs + 32 * kt * 8;  // key 32 kt of every plane (the XOR keeps bit 5)
          const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4i16*)(vk + voff[dt][st][0]));
          const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) v4i16*)(vk + voff[dt][st][1]));
          const short __attribute__((ext_vector_type(8))) av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const bf16x8 vf = __builtin_bit_cast(bf16x8, av);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt)
            oacc[qt][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[qt], oacc[qt][dt], 0, 0, 0);
        }
      }
    }
  };
  const int nfull = a.nk / KT;
  for (int t = 0; t < nfull; ++t) tile(t, std::false_type{});
  if (nfull < ntile) tile(nfull, std::true_type{});
  // l = O^T row 40: d tile 1, row 8 -> register 4 of the half hh = 0
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float lt = __shfl(oacc[qt][1][4], r32, 64);
    const float inv = 1.f / lt;
    const int q = q0 + qt * 32 + r32;
    if (q < a.nq) {
      u16* orow = ob + (long)q * a.o_si;
#pragma unroll
      for (int g = 0; g < 5; ++g) {  // d = 8 g' + 4 hh .. +3: dt 0 rows 4g..4g+3 (g < 4), dt 1 rows 0..3
        const int dt = g >> 2, rg = g & 3;
        const int d = 32 * dt + 8 * rg + 4 * hh;
        uint2 w;
        w.x = pack2(oacc[qt][dt][4 * rg] * inv, oacc[qt][dt][4 * rg + 1] * inv);
        w.y = pack2(oacc[qt][dt][4 * rg + 2] * inv, oacc[qt][dt][4 * rg + 3] * inv);
        *(uint2*)(orow + d) = w;
      }
    }
  }
}

template <int DSUM>
static int launch_attn6(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  const int nqb = cdiv(a.nq, 4 * 64);
  const long nblk = (long)nqb * heads * batch;
  if (nblk > 0x7fffffff) return fail(LS_ERR_INVALID, "ls_attention: grid too large");
  const size_t shm = (3 * (size_t)(6 + 8) + 1) * 64 * 8 * sizeof(u16);
  LS_SET_MAX_DYN_SHM((attn6_kernel<DSUM>), (int)shm);
  attn6_kernel<DSUM><<<(int)nblk, 256, shm, s>>>(a, nqb, heads);
  return check_launch("attn6_kernel");
}

#endif  // LS_DIAG_KERNELS

// attnw: wide heads -- the SD-VAE mid-block attention (1 head, d = 512, N = h w tokens;
// diffusers Attention).  Replaces attn_kernel<512,4> (0.068 of the
// dense peak: K / V staged synchronously behind two barriers per tile, no prefetch, one
// 4-wave block per CU).  A wave owns QG 16-query fragments at the full head dim (Q and
// the O^T accumulator in registers: 64 + 128 VGPRs at QG = 1, so two waves per SIMD and
// eight per block share each K / V tile; QG = 2 would halve the LDS fragment reads per
// MFMA but needs 384 registers, and the compiler spills it even at one wave per SIMD).
//   * 32-key tiles by buffer_load ... lds DMA, "chunk-plane" layout (plane c = dims
//     8c .. 8c + 7 of the tile's 32 keys; one wave-instruction moves two planes), K planes
//     plain (ds_read_b128 fragments conflict-free), V planes with the key rotated by 8 per
//     plane (the ds_read_b64_tr_b16 V^T reads conflict-free, as attn5); two 64-KB stages,
//     the next tile's DMA issued under the current tile's MFMAs.
//   * fragment reads software-pipelined PF k-steps ahead from one lane base plus
//     immediate offsets (per-fragment addresses hoisted out of the tile loop each held a
//     register and spilled the kernel);
//   * S^T = K Q^T with the running max subtracted by the MFMA (C = -m), lazy rescale
//     (threshold 10, one ballot per tile), bf16 P straight into O^T += V^T P^T (attn5's
//     arithmetic).
template <int D, int QG, int NW, int PF = 1, bool SB = true>
__global__ void __launch_bounds__(NW * 64, 1) attnw_kernel(AttnArgs a, int nqb, int heads) {
  constexpr int KT = 32;                  // keys per tile
  constexpr int NPL = D / 8;              // 16-B planes per operand row
  constexpr int PLANE = KT * 8;           // u16 per plane
  constexpr int STAGE = 2 * NPL * PLANE;  // K planes, then V planes
  constexpr int KC = D / 32;              // QK^T k-steps
  constexpr int ND = D / 16;              // O^T fragments per query group
  constexpr int QPB = NW * 16 * QG;       // queries per block
  constexpr int NDMA = NPL / NW;          // DMA wave-instructions per wave per tile (2 planes each)
  constexpr float TAU = 10.f;
  static_assert(D % 64 == 0 && NPL % NW == 0, "attnw: d multiple of 64");
  extern __shared__ __attribute__((aligned(16))) u16 sm[];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lb = attn_xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lb % nqb, pair = lb / nqb;
  const int h = pair % heads;
  const int b = pair / heads;
  const long b1 = b / a.z2, b2 = b - b1 * a.z2;
  const u16* qb = a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)h * a.q_sh;
  const u16* kb = a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + (long)h * a.k_sh;
  const u16* vb = a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + (long)h * a.v_sh;
  u16* ob = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)h * a.o_sh;
  const int q0 = qblk * QPB + wid * 16 * QG;
  const int lq = lane & 15, lg = lane >> 4;

  const float c2 = a.scale_log2;
  bf16x8 qf[QG][KC];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int q = q0 + g * 16 + lq;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (q < a.nq) v = *(const uint4*)(qb + (long)q * a.q_si + kc * 32 + lg * 8);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= c2;
      qf[g][kc] = __builtin_bit_cast(bf16x8, pack8(f));
    }

  // DMA of tile t: wave w issues instructions j = w + NW i; j < NPL / 2 moves K planes
  // 2j, 2j + 1 (lane: plane 2j + lane / 32, key lane % 32), the rest V planes with the
  // key rotated by 8 per plane (position (key + 8 c) % 32)
  const uint32_t kst = (uint32_t)a.k_si * 2, vst = (uint32_t)a.v_si * 2;
  const i32x4 krs = buffer_rsrc(kb, (uint32_t)(a.nk - 1) * kst + D * 2);
  const i32x4 vrs = buffer_rsrc(vb, (uint32_t)(a.nk - 1) * vst + D * 2);
  auto issue = [&](int t) {
    u16* st = sm + (t & 1) * STAGE;
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
      const int j = wid + NW * i;  // wave-uniform
      const bool isv = j >= NPL / 2;
      const int jj = isv ? j - NPL / 2 : j;
      const int c = 2 * jj + (lane >> 5);
      const int key = isv ? (((lane & 31) - 8 * c) & 31) : (lane & 31);
      ls_raw_buffer_load_lds(isv ? vrs : krs,
                             (__attribute__((address_space(3))) void*)(st + (isv ? NPL : 0) * PLANE + 2 * jj * PLANE), 16,
                             key * (int)(isv ? vst : kst) + c * 16, t * KT * (int)(isv ? vst : kst), 0, 0);
    }
  };

  f32x4 oacc[QG][ND];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int i = 0; i < ND; ++i) oacc[g][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[QG], l[QG];
  f32x4 negm[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    m[g] = 0.f;
    l[g] = 0.f;
    negm[g] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  const int ntile = (a.nk + KT - 1) / KT;
  issue(0);
  for (int t = 0; t < ntile; ++t) {
    attn_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t landed everywhere; every wave is past tile t - 1
    asm volatile("" ::: "memory");
    if (t + 1 < ntile) issue(t + 1);
    const u16* Ks = sm + (t & 1) * STAGE;
    const u16* Vs = Ks + NPL * PLANE;
    // (software-pipelined PF k-steps ahead; SB fences each step with sched_barrier)
    f32x4 s[QG][2];
    // (one lane base + immediate offsets: per-fragment addresses hoisted out of the tile
    // loop would each hold a register)
    const u16* kl = Ks + lg * PLANE + lq * 8;
    auto kread = [&](int kc, int f) {
      return __builtin_bit_cast(bf16x8, *(const uint4*)(kl + kc * 4 * PLANE + f * 128));
    };
    bf16x8 kq[PF][2];  // fragments of k-steps kc .. kc + PF - 1 in flight
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      kq[p][0] = kread(p, 0);
      kq[p][1] = kread(p, 1);
    }
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const bf16x8 k0 = kq[kc % PF][0], k1 = kq[kc % PF][1];
      if (kc + PF < KC) {
        kq[kc % PF][0] = kread(kc + PF, 0);
        kq[kc % PF][1] = kread(kc + PF, 1);
      }
#pragma unroll
      for (int g = 0; g < QG; ++g) {
        s[g][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[g][kc], kc == 0 ? negm[g] : s[g][0], 0, 0, 0);
        s[g][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[g][kc], kc == 0 ? negm[g] : s[g][1], 0, 0, 0);
      }
      if (SB) __builtin_amdgcn_sched_barrier(0);
    }
    const int t0 = t * KT;
    float mt[QG];
    bool need_any = t == 0;
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      if (t0 + KT > a.nk) {
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (t0 + 16 * f + 4 * lg + r >= a.nk) s[g][f][r] = -INFINITY;
      }
      float x = __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][0][0], s[g][0][1]),
                                              __builtin_elementwise_maximum(s[g][0][2], s[g][0][3]));
      x = __builtin_elementwise_maximum(
          x, __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][1][0], s[g][1][1]),
                                           __builtin_elementwise_maximum(s[g][1][2], s[g][1][3])));
      mt[g] = xor16_32_max(x);
      need_any |= mt[g] > TAU;
    }
    if (__builtin_amdgcn_ballot_w64(need_any)) {
#pragma unroll
      for (int g = 0; g < QG; ++g) {
        const bool need = t == 0 || mt[g] > TAU;
        const float dlt = need ? mt[g] : 0.f;
        const float alpha = t == 0 ? 0.f : fast_exp2(-dlt);
        m[g] += dlt;
        negm[g] = (f32x4){-m[g], -m[g], -m[g], -m[g]};
#pragma unroll
        for (int f = 0; f < 2; ++f) s[g][f] -= dlt;
#pragma unroll
        for (int i = 0; i < ND; ++i) oacc[g][i] *= alpha;
        l[g] *= alpha;
      }
    }
    bf16x8 pb[QG];
#pragma unroll
    for (int g = 0; g < QG; ++g) {
      float ps = 0.f;
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const __bf16 pr = (__bf16)fast_exp2(s[g][f][r]);
          ps += (float)pr;  // the denominator sums the bf16 P that P.V consumes (as tattn_fused)
          pb[g][4 * f + r] = pr;
        }
      l[g] += ps;
    }
    // O^T += V^T P^T: a lane reads 4 dims of key 4 lg + qq (and + 16) from plane
    // 2 nd + pp / 2 at its rotated position
    // plane pl = 2 nd + pp / 2 holds key k at position (k + 8 pl) % 32: for even nd the
    // low read (key) sits at rotation re, the high one (key + 16) at ro; odd nd swaps them
    const int qq = lq >> 2, pp = lq & 3;
    const int key = 4 * lg + qq;
    const u16* vl = Vs + (pp >> 1) * PLANE + (pp & 1) * 4;
    const u16* pe = vl + ((key + 8 * (pp >> 1)) & 31) * 8;
    const u16* po = vl + ((key + 16 + 8 * (pp >> 1)) & 31) * 8;
    auto vread = [&](int nd) {
      const u16* lop = ((nd & 1) ? po : pe) + 2 * nd * PLANE;
      const u16* hip = ((nd & 1) ? pe : po) + 2 * nd * PLANE;
      const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)lop);
      const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)hip);
      const short __attribute__((ext_vector_type(8))) av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, av);
    };
    bf16x8 vq[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) vq[p] = vread(p);
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) {
      const bf16x8 vf = vq[nd % PF];
      if (nd + PF < ND) vq[nd % PF] = vread(nd + PF);
#pragma unroll
      for (int g = 0; g < QG; ++g) oacc[g][nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[g], oacc[g][nd], 0, 0, 0);
      if (SB) __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    const float inv = 1.f / xor16_32_sum(l[g]);
    const int q = q0 + g * 16 + lq;
    if (q < a.nq) {
      u16* orow = ob + (long)q * a.o_si;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd)
        *(uint2*)(orow + nd * 16 + 4 * lg) = make_uint2(pack2(oacc[g][nd][0] * inv, oacc[g][nd][1] * inv),
                                                        pack2(oacc[g][nd][2] * inv, oacc[g][nd][3] * inv));
    }
  }
}

template <int D, int QG, int NW, int PF, bool SB>
static int launch_attnw(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  const int nqb = cdiv(a.nq, NW * 16 * QG);
  const long nblk = (long)nqb * heads * batch;
  if (nblk > 0x7fffffff) return fail(LS_ERR_INVALID, "ls_attention: grid too large");
  const size_t shm = (size_t)2 * 2 * (D / 8) * 32 * 8 * sizeof(u16);  // two stages of K + V tiles
  LS_SET_MAX_DYN_SHM((attnw_kernel<D, QG, NW, PF, SB>), (int)shm);
  attnw_kernel<D, QG, NW, PF, SB><<<(int)nblk, NW * 64, shm, s>>>(a, nqb, heads);
  return check_launch("attnw_kernel");
}

static const int g_attnw_variant = ls_env("LS_ATTNW_VARIANT") ? atoi(ls_env("LS_ATTNW_VARIANT")) : 0;  // A/B switch

static int launch_attnw512(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  // same-box A/B (scripts/attn_bench.py VAE=1, 512 images at 32^2 / 64 at 64^2):
  // PF 1 fenced 1673 / 2934 us, PF 1 unfenced 1609 / 2818, PF 2 fenced 1598 / 2793,
  // PF 2 unfenced 1609 / 2812 (attn_kernel<512,4> before: 6449 / 11858)
  switch (g_attnw_variant) {
    case 1: return launch_attnw<512, 1, 8, 1, false>(a, batch, heads, s);
    case 2: return launch_attnw<512, 1, 8, 1, true>(a, batch, heads, s);
    case 3: return launch_attnw<512, 1, 8, 2, false>(a, batch, heads, s);
    default: return launch_attnw<512, 1, 8, 2, true>(a, batch, heads, s);
  }
}

template <int KC, int ND, int DSUM, bool ONE>
static int launch_attn3_(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  const dim3 grid(cdiv(a.nq, 128), heads, batch);
  const size_t shm = (ONE ? 1 : 2) * 2 * (size_t)64 * (KC * 32 + 8) * sizeof(u16);
  if (shm > 64 * 1024) {
    LS_SET_MAX_DYN_SHM((attn3_kernel<KC, ND, DSUM, ONE>), (int)shm);
  }
  attn3_kernel<KC, ND, DSUM, ONE><<<grid, 256, shm, s>>>(a);
  return check_launch("attn3_kernel");
}

static bool g_attn3_two = ls_env("LS_ATTN3_TWO_STAGE") != nullptr;  // A/B switch: no single-tile variant

template <int KC, int ND, int DSUM>
static int launch_attn3(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  if (a.nk <= 64 && !g_attn3_two) return launch_attn3_<KC, ND, DSUM, true>(a, batch, heads, s);
  return launch_attn3_<KC, ND, DSUM, false>(a, batch, heads, s);
}

template <int DP, int NKF>
static int launch_attn(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  const int nwant = cdiv(a.nq, 16);
  const int nw = std::min(4, nwant);
  const dim3 grid(cdiv(nwant, nw), heads, batch);
  const size_t shm = 2 * (size_t)(16 * NKF) * (DP + 8) * sizeof(u16);
  if (shm > 64 * 1024) {
    LS_SET_MAX_DYN_SHM((attn_kernel<DP, NKF>), (int)shm);
  }
  attn_kernel<DP, NKF><<<grid, nw * 64, shm, s>>>(a);
  return check_launch("attn_kernel");
}


// ------------------------------------------------- short sequences (temporal)
// VersatileAttention over the 16 frames of a window (motion_module.py:203-239) is
// 16 queries x 16 keys per (pixel, head): far too small for MFMA tiles, and the
// flash kernel above spent a 256-thread block per (pixel, head) re-reading 80-B
// head slices.  Here a block owns NB whole (pixel) sequences -- all heads, i.e.
// full contiguous C-channel rows of K and V, read once with 16-B loads -- stages
// them row-major in LDS, and every thread computes one (sequence, head, query):
// QK^T with packed-bf16 dot products (v_dot2_f32_bf16, fp32 accumulation), fp32
// softmax, P V as fp32 FMAs over the 16 keys.  TS threads split the head dim
// (partial dots summed with lane shuffles, D/TS output dims each).  All LDS reads
// are broadcasts within a (sequence, head) lane group.  HBM bound: q, k, v read
// once, o written once.
// Host contract: nq == nk <= 16, heads contiguous (q/k/v/o head stride == D),
// D / TS == 40, heads * 16 * TS divides the block (256 or 512), 16-B aligned rows.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int D, int TS, int NT>
__global__ void __launch_bounds__(NT, 4) attn_seq_kernel(AttnArgs a, int H, int nbatch) {
  constexpr int DT = D / TS;                  // head dims per thread (40)
  constexpr int DC = DT / 8;                  // 16-B chunks per thread slice
  const int C = H * D;
  const int F = a.nk;
  const int NB = NT / (H * 16 * TS);          // sequences per block
  extern __shared__ __attribute__((aligned(16))) u16 sm[];
  u16* Ks = sm;                               // [NB][16][C]
  u16* Vs = sm + NB * 16 * C;                 // [NB][16][C]
  const int tid = threadIdx.x;
  const int bz0 = blockIdx.x * NB;

  // ---- stage K and V rows of the block's sequences (zero rows past F / nbatch)
  const int cpr = C / 8;  // 16-B chunks per row
  for (int q = tid; q < NB * 16 * cpr; q += NT) {
    const int nb = q / (16 * cpr), r = q - nb * 16 * cpr;
    const int j = r / cpr, c8 = (r - j * cpr) * 8;
    const int bz = bz0 + nb;
    uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (bz < nbatch && j < F) {
      const long b1 = bz / a.z2, b2 = bz - b1 * a.z2;
      kv = *(const uint4*)(a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + j * a.k_si + c8);
      vv = *(const uint4*)(a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + j * a.v_si + c8);
    }
    *(uint4*)(Ks + (nb * 16 + j) * C + c8) = kv;
    *(uint4*)(Vs + (nb * 16 + j) * C + c8) = vv;
  }

  // ---- this thread's item: lane = query * TS + ts inside a 16*TS-lane (sequence, head) group
  const int grp = tid / (16 * TS), in = tid - grp * 16 * TS;
  const int qi = in / TS, ts = in - qi * TS;
  const int nb = grp / H, h = grp - nb * H;
  const int bz = bz0 + nb;
  const bool live = bz < nbatch && qi < F;
  const long b1 = bz / a.z2, b2 = bz - b1 * a.z2;
  bf16x2 qv[DT / 2];
  {
    const u16* qp = a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)qi * a.q_si + (long)h * a.q_sh + ts * DT;
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      const uint4 u = live ? *(const uint4*)(qp + c * 8) : make_uint4(0, 0, 0, 0);
      qv[4 * c + 0] = __builtin_bit_cast(bf16x2, u.x); qv[4 * c + 1] = __builtin_bit_cast(bf16x2, u.y);
      qv[4 * c + 2] = __builtin_bit_cast(bf16x2, u.z); qv[4 * c + 3] = __builtin_bit_cast(bf16x2, u.w);
    }
  }
  __syncthreads();

  // ---- scores (log2 domain), softmax over the F keys
  const int off = nb * 16 * C + h * D + ts * DT;
  float sc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < DC; ++c) {
      const uint4 u = *(const uint4*)(Ks + off + j * C + c * 8);
      acc = __builtin_amdgcn_fdot2_f32_bf16(qv[4 * c + 0], __builtin_bit_cast(bf16x2, u.x), acc, false);
      acc = __builtin_amdgcn_fdot2_f32_bf16(qv[4 * c + 1], __builtin_bit_cast(bf16x2, u.y), acc, false);
      acc = __builtin_amdgcn_fdot2_f32_bf16(qv[4 * c + 2], __builtin_bit_cast(bf16x2, u.z), acc, false);
      acc = __builtin_amdgcn_fdot2_f32_bf16(qv[4 * c + 3], __builtin_bit_cast(bf16x2, u.w), acc, false);
    }
#pragma unroll
    for (int o = 1; o < TS; o <<= 1) acc += __shfl_xor(acc, o, 64);
    sc[j] = j < F ? acc * a.scale_log2 : -INFINITY;
  }
  float m = sc[0];
#pragma unroll
  for (int j = 1; j < 16; ++j) m = fmaxf(m, sc[j]);
  float l = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    // probabilities rounded to bf16 as the PV operand of a bf16 SDPA would be
    sc[j] = (float)(__bf16)fast_exp2(sc[j] - m);
    l += sc[j];
  }
  const float inv = 1.f / l;

  // ---- O[dims ts*DT .. +DT) = sum_j p_j V[j][dim] / l, one 8-dim chunk at a time
  u16* op = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)qi * a.o_si + (long)h * a.o_sh + ts * DT;
#pragma unroll
  for (int c = 0; c < DC; ++c) {
    float o8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float v8[8];
      unpack8(*(const uint4*)(Vs + off + j * C + c * 8), v8);
#pragma unroll
      for (int e = 0; e < 8; ++e) o8[e] = fmaf(sc[j], v8[e], o8[e]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o8[e] *= inv;
    if (live) *(uint4*)(op + c * 8) = pack8(o8);
  }
}

// attn_seqm: the same short-sequence attention on the matrix cores.  A block owns one
// (pixel) sequence -- K and V rows of all heads staged in LDS exactly as above -- and
// each wave takes whole (sequence, head) pairs: S^T = K Q^T as ceil(D/32) 16x16x32
// MFMAs (B = Q^T straight from global, 64-B row segments), the 16 keys of a query
// held 4 per lane so the softmax is 4 registers + two cross-row swaps, and
// O^T = V^T P^T as ceil(D/16) 16x16x16 MFMAs whose B operand is the bf16 P already
// in place and whose A operand comes from ds_read_b64_tr_b16.  Per (pixel, head)
// that is ~60 wave instructions where the dot-product kernel spends ~450, which
// leaves the kernel bound by the q/k/v/o stream.
// Host contract: nq == nk <= 16, heads <= 8 (two per wave), heads contiguous,
// D in {40, 80, 160}, rows 8-element aligned (16-B loads and stores).  HS > 1 splits a
// sequence's heads over HS blocks (blockIdx.y), each staging only its heads' channels:
// d = 160 with all 8 heads would need 82 KB of LDS (one block per CU), 4 heads 41 KB.
template <int D, int HS = 1>
__global__ void __launch_bounds__(256) attn_seqm_kernel(AttnArgs a, int H, int nbatch) {
  constexpr int KC = (D + 31) / 32, ND = (D + 15) / 16;
  const int HB = H / HS;                        // heads of this block
  const int C = HB * D, P = C + 8;              // staged channels, LDS row pitch (elements)
  const int h0 = blockIdx.y * HB;
  const int F = a.nk;
  extern __shared__ __attribute__((aligned(16))) u16 sm[];
  u16* Ks = sm;           // [16][P]
  u16* Vs = sm + 16 * P;  // [16][P]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int lq = lane & 15, lg = lane >> 4;
  const int bz = blockIdx.x;
  if (bz >= nbatch) return;
  const long b1 = bz / a.z2, b2 = bz - b1 * a.z2;

  // Q^T fragments (B operand) of this wave's heads wid and wid + 4, issued first
  bf16x8 qf[2][KC];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int h = wid + 4 * i;  // head within the block
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int d = kc * 32 + lg * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (h < HB && lq < F && d < D)
        v = *(const uint4*)(a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)lq * a.q_si + (long)(h0 + h) * D + d);
      qf[i][kc] = __builtin_bit_cast(bf16x8, v);
    }
  }

  // stage the sequence's K and V rows (zero rows past F)
  const int cpr = C / 8;
  for (int i = tid; i < 16 * cpr; i += 256) {
    const int j = i / cpr, c8 = (i - j * cpr) * 8;
    uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (j < F) {
      kv = *(const uint4*)(a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + (long)j * a.k_si + h0 * D + c8);
      vv = *(const uint4*)(a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + (long)j * a.v_si + h0 * D + c8);
    }
    *(uint4*)(Ks + j * P + c8) = kv;
    *(uint4*)(Vs + j * P + c8) = vv;
  }
  __syncthreads();

  const int qq = lq >> 2, pp = lq & 3;
  u16* ob = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)lq * a.o_si + (long)h0 * D;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int h = wid + 4 * i;
    if (h >= HB) break;
    // s[r] = score(key 4 lg + r, query lq)
    f32x4 s = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int d = kc * 32 + lg * 8;
      uint4 kv = *(const uint4*)(Ks + lq * P + h * D + (d < D ? d : 0));
      if (d >= D) kv = make_uint4(0, 0, 0, 0);  // past the head (pad / next head)
      s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kv), qf[i][kc], s, 0, 0, 0);
    }
    float mt = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] = 4 * lg + r < F ? s[r] * a.scale_log2 : -INFINITY;
      mt = fmaxf(mt, s[r]);
    }
    mt = xor16_32_max(mt);
    float l = 0.f;
    v4i16 pb;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // probabilities rounded to bf16 as the PV operand of a bf16 SDPA would be
      const __bf16 p = (__bf16)fast_exp2(s[r] - mt);
      l += (float)p;
      pb[r] = __builtin_bit_cast(short, p);
    }
    const float inv = 1.f / xor16_32_sum(l);
    const u16* va = Vs + (4 * lg + qq) * P + h * D + 4 * pp;
    uint2 w[ND + 1];
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) {
      const v4i16 vt = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(va + nd * 16));
      const f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vt, pb, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      w[nd] = make_uint2(pack2(o[0] * inv, o[1] * inv), pack2(o[2] * inv, o[3] * inv));
    }
    w[ND] = make_uint2(0, 0);
    // 16-B stores: fragments 2p and 2p+1 trade halves between lane groups (permlane16
    // swap), so every lane holds 8 consecutive dims -- lane group g stores dims
    // 32 p + 16 (g & 1) + 4 (g & 2) .. + 7 (8-B stores were store-issue bound)
#pragma unroll
    for (int p = 0; p < (ND + 1) / 2; ++p) {
      const auto rx = __builtin_amdgcn_permlane16_swap(w[2 * p].x, w[2 * p + 1].x, false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(w[2 * p].y, w[2 * p + 1].y, false, false);
      const int d = 32 * p + 16 * (lg & 1) + 4 * (lg & 2);
      if (lq < F && d < D) *(uint4*)(ob + h * D + d) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
  }
}

template <int D, int HS = 1>
static int launch_seqm(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  const size_t shm = (size_t)2 * 16 * (heads / HS * D + 8) * sizeof(u16);
  if (shm > 64 * 1024) {
    LS_SET_MAX_DYN_SHM((attn_seqm_kernel<D, HS>), (int)shm);
  }
  attn_seqm_kernel<D, HS><<<dim3(batch, HS), 256, shm, s>>>(a, heads, batch);
  return check_launch("attn_seqm_kernel");
}

template <int D, int TS, int NT>
static int launch_seq(const AttnArgs& a, int batch, int heads, hipStream_t s) {
  const int nb = NT / (heads * 16 * TS);
  const int C = heads * D;
  const size_t shm = (size_t)nb * 16 * C * 2 * sizeof(u16);
  LS_SET_MAX_DYN_SHM((attn_seq_kernel<D, TS, NT>), (int)shm);
  attn_seq_kernel<D, TS, NT><<<cdiv(batch, nb), NT, shm, s>>>(a, heads, batch);
  return check_launch("attn_seq_kernel");
}

// ------------------------------------------------- fp8 P V (configs[4])
// attn8: attn5's scheme with the P V product on the block-scaled fp8 MFMA
// (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 x e4m3, fp32 accumulate: twice the bf16
// rate per clock and a quarter of the PV instructions).  QK^T stays on bf16 MFMA:
// at d = 40 the K = 128 fp8 shape would pad the head dim 3.2x, and the softmax is
// the precision-sensitive half.
//
// Operands of O^T += V^T P^T over a 128-key tile, per lane (lq = lane & 15,
// lg = lane >> 4): element j of the 32-byte fragment is key 16 (j >> 2) + 4 lg + (j & 3)
// -- exactly the 32 scores the lane already holds in S^T (keys 16 f + 4 lg + r), so P
// is packed in place (v_cvt_pk_fp8_f32, 16 per 16 queries) with no data movement.
//   P  (B operand): e4m3 with scale 1.  The reference "max" m is an integer 7 below the
//      ceil of the largest score seen when it last moved, so a fresh maximum has p in
//      (2^6, 2^7] and e4m3's normal range (down to 2^-6) reaches 2^-13 below it (with
//      m = max, everything under 2^-6 of the max -- a quarter of a flat softmax row --
//      would sit in e4m3's 2^-9-step subnormals: 1-2 % output error on its own).  m moves
//      when a tile max exceeds it by more than 8, so p <= 2^8 < 448 (e4m3 max).  Being an
//      integer, m only scales every p by a power of two, which e4m3 rounds identically:
//      the result does not depend on the order keys arrive in.
//   V^T (A operand): quantised by vt8_quant_kernel into the caller's workspace, one
//      e8m0 scale per (head dim, 128-key tile) with the row max mapped into [128, 256).
//      Every lane group of a row passes the same scale: a finer per-32-key scale would
//      tie the result to which k the hardware groups under one scale, and a lane-group
//      assignment that differs from it was measured wrong (67 % error) on the box.  Row D
//      is the constant 1.0 column, so O^T row D accumulates sum_k p_k of the same e4m3 p
//      the numerator uses.
// Workspace layout per (batch, head) pair: ceil(nk / 128) tiles of
//   [ND * 16 rows][128 B]  e4m3, row d at d * 128, 16-B chunk c stored at chunk
//                          c ^ ((d >> 1) & 7) (conflict-free ds_read_b128 of 16 rows)
//   [ceil(ND / 4)][64 lanes][4] e8m0 scales: byte nd & 3 of lane (lg, lq)'s dword in
//                          block nd >> 2 is the scale of row 16 nd + lq (equal for all lg)
// so one tile is a contiguous run the attention kernel DMAs straight into LDS.
template <int D>
struct Fp8Tile {
  static constexpr int KC = (D + 31) / 32;       // 32-wide QK^T k-steps (bf16)
  static constexpr int ND = (D + 16) / 16;       // 16-row O^T fragments incl. the sum row
  static constexpr int CPR = D / 8;              // 16-B chunks per K row
  static constexpr int VBYTES = ND * 16 * 128;
  static constexpr int NSC = (ND + 3) / 4;
  static constexpr int TB = VBYTES + NSC * 256;  // workspace bytes per tile
};

__device__ __forceinline__ int fp8_key_of(int lg, int j) { return 16 * (j >> 2) + 4 * lg + (j & 3); }

// e4m3 x e4m3 block-scaled MFMA, A scale = byte `sel` of sa (sel folds to an immediate
// after unrolling), B scale 2^0
__device__ __forceinline__ f32x4 mfma_fp8_mx(const v8i32& a, const v8i32& b, f32x4 c, int sel, int sa) {
  switch (sel) {
    case 0: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 127);
    case 1: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 1, sa, 0, 127);
    case 2: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 2, sa, 0, 127);
    default: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 3, sa, 0, 127);
  }
}

template <int D>
__global__ void __launch_bounds__(256) vt8_quant_kernel(AttnArgs a, uint8_t* ws, long pair_bytes, int heads) {
  using T = Fp8Tile<D>;
  constexpr int R = T::ND * 16;
  constexpr int PITCH = D + 2;  // odd word pitch: column reads are conflict-free
  __shared__ u16 vs[128 * PITCH];
  const int t = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const long b1 = b / a.z2, b2 = b - b1 * a.z2;
  const u16* vb = a.v + b1 * a.v_sb1 + b2 * a.v_sb2 + (long)h * a.v_sh;
  uint8_t* tile = ws + ((long)b * heads + h) * pair_bytes + (long)t * T::TB;
  const int t0 = t * 128;
  for (int i = threadIdx.x; i < 128 * T::CPR; i += 256) {
    const int r = i / T::CPR, c = i - r * T::CPR;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (t0 + r < a.nk) v = *(const uint4*)(vb + (long)(t0 + r) * a.v_si + c * 8);
    uint32_t* dst = (uint32_t*)(vs + r * PITCH + c * 8);
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  __syncthreads();
  // item (d, lg) = thread 4 d + lg: the 4 lane-group blocks of a row sit in adjacent
  // lanes, so the row max is two xor shuffles
  for (int base = 0; base < 4 * R; base += 256) {
    const int it = base + threadIdx.x;
    const int d = it >> 2, lg = it & 3;
    float v[32];
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      v[j] = d < D ? bf2f(vs[fp8_key_of(lg, j) * PITCH + d]) : 0.f;
      amax = fmaxf(amax, fabsf(v[j]));
    }
    amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
    amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
    if (d >= R) continue;
    uint32_t w[8];
    int e8 = 127;
    if (d < D) {
      // row max into [128, 256): floor(log2 amax) - 7 (denormal / zero rows: 2^-127)
      const int ex = (int)((__float_as_uint(amax) >> 23) & 0xff) - 127;
      const int e = amax > 0.f ? ex - 7 : -127;
      e8 = max(0, min(254, e + 127));
      const float inv_s = __uint_as_float((uint32_t)(254 - e8) << 23);  // 2^(127 - e8), e8 <= 247
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        int p = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * f] * inv_s, v[4 * f + 1] * inv_s, 0, false);
        w[f] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v[4 * f + 2] * inv_s, v[4 * f + 3] * inv_s, p, true);
      }
    } else {
      const uint32_t c = d == D ? 0x38383838u : 0u;  // e4m3 1.0: the row-sum column
#pragma unroll
      for (int f = 0; f < 8; ++f) w[f] = c;
    }
    uint8_t* row = tile + d * 128;
    const int sw = (d >> 1) & 7;
    *(uint4*)(row + (((2 * lg) ^ sw) << 4)) = make_uint4(w[0], w[1], w[2], w[3]);
    *(uint4*)(row + (((2 * lg + 1) ^ sw) << 4)) = make_uint4(w[4], w[5], w[6], w[7]);
    const int nd = d >> 4, lq = d & 15;
    tile[T::VBYTES + (nd >> 2) * 256 + (lg * 16 + lq) * 4 + (nd & 3)] = (uint8_t)e8;
  }
}

template <int D, int QG, int NST, bool SB = true, int OCC = 2>
__global__ void __launch_bounds__(256, OCC) attn8_kernel(AttnArgs a, const uint8_t* ws, long pair_bytes, int nqb,
                                                       int heads) {
  using T = Fp8Tile<D>;
  constexpr int KC = T::KC, ND = T::ND, CPR = T::CPR;
  constexpr int KT = 128;
  constexpr int KPL = KC * 4;                       // K planes per 64-key half
  constexpr int PLANE = 64 * 8;                     // u16 per plane (64 keys x 16 B)
  constexpr int KBYTES = 2 * KPL * PLANE * 2;
  constexpr int STAGE = KBYTES + T::TB;             // bytes
  constexpr int NJ = 2 * CPR + 2 * ND + T::NSC;     // DMA instructions per tile
  constexpr int NDMA = (NJ + 3) / 4;                // per wave (dummies pad the rest)
  constexpr float TAU = 8.f;                        // p <= 2^8 < 448 (e4m3 max)
  constexpr int DSUM = D;
  static_assert(NST == 2 || NST == 3, "ring depth");
  extern __shared__ __attribute__((aligned(16))) uint8_t smb[];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lb = attn_xcd_remap(blockIdx.x, gridDim.x);
  const int qblk = lb % nqb, pair = lb / nqb;
  const int h = pair % heads;
  const int b = pair / heads;
  const long b1 = b / a.z2, b2 = b - b1 * a.z2;
  const u16* qb = a.q + b1 * a.q_sb1 + b2 * a.q_sb2 + (long)h * a.q_sh;
  const u16* kb = a.k + b1 * a.k_sb1 + b2 * a.k_sb2 + (long)h * a.k_sh;
  u16* ob = a.o + b1 * a.o_sb1 + b2 * a.o_sb2 + (long)h * a.o_sh;
  const uint8_t* wsp = ws + (long)pair * pair_bytes;
  const int q0 = (qblk * 4 + wid) * 16 * QG;
  const int lq = lane & 15, lg = lane >> 4;

  // K planes past the head dim: zero in every stage and both halves
  for (int i = tid; i < NST * 2 * (KPL - CPR) * 64; i += 256) {
    const int r = i % 64, c = CPR + (i / 64) % (KPL - CPR), hf = (i / (64 * (KPL - CPR))) % 2,
              st = i / (64 * (KPL - CPR) * 2);
    *(uint4*)(smb + st * STAGE + ((hf * KPL + c) * PLANE + r * 8) * 2) = make_uint4(0, 0, 0, 0);
  }

  const float c2 = a.scale_log2;
  bf16x8 qf[QG][KC];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int d = kc * 32 + lg * 8;
      const int q = q0 + g * 16 + lq;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (q < a.nq && d < D) v = *(const uint4*)(qb + (long)q * a.q_si + d);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= c2;
      qf[g][kc] = __builtin_bit_cast(bf16x8, pack8(f));
    }

  const uint32_t kst = (uint32_t)a.k_si * 2;
  const i32x4 krs = buffer_rsrc(kb, (uint32_t)(a.nk - 1) * kst + CPR * 16);
  const i32x4 wrs = buffer_rsrc(wsp, (uint32_t)pair_bytes);
  uint8_t* dummy = smb + NST * STAGE;
  auto issue = [&](int t) {
    uint8_t* st = smb + (t % NST) * STAGE;
#pragma unroll
    for (int u = 0; u < NDMA; ++u) {
      const int j = wid + 4 * u;  // wave-uniform job
      if (j < 2 * CPR) {
        const int hf = j / CPR, c = j - hf * CPR;
        ls_raw_buffer_load_lds(krs, (__attribute__((address_space(3))) void*)(st + (hf * KPL + c) * PLANE * 2), 16,
                               lane * (int)kst + c * 16, (t * KT + 64 * hf) * (int)kst, 0, 0);
      } else if (j < 2 * CPR + 2 * ND) {
        const int i = j - 2 * CPR;
        ls_raw_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(st + KBYTES + i * 1024), 16, lane * 16,
                               t * T::TB + i * 1024, 0, 0);
      } else if (j < NJ) {
        const int i = j - 2 * CPR - 2 * ND;
        ls_raw_buffer_load_lds(wrs, (__attribute__((address_space(3))) void*)(st + KBYTES + T::VBYTES + i * 256), 4,
                               lane * 4, t * T::TB + T::VBYTES + i * 256, 0, 0);
      } else {
        ls_raw_buffer_load_lds(krs, (__attribute__((address_space(3))) void*)dummy, 16, lane * (int)kst,
                               t * KT * (int)kst, 0, 0);
      }
    }
  };

  f32x4 oacc[QG][ND];
#pragma unroll
  for (int g = 0; g < QG; ++g)
#pragma unroll
    for (int i = 0; i < ND; ++i) oacc[g][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // running reference max m (an integer), subtracted through the MFMA's C operand
  float m[QG];
  f32x4 negm[QG];
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    m[g] = 0.f;
    negm[g] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  const int ntile = (a.nk + KT - 1) / KT;
  issue(0);
  if (NST == 3 && ntile > 1) issue(1);
  auto tile = [&](int t, auto partial_tag) {
    constexpr bool PARTIAL = decltype(partial_tag)::value;
    const int t0 = t * KT;
    if (NST == 3 && t + 1 < ntile) attn_wait_vm<NDMA>();  // tile t landed; t+1 may fly
    else attn_wait_vm<0>();
    __syncthreads();                                      // everyone's; slot (t-1) % NST free
    if (t + NST - 1 < ntile) issue(t + NST - 1);
    const uint8_t* st = smb + (t % NST) * STAGE;
    const u16* Ks = (const u16*)st;
    const uint8_t* Vt = st + KBYTES;
    const uint32_t* Sc = (const uint32_t*)(st + KBYTES + T::VBYTES);
    auto pv = [&](const v8i32* pkv) {
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) {
      const int d = 16 * nd + lq;
      const uint8_t* row = Vt + d * 128;
      const int sw = (d >> 1) & 7;
      const uint4 lo = *(const uint4*)(row + (((2 * lg) ^ sw) << 4));
      const uint4 hi = *(const uint4*)(row + (((2 * lg + 1) ^ sw) << 4));
      const v8i32 va = {(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
      const int sc = (int)Sc[(nd >> 2) * 64 + lane];
#pragma unroll
      for (int g = 0; g < QG; ++g)
        oacc[g][nd] = mfma_fp8_mx(va, pkv[g], oacc[g][nd], nd & 3, sc);
    }
    };
    // two 64-key halves: scores of one half live in registers at a time (QG * 16
    // VGPRs); each half's P goes to e4m3 at once (8 bytes per f32x4 of scores)
    v8i32 pk[QG];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      bool first = t == 0 && hf == 0;
      f32x4 s[QG][4];
      auto qk = [&]() {
#pragma unroll
      for (int f = 0; f < 4; ++f) {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const bf16x8 kf = __builtin_bit_cast(
              bf16x8, *(const uint4*)(Ks + (hf * KPL + kc * 4 + lg) * PLANE + (16 * f + lq) * 8));
#pragma unroll
          for (int g = 0; g < QG; ++g)
            s[g][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[g][kc], kc == 0 ? negm[g] : s[g][f], 0,
                                                              0, 0);
        }
      }
      };
      qk();
      bool again;
      {
        float mt[QG];
        bool need_any = first;
#pragma unroll
        for (int g = 0; g < QG; ++g) {
          if (PARTIAL) {
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (t0 + 64 * hf + 16 * f + 4 * lg + r >= a.nk) s[g][f][r] = -INFINITY;
          }
          float x = __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][0][0], s[g][0][1]),
                                                  __builtin_elementwise_maximum(s[g][0][2], s[g][0][3]));
#pragma unroll
          for (int f = 1; f < 4; ++f)
            x = __builtin_elementwise_maximum(
                x, __builtin_elementwise_maximum(__builtin_elementwise_maximum(s[g][f][0], s[g][f][1]),
                                                 __builtin_elementwise_maximum(s[g][f][2], s[g][f][3])));
          mt[g] = xor16_32_max(x);
          need_any |= mt[g] > TAU;
        }
        again = __builtin_amdgcn_ballot_w64(need_any) != 0;
        if (again) {
          if (hf == 1) {
            // the first half's P was packed against the old m: accumulate it now (second
            // half zero) so the rescale below applies to it
#pragma unroll
            for (int g = 0; g < QG; ++g)
#pragma unroll
              for (int f = 4; f < 8; ++f) pk[g][f] = 0;
            pv(pk);
#pragma unroll
            for (int g = 0; g < QG; ++g)
#pragma unroll
              for (int f = 0; f < 4; ++f) pk[g][f] = 0;
          }
#pragma unroll
          for (int g = 0; g < QG; ++g) {
            const bool need = first || mt[g] > TAU;
            // new m: an integer 7 below the ceil of the tile max (its p in (2^6, 2^7])
            const float dlt = need ? ceilf(mt[g]) - 7.f : 0.f;
            const float alpha = first ? 0.f : fast_exp2(-dlt);
            m[g] += dlt;
            negm[g] = (f32x4){-m[g], -m[g], -m[g], -m[g]};
#pragma unroll
            for (int f = 0; f < 4; ++f) s[g][f] -= dlt;
#pragma unroll
            for (int i = 0; i < ND; ++i) oacc[g][i] *= alpha;
          }
          first = false;
        }
      }
      // P^T in e4m3, element j = 4 f + r at byte j (key 16 f + 4 lg + r, f = 4 hf + f')
#pragma unroll
      for (int g = 0; g < QG; ++g)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const int lo = __builtin_amdgcn_cvt_pk_fp8_f32(fast_exp2(s[g][f][0]), fast_exp2(s[g][f][1]), 0, false);
          pk[g][4 * hf + f] = __builtin_amdgcn_cvt_pk_fp8_f32(fast_exp2(s[g][f][2]), fast_exp2(s[g][f][3]), lo, true);
        }
      if (SB) __builtin_amdgcn_sched_barrier(0);  // keep one half's scores live at a time
    }
    pv(pk);
  };
  const int nfull = a.nk / KT;
  for (int t = 0; t < nfull; ++t) tile(t, std::false_type{});
  if (nfull < ntile) tile(nfull, std::true_type{});
#pragma unroll
  for (int g = 0; g < QG; ++g) {
    constexpr int NDL = DSUM / 16, LGL = (DSUM % 16) / 4, RL = DSUM % 4;
    const float lt = __shfl(oacc[g][NDL][RL], LGL * 16 + lq, 64);
    const float inv = 1.f / lt;
    const int q = q0 + g * 16 + lq;
    if (q < a.nq) {
      u16* orow = ob + (long)q * a.o_si;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        const int d = nd * 16 + 4 * lg;
        if (d + 3 < D) {
          uint2 w;
          w.x = pack2(oacc[g][nd][0] * inv, oacc[g][nd][1] * inv);
          w.y = pack2(oacc[g][nd][2] * inv, oacc[g][nd][3] * inv);
          *(uint2*)(orow + d) = w;
        }
      }
    }
  }
}

template <int D>
static long fp8_pair_bytes(int nk) {
  return (long)cdiv(nk, 128) * Fp8Tile<D>::TB;
}

template <int D, int QG, int NST, bool SB = true, int OCC = 2>
static int launch_attn8(const AttnArgs& a, int batch, int heads, uint8_t* ws, hipStream_t s) {
  using T = Fp8Tile<D>;
  const long pb = fp8_pair_bytes<D>(a.nk);
  if (pb >= (1L << 31)) return fail(LS_ERR_INVALID, "ls_attention_fp8: key set too long");
  vt8_quant_kernel<D><<<dim3(cdiv(a.nk, 128), heads, batch), 256, 0, s>>>(a, ws, pb, heads);
  int rc = check_launch("vt8_quant_kernel");
  if (rc) return rc;
  const int nqb = cdiv(a.nq, 4 * 16 * QG);
  const long nblk = (long)nqb * heads * batch;
  if (nblk > 0x7fffffff) return fail(LS_ERR_INVALID, "ls_attention_fp8: grid too large");
  constexpr int STAGE = 2 * T::KC * 4 * 64 * 8 * 2 + T::TB;
  const size_t shm = (size_t)NST * STAGE + 1024;
  LS_SET_MAX_DYN_SHM((attn8_kernel<D, QG, NST, SB, OCC>), (int)shm);
  attn8_kernel<D, QG, NST, SB, OCC><<<(int)nblk, 256, shm, s>>>(a, ws, pb, nqb, heads);
  return check_launch("attn8_kernel");
}

}  // namespace ls

using namespace ls;

static bool g_attn_v1 = ls_env("LS_ATTN_V1") != nullptr;  // A/B switch: force the 16-query kernel
static bool g_attn_v3 = ls_env("LS_ATTN_V3") != nullptr;  // A/B switch: attn3 for d = 40 too
// A/B switch: d = 40 self attention on attn6 (32x32x16); measured 3 % slower than attn5 at 48
// windows (1670 vs 1620 us per call, profiles/r04b_attn6_vs_attn5_ab.txt), so attn5 stays the default
#ifdef LS_DIAG_KERNELS
static bool g_attn6 = ls_env("LS_ATTN6") != nullptr;
#else
static bool g_attn6 = false;
#endif
namespace ls {
void attn_set_attn6(bool on) { g_attn6 = on; }  // ls_set_tuning key 9 (diagnostics build)
}
static bool g_attnw_off = ls_env("LS_ATTNW_OFF") != nullptr;  // A/B switch: d = 512 on attn_kernel
static bool g_seq_valu = ls_env("LS_ATTN_SEQ_VALU") != nullptr;  // A/B switch: dot-product short-sequence kernel
static bool g_seq160_valu = ls_env("LS_ATTN_SEQ160_VALU") != nullptr;  // A/B switch: ... for d = 160 only

static AttnArgs attn_args(const ls_attn_desc* d) {
  AttnArgs a;
  a.q = d->q; a.k = d->k; a.v = d->v; a.o = d->o;
  a.q_sb1 = d->q_sb1; a.q_sb2 = d->q_sb2; a.q_si = d->q_si; a.q_sh = d->q_sh;
  a.k_sb1 = d->k_sb1; a.k_sb2 = d->k_sb2; a.k_si = d->k_si; a.k_sh = d->k_sh;
  a.v_sb1 = d->v_sb1; a.v_sb2 = d->v_sb2; a.v_si = d->v_si; a.v_sh = d->v_sh;
  a.o_sb1 = d->o_sb1; a.o_sb2 = d->o_sb2; a.o_si = d->o_si; a.o_sh = d->o_sh;
  a.z2 = d->z2; a.nq = d->nq; a.nk = d->nk; a.D = d->head_dim;
  a.scale_log2 = d->scale * 1.4426950408889634f;
  a.o16 = ((uintptr_t)d->o & 15) == 0 && d->o_si % 8 == 0 && d->o_sh % 8 == 0 && d->o_sb1 % 8 == 0 &&
          d->o_sb2 % 8 == 0;
  return a;
}

static int attn_check(const ls_attn_desc* d, const char* who) {
  if (!d || !d->q || !d->k || !d->v || !d->o) return fail(LS_ERR_INVALID, std::string(who) + ": null pointer");
  if (d->head_dim % 2 || d->head_dim <= 0 || d->head_dim > 512 || d->nq <= 0 || d->nk <= 0 || d->batch <= 0 ||
      d->z2 <= 0 || d->heads <= 0)
    return fail(LS_ERR_INVALID, std::string(who) + ": bad shape (head_dim even, <= 512)");
  return LS_OK;
}

extern "C" size_t ls_attention_fp8_workspace_bytes(const ls_attn_desc* d) {
  if (!d || d->nk <= 0 || d->batch <= 0 || d->heads <= 0) return 0;
  const long pairs = (long)d->batch * d->heads;
  switch (d->head_dim) {
    case 40: return (size_t)(pairs * fp8_pair_bytes<40>(d->nk));
    case 80: return (size_t)(pairs * fp8_pair_bytes<80>(d->nk));
    default: return 0;
  }
}

extern "C" int ls_attention_fp8(const ls_attn_desc* d, void* workspace, size_t workspace_bytes, void* stream) {
  if (int rc = attn_check(d, "ls_attention_fp8")) return rc;
  const int D = d->head_dim;
  if (D != 40 && D != 80) return fail(LS_ERR_INVALID, "ls_attention_fp8: head_dim must be 40 or 80");
  const bool aligned = d->q_si % 8 == 0 && d->k_si % 8 == 0 && d->v_si % 8 == 0 && d->q_sh % 8 == 0 &&
                       d->k_sh % 8 == 0 && d->v_sh % 8 == 0 && d->q_sb1 % 8 == 0 && d->q_sb2 % 8 == 0 &&
                       d->k_sb1 % 8 == 0 && d->k_sb2 % 8 == 0 && d->v_sb1 % 8 == 0 && d->v_sb2 % 8 == 0 &&
                       (((uintptr_t)d->q | (uintptr_t)d->k | (uintptr_t)d->v) & 15) == 0 && d->o_si % 2 == 0 &&
                       d->o_sh % 2 == 0 && d->o_sb1 % 2 == 0 && d->o_sb2 % 2 == 0 && ((uintptr_t)d->o & 7) == 0;
  if (!aligned) return fail(LS_ERR_INVALID, "ls_attention_fp8: q/k/v rows must be 16-B aligned, o rows 8-B");
  if (((long)d->nk + 128) * d->k_si * 2 >= (1L << 31)) return fail(LS_ERR_INVALID, "ls_attention_fp8: key set too long");
  const size_t need = ls_attention_fp8_workspace_bytes(d);
  if (!workspace || workspace_bytes < need || ((uintptr_t)workspace & 15))
    return fail(LS_ERR_WORKSPACE, "ls_attention_fp8: workspace missing, unaligned or smaller than "
                                  "ls_attention_fp8_workspace_bytes");
  const AttnArgs a = attn_args(d);
  hipStream_t s = (hipStream_t)stream;
  uint8_t* ws = (uint8_t*)workspace;
  static const int variant = ls_env("LS_ATTN8_VARIANT") ? atoi(ls_env("LS_ATTN8_VARIANT")) : 0;  // A/B switch
  if (D == 40) {
    if (variant == 1) return launch_attn8<40, 2, 2, false, 3>(a, d->batch, d->heads, ws, s);
    if (variant == 2) return launch_attn8<40, 2, 2, true, 2>(a, d->batch, d->heads, ws, s);
    if (variant == 3) return launch_attn8<40, 3, 3, true, 2>(a, d->batch, d->heads, ws, s);
    return launch_attn8<40, 2, 2, true, 3>(a, d->batch, d->heads, ws, s);
  }
  return launch_attn8<80, 2, 2>(a, d->batch, d->heads, ws, s);
}

extern "C" int ls_attention(const ls_attn_desc* d, void* stream) {
  if (int rc = attn_check(d, "ls_attention")) return rc;
  const AttnArgs a = attn_args(d);
  hipStream_t s = (hipStream_t)stream;
  const bool small = d->nk <= 32;
  const int D = d->head_dim;
  // short sequences (the temporal attention over a window's frames): whole-row kernel
  {
    const int H = d->heads, TS = D / 40;
    const bool heads_packed = d->q_sh == D && d->k_sh == D && d->v_sh == D && d->o_sh == D;
    const bool aligned = d->q_si % 8 == 0 && d->k_si % 8 == 0 && d->v_si % 8 == 0 && d->o_si % 8 == 0 &&
                         d->q_sb1 % 8 == 0 && d->q_sb2 % 8 == 0 && d->k_sb1 % 8 == 0 && d->k_sb2 % 8 == 0 &&
                         d->v_sb1 % 8 == 0 && d->v_sb2 % 8 == 0 && d->o_sb1 % 8 == 0 && d->o_sb2 % 8 == 0 &&
                         (((uintptr_t)d->q | (uintptr_t)d->k | (uintptr_t)d->v | (uintptr_t)d->o) & 15) == 0;
    if (!g_attn_v1 && d->nq == d->nk && d->nk <= 16 && heads_packed && aligned && D % 40 == 0 &&
        (TS == 1 || TS == 2 || TS == 4) && H * 16 * TS <= 512 && 512 % (H * 16 * TS) == 0) {
      // heads split over 2 blocks at d = 80 (20 KB of LDS per block: 146 -> 142 us at 32 windows)
      // and d = 160 (41 KB: 111 -> 83 us); d = 40 keeps all heads in one block (295 vs 340 us)
      if (!g_seq_valu && D == 40 && H <= 8) return launch_seqm<40>(a, d->batch, H, s);
      if (!g_seq_valu && D == 80 && H <= 8)
        return H % 2 == 0 ? launch_seqm<80, 2>(a, d->batch, H, s) : launch_seqm<80>(a, d->batch, H, s);
      if (!g_seq_valu && !g_seq160_valu && D == 160 && H <= 8 && H % 2 == 0)
        return launch_seqm<160, 2>(a, d->batch, H, s);
      // 256-thread blocks (several per CU desynchronise the load and compute phases)
      // wherever one (sequence, head) set fits
      const bool small_blk = H * 16 * TS <= 256 && 256 % (H * 16 * TS) == 0;
      if (D == 40) return small_blk ? launch_seq<40, 1, 256>(a, d->batch, H, s) : launch_seq<40, 1, 512>(a, d->batch, H, s);
      if (D == 80) return small_blk ? launch_seq<80, 2, 256>(a, d->batch, H, s) : launch_seq<80, 2, 512>(a, d->batch, H, s);
      if (D == 160) return launch_seq<160, 4, 512>(a, d->batch, H, s);
    }
  }
  if (!small && D % 8 == 0 && D <= 160 && !g_attn_v1) {
    // d = 40 self attention (the UNet's 32x32 / 64x64 levels): the DMA-fed kernel, 64
    // queries per wave, row sums from the PV MFMA; short key sets (the 50 audio tokens)
    // and other head dims: attn3 (register-staged tiles)
    if (D == 40 && !g_attn_v3 && d->nk > 128 && ((long)(d->nk - 1) * std::max(d->k_si, d->v_si) + D) * 2 < (1L << 31))
#ifdef LS_DIAG_KERNELS
      if (g_attn6) return launch_attn6<40>(a, d->batch, d->heads, s);
#endif
      return launch_attn5<2, 3, 40, 4>(a, d->batch, d->heads, s);
    if (D == 40) return launch_attn3<2, 3, 40>(a, d->batch, d->heads, s);
    switch ((D + 15) / 16) {
      case 1: case 2: return launch_attn3<1, 2, 0>(a, d->batch, d->heads, s);
      case 3: return launch_attn3<2, 3, 0>(a, d->batch, d->heads, s);
      case 4: return launch_attn3<2, 4, 0>(a, d->batch, d->heads, s);
      case 5: return launch_attn3<3, 5, 0>(a, d->batch, d->heads, s);
      case 6: return launch_attn3<3, 6, 0>(a, d->batch, d->heads, s);
      case 7: case 8: return launch_attn3<4, 8, 0>(a, d->batch, d->heads, s);
      default: return launch_attn3<5, 10, 0>(a, d->batch, d->heads, s);
    }
  }
  // d = 512 (the VAE mid attention): the head dim split over wave pairs (attnw)
  if (D == 512 && !g_attn_v1 && !g_attnw_off && d->q_si % 8 == 0 && d->k_si % 8 == 0 && d->v_si % 8 == 0 &&
      d->o_si % 4 == 0 && (((uintptr_t)d->q | (uintptr_t)d->k | (uintptr_t)d->v) & 15) == 0 &&
      ((uintptr_t)d->o & 7) == 0 && (d->q_sb1 | d->q_sb2 | d->q_sh | d->k_sb1 | d->k_sb2 | d->k_sh | d->v_sb1 |
                                      d->v_sb2 | d->v_sh) % 8 == 0 &&
      (d->o_sb1 | d->o_sb2 | d->o_sh) % 4 == 0 &&
      ((long)(d->nk + 32) * std::max(d->k_si, d->v_si) + D) * 2 < (1L << 31))
    return launch_attnw512(a, d->batch, d->heads, s);
#define LS_ATTN(DPV)                                                              \
  return small ? launch_attn<DPV, 2>(a, d->batch, d->heads, s)                    \
               : launch_attn<DPV, 4>(a, d->batch, d->heads, s);
  if (D <= 64) { LS_ATTN(64) }
  if (D <= 96) { LS_ATTN(96) }
  if (D <= 160) { LS_ATTN(160) }
  if (D <= 256) { LS_ATTN(256) }
  LS_ATTN(512)
#undef LS_ATTN
}
