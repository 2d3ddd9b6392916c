// Temporal self-attention of the motion module fused with its input projections
// (gfx950).  Replaces, per VersatileAttention block of a TemporalTransformerBlock
// (latentsync/models/motion_module.py:203-218 norms + :262-313 forward):
//
//   norm_hidden = LayerNorm(h)                                  (:207, nn.LayerNorm, eps 1e-5)
//   x = rearrange(norm_hidden, "(b f) s c -> (b s) f c") + pe[:f] (:281-285, PositionalEncoding)
//   q, k, v = to_q(x), to_k(x), to_v(x)                          (:296-303, no bias)
//   o = SDPA(q, k, v) over the f frames, 8 heads                 (:300)
//   o -> "(b s) f c -> (b f) s c"                                (:311)
//
// i.e. everything up to (not including) to_out, which stays the row-block GEMM with
// its residual epilogue.  Before this kernel the path was: a q|k|v GEMM writing 3C
// per row to HBM, then a short-sequence attention kernel reading it back and writing
// o -- two launches and two extra full-tensor round trips per attention block.
//
// Layout.  A workgroup owns 2*WAVES pixels of one sample x all F (<= 16) frames; wave
// w owns FM pixels as FM 16-row MFMA fragments whose row (lane & 15) is the
// FRAME.  So a fragment is exactly one pixel's temporal sequence: the attention over
// frames is wave-local, with no rearrange and no LDS.  The rows are gathered straight
// from the (b f) s c activation (row (b*F + f)*S + s).
//   * The wave's A rows (2 x 16 rows x C, bf16) live in registers; LayerNorm (+ the
//     positional-encoding row of the lane's frame) is applied to them in place.
//   * The packed q|k|v weights stream through an LDS ring by global_load_lds DMA, in
//     sub-chunks of 48 (C = 320, 2 stages) or 16 (C = 640, 3 stages) output columns.  Columns are packed per
//     80-wide group (2 heads at d = 40, 1 head at d = 80) as (q_t, k_t, v_t), t = 0..4:
//     16-channel tiles of q, k and v in turn.
//   * q and k tiles are computed transposed (C^T = W A^T: a lane holds 4 consecutive
//     columns of its frame row), v tiles non-transposed (C = A W^T: a lane holds one
//     channel d for 4 consecutive frames) -- which is exactly the A operand V^T of the
//     16x16x16 P.V MFMA, so V is never transposed through LDS.
//   * S^T = K Q^T accumulates per 16-channel tile as soon as q_t and k_t exist (16x16x16
//     MFMAs whose operands are the C^T accumulators as they stand: key / query row,
//     4 channels; Q masked to the head), so q and k never wait in registers; at the
//     group's end the softmax over the 16 keys is 4 registers + two cross-row swaps
//     and O^T = V^T P^T (16x16x16) lands as 4 consecutive channels of the query
//     frame's row: the layout of the o tensor, stored 16 B per lane.
// The q rows of W are pre-scaled by log2(e)/sqrt(d) on the host, so scores are in
// log2 units and the softmax uses the bare v_exp_f32.
// Config (TCfg): 4-wave blocks, C = 320 (d 40) two pixels per wave, two blocks per CU;
// C = 640 (d 80) one pixel per wave.
#include "ls_common.h"

typedef short v4i16 __attribute__((ext_vector_type(4)));

namespace ls {

struct TAttnArgs {
  const u16* x;
  const float* gamma;  // [C] LayerNorm weight
  const float* bpe;    // [16][C] LayerNorm bias + positional-encoding row f
  const u16* w;        // [3C][C] packed q|k|v rows (see above)
  u16* o;
  int ldx, ldo, F, S, blocks_per_sample;
  float eps;
  int ablate;  // diagnostic builds only (-DLS_TATTN_ABLATE, env LS_TATTN_ABLATE): parts skipped
};

#ifdef LS_TATTN_ABLATE
#define ABL(bit) (a.ablate & (bit))
#else
#define ABL(bit) false
#endif

// Blocks are small enough that two run on a CU at once: one
// block's row gather, LayerNorm, softmax and o stores then overlap another block's
// MFMAs (with one 8-wave block per CU those phases left the matrix pipe idle: ablation,
// DESIGN.md §3).
template <int C>
struct TCfg {
  static constexpr int WAVES = 4;
  static constexpr int FM = C == 320 ? 2 : 1;       // 16-row fragments (= pixels) per wave
  static constexpr int MINB = 2;                    // resident blocks per CU
  static constexpr int NT = WAVES * 64;
  static constexpr int KT = C / 32;                 // 32-wide k-steps of the A rows
  static constexpr int NG = C / 80;                 // 80-column groups
  static constexpr int D = C / 8;                   // head dim
  static constexpr int HG = 80 / D;                 // heads per group
  static constexpr int FN = C == 320 ? 3 : 1;       // 16-column tiles per W sub-chunk
  static constexpr int NSC = 15 / FN;               // sub-chunks per group (tiles q_t, k_t, v_t)
  static constexpr int BN = 16 * FN;                // W rows per sub-chunk
  static constexpr int STAGE = (C / 64) * BN * 8;   // 16-B slots per LDS stage
  static constexpr int NST = C == 320 ? 2 : 3;      // LDS ring depth (30 / 20 KB stages, <= 80 KB per block)
  static constexpr int DPW = (STAGE / 64 + WAVES - 1) / WAVES;  // DMA wave-instructions per wave per stage
  static constexpr int PPB = FM * WAVES;            // pixels per block
};

__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ uint2 pack4(const f32x4& v, float s) {
  return make_uint2(pack2(v[0] * s, v[1] * s), pack2(v[2] * s, v[3] * s));
}

// 8 bf16 (a 32-wide k-step operand) from two 4-column tile halves
__device__ __forceinline__ bf16x8 kstep(uint2 lo, uint2 hi) {
  return __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

template <int C>
__global__ void __launch_bounds__(TCfg<C>::NT, TCfg<C>::MINB) tattn_fused_kernel(TAttnArgs a) {
  using T = TCfg<C>;
  constexpr int KT = T::KT, NT = T::NT, BN = T::BN, STAGE = T::STAGE, NSC = T::NSC, NG = T::NG;
  constexpr int D = T::D, HG = T::HG, FN = T::FN, FM = T::FM;
  extern __shared__ __attribute__((aligned(16))) uint4 lds_w[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, lg = lane >> 4;
  const int b = blockIdx.x / a.blocks_per_sample, pg = blockIdx.x - b * a.blocks_per_sample;
  const int s0 = pg * T::PPB + FM * wid;  // this wave's pixels s0 .. s0 + FM - 1
  const int f = l16;                             // the frame of this lane's rows
  const bool live = f < a.F;
  const long row0 = ((long)b * a.F + f) * a.S + s0;

  // sub-chunk c (W rows [c BN, c BN + BN) x all C) -> stage: KT/2 64-wide swizzled images.
  // Every wave issues exactly DPW DMA instructions per stage (the spare ones re-fetch
  // row 0 into a dummy slot), so "stage c landed" is one constant vmcnt for all waves.
  // (round 6) buffer-descriptor DMA: per-thread byte offsets fixed over the sub-chunks, the
  // sub-chunk in the uniform soffset, LDS-space destinations, and the live / spare choice on
  // the scalar wave index -- the generic-address form spent ~5 VALU / SALU per DMA on a 64-bit
  // address, a readfirstlane for M0 and an exec-masked branch
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  __builtin_assume(wid_u >= 0 && wid_u < T::WAVES);
  const i32x4 rs_w = buffer_rsrc(a.w, (uint32_t)min(3L * C * C * 2, 0x7FFFFFFFL));
  int wvo[T::DPW];
#pragma unroll
  for (int p = 0; p < T::DPW; ++p) {
    const int u = p * T::WAVES + wid_u;  // wave-instruction index within the stage
    const int q = u * 64 + lane, t = q / (8 * BN), row = (q >> 3) % BN, pc = q & 7;
    const int lc = pc ^ ((row >> 1) & 7);
    wvo[p] = (STAGE % (64 * T::WAVES) == 0 || u < STAGE / 64) ? (row * C + t * 64 + lc * 8) * 2 : lane * 16;
  }
  lds_u4* const lbase = (lds_u4*)lds_w;
  lds_u4* const dummy_l = lbase + T::NST * STAGE;
  auto issue = [&](int c) {
    lds_u4* const dst = lbase + (c % T::NST) * STAGE;
#pragma unroll
    for (int p = 0; p < T::DPW; ++p) {
      const int u = p * T::WAVES + wid_u;  // (wave-uniform)
      const bool live = STAGE % (64 * T::WAVES) == 0 || u < STAGE / 64;
      ls_raw_buffer_load_lds(rs_w, (__attribute__((address_space(3))) void*)(live ? dst + u * 64 : dummy_l), 16, wvo[p],
                             c * BN * C * 2, 0, 0);
    }
  };

  // ---- A rows -> registers (lane: frame row, 8 consecutive channels per k-step)
  bf16x8 ar[FM][KT];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const u16* src = a.x + (row0 + i) * a.ldx + lg * 8;
#pragma unroll
    for (int s = 0; s < KT; ++s)
      ar[i][s] = live && !ABL(16) ? *(const bf16x8*)(src + s * 32) : __builtin_bit_cast(bf16x8, make_uint4(0, 0, 0, 0));
  }
  constexpr int NC = NG * NSC;  // sub-chunks in all
  constexpr int PD = T::NST - 1;  // prefetch distance
#pragma unroll
  for (int c = 0; c < PD; ++c) issue(c);
  // ---- LayerNorm over the C channels of each row (the 4 lane groups of a frame hold
  // disjoint quarters), two-pass in fp32; then (x - mean) rstd gamma + (beta + pe[f])
  float mean[FM], rstd[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    float t = 0.f;
#pragma unroll
    for (int s = 0; s < KT; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) t += (float)ar[i][s][e];
    mean[i] = xor16_32_sum(t) * (1.f / C);
    float q = 0.f;
#pragma unroll
    for (int s = 0; s < KT; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (float)ar[i][s][e] - mean[i];
        q = fmaf(d, d, q);
      }
    rstd[i] = rsqrtf(xor16_32_sum(q) * (1.f / C) + a.eps);
  }
  {
    const float* bp = a.bpe + f * C + lg * 8;
    const float* gm = a.gamma + lg * 8;
#pragma unroll
    for (int s = 0; s < KT; ++s) {
      float g8[8], b8[8];
      load8f(gm + s * 32, g8);
      load8f(bp + s * 32, b8);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        bf16x8 v = ar[i][s];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (__bf16)fmaf(((float)v[e] - mean[i]) * rstd[i], g8[e], b8[e]);
        ar[i][s] = v;
      }
    }
  }
  // The packed rows of a group come as (q_t, k_t, v_t) for t = 0..4 (16 channels each), so
  // S^T = K Q^T accumulates tile by tile (16x16x16 MFMAs straight from the q / k
  // accumulators) and only v^T has to stay in registers until the softmax.
  f32x4 sacc[FM][HG];  // S^T of (fragment, head): key 4 lg + r, query l16
  uint2 qt[FM];        // the current tile's q (C^T layout: frame row, 4 channels)
  v4i16 vt[FM][5];     // v^T tiles (channel rows, 4 frames per lane)

  for (int g = 0; g < NG; ++g) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int hh = 0; hh < HG; ++hh) sacc[i][hh] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sc = 0; sc < NSC; ++sc) {
      const int c = g * NSC + sc;
      // this wave's DMA of sub-chunk c landed (the PD - 1 younger sub-chunks may still fly;
      // o stores issued since are younger still: waiting past them is only early)
      const int younger = NC - 1 - c < PD - 1 ? NC - 1 - c : PD - 1;
      if (younger >= PD - 1) wait_vm<(PD - 1) * T::DPW>();
      else if (PD >= 3 && younger == 1) wait_vm<T::DPW>();
      else wait_vm<0>();
      lds_sync();  // ... everyone's; the stage of sub-chunk c - 1 is free again
      if (c + PD < NC && !ABL(4)) issue(c + PD);
      const uint4* cur = lds_w + (c % T::NST) * STAGE;
      f32x4 acc[FM][FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      // fragments of k-step s + 1 are read while the MFMAs of k-step s issue (double
      // buffer), so the LDS latency hides behind this wave's own matrix work
      auto frag = [&](int s, int j) {
        return __builtin_bit_cast(bf16x8, cur[(s >> 1) * (8 * BN) + swz_bk<64>(j * 16 + l16, (s & 1) * 4 + lg)]);
      };
      bf16x8 bw[2][FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bw[0][j] = frag(0, j);
#pragma unroll
      for (int s = 0; s < (ABL(2) ? 0 : KT); ++s) {
        if (s + 1 < KT) {
#pragma unroll
          for (int j = 0; j < FN; ++j) bw[(s + 1) & 1][j] = frag(s + 1, j);
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if ((sc * FN + j) % 3 == 2)  // v: C = A W^T
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar[i][s], bw[s & 1][j], acc[i][j], 0, 0, 0);
            else                         // q, k: C^T = W A^T
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[s & 1][j], ar[i][s], acc[i][j], 0, 0, 0);
          }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int idx = sc * FN + j, kind = idx % 3, t = idx / 3;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const uint2 pk = pack4(acc[i][j], 1.f);
          if (kind == 0) {
            qt[i] = pk;
          } else if (kind == 1) {
            // S^T += K_t Q_t^T over the tile's 16 channels, per head (Q masked to it)
#pragma unroll
            for (int hh = 0; hh < HG; ++hh) {
              if (16 * t >= hh * D + D || 16 * t + 16 <= hh * D) continue;  // (compile time)
              const int cl = 16 * t + 4 * lg;
              const uint2 q = (cl >= hh * D && cl < hh * D + D) ? qt[i] : make_uint2(0, 0);
              sacc[i][hh] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(
                  __builtin_bit_cast(v4i16, pk), __builtin_bit_cast(v4i16, q), sacc[i][hh], 0, 0, 0);
            }
          } else {
            vt[i][t] = __builtin_bit_cast(v4i16, pk);
          }
        }
      }

      if (sc == NSC - 1 && !ABL(1)) {
        // ---- softmax + P V of this group's heads, per fragment (pixel)
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          uint2 ot[6];
          ot[5] = make_uint2(0, 0);
#pragma unroll
          for (int hh = 0; hh < HG; ++hh) {
            const int d0 = hh * D, d1 = d0 + D;  // the head's columns within the group
            f32x4 sv = sacc[i][hh];              // score(key 4 lg + r, query l16), log2 units
            float m = -INFINITY;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (4 * lg + r >= a.F) sv[r] = -INFINITY;
              m = fmaxf(m, sv[r]);
            }
            m = xor16_32_max(m);
            float l = 0.f;
            v4i16 pb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              // probabilities rounded to bf16, as the P.V operand of a bf16 SDPA
              const __bf16 p = (__bf16)fast_exp2(sv[r] - m);
              l += (float)p;
              pb[r] = __builtin_bit_cast(short, p);
            }
            const float inv = 1.f / xor16_32_sum(l);
#pragma unroll
            for (int dt = 0; dt < 5; ++dt) {
              if (16 * dt >= d1 || 16 * dt + 16 <= d0) continue;  // (compile time)
              const f32x4 o = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(vt[i][dt], pb, (f32x4){0.f, 0.f, 0.f, 0.f},
                                                                         0, 0, 0);
              const uint2 w = pack4(o, inv);  // O^T: channels 16 dt + 4 lg + r of query frame l16
              const int cl = 16 * dt + 4 * lg;
              if (16 * dt >= d0 && 16 * dt + 16 <= d1) ot[dt] = w;
              else if (cl >= d0 && cl < d1) ot[dt] = w;
              else if (hh == 0) ot[dt] = make_uint2(0, 0);
            }
          }
          // 16-B stores: tiles 2p and 2p+1 trade halves between lane groups (permlane16
          // swap) so lane group q holds channels 32p + 16 (q & 1) + 4 (q & 2) .. + 7
          u16* orow = a.o + (row0 + i) * a.ldo + g * 80;
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            const auto rx = __builtin_amdgcn_permlane16_swap(ot[2 * p].x, ot[2 * p + 1].x, false, false);
            const auto ry = __builtin_amdgcn_permlane16_swap(ot[2 * p].y, ot[2 * p + 1].y, false, false);
            const int d = 32 * p + 16 * (lg & 1) + 4 * (lg & 2);
            if (live && d < 80 && !ABL(8)) *(uint4*)(orow + d) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
          }
        }
      }
    }
  }
}

template <int C>
static int launch_tattn(const TAttnArgs& a, int grid, hipStream_t s) {
  using T = TCfg<C>;
  const size_t shm = ((size_t)T::NST * T::STAGE + 64) * 16;  // ring + the dummy DMA slot
  LS_SET_MAX_DYN_SHM((tattn_fused_kernel<C>), (int)shm);
  tattn_fused_kernel<C><<<grid, T::NT, shm, s>>>(a);
  return check_launch("tattn_fused_kernel");
}

}  // namespace ls

using namespace ls;

extern "C" int ls_temporal_attention(const ls_tattn_desc* d, void* stream) {
  if (!d || !d->x || !d->gamma || !d->bpe || !d->w || !d->o) return fail(LS_ERR_INVALID, "ls_temporal_attention: null pointer");
  if (d->C != 320 && d->C != 640) return fail(LS_ERR_INVALID, "ls_temporal_attention: C must be 320 or 640");
  if (d->heads != 8) return fail(LS_ERR_INVALID, "ls_temporal_attention: 8 heads");
  if (d->F < 1 || d->F > 16) return fail(LS_ERR_INVALID, "ls_temporal_attention: 1 <= F <= 16 frames");
  const int ppb = d->C == 320 ? TCfg<320>::PPB : TCfg<640>::PPB;  // pixels per block
  if (d->S <= 0 || d->S % ppb || d->n_samples <= 0)
    return fail(LS_ERR_INVALID, "ls_temporal_attention: S must be a positive multiple of the block's pixels");
  if (d->ldx % 8 || d->ldo % 8 || d->ldx < d->C || d->ldo < d->C)
    return fail(LS_ERR_INVALID, "ls_temporal_attention: row pitches must be multiples of 8 and >= C");
  if (((uintptr_t)d->x | (uintptr_t)d->o | (uintptr_t)d->w | (uintptr_t)d->gamma | (uintptr_t)d->bpe) & 15)
    return fail(LS_ERR_INVALID, "ls_temporal_attention: pointers must be 16-B aligned");
  if ((long)d->n_samples * d->F * d->S >= (1L << 31)) return fail(LS_ERR_INVALID, "ls_temporal_attention: too many rows");
  TAttnArgs a;
  a.x = (const u16*)d->x; a.gamma = d->gamma; a.bpe = d->bpe; a.w = (const u16*)d->w; a.o = (u16*)d->o;
  a.ldx = d->ldx; a.ldo = d->ldo; a.F = d->F; a.S = d->S; a.blocks_per_sample = d->S / ppb;
  a.eps = d->eps > 0.f ? d->eps : 1e-5f;
  a.ablate = 0;
#ifdef LS_TATTN_ABLATE
  if (const char* e = ls_env("LS_TATTN_ABLATE")) a.ablate = atoi(e);
#endif
  const int grid = d->n_samples * a.blocks_per_sample;
  hipStream_t s = (hipStream_t)stream;
  return d->C == 320 ? launch_tattn<320>(a, grid, s) : launch_tattn<640>(a, grid, s);
}
