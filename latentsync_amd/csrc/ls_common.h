// Shared device helpers for libls_hip.so (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <atomic>
#include <string>

#include "../../include/ls_hip.h"

// A/B switches read from the environment exist only in the diagnostics build
// (LS_DIAG_KERNELS, LS_DIAG_BUILD=1): in the default library no dispatch decision and no
// weight layout depends on the environment -- tuning goes through ls_set_tuning.
static inline const char* ls_env(const char* name) {
#ifdef LS_DIAG_KERNELS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// buffer_load ... lds (LDS-DMA through a buffer descriptor): LDS destination = M0 base
// + lane * size; the global byte offset = voffset (per lane) + soffset (uniform); a
// piece whose voffset + soffset reaches num_records reads zeros.
__device__ void ls_raw_buffer_load_lds(i32x4 rsrc, __attribute__((address_space(3))) void* lds, int size, int voffset,
                                       int soffset, int offset, int aux) __asm("llvm.amdgcn.raw.buffer.load.lds");

__device__ __forceinline__ i32x4 buffer_rsrc(const void* base, uint32_t bytes) {
  const unsigned long long b = (unsigned long long)base;
  i32x4 r;
  r[0] = (int)(uint32_t)b;
  r[1] = (int)(uint32_t)(b >> 32);  // stride 0
  r[2] = (int)bytes;                // num_records (bytes): loads at or past it return 0
  r[3] = 0x00020000;                // gfx9 raw-buffer dword 3
  return r;
}
typedef uint16_t u16;
// a 16-B LDS slot as an LDS-space (32-bit) pointer: LDS-DMA destinations computed in this
// space need no generic -> LDS null check per instruction
typedef __attribute__((address_space(3))) uint4 lds_u4;

namespace ls {

void set_error(const std::string& msg);
int fail(ls_status code, const std::string& msg);
int check_launch(const char* what);

__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ u16 f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN preserved
  return __builtin_bit_cast(u16, b);
}

// two floats -> one dword of bf16 (a low): ONE v_cvt_pk_bf16_f32 on both.  (Two scalar
// casts combined with shift / or compile to 2 converts + v_lshlrev + v_or_sdwa.)
typedef __bf16 bf16x2_cv __attribute__((ext_vector_type(2)));
typedef float f32x2_cv __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  const f32x2_cv v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_cv));
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

// 2^x as the bare v_exp_f32: exp2f() wraps it in a denormal-range fix-up (compare,
// two selects and a v_ldexp around every call -- 5 VALU ops where the softmax and
// GELU need 1).  Results below 2^-126 flush to 0, which every caller tolerates
// (softmax terms, erf tails).
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// x * sigmoid(x) with the hardware reciprocal v_rcp_f32 (1 ulp; outputs are bf16).
// (__frcp_rn is the correctly rounded reciprocal: a 10-instruction division sequence.)
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.0f + fast_exp2(x * -1.4426950408889634f));
}
// silu(t) from u = t log2(e) (a producer that folds log2(e) into its affine): 5 VALU with
// the affine's fma -- e = 2^-u, r = 1 / ((1 + e) log2 e) by one fma + v_rcp_f32, u r = t / (1 + e^-t)
__device__ __forceinline__ float silu_log2(float u) {
  const float e = fast_exp2(-u);
  return u * __builtin_amdgcn_rcpf(fmaf(e, 1.4426950408889634f, 1.4426950408889634f));
}

// exact-erf GELU (diffusers GEGLU / whisper MLP), branch-free, as x * sigmoid(s(x)) with
// s(x) = x (a + b x^2 + c x^4): (a, b, c) fitted minimax to the fp64 erf GELU, x^2 clamped
// at 36 (beyond |x| = 6 the sigmoid is saturated either way and the quartic would turn
// over).  Abs error 2.6e-5 on all of R in fp32 -- the accuracy of the Abramowitz & Stegun
// 7.1.25 erf form this replaces (a twentieth of a bf16 ulp at the GELU's largest negative
// output, |y| = 0.17) -- in 7 VALU ops + v_exp_f32 + v_rcp_f32 instead of 10 + the same two
// (round 6: the GEGLU epilogues and the FeedForward kernels are VALU-issue-bound).  log2(e)
// and the sign are folded into the coefficients: e = 2^(x t) = e^(-s(x)).
__device__ __forceinline__ float gelu_erf(float x) {
  const float x2 = fminf(x * x, 36.0f);
  const float t = fmaf(x2, fmaf(x2, 0.001014263f, -0.10677572f), -2.3011212f);
  return x * __builtin_amdgcn_rcpf(1.0f + fast_exp2(x * t));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// max / sum over the 4 lanes {L, L^16, L^32, L^48} (the lane groups of a 16x16 MFMA
// accumulator column) with gfx950's cross-row swaps: VALU only, no LDS round trip
// (a ds_bpermute per step costs a dependent LDS latency).
__device__ __forceinline__ float xor16_32_max(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  v = __builtin_elementwise_maximum(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const uint32_t w = __float_as_uint(v);
  const auto b = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return __builtin_elementwise_maximum(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float xor16_32_sum(float v) {
  const uint32_t u = __float_as_uint(v);
  const auto a = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const uint32_t w = __float_as_uint(v);
  const auto b = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// 16 B per lane global -> LDS DMA (global_load_lds_dwordx4): the wave-instruction
// writes 64 consecutive 16-B slots from lds_dst (lane-linear), each lane's own source
__device__ __forceinline__ void glds16(const void* src, uint4* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_dst, 16, 0, 0);
}

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// LDS image of one operand tile: rows of BK bf16, 16-B chunks XOR-swizzled so
// the 16-lane groups of a ds_read_b128 fragment read hit distinct bank slots.
template <int BK>
__device__ __forceinline__ int swz_bk(int row, int c) {
  if (BK == 64) return row * 8 + (c ^ ((row >> 1) & 7));
  return row * 4 + (c ^ ((-(row >> 2)) & 3));
}

__device__ __forceinline__ void load8f(const float* __restrict__ p, float* d) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

}  // namespace ls

// hipFuncSetAttribute is a per-device setting: apply it once per (call site, device) --
// a process-wide `static bool` would skip every device after the first one it ran on.
inline void ls_set_max_dyn_shm(const void* fn, int shm, std::atomic<unsigned long long>& done) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const unsigned long long bit = 1ull << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return;
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, shm);
  done.fetch_or(bit, std::memory_order_acq_rel);
}
#define LS_SET_MAX_DYN_SHM(fn, shm)                                  \
  do {                                                               \
    static std::atomic<unsigned long long> ls_shm_done_{0};          \
    ls_set_max_dyn_shm((const void*)(fn), (int)(shm), ls_shm_done_); \
  } while (0)
