// gpsig_amd -- shared device helpers for the gfx950 (CDNA4) signature-kernel kernels.
//
// Wave64 everywhere: cross-lane steps use DPP (row_shr / row_bcast / wave_shl), which on
// gfx950 are single VALU-issue operations, instead of LDS round trips.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gpsig_amd.h"

#define GPSIG_DEV __device__ __forceinline__

namespace gpsig {

// ---------------------------------------------------------------------------------------------
// DPP cross-lane helpers (gfx9 encodings: row_shr:n = 0x110|n, row_bcast:15 = 0x142,
// row_bcast:31 = 0x143, wave_shl:1 = 0x130, wave_shr:1 = 0x138).
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF, bool BOUND_ZERO = true>
GPSIG_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK,
                                                               BANK_MASK, BOUND_ZERO));
}
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF, bool BOUND_ZERO = true>
GPSIG_DEV double dpp_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Inclusive prefix sum over aligned groups of LP lanes (LP = 16, 32 or 64).
template <int LP>
GPSIG_DEV float group_incl_scan(float v) {
  static_assert(LP == 16 || LP == 32 || LP == 64, "LP");
  v += dpp_f<0x111>(v);
  v += dpp_f<0x112>(v);
  v += dpp_f<0x114>(v);
  v += dpp_f<0x118>(v);
  if constexpr (LP >= 32) v += dpp_f<0x142, 0xA>(v);
  if constexpr (LP >= 64) v += dpp_f<0x143, 0xC>(v);
  return v;
}

// N independent inclusive group scans, step-interleaved so consecutive DPP reads never wait on the
// VALU result of the previous step (the VALU-write -> DPP-read hazard otherwise costs s_nops).
template <int LP, int N>
GPSIG_DEV void group_incl_scan_n(float (&v)[N]) {
  static_assert(LP == 16 || LP == 32 || LP == 64, "LP");
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_f<0x111>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_f<0x112>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_f<0x114>(v[k]);
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] += dpp_f<0x118>(v[k]);
  // The row broadcasts run over all rows and their term is weighted by a per-lane 0/1 factor
  // instead of a row-masked DPP (which needs a freshly zeroed destination per step): row_bcast:15
  // feeds rows 1 and 3 only (row 2 belongs to the next group at LP = 32 and takes rows 0-1 through
  // row_bcast:31 at LP = 64).
  const int row = (int)(__lane_id() >> 4);
  if constexpr (LP >= 32) {
    const float f = (row & 1) ? 1.0f : 0.0f;
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = __builtin_fmaf(dpp_f<0x142>(v[k]), f, v[k]);
  }
  if constexpr (LP >= 64) {
    const float f = (row >= 2) ? 1.0f : 0.0f;
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = __builtin_fmaf(dpp_f<0x143>(v[k]), f, v[k]);
  }
}

// Lane groups that are not aligned to DPP rows: LP = 10 or 20 lanes per group, groups at lanes 0, LP,
// 2 LP, ... (64 / LP of them; the remaining lanes form a partial group whose results are discarded).
// Such a group straddles a 16-lane DPP row at a position that depends on its slot (row offsets 0, 10, 4, 14,
// 8, 2 for LP = 10), and a DPP scan (row_shr inside rows, row_bcast across them) would then combine the
// partial sums in a slot-dependent order: a pair moved to another slot would differ by fp32 rounding.  So the
// scan is a plain Hillis-Steele scan over the whole wave, every step reading lane - s through ds_bpermute
// (the LDS crossbar; no LDS storage, no VALU issue), its term weighted by a per-lane 0/1 factor (source in
// the same group: gl >= s).  Every lane of every group then evaluates the same tree,
//   S_1(gl) = v(gl) + v(gl-1),  S_2(gl) = S_1(gl) + S_1(gl-2),  ...,
// so results are bitwise independent of the slot (K(X)[S, S] == K(X[S])).
template <int LP>
struct SegFactors {
  static constexpr int NS = LP > 16 ? 5 : 4;  // steps 1, 2, 4, 8 (, 16)
  float f[NS];
  int base;  // 4 lane: ds_bpermute takes address bits [7:2], so base + 256 - 4 s addresses lane - s mod 64
             // (the constant folds into the instruction's offset; wrapped sources are masked)
  GPSIG_DEV SegFactors() {
    const int lane = (int)__lane_id(), gl = lane % LP;
    base = 4 * lane;
#pragma unroll
    for (int t = 0; t < NS; ++t) f[t] = gl >= (1 << t) ? 1.0f : 0.0f;
  }
};
// v[k] from lane - S (mod 64) for N values: ds_bpermute with the shift in the instruction's offset field (the
// compiler materialises a register per constant address otherwise), one lgkmcnt wait for the batch.
template <int S, int N>
GPSIG_DEV void bperm_sub_n(int base, const float (&v)[N], float (&u)[N]) {
  constexpr int OFF = 256 - 4 * S;
#pragma unroll
  for (int k = 0; k < N; ++k)
    asm volatile("ds_bpermute_b32 %0, %1, %2 offset:%3" : "=v"(u[k]) : "v"(base), "v"(v[k]), "i"(OFF));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // the results exist only after the wait: tie every later use to it (volatile asm keeps this order)
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" : "+v"(u[k]));
}
template <int LP, int N>
GPSIG_DEV void seg_incl_scan_n(float (&v)[N], const SegFactors<LP> &f) {
  static_assert(LP == 10 || LP == 20, "segmented groups");
  float u[N];
#define GPSIG_SEG_STEP(t)                                                         \
  bperm_sub_n<(1 << t), N>(f.base, v, u);                                         \
  _Pragma("unroll") for (int k = 0; k < N; ++k) v[k] = __builtin_fmaf(u[k], f.f[t], v[k]);
  GPSIG_SEG_STEP(0)
  GPSIG_SEG_STEP(1)
  GPSIG_SEG_STEP(2)
  GPSIG_SEG_STEP(3)
  if constexpr (SegFactors<LP>::NS > 4) { GPSIG_SEG_STEP(4) }
#undef GPSIG_SEG_STEP
}

// Sum over a segmented group (LP = 10 / 20), valid in the group's first lane (gl == 0).
template <int LP>
GPSIG_DEV float seg_group_sum(float v, const SegFactors<LP> &f) {
  float t[1] = {v};
  seg_incl_scan_n<LP, 1>(t, f);
  const int lane = (int)__lane_id();
  const int last = lane - lane % LP + LP - 1;
  return __shfl(t[0], last < 64 ? last : 63, 64);
}

// Value of lane (lane+1) of the wave (0 for lane 63).
GPSIG_DEV float lane_next(float v) { return dpp_f<0x130>(v); }
// Value of lane (lane-1) of the wave (`edge` for lane 0 is handled by the caller).
GPSIG_DEV float lane_prev(float v) { return dpp_f<0x138>(v); }
GPSIG_DEV double lane_prev(double v) { return dpp_d<0x138>(v); }

// Reduce-scatter of 4K per-lane values over the 64 lanes of a wave (gfx950 v_permlane32_swap /
// v_permlane16_swap halve the live values twice, DPP row rotations finish each 16-lane row): on return
// every lane of row R (lanes 16R .. 16R+15) holds in out[i] the wave total of v[4i + ROW_SLOT[R]].
// 2K + K swaps and adds plus 4K row steps for 4K totals (a wave-wide scan per value costs 6 steps each).
constexpr int ROW_SLOT[4] = {0, 2, 1, 3};
template <int K>
GPSIG_DEV void wave_reduce_scatter4(const float (&v)[4 * K], float (&out)[K]) {
  // The swaps are issued as inline asm: ROCm 7.2's __builtin_amdgcn_permlane{16,32}_swap lowering reuses
  // the first result register for the second (tools/permlane_probe2.hip shows v_add v2, v4, v4 after
  // v_permlane32_swap v4, v5).  s_nop 1 covers the VALU-write -> permlane-read hazard of the operands.
  float s1[2 * K];
#pragma unroll
  for (int i = 0; i < 2 * K; ++i) {
    float a = v[2 * i], b = v[2 * i + 1];
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    s1[i] = a + b;  // lanes < 32: v[2i], lanes >= 32: v[2i+1]
  }
#pragma unroll
  for (int i = 0; i < K; ++i) {
    float a = s1[2 * i], b = s1[2 * i + 1];
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
    out[i] = a + b;
  }
#pragma unroll
  for (int i = 0; i < K; ++i) out[i] += dpp_f<0x128>(out[i]);  // row_ror:8
#pragma unroll
  for (int i = 0; i < K; ++i) out[i] += dpp_f<0x124>(out[i]);  // row_ror:4
#pragma unroll
  for (int i = 0; i < K; ++i) out[i] += dpp_f<0x122>(out[i]);  // row_ror:2
#pragma unroll
  for (int i = 0; i < K; ++i) out[i] += dpp_f<0x121>(out[i]);  // row_ror:1
}

// Sum over an aligned group of LP lanes, result in every lane of the group.
template <int LP>
GPSIG_DEV float group_sum(float v) {
#pragma unroll
  for (int o = LP / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

GPSIG_DEV int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Read-only view of data no launch in flight writes (feature records): loads through the constant
// address space may use the scalar unit even when the kernel also stores or issues atomics, which
// would otherwise keep wave-uniform global loads on the vector path (behind the atomics in vmcnt).
using cfloat = const __attribute__((address_space(4))) float;
GPSIG_DEV cfloat *as_const(const float *p) { return (cfloat *)p; }

// ---------------------------------------------------------------------------------------------
// expm1 on |x| <= 0.5 as x * P5(x): minimax (Lawson) fit of expm1(x)/x on [-0.5, 0.5], max
// relative error 2.2e-7 in fp32 with FMA Horner (tests/test_numerics.py pins it).  Only used where
// the caller has already checked |x| < EM1_TAU; outside that range the value is discarded.
constexpr float EM1_TAU = 0.5f;
GPSIG_DEV float em1_small(float x) {
  float p = 1.388882549e-03f;
  p = __builtin_fmaf(p, x, 8.407682727e-03f);
  p = __builtin_fmaf(p, x, 4.166870013e-02f);
  p = __builtin_fmaf(p, x, 1.666597426e-01f);
  p = __builtin_fmaf(p, x, 4.999998314e-01f);
  p = __builtin_fmaf(p, x, 1.000000095e+00f);
  return p * x;
}

// Packed fp32 pairs: on gfx950 v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 process two fp32 values
// per lane in one VALU issue (a wave-uniform SGPR operand is broadcast through op_sel), so every
// per-cell evaluation is written on column pairs.
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
GPSIG_DEV f2 splat2(float v) { return (f2){v, v}; }
GPSIG_DEV f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
GPSIG_DEV f2 em1_small2(f2 x) {
  f2 p = splat2(1.388882549e-03f);
  p = fma2(p, x, splat2(8.407682727e-03f));
  p = fma2(p, x, splat2(4.166870013e-02f));
  p = fma2(p, x, splat2(1.666597426e-01f));
  p = fma2(p, x, splat2(4.999998314e-01f));
  p = fma2(p, x, splat2(1.000000095e+00f));
  return p * x;
}

// N independent em1 evaluations, Horner steps interleaved across the N chains (back-to-back
// dependent v_pk_fma_f32 would otherwise be padded with s_nop).
template <int N>
GPSIG_DEV void em1_small2_n(const f2 (&x)[N], f2 (&out)[N]) {
  constexpr float c[6] = {1.388882549e-03f, 8.407682727e-03f, 4.166870013e-02f,
                          1.666597426e-01f, 4.999998314e-01f, 1.000000095e+00f};
#pragma unroll
  for (int k = 0; k < N; ++k) out[k] = fma2(splat2(c[0]), x[k], splat2(c[1]));
#pragma unroll
  for (int s = 2; s < 6; ++s)
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = fma2(out[k], x[k], splat2(c[s]));
#pragma unroll
  for (int k = 0; k < N; ++k) out[k] = out[k] * x[k];
}

// expm1 on |x| < EM1_LO_TAU as x * P3(x): minimax (Lawson) fit of expm1(x)/x on [-1/16, 1/16], 1.6e-8
// relative in exact arithmetic, 1.4e-7 with fp32 FMA Horner.  For arguments the caller has bounded a
// priori (the increment products of a pair whose increments are all small).
constexpr float EM1_LO_TAU = 0.0625f;
template <int N>
GPSIG_DEV void em1_lo2_n(const f2 (&x)[N], f2 (&out)[N]) {
  constexpr float c[4] = {4.166666667e-02f, 1.666992186e-01f, 5.000000132e-01f, 9.999999841e-01f};
#pragma unroll
  for (int k = 0; k < N; ++k) out[k] = fma2(splat2(c[0]), x[k], splat2(c[1]));
#pragma unroll
  for (int s = 2; s < 4; ++s)
#pragma unroll
    for (int k = 0; k < N; ++k) out[k] = fma2(out[k], x[k], splat2(c[s]));
#pragma unroll
  for (int k = 0; k < N; ++k) out[k] = out[k] * x[k];
}

// Maximum over the 64 lanes of a wave (result in every lane).
GPSIG_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = __builtin_fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// exp(x) = 2^(x log2 e) on the hardware transcendental unit (v_exp_f32, ~1 ulp).
GPSIG_DEV float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

}  // namespace gpsig
