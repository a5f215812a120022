// gpsig_amd -- gradient (VJP) of the first-order signature-kernel Gram on column pairs (round 6).
//
// The same reverse sweep as sig_bwd_kernel (sig_bwd.h: forward state recovered by inverting the row update,
// adjoint column sums, second-difference adjoint, point gradients), with every per-column quantity held as a
// packed fp32 pair: lane gl owns the W columns gl W .. gl W + W - 1 as W/2 pairs (w2, w2 + W/2), so the cell
// regeneration, the inversion and adjoint updates, the in-lane parts of the column scans and the emission
// run on v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 (two columns per issue; sig_fo.h's layout).  Only the
// cross-lane steps of the scans stay one value per lane.
//
// Level 1 leaves the cells: its adjoint is the constant g_1 = dLoss/dK_1 on every cell, whose
// second-difference adjoint is +-g_1 on the four corner points alone (K_1 telescopes to
// k(x_L, y_L) - k(x_L, y_0) - k(x_0, y_L) + k(x_0, y_0), sig_common.h level1_closed), so the kernel adds the
// corner gradients in fp64 and runs the cells with Ĉ_1 - g_1.  That removes the exp/fp32 rounding of the
// corner terms, which for one-level or short sequences are the whole gradient (tests/test_grad_gpu.py
// test_gram_vjp_shapes[1-1-8]), and at M = 1 the sweep itself.
//
// Covered: RBF / linear difference seeds, one column block (l2 <= LP W), any pair mode, with or without the
// forward's saved state.  Longer sequences, difference=False and wide channel counts keep sig_bwd_kernel.
#pragma once
#include "sig_bwd.h"

namespace gpsig {

// Exclusive scan over the group's columns of N packed column-pair arrays (pair w2 = columns (w2, w2 + W2)),
// in place: the in-lane prefix of each half as one packed chain, the lane totals scanned across the group.
template <int LP, int W2, int N, class SF>
GPSIG_DEV void pk_excl_n(f2 (&v)[N][W2], const SF &sf) {
  float T[N], incl[N], h0[N];
#pragma unroll
  for (int n = 0; n < N; ++n) {
    f2 run = v[n][0];
    v[n][0] = splat2(0.0f);
#pragma unroll
    for (int k = 1; k < W2; ++k) {
      const f2 t = v[n][k];
      v[n][k] = run;
      run += t;
    }
    h0[n] = run[0];
    T[n] = run[0] + run[1];
    incl[n] = T[n];
  }
  if constexpr (64 % LP != 0)
    seg_incl_scan_n<LP, N>(incl, sf);
  else
    group_incl_scan_n<LP, N>(incl);
#pragma unroll
  for (int n = 0; n < N; ++n) {
    const float b = incl[n] - T[n];
    const f2 off = (f2){b, b + h0[n]};
#pragma unroll
    for (int k = 0; k < W2; ++k) v[n][k] = (k == 0) ? off : v[n][k] + off;
  }
}

// Group total of an inclusive scan, in every lane of the group: the last lane's value (v_readlane for the
// 32- and 64-lane groups, a ds_bpermute read otherwise).
template <int LP>
GPSIG_DEV float group_total(float incl) {
  if constexpr (LP == 64) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 63));
  } else if constexpr (LP == 32) {
    const float t0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 31));
    const float t1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, incl), 63));
    return __lane_id() < 32 ? t0 : t1;
  } else {
    const int l0 = (int)__lane_id() - (int)__lane_id() % LP + LP - 1;
    return __shfl(incl, l0 < 64 ? l0 : 63, 64);
  }
}

// One exclusive scan (a, in place) and one reverse-exclusive scan (b, in place) of packed column-pair arrays,
// their lane totals scanned across the group together (two independent DPP chains: no step waits on the
// previous step's result).
template <int LP, int W2, class SF>
GPSIG_DEV void pk_excl_rexcl(f2 (&a)[W2], f2 (&b)[W2], const SF &sf) {
  f2 ra = a[0];
  a[0] = splat2(0.0f);
#pragma unroll
  for (int k = 1; k < W2; ++k) {
    const f2 t = a[k];
    a[k] = ra;
    ra += t;
  }
  f2 rb = b[W2 - 1];
  b[W2 - 1] = splat2(0.0f);
#pragma unroll
  for (int k = W2 - 2; k >= 0; --k) {
    const f2 t = b[k];
    b[k] = rb;
    rb += t;
  }
  const float Ta = ra[0] + ra[1], Tb = rb[0] + rb[1];
  float incl[2] = {Ta, Tb};
  if constexpr (64 % LP != 0)
    seg_incl_scan_n<LP, 2>(incl, sf);
  else
    group_incl_scan_n<LP, 2>(incl);
  const float ba = incl[0] - Ta;
  const f2 offa = (f2){ba, ba + ra[0]};
  const float after = group_total<LP>(incl[1]) - incl[1];
  const f2 offb = (f2){after + rb[1], after};
#pragma unroll
  for (int k = 0; k < W2; ++k) {
    a[k] = (k == 0) ? offa : a[k] + offa;
    b[k] = (k == W2 - 1) ? offb : b[k] + offb;
  }
}

template <int DP, int W, int LP, int M, int SEED>
#ifndef GPSIG_BWDPK_WPE
#define GPSIG_BWDPK_WPE 2
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GPSIG_BWDPK_WPE))) void sig_bwd_pk_kernel(BwdArgs p) {
  static_assert(W % 2 == 0, "column pairs");
  static_assert(SEED == SEED_RBF_DIFF || SEED == SEED_LIN_DIFF, "difference seeds");
  constexpr int FS = feat_stride(DP);
  constexpr int W2 = W / 2;
  constexpr int G = 64 / LP;
  constexpr bool SEG = (64 % LP) != 0;
  constexpr bool RBF = SEED == SEED_RBF_DIFF;
  constexpr float NHL2E = -0.72134752044448170f;  // exp(-d2/2) = exp2(d2 * NHL2E)
  constexpr float L2E = 1.4426950408889634f;
  constexpr int RC = 4;  // rows per regenerated chunk (RbfSeed cells), LDS: 4 waves x RC x W x 64 f2
  constexpr int ML = M > 1 ? M - 1 : 1;
  __shared__ __attribute__((aligned(16))) f2 cbuf[RBF ? 4 : 1][RBF ? RC : 1][W][64];
  __shared__ float tbuf[4][4][DP][64];  // x-gradient row batches

  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int g = lane / LP;
  const int gl = lane % LP;
  const bool diag = p.pair_mode == GPSIG_PAIRS_DIAG;
  const long long lblk = p.blk0 + (long long)blockIdx.x;

  // ---- which pair (sig_bwd_kernel's enumeration)
  int a, b;
  if (diag) {
    a = p.row_begin + (int)lblk * 4 + wave;
    b = a;
    if (a >= p.row_end) return;
  } else {
    int ta, tb;
    if (p.pair_mode == GPSIG_PAIRS_UPPER) {
      Tile t;
      if constexpr (SEG)
        t = upper_tile_g<G>(p.tile_base + lblk, p.ntb);
      else
        t = upper_tile(p.tile_base + lblk, p.ntb, 4 / G);
      ta = t.ta;
      tb = t.tb;
    } else {
      ta = p.tiles_a0 + (int)(lblk / p.ntb);
      tb = (int)(lblk % p.ntb);
    }
    a = ta * 4 + wave;
    b = tb * G + (SEG && g >= G ? G - 1 : g);
    if (a < p.row_begin || a >= p.row_end) return;
  }
  bool pair_ok = b < p.n2;
  if (p.pair_mode == GPSIG_PAIRS_UPPER) pair_ok = pair_ok && b >= a;
  if (SEG) pair_ok = pair_ok && g < G;
  if (diag) pair_ok = (g == 0);
  const int bl = b < p.n2 ? b : p.n2 - 1;
  const int l1 = p.l1, l2 = p.l2;
  const int nrows = l1 - 1, ncells = l2 - 1;

  const float *__restrict__ fx = p.FX + (long long)a * l1 * FS;
  cfloat *fxc = as_const(fx);  // row records: scalar loads
  const float *__restrict__ fy = p.FY + (long long)bl * l2 * FS;
  using SegF = std::conditional_t<SEG, SegFactors<SEG ? LP : 10>, char>;
  const SegF segf{};

  // ---- column data: pair w2 of this lane holds columns j = gl W + w2 + h W2 (h = 0, 1); points past the
  // sequence clamp to its last one, columns without a cell get a zero increment (their product-form cells
  // are exact zeros) and a zero cell mask
  f2 y[W2][DP], dy[W2][DP];
#pragma unroll
  for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = gl * W + w2 + h * W2;
      const bool cell = j < ncells;
      const float *f = fy + (long long)(j < l2 ? j : l2 - 1) * FS;
#pragma unroll
      for (int k = 0; k < DP; ++k) {
        y[w2][k][h] = f[k];
        dy[w2][k][h] = cell ? f[DP + k] : 0.0f;
      }
    }
  const int nv = ncells - gl * W;  // this lane's columns w < nv carry a cell
  // |dy_j|^2 / 2 of a column pair (recomputed where needed: two registers per pair fewer)
  auto hdy_of = [&](int w2) {
    f2 h = dy[w2][0] * dy[w2][0];
#pragma unroll
    for (int k = 1; k < DP; ++k) h = fma2(dy[w2][k], dy[w2][k], h);
    return h * splat2(0.5f);
  };
  // the lane's last column: a cell whose right point sits in the next lane (the naive corner needs it)
  const bool valid_last = gl * W + W - 1 < ncells;

  // |c_ij| <= 2 sqrt(hdx_i hdy_j): when the bound over the pair block stays below EM1_LO_TAU the cells take
  // the cubic expm1 of c and only |p| is range-checked (RbfSeedPk::bound_c)
  bool clo = false;
  if constexpr (RBF) {
    float hx = 0.0f, hy = 0.0f;
    for (int i = lane; i < nrows; i += 64) hx = __builtin_fmaxf(hx, fx[(long long)i * FS + 2 * DP]);
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      const f2 hd = hdy_of(w2);
      hy = __builtin_fmaxf(hy, __builtin_fmaxf(hd[0], hd[1]));
    }
    hx = wave_max(hx);
    hy = wave_max(hy);
    clo = wave_uniform(4.0f * hx * hy < 0.98f * EM1_LO_TAU * EM1_LO_TAU ? 1 : 0) != 0;
  }

  // exact k(x, y_j) and expm1(q_j) (q = <x - y_j, dy_j> - |dy_j|^2/2) of the row with point x
  auto exact_row = [&](cfloat *xr, f2 (&k)[W2], f2 (&Eq)[W2]) {
    float xv[DP];
#pragma unroll
    for (int c = 0; c < DP; ++c) xv[c] = xr[c];
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      f2 s2 = splat2(0.0f), q = -hdy_of(w2);
#pragma unroll
      for (int c = 0; c < DP; ++c) {
        const f2 df = splat2(xv[c]) - y[w2][c];
        s2 = fma2(df, df, s2);
        q = fma2(df, dy[w2][c], q);
      }
      s2 = s2 * splat2(NHL2E);
      Eq[w2] = em1_small2(q);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        k[w2][h] = __builtin_amdgcn_exp2f(s2[h]);
        if (!(__builtin_fabsf(q[h]) < EM1_TAU)) Eq[w2][h] = __builtin_amdgcn_exp2f(q[h] * L2E) - 1.0f;
      }
    }
  };

  // cells of rows i0 .. i0 + nr - 1 (RBF) into this wave's LDS chunk: an exact row, then the forward seed's
  // exp-free recurrences (sig_common.h RbfSeedPk::row: the column recurrence of p from the lane's first pair,
  // k and expm1(q) row to row); cells outside the polynomial range take the corner difference of an exact
  // next row (wave-uniform branch).  Slot [r][w2] holds the cells, [r][W2 + w2] the k row of point i0 + r.
  f2(*cb)[W][64] = cbuf[RBF ? wave : 0];
  auto chunk = [&](auto clo_t, int i0, int nr) {
    constexpr bool CLO = decltype(clo_t)::value;
    f2 kc[W2], Eq[W2];
    exact_row(fxc + (long long)i0 * FS, kc, Eq);
#pragma unroll 1
    for (int r = 0; r < nr; ++r) {
      cfloat *fr = fxc + (long long)(i0 + r) * FS;
      float dxv[DP];
#pragma unroll
      for (int c = 0; c < DP; ++c) dxv[c] = fr[DP + c];
      const float gi = fr[2 * DP + 1];
      f2 c2[W2], p2[W2];
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        f2 cc = dy[w2][0] * splat2(dxv[0]);
#pragma unroll
        for (int k = 1; k < DP; ++k) cc = fma2(dy[w2][k], splat2(dxv[k]), cc);
        c2[w2] = cc;
      }
      {
        f2 pp = splat2(-gi);
#pragma unroll
        for (int k = 0; k < DP; ++k) pp = fma2(y[0][k], splat2(dxv[k]), pp);
        p2[0] = pp;
      }
#pragma unroll
      for (int w2 = 1; w2 < W2; ++w2) p2[w2] = p2[w2 - 1] + c2[w2 - 1];
      f2 Ec[W2];
      if constexpr (CLO)
        em1_lo2_n<W2>(c2, Ec);
      else
        em1_small2_n<W2>(c2, Ec);
      f2 Ep = em1_small2(p2[0]);
      f2 dM[W2], kn[W2], Eqn[W2];
      float mx = 0.0f;
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        f2 t = fma2(Ep, Ec[w2], Ec[w2]);  // (1 + Ep) Ec
        const f2 Epw = Ep;
        Ep = Ep + t;
        const f2 t2 = fma2(Eq[w2], t, t);
        dM[w2] = kc[w2] * fma2(Epw, Eq[w2], t2);
        kn[w2] = fma2(kc[w2], Epw, kc[w2]);
        Eqn[w2] = fma2(Eq[w2], Ec[w2], Eq[w2] + Ec[w2]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if constexpr (CLO) {  // the pairs after the first follow the exact Ep chain (RbfSeedPk::row)
            if (w2 == 0) mx = __builtin_fmaxf(mx, __builtin_fabsf(p2[w2][h]));
          } else {
            mx = __builtin_fmaxf(__builtin_fmaxf(mx, __builtin_fabsf(p2[w2][h])), __builtin_fabsf(c2[w2][h]));
          }
        }
      }
      if (__builtin_amdgcn_ballot_w64(mx >= EM1_TAU) != 0) {
        // an out-of-range cell may have spoilt the chained Ep after it: every in-range cell from its own p,
        // the others by the corner difference of the k grid with an exact next row
        exact_row(fr + FS, kn, Eqn);
        const float knR = lane_next(kn[0][0]), kcR = lane_next(kc[0][0]);
        f2 Epd[W2], Ecd[W2];
        em1_small2_n<W2>(p2, Epd);
        em1_small2_n<W2>(c2, Ecd);
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const int w2 = w % W2, h = w / W2;
          const float kn1 = (w + 1 < W) ? kn[(w + 1) % W2][(w + 1) / W2] : knR;
          const float kc1 = (w + 1 < W) ? kc[(w + 1) % W2][(w + 1) / W2] : kcR;
          const float naive = (kn1 - kn[w2][h]) - (kc1 - kc[w2][h]);
          const float m = __builtin_fmaxf(__builtin_fabsf(p2[w2][h]), __builtin_fabsf(c2[w2][h]));
          float t = __builtin_fmaf(Epd[w2][h], Ecd[w2][h], Ecd[w2][h]);
          t = __builtin_fmaf(Eq[w2][h], t, t);
          const float prod = kc[w2][h] * __builtin_fmaf(Epd[w2][h], Eq[w2][h], t);
          float v = m < EM1_TAU ? prod : naive;
          if (w + 1 == W && !valid_last) v = 0.0f;
          dM[w2][h] = w < nv ? v : 0.0f;
        }
      }
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        cb[r][w2][lane] = dM[w2];
        cb[r][W2 + w2][lane] = kc[w2];
        kc[w2] = kn[w2];
        Eq[w2] = Eqn[w2];
      }
    }
  };
  // linear seed: the cells are <dx_i, dy_j>, the k row is 1
  auto lin_cells = [&](int i, f2 (&dM)[W2]) {
    cfloat *fr = fxc + (long long)i * FS;
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      f2 cc = dy[w2][0] * splat2(fr[DP]);
#pragma unroll
      for (int k = 1; k < DP; ++k) cc = fma2(dy[w2][k], splat2(fr[DP + k]), cc);
      dM[w2] = cc;
    }
  };

  // ---- forward state at the end of the sweep: saved by the forward launch, or a forward sweep on the
  // same regenerated cells
  f2 C[ML][W2];
#pragma unroll
  for (int m = 0; m < ML; ++m)
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) C[m][w2] = splat2(0.0f);
  float K[M + 1];
  K[0] = 1.0f;
  const bool saved = p.state != nullptr;
  if (saved) {
    const float *__restrict__ st =
        p.state + (pair_ok ? state_slot(a, bl, p.n2, p.pair_mode == GPSIG_PAIRS_UPPER) * state_stride(M, l2) : 0);
#pragma unroll
    for (int m = 1; m <= M; ++m) K[m] = pair_ok ? st[(long long)(M - 1) * ncells + m - 1] : 0.0f;
    if constexpr (M > 1) {
#pragma unroll
      for (int m = 0; m + 1 < M; ++m)
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int j = gl * W + w2 + h * W2;
            C[m][w2][h] = (pair_ok && j < ncells) ? st[(long long)m * ncells + j] : 0.0f;
          }
    }
  } else {
    // K_1 in closed form, K_2 .. K_{M-1} from the end column sums, K_M = sum of the top level's products
    float KM = 0.0f;
    if constexpr (M > 1) {
      auto fwd_row = [&](const f2 (&dM)[W2]) {
        f2 S[ML][W2];
#pragma unroll
        for (int m = 0; m < ML; ++m)
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) S[m][w2] = C[m][w2];
        pk_excl_n<LP, W2, ML>(S, segf);
        f2 km = dM[0] * S[ML - 1][0];
#pragma unroll
        for (int w2 = 1; w2 < W2; ++w2) km = fma2(dM[w2], S[ML - 1][w2], km);
        KM += km[0] + km[1];
#pragma unroll
        for (int m = ML - 1; m >= 1; --m)
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) C[m][w2] = fma2(dM[w2], S[m - 1][w2], C[m][w2]);
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) C[0][w2] += dM[w2];
      };
      if constexpr (RBF) {
        auto sweep = [&](auto clo_t) {
          for (int i0 = 0; i0 < nrows; i0 += RC) {
            const int nr = nrows - i0 < RC ? nrows - i0 : RC;
            chunk(clo_t, i0, nr);
#pragma unroll 1
            for (int r = 0; r < nr; ++r) {
              f2 dM[W2];
#pragma unroll
              for (int w2 = 0; w2 < W2; ++w2) dM[w2] = cb[r][w2][lane];
              fwd_row(dM);
            }
          }
        };
        if (clo)
          sweep(std::true_type{});
        else
          sweep(std::false_type{});
      } else {
        for (int i = 0; i < nrows; ++i) {
          f2 dM[W2];
          lin_cells(i, dM);
          fwd_row(dM);
        }
      }
    }
    K[1] = level1_closed<DP, SEED>(fx, fy, l1, l2);
#pragma unroll
    for (int m = 2; m <= M; ++m) {
      float s1;
      if (m < M) {
        f2 s2 = C[m - 1][0];
#pragma unroll
        for (int w2 = 1; w2 < W2; ++w2) s2 += C[m - 1][w2];
        s1 = s2[0] + s2[1];
      } else {
        s1 = KM;
      }
      if constexpr (SEG)
        K[m] = seg_group_sum<LP>(s1, segf);
      else
        K[m] = group_sum<LP>(s1);
    }
  }

  // ---- per-level weights g_m = dLoss/dK_m(a, b) and the normalisation / scale factors of this pair
  const bool upper_off = p.pair_mode == GPSIG_PAIRS_UPPER && a != bl;
  const float jit = (p.pair_mode == GPSIG_PAIRS_UPPER && a == bl) ? p.jitter : 0.0f;
  auto pair_terms = [&](float (&gs)[M + 1], float (&sc)[M + 1], float (&r1)[M + 1], float (&r2)[M + 1]) {
    float gsum = 0.0f;
    if (!diag && !p.gout_levels) {
      gsum = p.gout[(long long)a * p.g_ld + bl];
      if (upper_off) gsum += p.gout[(long long)bl * p.g_ld + a];
    }
#pragma unroll
    for (int m = 0; m <= M; ++m) {
      float gg;
      if (diag) {
        gg = p.gout[(long long)m * p.g_lvl + a];
      } else if (p.gout_levels) {
        gg = p.gout[(long long)m * p.g_lvl + (long long)a * p.g_ld + bl];
        if (upper_off) gg += p.gout[(long long)m * p.g_lvl + (long long)bl * p.g_ld + a];
      } else {
        gg = gsum;
      }
      gs[m] = pair_ok ? gg : 0.0f;
      sc[m] = p.scale ? p.scale[m] : 1.0f;
      r1[m] = p.rs1 ? p.rs1[(long long)m * p.n1 + a] : 1.0f;
      r2[m] = p.rs2 ? p.rs2[(long long)m * p.n2 + bl] : 1.0f;
    }
  };
  float gw[M + 1];
  {
    float gs[M + 1], sc[M + 1], r1[M + 1], r2[M + 1];
    pair_terms(gs, sc, r1, r2);
#pragma unroll
    for (int m = 0; m <= M; ++m) gw[m] = gs[m] * sc[m] * r1[m] * r2[m];
  }
  const float g1 = gw[1];
  const float gM = gw[M];

  // level 1 at the corner points, in fp64: dLoss/dx_p of g_1 [k(x_L, y_L) - k(x_L, y_0) - k(x_0, y_L) +
  // k(x_0, y_0)] (linear: g_1 <x_L - x_0, y_L - y_0>); side 0 = x (rows 0, L1), side 1 = y (columns 0, L2)
  auto corner = [&](int side, bool last, double (&o)[DP]) {
    const float *u0 = side ? fy : fx;                             // the point's own sequence
    const float *v0 = side ? fx : fy;                             // the partner sequence
    const int lu = side ? l2 : l1, lv = side ? l1 : l2;
    const float *pu = u0 + (long long)(last ? lu - 1 : 0) * FS;   // the point
    const float *vL = v0 + (long long)(lv - 1) * FS, *vF = v0;    // partner's last and first points
    const double sgn = last ? 1.0 : -1.0;
#pragma unroll
    for (int c = 0; c < DP; ++c) o[c] = 0.0;
    if constexpr (RBF) {
      auto term = [&](const float *q, double s) {
        double d2 = 0.0;
#pragma unroll
        for (int c = 0; c < DP; ++c) {
          const double d = (double)q[c] - (double)pu[c];
          d2 = __builtin_fma(d, d, d2);
        }
        const double kv = s * exp(-0.5 * d2);
#pragma unroll
        for (int c = 0; c < DP; ++c) o[c] = __builtin_fma(kv, (double)q[c] - (double)pu[c], o[c]);
      };
      term(vL, sgn);   // k(p, v_L) with the sign of the corner (p, v_L)
      term(vF, -sgn);  // k(p, v_0)
    } else {
#pragma unroll
      for (int c = 0; c < DP; ++c) o[c] = sgn * ((double)vL[c] - (double)vF[c]);
    }
#pragma unroll
    for (int c = 0; c < DP; ++c) o[c] *= (double)g1;
  };

  // ---- reverse sweep
  float *__restrict__ gxa = p.gX + (long long)a * l1 * p.d;
  const int d = p.d;
  f2 Ch[ML][W2];
#pragma unroll
  for (int m = 0; m < ML; ++m)
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) Ch[m][w2] = splat2(m == 0 ? 0.0f : gw[m + 1]);  // level 1 - g_1 (corners)
  f2 EpA[W2], A[W2], B[W2][DP];
#pragma unroll
  for (int w2 = 0; w2 < W2; ++w2) {
    EpA[w2] = splat2(0.0f);
    A[w2] = splat2(0.0f);
#pragma unroll
    for (int k = 0; k < DP; ++k) B[w2][k] = splat2(0.0f);
  }
  int nslot = 0, pi0 = 0;
  auto flush = [&]() {
    float v[4 * DP], o[DP];
#pragma unroll
    for (int k = 0; k < DP; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[4 * k + r] = tbuf[wave][r][k][lane];
    wave_reduce_scatter4<DP>(v, o);
    const int R = lane >> 4;
    const int slot = R == 0 ? 0 : R == 1 ? 2 : R == 2 ? 1 : 3;  // ROW_SLOT
    if ((lane & 15) == 0 && slot < nslot) {
#pragma unroll
      for (int k = 0; k < DP; ++k)
        if (k < d) unsafeAtomicAdd(gxa + (long long)(pi0 - slot) * d + k, o[k]);
    }
    nslot = 0;
  };
  // point row pi receives dLoss/dk(x_pi, y_j) = Kh: x-gradient reduced over the wave (its pairs share a),
  // y-gradient accumulated per column
  auto emit = [&](int pi, const f2 (&Kh)[W2], const f2 (&kr)[W2]) {
    cfloat *xp = fxc + (long long)pi * FS;
    float xi[DP];
#pragma unroll
    for (int k = 0; k < DP; ++k) xi[k] = xp[k];
    f2 wg[W2];
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) wg[w2] = RBF ? Kh[w2] * kr[w2] : Kh[w2];
    f2 s[DP], st = wg[0];
#pragma unroll
    for (int k = 0; k < DP; ++k) s[k] = wg[0] * y[0][k];
#pragma unroll
    for (int w2 = 1; w2 < W2; ++w2) {
      st += wg[w2];
#pragma unroll
      for (int k = 0; k < DP; ++k) s[k] = fma2(wg[w2], y[w2][k], s[k]);
    }
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      A[w2] += wg[w2];
#pragma unroll
      for (int k = 0; k < DP; ++k) B[w2][k] = fma2(wg[w2], splat2(xi[k]), B[w2][k]);
    }
    const float sw = st[0] + st[1];
    float t[DP];
#pragma unroll
    for (int k = 0; k < DP; ++k) {
      const float sk = s[k][0] + s[k][1];
      t[k] = RBF ? __builtin_fmaf(-sw, xi[k], sk) : sk;
    }
    if (pi == 0 || pi == nrows) {  // the level-1 corner terms of the pair's rows 0 and L1 (group leader)
      if (gl == 0 && pair_ok) {
        double o[DP];
        corner(0, pi == nrows, o);
#pragma unroll
        for (int k = 0; k < DP; ++k) t[k] += (float)o[k];
      }
    }
    if (nslot == 0) pi0 = pi;
#pragma unroll
    for (int k = 0; k < DP; ++k) tbuf[wave][nslot][k][lane] = t[k];
    if (++nslot == 4) flush();
  };

  // one row of the reverse sweep from its cells dM(i, .) and the k row of point i
  f2 kr1[W2];  // k row of point i + 1
  auto rev_row = [&](int i, const f2 (&dM)[W2], const f2 (&k0)[W2]) {
    f2 Dh[W2];
    if constexpr (M > 1) {
      // adjoint column sums from the old Ch: v_m = dM Ch_{m+1}, reverse-exclusive over j
      f2 v[ML][W2];
#pragma unroll
      for (int m = 0; m < ML; ++m)
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) v[m][w2] = dM[w2] * ((m + 1 < ML) ? Ch[m + 1][w2] : splat2(gM));
      // forward state of row i by inversion, ascending levels (C[m] = level m + 1, S_0 = 1), and
      // dLoss/d dM(i, j) = sum_m Ch_m(i+1, j) S_{m-1}(i, j) (with Ch_1 - g_1); each inversion scan (a chain
      // through the levels) shares its cross-lane steps with one of the independent adjoint scans
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) {
        C[0][w2] -= dM[w2];
        Dh[w2] = Ch[0][w2];
      }
#pragma unroll
      for (int s = 1; s < M; ++s) {
        f2 Sm[W2];
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) Sm[w2] = C[s - 1][w2];
        pk_excl_rexcl<LP, W2>(Sm, v[s - 1], segf);
#pragma unroll
        for (int w2 = 0; w2 < W2; ++w2) {
          if (s + 1 < M) C[s][w2] = fma2(-dM[w2], Sm[w2], C[s][w2]);
          const f2 chn = (s + 1 < M) ? Ch[s < ML ? s : 0][w2] : splat2(gM);  // old Ch_{s+1}
          Dh[w2] = fma2(chn, Sm[w2], Dh[w2]);
          Ch[s - 1][w2] += v[s - 1][w2];  // Ch_s(i) (its old value was last read above, at step s - 1)
        }
      }
    } else {
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) Dh[w2] = splat2(0.0f);  // M = 1: level 1 is all corners
    }
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (w2 + h * W2 >= nv) Dh[w2][h] = 0.0f;
    // adjoint of the second difference: E(i, j) = Dh(i, j-1) - Dh(i, j); Kh(i+1, j) = E(i, j) - E(i+1, j)
    float left = lane_prev(Dh[W2 - 1][1]);
    if (gl == 0) left = 0.0f;
    f2 Kh[W2];
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) {
      const f2 lf = (w2 == 0) ? (f2){left, Dh[W2 - 1][0]} : Dh[w2 - 1];
      const f2 e = lf - Dh[w2];
      Kh[w2] = e - EpA[w2];
      EpA[w2] = e;
    }
    emit(i + 1, Kh, kr1);
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) kr1[w2] = k0[w2];
  };

  if constexpr (RBF) {
    f2 Eqd[W2];
    exact_row(fxc + (long long)nrows * FS, kr1, Eqd);  // k row of the last point
    auto sweep = [&](auto clo_t) {
      for (int i0 = ((nrows - 1) / RC) * RC; i0 >= 0; i0 -= RC) {
        const int nr = nrows - i0 < RC ? nrows - i0 : RC;
        chunk(clo_t, i0, nr);
#pragma unroll 1
        for (int r = nr - 1; r >= 0; --r) {
          f2 dM[W2], k0[W2];
#pragma unroll
          for (int w2 = 0; w2 < W2; ++w2) {
            dM[w2] = cb[r][w2][lane];
            k0[w2] = cb[r][W2 + w2][lane];
          }
          rev_row(i0 + r, dM, k0);
        }
      }
    };
    if (clo)
      sweep(std::true_type{});
    else
      sweep(std::false_type{});
  } else {
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) kr1[w2] = splat2(1.0f);
    for (int i = nrows - 1; i >= 0; --i) {
      f2 dM[W2], k0[W2];
      lin_cells(i, dM);
#pragma unroll
      for (int w2 = 0; w2 < W2; ++w2) k0[w2] = splat2(1.0f);
      rev_row(i, dM, k0);
    }
  }
  {
    f2 Kh[W2];
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2) Kh[w2] = -EpA[w2];
    emit(0, Kh, kr1);
  }
  if (nslot > 0) flush();

  // ---- y-gradient of the pair's points (+ the level-1 corner terms of columns 0 and L2)
  if (pair_ok) {
    float *__restrict__ gyb = (diag ? p.gX : p.gY) + (long long)bl * l2 * d;
#pragma unroll
    for (int w2 = 0; w2 < W2; ++w2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = gl * W + w2 + h * W2;
        if (j >= l2) continue;
        float v[DP];
#pragma unroll
        for (int k = 0; k < DP; ++k) v[k] = RBF ? __builtin_fmaf(-A[w2][h], y[w2][k][h], B[w2][k][h]) : B[w2][k][h];
        if ((j == 0 || j == l2 - 1)) {
          double o[DP];
          corner(1, j == l2 - 1, o);
#pragma unroll
          for (int k = 0; k < DP; ++k) v[k] += (float)o[k];
        }
#pragma unroll
        for (int k = 0; k < DP; ++k)
          if (k < d) unsafeAtomicAdd(gyb + (long long)j * d + k, v[k]);
      }
  }

  // ---- dLoss/drs and dLoss/dscale of this pair (after the sweep: sig_bwd_kernel's norm_terms)
  if (diag || !(p.gscale || (p.rs1 && (p.grs1 || p.grs2)))) return;
  float gs[M + 1], sc[M + 1], r1[M + 1], r2[M + 1];
  pair_terms(gs, sc, r1, r2);
  const bool lead = gl == 0 && pair_ok;
  float g1v[M + 1], g2v[M + 1], gsc[M + 1];
#pragma unroll
  for (int m = 0; m <= M; ++m) {
    const float t = gs[m] * sc[m] * (K[m] + jit);
    g1v[m] = lead ? t * r2[m] : 0.0f;
    g2v[m] = t * r1[m];
    gsc[m] = lead ? gs[m] * (K[m] + jit) * r1[m] * r2[m] : 0.0f;
  }
  if (p.rs1 && p.grs1) {
    wave_sum_last_n<M + 1>(g1v);
    if (lane == 63)
      for (int m = 0; m <= M; ++m) unsafeAtomicAdd(p.grs1 + (long long)m * p.n1 + a, g1v[m]);
  }
  if (p.rs1 && p.grs2 && lead) {
#pragma unroll
    for (int m = 0; m <= M; ++m) unsafeAtomicAdd(p.grs2 + (long long)m * p.n2 + bl, g2v[m]);
  }
  if (p.gscale) {
    wave_sum_last_n<M + 1>(gsc);
    if (lane == 63) {
      float *slot = p.gscale + (long long)(lblk & (GSCALE_SLOTS - 1)) * (M + 1);
      for (int m = 0; m <= M; ++m) unsafeAtomicAdd(slot + m, gsc[m]);
    }
  }
}

// Column geometry of the packed VJP (one column block, LP W >= l2): W = 6 columns (3 pairs) per lane for the
// linear seed (DP <= 5, M <= 6: within 256 VGPRs), else 4 (the RBF seed's chunk state makes W = 6 spill);
// the narrowest lane group that covers l2 (most pairs per wave).
inline BwdGeo bwd_pk_geometry(int l2, int DP, int M, bool rbf) {
  if (DP > 8 || M > 8 || l2 < 2) return {0, 0};
  const bool w6 = !rbf && DP <= 5 && M <= 6;
  if (l2 <= 64) return {4, 16};
  if (w6 && l2 <= 120) return {6, 20};
  if (l2 <= 128) return {4, 32};
  if (w6 && l2 <= 192) return {6, 32};
  if (l2 <= 256) return {4, 64};
  return {0, 0};
}

}  // namespace gpsig
