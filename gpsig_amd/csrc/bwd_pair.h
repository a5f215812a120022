// gpsig_amd -- per-pair terms of the tile-emitting Gram VJPs (sig_bwd_wide.h, sig_ho_bwd.h): the level
// weights g_m = dLoss/dK_m(a, b) with the normalisation and scale factors, and the pair's contributions to
// dLoss/drs1, dLoss/drs2 and dLoss/dscale (as sig_bwd.h, whose kernel keeps its own inline copy).
#pragma once
#include "sig_bwd.h"

namespace gpsig {

template <int M>
struct PairTerms {
  const BwdArgs &p;
  int a, bl, gl;
  bool pair_ok, diag, upper_off;
  float jit;
  long long lblk;

  GPSIG_DEV PairTerms(const BwdArgs &p_, int a_, int bl_, int gl_, bool ok, long long lblk_)
      : p(p_), a(a_), bl(bl_), gl(gl_), pair_ok(ok), lblk(lblk_) {
    diag = p.pair_mode == GPSIG_PAIRS_DIAG;
    upper_off = p.pair_mode == GPSIG_PAIRS_UPPER && a != bl;
    jit = (p.pair_mode == GPSIG_PAIRS_UPPER && a == bl) ? p.jitter : 0.0f;
  }

  // upstream gradient (both triangle entries of an off-diagonal UPPER pair), scale, rs1, rs2 per level
  GPSIG_DEV void load(float (&gs)[M + 1], float (&sc)[M + 1], float (&r1)[M + 1], float (&r2)[M + 1]) const {
    float gsum = 0.0f;
    if (!diag && !p.gout_levels) {
      gsum = p.gout[(long long)a * p.g_ld + bl];
      if (upper_off) gsum += p.gout[(long long)bl * p.g_ld + a];
    }
#pragma unroll
    for (int m = 0; m <= M; ++m) {
      float gv;
      if (diag) {
        gv = p.gout[(long long)m * p.g_lvl + a];
      } else if (p.gout_levels) {
        gv = p.gout[(long long)m * p.g_lvl + (long long)a * p.g_ld + bl];
        if (upper_off) gv += p.gout[(long long)m * p.g_lvl + (long long)bl * p.g_ld + a];
      } else {
        gv = gsum;
      }
      gs[m] = pair_ok ? gv : 0.0f;
      sc[m] = p.scale ? p.scale[m] : 1.0f;
      r1[m] = p.rs1 ? p.rs1[(long long)m * p.n1 + a] : 1.0f;
      r2[m] = p.rs2 ? p.rs2[(long long)m * p.n2 + bl] : 1.0f;
    }
  }

  // g_m = dLoss/dK_m(a, b) of the raw levels
  GPSIG_DEV void weights(float (&gw)[M + 1]) const {
    float gs[M + 1], sc[M + 1], r1[M + 1], r2[M + 1];
    load(gs, sc, r1, r2);
#pragma unroll
    for (int m = 0; m <= M; ++m) gw[m] = gs[m] * sc[m] * r1[m] * r2[m];
  }

  // dLoss/drs and dLoss/dscale of this pair from its raw levels K (after the sweep: the factors are
  // reloaded here so only K stays live through it): grs1[m, a] summed over the wave (its pairs share a),
  // grs2[m, b] per pair, gscale into one of GSCALE_SLOTS partial sums
  GPSIG_DEV void norm(const float (&K)[M + 1]) const {
    if (diag || !(p.gscale || (p.rs1 && (p.grs1 || p.grs2)))) return;
    float gs[M + 1], sc[M + 1], r1[M + 1], r2[M + 1];
    load(gs, sc, r1, r2);
    const bool lead = gl == 0 && pair_ok;
    float g1[M + 1], g2[M + 1], gsc[M + 1];
#pragma unroll
    for (int m = 0; m <= M; ++m) {
      const float t = gs[m] * sc[m] * (K[m] + jit);
      g1[m] = lead ? t * r2[m] : 0.0f;
      g2[m] = t * r1[m];
      gsc[m] = lead ? gs[m] * (K[m] + jit) * r1[m] * r2[m] : 0.0f;
    }
    const int lane = (int)__lane_id();
    if (p.rs1 && p.grs1) {
      wave_sum_last_n<M + 1>(g1);
      if (lane == 63)
        for (int m = 0; m <= M; ++m) unsafeAtomicAdd(p.grs1 + (long long)m * p.n1 + a, g1[m]);
    }
    if (p.rs1 && p.grs2 && lead) {
#pragma unroll
      for (int m = 0; m <= M; ++m) unsafeAtomicAdd(p.grs2 + (long long)m * p.n2 + bl, g2[m]);
    }
    if (p.gscale) {
      wave_sum_last_n<M + 1>(gsc);
      if (lane == 63) {
        float *slot = p.gscale + (long long)(lblk & (GSCALE_SLOTS - 1)) * (M + 1);
        for (int m = 0; m <= M; ++m) unsafeAtomicAdd(slot + m, gsc[m]);
      }
    }
  }
};

}  // namespace gpsig
