/*
 * gpsig_amd -- C ABI of the MI355X (gfx950) signature-kernel evaluator.
 *
 * Drop-in boundary for the hot path of maudl3116/GPSig (paths relative to the reference root):
 *   - the per-pair level-M iterated-sums recursion behind SignatureKernel.K/Kdiag/K_tens_vs_seq
 *       gpsig/kernels.py:190-341 (_K_seq_diag/_K_seq/_K_tens/_K_tens_vs_seq, the algorithm seam)
 *       gpsig/signature_algs.py:8-160, gpsig/signature_algs_vosf.py:11-48
 *   - the Goursat-PDE solve behind kernels_pde.UntruncSignatureKernel.Kdiag
 *       gpsig/sigKer_fast.pyx:15-62 (Cython, OpenMP)
 *       gpsig/covariance_op/untrunc_cov_op_gpu.cu:5-94 + untrunc_cov_op_gpu.cc:13-150 (CUDA TF op)
 *
 * Conventions (all entry points):
 *   - device pointers, caller-owned buffers, row-major contiguous float32;
 *   - sequences are (n, l, d): n sequences of l points in R^d (the reference's (N, L*D) input after
 *     the reshape at gpsig/kernels.py:418-420, with scaling/lags already applied by the host);
 *   - every call is stream-ordered on `stream` (the caller's current HIP stream), allocates nothing
 *     (scratch comes from the caller's workspace, sized by the *_workspace_bytes query), performs no
 *     host synchronisation, and is therefore capturable in a hipGraph;
 *   - the return value is GPSIG_OK (0) or a negative error code (no exceptions, no aborts).
 */
#ifndef GPSIG_AMD_H
#define GPSIG_AMD_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *gpsig_stream_t; /* == hipStream_t */

enum gpsig_status {
  GPSIG_OK = 0,
  GPSIG_EINVAL = -1,       /* bad shape / argument */
  GPSIG_EUNSUPPORTED = -2, /* configuration outside the compiled instantiations */
  GPSIG_ELAUNCH = -3,      /* HIP launch error (hipGetLastError after the launch) */
  GPSIG_EWORKSPACE = -4    /* workspace too small */
};

/* Base (state-space) kernels, gpsig/kernels.py:966-1173. */
enum gpsig_base_kind {
  GPSIG_BASE_RBF = 0,    /* SignatureRBF._rbf      kernels.py:1042 : exp(-|x-y|^2/2)  */
  GPSIG_BASE_LINEAR = 1, /* SignatureLinear._lin   kernels.py:979  : <x, y>           */
  /* Flag OR-ed into base_kind of gpsig_sig_gram / gpsig_sig_diag (RBF, order 1, difference 1, no saved
   * state): evaluate the seed's increment inner products <y_j, dx_i>, <dy_j, dx_i> (the reference's
   * seed GEMM, kernels.py:946-957 + 1042-1044) on the matrix cores (v_mfma_f32_4x4x1_16b_f32) instead of
   * packed VALU FMAs.  Bitwise the same results; slower on MI355X, kept as the A/B arm. */
  GPSIG_BASE_SEED_MFMA = 0x100,
  /* Flag OR-ed into base_kind of gpsig_sig_gram (RBF, order 1, difference 1, Gram pairs, no saved state,
   * sequences within one lane group): the split design of SURVEY.md 8d as a diagnostic -- a producer
   * launch writes every pair's cells dM (fp32) to the workspace, a consumer launch streams them from HBM
   * through the recursion, in chunks of pairs.  Same results as the fused kernel; the consumer's HBM
   * traffic is the recursion's algorithmic bytes.  Workspace: gpsig_sig_workspace_bytes(...) +
   * gpsig_sig_split_bytes(...). */
  GPSIG_GRAM_SPLIT = 0x200
};

/* Which (a, b) sequence pairs a Gram call evaluates. */
enum gpsig_pair_mode {
  GPSIG_PAIRS_RECT = 0,  /* all a in [row_begin,row_end) x all b in [0,n2)           (K(X, X2)) */
  GPSIG_PAIRS_UPPER = 1, /* a in [row_begin,row_end), b in [a, n)  (Y == X, K(X))  + mirrored store */
  GPSIG_PAIRS_DIAG = 2   /* (a, a) for a in [row_begin,row_end)           (_K_seq_diag) */
};

/* What a Gram / diag call writes. L = num_levels. */
enum gpsig_out_mode {
  GPSIG_OUT_LEVELS = 0,      /* raw per-level values K_m, out (L+1, out_rows, n2) [diag: (L+1, n)] */
  GPSIG_OUT_NORM_LEVELS = 1, /* scale[m] * (K_m + jit) * rs1[m,a] * rs2[m,b], (L+1, out_rows, n2) */
  GPSIG_OUT_NORM_SUM = 2,    /* sum over m of the above, (out_rows, n2)                             */
  GPSIG_OUT_RSQRT = 3        /* diag only: 1/sqrt(K_m(a,a) + jitter), (L+1, n)                      */
};

/* ---------------------------------------------------------------------------------------------
 * Truncated signature kernel, seq x seq.
 *
 * Replaces _K_seq / _K_seq_diag (kernels.py:190-238) = base kernel tensor (kernels.py:946-1044)
 * + signature_kern_first_order (signature_algs.py:8-35, order == 1) or
 * signature_kern_higher_order (signature_algs.py:37-74, order > 1), with the normalisation and
 * sigma*variances epilogue of SignatureKernel.K (kernels.py:431-477) fused in (out_mode 1/2).
 *
 *   X (n1, l1, d), Y (n2, l2, d); for GPSIG_PAIRS_UPPER / DIAG pass Y == X (n2 == n1, l2 == l1).
 *   order: 1 = first order; >1 = higher order (clamped by the caller as kernels.py:58 does).
 *   difference: kernels.py `difference` flag (second-difference the base-kernel grid).
 *   rs1 (L+1, n1), rs2 (L+1, n2): 1/sqrt(diag + jitter) from gpsig_sig_diag(GPSIG_OUT_RSQRT), or
 *     NULL for "no normalisation".  scale (L+1): sigma * variances (NULL = ones).
 *   jitter: added to K_m(a,a) before normalising in GPSIG_PAIRS_UPPER (kernels.py:432).
 *   out rows are a - out_row0 for a in [out_row0, out_row0 + out_rows); in UPPER mode the mirrored
 *     entry (b, a) is also stored when b lies in that row window.
 */
size_t gpsig_sig_workspace_bytes(int n1, int l1, int n2, int l2, int d);
/* The workspace of one gpsig_sig_gram / gpsig_sig_diag call given its order and pair mode: as above,
 * except the higher-order recursion past 32 channels, whose cells come from a tile -- for the linear base
 * kernel the reference's tf.matmul (kernels.py:1042-1044), a matrix-core GEMM per chunk of x-rows; for the
 * RBF base kernel the matrix-core cell producer of the wide first-order Gram -- the increments plus one
 * chunk's tile (<= 1 GiB).  Channel bound of the RBF higher order past 32 channels: the producer keeps one
 * y-sequence's increments in LDS (160 KiB), which holds d up to about 180 channels at 129-160 points and
 * about 240 otherwise; past that the call returns GPSIG_EUNSUPPORTED (the linear kernel has no bound). */
size_t gpsig_sig_workspace_bytes_ex(int n1, int l1, int n2, int l2, int d, int order, int pair_mode);
/* Extra workspace of a GPSIG_GRAM_SPLIT call (one chunk of pairs' cells); 0 where the split does not apply. */
size_t gpsig_sig_split_bytes(int l1, int l2, int d, int num_levels);

int gpsig_sig_gram(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int num_levels,
                   int order, int base_kind, int difference, int pair_mode, int row_begin, int row_end,
                   const float *rs1, const float *rs2, const float *scale, float jitter, int out_mode,
                   float *out, int out_row0, int out_rows, void *workspace, size_t workspace_bytes,
                   gpsig_stream_t stream);

/* Training variant of gpsig_sig_gram: also saves, per evaluated pair (a, b), the forward state the
 * VJP would otherwise recompute -- the column sums C_m(L1-1, j) of levels 1..L-1 at the end of the row
 * sweep (j < l2-1) and the raw levels K_1..K_L -- so that gpsig_sig_gram_vjp given the same `state`
 * skips its forward sweep.  The reference keeps every (N1, L1, N2, L2) intermediate of the TF graph
 * alive for autodiff (kernels.py:209-238); this keeps (L-1)(l2-1) + L floats per pair.
 * Pair slot: RECT a*n2 + b; UPPER the row-major upper triangle a*n2 - a(a-1)/2 + (b - a).
 * order == 1, difference == 1, pair_mode RECT or UPPER; state_bytes >= gpsig_sig_state_bytes(...). */
size_t gpsig_sig_state_bytes(int n1, int n2, int l2, int num_levels, int pair_mode);
int gpsig_sig_gram_state(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int num_levels,
                         int base_kind, int pair_mode, int row_begin, int row_end, const float *rs1,
                         const float *rs2, const float *scale, float jitter, int out_mode, float *out,
                         int out_row0, int out_rows, float *state, size_t state_bytes, void *workspace,
                         size_t workspace_bytes, gpsig_stream_t stream);

/* Diagonal k(x_a, x_a) per level: _K_seq_diag (kernels.py:190-207).  out_mode LEVELS or RSQRT. */
int gpsig_sig_diag(const float *X, int n, int l, int d, int num_levels, int order, int base_kind, int difference,
                   float jitter, int out_mode, float *out, void *workspace, size_t workspace_bytes,
                   gpsig_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Gradient of the first-order Gram (vector-Jacobian product).
 *
 * The reference obtains dLoss/dX of K (and through the host-side scaling dLoss/dlengthscales) by TF
 * autodiff of the graph kernels.py:209-238 (base kernel, kernels.py:946-1044) ->
 * signature_algs.py:8-35 -> kernels.py:431-477 (jitter, normalisation, sigma*variances).  This entry
 * evaluates the same derivative for order == 1, RBF and linear base kernels, difference == 1 (second
 * difference of the base-kernel grid, the default) or 0 (the grid itself, kernels.py:19 `difference`):
 *
 *   gout_levels == 0: gout (n1, n2) is dLoss/dK for out_mode GPSIG_OUT_NORM_SUM;
 *   gout_levels == 1: gout (L+1, n1, n2) is dLoss/dK_m for GPSIG_OUT_LEVELS / GPSIG_OUT_NORM_LEVELS;
 *   GPSIG_PAIRS_DIAG: gout (L+1, n1) per-level dLoss/dK_m(a, a) of gpsig_sig_diag (gout_levels = 1).
 *   rs1/rs2/scale/jitter: as in the forward call (NULL = none).  Accumulated (+=) outputs:
 *   gX (n1, l1, d) and gY (n2, l2, d) (UPPER / DIAG: Y == X and everything goes to gX);
 *   grs1 (L+1, n1), grs2 (L+1, n2) = dLoss/drs (the host chains them through rs = (diag+jitter)^-1/2
 *   into a DIAG call); gscale (L+1) = dLoss/dscale.  Any of grs1/grs2/gscale may be NULL.
 *   state: NULL, or the buffer a gpsig_sig_gram_state call with the same inputs filled (RECT/UPPER).
 *   Workspace: gpsig_sig_vjp_workspace_bytes(n1, l1, n2, l2, d, num_levels, difference): the feature
 *   records, for sequences longer than one lane group covers (column blocks) the per-row carries of
 *   one launch chunk, and the partial sums of gscale (reduced into gscale after the launch, on the
 *   same stream).  Any length up to 16 channels; above 16 (wide channels) l2 <= 512, the point weights
 *   of a chunk of pairs go to a tile in the workspace and the matrix-core GEMMs (gpsig_gemm_f32) contract
 *   them with the points.
 */
size_t gpsig_sig_vjp_workspace_bytes(int n1, int l1, int n2, int l2, int d, int num_levels, int difference);
int gpsig_sig_gram_vjp(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int num_levels,
                       int base_kind, int difference, int pair_mode, int row_begin, int row_end, const float *gout, int gout_levels,
                       const float *rs1, const float *rs2, const float *scale, float jitter, float *gX, float *gY,
                       float *grs1, float *grs2, float *gscale, const float *state, void *workspace,
                       size_t workspace_bytes, gpsig_stream_t stream);

/* Gradient of the higher-order Gram (order > 1): TF autodiff of signature_kern_higher_order
 * (signature_algs.py:37-74) behind _K_seq / K.  Arguments as gpsig_sig_gram_vjp (difference = 1, no
 * saved state); order 1 forwards to it.  Supported: RBF / linear, any channel count, l2 <= 512, and
 * min(order, num_levels) <= 6 where the row state fits the LDS (l2 <= 256: order 2-4 to 8 levels,
 * order 5 to 7, order 6 at 6; l2 <= 512: order 2 to 8 levels, 3 to 7, 4 to 5, 5 at 5), and 510 <= l2 <= 1017
 * at order 2 to 7 levels, 3 to 6, 4 and 5 to 5 (8 waves per pair, the multiplier slabs in the workspace: the
 * workspace query includes them); otherwise GPSIG_EUNSUPPORTED, and the workspace query returns 0. */
size_t gpsig_sig_vjp_ho_workspace_bytes(int n1, int l1, int n2, int l2, int d, int num_levels, int order,
                                        int base_kind);
int gpsig_sig_gram_vjp_ho(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int num_levels,
                          int order, int base_kind, int pair_mode, int row_begin, int row_end, const float *gout,
                          int gout_levels, const float *rs1, const float *rs2, const float *scale, float jitter,
                          float *gX, float *gY, float *grs1, float *grs2, float *gscale, void *workspace,
                          size_t workspace_bytes, gpsig_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Inducing tensors (sparse rank-1 tensors z = (z_{m,1} (x) ... (x) z_{m,m})_m).
 *
 * gpsig_tens_vs_seq replaces _K_tens_vs_seq (kernels.py:314-341) = base kernel between tensor
 * components and sequence points + signature_kern_tens_vs_seq_first_order / _higher_order
 * (signature_algs.py:101-160).  Z (LT, T, d), or (LT, T, 2, d) with increments (kernels.py:328-331),
 * LT = num_levels (num_levels+1) / 2; X (n, l, d).  out (num_levels+1, T, n), raw (unnormalised).
 *
 * gpsig_tens_gram replaces _K_tens (kernels.py:264-284) + tensor_kern (signature_algs.py:76-99):
 * out (num_levels+1, T, T).
 *
 * gpsig_rescaled replaces _Mahalanobis_term_approx_posterior (kernels.py:800-822, linear embedding
 * = 0; kernels_pde.py:191-222, per-coordinate RBF embedding = 1) + signature_kern_rescaled_higher_order
 * (signature_algs_vosf.py:11-48): <S(x_n), (I - Lambda_t) S(x_n)> per level with Lambda_t the rank-1
 * diagonal built from Z (LT, T, d).  out (num_levels+1, n, T).
 */
/* Workspace of gpsig_tens_vs_seq for n sequences of l points in d channels and lt x t components. */
size_t gpsig_tens_workspace_bytes(int n, int l, int d, int lt, int t);

int gpsig_tens_vs_seq(const float *Z, int lt, int t, int increments, int d, const float *X, int n, int l,
                      int num_levels, int order, int base_kind, int difference, float *out, void *workspace,
                      size_t workspace_bytes, gpsig_stream_t stream);

/* Tensor Gram (_K_tens, kernels.py:264-284): out (num_levels+1, T, T).  Channel counts past 32 run as pair
 * tiles (the VJP's component-kernel tile kernel) and need the workspace the query names (0 for d <= 32). */
size_t gpsig_tens_gram_workspace_bytes(int lt, int t, int d);
int gpsig_tens_gram(const float *Z, int lt, int t, int increments, int d, int num_levels, int base_kind, float *out,
                    void *workspace, size_t workspace_bytes, gpsig_stream_t stream);

/* Gradient of gpsig_tens_gram (tensor_kern, signature_algs.py:76-99, over _K_tens, kernels.py:264-284):
 * gout (num_levels+1, T, T) = dLoss/d(raw per-level output); accumulates (+=) gZ (same layout as Z).
 * Channel counts past 32 run as pair tiles + matrix-core GEMMs and need the workspace the query names
 * (0 for d <= 32: workspace may be NULL). */
size_t gpsig_tens_gram_vjp_workspace_bytes(int lt, int t, int increments, int d, int num_levels, int base_kind);
int gpsig_tens_gram_vjp(const float *Z, int lt, int t, int increments, int d, int num_levels, int base_kind,
                        const float *gout, float *gZ, void *workspace, size_t workspace_bytes, gpsig_stream_t stream);

/* gpsig_tens_vs_seq for a training step: the same output (order 1, difference 1, RBF or linear, d <= 8,
 * num_levels <= 6 -- the packed fast paths; GPSIG_EUNSUPPORTED otherwise, nothing launched) plus the
 * VJP's saved state: state (T, n, LT) = every component's end-of-sweep running sum (the TF graph's
 * saved intermediates for autodiff of _K_tens_vs_seq, kernels.py:314-341).  Workspace as
 * gpsig_tens_vs_seq. */
int gpsig_tens_vs_seq_state(const float *Z, int lt, int t, int increments, int d, const float *X, int n, int l,
                            int num_levels, int base_kind, float *out, float *state, void *workspace,
                            size_t workspace_bytes, gpsig_stream_t stream);

/* Gradient of gpsig_tens_vs_seq (order 1, difference 1 or 0, RBF or linear, num_levels <= 8, any d):
 * the reference differentiates _K_tens_vs_seq (kernels.py:314-341 + signature_algs.py:101-127) by TF
 * autodiff.  gout (num_levels+1, T, n) = dLoss/d(raw per-level output); accumulates (+=) gZ (same
 * layout as Z) and gX (n, l, d).  state: NULL, or the buffer a gpsig_tens_vs_seq_state call on the same
 * inputs filled (difference 1): the VJP then skips its forward sweep.  Workspace:
 * gpsig_tens_vjp_workspace_bytes(n, l, d) for d <= 16, gpsig_tens_vjp_wide_workspace_bytes(...) above. */
size_t gpsig_tens_vjp_workspace_bytes(int n, int l, int d);
/* Workspace of gpsig_tens_vs_seq_vjp at d > 16 (point-weight tiles of a chunk of sequences and the emission
 * GEMMs on the matrix cores; any channel count). */
size_t gpsig_tens_vjp_wide_workspace_bytes(int n, int l, int d, int lt, int t);

int gpsig_tens_vs_seq_vjp(const float *Z, int lt, int t, int increments, int d, const float *X, int n, int l,
                          int num_levels, int base_kind, int difference, const float *gout, float *gZ, float *gX,
                          const float *state, void *workspace, size_t workspace_bytes, gpsig_stream_t stream);

size_t gpsig_rescaled_workspace_bytes(int n, int num_levels);

int gpsig_rescaled(const float *Z, int lt, int t, const float *X, int n, int l, int d, int num_levels,
                   int embedding, float *out, void *workspace, size_t workspace_bytes, gpsig_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Goursat PDE (untruncated signature kernel).
 *
 * Replaces sig_kern_diag (sigKer_fast.pyx:15-62) and the UntruncCov op
 * (untrunc_cov_op_gpu.cc:13-25 -> UntruncCovKernelLauncher, untrunc_cov_op_gpu.cu:71-81), which
 * solve k(x, x) only; gpsig_pde_gram adds the cross Gram the reference lacks (kernels_pde.py:107
 * calls an undefined K).  dyadic = the reference `order`/`n` (grid refined 2^dyadic per increment),
 * solver 1 = explicit scheme (sigKer_fast.pyx:48 / .cu:29), 0 = first-order scheme (:46).
 * out: final corner K[-1,-1] per pair (kernels_pde.py:185 takes K_diag[:, -1, -1]).
 */
int gpsig_pde_gram(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                   int pair_mode, int row_begin, int row_end, float *out, int out_row0, int out_rows,
                   gpsig_stream_t stream);

int gpsig_pde_diag(const float *X, int n, int l, int d, int dyadic, int solver, float *out, gpsig_stream_t stream);

/* Channel counts past 16 and dyadic orders past 4 run the solver on increment tiles: the coarse increment Gram
 * <dx_i, dy_j> of a chunk of pairs is one matrix-core GEMM (the reference's own split, kernels_pde.py:176
 * tf.matmul before the op), the solver reads it; any channel count, dyadic <= 8.  Those calls need a scratch
 * of gpsig_pde_scratch_bytes(...) bytes (0 otherwise; the entries above pass none and return
 * GPSIG_EWORKSPACE there). */
size_t gpsig_pde_scratch_bytes(int n1, int l1, int n2, int l2, int d, int dyadic, int pair_mode);
int gpsig_pde_gram_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                      int pair_mode, int row_begin, int row_end, float *out, int out_row0, int out_rows, void *scratch,
                      size_t scratch_bytes, gpsig_stream_t stream);
int gpsig_pde_diag_ex(const float *X, int n, int l, int d, int dyadic, int solver, float *out, void *scratch,
                      size_t scratch_bytes, gpsig_stream_t stream);

/* Gradient of gpsig_pde_gram / gpsig_pde_diag: the reference's own adjoint (kernels_pde.py:465-509,
 * _KdiagGrad; covariance_op/_untrunc_cov_grad.py:25-77): KK = K (.) flip(K_rev) with K_rev solved on the
 * time-reversed paths by the first-order scheme, contracted with the increments.  pair_mode DIAG
 * (gout (n1,), dLoss/dk(x_a, x_a); the reference's factor 2 for the symmetric pair) or RECT (gout
 * (n1, n2); gX and gY).  Accumulates (+=) gX (n1, l1, d), gY (n2, l2, d).  No grid is stored: K_rev
 * is re-solved on the mirrored wavefront and meets the forward sweep lane by lane; the workspace holds
 * the forward sweep's fronts (fp32, every few coarse steps, about (1 + REP/W) I J / H floats per pair;
 * I = 2^dyadic (l1-1), J = 2^dyadic (l2-1)), gpsig_pde_vjp_workspace_bytes(pairs, l1, l2, dyadic), which
 * returns 0 where the kernel does not apply.  Wider grids than one wave's 64 W columns are swept in column
 * blocks; their fp64 boundary columns are part of the workspace.  Past dyadic 3 (and past 16 channels) the
 * _ex entries below apply (the fronts then follow the grid refined 2^(dyadic - 3) per tile cell).  dyadic <= 8,
 * as the forward. */
size_t gpsig_pde_vjp_workspace_bytes(int npairs, int l1, int l2, int dyadic);

int gpsig_pde_vjp(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                  int pair_mode, int row_begin, int row_end, const float *gout, float *gX, float *gY, void *workspace,
                  size_t workspace_bytes, gpsig_stream_t stream);

/* The forward of a training step split off gpsig_pde_vjp: gpsig_pde_fronts evaluates k(x_a, y_b) of the
 * pairs (pair_mode RECT: out[(a - row_begin) * n2 + b]; DIAG: out[a - row_begin]; the values of
 * gpsig_pde_gram / gpsig_pde_diag, same cells) and leaves the adjoint's forward fronts in `fronts`
 * (gpsig_pde_vjp_workspace_bytes(pairs, l1, l2, dyadic) bytes); gpsig_pde_vjp_fronts on the same inputs
 * and rows then runs only the adjoint's backward sweeps (one solve of the grid fewer than gpsig_pde_vjp). */
int gpsig_pde_fronts(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                     int pair_mode, int row_begin, int row_end, float *out, void *fronts, size_t fronts_bytes,
                     gpsig_stream_t stream);

int gpsig_pde_vjp_fronts(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                         int solver, int pair_mode, int row_begin, int row_end, const float *gout, float *gX,
                         float *gY, const void *fronts, size_t fronts_bytes, gpsig_stream_t stream);

/* The adjoint entries with the scratch of the increment-tile path (d > 16 or dyadic > 3: the increment
 * tile, the adjoint's coarse-cell sums as dLoss/d<dx_i, dy_j> in a tile of the same layout, contracted with
 * the increments by two matrix-core GEMMs); gpsig_pde_vjp_scratch_bytes(...) bytes, 0 where the fixed
 * kernels apply. */
size_t gpsig_pde_vjp_scratch_bytes(int n1, int l1, int n2, int l2, int d, int dyadic, int pair_mode);
int gpsig_pde_vjp_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                     int pair_mode, int row_begin, int row_end, const float *gout, float *gX, float *gY,
                     void *workspace, size_t workspace_bytes, void *scratch, size_t scratch_bytes,
                     gpsig_stream_t stream);
int gpsig_pde_fronts_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic, int solver,
                        int pair_mode, int row_begin, int row_end, float *out, void *fronts, size_t fronts_bytes,
                        void *scratch, size_t scratch_bytes, gpsig_stream_t stream);
int gpsig_pde_vjp_fronts_ex(const float *X, int n1, int l1, const float *Y, int n2, int l2, int d, int dyadic,
                            int solver, int pair_mode, int row_begin, int row_end, const float *gout, float *gX,
                            float *gY, const void *fronts, size_t fronts_bytes, void *scratch, size_t scratch_bytes,
                            gpsig_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Truncated signatures (replaces iisignature.sig behind iisignature_tensorflow.Sig,
 * gpsig/iisignature_tensorflow.py:87, used by the VOSF Kuf, gpsig/inducing_variables_vosf.py:120-146).
 * X (n, l, d) -> out (n, gpsig_signature_channels(d, depth)): levels 1..depth, each flattened
 * first-index-major, concatenated (iisignature.sig's layout).  Any size the int32 entry index takes (channels
 * < 2^29, d channels < 2^32): while (channels + d) * 4 <= 160 KiB the levels live in a CU's LDS, past it in
 * per-path slabs of the caller's workspace (gpsig_signature_workspace_bytes, 0 for the LDS case).
 */
long long gpsig_signature_channels(int d, int depth);

/* Workspace of gpsig_signature_ex (vjp = 0) / gpsig_signature_vjp_ex (vjp = 1): 0 when the levels fit the
 * LDS, else the slabs of one launch chunk of paths (at most 1 GiB, at least one path). */
size_t gpsig_signature_workspace_bytes(int n, int d, int depth, int vjp);

int gpsig_signature_ex(const float *X, int n, int l, int d, int depth, float *out, void *workspace,
                       size_t workspace_bytes, gpsig_stream_t stream);

/* gpsig_signature_ex without a workspace: GPSIG_EWORKSPACE past the LDS. */
int gpsig_signature(const float *X, int n, int l, int d, int depth, float *out, gpsig_stream_t stream);

/* Gradient of gpsig_signature (iisignature.sigbackprop behind the Sig op's gradient): gout (n, channels)
 * = dLoss/dsig; accumulates (+=) gX (n, l, d).  The levels, their adjoints and two tables of the step's
 * exponential: (4 channels + 2 d) * 4 bytes in LDS up to 160 KiB, past it in the workspace. */
int gpsig_signature_vjp_ex(const float *X, int n, int l, int d, int depth, const float *gout, float *gX,
                           void *workspace, size_t workspace_bytes, gpsig_stream_t stream);

int gpsig_signature_vjp(const float *X, int n, int l, int d, int depth, const float *gout, float *gX,
                        gpsig_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * Multi-GPU assembly helper (no reference counterpart: the reference has no distributed code).
 * After an all-gather of UPPER-mode row blocks, build the full symmetric matrix:
 *   dst[l][a][b] = src[row_off[a] + l*level_stride + b]   for b >= a,
 *                  src[row_off[b] + l*level_stride + a]   otherwise;   dst (levels, n, n).
 * row_off (n): element offset of global row a (level 0) inside the gathered buffer.
 */
int gpsig_sym_assemble(const float *src, const long long *row_off, long long level_stride, int n, int levels,
                       float *dst, gpsig_stream_t stream);

/* ---------------------------------------------------------------------------------------------
 * fp32 GEMM on the matrix cores (v_mfma_f32_32x32x2_f32), the engine of the wide-channel paths' inner-
 * product GEMMs (the PDE increment Gram, the VJPs' emission products).  Exposed for tests:
 *   C = alpha op(A) op(B) + beta C, row-major, op(A) M x K, op(B) K x N; trans* = 1 transposes.
 */
int gpsig_gemm_f32(int transA, int transB, int M, int N, int K, float alpha, const float *A, long long lda,
                   const float *B, long long ldb, float beta, float *C, long long ldc, gpsig_stream_t stream);
/* The same with K split into slices whose partial products are summed in a fixed order (products with few
 * output tiles and a long K); workspace of gpsig_gemm_splitk_bytes(M, N, K) bytes (0: no split). */
size_t gpsig_gemm_splitk_bytes(int M, int N, int K);
int gpsig_gemm_f32_splitk(int transA, int transB, int M, int N, int K, float alpha, const float *A, long long lda,
                          const float *B, long long ldb, float beta, float *C, long long ldc, void *workspace,
                          size_t workspace_bytes, gpsig_stream_t stream);

/* Library identification (for tests: the loaded object must be this build). */
const char *gpsig_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GPSIG_AMD_H */
