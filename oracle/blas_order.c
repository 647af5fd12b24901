/*
 * TEST INFRASTRUCTURE (oracle) -- never linked into or called by the product.
 *
 * The reference's non-causal backward pass (src/maxent.py:140-159) restated in
 * the exact floating-point order numpy 2.2 / OpenBLAS 0.3.29 give it on x86-64
 * hosts whose OpenBLAS core is Haswell-family (Haswell, SkylakeX, Zen -- the
 * DYNAMIC_ARCH kernels that share dgemv_t_4.c with the Haswell micro-kernel),
 * single-threaded partition (OPENBLAS_NUM_THREADS=1, or any thread count for
 * S <= 625).  Pinned bit for bit against the reference's own outputs
 * (tests/golden/maxent_small.npz, config1.npz) and against np.dot on the host
 * (tests/test_oracle_blas_order.py).  The order, established by probing np.dot
 * with one-, two- and three-nonzero rows (fma vs. separately rounded sums):
 *
 *   maxent.py:155  p[a].dot(zs), p[a] C-contiguous S x S  ->  cblas dgemv,
 *                  OpenBLAS dgemv_t on the column-major view; per output row s:
 *     - the first m1 = S - S % 4 columns in blocks of 2048 (NBMAX); inside a
 *       block four lane accumulators, lane = column % 4, starting at 0:
 *         rows s <  S & ~3 (dgemv_kernel_4x4): lane = fma(a, x, lane)
 *         rows s >= S & ~3 (dgemv_kernel_4x1): lane = lane + a * x (rounded product)
 *       block sum (l0 + l2) + (l1 + l3); y = ((0 + block0) + block1) ...
 *     - the remaining S % 4 columns: y = fma(a, x, y), ascending (S % 4 == 1;
 *       S % 4 in {2, 3} use other kernels and are not restated: rejected)
 *   maxent.py:155  er * dot        one rounded product
 *   maxent.py:156  za.sum(axis=1)  ((za0 + za1) + za2) + za3, sequential
 *   maxent.py:159  za / zs         IEEE division
 *
 * Zero entries contribute fma(0, x, acc) = acc exactly while x is finite; a
 * non-finite partition value makes every later dot NaN (0 * inf), which the
 * dense restatement below reproduces by running over all S columns.
 */

#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NBMAX 2048

/* y[s] = sum_t M[s][t] x[t], M row-major n x n, in OpenBLAS Haswell dgemv_t order
 * with column blocks of nbmax (the tests run it with an unbounded block too, to
 * show that numpy's results at S > 2048 do depend on the NBMAX split). */
int blas_order_dgemv_rows_nb(const double* M, int n, const double* x, double* y, int nbmax) {
  if (n <= 0 || (n & 3) > 1 || nbmax <= 0) return -1;
  const int m1 = n - (n & 3), n4 = n & ~3;
  for (int s = 0; s < n; ++s) {
    const double* a = M + (size_t)s * n;
    const int fused = s < n4;
    double out = 0.0;
    for (int lo = 0; lo < m1; lo += nbmax) {
      const int hi = nbmax < m1 - lo ? lo + nbmax : m1;
      double l[4] = {0.0, 0.0, 0.0, 0.0};
      for (int t = lo; t < hi; ++t) {
        const int q = (t - lo) & 3;
        l[q] = fused ? fma(a[t], x[t], l[q]) : l[q] + a[t] * x[t];
      }
      out = out + ((l[0] + l[2]) + (l[1] + l[3]));
    }
    for (int t = m1; t < n; ++t) out = fma(a[t], x[t], out);
    y[s] = out;
  }
  return 0;
}

int blas_order_dgemv_rows(const double* M, int n, const double* x, double* y) {
  return blas_order_dgemv_rows_nb(M, n, x, y, NBMAX);
}

/*
 * local_action_probabilities (maxent.py:119-159) in that order.
 *   P  [S][S][A] C order (the reference's p_transition), term [S] (1 = terminal),
 *   er [S] = np.exp(reward) computed by the caller with numpy (maxent.py:142),
 *   pi [S][A] out.
 */
int blas_order_backward_maxent(const double* P, int S, int A, const uint8_t* term, const double* er,
                               double* pi) {
  if (S <= 0 || A <= 0 || (S & 3) > 1) return -1;
  double* pa = malloc((size_t)A * S * S * sizeof(double));
  double* zs = malloc((size_t)S * sizeof(double));
  double* dot = malloc((size_t)S * sizeof(double));
  double* za = malloc((size_t)S * A * sizeof(double));
  if (!pa || !zs || !dot || !za) {
    free(pa); free(zs); free(dot); free(za);
    return -2;
  }
  for (int a = 0; a < A; ++a)  /* maxent.py:143: the C-contiguous slices p[a] */
    for (int s = 0; s < S; ++s)
      for (int t = 0; t < S; ++t) pa[((size_t)a * S + s) * S + t] = P[((size_t)s * S + t) * A + a];
  for (int s = 0; s < S; ++s) zs[s] = term[s] ? 1.0 : 0.0;  /* maxent.py:146-147 */
  for (int it = 0; it < 2 * S; ++it) {                      /* maxent.py:154 */
    for (int a = 0; a < A; ++a) {
      blas_order_dgemv_rows(pa + (size_t)a * S * S, S, zs, dot);
      for (int s = 0; s < S; ++s) za[(size_t)s * A + a] = er[s] * dot[s];
    }
    for (int s = 0; s < S; ++s) {
      double z = za[(size_t)s * A];
      for (int a = 1; a < A; ++a) z = z + za[(size_t)s * A + a];
      zs[s] = z;
    }
  }
  for (int s = 0; s < S; ++s)
    for (int a = 0; a < A; ++a) pi[(size_t)s * A + a] = za[(size_t)s * A + a] / zs[s];
  free(pa); free(zs); free(dot); free(za);
  return 0;
}

/*
 * value_iteration / stochastic_value_iteration (solver.py:9-52, 55-104) in that
 * order: q_a = discount * (p[a] @ v) (np.matrix @ 1-d: the same dgemv), then
 * v = reward + max_a q_a (exact; NaN propagates as np.max does) or
 * reward + ((q_0 + q_1) + ...) / A (np.average over axis 0), until
 * max|v_old - v| <= eps.  P [S][S][A] C order; returns the sweep count (or < 0).
 */
long long blas_order_value_iteration(const double* P, int S, int A, const double* reward, double discount,
                                     double eps, int average, long long max_iter, double* v) {
  if (S <= 0 || A <= 0 || (S & 3) > 1) return -1;
  double* pa = malloc((size_t)A * S * S * sizeof(double));
  double* q = malloc((size_t)A * S * sizeof(double));
  double* vo = malloc((size_t)S * sizeof(double));
  if (!pa || !q || !vo) {
    free(pa); free(q); free(vo);
    return -2;
  }
  for (int a = 0; a < A; ++a)
    for (int s = 0; s < S; ++s)
      for (int t = 0; t < S; ++t) pa[((size_t)a * S + s) * S + t] = P[((size_t)s * S + t) * A + a];
  for (int s = 0; s < S; ++s) v[s] = 0.0;  /* solver.py:29 */
  long long it = 0;
  double delta = INFINITY;
  while (delta > eps && (max_iter <= 0 || it < max_iter)) {
    for (int s = 0; s < S; ++s) vo[s] = v[s];
    for (int a = 0; a < A; ++a) {
      blas_order_dgemv_rows(pa + (size_t)a * S * S, S, vo, q + (size_t)a * S);
      for (int s = 0; s < S; ++s) q[(size_t)a * S + s] = discount * q[(size_t)a * S + s];
    }
    delta = 0.0;
    for (int s = 0; s < S; ++s) {
      double m = q[s];
      for (int a = 1; a < A; ++a) {
        const double x = q[(size_t)a * S + s];
        if (average) m = m + x;
        else if (m == m && (x != x || x > m)) m = x;  /* np.max: NaN wins */
      }
      v[s] = reward[s] + (average ? m / (double)A : m);
      const double d = fabs(vo[s] - v[s]);
      if (d != d || d > delta) delta = d != d ? NAN : (delta != delta ? delta : d);
    }
    ++it;
  }
  free(pa); free(q); free(vo);
  return it;
}

/*
 * y[t] = sum_s M[s][t] x[s] -- numpy's M.T.dot(x) for a C-contiguous square M
 * (maxent.py:109: p_transition[a].T.dot(...)), i.e. OpenBLAS dgemv_n on the
 * column-major view, in its Haswell order (probed like dgemv_t above): for
 * outputs t < n & ~3, per group of four sources s = 4g .. 4g + 3 a chain
 * round(a1 x1), fma a0, fma a2, fma a3, added to y group after group, then the
 * remaining n % 4 sources as rounded products added one by one; the last
 * n % 4 outputs one fma chain over all sources in order.
 */
int blas_order_dgemv_cols(const double* M, int n, const double* x, double* y) {
  if (n <= 0 || (n & 3) > 1) return -1;
  const int n4 = n & ~3;
  for (int t = 0; t < n; ++t) {
    double out = 0.0;
    if (t >= n4) {
      for (int s = 0; s < n; ++s) out = fma(M[(size_t)s * n + t], x[s], out);
    } else {
      for (int s = 0; s < n4; s += 4) {
        double c = M[(size_t)(s + 1) * n + t] * x[s + 1];
        c = fma(M[(size_t)s * n + t], x[s], c);
        c = fma(M[(size_t)(s + 2) * n + t], x[s + 2], c);
        c = fma(M[(size_t)(s + 3) * n + t], x[s + 3], c);
        out = out + c;
      }
      for (int s = n4; s < n; ++s) out = out + M[(size_t)s * n + t] * x[s];
    }
    y[t] = out;
  }
  return 0;
}

/*
 * expected_svf_from_policy (maxent.py:63-114) in that order: P' = P with the
 * terminal rows zeroed (98-99); per sweep x_a = pi[:, a] * d (rounded),
 * y_a = P'_a^T . x_a (blas_order_dgemv_cols), d_ = p0 + (((y_0 + y_1) + y_2) + ...)
 * (np.array(d_).sum(axis=0), then + p_initial), delta = max|d_ - d| (NaN wins),
 * until delta <= eps (or max_iter sweeps when > 0).  Returns the sweep count.
 */
long long blas_order_forward_svf(const double* P, int S, int A, const double* p0, const uint8_t* term,
                                 const double* pi, double eps, long long max_iter, double* d) {
  if (S <= 0 || A <= 0 || (S & 3) > 1) return -1;
  double* pa = malloc((size_t)A * S * S * sizeof(double));
  double* x = malloc((size_t)S * sizeof(double));
  double* y = malloc((size_t)A * S * sizeof(double));
  double* dn = malloc((size_t)S * sizeof(double));
  if (!pa || !x || !y || !dn) {
    free(pa); free(x); free(y); free(dn);
    return -2;
  }
  for (int a = 0; a < A; ++a)  /* maxent.py:98-102: the terminal rows cleared, then the slices */
    for (int s = 0; s < S; ++s)
      for (int t = 0; t < S; ++t) pa[((size_t)a * S + s) * S + t] = term[s] ? 0.0 : P[((size_t)s * S + t) * A + a];
  for (int s = 0; s < S; ++s) d[s] = 0.0;
  long long it = 0;
  double delta = INFINITY;
  while (delta > eps && (max_iter <= 0 || it < max_iter)) {
    for (int a = 0; a < A; ++a) {
      for (int s = 0; s < S; ++s) x[s] = pi[(size_t)s * A + a] * d[s];
      blas_order_dgemv_cols(pa + (size_t)a * S * S, S, x, y + (size_t)a * S);
    }
    delta = 0.0;
    for (int t = 0; t < S; ++t) {
      double v = y[t];
      for (int a = 1; a < A; ++a) v = v + y[(size_t)a * S + t];
      dn[t] = p0[t] + v;
      const double dd = fabs(dn[t] - d[t]);
      if (dd != dd || (delta == delta && dd > delta)) delta = dd;
    }
    for (int t = 0; t < S; ++t) d[t] = dn[t];
    ++it;
  }
  free(pa); free(x); free(y); free(dn);
  return it;
}

/*
 * The same dgemv_t order over a sparse matrix (CSR, ascending columns per row):
 * numpy's dense dot products with the zero entries skipped.  A skipped entry
 * contributes fma(0, x, acc) = acc (or acc + 0 * x = acc) exactly while x is
 * finite -- the lane accumulators start at +0 and never become -0 -- so the
 * result equals blas_order_dgemv_rows on the dense matrix bit for bit
 * (tests/test_oracle_blas_order.py pins it), at O(nnz) instead of O(S^2): the
 * restatement then reaches 64x64 grids (S = 4096, the two NBMAX blocks).
 */
int blas_order_dgemv_rows_csr(const int64_t* indptr, const int32_t* indices, const double* data, int n,
                              const double* x, double* y) {
  if (n <= 0 || (n & 3) > 1) return -1;
  const int m1 = n - (n & 3), n4 = n & ~3;
  for (int s = 0; s < n; ++s) {
    const int fused = s < n4;
    int64_t e = indptr[s];
    const int64_t e1 = indptr[s + 1];
    double out = 0.0;
    for (int lo = 0; lo < m1; lo += NBMAX) {
      const int hi = lo + NBMAX < m1 ? lo + NBMAX : m1;
      double l[4] = {0.0, 0.0, 0.0, 0.0};
      for (; e < e1 && indices[e] < hi; ++e) {
        const int t = indices[e];
        const int q = (t - lo) & 3;
        l[q] = fused ? fma(data[e], x[t], l[q]) : l[q] + data[e] * x[t];
      }
      out = out + ((l[0] + l[2]) + (l[1] + l[3]));
    }
    for (; e < e1; ++e) out = fma(data[e], x[indices[e]], out);
    y[s] = out;
  }
  return 0;
}

/*
 * local_action_probabilities (maxent.py:119-159) in numpy's order on per-action
 * CSR matrices P_a[s, t] (the slices p[a] of maxent.py:143), stacked as one CSR
 * of A * S rows: the statements of blas_order_backward_maxent with
 * blas_order_dgemv_rows_csr for the dot products.
 */
int blas_order_backward_maxent_csr(const int64_t* indptr, const int32_t* indices, const double* data, int S, int A,
                                   const uint8_t* term, const double* er, double* pi) {
  if (S <= 0 || A <= 0 || (S & 3) > 1) return -1;
  double* zs = malloc((size_t)S * sizeof(double));
  double* dot = malloc((size_t)S * sizeof(double));
  double* za = malloc((size_t)S * A * sizeof(double));
  if (!zs || !dot || !za) {
    free(zs); free(dot); free(za);
    return -2;
  }
  for (int s = 0; s < S; ++s) zs[s] = term[s] ? 1.0 : 0.0;
  for (int it = 0; it < 2 * S; ++it) {
    for (int a = 0; a < A; ++a) {
      blas_order_dgemv_rows_csr(indptr + (size_t)a * S, indices, data, S, zs, dot);
      for (int s = 0; s < S; ++s) za[(size_t)s * A + a] = er[s] * dot[s];
    }
    for (int s = 0; s < S; ++s) {
      double z = za[(size_t)s * A];
      for (int a = 1; a < A; ++a) z = z + za[(size_t)s * A + a];
      zs[s] = z;
    }
  }
  for (int s = 0; s < S; ++s)
    for (int a = 0; a < A; ++a) pi[(size_t)s * A + a] = za[(size_t)s * A + a] / zs[s];
  free(zs); free(dot); free(za);
  return 0;
}

/*
 * TEST INFRASTRUCTURE (oracle).  np.exp / np.log for float64 as numpy 2.2.6
 * computes them on an AVX512_SKX host: the contiguous loops
 * DOUBLE_exp_AVX512_SKX / DOUBLE_log_AVX512_SKX call SVML's __svml_exp8_ha /
 * __svml_log8_ha (numpy's vendored SVML, no source in this image).  Restated
 * from their instruction sequence (constants as stored in numpy's rodata),
 * one scalar lane at a time, with the two non-portable steps replaced by exact
 * equivalents:
 *   exp: the {rz-sae} fma x / ln2 + shifter -- round to nearest, then step
 *        down one grid point (1/16) when the exact residual is negative;
 *   log: vrcp14pd + vrndscalepd(0x58) of the mantissa -- rcp14 reads the top
 *        16 mantissa bits u only, and the rounded result R = (32 - n) / 32
 *        with n = #{t : u >= t} over 16 thresholds found by evaluating the
 *        instruction for all 65,536 u (tools/gen_npmath.py).
 * Inputs SVML sends to its scalar rare path (exp: |x| >= 707.70, NaN; log:
 * x <= 0, inf, NaN) use libm here.  The device twins are np_exp / np_log in
 * irl-maxent_amd/csrc/common.h; both are pinned against np.exp / np.log
 * (tests/golden/npmath.npz, tests/test_npmath.py, tests/test_gpu_npmath.py).
 */
static const double kExpT0[16] = {
    0x1.0000000000000p+0, 0x1.0b5586cf9890fp+0, 0x1.172b83c7d517bp+0, 0x1.2387a6e756238p+0,
    0x1.306fe0a31b715p+0, 0x1.3dea64c123422p+0, 0x1.4bfdad5362a27p+0, 0x1.5ab07dd485429p+0,
    0x1.6a09e667f3bcdp+0, 0x1.7a11473eb0187p+0, 0x1.8ace5422aa0dbp+0, 0x1.9c49182a3f090p+0,
    0x1.ae89f995ad3adp+0, 0x1.c199bdd85529cp+0, 0x1.d5818dcfba487p+0, 0x1.ea4afa2a490dap+0};
static const double kExpT1[16] = {
    0x0.0p+0, 0x1.79aa65d837b6dp-54, -0x1.01b15eaa59348p-55, 0x1.68efde3a8a894p-54,
    0x1.34d754db0abb6p-55, 0x1.59f48a72a4c6dp-55, 0x1.690cebb7aafb0p-56, 0x1.063e1e21c5409p-54,
    -0x1.3b3efbf5e2228p-54, -0x1.b32dcb94da51dp-56, 0x1.db72fc1f0eab4p-55, 0x1.1affc2b91ce27p-56,
    0x1.c1a7792cb3387p-55, 0x1.36eae30af0cb3p-56, 0x1.4a385a63d07a7p-56, -0x1.ff7128fd391f0p-55};
static const double kLogTH[16] = {
    0x0.0p+0, -0x1.f0a30c0120000p-5, -0x1.e27076e2b0000p-4, -0x1.5ff3070a78000p-3,
    -0x1.c8ff7c79a8000p-3, -0x1.1675cababc000p-2, -0x1.4618bc21c4000p-2, -0x1.739d7f6bbc000p-2,
    0x1.269621134c000p-2, 0x1.f991c6cb38000p-3, 0x1.a93ed3c8b0000p-3, 0x1.5bf406b540000p-3,
    0x1.1178e82280000p-3, 0x1.9335e5d590000p-4, 0x1.08598b59e0000p-4, 0x1.0415d89e80000p-5};
static const double kLogTL[16] = {
    0x0.0p+0, 0x1.3ab33d066d1d2p-42, 0x1.a342c2af0003cp-45, -0x1.3d3c873e20a07p-43,
    -0x1.a21ac25d81ef3p-43, 0x1.9f1fc63382a8fp-42, -0x1.ec27d0b7b37b3p-42, -0x1.0069ce24c53fbp-42,
    0x1.b92783beb7677p-42, 0x1.9bcbecca0cdf3p-42, -0x1.30e486a0ac42dp-42, 0x1.ed8fdc149767ep-42,
    -0x1.b8421cc74be04p-43, 0x1.2622b8757a8fbp-42, 0x1.d034451fecdfbp-43, -0x1.77771fd187145p-42};
static const unsigned kRcpSteps[16] = {1039u, 3223u, 5556u, 8048u, 10726u, 13603u, 16707u, 20063u,
                                       23705u, 27669u, 32007u, 36764u, 42010u, 47824u, 54300u, 61568u};

static double np_exp1(double x) {
  if (!(fabs(x) < 0x1.61da04cbafe44p+9)) {
    if (x <= -746.0) return 0.0;
    if (x >= 710.0) return INFINITY;
    return exp(x);
  }
  const double shift = 0x1.8000000003ff0p+48, inv_ln2 = 0x1.71547652b82fep+0;
  double xs = fma(x, inv_ln2, shift);
  if (fma(x, inv_ln2, shift - xs) < 0.0) xs -= 0x1p-4;
  const double n = xs - shift;
  uint64_t bits;
  memcpy(&bits, &xs, 8);
  const int j = (int)(bits & 15);
  double r = fma(-n, 0x1.62e42fefa39efp-1, x);
  r = fma(-0x1.abc9e3b39803fp-56, n, r);
  const double r2 = r * r;
  const double a = fma(r, 0x1.7411836940c04p-10, 0x1.1101cbbc265c0p-7);
  const double b = fma(r, 0x1.55557242d68fep-5, 0x1.5555553939732p-3);
  const double c = fma(r, 0x1.000000000d008p-1, 0x1.fffffffffff70p-1);
  double p = fma(r2, a, b);
  p = fma(r2, p, c);
  double q = fma(p, r, kExpT1[j]);
  q = fma(kExpT0[j], q, kExpT0[j]);
  return ldexp(q, (int)floor(n));
}

static double np_log1(double x) {
  if (!(x > 0.0) || isinf(x)) return log(x);
  int e;
  const double m = ldexp(frexp(x, &e), 1);
  double E = (double)(e - 1);
  uint64_t bits;
  memcpy(&bits, &m, 8);
  const unsigned u = (unsigned)(bits >> 36) & 0xffffu;
  int nd = 0;
  for (int i = 0; i < 16; ++i) nd += u >= kRcpSteps[i];
  const double R = (double)(32 - nd) * 0x1p-5;
  const double r = fma(R, m, -1.0);
  if (nd > 8) E += 1.0;
  const int idx = (16 - nd) & 15;
  const double p1 = fma(r, 0x1.249229cee81efp-3, -0x1.55553fb28db06p-3);
  double p2 = fma(r, 0x1.c81cd309d7c70p-4, -0x1.007357e93af62p-3);
  const double r2 = r * r;
  double p3 = fma(r, 0x1.9999999cc9f5cp-3, -0x1.00000000c05bdp-2);
  p2 = fma(r2, p2, p1);
  const double r4 = r2 * r2;
  const double p4 = fma(r, 0x1.5555555555466p-2, -0x1.fffffffffffc6p-2);
  p3 = fma(r2, p3, p4);
  const double hi = fma(E, 0x1.62e42fefa0000p-1, kLogTH[idx]);
  p2 = fma(r4, p2, p3);
  const double s = hi + r;
  const double rl = r - (s - hi);
  p2 = fma(r2, p2, rl);
  const double lo = fma(0x1.cf79abc9e0000p-40, E, kLogTL[idx]);
  return s + (p2 + lo);
}

void numpy_exp_restated(const double* x, double* y, long long n) {
  for (long long i = 0; i < n; ++i) y[i] = np_exp1(x[i]);
}
void numpy_log_restated(const double* x, double* y, long long n) {
  for (long long i = 0; i < n; ++i) y[i] = np_log1(x[i]);
}
