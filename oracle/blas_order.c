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
