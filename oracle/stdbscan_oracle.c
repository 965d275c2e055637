/*
 * TEST INFRASTRUCTURE ONLY — the parity oracle.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this; the product (librpt.so) never does.
 *
 * CPU restatement of the reference ST-DBSCAN, following the sequential BFS of
 *   PointCloudWork/3_stdbscan_point_clouds.py:101-136  (and the identical loop in
 *   radar_pipeline/processors/clustering.py:80-115, 4_temporal_object_tracker.py:469-506):
 *   - visit points in index order; a point with fewer than min_samples space-time neighbours
 *     (itself included) stays -1 (:118-121);
 *   - otherwise it opens cluster `cid` and a seed set of its neighbours is drained; a popped
 *     unvisited point is visited and, if it is core, its neighbours join the seeds (:125-131);
 *     every popped point still labelled -1 receives cid (:132-133).
 *   Neighbour predicate, as sklearn BallTree.query_radius (float64 copy of the input, rdist
 *   = sum of squared differences, left to right) and the reference's float32 time filter:
 *     d2 = (xi-xj)^2 + (yi-yj)^2 [+ (zi-zj)^2] <= eps^2   (float64, no FMA)
 *     |float32(t_j - t_i)| <= float32(eps_t)               (NEP 50: Python float -> float32)
 * Neighbour search: points sorted by time; each query scans the time window (with generous
 * slack) and applies the exact predicate, so the oracle is exact and O(n * window).
 * Build: gcc -O2 -ffp-contract=off -shared -fPIC (oracle/Makefile, __graft_entry__.build()).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  const float* c;
  int dim;
  const float* t;
  double eps2;
  float epst;
  int64_t n;
  int64_t* order; /* indices sorted by time (non-finite last) */
  float* tsorted;
  int64_t n_finite;
} ctx_t;

static const float* g_t_for_sort;

static int cmp_time(const void* a, const void* b) {
  int64_t i = *(const int64_t*)a, j = *(const int64_t*)b;
  float ti = g_t_for_sort[i], tj = g_t_for_sort[j];
  int fi = isfinite(ti), fj = isfinite(tj);
  if (fi != fj) return fi ? -1 : 1;
  if (fi) {
    if (ti < tj) return -1;
    if (ti > tj) return 1;
  }
  return (i < j) ? -1 : (i > j);
}

static int adjacent(const ctx_t* x, int64_t i, int64_t j) {
  const float* a = x->c + i * x->dim;
  const float* b = x->c + j * x->dim;
  double d2 = 0.0;
  for (int k = 0; k < x->dim; ++k) {
    double d = (double)a[k] - (double)b[k];
    double sq = d * d;
    d2 = d2 + sq;
  }
  float dt = x->t[j] - x->t[i];
  dt = fabsf(dt);
  return (d2 <= x->eps2) && (dt <= x->epst);
}

/* writes neighbours of i into buf (capacity n); returns count */
static int64_t neighbours(const ctx_t* x, int64_t i, int64_t* buf) {
  float ti = x->t[i];
  if (!isfinite(ti) || !(x->epst >= 0.0f) || !(x->eps2 >= 0.0)) return 0;
  double slack = 1e-3 * (fabs((double)x->epst) + fabs((double)ti)) + 1e-6;
  double lo = (double)ti - (double)x->epst - slack;
  double hi = (double)ti + (double)x->epst + slack;
  /* lower_bound on tsorted[0..n_finite) */
  int64_t a = 0, b = x->n_finite;
  while (a < b) {
    int64_t m = (a + b) / 2;
    if ((double)x->tsorted[m] < lo) a = m + 1; else b = m;
  }
  int64_t cnt = 0;
  for (int64_t k = a; k < x->n_finite && (double)x->tsorted[k] <= hi; ++k) {
    int64_t j = x->order[k];
    if (adjacent(x, i, j)) buf[cnt++] = j;
  }
  return cnt;
}

/* labels: int32[n] out.  coords: float32 [n][dim] row-major.  Returns #clusters or -1. */
int32_t oracle_stdbscan(const float* coords, int32_t dim, const float* times, int64_t n,
                        double eps_space, double eps_time, int32_t min_samples,
                        int32_t* labels) {
  ctx_t x;
  x.c = coords;
  x.dim = dim;
  x.t = times;
  x.eps2 = eps_space * eps_space;
  if (!(eps_space >= 0.0)) x.eps2 = -1.0;
  x.epst = (float)eps_time;
  x.n = n;
  x.order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  x.tsorted = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
  int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t* nb2 = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t* stack = (int64_t*)malloc(sizeof(int64_t) * (size_t)(2 * n + 1));
  uint8_t* visited = (uint8_t*)calloc((size_t)(n > 0 ? n : 1), 1);
  uint8_t* inseed = (uint8_t*)calloc((size_t)(n > 0 ? n : 1), 1);
  if (!x.order || !x.tsorted || !nb || !nb2 || !stack || !visited || !inseed) return -1;
  for (int64_t i = 0; i < n; ++i) x.order[i] = i;
  g_t_for_sort = times;
  qsort(x.order, (size_t)n, sizeof(int64_t), cmp_time);
  x.n_finite = 0;
  for (int64_t k = 0; k < n; ++k) {
    x.tsorted[k] = times[x.order[k]];
    if (isfinite(x.tsorted[k])) x.n_finite = k + 1;
  }
  for (int64_t i = 0; i < n; ++i) labels[i] = -1;
  int32_t cid = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (visited[i]) continue;
    visited[i] = 1;
    int64_t cnt = neighbours(&x, i, nb);
    if (cnt < (int64_t)min_samples) continue; /* labels[i] stays -1 */
    labels[i] = cid;
    int64_t sp = 0;
    for (int64_t k = 0; k < cnt; ++k)
      if (!inseed[nb[k]]) { inseed[nb[k]] = 1; stack[sp++] = nb[k]; }
    while (sp > 0) {
      int64_t pt = stack[--sp];
      inseed[pt] = 0;
      if (!visited[pt]) {
        visited[pt] = 1;
        int64_t c2 = neighbours(&x, pt, nb2);
        if (c2 >= (int64_t)min_samples)
          for (int64_t k = 0; k < c2; ++k)
            if (!inseed[nb2[k]]) { inseed[nb2[k]] = 1; stack[sp++] = nb2[k]; }
      }
      if (labels[pt] == -1) labels[pt] = cid;
    }
    ++cid;
  }
  free(x.order); free(x.tsorted); free(nb); free(nb2); free(stack); free(visited); free(inseed);
  return cid;
}

/* neighbour counts (incl. self) per point — used to pin core flags */
int32_t oracle_neighbour_counts(const float* coords, int32_t dim, const float* times, int64_t n,
                                double eps_space, double eps_time, int64_t* counts) {
  ctx_t x;
  x.c = coords; x.dim = dim; x.t = times; x.n = n;
  x.eps2 = (eps_space >= 0.0) ? eps_space * eps_space : -1.0;
  x.epst = (float)eps_time;
  x.order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  x.tsorted = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
  int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  if (!x.order || !x.tsorted || !nb) return -1;
  for (int64_t i = 0; i < n; ++i) x.order[i] = i;
  g_t_for_sort = times;
  qsort(x.order, (size_t)n, sizeof(int64_t), cmp_time);
  x.n_finite = 0;
  for (int64_t k = 0; k < n; ++k) {
    x.tsorted[k] = times[x.order[k]];
    if (isfinite(x.tsorted[k])) x.n_finite = k + 1;
  }
  for (int64_t i = 0; i < n; ++i) counts[i] = neighbours(&x, i, nb);
  free(x.order); free(x.tsorted); free(nb);
  return 0;
}
