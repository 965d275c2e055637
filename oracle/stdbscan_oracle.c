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
 * Neighbour search (candidates only; the exact predicate above decides): when every finite
 * time is an integer (frame ids) a sorted (slab, cell) key grid with cell side >= eps is probed
 * over +-1 cells and floor(eps_t)+1 slabs; otherwise points are sorted by time and the time
 * window (with generous slack) is scanned.
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
  /* grid mode (all finite times integral): key = ((slab*nz + cz)*ny + cy)*nx + cx */
  int grid;
  double lo[3], cs;
  int64_t nd[3];
  double tmin;
  int64_t smax;
  int64_t* gkey;   /* sorted keys */
  int64_t* gidx;   /* point index per sorted key */
  float* gc;       /* coords of the sorted points, component-major: gc[d * n_grid + k] */
  float* gt;       /* times of the sorted points */
  int64_t n_grid;
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

static int64_t cell1(double v, double lo, double cs, int64_t n) {
  double q = floor((v - lo) / cs);
  if (q < 0) return 0;
  if (q >= (double)n) return n - 1;
  return (int64_t)q;
}

static int64_t key_of(const ctx_t* x, int64_t slab, const int64_t* c) {
  int64_t k = slab;
  for (int d = x->dim - 1; d >= 0; --d) k = k * x->nd[d] + c[d];
  return k;
}

static int cmp_pair(const void* a, const void* b) {
  const int64_t* p = (const int64_t*)a;
  const int64_t* q = (const int64_t*)b;
  if (p[0] != q[0]) return p[0] < q[0] ? -1 : 1;
  return (p[1] < q[1]) ? -1 : (p[1] > q[1]);
}

/* grid mode: used when every finite time is an integer below 2^24 (frame ids) and eps >= 0 */
static void build_grid(ctx_t* x) {
  x->grid = 0;
  if (!(x->epst >= 0.0f) || !(x->eps2 >= 0.0) || x->dim > 3) return;
  double tmin = INFINITY, tmax = -INFINITY;
  for (int d = 0; d < x->dim; ++d) { x->lo[d] = INFINITY; }
  double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = 0; i < x->n; ++i) {
    float t = x->t[i];
    if (!isfinite(t)) continue;
    if (t != floorf(t) || fabsf(t) >= 16777216.f) return;
    if (t < tmin) tmin = t;
    if (t > tmax) tmax = t;
    for (int d = 0; d < x->dim; ++d) {
      double v = x->c[i * x->dim + d];
      if (v < x->lo[d]) x->lo[d] = v;
      if (v > hi[d]) hi[d] = v;
    }
  }
  if (!(tmin <= tmax)) return;
  double eps = sqrt(x->eps2);
  x->cs = (eps > 0 ? eps : 1.0) * (1.0 + 1.0 / 1048576.0);
  double cells = 1.0;
  for (int d = 0; d < x->dim; ++d) {
    if (!isfinite(x->lo[d]) || !isfinite(hi[d])) return;
    /* keep the composite key in range; coarser cells stay exact (neighbours within +-1) */
    double nd = floor((hi[d] - x->lo[d]) / x->cs) + 1.0;
    while (nd > 4.0e5) { x->cs *= 2.0; nd = floor((hi[d] - x->lo[d]) / x->cs) + 1.0; }
    x->nd[d] = (int64_t)nd;
    cells *= nd;
  }
  if (cells * (tmax - tmin + 1.0) > 9.0e18) return;
  x->tmin = tmin;
  x->smax = (int64_t)(tmax - tmin);
  int64_t* pairs = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)(x->n > 0 ? x->n : 1));
  x->gkey = (int64_t*)malloc(sizeof(int64_t) * (size_t)(x->n > 0 ? x->n : 1));
  x->gidx = (int64_t*)malloc(sizeof(int64_t) * (size_t)(x->n > 0 ? x->n : 1));
  int64_t m = 0;
  for (int64_t i = 0; i < x->n; ++i) {
    float t = x->t[i];
    if (!isfinite(t)) continue;
    int64_t c[3];
    for (int d = 0; d < x->dim; ++d) c[d] = cell1(x->c[i * x->dim + d], x->lo[d], x->cs, x->nd[d]);
    pairs[2 * m] = key_of(x, (int64_t)((double)t - tmin), c);
    pairs[2 * m + 1] = i;
    ++m;
  }
  /* (key, index) order: a stable counting sort when the key range is small (same order as
   * the comparison sort, linear time on stacks of tens of millions of points) */
  const double nkeys = cells * (double)(x->smax + 1);
  if (nkeys <= 4.0 * (double)m + 16777216.0) {
    const int64_t K = (int64_t)nkeys;
    int64_t* cnt = (int64_t*)calloc((size_t)K + 1, sizeof(int64_t));
    int64_t* tmp = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)(m > 0 ? m : 1));
    for (int64_t k = 0; k < m; ++k) ++cnt[pairs[2 * k] + 1];
    for (int64_t k = 0; k < K; ++k) cnt[k + 1] += cnt[k];
    for (int64_t k = 0; k < m; ++k) {
      const int64_t d = cnt[pairs[2 * k]]++;
      tmp[2 * d] = pairs[2 * k];
      tmp[2 * d + 1] = pairs[2 * k + 1];
    }
    free(cnt);
    free(pairs);
    pairs = tmp;
  } else {
    qsort(pairs, (size_t)m, 2 * sizeof(int64_t), cmp_pair);
  }
  x->gc = (float*)malloc(sizeof(float) * (size_t)(m > 0 ? m : 1) * (size_t)x->dim);
  x->gt = (float*)malloc(sizeof(float) * (size_t)(m > 0 ? m : 1));
  for (int64_t k = 0; k < m; ++k) {
    const int64_t i = pairs[2 * k + 1];
    x->gkey[k] = pairs[2 * k];
    x->gidx[k] = i;
    for (int d = 0; d < x->dim; ++d) x->gc[(int64_t)d * m + k] = x->c[i * x->dim + d];
    x->gt[k] = x->t[i];
  }
  free(pairs);
  x->n_grid = m;
  x->grid = 1;
}

static int64_t lower_key(const ctx_t* x, int64_t key) {
  int64_t a = 0, b = x->n_grid;
  while (a < b) {
    int64_t m = (a + b) / 2;
    if (x->gkey[m] < key) a = m + 1; else b = m;
  }
  return a;
}

/* candidates [p0, p1) of the sorted arrays: the predicate of adjacent(), evaluated in the same
 * order of operations on contiguous copies (the compiler vectorises the arithmetic) */
static int64_t scan_range(const ctx_t* x, int64_t i, int64_t p0, int64_t p1, int64_t* out) {
  const int64_t m = x->n_grid;
  const double eps2 = x->eps2;
  const float epst = x->epst;
  const float ti = x->t[i];
  const double ax = x->c[i * x->dim];
  const double ay = x->dim >= 2 ? (double)x->c[i * x->dim + 1] : 0.0;
  const float* gx = x->gc;
  const float* gy = x->gc + m;
  const float* gt = x->gt;
  int64_t cnt = 0;
  if (x->dim == 2) {
    for (int64_t p = p0; p < p1; ++p) {
      const double dx = ax - (double)gx[p];
      const double dy = ay - (double)gy[p];
      const double d2 = dx * dx + dy * dy;
      const float dt = fabsf(gt[p] - ti);
      out[cnt] = x->gidx[p];
      cnt += (d2 <= eps2) & (dt <= epst);
    }
    return cnt;
  }
  const double az = x->dim == 3 ? (double)x->c[i * x->dim + 2] : 0.0;
  const float* gz = x->gc + 2 * m;
  for (int64_t p = p0; p < p1; ++p) {
    double d2 = 0.0;
    if (x->dim >= 1) { const double d = ax - (double)gx[p]; d2 = d2 + d * d; }
    if (x->dim >= 2) { const double d = ay - (double)gy[p]; d2 = d2 + d * d; }
    if (x->dim >= 3) { const double d = az - (double)gz[p]; d2 = d2 + d * d; }
    const float dt = fabsf(gt[p] - ti);
    out[cnt] = x->gidx[p];
    cnt += (d2 <= eps2) & (dt <= epst);
  }
  return cnt;
}

/* window of point i in grid mode: its slab +- floor(eps_t)+1 (clipped), cells +-1 per
 * dimension; the candidates are the sorted positions [r[2k], r[2k+1]) for k < return value.
 * r needs room for 2 * max_ranges(x) entries. */
static int64_t max_ranges(const ctx_t* x) {
  double dsd = floor((double)x->epst) + 1.0;
  int64_t ds = dsd > (double)(x->smax + 1) ? x->smax + 1 : (int64_t)dsd;
  return (2 * ds + 1) * (x->dim == 3 ? 9 : 3);
}

static int64_t grid_ranges(const ctx_t* x, int64_t i, int64_t* r) {
  float ti = x->t[i];
  int64_t slab = (int64_t)((double)ti - x->tmin);
  double dsd = floor((double)x->epst) + 1.0;
  int64_t ds = dsd > (double)(x->smax + 1) ? x->smax + 1 : (int64_t)dsd;
  int64_t c0[3] = {0, 0, 0}, lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
  for (int d = 0; d < x->dim; ++d) {
    c0[d] = cell1(x->c[i * x->dim + d], x->lo[d], x->cs, x->nd[d]);
    lo[d] = c0[d] > 0 ? c0[d] - 1 : 0;
    hi[d] = c0[d] + 1 < x->nd[d] ? c0[d] + 1 : x->nd[d] - 1;
  }
  int64_t k = 0;
  for (int64_t s = slab - ds; s <= slab + ds; ++s) {
    if (s < 0 || s > x->smax) continue;
    int64_t c[3];
    for (c[2] = (x->dim == 3 ? lo[2] : 0); c[2] <= (x->dim == 3 ? hi[2] : 0); ++c[2])
      for (c[1] = lo[1]; c[1] <= hi[1]; ++c[1]) {
        c[0] = lo[0];
        const int64_t k0 = key_of(x, s, c);
        c[0] = hi[0];
        const int64_t k1 = key_of(x, s, c);
        r[2 * k] = lower_key(x, k0);
        r[2 * k + 1] = lower_key(x, k1 + 1);
        ++k;
      }
  }
  return k;
}

static int64_t neighbours_grid(const ctx_t* x, int64_t i, int64_t* buf) {
  int64_t rr[2 * 7 * 9];
  int64_t* r = max_ranges(x) <= 7 * 9 ? rr : (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)max_ranges(x));
  const int64_t nr = grid_ranges(x, i, r);
  int64_t cnt = 0;
  for (int64_t k = 0; k < nr; ++k) cnt += scan_range(x, i, r[2 * k], r[2 * k + 1], buf + cnt);
  if (r != rr) free(r);
  return cnt;
}

/* writes neighbours of i into buf (capacity n); returns count */
static int64_t neighbours(const ctx_t* x, int64_t i, int64_t* buf) {
  float ti = x->t[i];
  if (!isfinite(ti) || !(x->epst >= 0.0f) || !(x->eps2 >= 0.0)) return 0;
  if (x->grid) return neighbours_grid(x, i, buf);
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
  x.gkey = x.gidx = NULL;
  x.gc = x.gt = NULL;
  build_grid(&x);
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
  free(x.gkey); free(x.gidx); free(x.gc); free(x.gt);
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
  x.gkey = x.gidx = NULL;
  x.gc = x.gt = NULL;
  build_grid(&x);
  for (int64_t i = 0; i < n; ++i) counts[i] = neighbours(&x, i, nb);
  free(x.order); free(x.tsorted); free(nb); free(x.gkey); free(x.gidx); free(x.gc);
  free(x.gt);
  return 0;
}

/* For sample points idx[0..m): the exact neighbour count (self included) and, given a claimed
 * labelling (core flags + labels of ALL points, e.g. a device run's), the smallest and largest
 * label among the core neighbours (-1 / -1 when none).  A full-size invariant check: core flags
 * of the sample must equal count >= min_samples, a core sample's core neighbours all share its
 * label, a non-core sample takes the smallest adjacent label.  OpenMP. */
static int pair_ok(const ctx_t* x, int64_t i, int64_t p);

int32_t oracle_sample_check(const float* coords, int32_t dim, const float* times, int64_t n,
                            double eps_space, double eps_time, const int64_t* idx, int64_t m,
                            const uint8_t* core, const int32_t* labels, int64_t* count_out,
                            int32_t* lo_out, int32_t* hi_out) {
  ctx_t x;
  memset(&x, 0, sizeof(x));
  x.c = coords;
  x.dim = dim;
  x.t = times;
  x.eps2 = (eps_space >= 0.0) ? eps_space * eps_space : -1.0;
  x.epst = (float)eps_time;
  x.n = n;
  build_grid(&x);
  if (!x.grid) {
    free(x.gkey); free(x.gidx); free(x.gc); free(x.gt);
    return -1;
  }
  const int64_t mr = max_ranges(&x);
#pragma omp parallel
  {
    int64_t* r = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)mr);
#pragma omp for schedule(dynamic, 16)
    for (int64_t k = 0; k < m; ++k) {
      const int64_t i = idx[k];
      int64_t cnt = 0;
      int32_t lo = -1, hi = -1;
      if (isfinite(x.t[i])) {
        const int64_t nr = grid_ranges(&x, i, r);
        for (int64_t q = 0; q < nr; ++q)
          for (int64_t p = r[2 * q]; p < r[2 * q + 1]; ++p) {
            if (!pair_ok(&x, i, p)) continue;
            ++cnt;
            const int64_t j = x.gidx[p];
            if (core[j]) {
              const int32_t l = labels[j];
              if (lo < 0 || l < lo) lo = l;
              if (hi < 0 || l > hi) hi = l;
            }
          }
      }
      count_out[k] = cnt;
      lo_out[k] = lo;
      hi_out[k] = hi;
    }
    free(r);
  }
  free(x.gkey); free(x.gidx); free(x.gc); free(x.gt);
  return 0;
}

/* ---------------------------------------------------------------------------------------
 * oracle_stdbscan_uf — the same labels as oracle_stdbscan, by the set formulation the BFS
 * computes (checked against the BFS in tests/test_oracle_golden.py):
 *   core_i   = |{ j : adjacent(i, j) }| >= min_samples       (the BFS count, self included)
 *   clusters = connected components of the core-core adjacency, numbered in ascending order of
 *              their minimum index (the BFS opens cluster ids in index order);
 *   border   = a non-core point adjacent to a core point takes the smallest adjacent cluster id
 *              (the first cluster whose BFS reaches it); every other point is -1.
 * OpenMP over points (lock-free union-find hooking the larger root under the smaller, so every
 * root is its component's minimum index whatever the order).  Grid mode only (integral finite
 * times); other inputs fall back to the BFS.  Used as the checker for stacks whose summed
 * neighbourhood sizes (10^10 pairs at the bench's 100 frames) make the sequential BFS too slow.
 */
static int64_t uf_find(int64_t* par, int64_t i) {
  for (;;) {
    const int64_t p = __atomic_load_n(&par[i], __ATOMIC_RELAXED);
    if (p == i) return i;
    const int64_t gp = __atomic_load_n(&par[p], __ATOMIC_RELAXED);
    if (gp != p) __atomic_compare_exchange_n(&par[i], (int64_t*)&p, gp, 0, __ATOMIC_RELAXED,
                                             __ATOMIC_RELAXED);
    i = p;
  }
}

static void uf_unite(int64_t* par, int64_t a, int64_t b) {
  for (;;) {
    a = uf_find(par, a);
    b = uf_find(par, b);
    if (a == b) return;
    if (a > b) { const int64_t t = a; a = b; b = t; }
    int64_t expect = b;
    if (__atomic_compare_exchange_n(&par[b], &expect, a, 0, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED))
      return;
  }
}

static int pair_ok(const ctx_t* x, int64_t i, int64_t p) {
  const int64_t m = x->n_grid;
  double d2 = 0.0;
  for (int d = 0; d < x->dim; ++d) {
    const double dd = (double)x->c[i * x->dim + d] - (double)x->gc[(int64_t)d * m + p];
    d2 = d2 + dd * dd;
  }
  const float dt = fabsf(x->gt[p] - x->t[i]);
  return (d2 <= x->eps2) & (dt <= x->epst);
}

int32_t oracle_stdbscan_uf(const float* coords, int32_t dim, const float* times, int64_t n,
                           double eps_space, double eps_time, int32_t min_samples,
                           int32_t* labels) {
  ctx_t x;
  memset(&x, 0, sizeof(x));
  x.c = coords;
  x.dim = dim;
  x.t = times;
  x.eps2 = (eps_space >= 0.0) ? eps_space * eps_space : -1.0;
  x.epst = (float)eps_time;
  x.n = n;
  build_grid(&x);
  if (!x.grid) {
    free(x.gkey); free(x.gidx); free(x.gc); free(x.gt);
    return oracle_stdbscan(coords, dim, times, n, eps_space, eps_time, min_samples, labels);
  }
  uint8_t* core = (uint8_t*)calloc((size_t)(n > 0 ? n : 1), 1);
  int64_t* par = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int32_t* cid = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  if (!core || !par || !cid) return -1;
  const int64_t mr = max_ranges(&x);
  /* 1. core flags: neighbour counts with early exit at min_samples */
#pragma omp parallel
  {
    int64_t* r = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)mr);
#pragma omp for schedule(dynamic, 1024)
    for (int64_t i = 0; i < n; ++i) {
      par[i] = i;
      int64_t cnt = 0;
      if (isfinite(x.t[i]) && cnt < (int64_t)min_samples) {
        const int64_t nr = grid_ranges(&x, i, r);
        for (int64_t k = 0; k < nr && cnt < (int64_t)min_samples; ++k)
          for (int64_t p = r[2 * k]; p < r[2 * k + 1]; ++p) cnt += pair_ok(&x, i, p);
      }
      core[i] = cnt >= (int64_t)min_samples;
    }
    free(r);
  }
  /* 2. components of the core-core adjacency: each pair once, from its lower sorted position
   * (the candidates above q form a contiguous tail of every range) */
  uint8_t* core_s = (uint8_t*)malloc((size_t)(x.n_grid > 0 ? x.n_grid : 1));
  if (!core_s) return -1;
  for (int64_t q = 0; q < x.n_grid; ++q) core_s[q] = core[x.gidx[q]];
#pragma omp parallel
  {
    int64_t* r = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)mr);
#pragma omp for schedule(dynamic, 256)
    for (int64_t q = 0; q < x.n_grid; ++q) {
      if (!core_s[q]) continue;
      const int64_t i = x.gidx[q];
      const int64_t nr = grid_ranges(&x, i, r);
      for (int64_t k = 0; k < nr; ++k)
        for (int64_t p = r[2 * k] > q + 1 ? r[2 * k] : q + 1; p < r[2 * k + 1]; ++p)
          if (core_s[p] && pair_ok(&x, i, p)) {
            const int64_t j = x.gidx[p];
            if (uf_find(par, j) != uf_find(par, i)) uf_unite(par, i, j);
          }
    }
    free(r);
  }
  free(core_s);
  /* 3. ids in ascending order of the component minimum (= the root) */
  int32_t ncl = 0;
  for (int64_t i = 0; i < n; ++i) {
    cid[i] = -1;
    if (core[i] && uf_find(par, i) == i) cid[i] = ncl++;
  }
  /* 4. labels: core -> its component's id; border -> the smallest adjacent id */
#pragma omp parallel
  {
    int64_t* r = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)mr);
#pragma omp for schedule(dynamic, 1024)
    for (int64_t i = 0; i < n; ++i) {
      if (core[i]) {
        labels[i] = cid[uf_find(par, i)];
        continue;
      }
      int32_t best = -1;
      if (isfinite(x.t[i])) {
        const int64_t nr = grid_ranges(&x, i, r);
        for (int64_t k = 0; k < nr; ++k)
          for (int64_t p = r[2 * k]; p < r[2 * k + 1]; ++p) {
            const int64_t j = x.gidx[p];
            if (core[j] && pair_ok(&x, i, p)) {
              const int32_t c = cid[uf_find(par, j)];
              if (best < 0 || c < best) best = c;
            }
          }
      }
      labels[i] = best;
    }
    free(r);
  }
  free(core); free(par); free(cid);
  free(x.gkey); free(x.gidx); free(x.gc); free(x.gt);
  return ncl;
}

/* ---- denoise variant: PointCloudWorkF/stdbscan_denoising_pipeline.py:264-369, restated as the
 * reference's own loop.  Same neighbour predicate as above (BallTree query_radius over float32
 * coords, float32 time filter :317-321).  Differences from oracle_stdbscan:
 *   - core (:308-315): len(neighbours) >= min_samples AND the neighbours' int32(times) frames
 *     (astype truncation, :305) number >= min_frames;
 *   - expansion (:340-367): FIFO queue seeded with ALL neighbours of the seed (visited or not),
 *     a popped unvisited core point appends its neighbours that are neither visited nor already
 *     queued in this cluster (in_queue, reset per cluster, :357-367); every popped point still
 *     labelled -1 takes the cluster id.
 * n == 0 returns 0 clusters (the reference returns an empty array, :286-287). */
static int cmp_i32(const void* a, const void* b) {
  const int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
  return (x > y) - (x < y);
}

static int32_t np_int32(float v) {
  /* numpy float32 -> int32 astype on x86-64: truncation; NaN / out of range -> INT32_MIN */
  if (!(v == v) || v >= 2147483648.0f || v < -2147483648.0f) return INT32_MIN;
  return (int32_t)v;
}

static int denoise_core(const ctx_t* x, const int64_t* nb, int64_t cnt, int32_t min_samples,
                        int32_t min_frames, int32_t* fbuf) {
  if (cnt < (int64_t)min_samples) return 0;
  for (int64_t k = 0; k < cnt; ++k) fbuf[k] = np_int32(x->t[nb[k]]);
  qsort(fbuf, (size_t)cnt, sizeof(int32_t), cmp_i32);
  int64_t uniq = cnt > 0 ? 1 : 0;
  for (int64_t k = 1; k < cnt; ++k) uniq += fbuf[k] != fbuf[k - 1];
  return uniq >= (int64_t)min_frames;
}

int32_t oracle_stdbscan_denoise(const float* coords, int32_t dim, const float* times, int64_t n,
                                double eps_space, double eps_time, int32_t min_samples,
                                int32_t min_frames, int32_t* labels) {
  if (n <= 0) return 0;
  ctx_t x;
  x.c = coords;
  x.dim = dim;
  x.t = times;
  x.eps2 = eps_space * eps_space;
  if (!(eps_space >= 0.0)) x.eps2 = -1.0;
  x.epst = (float)eps_time;
  x.n = n;
  x.order = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  x.tsorted = (float*)malloc(sizeof(float) * (size_t)n);
  int64_t* nb = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  int64_t* nb2 = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  int32_t* fbuf = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
  int64_t* queue = (int64_t*)malloc(sizeof(int64_t) * (size_t)(2 * n + 1));
  uint8_t* visited = (uint8_t*)calloc((size_t)n, 1);
  uint8_t* in_queue = (uint8_t*)calloc((size_t)n, 1);
  if (!x.order || !x.tsorted || !nb || !nb2 || !fbuf || !queue || !visited || !in_queue)
    return -1;
  for (int64_t i = 0; i < n; ++i) x.order[i] = i;
  g_t_for_sort = times;
  qsort(x.order, (size_t)n, sizeof(int64_t), cmp_time);
  x.n_finite = 0;
  for (int64_t k = 0; k < n; ++k) {
    x.tsorted[k] = times[x.order[k]];
    if (isfinite(x.tsorted[k])) x.n_finite = k + 1;
  }
  x.gkey = x.gidx = NULL;
  x.gc = x.gt = NULL;
  build_grid(&x);
  for (int64_t i = 0; i < n; ++i) labels[i] = -1;
  int32_t cid = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (visited[i]) continue;
    visited[i] = 1;
    const int64_t cnt = neighbours(&x, i, nb);
    if (!denoise_core(&x, nb, cnt, min_samples, min_frames, fbuf)) continue;
    labels[i] = cid;
    int64_t head = 0, tail = 0;
    for (int64_t k = 0; k < cnt; ++k) {
      queue[tail++] = nb[k];
      in_queue[nb[k]] = 1;
    }
    while (head < tail) {
      const int64_t pt = queue[head++];
      if (!visited[pt]) {
        visited[pt] = 1;
        const int64_t c2 = neighbours(&x, pt, nb2);
        if (denoise_core(&x, nb2, c2, min_samples, min_frames, fbuf))
          for (int64_t k = 0; k < c2; ++k)
            if (!visited[nb2[k]] && !in_queue[nb2[k]]) {
              queue[tail++] = nb2[k];
              in_queue[nb2[k]] = 1;
            }
      }
      if (labels[pt] == -1) labels[pt] = cid;
    }
    for (int64_t k = 0; k < tail; ++k) in_queue[queue[k]] = 0; /* in_queue[:] = False */
    ++cid;
  }
  free(x.order); free(x.tsorted); free(nb); free(nb2); free(fbuf); free(queue);
  free(visited); free(in_queue);
  free(x.gkey); free(x.gidx); free(x.gc); free(x.gt);
  return cid;
}
