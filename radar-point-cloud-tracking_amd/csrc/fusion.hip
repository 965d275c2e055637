// Max-intensity gain fusion on a regular grid: fuse_gains_max of
// PointCloudWork/5_gain_fusion_ply_builder.py:222-273 over a frame's concatenated per-gain points.
//
//   bins  = int(ceil(float32(max - min) / float32(res))) + 1          per axis (:251-252)
//   cell  = int(float32(v - min) / float32(res))                       truncation (:255-256)
//   grid  = np.maximum.at(zeros float32, cells, intensity)             (:259-260)
//   out   = cells with grid > 0 in np.where(valid.T) order, i.e. y-major then x (:263-264),
//           x = (float64(x_min) + ix * res) + res / 2 in float64, intensity float32 (:266-268)
//
// Intensities reaching this stage passed the loader's threshold (> 5), so they are positive and
// their float bit patterns order like unsigned integers: the max is one atomicMax per point on
// the cell's bits.  One pass over the points, one over the grid (flags in output order), a scan
// and a scatter: HBM-bound, ~12 B per point + ~8 B per cell.
#include <cmath>
#include <cstring>

#include "common.h"

namespace rpt {
int32_t bounds_xy(const float* x, const float* y, int64_t n, float* out4, hipStream_t st);
int32_t exclusive_scan_total_i32(const int32_t* in, int32_t* out, int64_t n, hipStream_t stream);

namespace {
constexpr int kBlock = 256;

__global__ void k_maxpool(const float* __restrict__ x, const float* __restrict__ y,
                          const float* __restrict__ v, int64_t n, float x0, float y0, float res,
                          int32_t ny, unsigned int* __restrict__ grid) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float tx = __fdiv_rn(__fsub_rn(x[i], x0), res);
    const float ty = __fdiv_rn(__fsub_rn(y[i], y0), res);
    const int64_t ix = (int64_t)tx;
    const int64_t iy = (int64_t)ty;
    const float val = v[i];
    if (val > 0.0f) atomicMax(grid + ix * ny + iy, __float_as_uint(val));
  }
}

// flags in output order k = iy * nx + ix (the transposed grid, row-major)
__global__ void k_fuse_flags(const unsigned int* __restrict__ grid, int32_t nx, int32_t ny,
                             int32_t* __restrict__ flag) {
  const int64_t cells = (int64_t)nx * ny;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cells;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t iy = k / nx, ix = k - iy * nx;
    flag[k] = grid[ix * ny + iy] != 0u;
  }
}

__global__ void k_fuse_scatter(const unsigned int* __restrict__ grid, int32_t nx, int32_t ny,
                               const int32_t* __restrict__ pos, double x0, double y0, double res,
                               double* __restrict__ ox, double* __restrict__ oy,
                               float* __restrict__ oi) {
  const int64_t cells = (int64_t)nx * ny;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cells;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t iy = k / nx, ix = k - iy * nx;
    const unsigned int b = grid[ix * ny + iy];
    if (b == 0u) continue;
    const int32_t p = pos[k];
    ox[p] = __dadd_rn(__dadd_rn(x0, __dmul_rn((double)ix, res)), res / 2.0);
    oy[p] = __dadd_rn(__dadd_rn(y0, __dmul_rn((double)iy, res)), res / 2.0);
    oi[p] = __uint_as_float(b);
  }
}
}  // namespace

int32_t fuse_gains_max(const float* x, const float* y, const float* v, int64_t n, double res,
                       double* ox, double* oy, float* oi, int64_t* n_out, hipStream_t st) {
  *n_out = 0;
  if (n <= 0) return RPT_OK;
  if (!(res > 0.0) || !std::isfinite(res)) {
    set_error("rpt_fuse_gains_max: grid_resolution must be positive");
    return RPT_EINVAL;
  }
  float b4[4];
  RPT_TRY(bounds_xy(x, y, n, b4, st));  // synchronises
  if (!std::isfinite(b4[0]) || !std::isfinite(b4[1]) || !std::isfinite(b4[2]) ||
      !std::isfinite(b4[3])) {
    set_error("rpt_fuse_gains_max: non-finite coordinates");
    return RPT_ENONFINITE;
  }
  const float rf = (float)res;  // NEP 50: the Python float joins float32 arithmetic as float32
  const double bx = std::ceil((double)((b4[1] - b4[0]) / rf)) + 1.0;
  const double by = std::ceil((double)((b4[3] - b4[2]) / rf)) + 1.0;
  if (bx * by >= 2147483647.0) {
    set_error("rpt_fuse_gains_max: grid of %.0f cells exceeds the int32 index space", bx * by);
    return RPT_ENOTSUP;
  }
  const int32_t nx = (int32_t)bx, ny = (int32_t)by;
  const int64_t cells = (int64_t)nx * ny;
  Scratch& sc = scratch(st);
  Budget bud;
  bud.add<unsigned int>(cells);
  bud.add<int32_t>(cells);
  bud.add<int32_t>(cells + 1);
  RPT_TRY(sc.reserve(bud.bytes, st));
  unsigned int* grid = sc.carve_n<unsigned int>(cells);
  int32_t* flag = sc.carve_n<int32_t>(cells);
  int32_t* pos = sc.carve_n<int32_t>(cells + 1);
  RPT_HIP(hipMemsetAsync(grid, 0, sizeof(unsigned int) * cells, st));
  hipLaunchKernelGGL(k_maxpool, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, st, x, y, v, n,
                     b4[0], b4[2], rf, ny, grid);
  hipLaunchKernelGGL(k_fuse_flags, dim3(grid_for(cells, kBlock, 4096)), dim3(kBlock), 0, st,
                     grid, nx, ny, flag);
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_total_i32(flag, pos, cells, st));
  hipLaunchKernelGGL(k_fuse_scatter, dim3(grid_for(cells, kBlock, 4096)), dim3(kBlock), 0, st,
                     grid, nx, ny, pos, (double)b4[0], (double)b4[2], res, ox, oy, oi);
  RPT_CHECK_LAUNCH();
  int32_t tot = 0;
  RPT_HIP(hipMemcpyAsync(&tot, pos + cells, sizeof(int32_t), hipMemcpyDeviceToHost, st));
  RPT_TRY(wait_stream(st));
  *n_out = tot;
  return RPT_OK;
}

}  // namespace rpt

extern "C" int32_t rpt_fuse_gains_max(const float* x, const float* y, const float* intensity,
                                      int64_t n, double grid_resolution, double* out_x,
                                      double* out_y, float* out_intensity, int64_t* n_out_host,
                                      void* stream) {
  rpt::clear_error();
  if (n < 0 || !n_out_host || (n > 0 && (!x || !y || !intensity || !out_x || !out_y ||
                                         !out_intensity))) {
    rpt::set_error("rpt_fuse_gains_max: bad arguments");
    return RPT_EINVAL;
  }
  if (n >= (int64_t(1) << 31) - 1) {
    rpt::set_error("rpt_fuse_gains_max: n exceeds the int32 index space");
    return RPT_ENOTSUP;
  }
  return rpt::fuse_gains_max(x, y, intensity, n, grid_resolution, out_x, out_y, out_intensity,
                             n_out_host, rpt::as_stream(stream));
}
