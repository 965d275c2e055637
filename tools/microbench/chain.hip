// Calibration: cost per step of a dependent float32 add chain on one wave (gfx950), the critical
// path of K9's order-preserving centroid sums.  Usage: ./chain  (prints cycles/step per variant)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int N = 1 << 16;

__global__ void k_scalar(const float* __restrict__ a, float* out, long long* cyc) {
  float s = a[0];
  long long t0 = clock64();
#pragma unroll 16
  for (int i = 1; i < N; ++i) s = s + a[i & 63];
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = s; cyc[0] = t1 - t0; }
}
__global__ void k_two(const float* __restrict__ a, float* out, long long* cyc) {
  float s = a[0], r = a[1];
  long long t0 = clock64();
#pragma unroll 16
  for (int i = 1; i < N; ++i) { s = s + a[i & 63]; r = r + a[(i + 7) & 63]; }
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = s + r; cyc[0] = t1 - t0; }
}
__global__ void k_packed(const float* __restrict__ a, float* out, long long* cyc) {
  f32x2 s = {a[0], a[1]};
  long long t0 = clock64();
#pragma unroll 16
  for (int i = 1; i < N; ++i) { f32x2 v = {a[i & 63], a[(i + 7) & 63]}; s = s + v; }
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = s.x + s.y; cyc[0] = t1 - t0; }
}
// operands in registers (values from lanes, no memory in the loop)
__global__ void k_regs(const float* __restrict__ a, float* out, long long* cyc) {
  const float v = a[threadIdx.x & 63];
  float s = 0.f;
  long long t0 = clock64();
  for (int r = 0; r < N / 64; ++r) {
#pragma unroll
    for (int l = 0; l < 64; ++l) s = s + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = s; cyc[0] = t1 - t0; }
}
__global__ void k_dep_only(float* out, long long* cyc, float seed) {
  float s = seed, d = seed * 0.5f;
  long long t0 = clock64();
#pragma unroll 64
  for (int i = 0; i < N; ++i) s = s + d;
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = s; cyc[0] = t1 - t0; }
}

__global__ void k_pk_dep(float* out, long long* cyc, float seed) {
  f32x2 s = {seed, seed * 2.f}, d = {seed * 0.5f, seed * 0.25f};
  long long t0 = clock64();
#pragma unroll 64
  for (int i = 0; i < N; ++i) s = s + d;
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = s.x + s.y; cyc[0] = t1 - t0; }
}
// k_summarize's shape: pairs staged in LDS, uniform broadcast reads double-buffered 16 ahead
__global__ void k_lds_pk(const float* __restrict__ a, float* out, long long* cyc) {
  __shared__ float2 sb[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) sb[i] = make_float2(a[i & 63], a[(i + 5) & 63]);
  __syncthreads();
  f32x2 acc = {0.f, 0.f};
  long long t0 = clock64();
  for (int rep = 0; rep < N / 1024; ++rep) {
    constexpr int V = 16;
    f32x2 cur[V], nxt[V];
#pragma unroll
    for (int u = 0; u < V; ++u) cur[u] = f32x2{sb[u].x, sb[u].y};
    for (int i = 0; i + 2 * V <= 1024; i += V) {
#pragma unroll
      for (int u = 0; u < V; ++u) nxt[u] = f32x2{sb[i + V + u].x, sb[i + V + u].y};
#pragma unroll
      for (int u = 0; u < V; ++u) acc = acc + cur[u];
#pragma unroll
      for (int u = 0; u < V; ++u) cur[u] = nxt[u];
    }
#pragma unroll
    for (int u = 0; u < V; ++u) acc = acc + cur[u];
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = acc.x + acc.y; cyc[0] = t1 - t0; }
}
// same, two scalar chains (x, y) instead of packed
__global__ void k_lds_two(const float* __restrict__ a, float* out, long long* cyc) {
  __shared__ float2 sb[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) sb[i] = make_float2(a[i & 63], a[(i + 5) & 63]);
  __syncthreads();
  float ax = 0.f, ay = 0.f;
  long long t0 = clock64();
  for (int rep = 0; rep < N / 1024; ++rep) {
    constexpr int V = 16;
    float2 cur[V], nxt[V];
#pragma unroll
    for (int u = 0; u < V; ++u) cur[u] = sb[u];
    for (int i = 0; i + 2 * V <= 1024; i += V) {
#pragma unroll
      for (int u = 0; u < V; ++u) nxt[u] = sb[i + V + u];
#pragma unroll
      for (int u = 0; u < V; ++u) { ax = ax + cur[u].x; ay = ay + cur[u].y; }
#pragma unroll
      for (int u = 0; u < V; ++u) cur[u] = nxt[u];
    }
#pragma unroll
    for (int u = 0; u < V; ++u) { ax = ax + cur[u].x; ay = ay + cur[u].y; }
  }
  long long t1 = clock64();
  if (threadIdx.x == 0) { out[0] = ax + ay; cyc[0] = t1 - t0; }
}

int main() {
  float *a, *o; long long* c;
  (void)hipMalloc(&a, 64 * 4); (void)hipMalloc(&o, 4); (void)hipMalloc(&c, 8);
  std::vector<float> h(64); for (int i = 0; i < 64; ++i) h[i] = 0.37f * i + 1.f;
  (void)hipMemcpy(a, h.data(), 256, hipMemcpyHostToDevice);
  long long cy;
  auto run = [&](const char* name, auto launch) {
    launch(); (void)hipDeviceSynchronize(); launch(); (void)hipDeviceSynchronize();
    (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    printf("%-12s %.2f cycles/step\n", name, (double)cy / N);
  };
  run("scalar", [&] { hipLaunchKernelGGL(k_scalar, 1, 64, 0, 0, a, o, c); });
  run("two-chains", [&] { hipLaunchKernelGGL(k_two, 1, 64, 0, 0, a, o, c); });
  run("packed", [&] { hipLaunchKernelGGL(k_packed, 1, 64, 0, 0, a, o, c); });
  run("readlane", [&] { hipLaunchKernelGGL(k_regs, 1, 64, 0, 0, a, o, c); });
  run("dep-only", [&] { hipLaunchKernelGGL(k_dep_only, 1, 64, 0, 0, o, c, 1.5f); });
  run("pk-dep", [&] { hipLaunchKernelGGL(k_pk_dep, 1, 64, 0, 0, o, c, 1.5f); });
  run("lds-pk", [&] { hipLaunchKernelGGL(k_lds_pk, 1, 64, 0, 0, a, o, c); });
  run("lds-two", [&] { hipLaunchKernelGGL(k_lds_two, 1, 64, 0, 0, a, o, c); });
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0); hipLaunchKernelGGL(k_dep_only, 1, 64, 0, 0, o, c, 1.5f); (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1); float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
  printf("dep-only wall %.1f us for %d steps, clock64 delta %lld -> %.2f GHz-equivalent\n", ms * 1e3, N, cy, cy / (ms * 1e6));
  return 0;
}
