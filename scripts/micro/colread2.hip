// Microbenchmark (diagnostics): the SAC weight-gradient operand pattern read right after another kernel wrote
// the matrices (192 blocks x 256 threads; lane reads 32 rows of dY and 32 rows of X, 128 B per half-wave per
// row, 1 KB row pitch) vs read again (clean), and with 16 rows per operand. Prints us per read launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CK(x) (void)(x)
__global__ __launch_bounds__(256) void writer(float* m, float v) {
  // 6 matrices [256][256]: block b writes rows [b * 8, b * 8 + 8) of every matrix (row-major, coalesced)
  for (int mat = 0; mat < 6; ++mat)
    for (int r = 0; r < 8; ++r) m[(size_t)mat * 65536 + (size_t)(blockIdx.x * 8 + r) * 256 + threadIdx.x] = v;
}
// the SAC store_slice pattern: block (row tile rt, column tile by) of a 64-block grid; the half-wave whose
// 32-column slice is column tile `by` writes its row's 128 B as 8 float4s per lane
__global__ __launch_bounds__(256) void writer_slice(float* m, float v) {
  const int L = blockIdx.x, by = L & 7, rt = L >> 3;  // 8 row tiles x 8 column tiles per matrix
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, kb = w * 64 + h * 32;
  if (kb / 32 != by) return;
  for (int mat = 0; mat < 6; ++mat)
    for (int rr = 0; rr < 1; ++rr) {
      float4* d = reinterpret_cast<float4*>(m + (size_t)mat * 65536 + (size_t)(rt * 32 + (lane & 31)) * 256 + kb);
      for (int q = 0; q < 8; ++q) d[q] = make_float4(v, v, v, v);
    }
}
template <int NR>
__global__ __launch_bounds__(256) void reader(const float* __restrict__ m, float* out) {
  const int b = blockIdx.x, t = b % 64, j0 = (t / 8) * 32, k0 = (t % 8) * 32, mat = b / 64;
  const float* dY = m + (size_t)(2 * mat) * 65536;
  const float* X = m + (size_t)(2 * mat + 1) * 65536;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  float a[NR], c[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int r = w * 64 + h * 32 + i;
    a[i] = dY[(size_t)r * 256 + j0 + (lane & 31)];
    c[i] = X[(size_t)r * 256 + k0 + (lane & 31)];
  }
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < NR; ++i) acc += a[i] * c[i];
  if (acc == 12345.f) out[b] = acc;
}
int main() {
  float *m, *out;
  CK(hipMalloc(&m, sizeof(float) * 6 * 65536));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(m, 0, sizeof(float) * 6 * 65536));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[5] = {"32 rows/operand after the writer", "32 rows/operand, clean (read twice)",
                          "16 rows/operand after the writer", "writer alone", "32 rows/operand after slice writer"};
  for (int mode = 0; mode < 5; ++mode) {
    float tot = 0; int n = 0;
    for (int rep = 0; rep < 300; ++rep) {
      if (mode == 4) {
        for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(writer_slice, dim3(64), dim3(256), 0, 0, m, (float)rep);
      } else {
        hipLaunchKernelGGL(writer, dim3(32), dim3(256), 0, 0, m, (float)rep);
      }
      if (mode == 1) hipLaunchKernelGGL(reader<32>, dim3(192), dim3(256), 0, 0, m, out);
      CK(hipEventRecord(e0));
      if (mode == 0 || mode == 1 || mode == 4) hipLaunchKernelGGL(reader<32>, dim3(192), dim3(256), 0, 0, m, out);
      else if (mode == 2) hipLaunchKernelGGL(reader<16>, dim3(192), dim3(256), 0, 0, m, out);
      else hipLaunchKernelGGL(writer, dim3(32), dim3(256), 0, 0, m, (float)rep);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep >= 20) { tot += ms; ++n; }
    }
    printf("%-40s %.2f us\n", names[mode], 1000 * tot / n);
  }
  return 0;
}
