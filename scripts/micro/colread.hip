// Microbenchmark (diagnostics): 192 blocks of 256 threads, each reading a 32-column x 256-row tile of a
// row-major [256][pitch] fp32 matrix (2 x 128 B per wave load instruction, as the SAC weight-gradient tiles do)
// vs reading the same bytes contiguously. Pitch 256 (1 KB rows) and 288 (padded). Prints us per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ __launch_bounds__(256) void tile_cols(const float* __restrict__ m, int pitch, float* out) {
  const int b = blockIdx.x, t = b % 64, j0 = (t / 8) * 32, mat = b / 64;
  const float* M = m + (size_t)mat * 256 * pitch;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5;
  float acc = 0.f;
  float v[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = M[(size_t)(w * 64 + h * 32 + i) * pitch + j0 + (lane & 31)];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc += v[i];
  if (acc == 12345.f) out[b] = acc;
}
__global__ __launch_bounds__(256) void tile_contig(const float* __restrict__ m, float* out) {
  const int b = blockIdx.x;
  const float* M = m + (size_t)(b % 64) * 8192 + (size_t)(b / 64) * 65536 * 4;
  float acc = 0.f;
  float v[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = M[i * 256 + threadIdx.x];
#pragma unroll
  for (int i = 0; i < 32; ++i) acc += v[i];
  if (acc == 12345.f) out[b] = acc;
}
int main() {
  float *m, *out;
  hipMalloc(&m, sizeof(float) * 3 * 256 * 512 * 4);
  hipMalloc(&out, 4096);
  hipMemset(m, 0, sizeof(float) * 3 * 256 * 512 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode) {
    float best = 1e9;
    for (int rep = 0; rep < 200; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(tile_cols, dim3(192), dim3(256), 0, 0, m, 256, out);
      else if (mode == 1) hipLaunchKernelGGL(tile_cols, dim3(192), dim3(256), 0, 0, m, 288, out);
      else hipLaunchKernelGGL(tile_contig, dim3(192), dim3(256), 0, 0, m, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 10 && ms < best) best = ms;
    }
    printf("%s: %.2f us\n", mode == 0 ? "column tiles, pitch 1024 B" : mode == 1 ? "column tiles, pitch 1152 B" : "contiguous", best * 1000);
  }
  return 0;
}
