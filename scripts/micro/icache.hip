// Microbenchmark (diagnostics): does a kernel's code stay in the instruction cache from one dispatch to the
// next? K distinct kernels of ~13 KB of straight-line code each (8 independent fmaf chains, a literal per
// instruction), 256 blocks x 256 threads (one block per CU), launched round-robin: K = 1 (the same code every
// launch), 3 (~39 KB), 4 (~52 KB), 6 (~77 KB, past a 64 KB cache). Prints us per launch (HIP events over
// 400 launches after 50 warmup). If code survives between dispatches, K = 1 / 3 / 4 run faster than K = 6.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int ID>
__global__ __launch_bounds__(256) void body(float* out, float x) {
  float a[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) a[c] = x + (float)c;
#pragma unroll
  for (int i = 0; i < 176; ++i)
#pragma unroll
    for (int c = 0; c < 8; ++c) a[c] = fmaf(a[c], 1.0f + (float)(ID * 4096 + i * 8 + c) * 1e-7f, (float)(i + c) * 1e-6f);
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += a[c];
  if (s == 12345.678f) out[blockIdx.x * 256 + threadIdx.x] = s;  // keeps the chains live
}

typedef void (*KFn)(float*, float);

int main() {
  float* out;
  if (hipMalloc(&out, 256 * 256 * sizeof(float)) != hipSuccess) return 1;
  KFn k[6] = {body<0>, body<1>, body<2>, body<3>, body<4>, body<5>};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int kinds[4] = {1, 3, 4, 6};
  for (int rep = 0; rep < 2; ++rep)
    for (int t = 0; t < 4; ++t) {
      const int K = kinds[t];
      for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k[i % K], dim3(256), dim3(256), 0, 0, out, 1.0f);
      (void)hipEventRecord(e0, 0);
      for (int i = 0; i < 400; ++i) hipLaunchKernelGGL(k[i % K], dim3(256), dim3(256), 0, 0, out, 1.0f);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("rep %d: K = %d distinct kernels round-robin: %.3f us per launch\n", rep, K, 1000.0f * ms / 400);
    }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
