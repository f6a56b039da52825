// Microbenchmark (diagnostics): L2->CU read rate of the SAC rows-kernel weight pattern, each block reading
// 8 x 256 KB fp32 matrices. Build: hipcc --offload-arch=gfx950 -O3 scripts/mb_weight_read.hip -o mb; run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdio.h>
// each block reads an HxH fp32 matrix (256 KB) NM times and does matvec-like FMAs
constexpr int H = 256;
// (a) column per thread, split-K KS groups of 256 threads: thread j reads W[k*H+j], k in its slice
template <int KS>
__global__ __launch_bounds__(256 * KS) void col_kernel(const float* W, int nm, float* out) {
  const int j = threadIdx.x % 256, kg = threadIdx.x / 256;
  __shared__ float x[H];
  if (threadIdx.x < H) x[threadIdx.x] = 0.001f * threadIdx.x;
  __syncthreads();
  float acc = 0;
  for (int m = 0; m < nm; ++m) {
    const float* Wm = W + (size_t)(m % 4) * H * H;
    const int len = H / KS, k0 = kg * len;
#pragma unroll 8
    for (int k = k0; k < k0 + len; ++k) acc = fmaf(Wm[k * H + j], x[k], acc);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
// (b) dwordx4: lane owns 4 columns, wave w takes rows k = w, w+NW, ...
template <int NWV>
__global__ __launch_bounds__(64 * NWV) void row_kernel(const float* W, int nm, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ float x[H];
  if (threadIdx.x < H) x[threadIdx.x] = 0.001f * threadIdx.x;
  __syncthreads();
  float a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  for (int m = 0; m < nm; ++m) {
    const float4* W4 = reinterpret_cast<const float4*>(W + (size_t)(m % 4) * H * H) + lane;
#pragma unroll 8
    for (int k = w; k < H; k += NWV) {
      const float4 v = W4[k * (H / 4)];
      const float xx = x[k];
      a0 = fmaf(v.x, xx, a0); a1 = fmaf(v.y, xx, a1); a2 = fmaf(v.z, xx, a2); a3 = fmaf(v.w, xx, a3);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
}
// (c) dwordx4 with a contiguous K slice per wave
template <int NWV>
__global__ __launch_bounds__(64 * NWV) void rowc_kernel(const float* W, int nm, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ float x[H];
  if (threadIdx.x < H) x[threadIdx.x] = 0.001f * threadIdx.x;
  __syncthreads();
  float a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  const int len = H / NWV;
  for (int m = 0; m < nm; ++m) {
    const float4* W4 = reinterpret_cast<const float4*>(W + (size_t)(m % 4) * H * H) + lane;
#pragma unroll 8
    for (int k = w * len; k < (w + 1) * len; ++k) {
      const float4 v = W4[k * (H / 4)];
      const float xx = x[k];
      a0 = fmaf(v.x, xx, a0); a1 = fmaf(v.y, xx, a1); a2 = fmaf(v.z, xx, a2); a3 = fmaf(v.w, xx, a3);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
}
int main() {
  float *W, *out;
  hipMalloc(&W, sizeof(float) * 4 * H * H);
  hipMalloc(&out, sizeof(float) * 256 * 1024);
  hipMemset(W, 0, sizeof(float) * 4 * H * H);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int nm = 8;  // 8 matrices of 256 KB per block = 2 MB, like the SAC rows kernel
  for (int nb : {256, 128}) {
    auto run = [&](const char* name, auto launch) {
      launch(); hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) launch();
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1000 / 20;
      printf("%-28s blocks %3d: %7.2f us/launch  %6.1f B/clk/CU (2.4 GHz)  %6.2f TB/s aggregate\n", name, nb, us,
             nm * 256.0 * 1024 / (us * 1e-6 * 2.4e9), nb * nm * 256.0 * 1024 / (us * 1e-6) / 1e12);
    };
    run("col KS=4 (1024 thr)", [&] { hipLaunchKernelGGL(col_kernel<4>, dim3(nb), dim3(1024), 0, 0, W, nm, out); });
    run("col KS=1 (256 thr)", [&] { hipLaunchKernelGGL(col_kernel<1>, dim3(nb), dim3(256), 0, 0, W, nm, out); });
    run("row x4 strided 16 waves", [&] { hipLaunchKernelGGL(row_kernel<16>, dim3(nb), dim3(1024), 0, 0, W, nm, out); });
    run("row x4 contiguous 16 waves", [&] { hipLaunchKernelGGL(rowc_kernel<16>, dim3(nb), dim3(1024), 0, 0, W, nm, out); });
    run("row x4 strided 4 waves", [&] { hipLaunchKernelGGL(row_kernel<4>, dim3(nb), dim3(256), 0, 0, W, nm, out); });
  }
  return 0;
}
