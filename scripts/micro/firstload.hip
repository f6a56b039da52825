// First-load burst at kernel start (scripts/micro/launch.hip found it): one float4 load per thread
// from a buffer no launch writes costs ~20 ns per 4 KiB page of the buffer read at the launch's start (256 KiB:
// +4.5 µs over a store-only launch; 2.5 MiB: +14 µs), while every thread reading one page is free. Here the same
// launch (448 blocks x 256 threads, ld1 of 256 KiB / 2.5 MiB, 30 launches in a graph) over buffers from different
// allocators: hipMalloc 8 MiB, a 2 MiB-aligned window of hipMalloc 512 MiB, hipExtMallocWithFlags fine-grained and
// uncached, and the same launches from the stream without a graph.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));          \
      exit(1);                                                                                   \
    }                                                                                            \
  } while (0)

__global__ __launch_bounds__(256) void k_ld1(const float4* in, float4* out, int n4) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < n4) out[t] = in[t];
}

// the same with the block's loads passed through LDS (a 4 KiB __shared__ array and a barrier), and a store-only
// launch with the same LDS use
__global__ __launch_bounds__(256) void k_ld1_lds(const float4* in, float4* out, int n4) {
  __shared__ float4 sh[256];
  const int t = blockIdx.x * 256 + threadIdx.x;
  sh[threadIdx.x] = t < n4 ? in[t] : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (t < n4) out[t] = sh[threadIdx.x ^ 1];
}
__global__ __launch_bounds__(256) void k_st_lds(const float4* in, float4* out, int n4) {
  __shared__ float4 sh[256];
  const int t = blockIdx.x * 256 + threadIdx.x;
  sh[threadIdx.x] = make_float4((float)t, 0.f, 0.f, 0.f);
  __syncthreads();
  if (t < n4 && in) out[t] = sh[threadIdx.x ^ 1];
}

typedef void (*kfn)(const float4*, float4*, int);
static kfn g_kern = k_ld1;

static float run(hipStream_t s, const float4* src, float4* dst, int n4, bool graph) {
  const int G = 448, K = 30, R = 50;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipGraphExec_t ge = nullptr;
  if (graph) {
    hipGraph_t g;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; ++k) hipLaunchKernelGGL(g_kern, dim3(G), dim3(256), 0, s, src, dst, n4);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
  }
  auto once = [&]() {
    if (graph) CK(hipGraphLaunch(ge, s));
    else
      for (int k = 0; k < K; ++k) hipLaunchKernelGGL(g_kern, dim3(G), dim3(256), 0, s, src, dst, n4);
  };
  for (int w = 0; w < 3; ++w) once();
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < R; ++r) once();
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  if (ge) CK(hipGraphExecDestroy(ge));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1e3f / (R * K);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float4 *dst, *a8, *big, *fg, *uc;
  CK(hipMalloc(&dst, 8 << 20));
  CK(hipMalloc(&a8, 8 << 20));
  CK(hipMalloc(&big, (size_t)512 << 20));
  CK(hipExtMallocWithFlags((void**)&fg, 8 << 20, hipDeviceMallocFinegrained));
  CK(hipExtMallocWithFlags((void**)&uc, 8 << 20, hipDeviceMallocUncached));
  for (float4* p : {dst, a8, fg, uc}) CK(hipMemset(p, 0, 8 << 20));
  CK(hipMemset(big, 0, (size_t)512 << 20));
  float4* win = (float4*)(((uintptr_t)big + (64u << 20)) & ~(uintptr_t)((2u << 20) - 1));
  struct { const char* name; const float4* p; } bufs[5] = {
      {"hipMalloc 8M", a8}, {"hipMalloc 512M window", win}, {"fine-grained", fg}, {"uncached", uc}, {"in == out", nullptr}};
  printf("buffer                  bytes     graph us/launch  stream us/launch\n");
  for (auto& b : bufs)
    for (int bytes : {256 << 10, (int)(2.5 * (1 << 20))}) {
      const int n4 = bytes / 16;
      const float4* src = b.p ? b.p : dst;  // in == out: reads the slot it then writes
      printf("%-22s %8d  %8.2f  %8.2f\n", b.name, bytes, run(s, src, dst, n4, true), run(s, src, dst, n4, false));
    }
  printf("kernel (hipMalloc 8M)    bytes     graph us/launch  stream us/launch\n");
  const kfn ks[3] = {k_ld1, k_ld1_lds, k_st_lds};
  const char* kn[3] = {"ld1", "ld1 via LDS", "store via LDS"};
  for (int k = 0; k < 3; ++k)
    for (int bytes : {256 << 10, (int)(2.5 * (1 << 20))}) {
      g_kern = ks[k];
      printf("%-22s %8d  %8.2f  %8.2f\n", kn[k], bytes, run(s, a8, dst, bytes / 16, true), run(s, a8, dst, bytes / 16, false));
    }
  CK(hipStreamDestroy(s));
  return 0;
}
