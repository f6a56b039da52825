// Launch-boundary cost on MI355X (the SAC step's three launches): a HIP graph of K back-to-back
// launches of one kernel shape, replayed R times, timed with HIP events — µs per launch for
//   empty  : no memory access (dispatch + completion of G blocks of 256 threads)
//   write  : every thread stores its share of `bytes` (the end-of-kernel write-back of that much dirty data)
//   (kinds chain .. ld8far: their kernels read the AQL dispatch packet — a private float4 promoted to LDS, indexed by
//    workitem id — which is what makes them slow; firstload.hip measures the same loads without that)
//   chain  : every thread reads what the previous launch wrote at another block's slot (so across XCDs) and
//            writes its own share: a dependent producer -> consumer pair per boundary, as P1 -> P2 -> P3
//   same / xcd / static : chain reading its own slot (same XCD as the writer), another block's slot on the same
//            XCD, or a buffer no launch of the graph writes
//   ld1 / ld4 / ld4far / ld8far : 1, 4 or 8 dependent loads per thread from that unwritten buffer (same line, or a
//            new 1 MiB-apart page each time)
// G in {48, 241, 384, 448} (the SAC launches' grids at B = 32 / 256), bytes in {0, 256 KiB, 2.5 MiB}.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ __launch_bounds__(256) void k_empty(float* out) {
  if (out && threadIdx.x == 1023) out[0] = 0.f;  // never true: keeps the argument live
}

__global__ __launch_bounds__(256) void k_write(float4* out, int n4) {
  const int t = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  for (int i = t; i < n4; i += stride) out[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

__global__ __launch_bounds__(256) void k_chain(const float4* in, float4* out, int n4, int shift) {
  // read the slot of block (b + shift) mod G: 37 = another XCD (blocks are dealt round-robin over the 8 XCDs),
  // 0 = the same block index (the same XCD), 16 = another block of the same XCD
  const int G = gridDim.x, b = (blockIdx.x + shift) % G, stride = G * 256;
  const int ts = b * 256 + threadIdx.x, td = blockIdx.x * 256 + threadIdx.x;
  for (int i = 0; ts + i < n4 && td + i < n4; i += stride) {
    float4 v = in[ts + i];
    v.x += 1.f;
    out[td + i] = v;
  }
}

// nload dependent loads per thread from a buffer no launch writes: each address depends on the previous value
// (always 0), at the next float4 of the same line (far = 0: warm after the first) or 1 MiB further (far = 1: a new
// page and line each time) — the first load's cost against a warm one's
__global__ __launch_bounds__(256) void k_dep(const float4* in, float4* out, int n4, int nload, int far) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n4) return;
  int idx = t;
  float4 v = in[idx];
  for (int k = 1; k < nload; ++k) {
    idx = (far ? (idx + 65536) % (1 << 19) : (idx ^ 1)) + (int)v.x;
    v = in[idx];
  }
  out[t] = v;
}

// one load per thread from a buffer no launch writes, every thread at one address (mode 0: c[0]) or within one
// 4 KiB page (mode 1: c[t & 255]): per-wave first-load cost without per-page or per-line traffic
__global__ __launch_bounds__(256) void k_narrow(const float4* in, float4* out, int n4, int mode) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n4) return;
  out[t] = in[mode ? (t & 255) : 0];
}

int main() {
  const int grids[4] = {48, 241, 384, 448};
  const size_t sizes[3] = {0, 256 << 10, (size_t)(2.5 * (1 << 20))};
  const int K = 30, R = 50;
  float4 *a, *b, *c;
  CK(hipMalloc(&a, 8 << 20));
  CK(hipMalloc(&b, 8 << 20));
  CK(hipMalloc(&c, 8 << 20));
  CK(hipMemset(a, 0, 8 << 20));
  CK(hipMemset(b, 0, 8 << 20));
  CK(hipMemset(c, 0, 8 << 20));
  const char* names[12] = {"empty", "write", "chain", "same", "xcd", "static", "ld1", "ld4", "ld4far", "ld8far", "bcast", "page1"};
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("kind   grid  bytes     us/launch\n");
  for (int kind = 0; kind < 12; ++kind)
    for (int gi = 0; gi < 4; ++gi)
      for (int si = 0; si < 3; ++si) {
        if (kind == 0 && si > 0) continue;
        if (kind > 0 && si == 0) continue;
        const int G = grids[gi];
        const int n4 = (int)(sizes[si] / 16);
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < K; ++k) {
          float4* src = (k & 1) ? b : a;
          float4* dst = (k & 1) ? a : b;
          if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(G), dim3(256), 0, s, (float*)nullptr);
          else if (kind == 1) hipLaunchKernelGGL(k_write, dim3(G), dim3(256), 0, s, dst, n4);
          else if (kind == 2) hipLaunchKernelGGL(k_chain, dim3(G), dim3(256), 0, s, src, dst, n4, 37);
          else if (kind == 3) hipLaunchKernelGGL(k_chain, dim3(G), dim3(256), 0, s, src, dst, n4, 0);
          else if (kind == 4) hipLaunchKernelGGL(k_chain, dim3(G), dim3(256), 0, s, src, dst, n4, 16);
          else if (kind == 5) hipLaunchKernelGGL(k_chain, dim3(G), dim3(256), 0, s, (const float4*)c, dst, n4, 37);
          else if (kind == 6) hipLaunchKernelGGL(k_dep, dim3(G), dim3(256), 0, s, (const float4*)c, dst, n4, 1, 0);
          else if (kind == 7) hipLaunchKernelGGL(k_dep, dim3(G), dim3(256), 0, s, (const float4*)c, dst, n4, 4, 0);
          else if (kind == 8) hipLaunchKernelGGL(k_dep, dim3(G), dim3(256), 0, s, (const float4*)c, dst, n4, 4, 1);
          else if (kind == 9) hipLaunchKernelGGL(k_dep, dim3(G), dim3(256), 0, s, (const float4*)c, dst, n4, 8, 1);
          else hipLaunchKernelGGL(k_narrow, dim3(G), dim3(256), 0, s, (const float4*)c, dst, n4, kind - 10);
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < R; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-6s %4d  %8zu  %.2f\n", names[kind], G, sizes[si],
               ms * 1e3 / (R * K));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
  CK(hipStreamDestroy(s));
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
