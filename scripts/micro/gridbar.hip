// Microbenchmark: cost of a software grid barrier (atomic arrive + acquire spin, agent scope) between the phases of one
// persistent launch, against a launch boundary. NB blocks x 256 threads, each block writes W floats per phase, then
// every block waits for all. The spin is bounded (a lost block ends the kernel with an error count, never a hang).
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/gridbar.hip -o scripts/micro/gridbar && ./scripts/micro/gridbar
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ bool grid_barrier(unsigned* arrive, unsigned target) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    long spins = 0;
    while (__hip_atomic_load(arrive, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1l << 22)) { ok = false; break; }
    }
  }
  __syncthreads();
  return ok;
}

__global__ __launch_bounds__(256) void phases(float* buf, int W, int iters, unsigned* arrive, unsigned* err) {
  const unsigned nb = gridDim.x;
  float acc = 0.0f;
  for (int it = 0; it < iters; ++it) {
    float* mine = buf + (size_t)blockIdx.x * W;
    for (int i = threadIdx.x; i < W; i += blockDim.x) mine[i] = (float)(it + i);
    if (!grid_barrier(arrive, nb * (unsigned)(it + 1))) {
      if (threadIdx.x == 0) atomicAdd(err, 1u);
      return;
    }
    // read another block's data (cross-XCD)
    const float* other = buf + (size_t)((blockIdx.x + 37) % nb) * W;
    acc += other[threadIdx.x % W];
  }
  if (acc == -1.0f) buf[0] = acc;
}
__global__ __launch_bounds__(256) void one_phase(float* buf, int W, int it) {
  const unsigned nb = gridDim.x;
  float* mine = buf + (size_t)blockIdx.x * W;
  const float* other = buf + (size_t)((blockIdx.x + 37) % nb) * W;
  float acc = other[threadIdx.x % W];
  for (int i = threadIdx.x; i < W; i += blockDim.x) mine[i] = (float)(it + i) + acc * 0.0f;
}

int main() {
  const int NBs[3] = {256, 448, 768};
  const int W = 8192, iters = 2000;
  float* buf; unsigned *arrive, *err;
  (void)hipMalloc(&buf, (size_t)1024 * W * sizeof(float));
  (void)hipMalloc(&arrive, 4); (void)hipMalloc(&err, 4);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipStream_t st; (void)hipStreamCreate(&st);
  for (int n = 0; n < 3; ++n) {
    const int NB = NBs[n];
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipMemsetAsync(arrive, 0, 4, st); (void)hipMemsetAsync(err, 0, 4, st);
      (void)hipEventRecord(e0, st);
      phases<<<NB, 256, 0, st>>>(buf, W, iters, arrive, err);
      (void)hipEventRecord(e1, st);
      (void)hipStreamSynchronize(st);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned h; (void)hipMemcpy(&h, err, 4, hipMemcpyDeviceToHost);
      printf("blocks %d: persistent, %d phases: %.3f us per phase (err %u)\n", NB, iters, ms * 1000.0f / iters, h);
    }
    // the same phases as separate launches captured in one graph
    hipGraph_t g; hipGraphExec_t ge;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int it = 0; it < 200; ++it) one_phase<<<NB, 256, 0, st>>>(buf, W, it);
    (void)hipStreamEndCapture(st, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0, st);
      (void)hipGraphLaunch(ge, st);
      (void)hipEventRecord(e1, st);
      (void)hipStreamSynchronize(st);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      printf("blocks %d: graph of 200 launches: %.3f us per launch\n", NB, ms * 1000.0f / 200);
    }
    (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(g);
  }
  return 0;
}
