// Device check of div_by (shipsim_device.hpp): n / d with the divisor's reciprocal formed once, against the
// compiler's own n / d, bitwise, over a sweep of operands (a test tool, not shipped).
//   hipcc --offload-arch=gfx950 -O3 -I include -I ast_sac_amd/csrc scripts/div_check.hip -o ast_sac_amd/lib/abl/div_check
//   ./div_check   -> per class: pairs tested, pairs differing (the documented domain must show 0)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "shipsim_device.hpp"

using namespace shipsim;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}
// a double with a random sign and mantissa and an exponent uniform in [e0, e1]
__device__ __forceinline__ double rnd(uint64_t k, int e0, int e1) {
  const uint64_t h = mix(k), g = mix(k ^ 0x9e3779b97f4a7c15ull);
  const int e = e0 + (int)(g % (uint64_t)(e1 - e0 + 1));
  const uint64_t bits = ((h >> 63) << 63) | ((uint64_t)(e + 1023) << 52) | (h & 0xfffffffffffffull);
  return __longlong_as_double((long long)bits);
}
// class 0: the documented domain (|d| in [2^-60, 2^60], |n| in [2^-900, 2^900]); class 1: n = +-0; class 2: the
// ship model's magnitudes (n in [2^-40, 2^40], d in [2^-10, 2^30]); class 3: outside (tiny numerators)
__global__ void check(uint64_t seed, long long per_thread, unsigned long long* out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  unsigned long long bad[4] = {0, 0, 0, 0};
  for (long long i = 0; i < per_thread; ++i) {
    const uint64_t k = seed ^ (t * 0x100000001b3ull + (uint64_t)i * 0x9e3779b97f4a7c15ull);
    const int cls = (int)(mix(k + 7) & 3);
    double n, d;
    if (cls == 0) { n = rnd(k, -900, 900); d = rnd(k + 1, -60, 60); }
    else if (cls == 1) { n = (k & 1) ? 0.0 : -0.0; d = rnd(k + 1, -60, 60); }
    else if (cls == 2) { n = rnd(k, -40, 40); d = rnd(k + 1, -10, 30); }
    else { n = rnd(k, -1074 + 52, -975); d = rnd(k + 1, -10, 30); }
    const double y = div_rcp(d);
    const double a = div_by(n, d, y);
    volatile double dv = d;  // (a plain division the compiler cannot rewrite)
    const double b = n / dv;
    if (__double_as_longlong(a) != __double_as_longlong(b)) bad[cls] += 1;
  }
  for (int c = 0; c < 4; ++c)
    if (bad[c]) atomicAdd(&out[c], bad[c]);
}

int main() {
  unsigned long long* d_out;
  hipMalloc(&d_out, 4 * sizeof(unsigned long long));
  hipMemset(d_out, 0, 4 * sizeof(unsigned long long));
  const int blocks = 4096, threads = 256;
  const long long per = 256;  // 2^28 pairs, a quarter per class
  check<<<blocks, threads>>>(0x5eed2025ull, per, d_out);
  unsigned long long h[4];
  hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
  const double tot = (double)blocks * threads * per / 4;
  const char* name[4] = {"domain |n| 2^-900..2^900, |d| 2^-60..2^60", "n = +-0", "ship-model magnitudes",
                         "outside: |n| < 2^-975 (v_div_scale scales)"};
  for (int c = 0; c < 4; ++c) printf("class %d (%s): ~%.0f pairs, %llu differ\n", c, name[c], tot, h[c]);
  hipFree(d_out);
  return (h[0] || h[1] || h[2]) ? 1 : 0;
}
