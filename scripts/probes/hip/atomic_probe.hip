// Probe: are fp32 atomicAdd (agent scope, no sc1) from all XCDs to the same addresses coherent
// within one kernel, and how fast are they? Each of B blocks adds 1.0 to every one of n words.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void add_all(float* p, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(p + i, 1.0f);
}
// each block adds into replica (blockIdx % rep)
__global__ void add_rep(float* p, int n, int rep) {
  float* q = p + (size_t)(blockIdx.x % rep) * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(q + i, 1.0f);
}
__global__ void store_part(float* p, int n) {  // split-K style: one slab per block
  float* q = p + (size_t)blockIdx.x * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) q[i] = 1.0f;
}

int main() {
  const int n = 16384, B = 256;
  float* d;
  hipMalloc(&d, (size_t)n * B * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<float> h(n);
  for (int rep : {1, 8, 64}) {
    hipMemset(d, 0, (size_t)n * rep * 4);
    hipEventRecord(e0);
    if (rep == 1) add_all<<<B, 256>>>(d, n); else add_rep<<<B, 256>>>(d, n, rep);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<float> all((size_t)n * rep);
    hipMemcpy(all.data(), d, all.size() * 4, hipMemcpyDeviceToHost);
    double tot = 0; int bad = 0;
    for (int r = 0; r < rep; ++r)
      for (int i = 0; i < n; ++i) tot += all[(size_t)r * n + i];
    for (int i = 0; i < n; ++i) {
      double s = 0;
      for (int r = 0; r < rep; ++r) s += all[(size_t)r * n + i];
      if (s != B) ++bad;
    }
    printf("rep %3d: %d blocks x %d atomics: %.1f us (%.1f G atomics/s), total %.0f (expect %d), bad words %d\n",
           rep, B, n, ms * 1e3, (double)B * n / (ms * 1e-3) / 1e9, tot, B * n, bad);
  }
  hipEventRecord(e0);
  store_part<<<B, 256>>>(d, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("split slabs: %d x %d stores %.1f us (%.2f TB/s)\n", B, n, ms * 1e3, (double)B * n * 4 / (ms * 1e-3) / 1e12);
  return 0;
}
