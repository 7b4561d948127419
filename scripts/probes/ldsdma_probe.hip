// L2 -> LDS DMA throughput probe: every workgroup streams STAGE-byte tiles of an L2-resident
// buffer into an NS-slot LDS ring with global_load_lds_dwordx4 (D = NS-1 stages in flight,
// counted vmcnt + barrier per stage, no compute), as the conv kernels' pipelines do.
// Build: hipcc --offload-arch=gfx950 -O3 ldsdma_probe.hip -o ldsdma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

template <int N>
__device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int NS, int G>
__global__ __launch_bounds__(256) void probe(const char* __restrict__ src, size_t span, int iters, float* sink) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  constexpr int STAGE = G * 4 * 1024;  // 4 waves x G wave-instructions x 1 KiB
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  size_t off = ((size_t)blockIdx.x * STAGE * 7) % span;
  auto issue = [&](int slot) {
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const char* p = src + off + (size_t)(i * 4 + wave) * 1024 + lane * 16;
      __builtin_amdgcn_global_load_lds((gbl_void*)p, (lds_void*)(smem + slot * STAGE + (i * 4 + wave) * 1024), 16, 0, 0);
    }
    off += STAGE;
    if (off + STAGE > span) off = 0;
  };
  constexpr int D = NS - 1;
#pragma unroll
  for (int s = 0; s < D; ++s) issue(s);
  float acc = 0.f;
  for (int t = 0; t < iters; ++t) {
    if (t + D - 1 < iters) vmwait<G * (D - 1)>(); else vmwait<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + D < iters) issue((t + D) % NS);
    acc += *reinterpret_cast<const float*>(smem + (t % NS) * STAGE + threadIdx.x * 4);
  }
  if (acc == 12345.f) sink[0] = acc;
}

template <int NS, int G>
void run(const char* buf, size_t span, int bpc, float* sink) {
  constexpr int STAGE = G * 4 * 1024;
  const int lds = NS * STAGE;
  hipFuncSetAttribute((const void*)probe<NS, G>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int grid = 256 * bpc, iters = 400;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((probe<NS, G>), dim3(grid), dim3(256), lds, 0, buf, span, iters, sink);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<NS, G>), dim3(grid), dim3(256), lds, 0, buf, span, iters, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double bytes = (double)grid * iters * STAGE;
  printf("NS=%d stage=%3d KiB blocks/CU=%d span=%6.1f MiB: %7.1f us  %6.1f GB/s/CU  %6.2f TB/s\n", NS, STAGE / 1024,
         bpc, span / 1048576.0, ms * 1e3, bytes / (ms * 1e-3) / 256 / 1e9, bytes / (ms * 1e-3) / 1e12);
}

int main() {
  char* buf;
  float* sink;
  const size_t big = 512ull << 20;
  hipMalloc(&buf, big);
  hipMalloc(&sink, 4);
  hipMemset(buf, 1, big);
  for (size_t span : {(size_t)2 << 20, (size_t)64 << 20, big}) {
    run<2, 8>(buf, span, 1, sink);
    run<2, 8>(buf, span, 2, sink);
    run<3, 8>(buf, span, 1, sink);
    run<4, 8>(buf, span, 1, sink);
    run<5, 8>(buf, span, 1, sink);
    run<3, 4>(buf, span, 2, sink);
    run<5, 4>(buf, span, 2, sink);
    run<8, 4>(buf, span, 1, sink);
    run<3, 8>(buf, span, 1, sink);
  }
  return 0;
}
