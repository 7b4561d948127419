// pool.hip — ImageNet stem max-pool 3x3/2 'SAME' (reference resnet_model_official.py:314-316)
// forward with a per-output uint8 argmax record, and the backward as a GATHER over the
// windows that selected each input element (no atomics, deterministic).
// TF 'SAME' geometry: P = ceil(H/stride), pad_beg = max((P-1)*stride + k - H, 0) / 2; padded
// taps never win (they are -inf for max pooling).
#include "drn_common.h"

namespace drn {

// One block per rows_per_block output rows (n, p); thread = (output column q, 8-channel group
// cv), so the row decode is one scalar division per row (the flat 64-bit index decode it
// replaces cost several 64-bit divisions per 16-byte output). With part set the block also
// reduces the per-channel sum / sum of squares of its bf16-rounded outputs -- the batch
// statistics of the first block's BatchNorm -- into replica blockIdx % rep (bn_stats_kernel's
// pattern), which saves the separate statistics pass over the pooled tensor.
// KC > 0: the window size is the compile-time KC (the ImageNet stem's 3x3), taps fully unrolled.
template <int KC>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C, int P,
                                                          int Q, int k, int stride, int pad_h, int pad_w,
                                                          int rows_per_block, float* __restrict__ part, int rep) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int CV = C / 8;
  const int tid = threadIdx.x;
  const int qstep = 256 / CV;  // output columns per pass (CV <= 256, host-checked)
  const int cv = tid % CV, q0 = tid / CV;
  float s[8], sq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = sq[j] = 0.f;
  const int row0 = blockIdx.x * rows_per_block;
  const int row1 = min(N * P, row0 + rows_per_block);
  if (q0 < qstep) {
    for (int row = row0; row < row1; ++row) {
      const int n = row / P, p = row - n * P;
      for (int q = q0; q < Q; q += qstep) {
        float best[8];
        uint8_t bi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
        if constexpr (KC > 0) {
          // fixed window: all KC*KC taps in flight together (out-of-image taps read as -inf and,
          // with the strict '>', never win -- the same first-maximum rule as the generic loop)
          uint4 v[KC * KC];
          const uint32_t ninf = 0xFF80FF80u;
#pragma unroll
          for (int r = 0; r < KC; ++r)
#pragma unroll
            for (int t = 0; t < KC; ++t) {
              const int h = p * stride - pad_h + r, w = q * stride - pad_w + t;
              v[r * KC + t] = ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
                                  ? *reinterpret_cast<const uint4*>(x + (((size_t)n * H + h) * W + w) * C + cv * 8)
                                  : make_uint4(ninf, ninf, ninf, ninf);
            }
#pragma unroll
          for (int tp = 0; tp < KC * KC; ++tp) {
            float f[8];
            unpack8(v[tp], f);
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (f[j] > best[j]) { best[j] = f[j]; bi[j] = (uint8_t)tp; }
          }
        } else {
          for (int r = 0; r < k; ++r) {
            const int h = p * stride - pad_h + r;
            if (h < 0 || h >= H) continue;
            for (int t = 0; t < k; ++t) {
              const int w = q * stride - pad_w + t;
              if (w < 0 || w >= W) continue;
              float f[8];
              unpack8(*reinterpret_cast<const uint4*>(x + (((size_t)n * H + h) * W + w) * C + cv * 8), f);
#pragma unroll
              for (int j = 0; j < 8; ++j)
                if (f[j] > best[j]) { best[j] = f[j]; bi[j] = (uint8_t)(r * k + t); }
            }
          }
        }
        const size_t o = ((size_t)row * Q + q) * CV + cv;
        const uint4 packed = pack8(best);
        reinterpret_cast<uint4*>(y)[o] = packed;
        uint2 a;
        a.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
        a.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
        reinterpret_cast<uint2*>(arg)[o] = a;
        if (part) {
          float f[8];
          unpack8(packed, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            s[j] += f[j];
            sq[j] += f[j] * f[j];
          }
        }
      }
    }
  }
  if (part == nullptr) return;  // uniform
  float* red = reinterpret_cast<float*>(smem);  // [256][17]: padded rows, conflict-free
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[tid * 17 + j] = s[j];
    red[tid * 17 + 8 + j] = sq[j];
  }
  __syncthreads();
  for (int t = tid; t < 2 * C; t += 256) {
    const int c = t >> 1, which = t & 1;
    const int cvv = c / 8, j = c % 8;
    float acc = 0.f;
    for (int r = 0; r < qstep; ++r) acc += red[(r * CV + cvv) * 17 + which * 8 + j];
    atomicAdd(part + ((size_t)(blockIdx.x % rep) * 2 + which) * C + c, acc);
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                          bf16_t* __restrict__ dx, int N, int H, int W, int C, int P,
                                                          int Q, int k, int stride, int pad_h, int pad_w) {
  const int CV = C / 8;
  const int64_t total = (int64_t)N * H * W * CV;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    int64_t t = i / CV;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // windows p with p*stride - pad_h <= h <= p*stride - pad_h + k - 1
    const int p_lo = max(0, (h + pad_h - k + stride) / stride);
    const int p_hi = min(P - 1, (h + pad_h) / stride);
    const int q_lo = max(0, (w + pad_w - k + stride) / stride);
    const int q_hi = min(Q - 1, (w + pad_w) / stride);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * stride - pad_h);
      if (r < 0 || r >= k) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * stride - pad_w);
        if (s < 0 || s >= k) continue;
        const int tap = r * k + s;
        const size_t o = (((size_t)n * P + p) * Q + q) * CV + cv;
        const uint2 a = reinterpret_cast<const uint2*>(arg)[o];
        float g[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], g);
        const uint8_t b[8] = {(uint8_t)(a.x), (uint8_t)(a.x >> 8), (uint8_t)(a.x >> 16), (uint8_t)(a.x >> 24),
                              (uint8_t)(a.y), (uint8_t)(a.y >> 8), (uint8_t)(a.y >> 16), (uint8_t)(a.y >> 24)};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (b[j] == tap) acc[j] += g[j];
      }
    }
    reinterpret_cast<uint4*>(dx)[i] = pack8(acc);
  }
}

// Stride-2 backward, one thread per 2x2 block of input pixels x 8 channels: the (at most 2x2)
// windows touching the block are each read once (dy + argmax) and scattered to the block's 4
// pixels in registers -- every window record is read ~1x instead of ~2.25x, and no thread loops
// over a data-dependent window count.
// NWD = max windows per dimension over a 2x2 input block: 2 for k <= 3, 3 for k = 4.
template <int NWD>
__device__ __forceinline__ void maxpool_bwd_s2_block(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                     bf16_t* __restrict__ dx, int n, int a, int b, int cv, int H,
                                                     int W, int CV, int P, int Q, int k, int pad_h, int pad_w) {
  const int h0 = 2 * a, w0 = 2 * b;
  float acc[2][2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[u][v][j] = 0.f;
  // windows p with p*2 - pad <= h <= p*2 - pad + k - 1 for h in {h0, h0 + 1}
  // (p_lo = ceil((h0 + pad - k + 1) / 2); C's truncation only matters below 0, where max() clamps)
  const int p_lo = max(0, (h0 + pad_h - k + 2) / 2), p_hi = min(P - 1, (h0 + 1 + pad_h) / 2);
  const int q_lo = max(0, (w0 + pad_w - k + 2) / 2), q_hi = min(Q - 1, (w0 + 1 + pad_w) / 2);
  // at most NWD windows per dimension touch a 2x2 block: all their records in flight together
  uint4 gv[NWD][NWD];
  uint2 av[NWD][NWD];
#pragma unroll
  for (int pi = 0; pi < NWD; ++pi)
#pragma unroll
    for (int qi = 0; qi < NWD; ++qi) {
      const int p = p_lo + pi, q = q_lo + qi;
      const bool ok = p <= p_hi && q <= q_hi;
      const size_t o = (((size_t)n * P + (ok ? p : 0)) * Q + (ok ? q : 0)) * CV + cv;
      gv[pi][qi] = ok ? reinterpret_cast<const uint4*>(dy)[o] : make_uint4(0u, 0u, 0u, 0u);
      av[pi][qi] = ok ? reinterpret_cast<const uint2*>(arg)[o] : make_uint2(~0u, ~0u);  // tap 255: never
    }
#pragma unroll
  for (int pi = 0; pi < NWD; ++pi) {
    const int p = p_lo + pi;
#pragma unroll
    for (int qi = 0; qi < NWD; ++qi) {
      const int q = q_lo + qi;
      const uint2 ar = av[pi][qi];
      float g[8];
      unpack8(gv[pi][qi], g);
      const uint8_t bt[8] = {(uint8_t)(ar.x), (uint8_t)(ar.x >> 8), (uint8_t)(ar.x >> 16), (uint8_t)(ar.x >> 24),
                             (uint8_t)(ar.y), (uint8_t)(ar.y >> 8), (uint8_t)(ar.y >> 16), (uint8_t)(ar.y >> 24)};
      const int r0 = h0 - (2 * p - pad_h), s0 = w0 - (2 * q - pad_w);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const int r = r0 + u, s = s0 + v;
          if (r >= 0 && r < k && s >= 0 && s < k) {
            const int tap = r * k + s;
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (bt[j] == tap) acc[u][v][j] += g[j];
          }
        }
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v)
      if (h0 + u < H && w0 + v < W)
        reinterpret_cast<uint4*>(dx)[(((size_t)n * H + h0 + u) * W + w0 + v) * CV + cv] = pack8(acc[u][v]);
}

// one thread per (2x2 block, 8-channel group), no loop: every thread's 2*NWD^2 loads are in
// flight at once (measured in-step at the ImageNet stem: 69 us vs 79 us for a row-per-block
// mapping whose threads looped over the row's columns, profiles/r4_experiments.md)
template <int NWD>
__global__ __launch_bounds__(256) void maxpool_bwd_s2_flat_kernel(const bf16_t* __restrict__ dy,
                                                                  const uint8_t* __restrict__ arg,
                                                                  bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                                                  int P, int Q, int k, int pad_h, int pad_w) {
  const int CV = C / 8;
  const int HB = (H + 1) / 2, WB = (W + 1) / 2;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * HB * WB * CV) return;
  const int cv = (int)(i % CV);
  const int64_t t = i / CV;
  const int b = (int)(t % WB);
  const int row = (int)(t / WB);
  const int n = row / HB, a = row - n * HB;
  maxpool_bwd_s2_block<NWD>(dy, arg, dx, n, a, b, cv, H, W, CV, P, Q, k, pad_h, pad_w);
}

static inline int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace drn

// part (optional): [rep][2][C] fp32 statistics accumulator of the output (sum, sum of squares)
DRN_API int drn_maxpool_fwd(const void* x, void* y, uint8_t* arg, int N, int H, int W, int C, int P, int Q, int k,
                            int stride, int pad_h, int pad_w, float* part, int rep, hipStream_t s) {
  if (C % 8 || C / 8 > 256 || (part != nullptr && rep < 1)) return (int)hipErrorInvalidValue;
  const int rows = N * P;
  const int rpb = rows >= 4096 ? 4 : 1;  // ~1.8K blocks at the ImageNet stem (128 x 56 rows)
  auto kern = k == 3 ? drn::maxpool_fwd_kernel<3> : drn::maxpool_fwd_kernel<0>;
  drn::launch(kern, dim3((rows + rpb - 1) / rpb), dim3(256), part ? 256 * 17 * 4 : 0, s, (const bf16_t*)x,
                     (bf16_t*)y, arg, N, H, W, C, P, Q, k, stride, pad_h, pad_w, rpb, part, rep);
  return (int)hipGetLastError();
}

DRN_API int drn_maxpool_bwd(const void* dy, const uint8_t* arg, void* dx, int N, int H, int W, int C, int P, int Q,
                            int k, int stride, int pad_h, int pad_w, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  if (stride == 2 && k <= 4) {
    const int64_t total = (int64_t)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
    auto kern = k <= 3 ? drn::maxpool_bwd_s2_flat_kernel<2> : drn::maxpool_bwd_s2_flat_kernel<3>;
    drn::launch(kern, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const bf16_t*)dy, arg,
                       (bf16_t*)dx, N, H, W, C, P, Q, k, pad_h, pad_w);
    return (int)hipGetLastError();
  }
  const int64_t total = (int64_t)N * H * W * (C / 8);
  drn::launch(drn::maxpool_bwd_kernel, dim3(drn::grid_for(total)), dim3(256), 0, s, (const bf16_t*)dy, arg,
                     (bf16_t*)dx, N, H, W, C, P, Q, k, stride, pad_h, pad_w);
  return (int)hipGetLastError();
}
