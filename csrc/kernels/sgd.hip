// sgd.hip — fused optimizer step and weight-layout maintenance on gfx950.
//
// Replaces TF's per-variable ApplyMomentum + L2Loss/AddN gradient of the weight-decay term
// (reference resnet_model.py:85-86 cost = xent + wd * sum(l2_loss(v)) over ALL trainable vars;
// :98-99 MomentumOptimizer(lr, 0.9), non-Nesterov) with ONE launch over the flat fp32
// master buffer (all 152/153 variables back to back):
//   g' = g * grad_scale + wd * w ;  m = mu * m + g' ;  w -= lr * m ;  w_bf16 = bf16(w)
// grad_scale folds the 1/world_size of the data-parallel average (SyncReplicas/Horovod mean).
// The learning rate is read from device memory so a captured HIP graph replays with the
// per-step LR written by the host (the reference feeds it through feed_dict each step,
// resnet_cifar_main.py:293-296).
#include "drn_common.h"

namespace drn {

// gradient element type: fp32 (local / fp32-wire gradients) or bf16 (the all-reduced bf16 wire
// buffer, consumed directly: no cast-back pass, half the gradient bytes)
__device__ __forceinline__ float4 grad4(const float* g, int64_t i) { return reinterpret_cast<const float4*>(g)[i]; }
__device__ __forceinline__ float4 grad4(const bf16_t* g, int64_t i) {
  const uint2 u = reinterpret_cast<const uint2*>(g)[i];
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

template <typename G>
__global__ __launch_bounds__(256) void sgd_momentum_kernel(float* __restrict__ w, float* __restrict__ m,
                                                           const G* __restrict__ g, bf16_t* __restrict__ wb,
                                                           int64_t n4, const float* __restrict__ lr_ptr, float mu,
                                                           float wd, float grad_scale, const int* __restrict__ skip) {
  // skip: the step's gradient exchange failed (P2P error word): apply no update at all
  if (skip != nullptr && *skip != 0) return;
  const float lr = *lr_ptr;
  auto upd = [&](float4& wv, float4& mv, const float4& gv) {
    float gg;
    gg = gv.x * grad_scale + wd * wv.x; mv.x = mu * mv.x + gg; wv.x -= lr * mv.x;
    gg = gv.y * grad_scale + wd * wv.y; mv.y = mu * mv.y + gg; wv.y -= lr * mv.y;
    gg = gv.z * grad_scale + wd * wv.z; mv.z = mu * mv.z + gg; wv.z -= lr * mv.z;
    gg = gv.w * grad_scale + wd * wv.w; mv.w = mu * mv.w + gg; wv.w -= lr * mv.w;
  };
  auto store = [&](int64_t i, const float4& wv, const float4& mv) {
    reinterpret_cast<float4*>(w)[i] = wv;
    reinterpret_cast<float4*>(m)[i] = mv;
    if (wb) {
      uint2 o;
      o.x = pack2bf(wv.x, wv.y);
      o.y = pack2bf(wv.z, wv.w);
      reinterpret_cast<uint2*>(wb)[i] = o;
    }
  };
  // two float4 groups in flight per thread (3 streams read, 3 written: one group per iteration
  // left the pass latency-bound at ~4.3 TB/s)
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    float4 w0 = reinterpret_cast<float4*>(w)[i], w1 = reinterpret_cast<float4*>(w)[i + stride];
    float4 m0 = reinterpret_cast<float4*>(m)[i], m1 = reinterpret_cast<float4*>(m)[i + stride];
    const float4 g0 = grad4(g, i), g1 = grad4(g, i + stride);
    upd(w0, m0, g0);
    upd(w1, m1, g1);
    store(i, w0, m0);
    store(i + stride, w1, m1);
  }
  if (i < n4) {
    float4 w0 = reinterpret_cast<float4*>(w)[i];
    float4 m0 = reinterpret_cast<float4*>(m)[i];
    const float4 g0 = grad4(g, i);
    upd(w0, m0, g0);
    store(i, w0, m0);
  }
}

__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                        int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    uint2 o;
    o.x = pack2bf(v.x, v.y);
    o.y = pack2bf(v.z, v.w);
    reinterpret_cast<uint2*>(y)[i] = o;
  }
}

// Data-gradient weights for a batch of convolutions described by a device-resident table (one
// launch for the whole network): Wt[c][u][v][k] = W[k][r0 + dr*u][s0 + ds*v][c], u < Ru, v < Sv.
// Full flip (stride-1 data gradient): Ru=R, r0=R-1, dr=-1. Stride-2 data gradients use one
// sub-kernel per output phase (taps of one parity, dr=-2), so no MFMA work is spent on the
// zeros of a dilated dY.
//
// For one tap the map is a K x C -> C x K matrix transpose, so the kernel is a tiled transpose:
// one workgroup per (descriptor, tap, 64-k tile, 64-c tile); rows of 64 c are read with 16-byte
// coalesced loads into LDS, and rows of 64 k leave with 16-byte coalesced stores. (An
// element-per-thread gather reads each 2-byte element from its own 32-byte sector.) The LDS row
// pitch of 66 elements (33 dwords) spreads the column reads of a wave over distinct banks.
struct TDesc {
  int64_t src, dst;       // element offsets into the flat bf16 weight buffers
  int32_t K, R, S, C;     // source KRSC dims (K, C multiples of 8)
  int32_t Ru, Sv, r0, s0; // destination taps and first source tap
  int32_t dr, ds, tk, tc; // tap steps; 64-wide tile counts along K and C
  int64_t begin;          // prefix sum of tile counts (Ru*Sv*tk*tc per descriptor)
};

constexpr int TF_T = 64, TF_PITCH = 66;

__global__ __launch_bounds__(256) void weight_tflip_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt,
                                                           const TDesc* __restrict__ table, int ntab) {
  __shared__ bf16_t tile[TF_T * TF_PITCH];
  // descriptor owning this tile (uniform scalar binary search)
  const int64_t b = blockIdx.x;
  int lo = 0, hi = ntab - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (table[mid].begin <= b) lo = mid; else hi = mid - 1;
  }
  const TDesc d = table[lo];
  int t = (int)(b - d.begin);
  const int taps = d.Ru * d.Sv;
  const int uv = t % taps; t /= taps;
  const int kt = t % d.tk, ct = t / d.tk;
  const int u = uv / d.Sv, v = uv - u * d.Sv;
  const int rs = d.r0 + d.dr * u, ss = d.s0 + d.ds * v;
  const int k0 = kt * TF_T, c0 = ct * TF_T;
  const int tid = threadIdx.x, ch = tid & 7, row = tid >> 3;  // 8 chunks of 8 elements x 32 rows
  const int64_t kstride = (int64_t)d.R * d.S * d.C;
  const bf16_t* src = w + d.src + ((int64_t)rs * d.S + ss) * d.C;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = k0 + row + h * 32, c = c0 + ch * 8;
    uint4 val = make_uint4(0, 0, 0, 0);
    if (k < d.K && c < d.C) val = *reinterpret_cast<const uint4*>(src + k * kstride + c);
    uint32_t* l = reinterpret_cast<uint32_t*>(tile + (row + h * 32) * TF_PITCH + ch * 8);
    l[0] = val.x; l[1] = val.y; l[2] = val.z; l[3] = val.w;
  }
  __syncthreads();
  bf16_t* dst = wt + d.dst + (int64_t)uv * d.K;
  const int64_t cstride = (int64_t)taps * d.K;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int cl = row + h * 32, c = c0 + cl, k = k0 + ch * 8;
    if (c < d.C && k < d.K) {
      uint32_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo16 = tile[(ch * 8 + 2 * j) * TF_PITCH + cl];
        const uint32_t hi16 = tile[(ch * 8 + 2 * j + 1) * TF_PITCH + cl];
        o[j] = lo16 | (hi16 << 16);
      }
      *reinterpret_cast<uint4*>(dst + c * cstride + k) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

__global__ void fill_f32_kernel(float* __restrict__ x, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) x[i] = v;
}

static inline int grid_for(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace drn

// skip (nullable device int): when *skip != 0 at run time the launch changes nothing;
// g_bf16: the gradient is bf16 (the all-reduced bf16 wire buffer), else fp32
DRN_API int drn_sgd_momentum(float* w, float* m, const void* g, int g_bf16, void* w_bf16, int64_t n,
                             const float* lr_ptr, float momentum, float wd, float grad_scale, const int* skip,
                             hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  if (g_bf16)
    drn::launch(drn::sgd_momentum_kernel<bf16_t>, dim3(drn::grid_for(n / 4)), dim3(256), 0, s, w, m,
                       (const bf16_t*)g, (bf16_t*)w_bf16, n / 4, lr_ptr, momentum, wd, grad_scale, skip);
  else
    drn::launch(drn::sgd_momentum_kernel<float>, dim3(drn::grid_for(n / 4)), dim3(256), 0, s, w, m,
                       (const float*)g, (bf16_t*)w_bf16, n / 4, lr_ptr, momentum, wd, grad_scale, skip);
  return (int)hipGetLastError();
}

DRN_API int drn_cast_bf16(const float* x, void* y, int64_t n, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  drn::launch(drn::cast_bf16_kernel, dim3(drn::grid_for(n / 4)), dim3(256), 0, s, x, (bf16_t*)y, n / 4);
  return (int)hipGetLastError();
}

// total = number of tiles (last begin + its count); every descriptor has K % 8 == C % 8 == 0.
DRN_API int drn_weight_tflip(const void* w, void* wt, const void* table, int ntab, int64_t total, hipStream_t s) {
  if (ntab < 1 || total < 1 || total > 0x7fffffff) return (int)hipErrorInvalidValue;
  drn::launch(drn::weight_tflip_kernel, dim3((unsigned)total), dim3(256), 0, s, (const bf16_t*)w,
                     (bf16_t*)wt, (const drn::TDesc*)table, ntab);
  return (int)hipGetLastError();
}

DRN_API int drn_fill_f32(float* x, int64_t n, float v, hipStream_t s) {
  drn::launch(drn::fill_f32_kernel, dim3(drn::grid_for(n)), dim3(256), 0, s, x, n, v);
  return (int)hipGetLastError();
}

DRN_API int drn_version() { return 1; }
