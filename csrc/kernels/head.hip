// head.hip — classifier head on gfx950: final BN-ReLU + global average pool, dense layer
// (fp32 GEMMs), softmax cross-entropy with one-hot labels and the batch precision metric.
//
// Reference: final batch_norm_relu + average_pooling2d(VALID, pool = H) + dense
// (resnet_model_official.py:268-275 CIFAR, :336-343 ImageNet); softmax + mean
// softmax_cross_entropy (resnet_model.py:77-80); train "precision" = mean(argmax p == argmax y)
// (resnet_cifar_main.py:270-272).
#include "drn_common.h"

namespace drn {

// pooled[n][c] = mean_hw relu(x[n][hw][c]*scale[c] + shift[c])   (scale==nullptr: no BN)
__global__ __launch_bounds__(256) void bnrelu_pool_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, float* __restrict__ pooled,
                                                          int HW, int C, int relu) {
  const int n = blockIdx.x;
  const int CV = C / 8;
  for (int cv = threadIdx.x; cv < CV; cv += blockDim.x) {
    const int c = cv * 8;
    float acc[8], sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc[j] = 0.f;
      sc[j] = scale ? scale[c + j] : 1.f;
      sh[j] = scale ? shift[c + j] : 0.f;
    }
    for (int hw = 0; hw < HW; ++hw) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(x + ((size_t)n * HW + hw) * C + c), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = f[j] * sc[j] + sh[j];
        if (relu) v = fmaxf(v, 0.f);
        acc[j] += v;
      }
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int j = 0; j < 8; ++j) pooled[(size_t)n * C + c + j] = acc[j] * inv;
  }
}

// C[M][N] = alpha * op(A) op(B) + beta * C (+ bias[N]); row-major; op = transpose if flag.
// Exact-fp32 MFMA (v_mfma_f32_16x16x4_f32, the f32-input matrix path: 16x the VALU-FMA work
// per instruction, bitwise a k-ordered fmaf chain). 64x64 block tile, 4 waves each 32x32
// (2x2 MFMA tiles), K staged 32 at a time through double-buffered LDS ([k][m] and [k][n], +1
// padding): the next slab's global loads are issued into registers before the current slab's
// MFMAs and stored to the other buffer after them (one barrier per slab), so their latency
// hides behind the MFMA chain -- the unpipelined load/barrier/MFMA loop, one workgroup per CU,
// was latency-bound (60 us for the 0.5 GFLOP ResNet-50 logits GEMM).
// Used for the dense layer of the head (logits, dW, dpool: <1 GFLOP each).
__global__ __launch_bounds__(256) void sgemm_kernel(int ta, int tb, int M, int N, int K, float alpha,
                                                    const float* __restrict__ A, int lda,
                                                    const float* __restrict__ B, int ldb, float beta,
                                                    float* __restrict__ Cm, int ldc, const float* __restrict__ bias) {
  constexpr int BM = 64, BN = 64, BK = 32;
  constexpr int LA = BK * BM / 256, LB = BK * BN / 256;  // slab elements per thread
  __shared__ float As[2][BK][BM + 1];
  __shared__ float Bs[2][BK][BN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
  // split-K over gridDim.z: slice z sums k in [kb, ke) and writes its partial tile to
  // Cm + z * M * ldc (beta/bias are then applied by sgemm_finish_kernel)
  const int ksz = (((K + gridDim.z - 1) / gridDim.z) + BK - 1) / BK * BK;
  const int kb = blockIdx.z * ksz, ke = min(K, kb + ksz);
  if (gridDim.z > 1) {
    Cm += (size_t)blockIdx.z * M * ldc;
    beta = 0.f;
    bias = nullptr;
    alpha = 1.f;
  }
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // element t of a slab: A at [k][m] = (t / BM, t % BM) when transposed (m contiguous in
  // memory), else (t % BK, t / BK) (k contiguous); likewise B with n
  float ra[LA], rb[LB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int t = tid + 256 * i;
      const int kk = ta ? t / BM : t % BK, mm = ta ? t % BM : t / BK;
      const int gm = m0 + mm, gk = k0 + kk;
      ra[i] = (gm < M && gk < ke) ? (ta ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk]) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int t = tid + 256 * i;
      const int kk = tb ? t % BK : t / BN, nn = tb ? t / BK : t % BN;
      const int gn = n0 + nn, gk = k0 + kk;
      rb[i] = (gn < N && gk < ke) ? (tb ? B[(size_t)gn * ldb + gk] : B[(size_t)gk * ldb + gn]) : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int t = tid + 256 * i;
      As[buf][ta ? t / BM : t % BK][ta ? t % BM : t / BK] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int t = tid + 256 * i;
      Bs[buf][tb ? t % BK : t / BN][tb ? t / BK : t % BN] = rb[i];
    }
  };
  if (kb < ke) {
    load(kb);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    const bool more = k0 + BK < ke;
    if (more) load(k0 + BK);  // in flight during this slab's MFMAs
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const int kr = kk + (lane >> 4);
      float a0 = As[buf][kr][wm + (lane & 15)], a1 = As[buf][kr][wm + 16 + (lane & 15)];
      float b0 = Bs[buf][kr][wn + (lane & 15)], b1 = Bs[buf][kr][wn + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    // the other buffer was last read before the previous barrier: safe to overwrite
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
        const int gn = n0 + wn + 16 * j + (lane & 15);
        if (gm < M && gn < N) {
          float v = alpha * acc[i][j][r];
          if (bias) v += bias[gn];
          if (beta != 0.f) v += beta * Cm[(size_t)gm * ldc + gn];
          Cm[(size_t)gm * ldc + gn] = v;
        }
      }
}

// C = alpha * sum_z ws[z] + beta * C (+ bias), fixed summation order (deterministic).
__global__ void sgemm_finish_kernel(const float* __restrict__ ws, int splits, int M, int N, int ldc, float alpha,
                                    float beta, float* __restrict__ Cm, const float* __restrict__ bias) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int m = idx / N, n = idx - m * N;
  float s = 0.f;
  for (int z = 0; z < splits; ++z) s += ws[(size_t)z * M * ldc + (size_t)m * ldc + n];
  float v = alpha * s;
  if (bias) v += bias[n];
  if (beta != 0.f) v += beta * Cm[(size_t)m * ldc + n];
  Cm[(size_t)m * ldc + n] = v;
}

// One block per sample: softmax, loss, dlogits = (p - y) * grad_scale, correct-count.
// labels: int32 class ids. out_loss[n] per-sample loss; probs optional.
__global__ __launch_bounds__(256) void softmax_xent_kernel(const float* __restrict__ logits,
                                                           const int* __restrict__ labels, int ncls,
                                                           float grad_scale, float* __restrict__ dlogits,
                                                           float* __restrict__ loss, float* __restrict__ probs,
                                                           int* __restrict__ correct) {
  const int n = blockIdx.x;
  const float* z = logits + (size_t)n * ncls;
  __shared__ float sred[8];
  __shared__ int sidx[8];
  float mx = -INFINITY;
  int amax = 0;
  for (int j = threadIdx.x; j < ncls; j += blockDim.x) {
    const float v = z[j];
    if (v > mx) { mx = v; amax = j; }
  }
  // block argmax (first index of the max)
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(mx, o, 64);
    const int oi = __shfl_xor(amax, o, 64);
    if (ov > mx || (ov == mx && oi < amax)) { mx = ov; amax = oi; }
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  if (l == 0) { sred[w] = mx; sidx[w] = amax; }
  __syncthreads();
  mx = sred[0]; amax = sidx[0];
  for (int i = 1; i < nw; ++i)
    if (sred[i] > mx || (sred[i] == mx && sidx[i] < amax)) { mx = sred[i]; amax = sidx[i]; }
  __syncthreads();
  float se = 0.f;
  for (int j = threadIdx.x; j < ncls; j += blockDim.x) se += __expf(z[j] - mx);
  se = wave_sum(se);
  if (l == 0) sred[w] = se;
  __syncthreads();
  se = 0.f;
  for (int i = 0; i < nw; ++i) se += sred[i];
  const int y = labels[n];
  const float lse = mx + __logf(se);
  const float inv = 1.f / se;
  for (int j = threadIdx.x; j < ncls; j += blockDim.x) {
    const float p = __expf(z[j] - mx) * inv;
    if (probs) probs[(size_t)n * ncls + j] = p;
    if (dlogits) dlogits[(size_t)n * ncls + j] = (p - (j == y ? 1.f : 0.f)) * grad_scale;
  }
  if (threadIdx.x == 0) {
    loss[n] = lse - z[y];
    if (correct) correct[n] = (amax == y) ? 1 : 0;
  }
}

// column sums: out[j] = scale * sum_n in[n][j]  (dense bias gradient)
// Column sums (the dense bias gradient, sum over the batch of dlogits): a block covers 32
// columns with 8 row slices of 32 lanes (coalesced 128-byte row segments, 4 independent loads
// in flight per lane), then a fixed-order LDS reduction over the slices (deterministic). The
// earlier one-thread-per-column loop ran 128 dependent-latency iterations: ~47 us for 128 x 1001.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ in, int rows, int cols,
                                                     float* __restrict__ out, float scale, int accumulate) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int j = blockIdx.x * 32 + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < cols) {
    int n = sl;
    for (; n + 24 < rows; n += 32) {
      s0 += in[(size_t)n * cols + j];
      s1 += in[(size_t)(n + 8) * cols + j];
      s2 += in[(size_t)(n + 16) * cols + j];
      s3 += in[(size_t)(n + 24) * cols + j];
    }
    for (; n < rows; n += 8) s0 += in[(size_t)n * cols + j];
  }
  red[sl][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (sl == 0 && j < cols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k][cl];
    out[j] = accumulate ? out[j] + scale * s : scale * s;
  }
}

}  // namespace drn

DRN_API int drn_bnrelu_pool(const void* x, const float* scale, const float* shift, float* pooled, int N, int HW,
                            int C, int relu, hipStream_t s) {
  if (C % 8) return (int)hipErrorInvalidValue;
  drn::launch(drn::bnrelu_pool_kernel, dim3(N), dim3(256), 0, s, (const bf16_t*)x, scale, shift, pooled, HW, C,
                     relu);
  return (int)hipGetLastError();
}

// splits > 1 needs ws with room for splits * M * ldc floats.
DRN_API int drn_sgemm(int ta, int tb, int M, int N, int K, float alpha, const float* A, int lda, const float* B,
                      int ldb, float beta, float* C, int ldc, const float* bias, int splits, float* ws,
                      hipStream_t s) {
  if (splits < 1 || (splits > 1 && ws == nullptr)) return (int)hipErrorInvalidValue;
  dim3 grid((N + 63) / 64, (M + 63) / 64, splits);
  drn::launch(drn::sgemm_kernel, grid, dim3(256), 0, s, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta,
                     splits > 1 ? ws : C, ldc, bias);
  if (splits > 1)
    drn::launch(drn::sgemm_finish_kernel, dim3((M * N + 255) / 256), dim3(256), 0, s, ws, splits, M, N, ldc,
                       alpha, beta, C, bias);
  return (int)hipGetLastError();
}

DRN_API int drn_softmax_xent(const float* logits, const int* labels, int N, int ncls, float grad_scale,
                             float* dlogits, float* loss, float* probs, int* correct, hipStream_t s) {
  drn::launch(drn::softmax_xent_kernel, dim3(N), dim3(256), 0, s, logits, labels, ncls, grad_scale, dlogits,
                     loss, probs, correct);
  return (int)hipGetLastError();
}

DRN_API int drn_colsum(const float* in, int rows, int cols, float* out, float scale, int accumulate, hipStream_t s) {
  drn::launch(drn::colsum_kernel, dim3((cols + 31) / 32), dim3(256), 0, s, in, rows, cols, out, scale,
                     accumulate);
  return (int)hipGetLastError();
}
