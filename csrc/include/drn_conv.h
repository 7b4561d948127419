// drn_conv.h — argument blocks for the implicit-GEMM convolution kernels.
//
// These are plain-old-data structs so that the Python runtime can build them once per layer
// at plan time (ctypes mirror in distributed_resnet_tensorflow_amd/ops/hip.py) and pass a
// pointer per launch; the field order here and there must match exactly.
#pragma once
#include <stdint.h>

// Magic-number unsigned division (n < 2^31): q = (umulhi(n, m) + n) >> s.
struct DrnFastDiv {
  uint32_t d, m, s, pad_;
};

#if defined(__HIPCC__)
// n / f.d for n < 2^31 in 3 VALU ops (a runtime-divisor integer division is ~40)
__device__ __forceinline__ uint32_t drn_fdiv(uint32_t n, const DrnFastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}
#endif

// BatchNorm finalize performed by the CONSUMER of the statistics (no separate finalize launch).
// Every workgroup of the consuming kernel derives the per-channel parameters it needs from the
// [G][2][C] statistics replicas in its prologue; the workgroup with blockIdx.x == 0 of the
// launch flagged `publish` also writes them to global memory for later kernels (and updates the
// moving averages / writes the parameter gradients). All consumers use the same device function,
// so locally derived and published values are bitwise identical.
//   forward : stats = (sum x, sum x^2); outputs scale/shift/mean/invstd (+ run_mean/run_var)
//   backward: stats = (sum g, sum g*xhat); inputs invstd; outputs dgamma = sum g*xhat,
//             dbeta = sum g
struct DrnBnFin {
  const float* stats;
  const float* gamma;
  const float* beta;
  float* run_mean;
  float* run_var;
  float* scale;
  float* shift;
  float* mean;
  float* invstd;
  float* dgamma;
  float* dbeta;
  int32_t G, C;
  float count, eps, momentum;
  int32_t publish;
};

#if defined(__HIPCC__)
// standalone forward finalize of a DrnBnFin (bn.hip; the fallback when no consumer kernel can
// finalize in its prologue)
extern "C" int drn_bn_fin_fwd_launch(const DrnBnFin* f, hipStream_t s);

// Sum of the G (<= DRN_BN_FIN_GMAX) replicas of channel c: every load is issued unconditionally
// (index clamped, the surplus masked after the load) so all 2*GMAX loads are in flight together
// instead of one dependent round trip per replica of a runtime-length loop.
#define DRN_BN_FIN_GMAX 8
__device__ __forceinline__ void drn_bn_fin_sums(const DrnBnFin& f, int c, float& s, float& q) {
  float sv[DRN_BN_FIN_GMAX], qv[DRN_BN_FIN_GMAX];
#pragma unroll
  for (int r = 0; r < DRN_BN_FIN_GMAX; ++r) {
    const int rr = r < f.G ? r : f.G - 1;
    sv[r] = f.stats[(size_t)(2 * rr) * f.C + c];
    qv[r] = f.stats[(size_t)(2 * rr + 1) * f.C + c];
  }
  s = 0.f;
  q = 0.f;
#pragma unroll
  for (int r = 0; r < DRN_BN_FIN_GMAX; ++r) {
    s += r < f.G ? sv[r] : 0.f;
    q += r < f.G ? qv[r] : 0.f;
  }
}

// forward finalize of channel c (fp32 from the fp32 sums: short dependent chain, it sits in
// the prologue of every consuming workgroup; TF fused-BN moving averages)
__device__ __forceinline__ void drn_bn_fin_fwd(const DrnBnFin& f, int c, bool pub, float& sc, float& sh) {
  float s, q;
  drn_bn_fin_sums(f, c, s, q);
  const float inv_n = 1.f / f.count;
  const float mean = s * inv_n;
  const float var = fmaxf(fmaf(-mean, mean, q * inv_n), 0.f);
  const float invstd = 1.f / sqrtf(var + f.eps);
  sc = f.gamma[c] * invstd;
  sh = fmaf(-mean, sc, f.beta[c]);
  if (pub) {
    f.scale[c] = sc;
    f.shift[c] = sh;
    f.mean[c] = mean;
    f.invstd[c] = invstd;
    if (f.run_mean != nullptr) {
      const float n = f.count;
      const float unbiased = n > 1.f ? var * (n / (n - 1.f)) : var;
      f.run_mean[c] = f.momentum * f.run_mean[c] + (1.f - f.momentum) * mean;
      f.run_var[c] = f.momentum * f.run_var[c] + (1.f - f.momentum) * unbiased;
    }
  }
}

// backward finalize of channel c: dx = k1 * (g - k2 - xhat * k3) with k1 = gamma * invstd,
// k2 = mean(g), k3 = mean(g * xhat); returned folded as dx = A*g + B*x + D
__device__ __forceinline__ void drn_bn_fin_bwd(const DrnBnFin& f, int c, bool pub, float& A, float& B, float& D) {
  float sg, sgx;
  drn_bn_fin_sums(f, c, sg, sgx);
  const float is = f.invstd[c], mu = f.mean[c];
  const float k1 = f.gamma[c] * is, k2 = sg / f.count, k3 = sgx / f.count;
  A = k1;
  B = -k1 * k3 * is;
  D = -k1 * k2 + k1 * k3 * is * mu;
  if (pub) {
    f.dbeta[c] = sg;
    f.dgamma[c] = sgx;
  }
}
#endif

// y[N][P][Q][K] = conv(x[N][H][W][C], w[K][R][S][C])  (NHWC / KRSC, bf16, fp32 accumulate)
//
// The same kernel runs the data-gradient of a convolution as a forward convolution of dY with
// the flipped, channel-transposed weights; `dil` = 2 selects the zero-dilated ("transposed")
// input indexing used for the gradient of a stride-2 convolution.
struct DrnConvFwdArgs {
  const void* x;          // bf16 [N][H][W][C]
  const void* w;          // bf16 [K][R][S][C]
  void* y;                // bf16 [N][P][Q][K]
  const float* in_scale;  // optional [C]: fused BN apply on the input: relu(x*scale+shift)
  const float* in_shift;  // optional [C]
  const void* residual;   // optional bf16 [N][P][Q][K]: y = conv + residual
  float* stats;           // optional [2][K] fp32 accumulator (+= sum, sumsq of y); pre-zeroed
  int32_t N, H, W, C, K, R, S, P, Q;
  int32_t stride, pad_h, pad_w, dil;
  int32_t relu_in;        // 1: relu after the fused scale/shift
  int32_t tiles_p;        // out: number of pixel tiles, filled by the host
  // Optional strided output mapping (phase-decomposed data gradient of a stride-2 conv): the
  // GEMM's P x Q output grid is written to y[n][i*out_stride + out_oh][j*out_stride + out_ow]
  // of a y tensor of spatial size out_H x out_W (residual uses the same mapping).
  // out_stride == 0 means the identity mapping (y is [N][P][Q][K]).
  int32_t out_H, out_W, out_stride, out_oh, out_ow;
  // Kernel configuration for drn_conv_fwd2: -1 automatic, 0..7 an LDS-DMA tile configuration
  // (DRN_GLDS_CONFIGS), 100 the register-staged kernel.
  int32_t cfg;
  // stats holds stats_rep replicas [rep][2][K]; block b adds into replica b % rep, so no
  // address collects more than blocks/rep atomics (same-address float atomics serialize).
  int32_t stats_rep;
  // Optional fused BatchNorm-backward reduction (data-gradient launches): when bn_x is set the
  // conv output v is d/d relu(bn(bn_x)); the epilogue stores the ReLU-masked gradient
  // g = v * [bn_x*scale+shift > 0] and accumulates stats[0][k] += g,
  // stats[1][k] += g * (bn_x - mean) * invstd instead of the forward statistics.
  const void* bn_x;       // bf16, same layout as y
  const float* bn_scale;
  const float* bn_shift;
  const float* bn_mean;
  const float* bn_invstd;
  // Optional fused BatchNorm finalize (needs stats): the workgroups of each BC-wide channel
  // column count themselves in fin_cnt[c0 / BC]; the last to arrive sums the stats replicas of
  // its channels and writes the BN parameters -- forward: fin_scale/shift/mean/invstd and the
  // moving averages; with bn_x set: fin_dgamma = sum g*xhat, fin_dbeta = sum g and
  // fin_coef[3][K] = (gamma*invstd, mean g, mean g*xhat) -- then re-arms its counter. Replaces
  // the separate finalize launch; with a multi-launch output (phase-decomposed data gradient)
  // only the last launch carries it.
  unsigned* fin_cnt;
  float fin_count, fin_eps, fin_momentum;
  // With a strided output map: 1 = the epilogue also stores zeros at the other phase positions
  // of every output pixel (single-phase data gradient, e.g. a 1x1 stride-2 projection), so the
  // output tensor needs no separate clearing pass.
  int32_t out_fill;
  const float* fin_gamma;
  const float* fin_beta;
  float* fin_run_mean;
  float* fin_run_var;
  float* fin_scale;
  float* fin_shift;
  float* fin_mean;
  float* fin_invstd;
  float* fin_dgamma;
  float* fin_dbeta;
  float* fin_coef;
  // pixel-index decode m -> (n, p, q): divisors P*Q and Q (filled by the host)
  DrnFastDiv fd_pq, fd_q;
  // Optional consumer-side finalize of the INPUT BatchNorm (LDS-DMA kernels with the fused
  // prologue): when in_fin.stats is set the prologue derives scale/shift from the statistics
  // instead of reading in_scale/in_shift (see DrnBnFin).
  DrnBnFin in_fin;
  // Split-K (LDS-DMA kernels, ksplit > 1): partial-tile workspace [tiles][ksplit][BP*BC] fp32 and
  // one zeroed ticket word per output tile (the last arriver re-arms it).
  // Stream-K (sk_blocks > 0): sk_blocks workgroups share the tiles x k-stages units evenly;
  // ksplit is then the partial slots per tile (>= drn_conv_sk_slots_cfg(args, cfg, sk_blocks)).
  float* ks_ws;
  unsigned* ks_tickets;
  int32_t ksplit;
  int32_t sk_blocks;
};

// dW[K][R][S][C] (+)= sum_{n,p,q} dy[n,p,q,k] * x[n, p*st-pad+r, q*st-pad+s, c]
// Split-K over output pixels: partial slabs out[split][K][R*S*C] (fp32); splits==1 writes
// the final gradient directly.
struct DrnConvWgradArgs {
  const void* x;          // bf16 [N][H][W][C] (forward input, pre-activation if fused)
  const void* dy;         // bf16 [N][P][Q][K]
  float* out;             // fp32 [splits][K][R*S*C]
  const float* in_scale;  // optional fused BN apply (recompute of the forward prologue)
  const float* in_shift;
  int32_t N, H, W, C, K, R, S, P, Q;
  int32_t stride, pad_h, pad_w;
  int32_t relu_in;
  int32_t splits, pix_per_split;
  DrnFastDiv fd_pq, fd_q;
  // 1: every split adds its tile into out = the final, pre-zeroed gradient with fp32 atomics
  // (no partial slabs, no drn_splitk_reduce)
  int32_t atomic_out;
};
