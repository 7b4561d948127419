// stem.hip — packed layout of the ImageNet stem convolution (7x7 / 2 over RGB).
//
// The images are stored NHWC with the 3 colour channels padded to 8 (16-byte pixels, the unit of
// every loader), so the stem's reduction k = (r, s, c) over 7 x 7 x 8 is 62.5 % zero channels:
// the forward ran 7 LDS-DMA stages of 64 (one filter row each) and the weight gradient 4 k-tiles
// of 128 for 147 useful k (reference resnet_model_official.py:301-306, the 7x7/2 stem conv).
// Packed stem (Executor.stem_pack): the input is re-laid out once per step as
//   xp[n][h][1 + w][c4]   (4 channels, one zero pixel column on each side of every row),
// so one 16-byte piece = TWO horizontally adjacent taps x 4 channels; with the filter padded to
// S = 8 taps (tap 7 zero) a filter row is 4 pieces and a 64-deep stage holds TWO filter rows:
// 4 forward stages instead of 7, and k = 7 x 8 x 4 = 224 -> 2 weight-gradient tiles of 128.
// The pad columns make a piece at w = -1 (pixels -1, 0) or w = W-1 (pixels W-1, W) valid without
// a per-pixel check: the conv kernels see an ordinary NHWC tensor of width W + 2, pad_w - 1.
// Weights: wp[k][r][s8][c4] = w[k][r][s][c] (s < 7, c < 4), refreshed after every update;
// gradient: dw[k][r][s][c] = dwp[k][r][s][c] for s < 7, c < 4, else 0.
#include "drn_common.h"

namespace drn {

// one thread per output piece: pixels (w0, w0 + 1) of one row -> 16 bytes (channels 0-3 each)
__global__ __launch_bounds__(256) void stem_pack_input_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xp,
                                                              int rows, int W, int64_t npieces) {
  const int WP = W / 2;  // pieces per row (W even, host-checked)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npieces;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / WP;
    const int j = (int)(i - row * WP);
    const uint4 a = *reinterpret_cast<const uint4*>(x + (row * W + 2 * j) * 8);
    const uint4 b = *reinterpret_cast<const uint4*>(x + (row * W + 2 * j + 1) * 8);
    // destination pixel 1 + 2j of a (W + 2)-wide row: 8-byte aligned, written as two uint2
    uint2* d = reinterpret_cast<uint2*>(xp + (row * (W + 2) + 1 + 2 * j) * 4);
    d[0] = make_uint2(a.x, a.y);
    d[1] = make_uint2(b.x, b.y);
  }
}

// wp[k][r][s8][c4] from w[k][r][s][c8] (bf16), zeros at s == 7 / c >= 4 of the source dropped
__global__ __launch_bounds__(256) void stem_pack_weights_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp,
                                                                int K, int R, int S, int C, int S8, int C4) {
  const int n = K * R * S8 * C4;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c = i % C4;
    int t = i / C4;
    const int s = t % S8;
    t /= S8;
    const int r = t % R, k = t / R;
    wp[i] = (s < S && c < C) ? w[((k * R + r) * S + s) * C + c] : (bf16_t)0;  // bf16 +0 is all-zero bits
  }
}

// dw[k][r][s][c8] (fp32) from dwp[k][r][s8][c4]; channels >= C4 and the padded tap get zero
__global__ __launch_bounds__(256) void stem_unpack_grad_kernel(const float* __restrict__ dwp, float* __restrict__ dw,
                                                               int K, int R, int S, int C, int S8, int C4) {
  const int n = K * R * S * C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c = i % C;
    int t = i / C;
    const int s = t % S;
    t /= S;
    const int r = t % R, k = t / R;
    dw[i] = c < C4 ? dwp[((k * R + r) * S8 + s) * C4 + c] : 0.f;
  }
}

}  // namespace drn

// x: [rows][W][8] bf16 (rows = N*H), xp: [rows][W + 2][4] bf16 whose pad columns the caller
// zeroed once (they are never written here).
DRN_API int drn_stem_pack_input(const void* x, void* xp, int rows, int W, hipStream_t s) {
  if (W % 2 || rows < 1) return (int)hipErrorInvalidValue;
  const int64_t np = (int64_t)rows * (W / 2);
  int64_t blocks = (np + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  drn::launch(drn::stem_pack_input_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const bf16_t*)x,
                     (bf16_t*)xp, rows, W, np);
  return (int)hipGetLastError();
}

DRN_API int drn_stem_pack_weights(const void* w, void* wp, int K, int R, int S, int C, int S8, int C4,
                                  hipStream_t s) {
  if (S8 < S || C4 > C) return (int)hipErrorInvalidValue;
  const int n = K * R * S8 * C4;
  drn::launch(drn::stem_pack_weights_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const bf16_t*)w,
                     (bf16_t*)wp, K, R, S, C, S8, C4);
  return (int)hipGetLastError();
}

DRN_API int drn_stem_unpack_grad(const float* dwp, float* dw, int K, int R, int S, int C, int S8, int C4,
                                 hipStream_t s) {
  if (S8 < S || C4 > C) return (int)hipErrorInvalidValue;
  const int n = K * R * S * C;
  drn::launch(drn::stem_unpack_grad_kernel, dim3((n + 255) / 256), dim3(256), 0, s, dwp, dw, K, R, S, C, S8,
                     C4);
  return (int)hipGetLastError();
}
