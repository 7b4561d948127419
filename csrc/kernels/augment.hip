// augment.hip — GPU-side input preprocessing producing NHWC bf16 images with the channel
// dimension zero-padded 3 -> 8 (16-byte vectors for the stem convolution's implicit GEMM).
//
// CIFAR (reference resnet_cifar_main.py:185-200): train = pad 4 px per side (zeros, raw 0..255
// values), random 32x32 crop, random left-right flip, then tf.image.per_image_standardization
// (x - mean) / max(stddev, 1/sqrt(H*W*C)); eval = standardization only. Crop/flip draws come
// from the host RNG per image (params[n] = {oy, ox, flip}).
//
// ImageNet (reference vgg_preprocessing.py:259-333 via resnet_imagenet_main.py:115-155): the
// decoded uint8 image (scaled to [0,1]) is aspect-preserving bilinear-resized (TF1 legacy
// mapping, src = dst * in/out, align_corners=False, no half-pixel offset) to (rh, rw), cropped
// at (cy, cx) to 224x224, optionally flipped, and the VGG RGB means (/255) are subtracted.
// Resize + crop + flip + mean-subtraction are fused: only the 224x224 output pixels are
// interpolated.
#include "drn_common.h"

namespace drn {

__global__ __launch_bounds__(256) void cifar_augment_kernel(const uint8_t* __restrict__ in, const int* __restrict__ params,
                                                            bf16_t* __restrict__ out, int H, int W, int pad) {
  const int n = blockIdx.x;
  const int oy = params[n * 3 + 0], ox = params[n * 3 + 1], flip = params[n * 3 + 2];
  const int HW = H * W;
  const uint8_t* img = in + (size_t)n * HW * 3;
  constexpr int MAXP = 8;  // up to 2048 pixels per image with 256 threads
  float v[MAXP][3];
  float s = 0.f, q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXP; ++i) {
    const int pix = threadIdx.x + i * 256;
    v[i][0] = v[i][1] = v[i][2] = 0.f;
    if (pix < HW) {
      const int y = pix / W, x = pix % W;
      const int xs = flip ? (W - 1 - x) : x;
      const int sy = y + oy - pad, sx = xs + ox - pad;
      if (sy >= 0 && sy < H && sx >= 0 && sx < W) {
        const uint8_t* p = img + ((size_t)sy * W + sx) * 3;
        v[i][0] = p[0]; v[i][1] = p[1]; v[i][2] = p[2];
      }
      s += v[i][0] + v[i][1] + v[i][2];
      q += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2];
    }
  }
  __shared__ float red[2][4];
  s = wave_sum(s);
  q = wave_sum(q);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = s; red[1][threadIdx.x >> 6] = q; }
  __syncthreads();
  s = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  q = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  const float cnt = (float)(HW * 3);
  const float mean = s / cnt;
  const float var = fmaxf(q / cnt - mean * mean, 0.f);
  const float adj = fmaxf(sqrtf(var), rsqrtf(cnt));
  const float inv = 1.f / adj;
#pragma unroll
  for (int i = 0; i < MAXP; ++i) {
    const int pix = threadIdx.x + i * 256;
    if (pix < HW) {
      float f[8] = {(v[i][0] - mean) * inv, (v[i][1] - mean) * inv, (v[i][2] - mean) * inv, 0.f, 0.f, 0.f, 0.f, 0.f};
      reinterpret_cast<uint4*>(out)[(size_t)n * HW + pix] = pack8(f);
    }
  }
}

struct ImgDesc {
  int64_t offset;       // byte offset of the HWC uint8 image in the packed buffer
  int32_t H, W;         // decoded size
  int32_t rh, rw;       // resized size (aspect preserving)
  int32_t cy, cx;       // crop origin in the resized image
  int32_t flip, pad_;
};

__global__ __launch_bounds__(256) void vgg_preprocess_kernel(const uint8_t* __restrict__ in,
                                                             const ImgDesc* __restrict__ desc,
                                                             bf16_t* __restrict__ out, int OH, int OW, float m0,
                                                             float m1, float m2) {
  const int n = blockIdx.y;
  const ImgDesc d = desc[n];
  const uint8_t* img = in + d.offset;
  const float sy = (float)d.H / (float)d.rh, sx = (float)d.W / (float)d.rw;
  for (int pix = blockIdx.x * blockDim.x + threadIdx.x; pix < OH * OW; pix += gridDim.x * blockDim.x) {
    const int y = pix / OW, x0 = pix % OW;
    const int x = d.flip ? (OW - 1 - x0) : x0;
    const float fy = (float)(y + d.cy) * sy, fx = (float)(x + d.cx) * sx;
    int y0 = (int)floorf(fy), xl = (int)floorf(fx);
    y0 = min(max(y0, 0), d.H - 1);
    xl = min(max(xl, 0), d.W - 1);
    const int y1 = min(y0 + 1, d.H - 1), x1 = min(xl + 1, d.W - 1);
    const float wy = fy - (float)y0, wx = fx - (float)xl;
    float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float a = img[((size_t)y0 * d.W + xl) * 3 + c], b = img[((size_t)y0 * d.W + x1) * 3 + c];
      const float e = img[((size_t)y1 * d.W + xl) * 3 + c], g = img[((size_t)y1 * d.W + x1) * 3 + c];
      const float top = a + (b - a) * wx, bot = e + (g - e) * wx;
      f[c] = (top + (bot - top) * wy) * (1.f / 255.f);
    }
    f[0] -= m0; f[1] -= m1; f[2] -= m2;
    reinterpret_cast<uint4*>(out)[(size_t)n * OH * OW + pix] = pack8(f);
  }
}

// Synthetic benchmark images: deterministic hash noise in [-1, 1) (3 live channels of 8).
__global__ void synthetic_images_kernel(bf16_t* __restrict__ out, int64_t npix, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix; i += (int64_t)gridDim.x * blockDim.x) {
    float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      uint32_t h = (uint32_t)(i * 3 + c) * 2654435761u ^ seed;
      h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
      f[c] = (float)(h >> 8) * (2.f / 16777216.f) - 1.f;
    }
    reinterpret_cast<uint4*>(out)[i] = pack8(f);
  }
}

}  // namespace drn

DRN_API int drn_cifar_augment(const uint8_t* in, const int* params, void* out, int N, int H, int W, int pad,
                              hipStream_t s) {
  if (H * W > 2048) return (int)hipErrorInvalidValue;
  drn::launch(drn::cifar_augment_kernel, dim3(N), dim3(256), 0, s, in, params, (bf16_t*)out, H, W, pad);
  return (int)hipGetLastError();
}

DRN_API int drn_vgg_preprocess(const uint8_t* in, const void* desc, void* out, int N, int OH, int OW, float m0,
                               float m1, float m2, hipStream_t s) {
  dim3 grid((OH * OW + 255) / 256, N);
  drn::launch(drn::vgg_preprocess_kernel, grid, dim3(256), 0, s, in, (const drn::ImgDesc*)desc, (bf16_t*)out,
                     OH, OW, m0, m1, m2);
  return (int)hipGetLastError();
}

DRN_API int drn_synthetic_images(void* out, int64_t npix, uint32_t seed, hipStream_t s) {
  int64_t b = (npix + 255) / 256;
  if (b > 8192) b = 8192;
  drn::launch(drn::synthetic_images_kernel, dim3((int)b), dim3(256), 0, s, (bf16_t*)out, npix, seed);
  return (int)hipGetLastError();
}
