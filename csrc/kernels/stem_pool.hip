// stem_pool.hip — the ImageNet stem's packed 7x7/2 convolution fused with its 3x3/2 max-pool
// (the packed layout itself: stem.hip). Kept out of stem.hip, whose text keys the kernel-selection
// database (ops/build.py tune_hash): this kernel is not tuned.
#include "drn_common.h"

#include <algorithm>

namespace drn {

// ---------------------------------------------------------------------------------------
// Fused ImageNet stem: the packed 7x7/2 convolution, the 3x3/2 'SAME' max-pool and the pooled
// output's BatchNorm statistics in ONE kernel (reference resnet_model_official.py:301-316: the v2
// stem is conv -> max-pool, the first BatchNorm acts on the pooled tensor). The two-kernel path
// wrote the 112x112x64 conv output (205 MB at bs 128) only for the pooling kernel to read it
// back; here a workgroup computes the conv rows of TWO pooled rows (5 conv rows, the shared
// 5th row recomputed by the next tile: 1.25x the stem's small MFMA work) into LDS and pools
// them there, so only the pooled tensor (51 MB) and its argmax bytes reach HBM.
//
// Workgroup (n, t, h): conv rows cr0 = 4t .. 4t + 4 of image n, output channels [h*32, h*32+32).
//   1. The 15 input rows those conv rows read (xp, packed 4-channel pixels) -> LDS, zero outside
//      the image (row) or the packed row (column), 16-byte pixel pairs, all loads in flight.
//   2. MFMA 16x16x32: A = weights (16 channels x one filter row r: taps 0-7 x 4 channels = 32 k,
//      held in VGPRs for the whole workgroup), B = 16 output pixels of one conv row x the same
//      32 k (one 16-byte tap-pair piece per lane, read from LDS); 7 MFMAs (r = 0..6) per
//      16-pixel x 16-channel block. The fp32 results are rounded to bf16 (as the two-kernel
//      path stores them) into an LDS tile.
//   3. Pooling from the LDS tile: max and first-max tap (r*3 + s, strict '>', out-of-image taps
//      -inf) per 8-channel group -> pooled y + argmax (the layout maxpool_bwd reads); the sums /
//      sums of squares of the pooled values -> the first block's BN statistics replica
//      blockIdx % rep (maxpool_fwd_kernel's fused-statistics contract).
// DRN_STEM_ISO_NOLOAD / _NOMMA / _NOPOOL: measurement builds without one phase
// (scripts/stem_pool_iso.py --variants).
// Host-checked: 7x7 filter packed to [K][7][8][4], stride 2, Q % 16 == 0 and Q <= 112, K % 32,
// the pooled geometry P' = ceil(P/2) with no leading pad (224 -> 112 -> 56).
constexpr int STEM_PQ_MAX = 112;                     // conv output columns (LDS tile width)
constexpr int STEM_IN_COLS = 2 * STEM_PQ_MAX + 8;    // LDS input row: packed cols -2 .. 2Q+5
constexpr int STEM_IN_ROWS = 15;                     // input rows of 5 conv rows (stride 2, 7 taps)
constexpr int STEM_CH = 32;                          // output channels per workgroup
constexpr int STEM_IN_BYTES = STEM_IN_ROWS * STEM_IN_COLS * 8;
constexpr int STEM_OUT_PITCH = STEM_CH * 2 + 16;    // bytes per pixel of the LDS output tile (padded)
constexpr int STEM_OUT_BYTES = 5 * STEM_PQ_MAX * STEM_OUT_PITCH;

struct StemPoolArgs {
  const bf16_t* xp;   // [N][H][W + 2][4]
  const bf16_t* w4;   // [K][7][8][4]
  bf16_t* y;          // [N][PP][QP][K] pooled
  uint8_t* arg;       // [N][PP][QP][K] first-max tap
  float* part;        // [rep][2][K] or nullptr
  int rep, N, H, W, P, Q, PP, QP, K, pad_h, pad_w4;
};

// LDS output tile: pixel px (0 .. 5Q-1, row-major over the 5 conv rows) x 32 channels bf16 =
// 8 chunks of 8 bytes, pixels 80 bytes apart: with the pooling's lane mapping (16 pooled columns x
// 4 channel groups per 64 lanes) its 16-byte reads are bank-conflict free (a 64-byte pitch put
// every pixel on the same few banks: 43 % of the LDS cycles were conflicts).
__device__ __forceinline__ int stem_out_off(int px, int cc) { return px * STEM_OUT_PITCH + cc * 8; }

// Persistent: workgroup b keeps channel half h = b % KH (its weights stay in VGPRs) and walks the
// (image, tile) pairs j = b / KH, += gridDim / KH; the next tile's input rows are loaded into
// registers while the current tile computes and pools (the load latency hides behind the work),
// and the BN statistics are accumulated across the workgroup's tiles and added once at the end.
__device__ __forceinline__ void stem_load_rows(const StemPoolArgs& a, int j, int TT, int tid, u32x4_t (&v)[7]) {
  const u32x4_t* __restrict__ xg = reinterpret_cast<const u32x4_t*>(a.xp);
  const int n = j / TT, t = j - n * TT;
  const int hb = 2 * (4 * t) - a.pad_h, WX = a.W + 2, npair = a.Q + 4, nld = STEM_IN_ROWS * npair;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const int i = tid + 256 * k;
    const int r = i / npair, c = i - r * npair;
    const int hh = hb + r, cx = 2 * c - 2;
    v[k] = u32x4_t{0u, 0u, 0u, 0u};
#ifndef DRN_STEM_ISO_NOLOAD
    if (i < nld && (unsigned)hh < (unsigned)a.H && (unsigned)cx < (unsigned)WX)
      v[k] = xg[(((size_t)n * a.H + hh) * WX + cx) >> 1];
#else
    v[k].x = hh + cx + i + nld;   // (isolation build: no global loads)
#endif
  }
}

__global__ __launch_bounds__(256) void stem_conv_pool_kernel(StemPoolArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* in = smem;                       // [15][STEM_IN_COLS][4] bf16
  char* out = smem + STEM_IN_BYTES;      // output tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kg = lane >> 4;
  const int KH = a.K / STEM_CH, TT = (a.PP + 1) / 2, NT = a.N * TT;
  const int h = blockIdx.x % KH, jstep = gridDim.x / KH;
  static_assert((STEM_IN_ROWS * STEM_IN_COLS / 2 + 255) / 256 == 7, "staging registers");
  u32x4_t v[7];
  int j = blockIdx.x / KH;
  if (j < NT) stem_load_rows(a, j, TT, tid, v);
  // weights of this workgroup's 32 channels: A fragments for (channel tile i, filter row r)
  bf16x8_t wa[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 7; ++r)
      wa[i][r] = *reinterpret_cast<const bf16x8_t*>(a.w4 + (size_t)(h * STEM_CH + i * 16 + (lane & 15)) * 224 +
                                                    r * 32 + kg * 8);
  // retire the weight loads here, before the tile loop: left pending, the compiler's waits for them
  // inside the loop (vmcnt counts in issue order) also drained each tile's prefetch every tile
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 7; ++r) asm volatile("" : "+v"(wa[i][r]));
  const int g = (tid >> 4) & 3;          // the thread's 8-channel group in the pooling phase
  float s[8], sq[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[q] = sq[q] = 0.f;
  const int npair = a.Q + 4, nld = STEM_IN_ROWS * npair;
  const int mpr = a.Q / 16, MT = 5 * mpr;
  // the staged rows of tile j -> LDS (`in` is free: every wave is past the conv phase)
  auto stage = [&](int jj) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const int i = tid + 256 * k;
      const int r = i / npair, c = i - r * npair;
      if (i < nld) *reinterpret_cast<u32x4_t*>(in + (r * STEM_IN_COLS + 2 * c) * 8) = v[k];
    }
  };
  // Pipeline: tile j's rows are in LDS when its iteration starts; the registers hold tile
  // j + jstep's rows, loaded during tile j - jstep's pooling and tile j's conv phase, written to
  // LDS right after that conv phase -- and the loads for tile j + 2 jstep are issued right then,
  // BEFORE tile j's pooling stores: vmcnt counts in issue order, so each wait for staged rows only
  // ever waits behind the stores of a pooling that ended a whole conv phase earlier.
  if (j < NT) {
    stage(j);
    if (j + jstep < NT) stem_load_rows(a, j + jstep, TT, tid, v);
  }
  for (; j < NT; j += jstep) {
    const int n = j / TT, t = j - n * TT;
    const int cr0 = 4 * t;
    // (orders this tile's staged rows before the conv phase, and the previous tile's pooling
    // reads of `out` before this conv phase's writes)
    __syncthreads();
    const bool more = j + jstep < NT;
    // 2. conv: 16-pixel blocks of the 5 conv rows, round-robin over the waves
    const int mend = min(MT, (a.P - cr0) * mpr);      // (rows past the image: never pooled)
#ifdef DRN_STEM_ISO_NOMMA
    if (mend < 0)   // (isolation build: no conv phase)
#endif
#pragma unroll 1
    for (int mt = wave; mt < mend; mt += 4) {
      const int rl = mt / mpr, q = (mt - rl * mpr) * 16 + (lane & 15);
      // packed col of this lane's piece for filter row r: 2q - pad_w4 + 2kg (LDS col - 2)
      const char* src = in + ((2 * rl) * STEM_IN_COLS + 2 * q - a.pad_w4 + 2 * kg + 2) * 8;
      bf16x8_t b[7];
#pragma unroll
      for (int r = 0; r < 7; ++r) b[r] = *reinterpret_cast<const bf16x8_t*>(src + r * STEM_IN_COLS * 8);
      f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 7; ++r) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][r], b[r], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1][r], b[r], acc1, 0, 0, 0);
      }
      // lane holds channels i*16 + 4*kg .. +3 of pixel (rl, q): one 8-byte chunk each
      const int px = rl * a.Q + q;
      *reinterpret_cast<uint2*>(out + stem_out_off(px, kg)) =
          make_uint2(pack2bf(acc0[0], acc0[1]), pack2bf(acc0[2], acc0[3]));
      *reinterpret_cast<uint2*>(out + stem_out_off(px, 4 + kg)) =
          make_uint2(pack2bf(acc1[0], acc1[1]), pack2bf(acc1[2], acc1[3]));
    }
    __syncthreads();
    if (more) {
      stage(j + jstep);
      if (j + 2 * jstep < NT) stem_load_rows(a, j + 2 * jstep, TT, tid, v);
    }
    // 3. pooling: item = (pooled column slot, 8-channel group g): per 64 items, 16 consecutive slots
    // (slot = pr * QP + pooled col over the tile's two pooled rows) x the 4 groups, so g = (tid /
    // 16) % 4 is fixed per thread; the 9 taps are read unconditionally (clamped address, one
    // 16-byte read each) and masked to -inf, all 9 reads of an item in flight together
#ifndef DRN_STEM_ISO_NOPOOL
    const int nslot = 2 * a.QP, nitems = (nslot + 15) / 16 * 64;
#else
    const int nslot = 2 * a.QP, nitems = 0;   // (isolation build: no pooling phase)
#endif
#pragma unroll 1
    for (int it = tid; it < nitems; it += 256) {
      const int slot = (it >> 6) * 16 + (it & 15);
      if (slot >= nslot) continue;
      const int pr = slot >= a.QP ? 1 : 0, qq = slot - pr * a.QP;
      const int pp = 2 * t + pr;
      if (pp >= a.PP) continue;
      // an out-of-image tap reads tap 0 of the window again (always inside): a repeat of an
      // earlier value never wins the strict '>' -- no per-element -inf masking
      uint4 tv[9];
      const int px0 = 2 * pr * a.Q + 2 * qq;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int rl = 2 * pr + tap / 3, qc = 2 * qq + tap % 3;
        const bool ok = cr0 + rl < a.P && qc < a.Q;
        tv[tap] = *reinterpret_cast<const uint4*>(out + stem_out_off(ok ? rl * a.Q + qc : px0, 2 * g));
      }
      // branch-free first-max (selects, not per-element branches: hipcc turned the conditional
      // byte stores into divergent branches, 2x the kernel's time)
      float best[8];
      int bi[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) { best[q] = -INFINITY; bi[q] = 0; }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        float f[8];
        unpack8(tv[tap], f);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const bool gt = f[q] > best[q];
          best[q] = gt ? f[q] : best[q];
          bi[q] = gt ? tap : bi[q];
        }
      }
      const size_t o = (((size_t)n * a.PP + pp) * a.QP + qq) * a.K + h * STEM_CH + g * 8;
      *reinterpret_cast<uint4*>(a.y + o) = pack8(best);   // (exact: maxima of bf16 values)
      uint2 av;
      av.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
      av.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
      *reinterpret_cast<uint2*>(a.arg + o) = av;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s[q] += best[q];
        sq[q] += best[q] * best[q];
      }
    }
  }
  if (a.part == nullptr) return;   // (uniform)
  // statistics: reduce the 64 threads of each channel group through LDS (`in` is dead: the last
  // conv phase ended at the barrier before the last pooling)
  float* red = reinterpret_cast<float*>(smem);   // [256][17]
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    red[tid * 17 + q] = s[q];
    red[tid * 17 + 8 + q] = sq[q];
  }
  __syncthreads();
  if (tid < 2 * STEM_CH) {
    const int c = tid >> 1, which = tid & 1;
    const int gg = c >> 3, q = c & 7;
    float acc = 0.f;
    for (int u = 0; u < 256; ++u)
      if (((u >> 4) & 3) == gg) acc += red[u * 17 + which * 8 + q];
    atomicAdd(a.part + ((size_t)((blockIdx.x / KH) % a.rep) * 2 + which) * a.K + h * STEM_CH + c, acc);
  }
}

}  // namespace drn

// Fused stem conv + 3x3/2 max-pool (+ pooled BN statistics when part != nullptr); see
// stem_conv_pool_kernel for the geometry it accepts.
DRN_API int drn_stem_conv_pool(const void* xp, const void* w4, void* y, uint8_t* arg, float* part, int rep, int N,
                               int H, int W, int P, int Q, int PP, int QP, int K, int pad_h, int pad_w4,
                               hipStream_t s) {
  // (pad_w4 <= 2: the LDS input row starts at packed column -2; rows outside the image read zero)
  if (Q % 16 || Q > drn::STEM_PQ_MAX || K % drn::STEM_CH || N < 1 || P < 1 || PP != (P + 1) / 2 ||
      QP != (Q + 1) / 2 || (part != nullptr && rep < 1) || pad_w4 < 0 || pad_w4 > 2 || pad_h < 0 || pad_h > 3 ||
      W + 2 < 2 * Q)
    return (int)hipErrorInvalidValue;
  drn::StemPoolArgs a{(const bf16_t*)xp, (const bf16_t*)w4, (bf16_t*)y, arg, part, rep > 0 ? rep : 1,
                      N, H, W, P, Q, PP, QP, K, pad_h, pad_w4};
  // persistent: two workgroups per CU (LDS-bound), a multiple of the channel halves
  const int KH = K / drn::STEM_CH, tiles = N * ((PP + 1) / 2) * KH;
  const int blocks = std::min(tiles, 512 / KH * KH);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(drn::stem_conv_pool_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, drn::STEM_IN_BYTES + drn::STEM_OUT_BYTES);
    attr_set = true;
  }
  drn::launch(drn::stem_conv_pool_kernel, dim3(blocks), dim3(256), drn::STEM_IN_BYTES + drn::STEM_OUT_BYTES, s, a);
  return (int)hipGetLastError();
}
